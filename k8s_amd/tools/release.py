"""Release packaging: native artefacts, image build contexts and the Helm chart with the image tag.

Parity: /root/reference/py/release.py:116-281 (build the operator + e2e binaries, copy them and the default
PS server into the Docker context, package the chart with values rewritten to the new image) and
py/build_and_push_image.py. Registry push and GCS upload are out of scope here (no network); the output
directory holds everything a CI job would push:

    <out>/operator-context/   Dockerfile + bin/tf_operator + bin/e2e + ps_server/grpc_tensorflow_server.py
    <out>/trainer-context/    Dockerfile + the k8s_amd package (with the gfx950 kernels .so) + bench.py
    <out>/tf-job-operator-chart-<version>.tgz   chart with image: <registry>/tf_operator:<tag>
    <out>/manifest.json       what was built (git sha, tag, files)

    python -m k8s_amd.tools.release --out dist --registry ghcr.io/me --tag v0.3.0-rocm7 [--skip-build]
"""
from __future__ import annotations

import argparse
import io
import json
import os
import shutil
import subprocess
import sys
import tarfile

import yaml

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
VERSION = "0.3.0"


def git_sha(short=True) -> str:
    try:
        return subprocess.run(["git", "rev-parse", "--short" if short else "HEAD"], cwd=REPO, capture_output=True,
                              text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return "unknown"


def update_values(values_text: str, image: str, test_image: str = None) -> str:
    """values.yaml with ``image`` (and optionally ``test_image``) replaced (release.py update_values)."""
    v = yaml.safe_load(values_text) or {}
    v["image"] = image
    if test_image:
        v["test_image"] = test_image
    return yaml.safe_dump(v, sort_keys=False)


def package_chart(chart_dir: str, out_dir: str, image: str, version: str, test_image: str = None) -> str:
    """tar.gz of the chart (helm package layout: <name>/...), Chart.yaml version/appVersion set."""
    chart = yaml.safe_load(open(os.path.join(chart_dir, "Chart.yaml")))
    name = chart["name"]
    chart["version"] = version
    chart["appVersion"] = version
    out = os.path.join(out_dir, "%s-%s.tgz" % (name, version))
    with tarfile.open(out, "w:gz") as tf:
        for root, _, files in os.walk(chart_dir):
            for f in sorted(files):
                p = os.path.join(root, f)
                rel = os.path.relpath(p, chart_dir)
                data = open(p, "rb").read()
                if rel == "Chart.yaml":
                    data = yaml.safe_dump(chart, sort_keys=False).encode()
                elif rel == "values.yaml":
                    data = update_values(data.decode(), image, test_image).encode()
                info = tarfile.TarInfo(os.path.join(name, rel))
                info.size = len(data)
                info.mode = 0o644
                tf.addfile(info, io.BytesIO(data))
    return out


def _copy(src, dst):
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    if os.path.isdir(src):
        shutil.copytree(src, dst, ignore=shutil.ignore_patterns("__pycache__", "*.o", "csrc"), dirs_exist_ok=True)
    else:
        shutil.copy2(src, dst)


def build_contexts(out: str) -> dict:
    files = {}
    op = os.path.join(out, "operator-context")
    _copy(os.path.join(REPO, "images", "operator", "Dockerfile"), os.path.join(op, "Dockerfile"))
    for b in ("tf_operator", "e2e"):
        _copy(os.path.join(REPO, "bin", b), os.path.join(op, "bin", b))
    _copy(os.path.join(REPO, "k8s_amd", "ps_server", "grpc_tensorflow_server.py"),
          os.path.join(op, "ps_server", "grpc_tensorflow_server.py"))
    files["operator"] = sorted(os.path.relpath(os.path.join(r, f), out) for r, _, fs in os.walk(op) for f in fs)
    tr = os.path.join(out, "trainer-context")
    _copy(os.path.join(REPO, "images", "trainer", "Dockerfile"), os.path.join(tr, "Dockerfile"))
    _copy(os.path.join(REPO, "k8s_amd"), os.path.join(tr, "k8s_amd"))
    _copy(os.path.join(REPO, "bench.py"), os.path.join(tr, "bench.py"))
    files["trainer"] = len([1 for _, _, fs in os.walk(tr) for _ in fs])
    return files


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", default="dist")
    ap.add_argument("--registry", default="k8s-amd")
    ap.add_argument("--tag", default=None, help="image tag (default: <version>-<git sha>)")
    ap.add_argument("--skip-build", action="store_true", help="package the already-built artefacts")
    a = ap.parse_args(argv)
    tag = a.tag or "%s-%s" % (VERSION, git_sha())
    out = os.path.abspath(a.out)
    os.makedirs(out, exist_ok=True)
    if not a.skip_build:
        from k8s_amd import _build

        _build.build_all()
    missing = [b for b in ("tf_operator", "e2e") if not os.path.exists(os.path.join(REPO, "bin", b))]
    if missing:
        print("missing binaries %s: run python -m k8s_amd._build" % missing, file=sys.stderr)
        return 1
    files = build_contexts(out)
    image = "%s/tf_operator:%s" % (a.registry, tag)
    chart = package_chart(os.path.join(REPO, "charts", "tf-job-operator"), out, image, tag.lstrip("v"),
                          test_image="%s/tf_sample:%s" % (a.registry, tag))
    tb = package_chart(os.path.join(REPO, "charts", "tensorboard"), out, "%s/trainer:%s" % (a.registry, tag),
                       tag.lstrip("v"))
    manifest = {"version": VERSION, "tag": tag, "git": git_sha(short=False), "operator_image": image,
                "trainer_image": "%s/trainer:%s" % (a.registry, tag), "charts": [os.path.basename(chart),
                                                                                 os.path.basename(tb)],
                "files": files}
    with open(os.path.join(out, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps({k: manifest[k] for k in ("tag", "operator_image", "charts")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
