"""Deploy / test / tear down the operator on a cluster of MI355X nodes (helm + kubectl), or on the one-box local
cluster.

Parity: /root/reference/py/deploy.py (``setup``: create a GKE cluster with GPU nodes, install the GPU driver
daemonset, ``helm install`` the chart and wait; ``test``: ``helm test tf-job`` with JUnit output; ``teardown``).
Cluster creation is a cloud API call with no MI355X equivalent here; ``setup`` starts from an existing
kubectl context, checks that the nodes advertise ``amd.com/gpu`` (the ROCm device plugin's resource, the
``nvidia.com/gpu`` wait in py/util.py:265-375), installs the chart with ``cloud=amd`` and the image tag, and
waits for the operator Deployment. ``--dryrun`` prints the commands instead of running them (py/util.py:31-70).

    python -m k8s_amd.tools.deploy setup --image ghcr.io/me/tf_operator:v0.3.0-rocm7 [--dryrun]
    python -m k8s_amd.tools.deploy test --junit out/junit_deploy.xml
    python -m k8s_amd.tools.deploy teardown
    python -m k8s_amd.tools.deploy local --junit out/junit_local.xml   # fake API server + kubelet + bin/e2e
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time
from typing import List, Optional

from k8s_amd.tools.junit import TestCase, create_junit_xml_file

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHART = os.path.join(REPO, "charts", "tf-job-operator")
RELEASE = "tf-job"


class Runner:
    def __init__(self, dryrun: bool):
        self.dryrun = dryrun
        self.log: List[str] = []

    def run(self, cmd: List[str], check: bool = True, capture: bool = False) -> str:
        line = " ".join(shlex.quote(c) for c in cmd)
        self.log.append(line)
        print("+ " + line, flush=True)
        if self.dryrun:
            return ""
        pipe = subprocess.PIPE if capture else None
        r = subprocess.run(cmd, stdout=pipe, stderr=subprocess.STDOUT if capture else None, text=True)
        if check and r.returncode != 0:
            raise RuntimeError("command failed (%d): %s\n%s" % (r.returncode, line, r.stdout or ""))
        return r.stdout or ""


def gpu_capacity(nodes_json: str, resource: str = "amd.com/gpu") -> int:
    """Total allocatable ``resource`` over the nodes of a ``kubectl get nodes -o json`` document."""
    total = 0
    for n in json.loads(nodes_json or "{}").get("items", []):
        v = n.get("status", {}).get("allocatable", {}).get(resource)
        if v is not None:
            total += int(str(v))
    return total


def setup(a, r: Runner) -> int:
    ctx = ["--context", a.context] if a.context else []
    if a.min_gpus > 0:
        end = time.time() + a.timeout
        while True:
            have = gpu_capacity(r.run(["kubectl"] + ctx + ["get", "nodes", "-o", "json"], capture=True))
            if r.dryrun or have >= a.min_gpus:
                break
            if time.time() > end:
                print("nodes advertise %d amd.com/gpu, need %d (is the ROCm device plugin installed?)"
                      % (have, a.min_gpus), file=sys.stderr)
                return 1
            time.sleep(10)
    repo, _, tag = a.image.rpartition(":")
    r.run(["helm"] + (["--kube-context", a.context] if a.context else []) +
          ["upgrade", "--install", RELEASE, a.chart, "--namespace", a.namespace, "--create-namespace", "--wait",
           "--timeout", "%ds" % int(a.timeout), "--set", "cloud=amd",
           "--set", "image=%s:%s" % (repo or a.image, tag or "latest"), "--set", "rbac.install=true"])
    r.run(["kubectl"] + ctx + ["-n", a.namespace, "rollout", "status", "deployment/tf-job-operator",
                               "--timeout=%ds" % int(a.timeout)])
    return 0


def test(a, r: Runner) -> int:
    t0 = time.time()
    ok, msg = True, ""
    try:
        r.run(["helm"] + (["--kube-context", a.context] if a.context else []) +
              ["test", RELEASE, "--namespace", a.namespace, "--timeout", "%ds" % int(a.timeout), "--logs"])
    except RuntimeError as e:
        ok, msg = False, str(e)
    if a.junit:
        create_junit_xml_file([TestCase("deploy", "helm-test", time.time() - t0, None if ok else msg)], a.junit)
    return 0 if ok else 1


def teardown(a, r: Runner) -> int:
    r.run(["helm"] + (["--kube-context", a.context] if a.context else []) +
          ["uninstall", RELEASE, "--namespace", a.namespace], check=False)
    r.run(["kubectl"] + (["--context", a.context] if a.context else []) +
          ["delete", "crd", "tfjobs.tensorflow.org", "--ignore-not-found"], check=False)
    return 0


def local(a, r: Runner) -> int:
    """The helm test against the one-box cluster: fake API server + local kubelet + the C++ operator + bin/e2e."""
    from k8s_amd.fakeapi.cluster import LocalCluster

    t0 = time.time()
    with LocalCluster(gpus=[]) as c:
        cmd = [os.path.join(REPO, "bin", "e2e"), "--image", "k8s-amd/tf_sample:rocm7", "--master", c.url,
               "--timeout", str(int(a.timeout)), "--num_jobs", str(a.num_jobs)]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=a.timeout + 60)
        print(p.stdout, end="")
    ok = p.returncode == 0
    if a.junit:
        create_junit_xml_file([TestCase("deploy-local", "e2e", time.time() - t0, None if ok else p.stdout[-2000:])],
                              a.junit)
    return 0 if ok else 1


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dryrun", action="store_true", help="print the commands, run nothing")
    ap.add_argument("--context", default="", help="kubectl / helm context")
    ap.add_argument("--namespace", default="default")
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--junit", default="")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("setup")
    s.add_argument("--image", default="k8s-amd/tf_operator:latest")
    s.add_argument("--chart", default=CHART)
    s.add_argument("--min-gpus", type=int, default=1, help="wait until the nodes advertise this many amd.com/gpu")
    sub.add_parser("test")
    sub.add_parser("teardown")
    lo = sub.add_parser("local")
    lo.add_argument("--num_jobs", type=int, default=1)
    a = ap.parse_args(argv)
    r = Runner(a.dryrun)
    return {"setup": setup, "test": test, "teardown": teardown, "local": local}[a.cmd](a, r)


if __name__ == "__main__":
    sys.exit(main())
