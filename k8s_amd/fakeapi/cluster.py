"""One-box "cluster": fake API server + local kubelet + the C++ tf_operator.

    with LocalCluster(gpus=[0]) as c:          # or gpus=[] on a CPU box
        c.create("examples/tf_job.yaml")
        job = c.wait("example-job")

``python -m k8s_amd.fakeapi.cluster up --port 8080`` runs it in the
foreground so the ``tfjob`` CLI (or the ``bin/e2e`` helm-test binary) can be
pointed at it with ``K8S_AMD_APISERVER=http://127.0.0.1:8080``.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from typing import List, Optional

from k8s_amd.fakeapi.client import ApiClient, create_tf_job, tfjobs_path, wait_for_job
from k8s_amd.fakeapi.kubelet import LocalKubelet
from k8s_amd.fakeapi.server import FakeApiServer

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OPERATOR_BIN = os.path.join(REPO, "bin", "tf_operator")
PS_SERVER = os.path.join(REPO, "k8s_amd", "ps_server", "grpc_tensorflow_server.py")

# controller config for MI355X nodes: amd.com/gpu -> ROCm user space + device nodes (chart's cloud=amd preset)
AMD_CONTROLLER_CONFIG = {
    "grpcServerFilePath": PS_SERVER,
    "accelerators": {
        "amd.com/gpu": {
            "volumes": [{"name": "rocm", "mountPath": "/opt/rocm", "hostPath": "/opt/rocm"}],
            "envVars": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
                        {"name": "NCCL_MIN_NCHANNELS", "value": "16"}],
        }
    },
}


def load_manifests(path: str) -> List[dict]:
    """YAML (multi-document) or JSON manifests, parsed by the C++ YAML reader (fallback: PyYAML)."""
    text = open(path).read()
    if path.endswith(".json"):
        d = json.loads(text)
        return d if isinstance(d, list) else [d]
    try:
        from k8s_amd import _operator

        return json.loads(_operator.yaml_all_to_json(text))
    except ImportError:
        import yaml

        return [d for d in yaml.safe_load_all(text) if d]


class LocalCluster:
    def __init__(self, gpus: Optional[List[int]] = None, port: int = 0, reconcile_interval: str = "500ms",
                 operator_bin: str = OPERATOR_BIN, log_dir: Optional[str] = None, extra_env=None,
                 chaos_level: int = -1, operator_args: Optional[List[str]] = None):
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="k8s_amd_cluster_")
        self.server = FakeApiServer(port=port)
        self.client = ApiClient(self.server.url)
        self.kubelet = LocalKubelet(self.client, gpus=gpus or [], log_dir=os.path.join(self.log_dir, "pods"),
                                    extra_env=extra_env)
        self.operator_bin = operator_bin
        self.reconcile_interval = reconcile_interval
        self.chaos_level = chaos_level
        self.operator_args = list(operator_args or [])
        self.op_proc = None
        self.t_start = None

    @property
    def url(self):
        return self.server.url

    def start(self):
        self.server.start()
        self.kubelet.start()
        cfg_path = os.path.join(self.log_dir, "controller_config_file.yaml")
        with open(cfg_path, "w") as f:
            json.dump(AMD_CONTROLLER_CONFIG, f)  # JSON is valid YAML
        if not os.path.exists(self.operator_bin):
            raise FileNotFoundError("%s missing: run `python -m k8s_amd._build --only operator`" % self.operator_bin)
        env = dict(os.environ, MY_POD_NAMESPACE="default", MY_POD_NAME="tf-operator-local-0")
        self.op_log = open(os.path.join(self.log_dir, "tf_operator.log"), "wb")
        self.op_proc = subprocess.Popen(
            [self.operator_bin, "-controller_config_file", cfg_path, "-master", self.server.url,
             "-reconcile-interval", self.reconcile_interval, "-chaos-level", str(self.chaos_level),
             "-alsologtostderr", "-v=1"] + self.operator_args,
            env=env, stdout=self.op_log, stderr=subprocess.STDOUT)
        # wait for the operator to register the CRD
        end = time.time() + 30
        while time.time() < end:
            if self.client.exists("/apis/apiextensions.k8s.io/v1/customresourcedefinitions/tfjobs.tensorflow.org"):
                return self
            if self.op_proc.poll() is not None:
                raise RuntimeError("tf_operator exited early:\n" + self.operator_log())
            time.sleep(0.05)
        raise TimeoutError("operator did not register the CRD")

    def operator_log(self) -> str:
        p = os.path.join(self.log_dir, "tf_operator.log")
        return open(p).read() if os.path.exists(p) else ""

    def stop(self):
        if self.op_proc and self.op_proc.poll() is None:
            self.op_proc.terminate()
            try:
                self.op_proc.wait(10)
            except subprocess.TimeoutExpired:
                self.op_proc.kill()
        self.kubelet.stop()
        self.server.stop()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    # ------------------------------------------------------------------ user surface
    def create(self, manifest, namespace="default") -> List[dict]:
        docs = load_manifests(manifest) if isinstance(manifest, str) else [manifest]
        out = []
        for d in docs:
            d.setdefault("metadata", {}).setdefault("namespace", namespace)
            out.append(create_tf_job(self.client, d))
        return out

    def get(self, name, namespace="default") -> dict:
        return self.client.get(tfjobs_path(namespace, name))

    def wait(self, name, namespace="default", timeout=120.0) -> dict:
        return wait_for_job(self.client, namespace, name, timeout=timeout, polling_interval=0.2)

    def delete(self, name, namespace="default"):
        return self.client.delete(tfjobs_path(namespace, name))

    def pods(self, namespace="default", selector=""):
        q = "?labelSelector=" + selector if selector else ""
        return self.client.get("/api/v1/namespaces/%s/pods%s" % (namespace, q))["items"]


def main(argv=None):
    ap = argparse.ArgumentParser(description="one-box TfJob cluster (fake API server + kubelet + tf_operator)")
    ap.add_argument("cmd", choices=["up"])
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--gpus", default="", help="comma-separated GPU ids the kubelet may hand out")
    a = ap.parse_args(argv)
    gpus = [int(x) for x in a.gpus.split(",") if x != ""]
    with LocalCluster(gpus=gpus, port=a.port) as c:
        print("cluster up: K8S_AMD_APISERVER=%s (logs in %s)" % (c.url, c.log_dir), flush=True)
        try:
            while True:
                time.sleep(1)
        except KeyboardInterrupt:
            pass


if __name__ == "__main__":
    sys.exit(main())
