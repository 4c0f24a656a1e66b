#!/usr/bin/env python3
"""End-to-end walkthrough: train a CIFAR-10-shaped ResNet as a TfJob and watch it in TensorBoard.

The reference's GKE notebook (`/root/reference/examples/gke/TF on GKE.ipynb`) deploys the operator, submits a
CIFAR-10 ResNet TfJob with a TensorBoard section, opens TensorBoard on the job's logDir and polls the job until
it is Done. This is the same flow on one box, with every piece real:

1. the one-box cluster: in-memory API server, local kubelet and the C++ ``tf_operator`` (``k8s_amd.fakeapi``);
2. a TfJob (MASTER, ``resnet_tiny`` = ResNet for 32x32x3 / 10 classes, synthetic CIFAR-shaped data -- no dataset
   download here) whose ``tensorboard.logDir`` is where the trainer writes ``events.out.tfevents.*``;
3. the operator's TensorBoard Deployment + Service (port 80 -> 6006), served on this box by
   ``k8s_amd.tools.tensorboard`` (TensorBoard's scalar REST API over the same event files);
4. the job polled to ``phase: Done``, then the loss curve read back through TensorBoard's HTTP API.

    python examples/walkthrough_cifar10_tensorboard.py [--steps 100] [--gpus 0]

Prints a JSON summary (job state, TensorBoard URL, runs/tags, the loss series) and exits 0 on success.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_amd.fakeapi.cluster import LocalCluster  # noqa: E402


def manifest(name: str, logdir: str, steps: int, gpu: bool) -> dict:
    container = {"name": "tensorflow", "image": "k8s-amd/trainer:rocm7-gfx950",
                 "args": ["--model", "resnet_tiny", "--steps", str(steps), "--log-every", "5", "--logdir", logdir],
                 "volumeMounts": [{"name": "logs", "mountPath": logdir}]}
    if gpu:
        container["resources"] = {"limits": {"amd.com/gpu": 1}}
    else:
        container["args"] += ["--device", "cpu"]
    vol = [{"name": "logs", "hostPath": {"path": logdir}}]
    return {"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob", "metadata": {"name": name},
            "spec": {"tensorboard": {"logDir": logdir, "serviceType": "ClusterIP", "volumes": vol,
                                     "volumeMounts": [{"name": "logs", "mountPath": logdir}]},
                     "replicaSpecs": [{"tfReplicaType": "MASTER", "replicas": 1, "tfPort": 2222,
                                       "template": {"spec": {"containers": [container], "volumes": vol,
                                                             "restartPolicy": "OnFailure"}}}]}}


def _get_json(url: str, timeout: float = 5.0):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return json.loads(r.read().decode())


def tensorboard_url(c: LocalCluster, job: str, ns: str = "default", timeout: float = 60.0) -> str:
    """Address of the job's TensorBoard Service (the local stand-in for cluster DNS / a port-forward)."""
    end = time.time() + timeout
    while time.time() < end:
        svcs = c.client.get("/api/v1/namespaces/%s/services?labelSelector=app=tensorboard" % ns).get("items", [])
        svcs = [s for s in svcs if s["metadata"]["name"].startswith(job)]
        if svcs:
            m = c.kubelet._service_map(ns)
            addr = m.get(svcs[0]["metadata"]["name"] + ":80")
            if addr:
                try:
                    urllib.request.urlopen("http://%s/data/runs" % addr, timeout=2).read()
                    return "http://" + addr
                except OSError:
                    pass
        time.sleep(0.25)
    raise TimeoutError("TensorBoard service of %s did not come up" % job)


def run(steps: int = 100, gpus=None, job: str = "cifar10-resnet", logdir: str = None, timeout: float = 900.0,
        verbose: bool = True) -> dict:
    logdir = logdir or tempfile.mkdtemp(prefix="k8s_amd_tb_")
    say = print if verbose else (lambda *a, **k: None)
    with LocalCluster(gpus=gpus or []) as c:
        c.create(manifest(job, logdir, steps, bool(gpus)))
        say("submitted TfJob %s (logDir %s)" % (job, logdir))
        tb = tensorboard_url(c, job)
        say("TensorBoard: %s" % tb)
        last, end = None, time.time() + timeout
        while time.time() < end:  # the notebook's polling cell: print every phase / state transition
            st = c.get(job).get("status", {})
            cur = (st.get("phase"), st.get("state"))
            if cur != last:
                say("  phase=%s state=%s" % cur)
                last = cur
            if st.get("phase") == "Done":
                break
            time.sleep(0.5)
        status = c.get(job).get("status", {})
        runs = _get_json(tb + "/data/runs")
        tags = _get_json(tb + "/data/plugin/scalars/tags")
        run_name = runs[0] if runs else "."
        loss = _get_json(tb + "/data/plugin/scalars/scalars?run=%s&tag=loss" % run_name) if runs else []
        index = urllib.request.urlopen(tb + "/", timeout=5).read().decode()
    out = {"job": job, "phase": status.get("phase"), "state": status.get("state"), "tensorboard": tb,
           "logdir": logdir, "runs": runs, "tags": {r: sorted(t) for r, t in tags.items()},
           "loss_points": len(loss), "loss_first": loss[0][2] if loss else None,
           "loss_last": loss[-1][2] if loss else None, "loss_steps": [p[1] for p in loss]}
    say(index.strip())
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--gpus", default="", help="GPU ids for the kubelet (empty: train on the CPU)")
    ap.add_argument("--timeout", type=float, default=900.0)
    a = ap.parse_args(argv)
    gpus = [int(x) for x in a.gpus.split(",") if x != ""]
    out = run(a.steps, gpus, timeout=a.timeout)
    print(json.dumps(out))
    return 0 if out["state"] == "Succeeded" and out["loss_points"] > 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
