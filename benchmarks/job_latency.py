#!/usr/bin/env python3
"""BASELINE.json's second metric: TfJob create -> step 0 latency.

Brings up the one-box cluster (fake API server + local kubelet + the C++
``tf_operator``), submits a single-MASTER ResNet-50 TfJob asking for
``amd.com/gpu: 1`` (CPU fallback: ``resnet_tiny`` without a GPU), and
measures from just before the create POST to the trainer's ``step0`` record
(first optimizer step finished, loss synced to host). Also reports the split:
create -> trainer process start (operator reconcile + kubelet), the process's
interpreter start + imports, setup (model / optimizer / synthetic data on the
GPU) and the first step itself, and the job's total time to ``Succeeded``.

    python benchmarks/job_latency.py [--runs 3] [--steps 5]

Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_amd.fakeapi.cluster import LocalCluster  # noqa: E402


def _manifest(name, model, steps, logdir, gpu, log_every=1):
    c = {"image": "k8s-amd/trainer:rocm7-gfx950", "name": "tensorflow",
         "args": ["--model", model, "--steps", str(steps), "--log-every", str(log_every), "--logdir", logdir]}
    if gpu:
        c["resources"] = {"limits": {"amd.com/gpu": 1}}
    else:
        c["args"] += ["--device", "cpu"]
    return {"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob", "metadata": {"name": name},
            "spec": {"replicaSpecs": [{"tfReplicaType": "MASTER", "replicas": 1,
                                       "template": {"spec": {"containers": [c], "restartPolicy": "OnFailure"}}}]}}


def _events(path, all_steps=None):
    out = {}
    if os.path.exists(path):
        for line in open(path):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            out.setdefault(r.get("event"), r)
            if all_steps is not None and r.get("event") == "step":
                all_steps.append(r)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default=None)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--log-every", type=int, default=1,
                    help="trainer log interval; with --steps 30 --log-every 10 the record also carries the TfJob "
                         "path's steady-state throughput (the trainer's per-interval rate, default batch = bench's)")
    a = ap.parse_args(argv)
    try:
        import torch

        gpu = torch.cuda.device_count() > 0  # does not initialise HIP in this process
    except ImportError:
        gpu = False
    model = a.model or ("resnet50" if gpu else "resnet_tiny")
    work = tempfile.mkdtemp(prefix="k8s_amd_latency_")
    results = []
    with LocalCluster(gpus=[0] if gpu else []) as c:
        for i in range(a.runs):
            name = "latency-%d" % i
            logdir = os.path.join(work, name)
            t0 = time.time()
            c.create(_manifest(name, model, a.steps, logdir, gpu, a.log_every))
            job = c.wait(name, timeout=a.timeout)
            t_done = time.time()
            steps_ev = []
            ev = _events(os.path.join(logdir, "metrics.jsonl"), steps_ev)
            state = job.get("status", {}).get("state")
            if state != "Succeeded" or "step0" not in ev:
                print(json.dumps({"error": "job %s ended %s" % (name, state), "events": list(ev)}), flush=True)
                return 1
            start = ev["start"]["start_time"]
            results.append({"create_to_step0_s": ev["step0"]["time"] - t0, "create_to_trainer_start_s": start - t0,
                            "trainer_start_to_step0_s": ev["step0"]["time"] - start,
                            "create_to_succeeded_s": t_done - t0})
            proc = ev["start"].get("process_start_time")
            if proc:  # operator + kubelet, then interpreter start + imports (torch, the extension)
                results[-1]["create_to_process_start_s"] = proc - t0
                results[-1]["process_imports_s"] = start - proc
            for k in ("setup_s", "first_step_s"):  # model / optimizer / data build, then step 0 itself
                if k in ev["step0"]:
                    results[-1]["step0_" + k] = ev["step0"][k]
            rates = [v for r in steps_ev for k, v in r.items() if k.endswith("_per_sec")]
            if len(rates) >= 2:  # the first interval includes the warm-up steps after step 0
                results[-1]["tfjob_steady_rate"] = statistics.median(rates[1:])
            c.delete(name)
            print(json.dumps({"run": i, **{k: round(v, 3) for k, v in results[-1].items()}}), file=sys.stderr,
                  flush=True)
    med = {k: round(statistics.median(r[k] for r in results if k in r), 3) for k in results[0]}
    print(json.dumps({"metric": "TfJob create -> step0 latency", "value": med["create_to_step0_s"], "unit": "s",
                      "higher_is_better": False, "runs": a.runs, "model": model, "gpu": gpu, "median": med,
                      "all": results}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
