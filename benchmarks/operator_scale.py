#!/usr/bin/env python3
"""Operator scale run at the reference's design target: O(100) concurrent TfJobs.

`/root/reference/tf_job_design_doc.md:24` sizes the operator for about a hundred concurrent TfJobs; the reference
reconciles each with its own goroutine, one Job GET + one Pod LIST per replica index every 8 s
(`/root/reference/pkg/trainer/replicas.go:415-492`). This drives the C++ operator with N TfJobs of
1 MASTER + 1 WORKER on the one-box cluster (in-memory API server + local kubelet; the containers are `sleep`s) and
measures, from the API server's side (requests counted by User-Agent):

* steady-state operator API requests per second, total and per job, while every job is Running;
* create -> every job Running, and release -> Succeeded per job: the MASTERs wait for a marker file, created after
  the steady-state window; the time from it to each TfJob's Succeeded status is the operator's detection latency
  (pod exit -> kubelet status -> operator -> TfJob status);
* the operator's thread count;
* cleanup: every TfJob deleted, every child Job / Pod / Service gone.

Run once with the shared watch caches (``-informers=true``, the default) and once with the reference's polling
reads (``-informers=false``) to compare the API load:

    python benchmarks/operator_scale.py --jobs 100 --informers both --out profiles/r05_operator_scale.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_amd.fakeapi.cluster import LocalCluster  # noqa: E402
from k8s_amd.fakeapi.client import tfjobs_path  # noqa: E402

OP_UA = "tf_operator-amd/"


def _job(name, marker):
    def rep(t, cmd):
        return {"replicas": 1, "tfReplicaType": t, "template": {"spec": {
            "containers": [{"name": "tensorflow", "image": "busybox", "command": ["sh", "-c", cmd]}],
            "restartPolicy": "OnFailure"}}}
    return {"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicaSpecs": [rep("MASTER", "while [ ! -f %s ]; do sleep 0.5; done" % marker),
                                      rep("WORKER", "exec sleep 600")]}}


def _threads(pid):
    try:
        for line in open("/proc/%d/status" % pid):
            if line.startswith("Threads:"):
                return int(line.split()[1])
    except OSError:
        pass
    return -1


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))] if xs else None


def run(jobs=100, informers=True, window=5.0, interval="2s", timeout=240.0, log=print):
    t_begin = time.time()
    args = ["-informers=%s" % ("true" if informers else "false")]
    with LocalCluster(reconcile_interval=interval, operator_args=args) as c:
        marker = os.path.join(c.log_dir, "release")
        names = ["scale-%03d" % i for i in range(jobs)]
        created = {}
        for n in names:
            c.create(_job(n, marker))
            created[n] = time.time()
        t_created = time.time()
        # every job Running with both pods up
        done, running_at = {}, None
        phases = {}
        end = time.time() + timeout
        while time.time() < end:
            items = c.client.get(tfjobs_path("default"))["items"]
            phases = {j["metadata"]["name"]: (j.get("status") or {}) for j in items}
            now = time.time()
            for n, st in phases.items():
                if st.get("phase") == "Done" and n not in done:
                    done[n] = (now, st.get("state"))
            n_running = sum(1 for st in phases.values() if st.get("phase") in ("Running", "Done"))
            pods = [p for p in c.pods() if (p.get("status") or {}).get("phase") == "Running"]
            if running_at is None and n_running == jobs and len(pods) >= 2 * jobs:
                running_at = now
                break
            time.sleep(0.25)
        if running_at is None:
            raise TimeoutError("only %d of %d jobs Running" % (sum(1 for st in phases.values()
                                                                  if st.get("phase") == "Running"), jobs))
        # steady state: every job Running, nothing changing -> what the operator asks the API server per second
        time.sleep(1.0)
        r0, t0 = c.server.request_counts(OP_UA), time.time()
        threads = _threads(c.op_proc.pid)
        time.sleep(window)
        r1, t1 = c.server.request_counts(OP_UA), time.time()
        steady = {k: r1.get(k, 0) - r0.get(k, 0) for k in set(r0) | set(r1)}
        qps = sum(steady.values()) / (t1 - t0)
        log("steady: %d jobs, informers=%s: %.1f req/s (%s), %d operator threads"
            % (jobs, informers, qps, steady, threads))
        # release every MASTER (exit 0) and wait for every job to finish
        open(marker, "w").close()
        t_release = time.time()
        while time.time() < end and len(done) < jobs:
            items = c.client.get(tfjobs_path("default"))["items"]
            now = time.time()
            for j in items:
                st = j.get("status") or {}
                n = j["metadata"]["name"]
                if st.get("phase") == "Done" and n not in done:
                    done[n] = (now, st.get("state"))
            time.sleep(0.2)
        states = {}
        for n, (_, s) in done.items():
            states[s] = states.get(s, 0) + 1
        lat = [done[n][0] - t_release for n in done]
        # cleanup: delete every TfJob; the operator deletes the children, ownerReferences GC the rest
        t_del = time.time()
        for n in names:
            c.delete(n)
        left = None
        while time.time() < t_del + 120:
            left = {p: len(c.client.get(p)["items"]) for p in (
                "/apis/batch/v1/namespaces/default/jobs", "/api/v1/namespaces/default/pods",
                "/api/v1/namespaces/default/services", tfjobs_path("default"))}
            if not any(left.values()):
                break
            time.sleep(0.25)
        cleanup_s = time.time() - t_del
        total = c.server.request_counts(OP_UA)
        op_log = c.operator_log()
    return {
        "jobs": jobs, "informers": informers, "reconcile_interval": interval,
        "create_all_s": round(t_created - t_begin, 3),
        "all_running_s": round(running_at - t_created, 3),
        "steady_window_s": round(t1 - t0, 3), "steady_requests": steady,
        "steady_qps": round(qps, 2), "steady_qps_per_job": round(qps / jobs, 4),
        "operator_threads": threads,
        "states": states,
        "release_to_succeeded_s": {"p50": round(_pct(lat, 0.5), 3), "p90": round(_pct(lat, 0.9), 3),
                                   "max": round(max(lat), 3)} if lat else None,
        "cleanup_s": round(cleanup_s, 3), "left_after_cleanup": left,
        "operator_requests_total": total,
        "operator_errors": sum(1 for line in op_log.splitlines() if " E" in line[:3] or "ERROR" in line),
        "wall_s": round(time.time() - t_begin, 3),
    }


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--jobs", type=int, default=100)
    ap.add_argument("--informers", choices=["true", "false", "both"], default="both")
    ap.add_argument("--window", type=float, default=5.0)
    ap.add_argument("--interval", default="2s", help="operator -reconcile-interval (reference: 8s)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    modes = {"true": [True], "false": [False], "both": [False, True]}[a.informers]
    out = [run(a.jobs, m, a.window, a.interval, log=lambda s: print(s, file=sys.stderr)) for m in modes]
    text = "\n".join(json.dumps(r) for r in out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
