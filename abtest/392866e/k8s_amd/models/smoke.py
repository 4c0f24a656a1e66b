"""tf_smoke equivalent: every task of the job executes a kernel.

Parity: /root/reference/examples/tf_sample/tf_sample/tf_smoke.py. The MASTER
reads TF_CONFIG, asks every ``/job:X/task:i`` (PS and WORKER tasks, and
itself) to run a 10x10 int32 elementwise multiply on its device, checks each
result and exits 0 -- which makes the MASTER replica Succeeded and the TfJob
Succeeded. PS and WORKER tasks serve until they are torn down (Q14: they never
exit on their own, exactly like the reference's ``server.join()``), unless
``--exit_after_master`` asks them to stop once the master shut them down.

    TF_CONFIG=... python -m k8s_amd.models.smoke
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

from k8s_amd.ps_server.grpc_tensorflow_server import call, parse_cluster_spec, serve  # noqa: F401


def run_master(cluster, task_index, shutdown_others=False, timeout=120.0, width=10, height=10):
    a = [[i * width + j for j in range(width)] for i in range(height)]
    b = [[2 + ((i + j) % 3) for j in range(width)] for i in range(height)]
    want = [[x * y for x, y in zip(ra, rb)] for ra, rb in zip(a, b)]
    results = {}
    for job in sorted(cluster):
        for i, addr in enumerate(cluster[job]):
            name = "/job:%s/task:%d" % (job, i)
            if job == "master" and i == task_index:
                results[name] = "local"
                continue
            deadline = time.time() + timeout
            while True:
                try:
                    r = call(addr, {"op": "multiply", "a": a, "b": b}, timeout=10)
                    break
                except OSError:
                    if time.time() > deadline:
                        print("task %s unreachable at %s" % (name, addr), flush=True)
                        return 1
                    time.sleep(0.2)
            if not r or not r.get("ok") or r["result"] != want:
                print("task %s returned a wrong result: %s" % (name, r), flush=True)
                return 1
            results[name] = r["device"]
            print("Result from %s (%s): ok" % (name, r["device"]), flush=True)
    if shutdown_others:
        for job in cluster:
            for i, addr in enumerate(cluster[job]):
                if not (job == "master" and i == task_index):
                    try:
                        call(addr, {"op": "shutdown"}, timeout=5)
                    except OSError:
                        pass
    print(json.dumps({"smoke": "ok", "tasks": results}), flush=True)
    return 0


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--exit_after_master", action="store_true",
                   help="master shuts the other tasks down at the end (so every replica exits 0)")
    a = p.parse_args(argv)
    tf_config = os.environ.get("TF_CONFIG", "{}")
    cfg = json.loads(tf_config)
    cluster = cfg.get("cluster", {})
    task = cfg.get("task", {})
    job, idx = task.get("type", "master"), int(task.get("index", 0))
    print("REPLICA_TYPE=%s REPLICA_INDEX=%d" % (job, idx), flush=True)
    if not cluster:
        print("TF_CONFIG has no cluster; nothing to do", flush=True)
        return 0
    if job == "master":
        # the master also serves, so other tasks may address it
        threading.Thread(target=serve, args=(cluster, job, idx), daemon=True).start()
        return run_master(cluster, idx, shutdown_others=a.exit_after_master)
    return serve(cluster, job, idx)


if __name__ == "__main__":
    sys.exit(main())
