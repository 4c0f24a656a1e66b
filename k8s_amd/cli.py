"""``tfjob`` -- the kubectl surface the reference's README uses, for TfJobs.

Reference usage (`/root/reference/README.md:14-28,364-457`):
``kubectl create -f examples/tf_job.yaml``, ``kubectl get tfjobs``,
``kubectl get -o yaml tfjobs $JOB``, ``kubectl delete tfjob $JOB``, plus the
Python client's ``wait_for_job`` (`/root/reference/py/tf_job_client.py:63-96`).

    python -m k8s_amd.cli create -f examples/tf_job.yaml
    python -m k8s_amd.cli get tfjobs [NAME] [-o yaml|json|wide]
    python -m k8s_amd.cli describe NAME        # replica statuses + pods
    python -m k8s_amd.cli wait NAME [--timeout S]   # exit 0 iff Succeeded
    python -m k8s_amd.cli delete tfjob NAME | delete -f FILE
    python -m k8s_amd.cli pods NAME            # the job's pods
    python -m k8s_amd.cli logs POD             # (local cluster) container output

The API server is ``--server`` or ``$K8S_AMD_APISERVER`` (a real cluster's
``kubectl proxy`` address, or ``python -m k8s_amd.fakeapi.cluster up``).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time
from typing import List

from k8s_amd.fakeapi.client import ApiClient, ApiError, create_tf_job, default_server, tfjobs_path, wait_for_job

_KINDS = ("tfjob", "tfjobs", "tfjob.tensorflow.org", "tfjobs.tensorflow.org")


def _load(path: str) -> List[dict]:
    from k8s_amd.fakeapi.cluster import load_manifests

    return load_manifests(path)


def _yaml(obj) -> str:
    import yaml

    return yaml.safe_dump(obj, default_flow_style=False, sort_keys=False)


def _age(ts: str) -> str:
    try:
        t = datetime.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc)
    except (TypeError, ValueError):
        return "<unknown>"
    s = int((datetime.datetime.now(datetime.timezone.utc) - t).total_seconds())
    return "%ds" % s if s < 120 else ("%dm" % (s // 60) if s < 7200 else "%dh" % (s // 3600))


def _table(rows, out):
    if not rows:
        return
    w = [max(len(str(r[i])) for r in rows) for i in range(len(rows[0]))]
    for r in rows:
        out.write("   ".join(str(c).ljust(w[i]) for i, c in enumerate(r)).rstrip() + "\n")


def _replica_summary(job) -> str:
    parts = []
    for rs in (job.get("status") or {}).get("replicaStatuses") or []:
        states = rs.get("ReplicasStates") or rs.get("replicasStates") or {}
        parts.append("%s:%s" % (rs.get("tf_replica_type", "?"),
                                ",".join("%s=%s" % (k, v) for k, v in sorted(states.items())) or rs.get("state", "")))
    return " ".join(parts)


def cmd_create(c: ApiClient, a, out) -> int:
    rc = 0
    for d in _load(a.filename):
        d.setdefault("metadata", {}).setdefault("namespace", a.namespace)
        try:
            create_tf_job(c, d)
            out.write('tfjob "%s" created\n' % d["metadata"].get("name"))
        except ApiError as e:
            sys.stderr.write("Error from server (%s): %s\n" % (e.reason or e.code, e))
            rc = 1
    return rc


def cmd_get(c: ApiClient, a, out) -> int:
    if a.kind not in _KINDS:
        sys.stderr.write('error: the server doesn\'t have a resource type "%s"\n' % a.kind)
        return 1
    ns = None if a.all_namespaces else a.namespace
    try:
        if a.name:
            items = [c.get(tfjobs_path(ns or a.namespace, a.name))]
        else:
            items = c.get(tfjobs_path(ns))["items"]
    except ApiError as e:
        sys.stderr.write("Error from server (%s): %s\n" % (e.reason or e.code, e))
        return 1
    if a.output in ("yaml", "json"):
        obj = items[0] if a.name else {"apiVersion": "v1", "kind": "List", "items": items}
        out.write(_yaml(obj) if a.output == "yaml" else json.dumps(obj, indent=2) + "\n")
        return 0
    hdr = ["NAME", "PHASE", "STATE", "RUNTIME-ID", "AGE"]
    if a.all_namespaces:
        hdr = ["NAMESPACE"] + hdr
    if a.output == "wide":
        hdr += ["REPLICAS"]
    rows = [hdr]
    for j in items:
        md, st, sp = j.get("metadata", {}), j.get("status") or {}, j.get("spec") or {}
        r = [md.get("name"), st.get("phase", ""), st.get("state", ""), sp.get("RuntimeId", sp.get("runtimeId", "")),
             _age(md.get("creationTimestamp"))]
        if a.all_namespaces:
            r = [md.get("namespace")] + r
        if a.output == "wide":
            r.append(_replica_summary(j))
        rows.append(r)
    if len(rows) == 1:
        sys.stderr.write("No resources found.\n")
        return 0
    _table(rows, out)
    return 0


def _pods(c: ApiClient, ns, name):
    return c.get("/api/v1/namespaces/%s/pods?labelSelector=tf_job_name=%s" % (ns, name))["items"]


def cmd_pods(c: ApiClient, a, out) -> int:
    rows = [["NAME", "STATUS", "RESTARTS", "JOB_TYPE", "TASK_INDEX"]]
    for p in _pods(c, a.namespace, a.name):
        st = p.get("status") or {}
        cs = (st.get("containerStatuses") or [{}])[0]
        lab = p["metadata"].get("labels", {})
        rows.append([p["metadata"]["name"], st.get("phase", ""), cs.get("restartCount", 0), lab.get("job_type", ""),
                     lab.get("task_index", "")])
    _table(rows, out)
    return 0


def cmd_describe(c: ApiClient, a, out) -> int:
    try:
        j = c.get(tfjobs_path(a.namespace, a.name))
    except ApiError as e:
        sys.stderr.write("Error from server (%s): %s\n" % (e.reason or e.code, e))
        return 1
    md, st, sp = j["metadata"], j.get("status") or {}, j.get("spec") or {}
    out.write("Name:        %s\nNamespace:   %s\nRuntimeId:   %s\nPhase:       %s\nState:       %s\n"
              "Reason:      %s\nCreated:     %s\n" % (md.get("name"), md.get("namespace"), sp.get("RuntimeId", ""),
                                                      st.get("phase", ""), st.get("state", ""), st.get("reason", ""),
                                                      md.get("creationTimestamp", "")))
    out.write("Replicas:\n")
    for r in sp.get("replicaSpecs") or []:
        out.write("  %-8s replicas=%s port=%s%s\n" % (r.get("tfReplicaType"), r.get("replicas"), r.get("tfPort"),
                                                     " (default PS)" if r.get("IsDefaultPS") else ""))
    out.write("Replica statuses:\n")
    for rs in st.get("replicaStatuses") or []:
        out.write("  %-8s %-10s %s\n" % (rs.get("tf_replica_type"), rs.get("state"),
                                         json.dumps(rs.get("ReplicasStates") or {})))
    out.write("Pods:\n")
    for p in _pods(c, a.namespace, a.name):
        out.write("  %s  %s\n" % (p["metadata"]["name"], (p.get("status") or {}).get("phase", "")))
    out.write("Events:\n")
    evs = job_events(c, a.namespace, a.name, md.get("uid"))
    if not evs:
        out.write("  <none>\n")
    else:
        out.write("  %-8s %-10s %-6s %-24s %s\n" % ("Type", "Reason", "Count", "Last seen", "Message"))
        for e in evs:
            out.write("  %-8s %-10s %-6s %-24s %s\n" % (e.get("type", ""), e.get("reason", ""), e.get("count", 1),
                                                        e.get("lastTimestamp", ""), e.get("message", "")))
    return 0


def job_events(c: ApiClient, namespace: str, name: str, uid=None):
    """core/v1 Events whose involvedObject is this TfJob (the operator's Created / Running / Succeeded / Failed),
    oldest first; with ``uid`` only those of that incarnation of the name."""
    try:
        items = c.get("/api/v1/namespaces/%s/events" % namespace).get("items") or []
    except ApiError:
        return []
    out = []
    for e in items:
        io = e.get("involvedObject") or {}
        if io.get("kind") == "TfJob" and io.get("name") == name and (not uid or io.get("uid") in (None, uid)):
            out.append(e)
    out.sort(key=lambda e: (e.get("firstTimestamp") or "", int((e.get("metadata") or {}).get("resourceVersion") or 0)))
    return out


def cmd_wait(c: ApiClient, a, out) -> int:
    try:
        j = wait_for_job(c, a.namespace, a.name, timeout=a.timeout, polling_interval=a.interval)
    except TimeoutError as e:
        sys.stderr.write("%s\n" % e)
        return 2
    st = j.get("status") or {}
    out.write("tfjob %s: phase=%s state=%s\n" % (a.name, st.get("phase"), st.get("state")))
    return 0 if st.get("state") == "Succeeded" else 1


def cmd_delete(c: ApiClient, a, out) -> int:
    targets = []
    if a.filename:
        for d in _load(a.filename):
            targets.append((d.get("metadata", {}).get("namespace", a.namespace), d["metadata"]["name"]))
    else:
        if a.kind not in _KINDS or not a.name:
            sys.stderr.write("usage: delete tfjob NAME | delete -f FILE\n")
            return 1
        targets.append((a.namespace, a.name))
    rc = 0
    for ns, name in targets:
        try:
            c.delete(tfjobs_path(ns, name))
            out.write('tfjob "%s" deleted\n' % name)
        except ApiError as e:
            sys.stderr.write("Error from server (%s): %s\n" % (e.reason or e.code, e))
            rc = 1
    return rc


def cmd_logs(c: ApiClient, a, out) -> int:
    from k8s_amd.fakeapi.kubelet import LOG_ANNOTATION

    try:
        p = c.get("/api/v1/namespaces/%s/pods/%s" % (a.namespace, a.pod))
    except ApiError as e:
        sys.stderr.write("Error from server (%s): %s\n" % (e.reason or e.code, e))
        return 1
    path = (p["metadata"].get("annotations") or {}).get(LOG_ANNOTATION)
    if not path or not os.path.exists(path):
        sys.stderr.write("no local log for pod %s (logs are only reachable on the local cluster)\n" % a.pod)
        return 1
    last = 0
    while True:
        with open(path) as f:
            f.seek(last)
            chunk = f.read()
            last = f.tell()
        out.write(chunk)
        out.flush()
        if not a.follow:
            return 0
        phase = (c.get("/api/v1/namespaces/%s/pods/%s" % (a.namespace, a.pod)).get("status") or {}).get("phase")
        if phase in ("Succeeded", "Failed"):
            return 0
        time.sleep(0.5)


def build_parser():
    ap = argparse.ArgumentParser(prog="tfjob", description="TfJob command line (kubectl-style)")
    ap.add_argument("--server", "-s", default=None, help="API server URL (default $K8S_AMD_APISERVER or %s)"
                    % "http://127.0.0.1:8080")
    ap.add_argument("--namespace", "-n", default="default")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("create")
    p.add_argument("-f", "--filename", required=True)
    p = sub.add_parser("get")
    p.add_argument("kind", nargs="?", default="tfjobs")
    p.add_argument("name", nargs="?")
    p.add_argument("-o", "--output", choices=["yaml", "json", "wide"], default=None)
    p.add_argument("--all-namespaces", "-A", action="store_true")
    p = sub.add_parser("describe")
    p.add_argument("name")
    p = sub.add_parser("wait")
    p.add_argument("name")
    p.add_argument("--timeout", type=float, default=300.0)
    p.add_argument("--interval", type=float, default=1.0)
    p = sub.add_parser("delete")
    p.add_argument("kind", nargs="?", default="tfjob")
    p.add_argument("name", nargs="?")
    p.add_argument("-f", "--filename")
    p = sub.add_parser("pods")
    p.add_argument("name")
    p = sub.add_parser("logs")
    p.add_argument("pod")
    p.add_argument("-f", "--follow", action="store_true")
    return ap


def main(argv=None, out=None) -> int:
    a = build_parser().parse_args(argv)
    out = out or sys.stdout
    c = ApiClient(a.server or default_server())
    fn = {"create": cmd_create, "get": cmd_get, "describe": cmd_describe, "wait": cmd_wait, "delete": cmd_delete,
          "pods": cmd_pods, "logs": cmd_logs}[a.cmd]
    try:
        return fn(c, a, out)
    except OSError as e:
        sys.stderr.write("The connection to the server %s was refused: %s\n" % (c.server, e))
        return 1


if __name__ == "__main__":
    sys.exit(main())
