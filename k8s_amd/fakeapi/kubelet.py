"""Local kubelet + batch-Job controller: runs TfJob replicas as host processes.

Stands in for the parts of Kubernetes below the API server (SURVEY.md §4,
implication 2) so a TfJob goes create -> pods -> train -> Succeeded on one
box, CPU or MI355X:

* batch Job controller: one Pod per Job (completions = parallelism = 1),
  pods labelled from the template and owned by the Job; Job.status.succeeded
  on exit 0, Failed after ``backoffLimit`` (default 6) failures.
* kubelet: runs the container named in the template as a subprocess with its
  ``env`` (TF_CONFIG), ``restartPolicy: OnFailure`` restarts in place and
  records ``lastState.terminated`` (the reference's retry state machine reads
  exactly that: pkg/trainer/replicas.go:383-409), ``Never`` fails the pod.
* devices: ``resources.limits["amd.com/gpu"] = n`` reserves n GPU ids from the
  node pool and exports ``HIP_VISIBLE_DEVICES`` to the container.
* networking: every Service gets a 127.0.0.1 port; the map is exported as
  ``K8S_AMD_SERVICE_MAP`` so workloads resolve TF_CONFIG host:port pairs
  (cluster DNS stand-in, see ``k8s_amd.parallel.dist``).
* volumes: configMap volumes are materialised in a scratch dir; command/args
  paths under a mountPath are rewritten to it; hostPath mounts likewise.
* Deployments: a TensorBoard Deployment (container command ``tensorboard --logdir ...``) runs the
  ``k8s_amd.tools.tensorboard`` stand-in on the 127.0.0.1 port of the Service that selects it, with the
  logdir rewritten through its volumes; other Deployments are marked available without a process.
* fault injection: ``kill_pod(name, exit_code)`` ends a container with a
  chosen exit code.
"""
from __future__ import annotations

import json
import os
import shlex
import signal
import subprocess
import sys
import tempfile
import threading
import time
import uuid
from typing import Dict, List, Optional

from k8s_amd.fakeapi.client import ApiClient
from k8s_amd.fakeapi.store import now_rfc3339

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# image -> default entrypoint when a container has no command (the "image" is our package)
DEFAULT_ENTRYPOINTS = [
    ("tf_sample", [sys.executable, "-m", "k8s_amd.models.smoke"]),
    ("k8s-amd/trainer", [sys.executable, "-m", "k8s_amd.trainer"]),
    ("tensorflow/tensorflow", [sys.executable, "-m", "k8s_amd.models.smoke"]),
]


LOG_ANNOTATION = "k8s-amd.io/log-path"


class _Container:
    def __init__(self, pod_name, proc, log_path):
        self.pod = pod_name
        self.proc = proc
        self.log_path = log_path
        self.forced_exit: Optional[int] = None


class LocalKubelet:
    def __init__(self, client: ApiClient, namespace: Optional[str] = None, gpus: Optional[List[int]] = None,
                 log_dir: Optional[str] = None, poll: float = 0.2, extra_env: Optional[Dict[str, str]] = None,
                 max_restarts: int = 6):
        self.api = client
        self.ns = namespace
        self.gpu_pool = list(gpus or [])
        self.gpu_used: Dict[str, List[int]] = {}
        self.gpu_history: Dict[str, List[int]] = {}  # every allocation ever made (tests)
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="k8s_amd_kubelet_")
        os.makedirs(self.log_dir, exist_ok=True)
        self.poll = poll
        self.extra_env = dict(extra_env or {})
        self.max_restarts = max_restarts
        self.running: Dict[str, _Container] = {}  # pod name -> container
        self.deploy_procs: Dict[str, subprocess.Popen] = {}  # ns/deployment -> TensorBoard stand-in
        self.pod_meta: Dict[str, dict] = {}  # pod name -> {"job":..., "ns":..., "restarts":..}
        self.service_ports: Dict[str, int] = {}
        self._published: Dict[str, str] = {}
        self.failures: Dict[str, int] = {}  # job -> failed pods
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self.events: List[dict] = []

    # ------------------------------------------------------------------ lifecycle
    def start(self):
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=10)
        for c in list(self.running.values()):
            self._kill(c.proc)
        for p in list(self.deploy_procs.values()):
            self._kill(p)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    # ------------------------------------------------------------------ helpers
    def _path(self, ns, plural, name=None, group=None):
        base = "/api/v1" if group is None else "/apis/" + group
        p = "%s/namespaces/%s/%s" % (base, ns, plural)
        return p + ("/" + name if name else "")

    def _namespaces(self):
        if self.ns:
            return [self.ns]
        seen = set()
        for it in self.api.get("/apis/batch/v1/jobs").get("items", []):
            seen.add(it["metadata"].get("namespace", "default"))
        return sorted(seen) or ["default"]

    @staticmethod
    def _kill(proc, sig=signal.SIGTERM):
        try:
            os.killpg(proc.pid, sig)
        except (ProcessLookupError, PermissionError):
            pass

    def kill_pod(self, pod_name: str, exit_code: int = 137):
        """Fault injection: terminate a running container; its status reports `exit_code`."""
        c = self.running.get(pod_name)
        if c:
            c.forced_exit = exit_code
            self._kill(c.proc, signal.SIGKILL)

    def pod_log(self, pod_name: str) -> str:
        for c in [self.running.get(pod_name)]:
            if c:
                return open(c.log_path).read()
        p = os.path.join(self.log_dir, pod_name + ".log")
        return open(p).read() if os.path.exists(p) else ""

    # ------------------------------------------------------------------ services / volumes / env
    def _service_port(self) -> int:
        """A free 127.0.0.1 port not handed out to another Service (the Service's ``tfPort`` stand-in; the
        trainer's rendezvous listens on the master Service's own port, parallel/dist.py)."""
        import socket

        taken = set(self.service_ports.values())
        for _ in range(64):
            a = socket.socket()
            try:
                a.bind(("127.0.0.1", 0))
                port = a.getsockname()[1]
            finally:
                a.close()
            if port not in taken:
                return port
        raise RuntimeError("no free port for a Service")

    def _service_map_file(self, ns) -> str:
        return os.path.join(self.log_dir, "service-map-%s.json" % ns)

    def _publish_service_map(self, ns) -> Dict[str, str]:
        """Cluster DNS stand-in that stays current: the map is rewritten (atomically) on every sync, and pods
        resolve through the file, so a pod started before a peer's Service existed still finds the peer
        (the operator creates a replica's Job before the next replica's Service)."""
        m = self._service_map(ns)
        path = self._service_map_file(ns)
        data = json.dumps(m, sort_keys=True)
        if self._published.get(ns) != data:
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                f.write(data)
            os.replace(tmp, path)
            self._published[ns] = data
        return m

    def _service_map(self, ns) -> Dict[str, str]:
        out = {}
        for s in self.api.get(self._path(ns, "services")).get("items", []):
            name = s["metadata"]["name"]
            key = ns + "/" + name
            if key not in self.service_ports:
                self.service_ports[key] = self._service_port()
            out[name] = "127.0.0.1:%d" % self.service_ports[key]
            for port in s.get("spec", {}).get("ports", []):
                out["%s:%s" % (name, port.get("port"))] = "127.0.0.1:%d" % self.service_ports[key]
        return out

    def _materialise_volumes(self, ns, pod_name, spec, container) -> Dict[str, str]:
        """mountPath -> host dir."""
        vols = {v["name"]: v for v in spec.get("volumes") or []}
        mapping = {}
        for vm in container.get("volumeMounts") or []:
            v = vols.get(vm["name"])
            if v is None:
                continue
            if "configMap" in v:
                cm = self.api.get(self._path(ns, "configmaps", v["configMap"]["name"]))
                d = os.path.join(self.log_dir, "volumes", pod_name, vm["name"])
                os.makedirs(d, exist_ok=True)
                for fname, content in (cm.get("data") or {}).items():
                    with open(os.path.join(d, fname), "w") as f:
                        f.write(content)
                mapping[vm["mountPath"]] = d
            elif "hostPath" in v:
                mapping[vm["mountPath"]] = v["hostPath"]["path"]
            elif "emptyDir" in v:
                d = os.path.join(self.log_dir, "volumes", pod_name, vm["name"])
                os.makedirs(d, exist_ok=True)
                mapping[vm["mountPath"]] = d
        return mapping

    @staticmethod
    def _rewrite(arg: str, mounts: Dict[str, str]) -> str:
        for mp, host in sorted(mounts.items(), key=lambda kv: -len(kv[0])):
            if arg == mp or arg.startswith(mp.rstrip("/") + "/"):
                return host + arg[len(mp.rstrip("/")):]
        return arg

    def _command(self, container, mounts) -> List[str]:
        cmd = list(container.get("command") or [])
        args = list(container.get("args") or [])
        if not cmd:
            img = container.get("image", "")
            for pat, ep in DEFAULT_ENTRYPOINTS:
                if pat in img:
                    cmd = list(ep)
                    break
            if not cmd:
                cmd = [sys.executable, "-m", "k8s_amd.trainer"]
        full = [self._rewrite(a, mounts) for a in cmd + args]
        if full and full[0] in ("python", "python3"):
            full[0] = sys.executable
        return full

    def _alloc_gpus(self, pod_name, container) -> Optional[List[int]]:
        lim = (container.get("resources") or {}).get("limits") or {}
        n = int(lim.get("amd.com/gpu", 0) or 0)
        if n <= 0:
            return []
        free = [g for g in self.gpu_pool if not any(g in v for v in self.gpu_used.values())]
        if len(free) < n:
            return None  # unschedulable for now (Pending)
        self.gpu_used[pod_name] = free[:n]
        self.gpu_history[pod_name] = free[:n]
        return free[:n]

    # ------------------------------------------------------------------ reconcile loop
    def _loop(self):
        while not self._stop.is_set():
            try:
                for ns in self._namespaces():
                    self._sync_jobs(ns)
                    self._sync_deployments(ns)
                    self._publish_service_map(ns)
                self._reap()
            except Exception as e:  # keep the node alive; log for the tests
                import traceback

                self.events.append({"type": "error", "message": repr(e), "trace": traceback.format_exc(),
                                    "time": time.time()})
            self._stop.wait(self.poll)

    def _sync_deployments(self, ns):
        deps = self.api.get(self._path(ns, "deployments", group="apps/v1")).get("items", [])
        live = set()
        for d in deps:
            key = ns + "/" + d["metadata"]["name"]
            live.add(key)
            if self._is_tensorboard(d) and (key not in self.deploy_procs or self.deploy_procs[key].poll() is not None):
                if not self._start_tensorboard(ns, d, key):
                    continue  # its Service is not there yet: retried on the next sync
            want = d.get("spec", {}).get("replicas", 1)
            st = d.get("status") or {}
            if st.get("availableReplicas") != want:
                d["status"] = {"replicas": want, "availableReplicas": want, "readyReplicas": want}
                self.api.request("PUT", self._path(ns, "deployments", d["metadata"]["name"], "apps/v1"), d)
        for key in [k for k in self.deploy_procs if k.startswith(ns + "/") and k not in live]:
            self._kill(self.deploy_procs.pop(key))  # Deployment deleted (job deleted / garbage collected)

    @staticmethod
    def _tb_container(d):
        cs = (((d.get("spec") or {}).get("template") or {}).get("spec") or {}).get("containers") or []
        return next((c for c in cs if os.path.basename((c.get("command") or [""])[0]) == "tensorboard"), None)

    def _is_tensorboard(self, d) -> bool:
        return self._tb_container(d) is not None

    def _start_tensorboard(self, ns, d, key) -> bool:
        tmpl = d["spec"]["template"]
        labels = (tmpl.get("metadata") or {}).get("labels") or {}
        svc = None
        for s in self.api.get(self._path(ns, "services")).get("items", []):
            sel = (s.get("spec") or {}).get("selector") or {}
            if sel and all(labels.get(k) == v for k, v in sel.items()):
                svc = s["metadata"]["name"]
                break
        if svc is None:
            return False
        self._publish_service_map(ns)
        port = self.service_ports[ns + "/" + svc]
        c = self._tb_container(d)
        mounts = self._materialise_volumes(ns, d["metadata"]["name"], tmpl.get("spec") or {}, c)
        argv = list(c.get("command") or [])[1:] + list(c.get("args") or [])
        logdir = argv[argv.index("--logdir") + 1] if "--logdir" in argv else "."
        cmd = [sys.executable, "-m", "k8s_amd.tools.tensorboard", "--logdir", self._rewrite(logdir, mounts),
               "--host", "127.0.0.1", "--port", str(port)]
        env = dict(os.environ)
        env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
        log_path = os.path.join(self.log_dir, d["metadata"]["name"] + ".log")
        with open(log_path, "ab") as logf:
            logf.write(("$ %s\n" % " ".join(shlex.quote(x) for x in cmd)).encode())
            logf.flush()
            self.deploy_procs[key] = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, cwd=REPO,
                                                      start_new_session=True)
        return True

    def _sync_jobs(self, ns):
        jobs = self.api.get(self._path(ns, "jobs", group="batch/v1")).get("items", [])
        pods = self.api.get(self._path(ns, "pods")).get("items", [])
        pods_by_job: Dict[str, List[dict]] = {}
        for p in pods:
            jn = (p["metadata"].get("labels") or {}).get("job-name")
            if jn:
                pods_by_job.setdefault(jn, []).append(p)
        live_names = {p["metadata"]["name"] for p in pods}
        # pods deleted out from under us (chaos / GC): stop their processes
        for pod_name in list(self.running):
            if pod_name not in live_names and self.pod_meta.get(pod_name, {}).get("ns") == ns:
                c = self.running.pop(pod_name)
                self._kill(c.proc, signal.SIGKILL)
                self.gpu_used.pop(pod_name, None)
        for j in jobs:
            name = j["metadata"]["name"]
            st = j.get("status") or {}
            if st.get("succeeded", 0) >= 1 or any(c.get("type") == "Failed" for c in st.get("conditions") or []):
                continue
            active = [p for p in pods_by_job.get(name, []) if p.get("status", {}).get("phase") in
                      (None, "Pending", "Running")]
            if not active:
                self._create_pod(ns, j)

    def _create_pod(self, ns, job):
        tmpl = job["spec"]["template"]
        jname = job["metadata"]["name"]
        pod_name = "%s-%s" % (jname, uuid.uuid4().hex[:5])
        labels = dict((tmpl.get("metadata") or {}).get("labels") or {})
        labels["job-name"] = jname
        labels["controller-uid"] = job["metadata"].get("uid", "")
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": pod_name, "namespace": ns, "labels": labels,
                            "ownerReferences": [{"apiVersion": "batch/v1", "kind": "Job", "name": jname,
                                                 "uid": job["metadata"].get("uid"), "controller": True,
                                                 "blockOwnerDeletion": True}]},
               "spec": tmpl.get("spec", {}),
               "status": {"phase": "Pending"}}
        code, created = self.api.request("POST", self._path(ns, "pods"), pod)
        if code >= 300:
            return
        self.pod_meta[pod_name] = {"job": jname, "ns": ns, "restarts": 0}
        self._start_container(ns, created)

    def _start_container(self, ns, pod):
        pod_name = pod["metadata"]["name"]
        spec = pod.get("spec", {})
        containers = spec.get("containers") or []
        if not containers:
            return
        # run the "tensorflow" container (the one the operator reads status from); others are sidecars we skip
        c = next((x for x in containers if x.get("name") == "tensorflow"), containers[0])
        gpus = self._alloc_gpus(pod_name, c)
        if gpus is None:
            return  # stays Pending; retried on the next sync when pods exit
        mounts = self._materialise_volumes(ns, pod_name, spec, c)
        env = dict(os.environ)
        env.update(self.extra_env)
        env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
        for e in c.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
        env["K8S_AMD_SERVICE_MAP"] = json.dumps(self._publish_service_map(ns))
        env["K8S_AMD_SERVICE_MAP_FILE"] = self._service_map_file(ns)
        env["POD_NAME"], env["POD_NAMESPACE"] = pod_name, ns
        if gpus:
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
        elif "amd.com/gpu" not in ((c.get("resources") or {}).get("limits") or {}):
            env.setdefault("K8S_AMD_NO_GPU", "1" if not self.gpu_pool else env.get("K8S_AMD_NO_GPU", "0"))
        cmd = self._command(c, mounts)
        log_path = os.path.join(self.log_dir, pod_name + ".log")
        logf = open(log_path, "ab")
        logf.write(("$ %s\n" % " ".join(shlex.quote(x) for x in cmd)).encode())
        logf.flush()
        wd = c.get("workingDir")
        proc = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, cwd=wd or REPO,
                                start_new_session=True)
        logf.close()
        self.running[pod_name] = _Container(pod_name, proc, log_path)
        self._set_pod_status(ns, pod_name, phase="Running",
                             cstatus={"name": c.get("name", "tensorflow"),
                                      "state": {"running": {"startedAt": now_rfc3339()}},
                                      "restartCount": self.pod_meta[pod_name]["restarts"]})

    def _set_pod_status(self, ns, pod_name, phase, cstatus, last=None):
        code, pod = self.api.request("GET", self._path(ns, "pods", pod_name))
        if code != 200:
            return
        c = self.running.get(pod_name)
        if c is not None:  # where `tfjob logs` finds the container output (the local stand-in for /log)
            pod["metadata"].setdefault("annotations", {})[LOG_ANNOTATION] = c.log_path
        st = pod.setdefault("status", {})
        st["phase"] = phase
        st.setdefault("startTime", now_rfc3339())
        if last is not None:
            cstatus["lastState"] = last
        else:
            prev = next((x for x in st.get("containerStatuses") or [] if x.get("name") == cstatus["name"]), None)
            if prev and prev.get("lastState"):
                cstatus["lastState"] = prev["lastState"]
        st["containerStatuses"] = [cstatus]
        self.api.request("PUT", self._path(ns, "pods", pod_name), pod)

    def _reap(self):
        for pod_name, c in list(self.running.items()):
            rc = c.proc.poll()
            if rc is None:
                continue
            del self.running[pod_name]
            self.gpu_used.pop(pod_name, None)
            meta = self.pod_meta.get(pod_name, {})
            ns, jname = meta.get("ns", "default"), meta.get("job")
            exit_code = c.forced_exit if c.forced_exit is not None else (rc if rc >= 0 else 128 - rc)
            reason = "Completed" if exit_code == 0 else "Error"
            code, pod = self.api.request("GET", self._path(ns, "pods", pod_name))
            if code != 200:
                continue
            cname = (pod.get("status", {}).get("containerStatuses") or [{}])[0].get("name", "tensorflow")
            term = {"terminated": {"exitCode": exit_code, "reason": reason, "finishedAt": now_rfc3339()}}
            policy = pod.get("spec", {}).get("restartPolicy", "Always")
            if exit_code == 0:
                self._set_pod_status(ns, pod_name, "Succeeded", {"name": cname, "state": term,
                                                                  "restartCount": meta.get("restarts", 0)})
                self._job_done(ns, jname, succeeded=True)
            elif policy in ("OnFailure", "Always") and meta.get("restarts", 0) < self.max_restarts:
                meta["restarts"] = meta.get("restarts", 0) + 1
                self._set_pod_status(ns, pod_name, "Running",
                                     {"name": cname, "state": {"waiting": {"reason": "CrashLoopBackOff"}},
                                      "restartCount": meta["restarts"]}, last=term)
                self._start_container(ns, pod)
            else:
                self._set_pod_status(ns, pod_name, "Failed", {"name": cname, "state": term,
                                                               "restartCount": meta.get("restarts", 0)})
                self.failures[jname] = self.failures.get(jname, 0) + 1
                if self.failures[jname] > self.max_restarts or policy in ("OnFailure", "Always"):
                    self._job_done(ns, jname, succeeded=False)

    def _job_done(self, ns, jname, succeeded):
        code, job = self.api.request("GET", self._path(ns, "jobs", jname, "batch/v1"))
        if code != 200:
            return
        st = job.setdefault("status", {})
        if succeeded:
            st["succeeded"] = 1
            st["conditions"] = [{"type": "Complete", "status": "True", "lastTransitionTime": now_rfc3339()}]
        else:
            st["failed"] = st.get("failed", 0) + 1
            st["conditions"] = [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                 "lastTransitionTime": now_rfc3339()}]
        self.api.request("PUT", self._path(ns, "jobs", jname, "batch/v1"), job)
