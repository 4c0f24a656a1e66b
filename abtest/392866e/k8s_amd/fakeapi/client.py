"""Minimal Kubernetes REST client (urllib + JSON) used by the CLI, the local
kubelet and the Python TfJob client.

Parity: /root/reference/py/tf_job_client.py (create_tf_job / wait_for_job)
and the REST paths of pkg/util/k8sutil/tf_job_client.go.
"""
from __future__ import annotations

import json
import os
import time
import urllib.error
import urllib.request
from typing import Iterator, Optional, Tuple

GROUP, VERSION, PLURAL = "tensorflow.org", "v1alpha1", "tfjobs"


def default_server() -> str:
    return os.environ.get("K8S_AMD_APISERVER", "http://127.0.0.1:8080")


class ApiError(Exception):
    def __init__(self, code, body):
        self.code = code
        self.body = body
        msg = body.get("message") if isinstance(body, dict) else str(body)
        super().__init__("HTTP %s: %s" % (code, msg))

    @property
    def reason(self):
        return self.body.get("reason") if isinstance(self.body, dict) else None


class ApiClient:
    def __init__(self, server: Optional[str] = None, timeout: float = 30.0):
        self.server = (server or default_server()).rstrip("/")
        self.timeout = timeout

    def request(self, method: str, path: str, body=None) -> Tuple[int, dict]:
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.server + path, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", "application/json")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                raw = r.read()
                return r.status, (json.loads(raw) if raw else {})
        except urllib.error.HTTPError as e:
            raw = e.read()
            try:
                return e.code, json.loads(raw)
            except ValueError:
                return e.code, {"message": raw.decode(errors="replace")}

    def _ok(self, method, path, body=None):
        code, out = self.request(method, path, body)
        if code >= 300:
            raise ApiError(code, out)
        return out

    def get(self, path):
        return self._ok("GET", path)

    def post(self, path, body):
        return self._ok("POST", path, body)

    def put(self, path, body):
        return self._ok("PUT", path, body)

    def delete(self, path, body=None):
        return self._ok("DELETE", path, body)

    def exists(self, path) -> bool:
        return self.request("GET", path)[0] == 200

    def watch(self, path: str, rv: Optional[str] = None) -> Iterator[dict]:
        sep = "&" if "?" in path else "?"
        url = self.server + path + sep + "watch=true" + ("&resourceVersion=%s" % rv if rv else "")
        with urllib.request.urlopen(url, timeout=None) as r:
            for line in r:
                line = line.strip()
                if line:
                    yield json.loads(line)


# ----------------------------------------------------------------------------- TfJob helpers
def tfjobs_path(ns: Optional[str] = "default", name: Optional[str] = None) -> str:
    p = "/apis/%s/%s" % (GROUP, VERSION)
    if ns:
        p += "/namespaces/" + ns
    p += "/" + PLURAL
    if name:
        p += "/" + name
    return p


def create_tf_job(client: ApiClient, spec: dict) -> dict:
    """Create a TfJob (py/tf_job_client.py:18-53)."""
    ns = spec.get("metadata", {}).get("namespace", "default")
    spec.setdefault("apiVersion", "%s/%s" % (GROUP, VERSION))
    spec.setdefault("kind", "TfJob")
    return client.post(tfjobs_path(ns), spec)


def wait_for_job(client: ApiClient, namespace: str, name: str, timeout: float = 300.0,
                 polling_interval: float = 1.0, status_callback=None) -> dict:
    """Poll until status.phase == Done (py/tf_job_client.py:63-96); raises TimeoutError."""
    end = time.time() + timeout
    while True:
        job = client.get(tfjobs_path(namespace, name))
        if status_callback:
            status_callback(job)
        if job.get("status", {}).get("phase") == "Done":
            return job
        if time.time() > end:
            raise TimeoutError("Timeout waiting for job %s in namespace %s to finish." % (name, namespace))
        time.sleep(polling_interval)
