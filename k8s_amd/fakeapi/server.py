"""HTTP front-end of the in-memory API server (``fakeapi.store.ApiStore``).

Speaks the subset of the Kubernetes REST protocol the operator, the e2e
binary, the kubelet and the ``tfjob`` CLI use: JSON bodies, Status error
objects, ``?labelSelector=``, and ``?watch=true&resourceVersion=N`` streams
delivered with chunked transfer encoding, one ``{"type","object"}`` JSON
event per line (410 Gone as an ERROR event when the version is compacted).

    python -m k8s_amd.fakeapi.server --port 8080
"""
from __future__ import annotations

import argparse
import json
import socket
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, urlparse

from k8s_amd.fakeapi.store import ApiStore


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    store: ApiStore = None  # set per server class

    def log_message(self, fmt, *args):  # quiet
        pass

    def _body(self) -> Optional[dict]:
        n = int(self.headers.get("Content-Length") or 0)
        if n <= 0:
            return None
        raw = self.rfile.read(n)
        try:
            return json.loads(raw)
        except ValueError:
            return None

    def _send(self, code: int, body):
        data = json.dumps(body).encode() if body is not None else b""
        try:
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
        except (BrokenPipeError, ConnectionResetError):
            pass  # the client went away (e.g. an operator shutting down mid-request)

    def _stall(self):
        """Fault injection: hold a matching request until its stall window ends (the client has usually given
        up by then), like an API server that stops answering."""
        ua = self.headers.get("User-Agent", "")
        for rule in list(self.server.stalls):
            if time.time() < rule["until"] and self.path.startswith(rule["path_prefix"]) and \
                    rule["user_agent"] in ua:
                time.sleep(max(0.0, rule["until"] - time.time()))

    def _dispatch(self, method):
        u = urlparse(self.path)
        if u.path == "/debug/stall" and method == "POST":
            # {"seconds": S, "path_prefix": "/api", "user_agent": "tf-operator-local-0"}: stall matching requests
            b = self._body() or {}
            self.server.stalls.append({"until": time.time() + float(b.get("seconds", 5)),
                                       "path_prefix": b.get("path_prefix", "/"),
                                       "user_agent": b.get("user_agent", "")})
            return self._send(200, {"stalls": len(self.server.stalls)})
        self._stall()
        for rule in list(self.server.failures):  # fault injection: answer matching requests with an error status
            is_watch = "watch=" in u.query
            if time.time() < rule["until"] and u.path.startswith(rule["path_prefix"]) and \
                    (rule["watch"] is None or rule["watch"] == is_watch):
                rule["hits"] += 1
                return self._send(rule["code"], {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                 "reason": "Injected", "code": rule["code"]})
        with self.server.count_lock:  # requests per client (User-Agent) and kind: the operator scale test's API load
            ua = self.headers.get("User-Agent", "")
            kind = "WATCH" if "watch=" in u.query else method
            self.server.ua_counts[(ua, kind)] = self.server.ua_counts.get((ua, kind), 0) + 1
        accept = self.server.accept_token
        if accept is not None:  # bearer-token check (credential refresh tests)
            auth = self.headers.get("Authorization", "")
            tok = auth[len("Bearer "):] if auth.startswith("Bearer ") else ""
            if not accept(tok):
                self.server.rejected.append(tok)
                return self._send(401, {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                        "reason": "Unauthorized", "code": 401})
            self.server.accepted.append(tok)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        body = self._body() if method in ("POST", "PUT", "PATCH", "DELETE") else None
        if method == "GET" and q.get("watch") in ("true", "1"):
            return self._watch(q.get("resourceVersion") or None, float(q.get("timeoutSeconds") or 0))
        if u.path in ("/healthz", "/readyz", "/livez"):
            data = b"ok"
            self.send_response(200)
            self.send_header("Content-Length", "2")
            self.end_headers()
            self.wfile.write(data)
            return
        if u.path == "/version":
            return self._send(200, {"major": "1", "minor": "30", "gitVersion": "v1.30.0-k8s-amd-fake"})
        code, out = self.store.handle_obj(method, self.path, body)
        self._send(code, out)

    def _chunk(self, data: bytes):
        self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
        self.wfile.flush()

    def _watch(self, rv, timeout_s=0.0):
        """Chunked watch stream; ends after ``timeout_s`` (``?timeoutSeconds=``) like the real API server. A watch
        open when a black-hole fault is injected (``FakeApiServer.blackhole_watches``) goes silent for good -- no
        events, no end of stream, the socket left open -- as a connection a NAT / load balancer dropped without
        telling either side."""
        started = time.time()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        try:
            for typ, obj in self.store.watch_from(self.path, rv):
                if started < self.server.blackhole_before:
                    while not self.server.stopping:  # half-open: hold the socket, never write again
                        time.sleep(0.2)
                    return
                if timeout_s and time.time() - started >= timeout_s:
                    break
                if typ is None:
                    continue  # heartbeat; a write failure below ends the stream
                self._chunk((json.dumps({"type": typ, "object": obj}) + "\n").encode())
                if typ == "ERROR":
                    break
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        self.close_connection = True

    def do_GET(self):
        self._dispatch("GET")

    def do_POST(self):
        self._dispatch("POST")

    def do_PUT(self):
        self._dispatch("PUT")

    def do_PATCH(self):
        self._dispatch("PATCH")

    def do_DELETE(self):
        self._dispatch("DELETE")


class _Server(ThreadingHTTPServer):
    # listen backlog: socketserver's default of 5 resets connections when ~100 reconciler threads, the kubelet and
    # the clients connect at once (the operator scale test)
    request_queue_size = 1024


class FakeApiServer:
    """Run an ApiStore behind HTTP on 127.0.0.1:<port> in a background thread."""

    def __init__(self, store: Optional[ApiStore] = None, port: int = 0, host: str = "127.0.0.1"):
        self.store = store or ApiStore()
        handler = type("Handler", (_Handler,), {"store": self.store})
        self.httpd = _Server((host, port), handler)
        self.httpd.daemon_threads = True
        self.httpd.stalls = []  # fault injection rules (POST /debug/stall, or stall() below)
        self.httpd.failures = []  # error-status injection rules (fail() below)
        self.httpd.blackhole_before = 0.0  # watches opened before this time are black holes (blackhole_watches)
        self.httpd.accept_token = None  # callable(token) -> bool: reject other bearer tokens with 401
        self.httpd.accepted, self.httpd.rejected = [], []
        self.httpd.stopping = False
        self.httpd.count_lock = threading.Lock()
        self.httpd.ua_counts = {}  # (User-Agent, GET/POST/PUT/DELETE/WATCH) -> requests
        self.port = self.httpd.server_address[1]
        self.url = "http://%s:%d" % (host, self.port)
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    def start(self):
        self.thread.start()
        return self

    def stall(self, seconds: float, path_prefix: str = "/", user_agent: str = ""):
        """Stop answering matching requests for ``seconds`` (requests arriving meanwhile hang until then)."""
        self.httpd.stalls.append({"until": time.time() + seconds, "path_prefix": path_prefix,
                                  "user_agent": user_agent})

    def fail(self, code: int, seconds: float, path_prefix: str = "/", watch: Optional[bool] = None) -> dict:
        """Answer matching requests with HTTP ``code`` (a Status body) for ``seconds``: ``watch`` True = only watch
        opens, False = only plain requests, None = both. Returns the rule (its ``hits`` counts the failed requests)."""
        rule = {"until": time.time() + seconds, "path_prefix": path_prefix, "code": int(code), "watch": watch,
                "hits": 0}
        self.httpd.failures.append(rule)
        return rule

    def request_counts(self, ua_prefix: str = "") -> dict:
        """{method: requests} of the clients whose User-Agent starts with ``ua_prefix`` (WATCH = watch opens)."""
        out = {}
        with self.httpd.count_lock:
            for (ua, kind), n in self.httpd.ua_counts.items():
                if ua.startswith(ua_prefix):
                    out[kind] = out.get(kind, 0) + n
        return out

    def blackhole_watches(self):
        """Every watch open right now silently stops: no more events and no end of stream (a half-open TCP
        connection); watches opened afterwards work normally."""
        self.httpd.blackhole_before = time.time()

    def stop(self):
        self.httpd.stopping = True
        self.httpd.shutdown()
        self.httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None):
    ap = argparse.ArgumentParser(description="in-memory Kubernetes API server (k8s_amd test double)")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--host", default="127.0.0.1")
    a = ap.parse_args(argv)
    srv = FakeApiServer(port=a.port, host=a.host)
    print("fake API server on %s" % srv.url, flush=True)
    srv.httpd.serve_forever()


if __name__ == "__main__":
    main()
