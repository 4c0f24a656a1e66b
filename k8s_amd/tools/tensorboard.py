"""TensorBoard stand-in for the TfJob TensorBoard replica (no tensorflow / tensorboard package in this stack).

The operator deploys ``tensorboard --logdir <logDir> --host 0.0.0.0`` behind a Service on port 80 -> 6006
(`/root/reference/pkg/trainer/tensorboard.go:140-177`). This server reads the same ``events.out.tfevents.*``
files the trainer writes (``k8s_amd.utils.tfevents``, CRC-checked) and serves TensorBoard's scalar REST API
shape, so the reference notebook's "watch the loss in TensorBoard" step works against a real HTTP endpoint:

    GET /data/runs                                  -> ["run", ...]   ("." = files directly in logdir)
    GET /data/plugin/scalars/tags                   -> {run: {tag: {"displayName": tag, "description": ""}}}
    GET /data/plugin/scalars/scalars?run=R&tag=T    -> [[wall_time, step, value], ...]
    GET /                                           -> a plain-text summary (latest value per run/tag)

    python -m k8s_amd.tools.tensorboard --logdir DIR [--host 127.0.0.1] [--port 6006]

Files are rescanned on every request, reading only bytes appended since the last scan.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import struct
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List
from urllib.parse import parse_qs, urlparse

from k8s_amd.utils.tfevents import decode_event, masked_crc


class _FileTail:
    """Incremental TFRecord reader: complete, CRC-valid records appended since the last call."""

    def __init__(self, path: str):
        self.path, self.pos = path, 0

    def new_events(self):
        out = []
        try:
            with open(self.path, "rb") as f:
                f.seek(self.pos)
                while True:
                    h = f.read(12)
                    if len(h) < 12:
                        break
                    n, lc = struct.unpack("<QI", h)
                    if masked_crc(h[:8]) != lc:
                        break
                    data = f.read(n)
                    tail = f.read(4)
                    if len(data) < n or len(tail) < 4 or masked_crc(data) != struct.unpack("<I", tail)[0]:
                        break
                    self.pos += 12 + n + 4
                    out.append(decode_event(data))
        except OSError:
            pass
        return out


class EventStore:
    def __init__(self, logdir: str):
        self.logdir = logdir
        self.tails: Dict[str, _FileTail] = {}
        self.data: Dict[str, Dict[str, List[list]]] = {}  # run -> tag -> [[wall, step, value]]
        self.lock = threading.Lock()

    def scan(self):
        with self.lock:
            for root, _, files in os.walk(self.logdir):
                for fn in sorted(files):
                    if "tfevents" not in fn:
                        continue
                    path = os.path.join(root, fn)
                    if path not in self.tails:
                        self.tails[path] = _FileTail(path)
                    run = os.path.relpath(root, self.logdir)
                    for ev in self.tails[path].new_events():
                        for tag, v in ev["scalars"].items():
                            self.data.setdefault(run, {}).setdefault(tag, []).append([ev["wall_time"], ev["step"],
                                                                                      v])
            return {r: {t: list(v) for t, v in tags.items()} for r, tags in self.data.items()}


def make_handler(store: EventStore):
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code, body, ctype="application/json"):
            raw = body.encode() if isinstance(body, str) else body
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(raw)))
            self.end_headers()
            self.wfile.write(raw)

        def do_GET(self):
            u = urlparse(self.path)
            q = parse_qs(u.query)
            data = store.scan()
            if u.path == "/data/runs":
                return self._send(200, json.dumps(sorted(data)))
            if u.path == "/data/plugin/scalars/tags":
                return self._send(200, json.dumps({r: {t: {"displayName": t, "description": ""} for t in tags}
                                                   for r, tags in data.items()}))
            if u.path == "/data/plugin/scalars/scalars":
                run, tag = q.get("run", [""])[0], q.get("tag", [""])[0]
                series = data.get(run, {}).get(tag)
                if series is None:
                    return self._send(404, json.dumps({"error": "no such run/tag"}))
                return self._send(200, json.dumps(sorted(series, key=lambda r: (r[1], r[0]))))
            if u.path in ("/", "/index.html"):
                lines = ["TensorBoard (k8s_amd stand-in) logdir=%s" % store.logdir]
                for r in sorted(data):
                    for t in sorted(data[r]):
                        w, st, v = data[r][t][-1]
                        lines.append("%s/%s step %d: %g (%d points)" % (r, t, st, v, len(data[r][t])))
                return self._send(200, "\n".join(lines) + "\n", "text/plain")
            return self._send(404, json.dumps({"error": "not found"}))

    return Handler


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=6006)
    a = ap.parse_args(argv)
    srv = ThreadingHTTPServer((a.host, a.port), make_handler(EventStore(a.logdir)))
    signal.signal(signal.SIGTERM, lambda *x: threading.Thread(target=srv.shutdown, daemon=True).start())
    print("TensorBoard stand-in serving %s on http://%s:%d/" % (a.logdir, a.host, a.port), flush=True)
    srv.serve_forever()
    srv.server_close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
