"""In-memory Kubernetes API server semantics (no network).

What the reference could only test on a real GKE cluster we
test against this: resourceVersion bookkeeping, optimistic concurrency (409
Conflict on stale resourceVersion), AlreadyExists / NotFound Status bodies,
label selectors, DeleteCollection, ownerReference garbage collection
(background and foreground), CRD registration with an Established
condition, and a bounded watch history that answers a too-old
resourceVersion with a 410 Gone ERROR event.

``ApiStore.handle(method, path, body_json)`` returns ``(code, body_json)`` and
is used directly by the C++ reconciler bindings (``k8s_amd._operator``) and
over HTTP by ``fakeapi.server``.
"""
from __future__ import annotations

import copy
import datetime
import json
import threading
import uuid
from collections import deque
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import parse_qs, unquote, urlparse

BUILTIN = {
    # (group/version) -> {plural: (kind, namespaced)}
    "v1": {"pods": ("Pod", True), "services": ("Service", True), "configmaps": ("ConfigMap", True),
           "endpoints": ("Endpoints", True), "namespaces": ("Namespace", False), "events": ("Event", True),
           "secrets": ("Secret", True), "persistentvolumeclaims": ("PersistentVolumeClaim", True)},
    "batch/v1": {"jobs": ("Job", True)},
    "apps/v1": {"deployments": ("Deployment", True), "replicasets": ("ReplicaSet", True)},
    "extensions/v1beta1": {"deployments": ("Deployment", True)},
    "coordination.k8s.io/v1": {"leases": ("Lease", True)},
    "apiextensions.k8s.io/v1": {"customresourcedefinitions": ("CustomResourceDefinition", False)},
    "apiextensions.k8s.io/v1beta1": {"customresourcedefinitions": ("CustomResourceDefinition", False)},
}


def now_rfc3339() -> str:
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def status_body(code: int, reason: str, message: str, details: Optional[dict] = None) -> dict:
    b = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": message,
         "reason": reason, "code": code}
    if details:
        b["details"] = details
    return b


def parse_selector(sel: str) -> List[Tuple[str, str, Optional[str]]]:
    """'a=b,c!=d,e' -> [(a, '=', b), (c, '!=', d), (e, 'exists', None)]"""
    out = []
    for part in [p for p in sel.split(",") if p.strip()]:
        part = part.strip()
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in part:
            k, v = part.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        elif part.startswith("!"):
            out.append((part[1:], "!exists", None))
        else:
            out.append((part, "exists", None))
    return out


def match_labels(sel, labels: Optional[dict]) -> bool:
    labels = labels or {}
    for k, op, v in sel:
        if op == "=" and labels.get(k) != v:
            return False
        if op == "!=" and labels.get(k) == v:
            return False
        if op == "exists" and k not in labels:
            return False
        if op == "!exists" and k in labels:
            return False
    return True


class _Route:
    __slots__ = ("gv", "plural", "ns", "name", "sub", "kind", "namespaced")

    def __init__(self, gv, plural, ns, name, sub, kind, namespaced):
        self.gv, self.plural, self.ns, self.name, self.sub = gv, plural, ns, name, sub
        self.kind, self.namespaced = kind, namespaced


class ApiStore:
    def __init__(self, history: int = 2000, established_delay: float = 0.0):
        self.lock = threading.RLock()
        self.cond = threading.Condition(self.lock)
        self.rv = 100
        # (gv, plural) -> {(ns, name): obj}
        self.objects: Dict[Tuple[str, str], Dict[Tuple[str, str], dict]] = {}
        self.crds: Dict[str, Dict[str, Tuple[str, bool]]] = {}  # gv -> plural -> (kind, namespaced)
        self.events = deque(maxlen=history)  # (rv, gv, plural, ns, type, obj)
        self.oldest_rv = self.rv
        self.request_log: List[Tuple[str, str]] = []
        self.hooks: List[Callable] = []  # fn(method, path, body) -> Optional[(code, body)] fault injection
        self.established_delay = established_delay
        self.live_uids = set()  # uids of every stored object (dangling-owner garbage collection)

    # ------------------------------------------------------------------ routing
    def _resources(self, gv):
        r = dict(BUILTIN.get(gv, {}))
        r.update(self.crds.get(gv, {}))
        return r

    def route(self, path: str) -> Optional[_Route]:
        parts = [unquote(p) for p in path.strip("/").split("/") if p]
        if not parts:
            return None
        if parts[0] == "api":
            if len(parts) < 2:
                return None
            gv, rest = parts[1], parts[2:]
        elif parts[0] == "apis":
            if len(parts) < 3:
                return None
            gv, rest = parts[1] + "/" + parts[2], parts[3:]
        else:
            return None
        res = self._resources(gv)
        ns = None
        if len(rest) >= 2 and rest[0] == "namespaces" and (len(rest) > 2 or gv != "v1"):
            ns, rest = rest[1], rest[2:]
        if not rest:
            return None
        plural = rest[0]
        if plural not in res:
            return None
        kind, namespaced = res[plural]
        name = rest[1] if len(rest) > 1 else None
        sub = rest[2] if len(rest) > 2 else None
        return _Route(gv, plural, ns, name, sub, kind, namespaced)

    # ------------------------------------------------------------------ helpers
    def _bump(self) -> str:
        self.rv += 1
        return str(self.rv)

    def _emit(self, gv, plural, ns, typ, obj):
        self.events.append((int(obj["metadata"]["resourceVersion"]), gv, plural, ns, typ, copy.deepcopy(obj)))
        if len(self.events) == self.events.maxlen:
            self.oldest_rv = self.events[0][0]
        self.cond.notify_all()

    def compact(self):
        """Drop the watch history (next watch from an old resourceVersion gets 410 Gone)."""
        with self.lock:
            self.events.clear()
            self.oldest_rv = self.rv

    def _table(self, gv, plural):
        return self.objects.setdefault((gv, plural), {})

    # ------------------------------------------------------------------ public API
    def handle(self, method: str, path: str, body: Optional[str] = None) -> Tuple[int, str]:
        code, b = self.handle_obj(method, path, json.loads(body) if body else None)
        return code, (json.dumps(b) if b is not None else "")

    def handle_obj(self, method: str, path: str, body: Optional[dict]) -> Tuple[int, Optional[dict]]:
        for h in self.hooks:
            r = h(method, path, body)
            if r is not None:
                return r
        u = urlparse(path)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        with self.lock:
            self.request_log.append((method, u.path))
            rt = self.route(u.path)
            if rt is None:
                return 404, status_body(404, "NotFound", "the server could not find the requested resource")
            if method == "GET":
                if rt.name:
                    return self._get(rt)
                return self._list(rt, q)
            if method == "POST":
                return self._create(rt, body or {})
            if method in ("PUT", "PATCH"):
                return self._update(rt, body or {}, merge=(method == "PATCH"))
            if method == "DELETE":
                if rt.name:
                    return self._delete(rt, body or {})
                return self._delete_collection(rt, q)
        return 405, status_body(405, "MethodNotAllowed", method)

    def _get(self, rt):
        o = self._table(rt.gv, rt.plural).get((rt.ns or "", rt.name))
        if o is None:
            return 404, status_body(404, "NotFound", '%s "%s" not found' % (rt.plural, rt.name),
                                    {"name": rt.name, "kind": rt.plural})
        return 200, copy.deepcopy(o)

    def _list(self, rt, q):
        sel = parse_selector(q.get("labelSelector", ""))
        items = []
        for (ns, _), o in sorted(self._table(rt.gv, rt.plural).items()):
            if rt.ns is not None and ns != rt.ns:
                continue
            if match_labels(sel, o["metadata"].get("labels")):
                items.append(copy.deepcopy(o))
        return 200, {"kind": rt.kind + "List", "apiVersion": rt.gv, "metadata": {"resourceVersion": str(self.rv)},
                     "items": items}

    def _create(self, rt, body):
        md = body.setdefault("metadata", {})
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                return 422, status_body(422, "Invalid", "metadata.name: Required value")
        ns = (rt.ns or md.get("namespace") or "default") if rt.namespaced else ""
        key = (ns, md["name"])
        tbl = self._table(rt.gv, rt.plural)
        if key in tbl:
            return 409, status_body(409, "AlreadyExists", '%s "%s" already exists' % (rt.plural, md["name"]),
                                    {"name": md["name"], "kind": rt.plural})
        if rt.namespaced:
            md["namespace"] = ns
        md["uid"] = str(uuid.uuid4())
        md["creationTimestamp"] = now_rfc3339()
        md["resourceVersion"] = self._bump()
        md.setdefault("generation", 1)
        body.setdefault("apiVersion", rt.gv)
        body.setdefault("kind", rt.kind)
        if rt.plural == "customresourcedefinitions":
            self._register_crd(body)
        tbl[key] = body
        self.live_uids.add(md["uid"])
        self._emit(rt.gv, rt.plural, ns, "ADDED", body)
        out = copy.deepcopy(body)
        refs = md.get("ownerReferences") or []
        if refs and not any(r.get("uid") in self.live_uids for r in refs):
            # every owner is already gone (e.g. a pod created for a Job deleted a moment earlier): the garbage
            # collector removes such a dependent right after its creation, as Kubernetes' GC does for dangling owners
            self._remove(rt.gv, rt.plural, ns, md["name"])
        return 201, out

    def _register_crd(self, crd):
        spec = crd.get("spec", {})
        group = spec.get("group")
        names = spec.get("names", {})
        versions = [v.get("name") for v in spec.get("versions", [])] or [spec.get("version")]
        for v in versions:
            if v:
                self.crds.setdefault("%s/%s" % (group, v), {})[names.get("plural")] = (
                    names.get("kind"), spec.get("scope", "Namespaced") == "Namespaced")
        crd["status"] = {"conditions": [
            {"type": "NamesAccepted", "status": "True", "reason": "NoConflicts"},
            {"type": "Established", "status": "True", "reason": "InitialNamesAccepted"}],
            "acceptedNames": names}

    def _update(self, rt, body, merge=False):
        if not rt.name:
            return 405, status_body(405, "MethodNotAllowed", "update needs a name")
        ns = (rt.ns or "default") if rt.namespaced else ""
        tbl = self._table(rt.gv, rt.plural)
        cur = tbl.get((ns, rt.name))
        if cur is None:
            return 404, status_body(404, "NotFound", '%s "%s" not found' % (rt.plural, rt.name))
        want_rv = (body.get("metadata") or {}).get("resourceVersion")
        if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
            return 409, status_body(409, "Conflict",
                                    'Operation cannot be fulfilled on %s "%s": the object has been modified; '
                                    "please apply your changes to the latest version and try again"
                                    % (rt.plural, rt.name))
        if merge:
            new = copy.deepcopy(cur)
            _merge(new, body)
        elif rt.sub == "status":
            new = copy.deepcopy(cur)
            new["status"] = body.get("status")
        else:
            new = copy.deepcopy(body)
            # immutable server-owned metadata
            for k in ("uid", "creationTimestamp", "namespace", "name"):
                new.setdefault("metadata", {})[k] = cur["metadata"].get(k)
            if "deletionTimestamp" in cur["metadata"]:
                new["metadata"]["deletionTimestamp"] = cur["metadata"]["deletionTimestamp"]
        new["metadata"]["resourceVersion"] = self._bump()
        new.setdefault("apiVersion", cur.get("apiVersion"))
        new.setdefault("kind", cur.get("kind"))
        tbl[(ns, rt.name)] = new
        self._emit(rt.gv, rt.plural, ns, "MODIFIED", new)
        return 200, copy.deepcopy(new)

    def _remove(self, gv, plural, ns, name):
        tbl = self._table(gv, plural)
        o = tbl.pop((ns, name), None)
        if o is None:
            return None
        self.live_uids.discard(o["metadata"].get("uid"))
        o["metadata"]["resourceVersion"] = self._bump()
        self._emit(gv, plural, ns, "DELETED", o)
        self._gc(o["metadata"]["uid"])
        return o

    def _gc(self, owner_uid):
        """Garbage-collect dependents whose ownerReferences point at owner_uid (cascading)."""
        for (gv, plural), tbl in list(self.objects.items()):
            for (ns, name), o in list(tbl.items()):
                refs = o["metadata"].get("ownerReferences") or []
                if any(r.get("uid") == owner_uid for r in refs):
                    self._remove(gv, plural, ns, name)

    def _delete(self, rt, opts):
        ns = (rt.ns or "default") if rt.namespaced else ""
        o = self._remove(rt.gv, rt.plural, ns, rt.name)
        if o is None:
            return 404, status_body(404, "NotFound", '%s "%s" not found' % (rt.plural, rt.name),
                                    {"name": rt.name, "kind": rt.plural})
        if rt.plural == "customresourcedefinitions":
            spec = o.get("spec", {})
            for v in spec.get("versions", []):
                self.crds.get("%s/%s" % (spec.get("group"), v.get("name")), {}).pop(spec.get("names", {}).get("plural"),
                                                                                    None)
        return 200, o

    def _delete_collection(self, rt, q):
        sel = parse_selector(q.get("labelSelector", ""))
        removed = []
        for (ns, name), o in list(self._table(rt.gv, rt.plural).items()):
            if rt.ns is not None and ns != rt.ns:
                continue
            if match_labels(sel, o["metadata"].get("labels")):
                removed.append(self._remove(rt.gv, rt.plural, ns, name))
        return 200, {"kind": rt.kind + "List", "apiVersion": rt.gv, "metadata": {}, "items": removed}

    # ------------------------------------------------------------------ watch
    def watch_from(self, path: str, rv: Optional[str]):
        """Generator of (type, obj) events for a collection path; yields ('ERROR', Status 410) if rv too old."""
        u = urlparse(path)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        rt = self.route(u.path)
        if rt is None:
            yield "ERROR", status_body(404, "NotFound", "no such resource")
            return
        sel = parse_selector(q.get("labelSelector", ""))
        start = int(rv) if rv else None
        with self.lock:
            if start is None:
                start = self.rv
            if start < self.oldest_rv:
                yield "ERROR", status_body(410, "Expired", "too old resource version: %d (%d)" % (start, self.oldest_rv))
                return
        last = start
        while True:
            batch = []
            with self.lock:
                while True:
                    batch = [e for e in self.events if e[0] > last]
                    if batch:
                        break
                    if not self.cond.wait(timeout=1.0):
                        batch = []
                        break
            if not batch:
                yield None, None  # heartbeat: lets the server detect closed connections
                continue
            for (erv, gv, plural, ns, typ, obj) in batch:
                last = max(last, erv)
                if gv != rt.gv or plural != rt.plural:
                    continue
                if rt.ns is not None and ns != rt.ns:
                    continue
                if not match_labels(sel, obj["metadata"].get("labels")):
                    continue
                yield typ, obj

    # ------------------------------------------------------------------ convenience for in-process users
    def get(self, path):
        return self.handle_obj("GET", path, None)

    def post(self, path, body):
        return self.handle_obj("POST", path, body)

    def put(self, path, body):
        return self.handle_obj("PUT", path, body)

    def delete(self, path, body=None):
        return self.handle_obj("DELETE", path, body)


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        elif v is None:
            dst.pop(k, None)
        else:
            dst[k] = v
