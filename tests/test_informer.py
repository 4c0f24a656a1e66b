"""The operator's shared watch cache (``csrc/operator/informer.cc``) under watch-open failures:
a watch that cannot be re-opened must not leave the cache frozen at its last list. A 410 / 403 on the watch open
relists at once, any other error relists after a run of failed opens, a resync period relists a healthy cache, and
``fresh()`` -- what the reconciler checks before trusting the cache over a direct GET / LIST (reconciler.cc) -- turns
false while neither a watch nor a list succeeds. Driven over the real HTTP transport against the fake API server's
error injection (``FakeApiServer.fail``)."""
import json
import time

import pytest

from k8s_amd.fakeapi.server import FakeApiServer

op = pytest.importorskip("k8s_amd._operator")
NS = "default"
PODS = "/api/v1/namespaces/%s/pods" % NS


def _pod(srv, name):
    body = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": NS,
                                                            "labels": {"tensorflow.org": ""}},
            "spec": {"containers": [{"name": "tensorflow", "image": "x"}]}}
    code, _ = srv.store.handle_obj("POST", PODS, json.loads(json.dumps(body)))
    assert code in (200, 201), code


def _until(pred, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


@pytest.fixture
def srv():
    with FakeApiServer() as s:
        yield s


def _informer(srv, **kw):
    args = dict(selector="tensorflow.org", watch_timeout_ms=1000, retry_ms=100, resync_ms=600000, relist_after=3,
                stale_ms=60000)
    args.update(kw)
    inf = op.Informer(srv.url, PODS, **args)
    inf.start()
    assert inf.wait_synced(5000)
    return inf


def test_watch_410_on_open_relists_at_once(srv):
    inf = _informer(srv)
    try:
        _pod(srv, "a")
        assert _until(lambda: "a" in inf.names(NS))
        lists = inf.lists()
        rule = srv.fail(410, 2.5, PODS, watch=True)
        _pod(srv, "b")  # may arrive on the still-open watch; "c" is created while every re-open gets 410
        assert _until(lambda: rule["hits"] >= 1, 5.0)
        _pod(srv, "c")
        # one 410 on open is enough to relist (LISTs still work): "c" shows up with no watch re-established
        assert _until(lambda: "c" in inf.names(NS), 5.0), inf.names(NS)
        assert inf.lists() > lists
        assert inf.fresh()
    finally:
        inf.stop()


def test_repeated_watch_failures_relist(srv):
    inf = _informer(srv, relist_after=3)
    try:
        rule = srv.fail(500, 3.0, PODS, watch=True)
        assert _until(lambda: rule["hits"] >= 1, 5.0)
        lists = inf.lists()
        _pod(srv, "late")
        # 500s are retried from the same rv, but after 3 in a row the informer relists and sees the new pod
        assert _until(lambda: "late" in inf.names(NS), 5.0), inf.names(NS)
        assert inf.lists() > lists and rule["hits"] >= 3
    finally:
        inf.stop()


def test_cache_not_fresh_while_watch_and_list_fail(srv):
    inf = _informer(srv, stale_ms=400)
    try:
        assert inf.fresh()
        srv.fail(500, 4.0, PODS, watch=None)  # lists and watch opens both fail
        # the open watch ends at its 1 s timeout; with nothing succeeding the cache goes stale -> readers go direct
        assert _until(lambda: not inf.fresh(), 5.0)
        assert inf.synced()  # still synced once: staleness, not the initial sync, is what flips
        # recovery: the next successful list / watch makes it fresh again
        assert _until(inf.fresh, 8.0)
    finally:
        inf.stop()


def test_resync_period_relists_a_healthy_cache(srv):
    inf = _informer(srv, watch_timeout_ms=60000, resync_ms=1000)
    try:
        lists = inf.lists()
        assert _until(lambda: inf.lists() >= lists + 2, 6.0)
        assert inf.fresh()
    finally:
        inf.stop()
