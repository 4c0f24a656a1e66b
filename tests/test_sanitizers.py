"""Host-side sanitizer runs of the C++ control plane (the reference ran `go test` without
`-race`; its controller mutates shared maps from several goroutines).

`tf_operator` and `e2e` are rebuilt with AddressSanitizer + UndefinedBehaviorSanitizer and, separately,
ThreadSanitizer (``python -m k8s_amd._build --only sanitizers`` -> ``bin/*-asan``, ``bin/*-tsan``), then
driven through the same local-cluster flows as tests/test_e2e_local.py: a MASTER + WORKER + 2 default-PS job
to Succeeded and deletion, and the e2e binary running two TfJobs concurrently (parallel reconciler threads,
watch thread, status writes). Any sanitizer report fails the test. CPU only.
"""
import glob
import os
import subprocess
import time

import pytest

from k8s_amd import _build
from k8s_amd.fakeapi.cluster import REPO, LocalCluster

BIN = os.path.join(REPO, "bin")


def _need(san):
    op, e2e = os.path.join(BIN, "tf_operator-" + san), os.path.join(BIN, "e2e-" + san)
    if not (os.path.exists(op) and os.path.exists(e2e)):
        try:
            _build.build_operator(sanitize=san)
        except Exception as e:  # toolchain without the sanitizer runtime
            pytest.skip("cannot build %s binaries: %s" % (san, str(e)[:200]))
    return op, e2e


def _reports(d):
    out = []
    for p in sorted(glob.glob(os.path.join(d, "san.*"))):
        txt = open(p, errors="replace").read()
        if txt.strip():
            out.append("%s:\n%s" % (p, txt[:4000]))
    return out


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_operator_under_sanitizer(san, tmp_path, monkeypatch):
    op, e2e = _need(san)
    rep = str(tmp_path / "reports")
    os.makedirs(rep)
    common = "log_path=%s/san:exitcode=66" % rep
    monkeypatch.setenv("ASAN_OPTIONS", common + ":detect_leaks=1:abort_on_error=0")
    monkeypatch.setenv("UBSAN_OPTIONS", common + ":print_stacktrace=1:halt_on_error=1")
    monkeypatch.setenv("TSAN_OPTIONS", common + ":second_deadlock_stack=1")
    monkeypatch.setenv("LSAN_OPTIONS", "log_path=%s/san" % rep)
    with LocalCluster(operator_bin=op, reconcile_interval="200ms", log_dir=str(tmp_path / "cluster")) as c:
        c.create(os.path.join(REPO, "examples", "tf_job.yaml"))
        end = time.time() + 90
        st = {}
        while time.time() < end:
            st = c.get("example-job").get("status", {})
            if st.get("phase") == "Done":
                break
            time.sleep(0.2)
        assert st.get("state") == "Succeeded", (st, c.operator_log()[-3000:])
        c.delete("example-job")
        r = subprocess.run([e2e, "--image", "k8s-amd/tf_sample:rocm7", "--master", c.url, "--timeout", "120",
                            "--num_jobs", "2"], capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:] + c.operator_log()[-3000:]
        assert c.op_proc.poll() is None, "operator died:\n" + c.operator_log()[-4000:]
    reports = _reports(rep)
    assert not reports, "\n\n".join(reports)
