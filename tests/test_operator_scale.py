"""Operator at the reference's design target: 100 concurrent TfJobs.

`/root/reference/tf_job_design_doc.md:24` sizes the operator for O(100) concurrent TfJobs. 100 jobs of
1 MASTER + 1 WORKER run on the one-box cluster, once with the shared Job / Pod watch caches (informers, the
default) and once with the reference's per-replica polling reads: every job must reach Succeeded and be cleaned up
within a fixed wall time, and the caches must cut the operator's steady-state API requests per job >= 2x (measured
from the API server's side, by User-Agent). ``benchmarks/operator_scale.py`` is the same run as a benchmark.
"""
import os

import pytest

from k8s_amd.fakeapi.cluster import OPERATOR_BIN

pytestmark = pytest.mark.skipif(not os.path.exists(OPERATOR_BIN), reason="bin/tf_operator not built")


def test_hundred_concurrent_tfjobs_with_and_without_informers():
    from benchmarks.operator_scale import run

    res = {m: run(jobs=100, informers=m, window=4.0, interval="2s", timeout=240.0, log=lambda s: None)
           for m in (False, True)}
    for m, r in res.items():
        assert r["states"] == {"Succeeded": 100}, (m, r)
        assert not any(r["left_after_cleanup"].values()), (m, r)
        assert r["operator_errors"] == 0, (m, r)
        assert r["wall_s"] < 150, (m, r)
        assert r["operator_threads"] <= 100 + 16, (m, r)  # one worker per job + a fixed few
    polled, cached = res[False]["steady_qps_per_job"], res[True]["steady_qps_per_job"]
    # polling: ~2 reads per replica per 2 s tick per job; cached: only status writes when something changes
    assert polled >= 0.5, res[False]
    assert cached * 2 <= polled, (cached, polled)
    # the caches' change callback pokes the owning job's worker: a finished MASTER is seen at watch latency, not at the
    # next resync tick
    assert res[True]["release_to_succeeded_s"]["p50"] <= res[False]["release_to_succeeded_s"]["p50"] + 1.0, res
