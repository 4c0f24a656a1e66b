"""Tracing (ROCTx step phases), the hang watchdog (exit 143 = retryable) and the kernel debug proxy
(NaN/+Inf checks, per-op synchronisation). SURVEY.md §5.1-5.3."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

from k8s_amd.utils import debug
from k8s_amd.utils.trace import EXIT_HANG, Tracer, Watchdog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tracer_phases_accumulate():
    t = Tracer(enabled=True, sync=True)
    for _ in range(3):
        with t.phase("forward"):
            time.sleep(0.01)
        with t.phase("backward"):
            pass
    s = t.summary_ms()
    assert set(s) == {"forward", "backward"} and s["forward"] >= 9.0
    assert t.summary_ms() == {}  # reset
    off = Tracer(enabled=False)
    with off.phase("x"):
        pass
    assert off.summary_ms() == {}


def test_watchdog_fires_without_kicks():
    codes = []
    w = Watchdog(0.2, exit_fn=codes.append, poll=0.02).start()
    time.sleep(0.6)
    w.stop()
    assert codes == [EXIT_HANG] and w.fired


def test_watchdog_quiet_while_kicked():
    codes = []
    w = Watchdog(0.3, exit_fn=codes.append, poll=0.02).start()
    for _ in range(10):
        time.sleep(0.05)
        w.kick()
    w.stop()
    assert codes == [] and not w.fired


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        env.pop(k, None)
    return env


def test_trainer_hang_exits_retryable():
    p = subprocess.run([sys.executable, "-m", "k8s_amd.trainer", "--device", "cpu", "--model", "resnet_tiny",
                        "--steps", "6", "--hang-at-step", "2", "--hang-timeout", "3"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == EXIT_HANG, p.stdout[-2000:] + p.stderr[-2000:]
    assert "watchdog" in p.stderr


def test_trainer_trace_sync_reports_phases():
    p = subprocess.run([sys.executable, "-m", "k8s_amd.trainer", "--device", "cpu", "--model", "resnet_tiny",
                        "--steps", "3", "--log-every", "1", "--trace", "sync"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    steps = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{") and '"event": "step"' in l]
    assert steps and {"step", "forward", "backward", "reduce+update"} <= set(steps[-1]["phase_ms"])


class _FakeExt:
    conv_stat_replicas = 32

    def bad(self, x):
        return x * float("nan")

    def good(self, x):
        return [x + 1, x.to(torch.int32)]

    def inplace(self, out):
        out.fill_(float("inf"))

    def neg_inf_ok(self, x):
        return torch.full_like(x, float("-inf"))


def test_checked_extension_numerics():
    ext = debug.CheckedExtension(_FakeExt(), check_numerics=True, sync=False)
    x = torch.ones(4)
    assert ext.conv_stat_replicas == 32
    assert torch.equal(ext.good(x)[0], x + 1)
    ext.neg_inf_ok(x)
    with pytest.raises(debug.NumericsError, match="bad"):
        ext.bad(x)
    with pytest.raises(debug.NumericsError, match="inplace"):
        ext.inplace(torch.zeros(3))


def test_maybe_wrap_is_identity_when_disabled(monkeypatch):
    monkeypatch.delenv("K8S_AMD_CHECK_NUMERICS", raising=False)
    monkeypatch.delenv("K8S_AMD_SYNC_OPS", raising=False)
    m = _FakeExt()
    assert debug.maybe_wrap(m) is m
    monkeypatch.setenv("K8S_AMD_SYNC_OPS", "1")
    assert isinstance(debug.maybe_wrap(m), debug.CheckedExtension)


@pytest.mark.gpu
def test_numerics_mode_on_gpu_catches_nan():
    code = r"""
import torch
from k8s_amd.ops import _ext
from k8s_amd.utils.debug import CheckedExtension, NumericsError
C = _ext.load()
assert isinstance(C, CheckedExtension)
from k8s_amd.ops import nn as K
from k8s_amd.parallel.flat import ParamStore, init_const
st = ParamStore()
pg = st.new("g", (256,), init_const(1.0), decay=False); pb = st.new("b", (256,), init_const(0.0), decay=False)
st.finalize(torch.device("cuda"))
x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
K.layer_norm(x, pg, pb)          # finite: passes
x[3, 7] = float("nan")
try:
    K.layer_norm(x, pg, pb)
except NumericsError as e:
    print("caught", e)
else:
    raise SystemExit("NaN not caught")
"""
    env = dict(os.environ, K8S_AMD_CHECK_NUMERICS="1", K8S_AMD_SYNC_OPS="1",
               PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "caught" in p.stdout, p.stdout[-2000:] + p.stderr[-3000:]
