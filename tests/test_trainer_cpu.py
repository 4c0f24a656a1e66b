"""The TfJob trainer on CPU: TF_CONFIG roles, gloo DP (all-reduce and sharded PS), checkpoint/resume,
exit-code contract (reference: pkg/trainer/training.go:45-73 retry rules)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from k8s_amd.fakeapi.server import free_port
from k8s_amd.utils import checkpoint as ckpt

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(tf_config=None):
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        env.pop(k, None)
    if tf_config is not None:
        env["TF_CONFIG"] = json.dumps(tf_config)
    return env


def _trainer(args, tf_config=None, **extra_env):
    env = _env(tf_config)
    env.update(extra_env)
    return subprocess.Popen([sys.executable, "-m", "k8s_amd.trainer", "--device", "cpu"] + args,
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def _events(out):
    recs = []
    for line in out.splitlines():
        if line.startswith("{"):
            try:
                recs.append(json.loads(line))
            except ValueError:
                pass
    return recs


def test_single_rank_checkpoint_resume(tmp_path):
    ck, lg = str(tmp_path / "ckpt"), str(tmp_path / "log")
    p = _trainer(["--model", "resnet_tiny", "--steps", "4", "--ckpt-dir", ck, "--logdir", lg, "--ckpt-every", "2",
                  "--log-every", "1"])
    out, _ = p.communicate(timeout=240)
    assert p.returncode == 0, out
    ev = _events(out)
    assert [e["event"] for e in ev][:2] == ["start", "step0"]
    assert ev[-1]["event"] == "done"
    latest, allp = ckpt.read_state(ck)
    assert latest == "model.ckpt-3" and allp == ["model.ckpt-1", "model.ckpt-3"]
    assert any(f.startswith("events.out.tfevents.") for f in os.listdir(lg))
    # resume: continues at step 4
    p = _trainer(["--model", "resnet_tiny", "--steps", "6", "--ckpt-dir", ck, "--log-every", "1"])
    out, _ = p.communicate(timeout=240)
    assert p.returncode == 0, out
    ev = _events(out)
    restored = [e for e in ev if e["event"] == "restored"]
    assert restored and restored[0]["step"] == 3
    assert [e for e in ev if e["event"] == "step0"][0]["step"] == 4
    step, tensors, meta = ckpt.load(ckpt.latest_checkpoint(ck))
    assert step == 5 and meta["optim_step"] == 6
    assert any(k.startswith("buffers/") and k.endswith("running_mean") for k in tensors)


def test_retryable_exit_then_resume(tmp_path):
    ck = str(tmp_path / "ckpt")
    args = ["--model", "resnet_tiny", "--steps", "4", "--ckpt-dir", ck, "--ckpt-every", "1", "--fail-at-step", "2"]
    p = _trainer(args)
    out, _ = p.communicate(timeout=240)
    assert p.returncode >= 128, out  # retryable per the operator's exit-code contract
    assert ckpt.read_state(ck)[0] == "model.ckpt-1"
    p = _trainer(args)  # the restarted replica resumes and finishes
    out, _ = p.communicate(timeout=240)
    assert p.returncode == 0, out
    assert ckpt.read_state(ck)[0] == "model.ckpt-3"


def test_bad_model_is_permanent_failure():
    p = subprocess.run([sys.executable, "-m", "k8s_amd.trainer", "--model", "nope"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert 0 < p.returncode < 128


def _distinct_ports(n):
    ports = []
    while len(ports) < n:
        p = free_port()
        if p not in ports:
            ports.append(p)
    return ports


def _run_job(tmp_path, strategy, with_ps):
    pm, pw, pp = _distinct_ports(3)
    cluster = {"master": ["127.0.0.1:%d" % pm], "worker": ["127.0.0.1:%d" % pw]}
    if with_ps:
        cluster["ps"] = ["127.0.0.1:%d" % pp]
    ck = str(tmp_path / strategy)
    common = ["--model", "resnet_tiny", "--steps", "3", "--strategy", strategy, "--ckpt-dir", ck, "--log-every", "1",
              "--optimizer", "adam", "--lr", "0.01"]
    procs = []
    if with_ps:
        procs.append(_trainer(common, {"cluster": cluster, "task": {"type": "ps", "index": 0},
                                       "environment": "cloud"}))
    procs.append(_trainer(common, {"cluster": cluster, "task": {"type": "master", "index": 0},
                                   "environment": "cloud"}))
    procs.append(_trainer(common, {"cluster": cluster, "task": {"type": "worker", "index": 0},
                                   "environment": "cloud"}))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=300)
        outs.append(out)
        assert p.returncode == 0, out
    _, tensors, meta = ckpt.load(ckpt.latest_checkpoint(ck))
    assert meta["world"] == 2
    return tensors, outs


def test_two_rank_allreduce_and_sharded_ps_agree(tmp_path):
    """1 MASTER + 1 WORKER (+ 1 PS task running the parameter server, shut down by the master): the
    sharded parameter service (reduce-scatter / owner update / all-gather) must produce the same weights
    and optimizer state as the all-reduce strategy."""
    a, _ = _run_job(tmp_path, "allreduce", with_ps=False)
    b, outs = _run_job(tmp_path, "ps", with_ps=True)
    assert "Started server /job:ps/task:0" in outs[0]
    checks = [e for e in _events(outs[1]) if e.get("event") == "transport_check"]
    assert checks and checks[0]["ok"] is True and checks[0]["transport"] == "zero1-fp32", outs[1][-2000:]
    for k in a:
        if k.startswith("params/") or k.startswith("optim/"):
            torch.testing.assert_close(a[k], b[k], rtol=1e-4, atol=1e-5, msg=k)


def test_service_resolution_follows_the_live_map_file(tmp_path, monkeypatch):
    """A pod started before a peer's Service existed must still resolve it: the local kubelet keeps
    $K8S_AMD_SERVICE_MAP_FILE current and resolvers read it on every lookup (the env snapshot is a fallback)."""
    import json

    from k8s_amd.parallel import dist
    from k8s_amd.ps_server import grpc_tensorflow_server as srv

    f = tmp_path / "service-map-default.json"
    monkeypatch.setenv("K8S_AMD_SERVICE_MAP", json.dumps({"a-master-x-0": "127.0.0.1:1000"}))
    monkeypatch.setenv("K8S_AMD_SERVICE_MAP_FILE", str(f))
    assert srv.resolve("a-ps-x-0:2222") == "a-ps-x-0:2222"  # no file yet: snapshot only
    assert dist.resolve("a-master-x-0:2222") == "127.0.0.1:1000"
    f.write_text(json.dumps({"a-master-x-0": "127.0.0.1:1000", "a-ps-x-0": "127.0.0.1:1002"}))
    assert srv.resolve("a-ps-x-0:2222") == "127.0.0.1:1002"
    assert dist.resolve("a-ps-x-0:2222") == "127.0.0.1:1002"


def test_ps_tasks_hold_the_variables_and_a_restarted_job_resumes_from_them(tmp_path):
    """1 MASTER + 1 WORKER + 2 PS: the chief pushes a versioned snapshot (weights, Adam state, BN buffers) to the
    PS tasks every 2 steps, sharded over them; both compute ranks then fail (retryable) at step 4 with NO
    checkpoint on disk, and the restarted ranks resume from the PS tasks' committed snapshot (step 3) -- the TF
    PS semantics (variables live on /job:ps, workers are stateless). The result equals an uninterrupted run."""
    from k8s_amd.ps_server.grpc_tensorflow_server import call

    pm, pw, p0, p1, rm, rw = _distinct_ports(6)
    cluster = {"master": ["127.0.0.1:%d" % pm], "worker": ["127.0.0.1:%d" % pw],
               "ps": ["127.0.0.1:%d" % p0, "127.0.0.1:%d" % p1]}
    run = str(tmp_path / "run")
    common = ["--model", "resnet_tiny", "--steps", "6", "--ckpt-dir", run, "--log-every", "1", "--optimizer",
              "adam", "--lr", "0.01", "--ps-sync-every", "2"]

    def tfc(role, i, cl=cluster):
        return {"cluster": cl, "task": {"type": role, "index": i}, "environment": "cloud"}

    ps = [_trainer(common, tfc("ps", 0)), _trainer(common, tfc("ps", 1))]
    try:
        first = [_trainer(common + ["--fail-at-step", "4"], tfc("master", 0)),
                 _trainer(common + ["--fail-at-step", "4"], tfc("worker", 0))]
        for p in first:
            out, _ = p.communicate(timeout=300)
            assert p.returncode >= 128, out
        assert ckpt.latest_checkpoint(run) is None  # nothing on disk: only the PS tasks hold the state
        for addr in cluster["ps"]:
            info = call(addr, {"op": "vinfo"})
            assert info["committed"] == [3], info  # older versions were dropped once 3 was committed everywhere
            assert {n for _, n, _ in info["shards"]} >= {"params", "optim/exp_avg", "optim/exp_avg_sq"}
        again = [_trainer(common + ["--fail-at-step", "4"], tfc("master", 0)),
                 _trainer(common + ["--fail-at-step", "4"], tfc("worker", 0))]  # markers: no second failure
        outs = []
        for p in again:
            out, _ = p.communicate(timeout=300)
            outs.append(out)
            assert p.returncode == 0, out
        ev = _events(outs[0])
        restored = [e for e in ev if e["event"] == "restored"]
        assert restored and restored[0]["source"] == "ps" and restored[0]["step"] == 3, restored
        assert [e for e in ev if e["event"] == "step0"][0]["step"] == 4
        for p in ps:  # the master shuts the PS tasks down after its last snapshot
            out, _ = p.communicate(timeout=120)
            assert p.returncode == 0, out
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    # an uninterrupted 2-rank run reaches the same weights and optimizer state
    ref_cluster = {"master": ["127.0.0.1:%d" % rm], "worker": ["127.0.0.1:%d" % rw]}
    ref = str(tmp_path / "ref")
    rargs = [a if a != run else ref for a in common]
    procs = [_trainer(rargs, tfc("master", 0, ref_cluster)), _trainer(rargs, tfc("worker", 0, ref_cluster))]
    for p in procs:
        out, _ = p.communicate(timeout=300)
        assert p.returncode == 0, out
    _, a, _ = ckpt.load(ckpt.latest_checkpoint(ref))
    _, b, _ = ckpt.load(ckpt.latest_checkpoint(run))
    for k in a:
        if k.startswith(("params/", "optim/", "buffers/")):
            torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-6, msg=k)


def test_ps_shard_ranges_cover_and_align():
    from k8s_amd.parallel.ps_vars import shard_ranges

    for n, parts in [(1000, 3), (64, 4), (5, 2), (4096 * 7 + 3, 5)]:
        r = shard_ranges(n, parts)
        assert len(r) == parts and r[0][0] == 0 and r[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        assert all(lo % 64 == 0 for lo, _ in r if lo < n)


def _ps_tasks(n):
    """n in-process default-PS task servers on free ports; returns (addresses, servers)."""
    import threading

    from k8s_amd.ps_server.grpc_tensorflow_server import TaskServer

    srvs, addrs = [], []
    for j in range(n):
        port = free_port()
        s = TaskServer(("127.0.0.1", port), "ps", j)
        threading.Thread(target=s.serve_forever, daemon=True).start()
        srvs.append(s)
        addrs.append("127.0.0.1:%d" % port)
    return addrs, srvs


def test_ps_snapshot_survives_a_chief_that_dies_mid_push():
    """a push of version v+1 must never destroy the committed version v. Three crash points
    of the two-phase push -- some shards of v+1 put on one task only, v+1 committed on one task only, v+1 committed
    everywhere but the old version not yet dropped -- each leave a whole snapshot readable on every task."""
    from k8s_amd.parallel.ps_vars import PsVariables, shard_ranges
    from k8s_amd.ps_server.grpc_tensorflow_server import call

    addrs, srvs = _ps_tasks(2)
    try:
        psv = PsVariables(addrs)
        v1 = {"params": torch.arange(1000, dtype=torch.float32), "optim/m": torch.full((300,), 2.0)}
        psv.push(1, v1, meta={"total": 1000})
        psv.wait()
        assert psv.latest()[0] == 1

        # (1) the chief dies in phase 1: part of version 2 reached task 0 only
        lo, hi = shard_ranges(1000, 2)[0]
        a = (torch.arange(1000, dtype=torch.float32) * -1).numpy()
        assert call(addrs[0], {"op": "vput", "name": "params", "lo": lo, "n": hi - lo, "version": 2},
                    payload=memoryview(a[lo:hi]))["ok"]
        v, meta = psv.latest()
        assert v == 1 and meta["total"] == 1000
        got = psv.pull(1)
        assert torch.equal(got["params"], v1["params"]) and torch.equal(got["optim/m"], v1["optim/m"])

        # (2) the chief dies in phase 2: version 2 committed on task 0 only
        assert call(addrs[0], {"op": "vcommit", "version": 2, "names": [["params", lo]], "meta": {}})["ok"]
        assert psv.latest()[0] == 1
        assert torch.equal(psv.pull(1)["params"], v1["params"])

        # (3) the chief dies between phase 2 and the old version's GC: both versions readable, newest wins
        v2 = {"params": torch.arange(1000, dtype=torch.float32) + 0.5, "optim/m": torch.full((300,), 3.0)}

        def die(stage):
            raise SystemExit("chief killed after %s" % stage)

        psv.fault_hook = die
        psv.push(2, v2, meta={"total": 1000})
        with pytest.raises(SystemExit):
            psv.wait()
        assert psv.latest()[0] == 2
        assert torch.equal(psv.pull(2)["params"], v2["params"])
        assert torch.equal(psv.pull(1)["params"], v1["params"])  # not dropped: GC never ran

        # a later complete push drops everything older than itself
        psv.fault_hook = None
        psv.push(3, v2, meta={"total": 1000})
        psv.wait()
        for addr in addrs:
            assert call(addr, {"op": "vinfo"})["committed"] == [3]
        with pytest.raises(RuntimeError):
            psv.pull(1)
    finally:
        for s in srvs:
            s.shutdown()
            s.server_close()


def test_default_ps_ignores_unknown_flags():
    """The reference's default PS parses with parse_known_args (grpc_tensorflow_server.py:159): extra flags from a
    user's PS template must not crash the pod."""
    from k8s_amd.ps_server import grpc_tensorflow_server as srv

    a, unknown = srv.build_parser().parse_known_args(
        ["--cluster_spec", "ps|127.0.0.1:1", "--job_name", "ps", "--task_id", "0", "--log_dir", "/tmp/x", "--foo"])
    assert a.job_name == "ps" and unknown == ["--log_dir", "/tmp/x", "--foo"]


def test_corrupted_gradient_transport_fails_the_job_at_step_0(tmp_path):
    """with a deliberately wrong reduction (K8S_AMD_FAULT_TRANSPORT) both ranks fail the
    step-0 transport self-check together and exit with a permanent code, before any training step."""
    pm, pw = _distinct_ports(2)
    cluster = {"master": ["127.0.0.1:%d" % pm], "worker": ["127.0.0.1:%d" % pw]}
    common = ["--model", "resnet_tiny", "--steps", "2", "--log-every", "1", "--grad-comm", "bf16"]
    procs = [_trainer(common, {"cluster": cluster, "task": {"type": t, "index": 0}, "environment": "cloud"},
                      K8S_AMD_FAULT_TRANSPORT="1") for t in ("master", "worker")]
    for p in procs:
        out, _ = p.communicate(timeout=300)
        assert 0 < p.returncode < 128, out
        ev = _events(out)
        assert not [e for e in ev if e.get("event") in ("step0", "step")], out[-2000:]
    checks = [e for e in _events(out) if e.get("event") == "transport_check"]
    assert checks and checks[0]["ok"] is False
