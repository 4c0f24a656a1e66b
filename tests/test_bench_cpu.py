"""bench.py and the collective benchmark under torch.distributed.run with 2 gloo ranks on CPU.

The driver launches ``bench.py`` exactly this way on an 8-GPU node (one rank per GPU over RCCL); this pins
the JSON-line contract and the multi-rank path (broadcast, bucketed all-reduce, MAX-over-ranks timing)."""
import json
import os
import subprocess
import sys

from k8s_amd.fakeapi.server import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = dict(os.environ)
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(script, args, nproc=2, timeout=300, launcher=True):
    cmd = [sys.executable, os.path.join(REPO, script)] + args
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, script)] + args
    r = subprocess.run(cmd, env=_env(), cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def test_bench_two_ranks_json_contract():
    recs = _run("bench.py", ["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "2", "--image", "64"])
    assert len(recs) == 1, recs  # rank 0 only, one line
    r = recs[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["global_batch"] == 4 and r["config"]["parallelism"] == "dp2"
    assert r["higher_is_better"] is True and r["scaling"] == "weak"
    # value is the whole-job aggregate: images / (max rank time)
    assert abs(r["value"] - 4 * 2 / (r["ms_per_step"] * 2 / 1000.0)) / r["value"] < 0.02
    assert r["final_loss"] == r["final_loss"]


def test_bench_eight_ranks_without_a_launcher():
    """``python bench.py --gpus 8`` with no torchrun starts its 8 local ranks itself (before
    any GPU call), rehearsed with 8 gloo ranks on the CPU: one JSON line, dp8, the whole-job value, identical
    replicas after the steps, and the exposed-communication time."""
    recs = _run("bench.py", ["--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "2", "--image", "32"],
                timeout=600, launcher=False)
    assert len(recs) == 1, recs
    r = recs[0]
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "dp8" and r["config"]["global_batch"] == 16
    assert abs(r["value"] - 16 * 2 / (r["ms_per_step"] * 2 / 1000.0)) / r["value"] < 0.02
    assert r["replicas_identical"] is True
    assert r["comm_exposed_ms"] >= 0 and r["grad_comm_fallbacks"] == {}
    # the record shows what the process group really ran on, and the step-0 transport
    # check passed for the full world
    assert r["comm"]["backend"] == "gloo" and r["comm"]["world_size"] == 8
    assert r["transport_check"]["ok"] is True and r["transport_check"]["world"] == 8
    assert r["transport_check"]["transport"] == "allreduce-fp32"


def _run_fail(args, nproc, **env_extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py")] + args
    return subprocess.run(cmd, env=_env(**env_extra), cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          text=True, timeout=300)


def test_bench_bf16_transport_self_check_passes_and_reports():
    recs = _run("bench.py", ["--gpus", "4", "--steps", "1", "--warmup", "1", "--batch", "2", "--image", "32",
                             "--grad-comm", "bf16"], nproc=4)
    r = recs[0]
    assert r["transport_check"]["ok"] is True and r["transport_check"]["transport"] == "allreduce-bf16"
    assert r["transport_check"]["max_err_over_tol"] < 1.0 and r["comm"]["world_size"] == 4


def test_bench_corrupted_transport_exits_nonzero():
    """A deliberately wrong reduction (K8S_AMD_FAULT_TRANSPORT: MAX instead of SUM for fp32, one rank's bf16 slice
    dropped) is caught by the step-0 self-check: exit 3 before any timed step, no JSON line."""
    for comm in ("fp32", "bf16"):
        r = _run_fail(["--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "2", "--image", "32",
                       "--grad-comm", comm], 2, K8S_AMD_FAULT_TRANSPORT="1")
        assert r.returncode != 0, (comm, r.stdout, r.stderr)
        assert not [line for line in r.stdout.splitlines() if line.startswith("{")]
        assert "transport self-check failed" in r.stderr, r.stderr[-2000:]


def test_bench_world_mismatch_fails_closed():
    """A world that is not the one asked for (here a single-rank env with --gpus 2) exits non-zero and prints no
    JSON line, instead of reporting a 1-GPU number as a 2-GPU one."""
    env = _env(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "0", "--batch", "2", "--image", "32"], env=env, cwd=REPO, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode != 0
    assert not [line for line in r.stdout.splitlines() if line.startswith("{")]
    assert "world size 1" in r.stderr


def test_collectives_bench_busbw():
    recs = _run("benchmarks/collectives.py", ["--device", "cpu", "--sizes-mb", "0.25", "--iters", "2",
                                              "--warmup", "1"])
    ops = {r["op"] for r in recs}
    assert ops == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    for r in recs:
        assert r["n"] == 2 and r["busbw_GBs"] > 0
        f = 1.0 if r["op"] == "all_reduce" else 0.5  # 2(n-1)/n and (n-1)/n at n=2
        assert abs(r["busbw_GBs"] - r["algbw_GBs"] * f) <= 1e-3
