"""bench.py and the collective benchmark under torch.distributed.run with 2 gloo ranks on CPU.

The driver launches ``bench.py`` exactly this way on an 8-GPU node (one rank per GPU over RCCL); this pins
the JSON-line contract and the multi-rank path (broadcast, bucketed all-reduce, MAX-over-ranks timing)."""
import json
import os
import subprocess
import sys

from k8s_amd.fakeapi.server import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, args, nproc=2, timeout=300):
    env = dict(os.environ)
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, script)] + args
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
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


def test_bench_eight_ranks_like_the_driver():
    """the driver's 8-GPU launch (torch.distributed.run, 8 ranks, one per GPU) rehearsed
    with 8 gloo ranks on the CPU: one JSON line, dp8, the whole-job value, identical replicas after the steps."""
    recs = _run("bench.py", ["--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "2", "--image", "32"],
                nproc=8, timeout=600)
    assert len(recs) == 1, recs
    r = recs[0]
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "dp8" and r["config"]["global_batch"] == 16
    assert abs(r["value"] - 16 * 2 / (r["ms_per_step"] * 2 / 1000.0)) / r["value"] < 0.02
    assert r["replicas_identical"] is True


def test_collectives_bench_busbw():
    recs = _run("benchmarks/collectives.py", ["--device", "cpu", "--sizes-mb", "0.25", "--iters", "2",
                                              "--warmup", "1"])
    ops = {r["op"] for r in recs}
    assert ops == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    for r in recs:
        assert r["n"] == 2 and r["busbw_GBs"] > 0
        f = 1.0 if r["op"] == "all_reduce" else 0.5  # 2(n-1)/n and (n-1)/n at n=2
        assert abs(r["busbw_GBs"] - r["algbw_GBs"] * f) <= 1e-3
