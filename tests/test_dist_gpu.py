"""The multi-rank training path on the GPU kernels: two ranks share the one GPU of the test box
(``K8S_AMD_GPU_OVERSUBSCRIBE=1``) and talk over gloo (``K8S_AMD_DIST_BACKEND=gloo``; RCCL refuses two ranks on
one device). What runs is exactly the driver's ``torch.distributed.run ... bench.py --gpus N`` path -- env
rendezvous, rank-0 broadcast, bucketed all-reduce hooks overlapped with the HIP backward, fused SGD, MAX-over-ranks
timing -- with only the transport swapped; RCCL itself is exercised by the driver's 8-GPU run."""
import json
import os
import subprocess
import sys

import pytest

from k8s_amd.fakeapi.server import free_port

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(script, args, nproc=2, timeout=240):
    env = dict(os.environ)
    env.update(K8S_AMD_GPU_OVERSUBSCRIBE="1", K8S_AMD_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, script)] + args
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


@pytest.mark.parametrize("mode", ["allreduce-fp32", "allreduce-bf16", "zero-bf16"])
def test_dp_replicas_stay_identical_on_gpu(mode):
    """All-reduce (fp32, and bf16 transport with its side-stream sum / all-gather / expansion) and the ZeRO-1
    service with the bf16 all-to-all push: after 3 steps every rank holds the same weights."""
    (rec,) = _torchrun("tests/dist_gpu_worker.py", [mode])
    assert rec["world"] == 2 and rec["replicas_identical"] == 1
    assert rec["loss"] == rec["loss"]


def test_zero_bf16_pull_matches_fp32_pull_on_gpu():
    """The ZeRO-1 bf16 working-copy pull (the GPU default: bucket-wise bf16 all-gather waited per bucket by the next
    forward, fp32 master sharded) trains bit-identically to the fp32-master pull on the GPU kernels."""
    (a,) = _torchrun("tests/dist_gpu_worker.py", ["zero-bf16"])
    (b,) = _torchrun("tests/dist_gpu_worker.py", ["zero-fp32pull-bf16"])
    assert (a["pull"], b["pull"]) == ("lowp", "fp32")
    assert a["replicas_identical"] == 1 and b["replicas_identical"] == 1
    assert a["wsum"] == b["wsum"] and a["loss"] == b["loss"]


def test_bench_two_ranks_on_gpu():
    (r,) = _torchrun("bench.py", ["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "16", "--image", "64"])
    assert r["n_gpus"] == 2 and r["dtype"] == "bf16" and r["config"]["parallelism"] == "dp2"
    assert r["config"]["global_batch"] == 32 and r["value"] > 0 and r["final_loss"] == r["final_loss"]


@pytest.mark.parametrize("mode", ["zero-bf16", "allreduce-bf16"])
def test_bf16_transport_memory_flat_on_gpu(mode):
    """The bf16 transports reuse one send / recv buffer pair per bucket (``parallel/ps.py`` CommBufferPool) instead
    of per-step allocations kept alive with ``record_stream``: the caching allocator's reservation is flat from the
    second step to the tenth on the 2-rank path."""
    (rec,) = _torchrun("tests/dist_gpu_worker.py", [mode, "10"])
    assert rec["replicas_identical"] == 1
    res = rec["reserved"]
    assert len(res) == 10 and res[-1] == res[1], res
