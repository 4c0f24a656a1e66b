"""RCCL on the test box's GPU: a one-rank ``nccl`` process group with the transports force-enabled
(``tests/rccl_worker.py``), and ``bench.py --force-dist`` recording ``comm.backend == "nccl"``. Every collective the
data-parallel and parameter-service transports issue runs as an RCCL kernel here, including the side-stream
ordering of the bf16 push (device-side ``Work.wait`` on a non-current stream) and the ZeRO-1 pull that the next
forward waits for lazily (``Param.weight``). Anchor: the reference's data plane is the distributed runtime between
replicas (`/root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:93`,
`/root/reference/examples/tf_sample/tf_sample/tf_smoke.py:100-118`)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG", "K8S_AMD_DIST_BACKEND",
              "K8S_AMD_GPU_OVERSUBSCRIBE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable] + args, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


@pytest.fixture(scope="module")
def rccl():
    (rec,) = _run([os.path.join(REPO, "tests", "rccl_worker.py")])
    return rec


def test_rccl_group_initialises(rccl):
    assert rccl["backend"] == "nccl" and rccl["world"] == 1


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_grad_reducer_over_rccl_is_exact(rccl, comm):
    r = rccl["reducer_" + comm]
    assert r["check"]["ok"] and r["check"]["transport"] == "allreduce-" + comm, r["check"]
    assert r["buckets"] > 3
    assert r["max_abs_err"] == 0.0, r
    assert r["reserved"][-1] == r["reserved"][1], r["reserved"]


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_sharded_service_over_rccl_is_exact(rccl, comm):
    r = rccl["service_" + comm]
    assert r["sharded"] and r["pull"] == "lowp"
    assert r["check"]["ok"] and r["check"]["pull"]["ok"], r["check"]
    assert r["max_abs_err_master"] == 0.0 and r["max_abs_err_half"] == 0.0, r
    assert r["reserved"][-1] == r["reserved"][1], r["reserved"]
    if comm == "bf16":
        assert r["pool_bytes"] > 0


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_bench_force_dist_runs_rccl(comm):
    (r,) = _run(["bench.py", "--force-dist", "--grad-comm", comm, "--steps", "2", "--warmup", "1", "--batch", "32",
                 "--image", "64"])
    assert r["comm"]["backend"] == "nccl" and r["comm"]["world_size"] == 1
    assert r["transport_check"]["ok"] and r["transport_check"]["transport"] == "allreduce-" + comm
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["final_loss"] == r["final_loss"]
