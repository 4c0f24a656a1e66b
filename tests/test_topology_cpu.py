"""BASELINE config 2's topology end to end on the CPU: ``examples/tf_job_resnet50_ps.yaml`` itself (1 MASTER + 7
WORKER, one ``amd.com/gpu`` each, + 2 default PS) through the local cluster (fake API server + kubelet with an
8-id GPU pool + the C++ operator) to Done/Succeeded -- the reference's e2e shape (MASTER + PS + WORKER driven to
Succeeded, `/root/reference/test/e2e/main.go:49-123`) at the rank count of the 8-GPU node. Only the model
(resnet_tiny), the step count and ``--device cpu`` (gloo) differ from the example."""
import io
import json
import os

import pytest
import yaml

from k8s_amd import cli
from k8s_amd.fakeapi.cluster import OPERATOR_BIN, LocalCluster

pytestmark = pytest.mark.skipif(not os.path.exists(OPERATOR_BIN), reason="bin/tf_operator not built")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(c, *argv):
    out = io.StringIO()
    rc = cli.main(["--server", c.url] + list(argv), out=out)
    return rc, out.getvalue()


def test_resnet50_ps_example_topology_runs_to_succeeded(tmp_path):
    with open(os.path.join(REPO, "examples", "tf_job_resnet50_ps.yaml")) as f:
        job = yaml.safe_load(f)
    logdir = str(tmp_path / "logs")
    ntrain = 0
    for spec in job["spec"]["replicaSpecs"]:
        if spec["tfReplicaType"] == "PS":
            assert "template" not in spec and spec["replicas"] == 2  # the default PS server
            continue
        ntrain += spec["replicas"]
        c0 = spec["template"]["spec"]["containers"][0]
        assert c0["resources"]["limits"]["amd.com/gpu"] == 1
        args = ["resnet_tiny" if a == "resnet50" else a for a in c0["args"]]
        args[args.index("--steps") + 1] = "3"
        args += ["--device", "cpu", "--log-every", "1", "--ps-sync-every", "2", "--batch", "2"]
        if spec["tfReplicaType"] == "MASTER":
            args += ["--logdir", logdir]
        c0["args"] = args
    assert ntrain == 8
    f = tmp_path / "job.yaml"
    f.write_text(yaml.safe_dump(job))
    with LocalCluster(gpus=list(range(8))) as c:
        c.kubelet.extra_env.update({"CUDA_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "1"})
        rc, out = _cli(c, "create", "-f", str(f))
        assert rc == 0, out
        rc, out = _cli(c, "wait", "resnet50-ps", "--timeout", "420", "--interval", "0.5")
        if rc != 0:
            logs = "\n".join(c.kubelet.pod_log(p["metadata"]["name"])[-1200:] for p in c.pods())
            pytest.fail(out + c.operator_log()[-2000:] + logs)
        assert "state=Succeeded" in out
        pods = c.pods()
        assert len(pods) == 10
        # every trainer pod got its own GPU id from the pool (HIP_VISIBLE_DEVICES), PS pods none
        used = sorted(v for vs in c.kubelet.gpu_history.values() for v in vs)
        assert used == list(range(8)), c.kubelet.gpu_history
    ev = [json.loads(line) for line in open(os.path.join(logdir, "metrics.jsonl"))]
    start = [e for e in ev if e["event"] == "start"][0]
    assert start["world"] == 8 and start["strategy"] == "ps" and start["zero1"] is True
    assert [e for e in ev if e["event"] == "ps_snapshot"][0]["step"] == 2  # committed on both PS tasks
    done = [e for e in ev if e["event"] == "done"][0]
    assert done["steps"] == 3 and done["loss"] == done["loss"]


MULTI = """
apiVersion: "tensorflow.org/v1alpha1"
kind: "TfJob"
metadata:
  name: "multi-gpu"
spec:
  replicaSpecs:
    - replicas: 1
      tfReplicaType: MASTER
      template:
        spec:
          containers:
            - image: k8s-amd/trainer:rocm7-gfx950
              name: tensorflow
              args: {args}
              resources:
                limits:
                  amd.com/gpu: 2
          restartPolicy: OnFailure
    - replicas: 1
      tfReplicaType: WORKER
      template:
        spec:
          containers:
            - image: k8s-amd/trainer:rocm7-gfx950
              name: tensorflow
              args: {args}
              resources:
                limits:
                  amd.com/gpu: 2
          restartPolicy: OnFailure
"""


@pytest.mark.parametrize("extra", [[], ["--zero", "1", "--optimizer", "adam", "--lr", "0.001"]])
def test_replicas_with_two_gpus_each_train_as_four_ranks(tmp_path, extra):
    """a replica given n GPUs runs n trainer processes (one per GPU, LOCAL_RANK i). A
    MASTER and a WORKER with ``amd.com/gpu: 2`` each (kubelet pool of 4 ids) train as world 4, the ranks ordered
    master 0-1, worker 2-3 (``TFJOB_TASK_GPUS`` from the operator), and all four replicas end bit-identical."""
    args = json.dumps(["--model", "resnet_tiny", "--steps", "3", "--device", "cpu", "--log-every", "1",
                       "--batch", "2"] + extra)
    f = tmp_path / "job.yaml"
    f.write_text(MULTI.format(args=args))
    with LocalCluster(gpus=[0, 1, 2, 3]) as c:
        c.kubelet.extra_env.update({"CUDA_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "1"})
        rc, out = _cli(c, "create", "-f", str(f))
        assert rc == 0, out
        rc, out = _cli(c, "wait", "multi-gpu", "--timeout", "300", "--interval", "0.5")
        logs = {p["metadata"]["name"]: c.kubelet.pod_log(p["metadata"]["name"]) for p in c.pods()}
        if rc != 0:
            pytest.fail(out + c.operator_log()[-2000:] + "\n".join(v[-1500:] for v in logs.values()))
        assert "state=Succeeded" in out
        assert sorted(len(v) for v in c.kubelet.gpu_history.values()) == [2, 2]
    ev = []
    for text in logs.values():
        for line in text.splitlines():
            if line.startswith("{"):
                try:
                    ev.append(json.loads(line))
                except ValueError:
                    pass
    starts = [e for e in ev if e.get("event") == "start"]
    assert sorted(e["rank"] for e in starts) == [0, 1, 2, 3] and {e["world"] for e in starts} == {4}
    done = [e for e in ev if e.get("event") == "done"]
    assert sorted(e["rank"] for e in done) == [0, 1, 2, 3]
    assert len({e["weights_sum"] for e in done}) == 1, done  # DP replicas bit-identical
