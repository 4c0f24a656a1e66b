"""`tfjob` CLI + trainer through the local cluster (fake API server + kubelet + C++ operator), on CPU.

The SURVEY §7.4 slice minus the GPU: create -f -> operator -> Services/Jobs with TF_CONFIG -> kubelet
starts MASTER + WORKER trainers (gloo, sharded-PS strategy) and the default PS server -> training,
tfevents, checkpoints -> master exits 0 and shuts the PS down -> TfJob Done/Succeeded; then get/describe/
pods/logs/delete through the CLI.
"""
import io
import os
import time

import pytest

from k8s_amd import cli
from k8s_amd.fakeapi.cluster import OPERATOR_BIN, LocalCluster
from k8s_amd.utils import checkpoint as ckpt

pytestmark = pytest.mark.skipif(not os.path.exists(OPERATOR_BIN), reason="bin/tf_operator not built")

JOB = """
apiVersion: "tensorflow.org/v1alpha1"
kind: "TfJob"
metadata:
  name: "tiny-train"
spec:
  tensorboard:
    logDir: {logdir}
  replicaSpecs:
    - replicas: 1
      tfReplicaType: MASTER
      template:
        spec:
          containers:
            - image: k8s-amd/trainer:rocm7-gfx950
              name: tensorflow
              args: ["--model", "resnet_tiny", "--steps", "4", "--strategy", "ps", "--device", "cpu",
                     "--log-every", "1", "--logdir", "{logdir}", "--ckpt-dir", "{ckpt}"]
          restartPolicy: OnFailure
    - replicas: 1
      tfReplicaType: WORKER
      template:
        spec:
          containers:
            - image: k8s-amd/trainer:rocm7-gfx950
              name: tensorflow
              args: ["--model", "resnet_tiny", "--steps", "4", "--strategy", "ps", "--device", "cpu",
                     "--log-every", "1", "--ckpt-dir", "{ckpt}"]
          restartPolicy: OnFailure
    - replicas: 1
      tfReplicaType: PS
"""


def _cli(c, *argv):
    out = io.StringIO()
    rc = cli.main(["--server", c.url] + list(argv), out=out)
    return rc, out.getvalue()


def test_cli_trainer_job(tmp_path):
    logdir, ck = str(tmp_path / "logs"), str(tmp_path / "ckpt")
    f = tmp_path / "job.yaml"
    f.write_text(JOB.format(logdir=logdir, ckpt=ck))
    with LocalCluster() as c:
        c.kubelet.extra_env.update({"CUDA_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "2"})
        rc, out = _cli(c, "create", "-f", str(f))
        assert rc == 0 and 'tfjob "tiny-train" created' in out
        rc, out = _cli(c, "create", "-f", str(f))
        assert rc == 1  # AlreadyExists
        rc, out = _cli(c, "wait", "tiny-train", "--timeout", "240", "--interval", "0.3")
        if rc != 0:
            logs = "\n".join(c.kubelet.pod_log(p["metadata"]["name"])[-1500:] for p in c.pods())
            pytest.fail(out + c.operator_log()[-2000:] + logs)
        assert "state=Succeeded" in out
        rc, out = _cli(c, "get", "tfjobs")
        assert rc == 0 and out.splitlines()[0].split()[:3] == ["NAME", "PHASE", "STATE"]
        assert "tiny-train" in out and "Done" in out and "Succeeded" in out
        rc, out = _cli(c, "get", "tfjobs", "tiny-train", "-o", "yaml")
        assert rc == 0 and "kind: TfJob" in out and "RuntimeId:" in out
        rc, out = _cli(c, "get", "tfjobs", "-o", "wide")
        assert "MASTER:" in out
        rc, out = _cli(c, "describe", "tiny-train")
        assert rc == 0 and "PS" in out and "(default PS)" in out
        end = time.time() + 30  # the PS pods stop right after the master (it shuts them down)
        while True:
            rc, out = _cli(c, "pods", "tiny-train")
            rows = out.splitlines()[1:]
            if all("Succeeded" in r for r in rows) or time.time() > end:
                break
            time.sleep(0.3)
        assert len(rows) == 3 and all("Succeeded" in r for r in rows), out
        master = next(r.split()[0] for r in rows if "MASTER" in r)
        rc, out = _cli(c, "logs", master)
        assert rc == 0 and '"event": "done"' in out
        # outputs of the chief
        assert any(n.startswith("events.out.tfevents.") for n in os.listdir(logdir))
        assert ckpt.read_state(ck)[0] == "model.ckpt-3"
        rc, out = _cli(c, "delete", "tfjob", "tiny-train")
        assert rc == 0
        end = time.time() + 20
        while time.time() < end and c.client.get("/api/v1/namespaces/default/pods")["items"]:
            time.sleep(0.2)
        assert not c.client.get("/api/v1/namespaces/default/pods")["items"]
        rc, _ = _cli(c, "get", "tfjobs", "tiny-train")
        assert rc == 1


def test_examples_default_and_validate():
    """Every shipped example manifest parses, defaults and validates (the CLI's create path)."""
    import glob
    import json

    from k8s_amd import _operator as op
    from k8s_amd.fakeapi.cluster import REPO, load_manifests

    files = sorted(glob.glob(os.path.join(REPO, "examples", "*.yaml")))
    assert len(files) >= 8
    for f in files:
        for d in load_manifests(f):
            assert d["kind"] == "TfJob" and d["apiVersion"] == "tensorflow.org/v1alpha1", f
            spec, err = op.set_defaults(json.dumps(d["spec"]))
            assert err == "", (f, err)
            assert op.validate(spec) == "", f
