"""Semantic ports of the reference Go unit tests (pkg/spec/tf_job_test.go,
pkg/trainer/replicas_test.go, training_test.go, tensorboard_test.go) against
the C++ control plane (k8s_amd._operator) and the in-memory API server.

Same inputs, same expected names / labels / owner references / TF_CONFIG /
states. Deliberate differences are called out inline.
"""
import json

import pytest

op = pytest.importorskip("k8s_amd._operator")

from k8s_amd.fakeapi.store import ApiStore  # noqa: E402


def container(name="tensorflow", **kw):
    c = {"name": name}
    c.update(kw)
    return c


def template(*containers):
    return {"spec": {"containers": list(containers)}}


ACC_CFG = {"accelerators": {"nvidia-gpu": {"volumes": [
    {"name": "cuda-lib", "hostPath": "/home/cuda", "mountPath": "/usr/local/cuda"}]}}}


# --------------------------------------------------------------------------- TestAddAccelertor
@pytest.mark.parametrize("where", ["requests", "limits"])
def test_configure_accelerators_requests_and_limits(where):
    spec = {"replicaSpecs": [{"replicas": 2, "tfPort": 10, "tfReplicaType": "PS",
                              "template": template(container(resources={where: {"nvidia-gpu": "1"}}))}]}
    out, err = op.configure_accelerators(json.dumps(spec), json.dumps(ACC_CFG))
    assert err == ""
    r = json.loads(out)["replicaSpecs"][0]
    pod = r["template"]["spec"]
    assert pod["volumes"] == [{"name": "cuda-lib", "hostPath": {"path": "/home/cuda"}}]
    assert pod["containers"][0]["volumeMounts"] == [{"name": "cuda-lib", "mountPath": "/usr/local/cuda"}]
    assert pod["containers"][0]["resources"] == {where: {"nvidia-gpu": "1"}}
    assert r["replicas"] == 2 and r["tfPort"] == 10


def test_configure_accelerators_no_accelerator_unchanged():
    spec = {"replicaSpecs": [{"replicas": 2, "tfPort": 10, "tfReplicaType": "PS",
                              "template": template(container())}]}
    out, err = op.configure_accelerators(json.dumps(spec), json.dumps(ACC_CFG))
    assert err == ""
    pod = json.loads(out)["replicaSpecs"][0]["template"]["spec"]
    assert "volumes" not in pod and "volumeMounts" not in pod["containers"][0]


def test_configure_accelerators_amd_gpu_rocm():
    """The MI355X deployment: amd.com/gpu limit -> ROCm user-space mounts + env, tensorflow container only."""
    cfg = {"accelerators": {"amd.com/gpu": {
        "volumes": [{"name": "rocm", "hostPath": "/opt/rocm", "mountPath": "/opt/rocm"},
                    {"name": "dri", "hostPath": "/dev/dri", "mountPath": "/dev/dri"}],
        "envVars": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]}}}
    spec = {"replicaSpecs": [{"replicas": 1, "tfPort": 2222, "tfReplicaType": "WORKER",
                              "template": template(container("sidecar", resources={"limits": {"amd.com/gpu": 1}}),
                                                   container(resources={"limits": {"amd.com/gpu": 8}}))}]}
    out, err = op.configure_accelerators(json.dumps(spec), json.dumps(cfg))
    assert err == ""
    pod = json.loads(out)["replicaSpecs"][0]["template"]["spec"]
    assert [v["name"] for v in pod["volumes"]] == ["rocm", "dri"]
    side, tf = pod["containers"]
    assert "volumeMounts" not in side and "env" not in side
    assert tf["env"] == [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]
    assert [m["mountPath"] for m in tf["volumeMounts"]] == ["/opt/rocm", "/dev/dri"]


# --------------------------------------------------------------------------- TestSetDefaults
def test_set_defaults_master():
    spec = {"replicaSpecs": [{"template": template(container())}], "tfImage": "tensorflow/tensorflow:1.3.0"}
    out, err = op.set_defaults(json.dumps(spec))
    assert err == ""
    s = json.loads(out)
    assert s["replicaSpecs"][0] == {"replicas": 1, "template": template(container()), "tfPort": 2222,
                                    "tfReplicaType": "MASTER", "IsDefaultPS": False}
    assert s["tfImage"] == "tensorflow/tensorflow:1.3.0"
    assert s["terminationPolicy"] == {"chief": {"replicaName": "MASTER", "replicaIndex": 0}}


def test_set_defaults_default_ps():
    spec = {"replicaSpecs": [{"tfReplicaType": "PS"}], "tfImage": "tensorflow/tensorflow:1.3.0"}
    s = json.loads(op.set_defaults(json.dumps(spec))[0])
    r = s["replicaSpecs"][0]
    assert r["IsDefaultPS"] is True
    assert r["replicas"] == 1 and r["tfPort"] == 2222
    c = r["template"]["spec"]["containers"][0]
    assert c["name"] == "tensorflow" and c["image"] == "tensorflow/tensorflow:1.3.0"
    assert c["volumeMounts"] == [{"name": "ps-config-volume", "mountPath": "/ps-server"}]
    assert r["template"]["spec"]["restartPolicy"] == "OnFailure"


def test_set_defaults_image_default():
    s = json.loads(op.set_defaults(json.dumps({"replicaSpecs": [{"template": template(container())}]}))[0])
    # deliberate: our default image is the ROCm trainer, not tensorflow/tensorflow:1.3.0 (pkg/spec/tf_job.go:87)
    assert s["tfImage"] == op.DEFAULT_TF_IMAGE


def test_validate_messages():
    base = {"replicaSpecs": [{"replicas": 2, "tfPort": 2222, "tfReplicaType": "MASTER",
                              "template": template(container())}]}
    assert op.validate(json.dumps(base)) == "The MASTER must have Replicas = 1"
    no_port = {"replicaSpecs": [{"replicas": 1, "tfReplicaType": "MASTER", "template": template(container())}]}
    assert op.validate(json.dumps(no_port)) == "tfReplicaSpec.TfPort can't be nil."
    bad_c = {"replicaSpecs": [{"replicas": 1, "tfPort": 1, "tfReplicaType": "WORKER", "template": template(container("x"))}]}
    assert op.validate(json.dumps(bad_c)) == "Replica type WORKER is missing a container named tensorflow"
    bad_t = {"replicaSpecs": [{"replicas": 1, "tfPort": 1, "tfReplicaType": "CHIEF", "template": template(container())}]}
    assert "must be one of [MASTER PS WORKER]" in op.validate(json.dumps(bad_t))
    bad_chief = {"replicaSpecs": [], "terminationPolicy": {"chief": {"replicaName": "WORKER", "replicaIndex": 0}}}
    assert op.validate(json.dumps(bad_chief)) == \
        "invalid termination policy, Chief should have replicaName=MASTER and index=0"
    # PS-only specs are accepted (Q8, pkg/trainer/training_test.go:187-211)
    ps_only = {"replicaSpecs": [{"replicas": 2, "tfPort": 10, "tfReplicaType": "PS", "template": template(container())}]}
    assert op.validate(json.dumps(ps_only)) == ""


def test_wire_format_go_names():
    j = {"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob", "metadata": {"name": "x"},
         "spec": {"replicaspecs": [{"TFREPLICATYPE": "WORKER", "tfport": 5}], "TensorBoard": {"logDir": "/l"}}}
    out = json.loads(op.normalize_tfjob(json.dumps(j)))
    # case-insensitive decode, Go field names/order on encode
    assert list(out["spec"].keys())[:3] == ["RuntimeId", "tensorboard", "replicaSpecs"]
    assert out["spec"]["replicaSpecs"][0] == {"tfPort": 5, "tfReplicaType": "WORKER", "IsDefaultPS": False}
    assert out["spec"]["tensorboard"] == {"logDir": "/l", "volumes": None, "volumeMounts": None, "serviceType": ""}
    assert out["status"] == {"phase": "", "reason": "", "controlPaused": False, "conditions": None, "state": "",
                             "replicaStatuses": None}
    # snake_case replica_specs is silently ignored (Q11)
    s = json.loads(op.normalize_tfjob(json.dumps({"spec": {"replica_specs": [{"tfReplicaType": "MASTER"}]}})))
    assert s["spec"]["replicaSpecs"] is None


# --------------------------------------------------------------------------- names / TF_CONFIG
def _job(name="some-job", rid="some-runtime", specs=None, uid="some-uid", ns="default"):
    return json.dumps({"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob",
                       "metadata": {"name": name, "uid": uid, "namespace": ns},
                       "spec": {"RuntimeId": rid, "replicaSpecs": specs or []}})


def test_transform_cluster_spec_for_default_ps():
    cs = {"master": ["master-0:2222"], "worker": ["worker-0:2222", "worker-1:2222"],
          "ps": ["localhost:2222", "ps-1:2222"]}
    assert op.default_ps_cluster_spec(cs) == \
        "master|master-0:2222,ps|localhost:2222;ps-1:2222,worker|worker-0:2222;worker-1:2222"


def test_cluster_spec():
    specs = [{"replicas": 2, "tfPort": 22, "tfReplicaType": "PS", "template": template(container())},
             {"replicas": 1, "tfPort": 42, "tfReplicaType": "MASTER", "template": template(container())},
             {"replicas": 3, "tfPort": 40, "tfReplicaType": "WORKER", "template": template(container())}]
    cs = op.cluster_spec(_job("myjob", "runtime", specs))
    assert cs == {"ps": ["myjob-ps-runtime-0:22", "myjob-ps-runtime-1:22"],
                  "master": ["myjob-master-runtime-0:42"],
                  "worker": ["myjob-worker-runtime-0:40", "myjob-worker-runtime-1:40", "myjob-worker-runtime-2:40"]}


def test_tf_config_exact_bytes():
    cs = {"worker": ["w-0:2222"], "master": ["m-0:2222"], "ps": ["p-0:2222", "p-1:2222"]}
    assert op.tf_config(cs, "worker", 0) == (
        '{"cluster":{"master":["m-0:2222"],"ps":["p-0:2222","p-1:2222"],"worker":["w-0:2222"]},'
        '"task":{"type":"worker","index":0},"environment":"cloud"}')


def test_name_truncation_40_runes():
    long = "a" * 50
    assert op.replica_job_name(_job(long, "ab12"), "WORKER", 3) == "a" * 40 + "-worker-ab12-3"
    assert op.tb_name(_job(long, "ab12")) == "a" * 40 + "-tensorboard-ab12"
    assert op.truncate_name("é" * 45) == "é" * 40
    assert op.default_ps_configmap_name(_job(rid="zz99")) == "cm-ps-zz99"


def test_rand_string():
    s = op.rand_string(4)
    assert len(s) == 4 and all(c in "0123456789abcdefghijklmnopqrstuvwxyz" for c in s)


# --------------------------------------------------------------------------- TestIsRetryableTerminationState
@pytest.mark.parametrize("code,reason,want", [(0, "", False), (1, "", False), (127, "", False), (128, "", True),
                                              (244, "", True), (244, "OOMKilled", False), (137, "", True)])
def test_retryable_termination(code, reason, want):
    assert op.is_retryable_termination(code, reason) is want


# --------------------------------------------------------------------------- TestTFReplicaSetStatusFromPodList
def _cs(name, state=None, last=None):
    d = {"name": name, "state": state or {}}
    if last:
        d["lastState"] = last
    return d


@pytest.mark.parametrize("pods,want", [
    ([{"status": {"containerStatuses": [_cs("master", {"running": {}})]}}], "Running"),
    ([{"status": {"containerStatuses": [_cs("master", {"terminated": {"exitCode": 0}})]}}], "Succeeded"),
    ([{"status": {"containerStatuses": [_cs("other", {"running": {}}),
                                        _cs("master", {"terminated": {"exitCode": 0}})]}}], "Succeeded"),
    ([{"status": {"containerStatuses": [_cs("master", {"running": {}},
                                            {"terminated": {"exitCode": 100, "message": "some reason"}})]}}], "Failed"),
    ([{"status": {"startTime": "2016-11-30T00:00:00Z", "containerStatuses": [_cs("master", {"running": {}})]}},
      {"status": {"startTime": "2017-11-30T00:00:00Z",
                  "containerStatuses": [_cs("master", {"terminated": {"exitCode": 100}})]}}], "Failed"),
    ([], "Running"),
    ([{"status": {"containerStatuses": [_cs("master", {"terminated": {"exitCode": 143}})]}}], "Running"),
])
def test_replica_state_from_pods(pods, want):
    assert op.replica_state_from_pods(json.dumps(pods), "master") == want


def test_aggregate_replica_states():
    assert op.aggregate_replica_states({"Failed": 1, "Running": 3}, 4) == "Failed"
    assert op.aggregate_replica_states({"Running": 1, "Succeeded": 3}, 4) == "Running"
    assert op.aggregate_replica_states({"Succeeded": 4}, 4) == "Succeeded"
    assert op.aggregate_replica_states({"Succeeded": 3, "Unknown": 1}, 4) == "Unknown"


# --------------------------------------------------------------------------- TestTFReplicaSet / TestTBReplicaSet
def _reconciler(store, job_json, cfg=None, ps_source=""):
    return op.Reconciler(store.handle, job_json, json.dumps(cfg) if cfg else "", ps_source)


def _seed(store, job):
    code, body = store.post("/apis/apiextensions.k8s.io/v1/customresourcedefinitions", json.loads(op.crd_manifest()))
    assert code == 201
    code, body = store.post("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs", job)
    assert code == 201, body
    return body


def test_replica_set_create():
    store = ApiStore()
    job = _seed(store, {"metadata": {"name": "some-job"}, "spec": {"RuntimeId": "some-runtime", "replicaSpecs": [
        {"replicas": 2, "tfPort": 10, "tfReplicaType": "PS", "template": template(container())}]}})
    r = _reconciler(store, json.dumps(job))
    r.reconcile()
    uid = job["metadata"]["uid"]
    owner = {"apiVersion": "tensorflow.org/v1alpha1", "kind": "TfJob", "name": "some-job", "uid": uid,
             "controller": True, "blockOwnerDeletion": True}
    _, svcs = store.get("/api/v1/namespaces/default/services")
    _, jobs = store.get("/apis/batch/v1/namespaces/default/jobs")
    assert len(svcs["items"]) == 2 and len(jobs["items"]) == 2
    for index in range(2):
        labels = {"tensorflow.org": "", "task_index": str(index), "job_type": "PS", "runtime_id": "some-runtime",
                  "tf_job_name": "some-job"}
        name = "some-job-ps-some-runtime-%d" % index
        s, j = svcs["items"][index], jobs["items"][index]
        assert s["metadata"]["name"] == name and j["metadata"]["name"] == name
        assert s["metadata"]["labels"] == labels and j["metadata"]["labels"] == labels
        assert s["metadata"]["ownerReferences"] == [owner] and j["metadata"]["ownerReferences"] == [owner]
        assert s["spec"]["ports"] == [{"name": "tf-port", "port": 10}] and s["spec"]["selector"] == labels
        assert j["spec"]["completions"] == 1 and j["spec"]["parallelism"] == 1
        cs = j["spec"]["template"]["spec"]["containers"]
        # TF_CONFIG (byte-compatible with the reference) plus our TFJOB_TASK_GPUS (GPUs per task of every replica
        # type, for replicas that drive several local GPUs; the reference's test pins only TF_CONFIG)
        assert len(cs) == 1 and [e["name"] for e in cs[0]["env"]] == ["TF_CONFIG", "TFJOB_TASK_GPUS"]
        assert json.loads(cs[0]["env"][1]["value"]) == {"ps": 0}
        tfc = json.loads(cs[0]["env"][0]["value"])
        # reference test sees an empty cluster because its job was never set up; ours is derived from the spec
        assert tfc == {"cluster": {"ps": ["some-job-ps-some-runtime-0:10", "some-job-ps-some-runtime-1:10"]},
                       "task": {"type": "ps", "index": index}, "environment": "cloud"}
        assert j["spec"]["template"]["metadata"]["labels"] == labels
    # delete: unlike client-go's fake, our store implements DeleteCollection, so Delete is verified here
    r.delete_resources()
    assert store.get("/api/v1/namespaces/default/services")[1]["items"] == []
    assert store.get("/apis/batch/v1/namespaces/default/jobs")[1]["items"] == []


def test_rendezvous_port_is_exposed_by_the_master_service():
    """The trainer's TCP-store rendezvous (parallel/dist.py) must dial a port the master's ClusterIP Service
    forwards: a multi-replica TfJob on a real cluster reaches the master only through that Service."""
    from k8s_amd.parallel.dist import rank_from_tf_config

    store = ApiStore()
    job = _seed(store, {"metadata": {"name": "dp"}, "spec": {"RuntimeId": "rid0", "replicaSpecs": [
        {"replicas": 1, "tfPort": 2222, "tfReplicaType": "MASTER", "template": template(container())},
        {"replicas": 3, "tfPort": 2222, "tfReplicaType": "WORKER", "template": template(container())}]}})
    _reconciler(store, json.dumps(job)).reconcile()
    _, svcs = store.get("/api/v1/namespaces/default/services")
    _, jobs = store.get("/apis/batch/v1/namespaces/default/jobs")
    ports = {s["metadata"]["name"]: {p["port"] for p in s["spec"]["ports"]} for s in svcs["items"]}
    for j in jobs["items"]:
        tfc = j["spec"]["template"]["spec"]["containers"][0]["env"][0]["value"]
        info = rank_from_tf_config(tfc)
        assert info.world_size == 4
        assert info.master_addr == "dp-master-rid0-0"
        assert info.master_port in ports[info.master_addr], (info.master_port, ports)


def test_tensorboard_create():
    store = ApiStore()
    job = _seed(store, {"metadata": {"name": "some-job"}, "spec": {
        "RuntimeId": "some-runtime", "tensorboard": {"logDir": "/tmp/tensorflow"},
        "replicaSpecs": [{"replicas": 1, "tfPort": 10, "tfReplicaType": "MASTER", "template": template(container())}]}})
    r = _reconciler(store, json.dumps(job))
    r.reconcile()
    name = "some-job-tensorboard-some-runtime"
    labels = {"tensorflow.org": "", "runtime_id": "some-runtime", "app": "tensorboard", "tf_job_name": "some-job"}
    code, s = store.get("/api/v1/namespaces/default/services/" + name)
    assert code == 200 and s["metadata"]["labels"] == labels
    assert s["spec"]["ports"][0] == {"name": "tb-port", "port": 80, "targetPort": 6006}
    assert s["spec"]["type"] == "ClusterIP"
    code, d = store.get("/apis/apps/v1/namespaces/default/deployments/" + name)
    assert code == 200 and d["metadata"]["labels"] == labels
    assert d["spec"]["template"]["spec"]["containers"][0]["command"] == [
        "tensorboard", "--logdir", "/tmp/tensorflow", "--host", "0.0.0.0"]
    assert d["metadata"]["ownerReferences"][0]["name"] == "some-job"


# --------------------------------------------------------------------------- TestJobSetup
@pytest.mark.parametrize("resources,tb,phase,state,reason,mounts", [
    ({}, None, "Creating", "Running", "", 0),
    ({"requests": {"nvidia-gpu": "1"}}, None, "Creating", "Running", "", 1),
    ({"requests": {"nvidia-gpu": "1"}}, {}, "Failed", "Failed", "tbReplicaSpec.LogDir must be specified", 0),
])
def test_job_setup(resources, tb, phase, state, reason, mounts):
    store = ApiStore()
    spec = {"replicaSpecs": [{"replicas": 2, "tfPort": 10, "tfReplicaType": "PS",
                              "template": template(container(resources=resources))}]}
    if tb is not None:
        spec["tensorboard"] = tb
    job = _seed(store, {"metadata": {"name": "j"}, "spec": spec})
    r = _reconciler(store, json.dumps(job), ACC_CFG)
    r.setup()
    st = json.loads(r.status())
    assert st["phase"] == phase and st["state"] == state and st["reason"] == reason
    j = json.loads(r.job())
    if state != "Failed":
        assert len(j["spec"]["RuntimeId"]) == 4
    pod = j["spec"]["replicaSpecs"][0]["template"]["spec"]
    assert len(pod.get("volumes") or []) == mounts
    assert len(pod["containers"][0].get("volumeMounts") or []) == mounts


# --------------------------------------------------------------------------- status machine (new coverage)
def _set_pod(store, job_name, exit_code=None, running=False, last=None):
    code, j = store.get("/apis/batch/v1/namespaces/default/jobs/" + job_name)
    labels = j["spec"]["template"]["metadata"]["labels"]
    st = {"running": {}} if running else {"terminated": {"exitCode": exit_code}}
    cst = {"name": "tensorflow", "state": st}
    if last:
        cst["lastState"] = last
    pod = {"metadata": {"name": job_name + "-pod", "labels": labels},
           "status": {"startTime": "2020-01-01T00:00:00Z", "containerStatuses": [cst]}}
    store.delete("/api/v1/namespaces/default/pods/" + job_name + "-pod")
    store.post("/api/v1/namespaces/default/pods", pod)


def _mw_job(store):
    job = _seed(store, {"metadata": {"name": "mw"}, "spec": {"replicaSpecs": [
        {"replicas": 1, "tfReplicaType": "MASTER", "template": template(container())},
        {"replicas": 2, "tfReplicaType": "WORKER", "template": template(container())},
        {"replicas": 1, "tfReplicaType": "PS"}]}})
    r = _reconciler(store, json.dumps(job), ps_source="print('ps')")
    r.reconcile()
    rid = json.loads(r.job())["spec"]["RuntimeId"]
    return r, rid


def test_master_decides_success_and_status_persisted():
    store = ApiStore()
    r, rid = _mw_job(store)
    st = json.loads(r.status())
    assert st["phase"] == "Running" and st["state"] == "Running"
    _set_pod(store, "mw-master-%s-0" % rid, 0)
    _set_pod(store, "mw-worker-%s-0" % rid, running=True)
    r.reconcile()
    st = json.loads(r.status())
    assert st["phase"] == "Done" and st["state"] == "Succeeded"
    code, stored = store.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs/mw")
    assert stored["status"]["state"] == "Succeeded" and stored["spec"]["RuntimeId"] == rid
    types = {s["tf_replica_type"]: s for s in stored["status"]["replicaStatuses"]}
    assert types["MASTER"]["ReplicasStates"] == {"Succeeded": 1}
    assert types["WORKER"]["state"] == "Running"


def test_worker_failure_does_not_fail_job_but_master_does():
    store = ApiStore()
    r, rid = _mw_job(store)
    _set_pod(store, "mw-worker-%s-1" % rid, 3)  # permanent worker error: ignored (master decides, Q7)
    _set_pod(store, "mw-master-%s-0" % rid, running=True)
    r.reconcile()
    assert json.loads(r.status())["state"] == "Running"
    _set_pod(store, "mw-master-%s-0" % rid, 139)  # retryable (>=128)
    r.reconcile()
    assert json.loads(r.status())["state"] == "Running"
    _set_pod(store, "mw-master-%s-0" % rid, running=True, last={"terminated": {"exitCode": 2}})
    r.reconcile()
    st = json.loads(r.status())
    assert st["phase"] == "Done" and st["state"] == "Failed"


def test_default_ps_configmap_idempotent_with_owner():
    """Q2: the PS ConfigMap AlreadyExists no longer aborts later ticks; Q9: it is owned by the TfJob."""
    store = ApiStore()
    r, rid = _mw_job(store)
    code, cm = store.get("/api/v1/namespaces/default/configmaps/cm-ps-" + rid)
    assert code == 200 and cm["data"]["grpc_tensorflow_server.py"] == "print('ps')"
    assert cm["metadata"]["ownerReferences"][0]["name"] == "mw"
    # external deletion of a worker Job is healed on a later tick
    store.delete("/apis/batch/v1/namespaces/default/jobs/mw-worker-%s-1" % rid)
    r.reconcile()
    r.reconcile()
    assert store.get("/apis/batch/v1/namespaces/default/jobs/mw-worker-%s-1" % rid)[0] == 200
    code, j = store.get("/apis/batch/v1/namespaces/default/jobs/mw-ps-%s-0" % rid)
    cmd = j["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[:2] == ["python", "/ps-server/grpc_tensorflow_server.py"]
    assert cmd[2] == "--cluster_spec" and cmd[4:] == ["--job_name", "ps", "--task_id", "0"]
    assert cmd[3].startswith("master|mw-master-%s-0:2222,ps|" % rid)
    assert {"name": "ps-config-volume", "configMap": {"name": "cm-ps-" + rid}} in j["spec"]["template"]["spec"]["volumes"]


def test_status_write_conflict_retry():
    """Q3: a stale resourceVersion gets re-GET + retry instead of a silently dropped write."""
    store = ApiStore()
    job = _seed(store, {"metadata": {"name": "c"}, "spec": {"replicaSpecs": [
        {"replicas": 1, "tfReplicaType": "MASTER", "template": template(container())}]}})
    # someone else modifies the object before our first status write
    store.put("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs/c",
              dict(job, metadata=dict(job["metadata"], labels={"touched": "yes"})))
    r = _reconciler(store, json.dumps(job))
    r.reconcile()
    code, stored = store.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs/c")
    assert stored["status"]["phase"] in ("Creating", "Running")


def test_api_errors_are_unknown_not_failed():
    """Q6: pod LIST errors make the replica Unknown, never Failed."""
    store = ApiStore()
    r, rid = _mw_job(store)
    store.hooks.append(lambda m, p, b: (500, {"kind": "Status", "code": 500}) if "/pods" in p and m == "GET" else None)
    r.reconcile()
    st = json.loads(r.status())
    assert st["state"] == "Running"
    assert all(s["state"] != "Failed" for s in st["replicaStatuses"])


def test_readopted_job_rebuilds_replicas():
    """Q1: a job whose status already has a phase (operator restart) still reconciles to Done."""
    store = ApiStore()
    r, rid = _mw_job(store)
    code, stored = store.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs/mw")
    r2 = _reconciler(store, json.dumps(stored), ps_source="x")
    _set_pod(store, "mw-master-%s-0" % rid, 0)
    r2.reconcile()
    assert json.loads(r2.status())["state"] == "Succeeded"


def test_invalid_spec_fails_job():
    store = ApiStore()
    job = _seed(store, {"metadata": {"name": "bad"}, "spec": {"replicaSpecs": [
        {"replicas": 2, "tfReplicaType": "MASTER", "template": template(container())}]}})
    r = _reconciler(store, json.dumps(job))
    r.reconcile()
    code, stored = store.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs/bad")
    assert stored["status"]["phase"] == "Failed" and stored["status"]["state"] == "Failed"
    assert stored["status"]["reason"] == "invalid job spec: The MASTER must have Replicas = 1"


def test_yaml_reader():
    text = """
# comment
apiVersion: "tensorflow.org/v1alpha1"
kind: "TfJob"
metadata:
  name: "example-job"
spec:
  replicaSpecs:
    - replicas: 1
      tfReplicaType: MASTER
      template:
        spec:
          containers:
            - image: gcr.io/tf-on-k8s-dogfood/tf_sample:dc944ff
              name: tensorflow
              args: ["--flag", 'x y']
          restartPolicy: OnFailure
    - replicas: 2
      tfReplicaType: PS
---
second: {a: 1, b: [true, null, 1.5]}
"""
    docs = json.loads(op.yaml_all_to_json(text))
    assert docs[0]["spec"]["replicaSpecs"][0]["template"]["spec"]["containers"][0]["args"] == ["--flag", "x y"]
    assert docs[0]["spec"]["replicaSpecs"][1] == {"replicas": 2, "tfReplicaType": "PS"}
    assert docs[1] == {"second": {"a": 1, "b": [True, None, 1.5]}}
