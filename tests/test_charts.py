"""Deployment artifacts: Helm charts (operator with the amd.com/gpu preset, RBAC incl. leases, helm test
running the e2e binary; TensorBoard chart) and the CRD manifest."""
import json
import os
import re

import yaml

from k8s_amd import _operator as op

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(REPO, "charts", "tf-job-operator")


def _read(*p):
    return open(os.path.join(*p)).read()


def test_templates_balanced():
    for root in (CHART, os.path.join(REPO, "charts", "tensorboard")):
        for dp, _, files in os.walk(root):
            for f in files:
                t = _read(dp, f)
                assert t.count("{{") == t.count("}}"), f
                yaml.safe_load(_read(root, "values.yaml")) if f == "values.yaml" else None


def _render_values(text, values):
    """The `{{ .Values.a.b | quote }}` placeholders of a template, filled from values.yaml (no helm binary here)."""
    def sub(m):
        v = values
        for k in m.group(1).split("."):
            v = v[k]
        return json.dumps(str(v)) if m.group(2) else str(v)
    return re.sub(r"\{\{\s*\.Values\.([\w.]+)\s*(\|\s*quote)?\s*\}\}", sub, text)


def test_amd_preset_controller_config():
    values = yaml.safe_load(_read(CHART, "values.yaml"))
    t = _render_values(_read(CHART, "templates", "config.yaml"), values)
    body = t.split("controller_config_file.yaml: |\n", 1)[1].split("{{-", 1)[0]
    body = "\n".join(line[4:] for line in body.splitlines())
    cfg = json.loads(op.controller_config(json.dumps(yaml.safe_load(body))))
    # Go field names: ControllerConfig has no json tags (pkg/spec/controller.go:3-11)
    acc = cfg["Accelerators"]["amd.com/gpu"]
    assert {v["MountPath"] for v in acc["Volumes"]} >= {"/opt/rocm", "/dev/kfd", "/dev/dri"}
    assert {"Name": "HSA_ENABLE_IPC_MODE_LEGACY", "Value": "0"} in acc["EnvVars"]
    assert {"Name": "NCCL_MIN_NCHANNELS", "Value": str(values["rccl"]["minChannels"])} in acc["EnvVars"]
    assert cfg["GrpcServerFilePath"].endswith("grpc_tensorflow_server.py")


def test_rbac_and_helm_test():
    rbac = _read(CHART, "templates", "rbac.yaml")
    for res in ("tfjobs", "customresourcedefinitions", "jobs", "pods", "services", "configmaps", "endpoints",
                "deployments", "leases"):
        assert re.search(r"\b%s\b" % res, rbac), res
    t = _read(CHART, "templates", "tests", "basic-test.yaml")
    assert "/opt/k8s-amd/bin/e2e" in t and '"helm.sh/hook": test' in t
    d = _read(CHART, "templates", "deployment.yaml")
    assert "MY_POD_NAMESPACE" in d and "MY_POD_NAME" in d and "apps/v1" in d


def test_crd_manifest_matches_operator():
    docs = [d for d in yaml.safe_load_all(_read(REPO, "manifests", "crd.yaml")) if d]
    assert docs == [json.loads(op.crd_manifest())]
