"""Release / CI tooling: JUnit XML (py/test_util_test.py semantics), the spec-driven test runner
(py/test_runner.py) against the local cluster, chart packaging with the image tag (py/release.py
update_values / update_chart) and the label-selector cleanup script (scripts/cleanup_clusters.sh)."""
import json
import os
import subprocess
import tarfile
import xml.etree.ElementTree as ET

import pytest
import yaml

from k8s_amd.fakeapi.cluster import OPERATOR_BIN, REPO, LocalCluster
from k8s_amd.tools import junit, release, test_runner


def test_junit_xml():
    cases = [junit.TestCase(class_name="some_test", name="first", time=10),
             junit.TestCase(class_name="some_test", name="first", time=10, failure="failed for some reason.")]
    root = ET.fromstring(junit.junit_xml(cases))
    assert root.tag == "testsuite" and root.get("failures") == "1" and root.get("tests") == "2"
    assert root.get("time") == "20"
    tcs = root.findall("testcase")
    assert [t.get("classname") for t in tcs] == ["some_test", "some_test"]
    assert tcs[0].find("failure") is None and tcs[1].find("failure").text == "failed for some reason."


def test_junit_escapes(tmp_path):
    p = junit.create_junit_xml_file([junit.TestCase("c<1>", "n&m", 1.5, 'bad "quote" <x>')],
                                    str(tmp_path / "sub" / "junit.xml"))
    root = ET.parse(p).getroot()
    assert root.find("testcase").get("name") == "n&m"
    assert root.find("testcase/failure").text == 'bad "quote" <x>'


def test_render_template():
    spec = test_runner.render("metadata:\n  name: j\nspec:\n  image: img:{{ image_tag }}\n", image_tag="abc")
    assert spec == {"metadata": {"name": "j"}, "spec": {"image": "img:abc"}}


def test_update_values_and_package_chart(tmp_path):
    out = release.package_chart(os.path.join(REPO, "charts", "tf-job-operator"), str(tmp_path),
                                "reg/tf_operator:v9", "9.9.9", test_image="reg/tf_sample:v9")
    with tarfile.open(out) as tf:
        names = tf.getnames()
        assert "tf-job-operator/Chart.yaml" in names and "tf-job-operator/templates/deployment.yaml" in names
        vals = yaml.safe_load(tf.extractfile("tf-job-operator/values.yaml").read())
        chart = yaml.safe_load(tf.extractfile("tf-job-operator/Chart.yaml").read())
    assert vals["image"] == "reg/tf_operator:v9" and vals["test_image"] == "reg/tf_sample:v9"
    assert vals["cloud"] == "amd"  # everything else untouched
    assert chart["version"] == "9.9.9"


@pytest.mark.skipif(not os.path.exists(OPERATOR_BIN), reason="operator not built")
def test_release_skip_build(tmp_path):
    assert release.main(["--out", str(tmp_path), "--registry", "reg", "--tag", "v1.2.3", "--skip-build"]) == 0
    m = json.load(open(tmp_path / "manifest.json"))
    assert m["operator_image"] == "reg/tf_operator:v1.2.3"
    assert "operator-context/bin/tf_operator" in m["files"]["operator"]
    assert "operator-context/ps_server/grpc_tensorflow_server.py" in m["files"]["operator"]
    assert os.path.exists(tmp_path / "trainer-context" / "k8s_amd" / "trainer" / "runner.py")


@pytest.mark.skipif(not os.path.exists(OPERATOR_BIN), reason="operator not built")
def test_test_runner_and_cleanup(tmp_path):
    spec = tmp_path / "job.yaml.template"
    spec.write_text(open(os.path.join(REPO, "examples", "tf_job.yaml")).read().replace(
        "name: \"example-job\"", "name: runner-{{ image_tag }}"))
    with LocalCluster() as c:
        junit_path = str(tmp_path / "junit.xml")
        rc = test_runner.main(["--spec", str(spec), "--junit_path", junit_path, "--image_tag", "t1",
                               "--server", c.url, "--timeout", "90", "--keep"])
        root = ET.parse(junit_path).getroot()
        assert rc == 0, ET.tostring(root).decode()
        assert root.get("failures") == "0" and root.find("testcase").get("name").startswith("runner-t1-")
        assert c.client.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs")["items"]
        r = subprocess.run([os.path.join(REPO, "scripts", "cleanup_jobs.sh"), "default", c.url],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert "tfjob/runner-t1-" in r.stdout
        assert not c.client.get("/apis/tensorflow.org/v1alpha1/namespaces/default/tfjobs")["items"]
        assert not c.client.get("/api/v1/namespaces/default/services?labelSelector=tensorflow.org")["items"]


def test_deploy_dryrun_commands(capsys):
    """tools/deploy.py (py/deploy.py parity): helm install with the amd preset + image tag, rollout wait, helm test,
    uninstall -- printed, not run, under --dryrun."""
    from k8s_amd.tools import deploy

    assert deploy.main(["--dryrun", "--namespace", "kubeflow", "setup", "--image", "reg.io/op:v1"]) == 0
    out = capsys.readouterr().out
    assert "kubectl get nodes -o json" in out
    assert "helm upgrade --install tf-job" in out and "cloud=amd" in out and "image=reg.io/op:v1" in out
    assert "rollout status deployment/tf-job-operator" in out
    assert deploy.main(["--dryrun", "test"]) == 0 and "helm test tf-job" in capsys.readouterr().out
    assert deploy.main(["--dryrun", "teardown"]) == 0 and "helm uninstall tf-job" in capsys.readouterr().out
    nodes = {"items": [{"status": {"allocatable": {"amd.com/gpu": "8"}}}, {"status": {"allocatable": {}}}]}
    assert deploy.gpu_capacity(json.dumps(nodes)) == 8


def test_deploy_local_e2e(tmp_path):
    import os

    from k8s_amd.fakeapi.cluster import OPERATOR_BIN
    from k8s_amd.tools import deploy

    if not os.path.exists(OPERATOR_BIN):
        pytest.skip("operator not built")
    junit = str(tmp_path / "junit.xml")
    assert deploy.main(["--timeout", "90", "--junit", junit, "local"]) == 0
    assert 'failures="0"' in open(junit).read()
