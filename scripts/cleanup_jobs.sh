#!/bin/bash
# Delete every TfJob and every object the operator created (label tensorflow.org) in a namespace.
# Parity: /root/reference/scripts/cleanup_clusters.sh (delete by the tensorflow.org= label selector).
#   scripts/cleanup_jobs.sh [namespace] [apiserver-url]
set -euo pipefail
NS=${1:-default}
SERVER=${2:-${K8S_AMD_APISERVER:-http://127.0.0.1:8080}}
cd "$(dirname "$0")/.."
python3 - "$NS" "$SERVER" <<'PY'
import sys
from k8s_amd.fakeapi.client import ApiClient
ns, server = sys.argv[1], sys.argv[2]
c = ApiClient(server)
for job in c.get("/apis/tensorflow.org/v1alpha1/namespaces/%s/tfjobs" % ns).get("items", []):
    c.request("DELETE", "/apis/tensorflow.org/v1alpha1/namespaces/%s/tfjobs/%s" % (ns, job["metadata"]["name"]))
    print("tfjob/%s deleted" % job["metadata"]["name"])
sel = "labelSelector=tensorflow.org"
for path in ("/apis/batch/v1/namespaces/%s/jobs", "/api/v1/namespaces/%s/pods", "/api/v1/namespaces/%s/services",
             "/api/v1/namespaces/%s/configmaps", "/apis/apps/v1/namespaces/%s/deployments"):
    p = path % ns
    for obj in c.get(p + "?" + sel).get("items", []):
        c.request("DELETE", p + "/" + obj["metadata"]["name"])
        print("%s/%s deleted" % (p.rsplit("/", 1)[1], obj["metadata"]["name"]))
PY
