#!/bin/bash
# A/B: scripts/diag_conv.py against older in-tree builds staged under abtest/<rev>/k8s_amd.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rev in $(ls abtest) current; do
  if [ "$rev" = current ]; then pp=$PWD; else pp=$PWD/abtest/$rev; fi
  echo "== $rev" >> gpurun_out/ab_conv.log
  K8S_AMD_ROOT=$pp timeout -k 10 120 python scripts/diag_conv.py >> gpurun_out/ab_conv.log 2>&1 || exit 1
done
