#!/bin/bash
# conv3x3 lean prologue A/B: kernel test, microbench (lean vs round-5 kernel, interleaved), bench on / off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_c3lean}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
C3_LEAN_AB=1 timeout -k 10 300 python -u scripts/bench_conv3x3.py --batch 3072 --rounds 3 > $O/micro.jsonl 2> $O/micro.err || { tail -20 $O/micro.err; exit 1; }
cat $O/micro.jsonl
bash scripts/gpurun/r6/envab.sh ${1:-r6_c3lean}_bench 2 3072 "lean:K8S_AMD_C3_LEAN=1" "old:K8S_AMD_C3_LEAN=0"
