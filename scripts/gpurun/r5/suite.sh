#!/bin/bash
# GPU job (round 5): whole GPU suite + smoke (as the driver runs them), then BERT b1024 and the ResNet-50 bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_suite; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 1; }
echo "bert b1024: $(grep '"event": "step"' $O/bert.log | tail -1 | cut -c1-120)"
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
