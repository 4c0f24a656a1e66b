#!/bin/bash
# GPU job (round 4): sub-wave grids off the stream-K tail -- gemm256 tests, BERT throughput and steady-state trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_tf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $O/g256_tests.log 2>&1 || { tail -30 $O/g256_tests.log; exit 1; }
tail -1 $O/g256_tests.log
timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 20 > $O/bert2.log 2>&1 || { tail -20 $O/bert2.log; exit 1; }
grep '"event": "step"' $O/bert2.log | tail -1 | cut -c1-120
rm -rf $O/prof_bert2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_bert2 -o bb -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 20 --log-every 10 > $O/prof_bert2.log 2>&1 || { tail -20 $O/prof_bert2.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof_bert2/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "BERT-base s128 b64, round 4" > $O/bert2.md && head -30 $O/bert2.md
