#!/bin/bash
# GPU job (round 5): 4-wave GEMM epilogue extras + tall-K split -- GEMM tests, BERT b1024 trainer, ResNet bench, BERT
# step profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_w4x; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 1; }
echo "bert b1024: $(grep '"event": "step"' $O/bert.log | tail -1 | cut -c1-120)"
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 8 --log-every 4 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "BERT-base s128 b1024, 4-wave GEMM extras + split" > $O/bert.md && head -35 $O/bert.md
rm -rf $O/pb
