#!/bin/bash
# GPU job (round 5): fused LayerNorm backward with three-row prefetch (K8S_AMD_NORM_PREFETCH=2: the two-slot form) --
# kernel tests, BERT b1024 A/B alternating, per-kernel profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_normpf; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_grads_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 3 2 3 2; do
  K8S_AMD_NORM_PREFETCH=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 prefetch=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
for v in 3 2; do
  K8S_AMD_NORM_PREFETCH=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb$v -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 6 --log-every 3 > $O/pb$v.log 2>&1 || { tail -20 $O/pb$v.log; exit 1; }
  python3 scripts/profile_report.py $(ls $O/pb$v/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "BERT-base s128 b1024, round 5 (LayerNorm backward prefetch $v)" > $O/bert_$v.md && head -4 $O/bert_$v.md && grep norm_bwd $O/bert_$v.md
  rm -rf $O/pb$v
done
