#!/bin/bash
# GPU job (round 6): GEMM products vs hipBLASLt, BERT b1024 products, attention vs SDPA -- on the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_kernels}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u scripts/bench_gemm256.py --rounds 5 > $O/gemm.jsonl 2> $O/gemm.err || { tail -30 $O/gemm.err; exit 1; }
echo "gemm rows: $(wc -l < $O/gemm.jsonl)"
timeout -k 10 300 python -u scripts/bench_bert_gemm.py --blas > $O/bert_gemm.jsonl 2> $O/bert_gemm.err || { tail -30 $O/bert_gemm.err; exit 1; }
echo "bert rows: $(wc -l < $O/bert_gemm.jsonl)"
timeout -k 10 300 python -u scripts/bench_attention.py > $O/attn.jsonl 2> $O/attn.err || { tail -30 $O/attn.err; exit 1; }
echo "attention rows: $(wc -l < $O/attn.jsonl)"
bash scripts/gpurun/r6/envab.sh r6_bstats_all 3 3072 "on:X=1" "off:K8S_AMD_BN_BSTATS=0"
