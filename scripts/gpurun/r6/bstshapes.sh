#!/bin/bash
# GPU job (round 6): per-shape cost of the tile kernel's BN-sums epilogue vs the plain data gradient it replaced.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bstshapes; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u scripts/microbench/bst_shapes.py > $O/b3072.jsonl 2> $O/b3072.err || { tail -20 $O/b3072.err; exit 1; }
cat $O/b3072.jsonl
BST_BATCH=1024 timeout -k 10 300 python -u scripts/microbench/bst_shapes.py > $O/b1024.jsonl 2> $O/b1024.err || { tail -20 $O/b1024.err; exit 1; }
cat $O/b1024.jsonl
