#!/bin/bash
# GPU job (round 5): the full-vocabulary BERT decoder test and the padded-vocab cross-entropy test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_vocab256b; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_kernels_gpu.py -k "full_vocab or padded_vocab or loss_matches" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
