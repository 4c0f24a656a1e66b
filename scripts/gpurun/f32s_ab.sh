#!/bin/bash
# GPU job: tests touching the fp32 epilogues, then ResNet bench and BERT trainer with K8S_AMD_F32S=0/1 alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_gemm256_gpu.py tests/test_resnet_gpu.py tests/test_wgrad_stream_gpu.py tests/test_transformer_grads_gpu.py > gpurun_out/f32s_test.log 2>&1 || { tail -40 gpurun_out/f32s_test.log; exit 1; }
tail -1 gpurun_out/f32s_test.log
for v in 1 0 1 0; do
  K8S_AMD_F32S=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 2> /tmp/b.err > /tmp/b.json || { tail -5 /tmp/b.err; exit 1; }
  echo "resnet F32S=$v $(python3 -c "import json;d=json.load(open('/tmp/b.json'));print(d['value'], d['ms_per_step'])")"
done
for v in 1 0; do
  K8S_AMD_F32S=$v timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > /tmp/bert.log 2>&1 || { tail -5 /tmp/bert.log; exit 1; }
  echo "bert F32S=$v $(grep '"step"' /tmp/bert.log | tail -1 | python3 -c "import json,sys;print(json.loads(sys.stdin.read())['tokens_per_sec'])")"
done
