#!/bin/bash
# fp16 on the MFMA convolutions: GPU tests, fp16 + bf16 ResNet-50 bench, ResNet-18 CIFAR fp16
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4t
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_bn_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s4t.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s4t.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --amp-dtype fp16 --json-out gpurun_out/bench_s4t.jsonl > gpurun_out/bench_s4t.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4t.jsonl >> gpurun_out/bench_s4t.txt 2>&1 || exit 5
R18="--model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 50 --warmup 20"
timeout -k 10 300 python bench.py $R18 --amp-dtype fp16 --json-out gpurun_out/bench_s4t.jsonl >> gpurun_out/bench_s4t.txt 2>&1 || exit 6
