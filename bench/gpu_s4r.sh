#!/bin/bash
# ResNet-18 / CIFAR shape (the reference's own workload): eager and hipGraph, bf16 and fp16
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4r
R18="--model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 50 --warmup 20"
timeout -k 10 300 python bench.py $R18 --json-out gpurun_out/bench_s4r.jsonl > gpurun_out/bench_s4r.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py $R18 --cuda-graph --json-out gpurun_out/bench_s4r.jsonl >> gpurun_out/bench_s4r.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py $R18 --amp-dtype fp16 --json-out gpurun_out/bench_s4r.jsonl >> gpurun_out/bench_s4r.txt 2>&1 || exit 5
timeout -k 10 300 python bench.py $R18 --amp-dtype fp16 --cuda-graph --json-out gpurun_out/bench_s4r.jsonl >> gpurun_out/bench_s4r.txt 2>&1 || exit 6
timeout -k 10 300 python bench.py $R18 --impl torch --amp-dtype fp16 --json-out gpurun_out/bench_s4r.jsonl >> gpurun_out/bench_s4r.txt 2>&1 || exit 7
