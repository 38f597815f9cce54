#!/bin/bash
# ResNet-18 / CIFAR: native-conv pixel threshold sweep (hipGraph and eager), ResNet-50 unchanged check
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4s
R18="--model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 50 --warmup 20"
for t in 0 3072 9000 40000; do
  DPT_CONV_MIN_PIXELS=$t timeout -k 10 300 python bench.py $R18 --cuda-graph --json-out gpurun_out/bench_s4s_$t.jsonl > gpurun_out/bench_s4s.txt 2>&1 || exit 3
  DPT_CONV_MIN_PIXELS=$t timeout -k 10 300 python bench.py $R18 --json-out gpurun_out/bench_s4s_$t.jsonl >> gpurun_out/bench_s4s.txt 2>&1 || exit 4
done
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4s_r50.jsonl >> gpurun_out/bench_s4s.txt 2>&1 || exit 5
