#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch8
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu8.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu8.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --cuda-graph --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8_graph.txt 2>&1 || exit 5
# the reference's own workload shape: ResNet-18, 32x32, 10 classes, batch 128 (eager vs graph vs stock)
timeout -k 10 300 python bench.py --find --model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 100 --warmup 20 --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8_r18.txt 2>&1 || exit 6
timeout -k 10 300 python bench.py --find --model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 100 --warmup 20 --cuda-graph --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8_r18g.txt 2>&1 || exit 7
timeout -k 10 300 python bench.py --find --model resnet18 --image-size 32 --num-classes 10 --batch-size 128 --steps 100 --warmup 20 --impl torch --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8_r18t.txt 2>&1 || exit 8
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --json-out gpurun_out/bench8.jsonl > gpurun_out/bench8_vit.txt 2>&1 || exit 9
