#!/bin/bash
# full GPU test suite, ViT bench, ResNet-50 throughput-vs-batch table (native)
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch15
timeout -k 10 700 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu15.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu15.txt
grep -q "pytest rc=0" gpurun_out/pytest_gpu15.txt || exit 3
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench15.jsonl > gpurun_out/bench15_vit.txt 2>&1 || exit 4
timeout -k 10 900 python bench/sweep.py --table batch --steps 20 --warmup 8 --timeout 420 --out gpurun_out/sweep_batch.jsonl > gpurun_out/sweep_batch.txt 2>&1 || exit 5
