#!/bin/bash
# current engine: throughput vs batch size, AMP vs FP32, native vs stock (ResNet-50, 1 GPU)
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4o
rm -f gpurun_out/sweep_s4o_*.jsonl
timeout -k 10 900 python bench/sweep.py --table batch --no-find --out gpurun_out/sweep_s4o_batch.jsonl > gpurun_out/sweep_s4o_batch.txt 2>&1 || exit 3
timeout -k 10 900 python bench/sweep.py --table amp --no-find --out gpurun_out/sweep_s4o_amp.jsonl > gpurun_out/sweep_s4o_amp.txt 2>&1 || exit 4
timeout -k 10 600 python bench/sweep.py --table impl --no-find --out gpurun_out/sweep_s4o_impl.jsonl > gpurun_out/sweep_s4o_impl.txt 2>&1 || exit 5
