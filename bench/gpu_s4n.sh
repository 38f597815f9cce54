#!/bin/bash
# ViT-B/16 (batch 128, AdamW): bench + per-step kernel profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4n
timeout -k 10 400 python bench.py --model vit_b_16 --batch-size 128 --optimizer adamw --no-channels-last --json-out gpurun_out/bench_s4n.jsonl > gpurun_out/bench_s4n.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s4n -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model vit_b_16 --batch-size 128 --optimizer adamw --no-channels-last --steps 6 --warmup 6 > $GRAFT_REPO_ROOT/gpurun_out/prof_s4n.txt 2>&1 || exit 6
