#!/bin/bash
# fused MFMA attention: numerics, ViT tests, ViT-B/16 bench A/B, ViT profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3o
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s3o.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3o.txt
[ $rc -le 1 ] || exit 3
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench_s3o.jsonl > gpurun_out/bench_s3o_vit.txt 2>&1 || exit 4
DPT_NATIVE_ATTN=0 timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench_s3o.jsonl > gpurun_out/bench_s3o_vit0.txt 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s3o -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 8 --warmup 4 --optimizer adamw > $GRAFT_REPO_ROOT/gpurun_out/prof_s3o.txt 2>&1 || exit 6
