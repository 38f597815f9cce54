#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch9
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --impl torch --json-out gpurun_out/bench9.jsonl > gpurun_out/bench9_vit_torch.txt 2>&1 || exit 4
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench9.jsonl > gpurun_out/bench9_vit_adamw.txt 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof9_vit -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 8 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof9.txt 2>&1 || exit 7
