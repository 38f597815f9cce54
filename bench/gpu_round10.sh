#!/bin/bash
# bf16 weight shadows: GPU tests, A/B bench (ResNet-50 + ViT-B/16), steady-state profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch10
timeout -k 10 700 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu10.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu10.txt
grep -q "pytest rc=0" gpurun_out/pytest_gpu10.txt || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench10.jsonl > gpurun_out/bench10.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --no-weight-shadow --json-out gpurun_out/bench10.jsonl > gpurun_out/bench10_ns.txt 2>&1 || exit 5
timeout -k 10 300 python bench.py --cuda-graph --json-out gpurun_out/bench10.jsonl > gpurun_out/bench10_graph.txt 2>&1 || exit 6
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench10.jsonl > gpurun_out/bench10_vit.txt 2>&1 || exit 7
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --impl torch --json-out gpurun_out/bench10.jsonl > gpurun_out/bench10_vitt.txt 2>&1 || exit 8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof10 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof10.txt 2>&1 || exit 9
