#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch7
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu7.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu7.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/bench7.jsonl > gpurun_out/bench7.txt 2>&1 || exit 4
timeout -k 10 300 python bench/conv1x1_vs_gemm.py > gpurun_out/conv1x1.md 2> gpurun_out/conv1x1.err || exit 5
