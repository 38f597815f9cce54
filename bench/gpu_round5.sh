#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch5
timeout -k 10 500 python -m pytest tests/test_bn_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu5.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu5.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/bench5.jsonl > gpurun_out/bench5.txt 2>&1 || exit 4
timeout -k 10 400 python bench/conv_roofline.py --batch 256 > gpurun_out/conv_roofline.md 2> gpurun_out/conv_roofline.err || exit 5
