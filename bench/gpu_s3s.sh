#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3s
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s3s.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3s.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s3s.jsonl > gpurun_out/bench_s3s.txt 2>&1 || exit 4
timeout -k 10 400 python -u bench/conv_bench.py > gpurun_out/conv_bench_s3s.md 2>&1 || exit 5
