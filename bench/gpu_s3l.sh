#!/bin/bash
# conv_kernels.hip v1: numerics vs fp32 reference, then per-shape timing vs MIOpen
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3l
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s3l.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3l.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python -u bench/conv_bench.py > gpurun_out/conv_bench_s3l.md 2>&1 || exit 4
