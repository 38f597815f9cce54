#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3q
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s3q.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3q.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s3q.jsonl > gpurun_out/bench_s3q.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s3q -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_s3q.txt 2>&1 || exit 6
