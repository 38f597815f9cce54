#!/bin/bash
# stem BN apply folded into the max-pool: tests, A/B bench, profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4v
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_bn_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s4v.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s4v.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4v.jsonl >> gpurun_out/bench_s4v.txt 2>&1 || exit 5
DPT_STEM_FUSE=0 timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4v.jsonl >> gpurun_out/bench_s4v.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s4v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_s4v.txt 2>&1 || exit 7
