#!/bin/bash
# 2x2-block stem max-pool forward: pool/BN tests, A/B bench, profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4y
timeout -k 10 600 python -u -m pytest tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s4y.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s4y.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4y.jsonl >> gpurun_out/bench_s4y.txt 2>&1 || exit 5
DPT_POOL_BLOCK2=0 timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4y.jsonl >> gpurun_out/bench_s4y.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s4y -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 4 --profile-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_s4y.txt 2>&1 || exit 7
