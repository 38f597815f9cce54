#!/bin/bash
# session-3 re-entry: full GPU test suite, headline bench (eager + hipGraph), ResNet-50 kernel profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3a
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s3a.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3a.txt
# test failures (rc 1) still allow the benches; crashes, aborts and time limits end the call
[ $rc -le 1 ] || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s3a.jsonl > gpurun_out/bench_s3a.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --cuda-graph --json-out gpurun_out/bench_s3a.jsonl > gpurun_out/bench_s3a_graph.txt 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s3a -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/prof_s3a.txt 2>&1 || exit 6
