#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch6
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu6.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu6.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/bench6.jsonl > gpurun_out/bench6.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof6 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof6.txt 2>&1 || exit 7
