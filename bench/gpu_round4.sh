#!/bin/bash
# GPU session 3: all GPU tests, headline bench (immediate mode), profile of the optimized BN.
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch4
timeout -k 10 500 python -m pytest tests/test_bn_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu4.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu4.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/bench4.jsonl > gpurun_out/bench4.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof4.txt 2>&1 || exit 7
