#!/bin/bash
# BN backward mask-from-x: BN GPU tests + bench + profile, then MIOpen tuning
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch11
timeout -k 10 600 python -m pytest tests/test_bn_gpu.py tests/test_engine_gpu.py -q -x > gpurun_out/pytest_gpu11.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu11.txt
grep -q "pytest rc=0" gpurun_out/pytest_gpu11.txt || exit 3
timeout -k 10 300 python bench.py --json-out gpurun_out/bench11.jsonl > gpurun_out/bench11.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof11 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof11.txt 2>&1 || exit 5
cd $GRAFT_REPO_ROOT
TUNE_SECONDS=700 bash bench/gpu_tune_miopen.sh t2
