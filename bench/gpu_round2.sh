#!/bin/bash
# GPU session 2: fused-BN numerics, bench A/B (fused vs MIOpen BN), MIOpen immediate mode, profile.
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch2
timeout -k 10 400 python -m pytest tests/test_bn_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu2.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu2.txt
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/bench2.jsonl > gpurun_out/bench2_fused.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-fused-bn --json-out gpurun_out/bench2.jsonl > gpurun_out/bench2_unfused.txt 2>&1 || exit 5
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-find --json-out gpurun_out/bench2.jsonl > gpurun_out/bench2_nofind.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.txt 2>&1 || exit 7
