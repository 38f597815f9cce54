#!/bin/bash
# full GPU test suite + smoke, then the reference README tables (throughput vs batch, AMP vs FP32)
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s3p
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s3p.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s3p.txt
[ $rc -le 1 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3p.txt 2>&1 || exit 4
timeout -k 10 900 python bench/sweep.py --table batch --steps 20 --warmup 8 --timeout 400 --out gpurun_out/sweep_batch_s3p.jsonl > gpurun_out/sweep_batch_s3p.txt 2>&1 || exit 5
timeout -k 10 900 python bench/sweep.py --table amp --steps 20 --warmup 8 --timeout 400 --out gpurun_out/sweep_amp_s3p.jsonl > gpurun_out/sweep_amp_s3p.txt 2>&1 || exit 6
