#!/bin/bash
# MIOpen exhaustive tuning for the bench config; tuned perf/find dbs land in gpurun_out/scratch_tune
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_tune
timeout -k 10 200 python bench.py --json-out gpurun_out/tune_bench.jsonl > gpurun_out/tune_before.txt 2>&1 || exit 3
MIOPEN_FIND_MODE=1 MIOPEN_FIND_ENFORCE=3 MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 \
  timeout -k 10 840 python bench.py --find --steps 3 --warmup 1 --json-out gpurun_out/tune_bench.jsonl > gpurun_out/tune_run.txt 2> gpurun_out/tune_log.txt
echo "tune rc=$?" >> gpurun_out/tune_run.txt
timeout -k 10 200 python bench.py --json-out gpurun_out/tune_bench.jsonl > gpurun_out/tune_after.txt 2>&1 || exit 5
