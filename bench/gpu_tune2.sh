#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune2/db gpurun_out/tune2/cache
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/tune2/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/tune2/cache
MIOPEN_FIND_MODE=1 MIOPEN_FIND_ENFORCE=4 MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=4 \
  timeout -k 10 960 python bench.py --find --steps 3 --warmup 1 --json-out gpurun_out/tune2_bench.jsonl > gpurun_out/tune2_run.txt 2> gpurun_out/tune2_log.txt
echo "tune rc=$?" >> gpurun_out/tune2_run.txt
timeout -k 10 200 python bench.py --json-out gpurun_out/tune2_bench.jsonl > gpurun_out/tune2_after.txt 2>&1 || exit 5
