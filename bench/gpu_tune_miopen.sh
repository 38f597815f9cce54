#!/bin/bash
# Exhaustive MIOpen perf-db tuning (FIND_ENFORCE=SEARCH) for the ResNet-50 B256 bf16 NHWC convs,
# starting from an EMPTY user db (so find really runs and tunes every solver), then an
# immediate-mode bench on the tuned databases.  Merge afterwards with
#   python bench/merge_miopen_db.py gpurun_out/scratch_<tag>/tune_db
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-t1}
export DPT_SCRATCH=$PWD/gpurun_out/scratch_$TAG
export MIOPEN_USER_DB_PATH=$DPT_SCRATCH/tune_db
export MIOPEN_CUSTOM_CACHE_DIR=$DPT_SCRATCH/cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
cp miopen_db/*.ukdb $MIOPEN_CUSTOM_CACHE_DIR/ 2>/dev/null
( while sleep 45; do echo "hb $(date +%T) $(cat $MIOPEN_USER_DB_PATH/*.udb.txt 2>/dev/null | wc -l) perf $(cat $MIOPEN_USER_DB_PATH/*.ufdb.txt 2>/dev/null | wc -l) find"; done ) &
HB=$!
MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 ${TUNE_SECONDS:-900} python bench.py --find --steps 3 --warmup 2 ${BENCH_ARGS} > gpurun_out/tune_$TAG.txt 2>&1
rc=$?
kill $HB
echo "tune rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 124 ] || exit 4
timeout -k 10 300 python bench.py ${BENCH_ARGS} --json-out gpurun_out/bench_$TAG.jsonl > gpurun_out/bench_$TAG.txt 2>&1 || exit 5
