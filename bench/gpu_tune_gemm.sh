#!/bin/bash
# Tune every GEMM shape of the benchmark workloads with PyTorch TunableOp (hipBLASLt + rocBLAS
# solutions, fastest measured wins) and write gpurun_out/tunableop_results*.csv; copy the
# result to gemm_db/tunableop_results.csv.  Then bench ViT with the tuned file.
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_gemm
( while sleep 45; do echo "hb $(date +%T) $(cat gpurun_out/tunableop_results*.csv 2>/dev/null | wc -l) tuned"; done ) &
HB=$!
# start from the shipped tunings: TunableOp reads the file (device ordinal appended) and
# writes it back with the new shapes added
cp gemm_db/tunableop_results.csv gpurun_out/tunableop_results0.csv 2>/dev/null
timeout -k 10 600 python -m pytest tests/test_vit_gpu.py -q -x > gpurun_out/pytest_gemm.txt 2>&1 || exit 3
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_results.csv
timeout -k 10 700 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 2 --warmup 2 --optimizer adamw > gpurun_out/tune_gemm_vit.txt 2>&1
rc1=$?
timeout -k 10 300 python bench.py --steps 2 --warmup 2 > gpurun_out/tune_gemm_r50.txt 2>&1
rc2=$?
kill $HB
echo "tune rc=$rc1 $rc2"
[ $rc1 -eq 0 ] || exit 4
unset PYTORCH_TUNABLEOP_ENABLED PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_FILENAME
f=$(ls gpurun_out/tunableop_results*.csv | head -1)
mkdir -p gemm_db && cp "$f" gemm_db/tunableop_results.csv
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench_gemm.jsonl > gpurun_out/bench_gemm_vit.txt 2>&1 || exit 5
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_gemm.jsonl > gpurun_out/bench_gemm_r50.txt 2>&1 || exit 6
