#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/bn_micro.txt
: > $O
timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 3
DPT_BN_MAX_CHUNKS=2048 timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 4
DPT_BN_MAX_CHUNKS=512 timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 5
DPT_BN_BWD_UNROLL=4 timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 6
DPT_BN_APPLY_MAX=2048 timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 7
DPT_BN_APPLY_MAX=32768 timeout -k 10 120 python bench/bn_micro.py >> $O 2>&1 || exit 8
