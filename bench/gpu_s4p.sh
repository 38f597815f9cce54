#!/bin/bash
# forward-conv statistics epilogue cost: with and without the partial stores
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/conv_stats_cost.py > gpurun_out/stats_cost_s4p.txt 2>&1 || exit 3
DPT_CONV_NO_PSTORE=1 timeout -k 10 300 python bench/conv_stats_cost.py >> gpurun_out/stats_cost_s4p.txt 2>&1 || exit 4
