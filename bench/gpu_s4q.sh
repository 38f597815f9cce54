#!/bin/bash
# forward-conv statistics epilogue: partial stores in the [Cout][m_tiles] vs [m_tiles][Cout] layout
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/conv_stats_cost.py > gpurun_out/stats_cost_s4q.txt 2>&1 || exit 3
DPT_CONV_NO_PSTORE=2 timeout -k 10 300 python bench/conv_stats_cost.py >> gpurun_out/stats_cost_s4q.txt 2>&1 || exit 4
