#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/bench/conv_pmc.py > $R/gpurun_out/pmc1.txt 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc2 -o run --output-format csv -- python3 $R/bench/conv_pmc.py > $R/gpurun_out/pmc2.txt 2>&1 || exit 4
