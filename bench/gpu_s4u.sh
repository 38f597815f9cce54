#!/bin/bash
# full GPU test suite (what the driver runs at round end) + smoke()
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s4u.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s4u.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s4u.txt 2>&1 || exit 4
