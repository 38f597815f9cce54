#!/bin/bash
# full GPU suite + smoke, headline bench (now with the post-window sync profile), kernel profile
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch_s4w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s4w.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_s4w.txt
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s4w.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_s4w.jsonl >> gpurun_out/bench_s4w.txt 2>&1 || exit 5
timeout -k 10 300 python bench.py --amp-dtype fp16 --json-out gpurun_out/bench_s4w.jsonl >> gpurun_out/bench_s4w.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s4w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 4 --profile-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_s4w.txt 2>&1 || exit 7
