#!/bin/bash
# GPU session: tests, bench (native vs stock torch), rocprof stats; MIOpen db exported.
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch
python -c "import distributed_pytorch_training_amd.ops as o; o.native(); print('native ok', o.native().rccl_version())" > gpurun_out/native.txt 2>&1 || exit 3
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.txt
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/bench.jsonl > gpurun_out/bench_native.txt 2>&1 || exit 4
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --impl torch --json-out gpurun_out/bench.jsonl > gpurun_out/bench_torch.txt 2>&1 || exit 5
mkdir -p gpurun_out/miopen_db && cp $DPT_SCRATCH/dpt_miopen_*/db/*.txt gpurun_out/miopen_db/ 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_native -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_native.txt 2>&1 || exit 6
