#!/bin/bash
# erf-approx GELU: ViT tests + bench + profile; ResNet-50 TunableOp A/B
set -o pipefail
mkdir -p gpurun_out
export DPT_SCRATCH=$PWD/gpurun_out/scratch14
timeout -k 10 600 python -m pytest tests/test_vit_gpu.py -q -x > gpurun_out/pytest_gpu14.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu14.txt
grep -q "pytest rc=0" gpurun_out/pytest_gpu14.txt || exit 3
timeout -k 10 400 python bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 20 --warmup 5 --optimizer adamw --json-out gpurun_out/bench14.jsonl > gpurun_out/bench14_vit.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --json-out gpurun_out/bench14.jsonl > gpurun_out/bench14.txt 2>&1 || exit 5
DPT_TUNABLEOP=0 timeout -k 10 300 python bench.py --json-out gpurun_out/bench14.jsonl > gpurun_out/bench14_nt.txt 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof14_vit -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --find --model vit_b_16 --batch-size 128 --no-channels-last --steps 8 --warmup 4 --optimizer adamw > $GRAFT_REPO_ROOT/gpurun_out/prof14.txt 2>&1 || exit 7
