"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` run into markdown.

    python bench/summarize_prof.py gpurun_out/prof_native [--steps N] > profiles/x.md

Groups kernels into families (convolution, batch-norm, elementwise, optimizer, RCCL, ...)
and lists the top kernels by total time, so per-step time can be attributed.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict

FAMILIES = [
    ("native: optimizer (fused SGD/Adam, grad_check, tail)", r"dpt::(sgd|adam|grad_check|optim_tail)"),
    ("native: MFMA convolutions (fwd/dgrad/wgrad + reduce/flip)", r"dpt::conv_"),
    ("native: fused BatchNorm(+add)(+ReLU)", r"dpt::bn_"),
    ("native: ViT block kernels", r"dpt::(ln_|gelu|rows_copy|colsum|sum_partials)"),
    ("native: flash attention (fwd / bwd phases)", r"dpt::attn"),
    ("native: metrics/augment/comm/pool kernels", r"dpt::"),
    ("RCCL", r"nccl|rccl|AllReduce|Broadcast"),
    ("conv (MIOpen/CK igemm, xdlops)", r"igemm|Conv|conv|xdlops|gridwise_gemm|DeviceGroupedConv|naive_conv|ImplicitGemm|kernel_grouped_conv"),
    ("batch-norm", r"batch_norm|batchnorm|BatchNorm|MIOpenBatchNorm|bn_"),
    ("GEMM (hipBLASLt/rocBLAS)", r"Cijk|gemm|Gemm|rocblas"),
    ("pooling", r"pool|Pool"),
    ("loss/softmax", r"softmax|nll|cross_entropy|log_softmax"),
    ("foreach / multi-tensor (stock optimizer, AMP)", r"multi_tensor|foreach|amp_|_amp"),
    ("elementwise / copy / reduce", r"elementwise|vectorized|reduce|copy|fill|unrolled|index|Memcpy|cat"),
]


def family(name: str) -> str:
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args(argv)
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        print(f"no kernel_stats.csv under {a.dir}", file=sys.stderr)
        return 1
    rows = list(csv.DictReader(open(files[0])))
    tot_key = "TotalDurationNs" if "TotalDurationNs" in rows[0] else [k for k in rows[0] if "Total" in k][0]
    fam = defaultdict(float)
    total = 0.0
    for r in rows:
        ns = float(r[tot_key])
        fam[family(r["Name"])] += ns
        total += ns
    div = a.steps or 1
    print(f"# rocprofv3 kernel summary: `{a.dir}`\n")
    print(f"Total kernel time {total/1e6:.2f} ms" + (f" = {total/1e6/div:.3f} ms/step over {div} steps" if a.steps else ""))
    print("\n| family | ms" + ("/step" if a.steps else "") + " | % |\n|---|---|---|")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v/1e6/div:.3f} | {100*v/total:.1f} |")
    print(f"\n| top kernels | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    rows.sort(key=lambda r: -float(r[tot_key]))
    for r in rows[: a.top]:
        name = r["Name"]
        name = name if len(name) < 110 else name[:107] + "..."
        name = name.replace("|", "/")
        calls = r.get("Calls", "?")
        avg = float(r.get("AverageNs", 0.0)) / 1e3
        print(f"| `{name}` | {calls} | {float(r[tot_key])/1e6:.2f} | {avg:.1f} | {float(r.get('Percentage', 0)):.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
