"""List the kernels of ONE training step from a rocprofv3 kernel trace (the step between the last
two fused-optimizer launches), grouped by name, optionally excluding name substrings.

    python bench/step_kernels.py gpurun_out/prof_x [--exclude dpt::conv dpt::bn] [--top 25]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
from collections import defaultdict


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--exclude", nargs="*", default=[])
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--marker", default="sgd", help="kernel-name substring that ends a step")
    a = ap.parse_args(argv)
    path = glob.glob(os.path.join(a.prof_dir, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows[lo:hi]:
        name = r["Kernel_Name"]
        if any(x in name for x in a.exclude):
            continue
        agg[name[:110]][0] += 1
        agg[name[:110]][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    span = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
    print(f"step span {span:.1f} us, {hi - lo} kernels")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{n:4d} {t:9.1f} us  {k}")


if __name__ == "__main__":
    main()
