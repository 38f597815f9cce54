"""One training step's kernels in launch order with their grid sizes and durations (rocprofv3
kernel trace), so per-shape conv times in the real step can be read off.

    python bench/step_shapes.py gpurun_out/prof/<host> [--marker sgd] [--filter conv_]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--marker", default="sgd", help="kernel-name substring that ends a step")
    ap.add_argument("--filter", default="", help="only kernels whose name contains this")
    a = ap.parse_args(argv)
    path = glob.glob(os.path.join(a.prof_dir, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    tot = 0.0
    for r in rows[lo:hi]:
        name = r["Kernel_Name"]
        if a.filter and a.filter not in name:
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += us
        short = name.split("(")[0].replace("void ", "")[:90]
        print(f"{us:8.1f} us  grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):6d}x{r['Grid_Size_Y']:>3}"
              f"  vgpr {r['VGPR_Count']:>3}+{r['Accum_VGPR_Count']:>3} lds {r['LDS_Block_Size']:>6}  {short}")
    print(f"total {tot / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
