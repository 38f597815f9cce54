"""The kernels of ONE training step in issue order, from a rocprofv3 kernel trace: duration, grid,
idle gap before each kernel, and a short template-stripped name - for attributing time to layers
and finding launch gaps.

    python bench/step_timeline.py gpurun_out/prof/<host> [--marker sgd] [--min-us 0] > profiles/x.txt
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re


def short(name: str) -> str:
    base = name.split("(")[0]
    m = re.match(r"(?:void )?(?:dpt::)?([\w:]+)(<.*>)?", base)
    if not m:
        return base[:60]
    tmpl = m.group(2) or ""
    return (m.group(1) + tmpl)[:90]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--marker", default="sgd", help="kernel-name substring that ends a step")
    ap.add_argument("--min-us", type=float, default=0.0, help="hide kernels shorter than this")
    a = ap.parse_args(argv)
    paths = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(paths[0])), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    t0 = int(rows[lo]["Start_Timestamp"])
    prev_end = t0
    busy = gaps = 0.0
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7} {'grid':>9} name")
    for r in rows[lo:hi]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur, gap = (e - s) / 1e3, max(0, s - prev_end) / 1e3
        busy += dur
        gaps += gap
        prev_end = max(prev_end, e)
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "1"
        try:
            blocks = int(grid) // max(1, int(wg))
        except ValueError:
            blocks = grid
        if dur >= a.min_us:
            print(f"{(s - t0) / 1e3:9.1f} {dur:8.1f} {gap:7.1f} {blocks:>9} {short(r['Kernel_Name'])}")
    span = (prev_end - t0) / 1e3
    print(f"\nstep span {span:.1f} us, {hi - lo} kernels, kernel busy {busy:.1f} us, idle gaps {gaps:.1f} us")


if __name__ == "__main__":
    main()
