"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv, restricted to the last N steps.

Steps are delimited by the fused-optimizer tail kernel (one per step, native engine) or by
an explicit --marker kernel-name regex.  Writes a markdown table (family ms/step, top kernels).
"""
import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_prof import family  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default=r"optim_tail|multi_tensor_apply_kernel.*SGD|amp_update_scale")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv)
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if re.search(a.marker, r["Kernel_Name"])]
    if len(marks) < a.steps + 1:
        print(f"only {len(marks)} step markers", file=sys.stderr)
        return 1
    lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
    win = rows[lo:hi]
    t_wall = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6
    fam, per = defaultdict(float), defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        busy += d
        fam[family(r["Kernel_Name"])] += d
        per[r["Kernel_Name"]][0] += 1
        per[r["Kernel_Name"]][1] += d
    n = a.steps
    print(f"# Per-step kernel breakdown (last {n} steps of `{a.dir}`)\n")
    print(f"- wall span {t_wall/n:.3f} ms/step, summed kernel time {busy/n:.3f} ms/step, "
          f"{len(win)/n:.0f} kernels/step\n")
    print("| family | ms/step | % of kernel time |\n|---|---|---|")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v/n:.3f} | {100*v/busy:.1f} |")
    print("\n| kernel | calls/step | ms/step | avg us |\n|---|---|---|---|")
    for name, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1])[: a.top]:
        nm = (name if len(name) < 100 else name[:97] + "...").replace("|", "/")
        print(f"| `{nm}` | {c/n:.1f} | {d/n:.3f} | {1e3*d/c:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
