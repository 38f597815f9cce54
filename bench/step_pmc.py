"""Per-kernel MFMA utilisation and HBM traffic of one ResNet-50 training step (VERDICT r4 next #2b),
from rocprofv3 --pmc passes over ``bench.py`` joined by position within the last step.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d D/pA -o run -- python3 bench.py ...
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/pB -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/pC -o run -- python3 bench.py ...
    rocprofv3 --kernel-trace --output-format csv -d D/kt -o run -- python3 bench.py ...
    python bench/step_pmc.py --passes D/pA D/pB D/pC --trace D/kt > profiles/step_pmc_r5.md

Each pass's dispatches are cut to the last full step (between the last two optimizer kernels);
the passes dispatch the same kernels in the same order, so position k of that step is one
dispatch in every pass (names are checked).  Derived per dispatch:
* MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs);
* HBM-side bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB; MI355X_MICROARCH.md: FETCH_SIZE tallies a
  wide coalesced stream's 128-B requests at 64 B, so the read side is doubled - an upper estimate
  for narrow or scattered reads); achieved TB/s over the kernel-trace duration, and its share of
  the 6.29 TB/s measured copy rate.
Rows aggregate dispatches of the same kernel instantiation.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

COPY_TBS = 6.29
OPT = re.compile(r"dpt::(sgd|adam)\w*_kernel")


def _last_step(rows):
    """rows: [(name, payload)] in dispatch order -> the last full step's slice."""
    opt = [i for i, (n, _) in enumerate(rows) if OPT.search(n)]
    if len(opt) < 2:
        raise SystemExit("fewer than two optimizer dispatches in a pass")
    return rows[opt[-2] + 1: opt[-1] + 1]


def load_pass(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    by = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        i = int(r["Dispatch_Id"])
        by[i][r["Counter_Name"]] = by[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    return _last_step([(names[i], by[i]) for i in sorted(by)])


def load_trace(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    return _last_step([(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                       for r in rows])


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name.replace("void ", ""))
    n = n.replace("dpt::", "").replace("false", "f").replace("true", "t").replace(" ", "")
    return n[:80]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", nargs="+", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    trace = load_trace(a.trace)
    merged = [dict() for _ in trace]
    for d in a.passes:
        p = load_pass(d)
        if len(p) != len(trace):
            raise SystemExit(f"{d}: {len(p)} dispatches in the last step vs {len(trace)} in the trace")
        for k, ((n, c), (tn, _)) in enumerate(zip(p, trace)):
            if short(n) != short(tn):
                raise SystemExit(f"{d}: dispatch {k} is {short(n)} in the pass, {short(tn)} in the trace")
            merged[k].update(c)
    agg = defaultdict(lambda: {"n": 0, "us": 0.0, "mfma_cyc": 0.0, "gui": 0.0, "rd": 0.0, "wr": 0.0})
    tot = {"us": 0.0, "bytes": 0.0, "mfma_cyc": 0.0}
    for (name, us), c in zip(trace, merged):
        e = agg[short(name)]
        e["n"] += 1
        e["us"] += us
        e["mfma_cyc"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        e["gui"] += c.get("GRBM_GUI_ACTIVE", 0.0)
        e["rd"] += 2 * 1024 * c.get("FETCH_SIZE", 0.0)
        e["wr"] += 1024 * c.get("WRITE_SIZE", 0.0)
        tot["us"] += us
        tot["bytes"] += 2 * 1024 * c.get("FETCH_SIZE", 0.0) + 1024 * c.get("WRITE_SIZE", 0.0)
    print(f"# One ResNet-50 bf16 batch-256 training step: MFMA busy and HBM traffic per kernel\n")
    print(f"{len(trace)} dispatches, kernel time {tot['us'] / 1e3:.3f} ms (trace run), HBM-side bytes "
          f"{tot['bytes'] / 1e9:.2f} GB -> {tot['bytes'] / (tot['us'] * 1e-6) / 1e12:.2f} TB/s averaged over "
          f"kernel time\n")
    print("| kernel | calls | us/step | share | MFMA busy | read GB | write GB | TB/s | % of copy rate |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, e in sorted(agg.items(), key=lambda kv: -kv[1]["us"])[:a.top]:
        busy = e["mfma_cyc"] / (e["gui"] / 8 * 256 * 4) if e["gui"] else 0.0
        tbs = (e["rd"] + e["wr"]) / (e["us"] * 1e-6) / 1e12 if e["us"] else 0.0
        print(f"| `{name}` | {e['n']} | {e['us']:.1f} | {e['us'] / tot['us']:.1%} | {busy:.0%} | "
              f"{e['rd'] / 1e9:.3f} | {e['wr'] / 1e9:.3f} | {tbs:.2f} | {tbs / COPY_TBS:.0%} |")


if __name__ == "__main__":
    main()
