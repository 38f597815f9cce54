"""Join rocprofv3 --pmc passes (one directory per pass) and a --kernel-trace run of the same
deterministic driver into one per-dispatch table of derived metrics.

    python bench/pmc_table.py --pass gpurun_out/pmc/p1 gpurun_out/pmc/p2 --trace gpurun_out/pmc/kt \
        [--filter conv_] > profiles/<name>_pmc.md

Derived (MI355X_MICROARCH.md §rocprofv3 PMC slots): MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE/8 XCDs * 32 CUs * 4 SIMDs); wait / issue-stall / active = SQ_WAIT_ANY /
SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES; LDS bank-conflict cycles per
LDS instruction; L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
from collections import defaultdict


def _short(name: str) -> str:
    n = name.replace("void ", "").split("(")[0]
    n = n.replace("dpt::", "").replace("false", "f").replace("true", "t").replace(" ", "")
    return n[:64]


def _load_pass(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        i = int(r["Dispatch_Id"])
        out[i][r["Counter_Name"]] = out[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    return out, names


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="passes", nargs="+", required=True)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--filter", default="conv_")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args(argv)
    ctr = defaultdict(dict)
    names = {}
    for d in a.passes:
        c, n = _load_pass(d)
        for i, v in c.items():
            ctr[i].update(v)
        names.update(n)
    dur = {}
    if a.trace:
        path = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)[0]
        rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
        # the trace run dispatches the same kernels in the same order
        for k, r in enumerate(rows, start=1):
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("| # | kernel | us | MFMA busy | wait | issue-stall | active | VALU/MFMA | LDS conf/instr | L2 hit |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for i in sorted(ctr):
        if a.filter not in names[i]:
            continue
        c = ctr[i]
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        mfma_busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        busy = f"{mfma_busy / (gui / 8 * a.cus * 4):.0%}" if mfma_busy and gui else "-"
        nm = c.get("SQ_INSTS_MFMA")
        valu = f"{c['SQ_INSTS_VALU'] / nm:.1f}" if nm and "SQ_INSTS_VALU" in c else "-"
        lds = f"{c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.2f}" if c.get("SQ_INSTS_LDS") and \
            "SQ_LDS_BANK_CONFLICT" in c else "-"
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        l2 = f"{h / (h + m):.0%}" if h is not None and m is not None and h + m > 0 else "-"
        share = (lambda k: f"{c[k] / wc:.0%}" if k in c else "-")
        us = f"{dur[i]:.1f}" if i in dur else "-"
        print(f"| {i} | `{_short(names[i])}` | {us} | {busy} | {share('SQ_WAIT_ANY')} | "
              f"{share('SQ_WAIT_INST_ANY')} | {share('SQ_ACTIVE_INST_ANY')} | {valu} | {lds} | {l2} |")


if __name__ == "__main__":
    main()
