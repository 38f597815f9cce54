"""Per-dispatch comparison of two arms of one bench/ab_step.py run under rocprofv3 --kernel-trace
(the conv_set_breg A/B of round 6, profiles/breg_r6.md): the last optimizer step of each arm,
dispatch by dispatch (the two arms launch the same kernel sequence), grouped by kernel family.

    python bench/breg_compare.py gpurun_out/r6/kt_breg/run_kernel_trace.csv
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict


def is_breg(name: str) -> bool:
    # conv_fwd_kernel's 19th template argument (BREG) is true
    m = re.match(r"void dpt::conv_fwd_kernel<(.*)>\(", name)
    return bool(m) and m.group(1).replace(" ", "").split(",")[-1] == "true"


def family(name: str) -> str:
    m = re.match(r"void dpt::(\w+)<(.*)>\(", name)
    if not m:
        return re.sub(r"\(.*", "", name)[:50]
    k, args = m.group(1), [a.strip() for a in m.group(2).split(",")]
    if k == "conv_fwd_kernel":
        halo = args[14] == "true"
        bnb = args[6] == "true"
        return f"conv_fwd {'3x3-halo' if halo else 'other'} {'dgrad(BNB)' if bnb else 'fwd'}"
    return k


def steps(rows):
    opt = [i for i, r in enumerate(rows) if re.search(r"dpt::(sgd|adam)\w*_kernel", r["Kernel_Name"])]
    return opt


def main(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first_breg = next(i for i, r in enumerate(rows) if is_breg(r["Kernel_Name"]))
    opt = steps(rows)
    a_end = max(i for i in opt if i < first_breg)
    a_start = max(i for i in opt if i < a_end)
    b_end = opt[-1]
    b_start = max(i for i in opt if i < b_end)
    A, B = rows[a_start + 1:a_end + 1], rows[b_start + 1:b_end + 1]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"base step: {len(A)} dispatches, kernel time {sum(map(dur, A)) / 1e3:.3f} ms; "
          f"breg step: {len(B)} dispatches, kernel time {sum(map(dur, B)) / 1e3:.3f} ms\n")
    if len(A) != len(B):
        print("dispatch sequences differ in length; per-family totals only\n")
    fam = defaultdict(lambda: [0.0, 0.0, 0])
    for r in A:
        f = fam[family(r["Kernel_Name"])]
        f[0] += dur(r)
        f[2] += 1
    for r in B:
        fam[family(r["Kernel_Name"])][1] += dur(r)
    print("| kernel family | calls | base us | breg us | delta us |")
    print("|---|---|---|---|---|")
    for k, (a, b, n) in sorted(fam.items(), key=lambda kv: -(kv[1][1] - kv[1][0])):
        if abs(b - a) > 1 or a > 100:
            print(f"| {k} | {n} | {a:.1f} | {b:.1f} | {b - a:+.1f} |")
    if len(A) == len(B):
        print("\nlargest per-dispatch changes (same position in the step):\n")
        print("| pos | kernel (base) | grid | base us | breg us | ratio |")
        print("|---|---|---|---|---|---|")
        pairs = [(dur(b) - dur(a), i, a, b) for i, (a, b) in enumerate(zip(A, B))]
        for d, i, a, b in sorted(pairs, key=lambda t: -abs(t[0]))[:25]:
            grid = int(a["Grid_Size_X"]) // max(1, int(a["Workgroup_Size_X"]))
            print(f"| {i} | {family(a['Kernel_Name'])} | {grid} | {dur(a):.1f} | {dur(b):.1f} | {dur(b) / max(dur(a), 1e-9):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])


def pmc(path: str) -> None:
    """MFMA busy, wait share and vector-memory read instructions per kernel family, last step of
    each arm, from a ``rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
    SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD`` run of the same A/B."""
    per = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = r
    ids = sorted(per)
    rows = [dict(meta[d], **{"Kernel_Name": meta[d]["Kernel_Name"]}) for d in ids]
    first_breg = next(i for i, r in enumerate(rows) if is_breg(r["Kernel_Name"]))
    opt = steps(rows)
    a_end = max(i for i in opt if i < first_breg)
    a_start = max(i for i in opt if i < a_end)
    b_end = opt[-1]
    b_start = max(i for i in opt if i < b_end)
    simds = 256 * 4
    for arm, lo, hi in (("base", a_start + 1, a_end + 1), ("breg", b_start + 1, b_end + 1)):
        fam = defaultdict(lambda: defaultdict(float))
        for i in range(lo, hi):
            c = per[ids[i]]
            f = fam[family(rows[i]["Kernel_Name"])]
            for k, v in c.items():
                f[k] += v
        print(f"\n{arm}: | kernel family | MFMA busy | wait / wave cycles | VMEM read instr (M) |")
        print("|---|---|---|---|")
        for k, f in sorted(fam.items()):
            if not k.startswith("conv_fwd"):
                continue
            # GRBM_GUI_ACTIVE sums the 8 XCDs (bench/step_pmc.py)
            busy = f["SQ_VALU_MFMA_BUSY_CYCLES"] / max(f["GRBM_GUI_ACTIVE"] / 8 * simds, 1)
            wait = f["SQ_WAIT_INST_ANY"] / max(f["SQ_WAVE_CYCLES"], 1)
            print(f"| {k} | {100 * busy:.1f} % | {100 * wait:.1f} % | {f['SQ_INSTS_VMEM_RD'] / 1e6:.2f} |")


if __name__ == "__main__" and len(sys.argv) > 2:
    pmc(sys.argv[2])
