"""Grid fill of every kernel in a training step (VERDICT r4 next #2a), from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace -d gpurun_out/kt -o run -- python3 bench.py --steps 5 --warmup 3 --stock-baseline off
    python bench/wave_efficiency.py gpurun_out/kt/.../run_kernel_trace.csv --steps 5 > profiles/...

Per dispatch: workgroups (tiles), the resident-block limit per CU from the trace's own LDS and
VGPR columns (gfx950: 160 KiB LDS and 512 unified VGPRs per SIMD lane, at most 8 waves per SIMD,
one wave per SIMD per 4-wave block), CU slots = 256 x that limit, waves = tiles / slots, and

    wave efficiency = tiles / (ceil(tiles / slots) * slots)

(the fraction of block slots doing work, averaged over the launch's duration, if every block
takes the same time).  ``lost`` = duration x (1 - efficiency) estimates the time a launch spends
with idle slots in its last wave.  Rows aggregate dispatches with the same kernel and grid.
Only the last ``--steps`` steps' worth of dispatches (the timed window) are used: the trace is cut
to its final N x (dispatches per step) rows, with dispatches per step taken from the repeats of
the most frequent kernel when not given.
"""
from __future__ import annotations

import argparse
import math
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from rocprof_rows import load_rows  # noqa: E402

CUS = 256
LDS_PER_CU = 160 * 1024
VGPRS_PER_LANE = 512
MAX_WAVES_PER_SIMD = 8


def granule(v: int, g: int = 8) -> int:
    return (v + g - 1) // g * g


# rocprofv3's VGPR_Count on gfx950 decodes the kernel descriptor's register granules as 4 VGPRs
# where gfx950 allocates 8: a kernel the compiler reports at 118-123 VGPRs
# (-Rpass-analysis=kernel-resource-usage) shows up as 64.  Scale it back.
TRACE_VGPR_SCALE = 2


def blocks_per_cu(lds: int, vgpr: int, agpr: int, wg_threads: int) -> int:
    waves_per_block = max(1, (wg_threads + 63) // 64)
    waves_per_simd_per_block = max(1, math.ceil(waves_per_block / 4))
    regs = granule(vgpr) + granule(agpr)
    by_vgpr = (VGPRS_PER_LANE // max(regs, 8)) // waves_per_simd_per_block
    by_waves = MAX_WAVES_PER_SIMD // waves_per_simd_per_block
    by_lds = LDS_PER_CU // lds if lds > 0 else 10 ** 9
    return max(0, min(by_vgpr, by_waves, by_lds))


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)
    return name[:110]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--filter", default="dpt::")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    rows = load_rows(a.trace)
    # the timed window: the last `steps` optimizer steps (one sgd/adam kernel per step)
    opt = [i for i, r in enumerate(rows) if re.search(r"dpt::(sgd|adam)\w*_kernel", r["Kernel_Name"])]
    if len(opt) >= a.steps + 1:
        rows = rows[opt[-a.steps - 1] + 1: opt[-1] + 1]
    step_ns = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / a.steps
    agg = defaultdict(lambda: {"n": 0, "ns": 0.0, "lost": 0.0})
    total = lost = 0.0
    # split of the estimate (4.63 vs 0.96 ms): grids of at least one full wave of
    # block slots lose their last wave's empty slots as tail time; a grid smaller than one wave
    # has no tail at all - its "empty slots" only mean fewer co-resident blocks, each of which
    # then gets a larger share of the CU, so that part of the estimate is an upper bound
    split = {"multi": [0.0, 0.0], "sub": [0.0, 0.0]}
    for r in rows:
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        total += dur
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        tiles = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) // max(wg, 1)
        bpc = blocks_per_cu(int(r["LDS_Block_Size"]), TRACE_VGPR_SCALE * int(r["VGPR_Count"]),
                            TRACE_VGPR_SCALE * int(r["Accum_VGPR_Count"]), wg)
        slots = CUS * max(bpc, 1)
        eff = tiles / (math.ceil(tiles / slots) * slots) if tiles else 1.0
        key = (short(r["Kernel_Name"]), tiles, bpc, int(r["LDS_Block_Size"]),
               granule(TRACE_VGPR_SCALE * int(r["VGPR_Count"])) + granule(TRACE_VGPR_SCALE * int(r["Accum_VGPR_Count"])))
        e = agg[key]
        e["n"] += 1
        e["ns"] += dur
        e["eff"] = eff
        e["lost"] += dur * (1 - eff)
        lost += dur * (1 - eff)
        sp = split["multi" if tiles >= slots else "sub"]
        sp[0] += dur
        sp[1] += dur * (1 - eff)
    print(f"# Grid fill over {a.steps} timed steps: `{a.trace}`\n")
    print(f"step (first dispatch start -> last end) {step_ns / 1e6:.3f} ms; kernel time {total / a.steps / 1e6:.3f} ms/step; "
          f"estimated last-wave idle time {lost / a.steps / 1e6:.3f} ms/step "
          f"({100 * lost / max(total, 1):.1f} % of kernel time)\n")
    print("| grids | kernel ms/step | estimated idle ms/step | what the estimate means |")
    print("|---|---|---|---|")
    print(f"| >= 1 wave of block slots | {split['multi'][0] / a.steps / 1e6:.3f} | {split['multi'][1] / a.steps / 1e6:.3f} | "
          "last-wave tail: slots really empty while the last blocks finish |")
    print(f"| < 1 wave (one partial wave) | {split['sub'][0] / a.steps / 1e6:.3f} | {split['sub'][1] / a.steps / 1e6:.3f} | "
          "upper bound: no tail; fewer co-resident blocks, each with a larger share of its CU |")
    print()
    print("| kernel | tiles | blocks/CU | LDS B | VGPR+AGPR | waves | wave eff | calls/step | ms/step | lost ms/step |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    items = sorted(agg.items(), key=lambda kv: -kv[1]["lost"])
    for (name, tiles, bpc, lds, regs), e in items[:a.top]:
        if a.filter and a.filter not in name:
            continue
        slots = CUS * max(bpc, 1)
        print(f"| `{name}` | {tiles} | {bpc} | {lds} | {regs} | {tiles / slots:.2f} | {e['eff']:.2f} | "
              f"{e['n'] / a.steps:g} | {e['ns'] / a.steps / 1e6:.4f} | {e['lost'] / a.steps / 1e6:.4f} |")


if __name__ == "__main__":
    sys.exit(main())
