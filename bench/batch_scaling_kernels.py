"""Which kernels make batch 256 less efficient per image than batch 512?

Two rocprofv3 kernel traces of ``bench.py`` (same steps, batch B1 and B2 = 2 B1): per kernel family
(name without arguments), ms per step at each batch and the per-image cost ratio
(t2 / B2) / (t1 / B1).  A ratio well below 1 marks a kernel with fixed or grid-fill cost at the
smaller batch - the candidates for the batch-256 headline (batch 512 reaches 7 % more
images/s).

    python bench/batch_scaling_kernels.py A_kernel_trace.csv 256 B_kernel_trace.csv 512 --steps 5
"""
from __future__ import annotations

import argparse
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from rocprof_rows import load_rows  # noqa: E402


def per_step(path: str, steps: int):
    rows = load_rows(path)
    opt = [i for i, r in enumerate(rows) if re.search(r"dpt::(sgd|adam)\w*_kernel", r["Kernel_Name"])]
    if len(opt) >= steps + 1:
        rows = rows[opt[-steps - 1] + 1: opt[-1] + 1]
    out = defaultdict(float)
    n = defaultdict(int)
    for r in rows:
        name = re.sub(r"\(.*$", "", r["Kernel_Name"])
        name = re.sub(r"<.*", "", name)[:60]
        out[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
        n[name] += 1
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6 / steps
    return out, {k: v / steps for k, v in n.items()}, span


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace1")
    ap.add_argument("batch1", type=int)
    ap.add_argument("trace2")
    ap.add_argument("batch2", type=int)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args(argv)
    t1, n1, s1 = per_step(a.trace1, a.steps)
    t2, n2, s2 = per_step(a.trace2, a.steps)
    k = a.batch2 / a.batch1
    print(f"# Per-kernel cost at batch {a.batch1} vs {a.batch2}\n")
    print(f"step span {s1:.3f} ms (batch {a.batch1}) vs {s2:.3f} ms (batch {a.batch2}): per-image ratio "
          f"{(s2 / a.batch2) / (s1 / a.batch1):.3f}; kernel sum {sum(t1.values()):.3f} vs {sum(t2.values()):.3f} ms\n")
    print(f"| kernel family | calls/step | ms/step @{a.batch1} | ms/step @{a.batch2} | per-image ratio | "
          f"excess ms/step @{a.batch1} vs linear |")
    print("|---|---|---|---|---|---|")
    rows = []
    for name in set(t1) | set(t2):
        x, y = t1.get(name, 0.0), t2.get(name, 0.0)
        excess = x - y / k          # what batch B1 pays beyond half of batch B2's time
        rows.append((excess, name, x, y))
    for excess, name, x, y in sorted(rows, reverse=True)[:30]:
        ratio = (y / k) / x if x > 0 else float("nan")
        print(f"| `{name}` | {n1.get(name, 0):g} | {x:.4f} | {y:.4f} | {ratio:.3f} | {excess:+.4f} |")
    tot = sum(e for e, *_ in rows)
    print(f"\ntotal excess at batch {a.batch1}: {tot:+.3f} ms/step")


if __name__ == "__main__":
    main()
