"""Teacher-forced bf16 numerics of the headline configuration (VERDICT r4 next #3a).

From the same fp32 master weights, BatchNorm buffers and batch (ResNet-50, 112 px, batch 64,
1000 classes, after 200 fp32 SGD steps on the learnable prototypes task: at random init the
gradient is chaotic - bf16 and fp32 gradients are nearly orthogonal in BOTH engines, rel-L2 1.2-1.3,
and nothing can be compared), one fp32 torch step is the reference; the native bf16 step's gradient (per
parameter group: stage x {conv, bn, fc}) and its SGD update must be no further from it than
1.25x what stock PyTorch's bf16 autocast step is, averaged over 16 teacher-forced steps
(bench/bf16_teacher.py; committed numbers in profiles/bf16_teacher_r5.md).  This is the check
with statistical power that free-running seed sweeps cannot give: an engine-level error of a few
percent in one layer's gradient shows up here as a ratio far above 1.
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))

# native may be worse than stock by at most this factor per group (mean over steps) ...
RATIO = 1.25
# ... plus this absolute slack for groups where both are at the fp32-rounding level
ABS = 2e-3


def test_native_bf16_step_is_as_close_to_fp32_as_stock_bf16(cuda):
    import bf16_teacher

    res = bf16_teacher.run(steps=16, batch=64, image_size=112, seed=0, log=lambda s: None, pretrain_steps=200,
                           task="prototypes")
    print(bf16_teacher.markdown(res))
    assert res["steps"] == 16
    assert all(r["found_inf"] == 0.0 for r in res["rows"]), [r["found_inf"] for r in res["rows"]]
    bad = {g: v for g, v in res["groups"].items() if v["native"] > RATIO * v["stock"] + ABS}
    assert not bad, bad
    u = res["update"]
    assert u["native"] <= RATIO * u["stock"] + ABS, u
    # the comparison has power: out of the chaotic regime (stock bf16 well correlated with fp32), and
    # bf16 still differs from fp32 measurably in both engines
    assert res["cos"]["stock"] > 0.8, res["cos"]
    assert res["groups"]["all"]["stock"] > 1e-4 and res["groups"]["all"]["native"] > 1e-4
