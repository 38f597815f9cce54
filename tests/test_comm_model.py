"""bench/comm_model.py: the ring all-reduce pricing and the comm-stream replay, and the design
decision it backs - the default 1 MiB tail bucket (--last-bucket-mb) lowers the modelled
exposed gradient sync of ResNet-50 at N = 2/4/8 (measured bucket ready times in
profiles/comm_model_r3_resnet50.jsonl, one MI355X)."""
import json
import os

import pytest

from bench import comm_model as cm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ring_cost_model():
    assert cm.ring_ms(1 << 20, 1, 100.0) == 0.0
    a, b = cm.ring_ms(1 << 20, 8, 100.0), cm.ring_ms(1 << 24, 8, 100.0)
    assert 0 < a < b
    # latency term: 2(N-1) steps of alpha
    assert cm.ring_ms(0, 8, 100.0) == pytest.approx(2 * 7 * cm.ALPHA_US * 1e-3)
    assert cm.busbw(8, "all-links") == pytest.approx(7 * cm.busbw(8, "1-link"))


def test_replay_serialises_the_comm_stream():
    # two buckets ready at 0 and 1 ms, 1 ms each (alpha 0): the second waits for the first
    bw = 2 * 3 / 4 * (1 << 20) / 1e9 / 1e-3  # GB/s that makes a 1 MiB 4-rank all-reduce take 1 ms
    busy, exposed, end = cm.simulate([0.0, 0.5], [1 << 20, 1 << 20], 1.0, 4, bw, alpha_us=0.0)
    assert busy == pytest.approx(2.0) and end == pytest.approx(2.0) and exposed == pytest.approx(1.0)
    # everything hidden behind a long backward
    assert cm.simulate([0.0], [1 << 20], 5.0, 4, bw, alpha_us=0.0)[1] == 0.0


def test_tail_bucket_lowers_modelled_exposed_comm_resnet50():
    with open(os.path.join(ROOT, "profiles", "comm_model_r3_resnet50.jsonl")) as f:
        ms = {m["last_bucket_mb"]: m for m in map(json.loads, f)}
    plain, tail = ms[0.0], ms[1.0]
    assert tail["buckets_mib"][-1] <= 1.0 < plain["buckets_mib"][-1]
    for n in (2, 4, 8):
        for mode in ("1-link", "all-links"):
            e0 = cm.simulate(plain["ready_ms"], [s * 2**20 for s in plain["buckets_mib"]], plain["bwd_end_ms"], n,
                             cm.busbw(n, mode))[1]
            e1 = cm.simulate(tail["ready_ms"], [s * 2**20 for s in tail["buckets_mib"]], tail["bwd_end_ms"], n,
                             cm.busbw(n, mode))[1]
            assert e1 < e0, (n, mode, e0, e1)
