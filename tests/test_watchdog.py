"""Communicator watchdog decision logic (csrc/watchdog.h WatchdogCore) with a fake clock.

The GPU watchdog thread (StreamWatchdog) feeds WatchdogCore real time and hipEventQuery; here
the clock and the completion predicate are explicit, so the timeout / async-error / FIFO
semantics are pinned on CPU.  Replaces the ProcessGroupNCCL watchdog the reference inherits
(reference train_ddp.py:65)."""
import pytest

from distributed_pytorch_training_amd import ops


@pytest.fixture(scope="module")
def C():
    if not ops.native_available():
        pytest.skip("native extension not built")
    return ops.native()


def test_completed_work_never_trips(C):
    w = C.WatchdogCore(10.0)
    done = set()
    for seq in range(5):
        w.enqueue(seq, float(seq))
    done.update({0, 1, 2})
    trip, completed = w.poll(11.5, lambda s: s in done)
    assert trip == "" and completed == [0, 1, 2]
    assert w.outstanding == 2
    done.update({3, 4})
    trip, completed = w.poll(100.0, lambda s: s in done)   # late but complete: fine
    assert trip == "" and completed == [3, 4] and not w.tripped


def test_timeout_trips_once_on_oldest(C):
    w = C.WatchdogCore(5.0)
    w.enqueue(7, 0.0)
    w.enqueue(8, 3.0)
    assert w.poll(4.9, lambda s: False)[0] == ""
    assert w.oldest_age(4.9) == pytest.approx(4.9)
    trip, _ = w.poll(5.1, lambda s: False)
    assert "collective #7" in trip and "5 s" in trip and "2 outstanding" in trip
    assert w.tripped and w.reason == trip
    assert w.poll(50.0, lambda s: False)[0] == ""    # reported once


def test_fifo_completion_only_pops_from_front(C):
    """One comm stream completes in order: a 'done' item behind a pending one stays queued
    (its event is not consulted out of order) and the pending head still times out."""
    w = C.WatchdogCore(1.0)
    w.enqueue(0, 0.0)
    w.enqueue(1, 0.0)
    asked = []

    def done(s):
        asked.append(s)
        return s == 1

    trip, completed = w.poll(0.5, done)
    assert completed == [] and asked == [0] and w.outstanding == 2
    assert w.poll(1.5, done)[0] != ""


def test_async_error_trips_immediately(C):
    w = C.WatchdogCore(1e9)
    trip, _ = w.poll(0.0, lambda s: True, "remote process exited")
    assert "asynchronous error" in trip and "remote process exited" in trip
    assert w.tripped


def test_idle_watchdog(C):
    w = C.WatchdogCore(1.0)
    assert w.poll(1e6, lambda s: True) == ("", [])
    assert w.oldest_age(5.0) == 0.0 and not w.tripped
