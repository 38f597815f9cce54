"""The framework RCCL communicator on a real MI355X: per-communicator channel (CTA) bounds and
the production watchdog / abort path (csrc/rccl_comm.cpp, csrc/watchdog.cpp).

These replace what the reference inherits from ProcessGroupNCCL (reference train_ddp.py:65:
default timeout, watchdog thread, abort on error).  Each case runs in
a fresh interpreter: an aborted communicator (and RCCL's NCCL_DEBUG log) must not leak into
the pytest process.  A 1-rank RcclComm is a real communicator (ncclCommInitRank[Config],
RCCL kernels on its own stream); one GPU cannot host two RCCL ranks.
"""
import os
import re
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(code: str, timeout: int = 120, **env_extra):
    env = dict(os.environ, **env_extra)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


_CHANNELS = """
    import torch
    from distributed_pytorch_training_amd.parallel.comm import make_comm
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    comm = make_comm(dev, 0, 1, rccl_channels={n})
    t = torch.ones(1 << 20, device=dev)
    comm.all_reduce(t, True)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.ones_like(t))
    print("ctas", comm.min_ctas, comm.max_ctas, flush=True)
    comm.destroy()
    print("ok", flush=True)
"""


def _channel_counts(log: str):
    """Channel counts RCCL reports at communicator init: "Channel 00/NN" ring lines and the
    "<n> coll channels" summary."""
    ring = {int(m) for m in re.findall(r"Channel \d+/(\d+)", log)}
    coll = {int(m) for m in re.findall(r"(\d+) coll channels", log)}
    return ring, coll


@pytest.mark.parametrize("n", [8, 16])
def test_rccl_channels_use_the_config_api(n):
    """``--rccl-channels N`` creates the framework communicator through ncclCommInitRankConfig
    with minCTAs = maxCTAs = N (the process-wide NCCL_*NCHANNELS environment is not touched).
    A 1-rank communicator always opens RCCL's maximum ring count (128 on this build, logged
    below), so the resulting channel count itself is only observable at N > 1; that the
    values land in RCCL's config parser is pinned by the next test."""
    r = _run(_CHANNELS.format(n=n), NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT")
    log = r.stdout + r.stderr
    assert r.returncode == 0 and "ok" in r.stdout, log[-4000:]
    assert f"ctas {n} {n}" in r.stdout
    assert "ncclCommInitRankConfig" in log, log[-3000:]
    assert "NCCL_MIN_NCHANNELS" not in os.environ and "NCCL_MAX_NCHANNELS" not in os.environ
    ring, coll = _channel_counts(log)
    print(f"channels={n}: 1-rank ring={sorted(ring)} coll={sorted(coll)}")


def test_rccl_config_values_reach_rccl():
    """The ncclConfig_t the framework builds (rccl.h 2.27 layout) is read field-for-field by the
    bundled RCCL 2.26: an inconsistent pair (minCTAs 24 > maxCTAs 12) is rejected by RCCL's own
    validation, which quotes exactly the two values we set (a layout mismatch would quote other
    numbers or accept it); a consistent pair is accepted."""
    r = _run("""
        import torch
        from distributed_pytorch_training_amd import ops
        C = ops.native()
        torch.cuda.set_device(0)
        try:
            C.RcclComm(C.RcclComm.new_unique_id(), 0, 1, 0, 24, 12)      # min > max
            print("accepted", flush=True)
        except RuntimeError as e:
            print("rejected:", e, flush=True)
        b = C.RcclComm(C.RcclComm.new_unique_id(), 0, 1, 0, 6, 9)
        assert (b.min_ctas, b.max_ctas) == (6, 9)
        b.destroy()
        print("ok", flush=True)
    """, NCCL_DEBUG="WARN")
    log = r.stdout + r.stderr
    assert r.returncode == 0 and "ok" in r.stdout, log[-4000:]
    assert "rejected: RCCL error invalid argument" in r.stdout, log[-3000:]
    assert "Invalid config min/max channels attribute value 24/12" in log, log[-3000:]


def test_rccl_default_channels_logged():
    """Reference point: what RCCL picks by itself for this communicator (ncclCommInitRank)."""
    r = _run(_CHANNELS.format(n=0), NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT")
    log = r.stdout + r.stderr
    assert r.returncode == 0 and "ok" in r.stdout, log[-4000:]
    assert "ctas 0 0" in r.stdout and "ncclCommInitRankConfig" not in log
    ring, coll = _channel_counts(log)
    print(f"default: ring={sorted(ring)} coll={sorted(coll)}")


def test_watchdog_aborts_a_stuck_collective():
    """A collective queued behind ~3 s of device work with a 1 s timeout: the watchdog thread
    trips within ~1-2 s (hipEventQuery polling), aborts the communicator (ncclCommAbort),
    ``check()`` raises at the next host touch point naming the collective, and ``destroy()``
    returns without hanging."""
    r = _run("""
        import time, torch
        from distributed_pytorch_training_amd.parallel.comm import make_comm
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        comm = make_comm(dev, 0, 1)
        comm.enable_watchdog(1.0, 0.05, -1.0)     # timeout 1 s, poll 50 ms, no process exit
        t = torch.ones(4096, device=dev)
        comm.all_reduce(t, False)                  # a normal collective completes: no trip
        torch.cuda.synchronize()
        time.sleep(1.5)
        assert not comm.watchdog_tripped and comm.watchdog_outstanding == 0
        comm.check()
        t0 = time.time()
        comm._test_spin(3000.0)                    # the "peer that never arrives"
        comm.all_reduce(t, False)                  # collective #1, behind the spin
        while not comm.watchdog_tripped and time.time() - t0 < 6.0:
            time.sleep(0.02)
        trip_s = time.time() - t0
        assert comm.watchdog_tripped, "watchdog did not trip"
        assert 0.9 <= trip_s <= 2.5, trip_s
        try:
            comm.check()
            raise AssertionError("check() did not raise")
        except RuntimeError as e:
            msg = str(e)
        assert "collective #1" in msg and "did not complete within 1 s" in msg, msg
        try:
            comm.all_reduce(t, False)
            raise AssertionError("an aborted communicator accepted work")
        except RuntimeError as e:
            assert "aborted" in str(e)
        t1 = time.time()
        comm.destroy()
        destroy_s = time.time() - t1
        torch.cuda.synchronize()                   # the spin drains; the device is idle at exit
        print(f"ok trip_s={trip_s:.2f} destroy_s={destroy_s:.2f}", flush=True)
        assert destroy_s < 5.0
    """)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "[dpt watchdog" in r.stderr and "aborting the communicator" in r.stderr
    print(r.stdout.strip())


def test_watchdog_async_error_branch():
    """An RCCL asynchronous error (injected through the test hook in place of a broken peer)
    trips the watchdog, aborts the communicator and surfaces at ``check()``."""
    r = _run("""
        import time, torch
        from distributed_pytorch_training_amd.parallel.comm import make_comm
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        comm = make_comm(dev, 0, 1)
        comm.enable_watchdog(60.0, 0.05, -1.0)
        assert comm.async_error() == ""
        comm.inject_async_error("remote process exited or there was a network error")
        t0 = time.time()
        while not comm.watchdog_tripped and time.time() - t0 < 3.0:
            time.sleep(0.02)
        assert comm.watchdog_tripped, "async error did not trip the watchdog"
        try:
            comm.check()
            raise AssertionError("check() did not raise")
        except RuntimeError as e:
            assert "asynchronous error: remote process exited" in str(e), str(e)
        comm.destroy()
        torch.cuda.synchronize()
        print(f"ok {time.time() - t0:.2f}", flush=True)
    """)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_graph_replay_is_tracked_by_the_watchdog():
    """``Collective.track`` (called by engine/graph.py after every replay) hands the watchdog a
    completion marker on the current stream: it is outstanding while the stream is busy and
    retires when the work finishes, so --dist-timeout also covers hipGraph steps."""
    r = _run("""
        import time, torch
        from distributed_pytorch_training_amd.parallel.comm import make_comm
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        comm = make_comm(dev, 0, 1)
        comm.enable_watchdog(30.0, 0.05, -1.0)
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            comm._test_spin(800.0, True)           # stands in for a replayed step
            comm.track()
        assert comm.watchdog_outstanding == 1
        torch.cuda.synchronize()
        t0 = time.time()
        while comm.watchdog_outstanding and time.time() - t0 < 3.0:
            time.sleep(0.02)
        assert comm.watchdog_outstanding == 0 and not comm.watchdog_tripped
        comm.destroy()
        print("ok", flush=True)
    """)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
