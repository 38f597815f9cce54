"""Host-code AddressSanitizer tier: the C++ reducer, communicators, watchdog
and bindings built with ``-fsanitize=address`` (``python csrc/build.py --asan`` ->
build/asan/, GPU kernels not instrumented) run the multi-process gloo DDP tests and the
watchdog tests with libasan preloaded.  Any heap overflow / use-after-free in the reducer's
bucket bookkeeping, hook teardown or comm objects aborts the child and fails this test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    except OSError:
        return None
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


def test_reducer_under_address_sanitizer(tmp_path):
    lib = _libasan()
    if lib is None:
        pytest.skip("gcc libasan not available")
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    import build as native_build

    so = native_build.build(jobs=min(8, os.cpu_count() or 4), asan=True)
    env = dict(os.environ, LD_PRELOAD=lib, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               DPT_NATIVE_LIB=str(so), PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    # the child must really run the sanitized extension
    probe = subprocess.run([sys.executable, "-c", "from distributed_pytorch_training_amd import ops;"
                            "print(ops.native().__file__)"], env=env, capture_output=True, text=True,
                           cwd=tmp_path, timeout=300)
    assert probe.returncode == 0 and str(so) in probe.stdout, probe.stdout + probe.stderr
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_ddp_gloo.py"),
                        os.path.join(ROOT, "tests", "test_watchdog.py")],
                       env=env, capture_output=True, text=True, cwd=tmp_path, timeout=1200)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
