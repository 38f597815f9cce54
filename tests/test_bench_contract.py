"""bench.py driver contract on the CPU: one JSON line from rank 0 with the required keys,
whole-job aggregate value, and the same line shape under torch.distributed.run (gloo, 2 ranks)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--model", "resnet18", "--batch-size", "4", "--image-size", "32", "--num-classes", "10",
        "--steps", "2", "--warmup", "1"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "pct_step_allreduce"}


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n):
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak" and rec["data"] == "synthetic"
    cfg = rec["config"]
    assert cfg["global_batch"] == 4 * n and cfg["parallelism"] == f"dp{n}" and "seq_len" in cfg
    # value is the whole-job images/s: global batch / step time
    assert rec["value"] == pytest.approx(4 * n * 1e3 / rec["ms_per_step"], rel=0.02)


def test_bench_single_process_cpu(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *TINY], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 1)
    # one rank: no collective, so the sync share is not a number (null), not a fake 0.0
    assert lines[0]["pct_step_allreduce"] is None
    assert lines[0]["comm"]["kind"] == "none"


def test_bench_fake_pg_eight_ranks(tmp_path):
    """The N=8 line shape (the driver's scaling run) on torch's fake process group: rank 0 of an
    8-rank job, every collective a no-op; the sync-profiling fields are present."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--fake-pg", *TINY],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    rec = lines[0]
    _check(rec, 8)
    for k in ("pct_step_allreduce", "pct_step_exposed_comm", "sync_profile_window", "comm"):
        assert k in rec, k
    comm = rec["comm"]
    assert comm["kind"] == "gloo" and comm["bucket_cap_mb"] == 25.0 and comm["first_bucket_mb"] == 1.0
    assert len(comm["buckets_mib"]) >= 2 and sum(comm["buckets_mib"]) > 40     # ResNet-18: 42.65 MiB
    assert "rccl_version" in comm

def test_bench_torchrun_gloo_two_ranks(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", *TINY]
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], 2)


def test_bench_self_launches_ranks_without_torchrun(tmp_path):
    """``python bench.py --gpus 2`` with no launcher environment spawns its own 2 ranks (the
    driver's whole-node invocation): the record says 2 GPUs, and the communicator itself saw a
    world of 2 on 2 rank processes."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = lines[0]
    _check(rec, 2)
    assert rec["comm"]["world_size"] == 2 and rec["comm"]["pg_backend"] == "gloo"
    assert len(rec["comm"]["rank_devices"]) == 2
    assert rec["config"]["launcher"] == "self" and isinstance(rec["config"]["env"], dict)
    # self-verification: identical parameters on both ranks after the window, an
    # exact rank+1 all-reduce (1 + 2 = 3) through the collective the gradients used, per-rank times
    v = rec["verify"]
    assert v["ok"] is True and v["params_consistent"] is True and v["selftest_ok"] is True, v
    assert v["selftest_expected"] == 3.0 and len(v["per_rank_ms_per_step"]) == 2
    assert rec["comm"]["selftest_ok"] is True
    # no RCCL communicator on gloo: nothing was opened, and the record says so (not a guess)
    assert v["rccl_channels_opened"] == [None, None]


def test_bench_launcher_never_initialises_hip(tmp_path, monkeypatch, capfd):
    """The self-launching parent must not touch the GPU runtime before it spawns the ranks
    (re-launching after HIP init is unsafe): run the launcher in-process with every torch entry
    point that could initialise HIP made to fail - the job still runs, and nothing was
    initialised in the parent."""
    import importlib.util

    import torch

    def boom(*a, **k):
        raise AssertionError("the launcher process touched the GPU runtime")

    for name in ("device_count", "init", "is_available", "set_device", "synchronize"):
        monkeypatch.setattr(torch.cuda, name, boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.chdir(tmp_path)
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rc = bench.main(["--gpus", "2", *TINY])
    out = capfd.readouterr()
    assert rc == 0, out.err[-3000:]
    assert not torch.cuda.is_initialized()
    lines = _json_lines(out.out)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2


def test_bench_dead_rank_fails_the_job(tmp_path):
    """A rank that dies makes the self-launched job exit non-zero (never a partial record)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--fail-rank", "1", *TINY],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "rank 1 exited with status 17" in r.stderr


def test_bench_launcher_world_size_mismatch_fails(tmp_path):
    """Under a launcher, ``--gpus`` must equal WORLD_SIZE: a 2-rank launch of ``--gpus 4`` is an
    error, not a silently smaller run."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29533")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", *TINY],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    assert not _json_lines(r.stdout)


@pytest.mark.parametrize("n", [1, 2])
def test_bench_same_box_stock_baseline(tmp_path, n):
    """the record carries a stock (--impl torch) number measured by a fresh
    child job of the same shape right after the native run, and vs_baseline divides by it."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--stock-baseline", "on",
                        *TINY], cwd=tmp_path, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    rec = lines[0]
    _check(rec, n)
    b = rec["baseline"]
    stock = b["stock_same_box"]
    assert stock["impl"] == "torch" and stock["n_gpus"] == n and stock["steps"] == 2, stock
    assert b["stock_same_box_img_s"] == stock["img_s"] > 0
    # the record's value is rounded to 2 decimals (tiny CPU runs: ~0.2 img/s), the ratio is not
    lo, hi = (rec["value"] - 0.005) / stock["img_s"], (rec["value"] + 0.005) / stock["img_s"]
    assert lo * 0.999 <= rec["vs_baseline"] <= hi * 1.001, (rec["vs_baseline"], lo, hi)
    assert b["vs_baseline_source"].startswith("stock_same_box")


def _fallback_run(tmp_path, extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DPT_TEST_FAIL_COMM_INIT_RANK"] = "1"      # rank 1 is never ready: every rank falls back
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *extra, *TINY],
                          cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)


def test_bench_fails_closed_on_comm_fallback(tmp_path):
    """when the framework RCCL communicator cannot be created and the ranks
    fall back to torch's communicator, the N > 1 bench exits non-zero and publishes no record."""
    r = _fallback_run(tmp_path, [])
    assert r.returncode == 4, (r.returncode, r.stderr[-3000:])
    assert not _json_lines(r.stdout)
    assert "fell back to torch's c10d communicator" in r.stderr
    assert "DPT_TEST_FAIL_COMM_INIT_RANK" in r.stderr          # the reason travels with the error


def test_bench_allowed_comm_fallback_is_recorded(tmp_path):
    r = _fallback_run(tmp_path, ["--allow-comm-fallback"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    comm = lines[0]["comm"]
    # rank 0 writes the record; its reason is that another rank was not ready
    assert comm["requested"] == "rccl" and "not created on any rank" in comm["fallback_reason"]


def test_bench_no_fallback_reason_without_fallback(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *TINY], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_lines(r.stdout)[0]["comm"]["fallback_reason"] is None


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_on_one_gpu(tmp_path):
    """The self-launch path on a real GPU: ``bench.py --gpus 2 --rehearse-shared-gpu`` without
    torchrun runs 2 rank processes on cuda:0 (gloo control plane, host-bridge collective)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch-size", "32",
           "--image-size", "64", "--steps", "2", "--warmup", "1", "--profile-steps", "2",
           "--rehearse-shared-gpu"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["comm"]["world_size"] == 2 and rec["comm"]["kind"] == "host-async"
    assert rec["config"]["launcher"] == "self"
    assert [d["device"] for d in rec["comm"]["rank_devices"]] == ["cuda:0", "cuda:0"]
    # self-verification through the host-async bridge: exact 1 + 2 and identical parameters
    assert rec["verify"]["ok"] is True and rec["verify"]["selftest_ok"] is True, rec["verify"]
    assert rec["verify"]["selftest_via"] == "host-async"


@pytest.mark.gpu
def test_bench_two_ranks_sharing_one_gpu(tmp_path):
    """bench.py's N > 1 path on a real GPU step (2 torchrun ranks on cuda:0, gloo control plane,
    host-bridge collective: --rehearse-shared-gpu): barrier + synchronize fences, MAX of the rank
    times, the second profiled window with per-bucket comm events, and the JSON line."""
    port = 29000 + os.getpid() % 2000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--batch-size", "32", "--image-size", "64", "--steps", "2", "--warmup", "1",
           "--profile-steps", "2", "--rehearse-shared-gpu"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]
    rec = lines[0]
    assert KEYS <= set(rec) and rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 64 and rec["comm"]["kind"] == "host-async"
    assert rec["value"] == pytest.approx(64 * 1e3 / rec["ms_per_step"], rel=0.02)
    # a real collective ran: the sync share is a measured number and buckets were formed
    assert isinstance(rec["pct_step_allreduce"], float) and rec["pct_step_allreduce"] > 0
    assert rec["comm"]["buckets_mib"] and rec["sync_profile_window"]["steps"] == 2


def test_extra_windows_plan():
    """BASELINE.json configs 4 and 5 ride on the driver's multi-GPU bench: the fp32 window at 4
    GPUs, ViT-B/16 bucket caps at 8, nothing at 1/2 (auto), never for an fp32 headline."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_script", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = bench.parse(["--gpus", "4"])
    plan = dict(bench.extra_windows_plan(a, 4))
    assert list(plan) == ["resnet50_fp32"]
    argv = plan["resnet50_fp32"]
    assert "--no-amp" in argv and argv[argv.index("--gpus") + 1] == "4"
    assert argv[argv.index("--extra-windows") + 1] == "off" and argv[argv.index("--stock-baseline") + 1] == "off"
    plan8 = dict(bench.extra_windows_plan(bench.parse(["--gpus", "8"]), 8))
    assert sorted(plan8) == ["resnet50_rccl_channels16", "resnet50_rccl_channels8", "vit_b16_bucket100mb",
                             "vit_b16_bucket25mb", "vit_b16_bucket400mb"]
    for name, argv in plan8.items():
        if name.startswith("vit"):
            assert argv[argv.index("--model") + 1] == "vit_b_16" and argv[argv.index("--optimizer") + 1] == "adamw"
            # the window's own cap is the last --bucket-cap-mb (argparse keeps the last)
            caps = [argv[i + 1] for i, t in enumerate(argv) if t == "--bucket-cap-mb"]
            assert caps[-1] == name[len("vit_b16_bucket"):-2]
        else:
            assert argv[argv.index("--rccl-channels") + 1] == name[len("resnet50_rccl_channels"):]
    assert bench.extra_windows_plan(bench.parse(["--gpus", "2"]), 2) == []
    plan1 = dict(bench.extra_windows_plan(bench.parse([]), 1))
    assert list(plan1) == ["vit_b16_bucket25mb", "vit_b16_stock", "resnet50_fp32"]
    assert plan1["vit_b16_stock"][-2:] == ["--impl", "torch"]
    assert plan1["vit_b16_bucket25mb"][plan1["vit_b16_bucket25mb"].index("--model") + 1] == "vit_b_16"
    assert bench.extra_windows_plan(bench.parse(["--gpus", "4", "--no-amp"]), 4) == []


def test_bench_extra_window_two_ranks(tmp_path):
    """N = 2: rank 0 runs the extra-window child job (itself two ranks) while rank 1 waits on the
    store; the record carries it and the job exits cleanly."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--extra-windows", "on",
                        "--extra-steps", "2", "--stock-baseline", "off", *TINY], cwd=tmp_path, capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 2)
    w = lines[0]["extra_windows"]["resnet50_fp32"]
    assert "error" not in w, w
    assert w["n_gpus"] == 2 and w["dtype"] == "fp32"


def test_bench_extra_window_record(tmp_path):
    """--extra-windows on: the fp32 child job runs after the headline and lands under
    extra_windows, outside the headline fields."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--extra-windows", "on",
                        "--extra-steps", "2", "--stock-baseline", "off", *TINY], cwd=tmp_path, capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    rec = lines[0]
    _check(rec, 1)
    w = rec["extra_windows"]["resnet50_fp32"]
    assert "error" not in w, w
    assert w["dtype"] == "fp32" and w["n_gpus"] == 1 and w["value"] > 0 and w["steps"] == 2
    assert rec["dtype"] == "bf16"


def _tagged_procs(tag: str):
    """Live processes (zombies excluded) whose environment carries DPT_TEST_TAG=tag."""
    import psutil
    out = []
    for p in psutil.process_iter(["pid"]):
        try:
            if p.status() == psutil.STATUS_ZOMBIE:
                continue
            if p.environ().get("DPT_TEST_TAG") == tag:
                out.append((p.pid, " ".join(p.cmdline())[:200]))
        except (psutil.NoSuchProcess, psutil.AccessDenied, psutil.ZombieProcess):
            continue
    return out


def test_bench_deadline_survives_hung_child_jobs(tmp_path):
    """child jobs (stock run, extra windows) whose ranks hang can neither cost
    the headline record nor leave rank processes behind.  With every child job hanging
    (DPT_TEST_HANG_CHILD), a 2-rank job with a 90 s --deadline still prints its one record in
    time, records the stock run and the extra window as errors, and no process of the job
    (launchers, ranks, child jobs or their ranks) is alive after it exits."""
    import time
    import uuid
    tag = uuid.uuid4().hex
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(DPT_TEST_HANG_CHILD="1", DPT_TEST_TAG=tag)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stock-baseline", "on",
                        "--extra-windows", "on", "--extra-steps", "2", "--deadline", "90", *TINY],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    _check(rec, 2)
    assert "error" in rec["baseline"]["stock_same_box"], rec["baseline"]
    assert rec["baseline"]["vs_baseline_source"] == "stock_reference_constant"
    w = rec["extra_windows"]["resnet50_fp32"]
    assert "error" in w and "cmd" in w, w
    # the record is written by the deadline (or, when the headline window itself ran past it on a
    # loaded CPU, right after the window: no child job is started then), plus the kill grace of a
    # timed-out child job; the job then exits promptly
    tm = rec["timing"]
    assert tm["deadline"] - t0 <= 90 + 5, tm
    assert tm["record"] <= max(tm["deadline"], tm["headline_done"]) + 12, tm
    assert t0 + wall - tm["record"] < 30, (tm, t0, wall)
    time.sleep(1.0)
    left = _tagged_procs(tag)
    assert not left, left


def test_bench_sigterm_during_child_jobs_still_prints_the_record(tmp_path):
    """The driver's time limit arriving while a child job runs: SIGTERM to the self-launching
    parent is forwarded to the ranks, rank 0 kills the child job's process group and prints its
    one record (the stock run marked as not measured), and nothing of the job is left running."""
    import signal
    import time
    import uuid
    tag = uuid.uuid4().hex
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(DPT_TEST_HANG_CHILD="1", DPT_TEST_TAG=tag)
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stock-baseline", "on",
                          "--deadline", "600", *TINY], cwd=tmp_path, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, env=env)
    t0 = time.time()
    seen = False
    while time.time() - t0 < 500:
        line = p.stderr.readline()
        if not line:
            break
        if "headline measured" in line:
            seen = True
            break
    assert seen, "no provisional record on stderr"
    time.sleep(5.0)                     # the (hanging) stock child job is running now
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=120)
    lines = _json_lines(out)
    assert len(lines) == 1, (out, err[-2000:])
    rec = lines[0]
    _check(rec, 2)
    assert "not measured: signal" in rec["baseline"]["stock_same_box"]["error"], rec["baseline"]
    time.sleep(1.0)
    left = _tagged_procs(tag)
    assert not left, left
