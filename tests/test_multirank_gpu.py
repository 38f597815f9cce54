"""World size 2 on ONE MI355X: the multi-rank GPU data path of the native engine.

Two processes share cuda:0.  RCCL needs one device per rank, so the native engine runs with
``--comm host``: the C++ reducer's bucket collectives go through the ``HostBridgeComm``
seam (csrc/host_comm.cpp) - comm-stream event ordering, steal-mode gathers, 16-bit weight
shadow gradients, the bf16 wire pack/unpack, the comm-stream non-finite check, the rank-0
parameter/buffer broadcasts and the bucket rebuild all run exactly as with RCCL; only the
``ncclAllReduce`` / ``ncclBroadcast`` call is replaced by D2H -> gloo (host) -> H2D.

Three checks:
* ``test_world_size_2_matches_ddp_semantics`` - 3 steps on plain torch layers (MIOpen convs)
  against the reference's DDP semantics (train_ddp.py:303-311 with torch DDP defaults,
  GradScaler + SGD train_ddp.py:339-346, 207-209) emulated in ONE process with plain torch
  (every rank's batch, rank-0 buffer broadcast before each forward, averaged gradients), each
  step from the parameter / buffer / optimizer / scaler state the native step started from.  No
  collective is involved in the emulation, so it cannot share a bug with the path under test
  (torch DDP over gloo with CUDA tensors is not used: in this environment gloo's CUDA
  all-reduce returned wrong sums in diagnostics, while host-tensor gloo is exact).  Ranks start
  from different seeds (rank 0's broadcast must win); under AMP rank 1's step-2 batch carries
  an inf, so that step must be skipped on BOTH ranks and the scale backed off.
* ``test_world_size_2_reduces_local_gradients_exactly`` - the FULL native engine (MFMA convs,
  fused BN, bf16 weight shadows, steal-mode gathers): one world-size-2 step must reduce to
  exactly the sum of the two ranks' local world-size-1 gradients (fp32 wire) or
  bf16(bf16(a) + bf16(b)) (bf16 wire).  Comparing MFMA-conv runs with MIOpen ones is not
  meaningful at this level (bf16 rounding flips max-pool argmaxes and ReLU masks, so even two
  conv implementations disagree by tens of percent on the stem gradients).
* ``test_world_size_2_native_engine_skips_inf_step_on_every_rank`` - full engine, inf on rank 1.
Every check also asserts that both ranks end with bit-identical parameters.
"""
import os
import socket
import time
import traceback

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 3
INF_STEP = 1          # 0-based step whose rank-1 batch carries an inf (AMP cases)
B = 32
LR = 0.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(rank, device, steps, inf_step):
    out = []
    for step in range(steps):
        g = torch.Generator().manual_seed(1000 * step + rank)
        x = torch.randn(B, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (B,), generator=g)
        if step == inf_step and rank == 1:
            x[0, 0, 0, 0] = float("inf")
        out.append((x.to(device).contiguous(memory_format=torch.channels_last), y.to(device)))
    return out


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().clone()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def _run_native(rank, ws, device, extra, amp, steps, inf_step, record=False):
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    argv = ["--model", "resnet18", "--dataset", "synthetic", "--no-cuda-graph", "--image-size", "32", "--num-classes", "10",
            "--batch-size", str(B), "--channels-last", "--lr", str(LR), "--comm", "host", "--ddp-debug", *extra]
    if amp:
        argv += ["--amp", "--amp-dtype", "bf16"]
    args = parse_args(argv)
    # ranks start different (rank 0's weights must win); a local (ws=1) run starts from rank 0's
    torch.manual_seed(1234 + (rank if ws > 1 else 0))
    model = build_model("resnet18", 10, device, image_size=32, channels_last=True)
    tr = Trainer(model, args, rank if ws > 1 else 0, ws, device, log=lambda s: None)
    ddp = tr.ddp

    def scale_now():
        return float(tr.scaler.scale_tensor.item()) if amp else 1.0

    snaps = []
    for x, y in _batches(rank, device, steps, inf_step):
        if record:   # the state this step starts from (teacher forcing for the emulation)
            torch.cuda.synchronize()
            snaps.append({"params": {n: _cpu(p) for n, p in model.named_parameters()},
                          "buffers": {n: _cpu(b) for n, b in model.named_buffers()},
                          "opt": _cpu(tr.optimizer.state_dict()),
                          "scaler": _cpu(tr.scaler.state_dict()) if amp else None})
        tr.train_step(x, y)
        if record:
            torch.cuda.synchronize()
            sc = scale_now()
            # the arena may have been rebuilt in gradient-ready order after the first step
            pos = {id(p): i for i, p in enumerate(ddp.arena.params)}
            grads = ddp.averaged_grads()
            snaps[-1].update(
                after_params={n: _cpu(p) for n, p in model.named_parameters()},
                after_buffers={n: _cpu(b) for n, b in model.named_buffers()},
                grads={n: (grads[pos[id(p)]] / snaps[-1]["scaler"]["scale"] if amp else grads[pos[id(p)]]).float().cpu()
                       for n, p in model.named_parameters()},
                after_scale=sc,
                after_tracker=float(tr.scaler.growth_tracker.item()) if amp else 0.0)
    torch.cuda.synchronize()
    if ws > 1:
        assert ddp.comm is not None and ddp.comm.kind.startswith("host")
    res = {"replays": tr.graphed.replays if tr.graphed is not None and tr.graphed.graph is not None else 0,
           "params": {n: p.detach().float().cpu() for n, p in model.named_parameters()},
           "buffers": {n: b.detach().float().cpu() for n, b in model.named_buffers()},
           "comm_ops": int(ddp.comm.ops) if ddp.comm is not None else 0,
           "buckets": int(ddp.reducer.num_buckets), "snaps": snaps}
    # the arena after the step: the last backward's (loss-scaled) gradient sum, as reduced
    pos = {id(p): i for i, p in enumerate(ddp.arena.params)}
    res["raw_grads"] = {n: ddp.arena.grad_views[pos[id(p)]].detach().float().cpu().clone()
                        for n, p in model.named_parameters()}
    scale = scale_now()
    grads = ddp.averaged_grads()       # last step's (loss-scaled) sum / world size
    res["grads"] = {n: (grads[pos[id(p)]] / scale).float().cpu() for n, p in model.named_parameters()}
    res["scale"] = scale
    res["tracker"] = float(tr.scaler.growth_tracker.item()) if amp else 0.0
    if ws > 1:
        tr.check_consistency()         # params bit-identical + collective sequence (--ddp-debug)
    tr.close()
    return res


def _emulate(ws, rank, device, amp, steps, inf_step, snaps0):
    """DDP semantics for ``ws`` ranks in one process with plain torch (see module doc), one step
    at a time from the state the native step started from (``snaps0``: rank 0's - the broadcast
    source - parameters, buffers, optimizer and scaler state before each step).  Teacher forcing
    keeps the comparison at rounding level: a free-running 3-step emulation diverges from a
    1-ulp optimizer rounding difference through ReLU / max-pool decision flips (round 3: 1.5e-3
    on some boxes), which says nothing about the semantics under test."""
    from distributed_pytorch_training_amd.models import build_model

    torch.manual_seed(1234)
    model = build_model("resnet18", 10, device, image_size=32, channels_last=True)
    params = list(model.named_parameters())
    data = [_batches(q, device, steps, inf_step) for q in range(ws)]
    out = []
    for step in range(steps):
        snap = snaps0[step]
        with torch.no_grad():
            for n, p in params:
                p.copy_(snap["params"][n])
        opt = torch.optim.SGD(model.parameters(), lr=LR, momentum=0.9, weight_decay=5e-4)
        opt.load_state_dict(snap["opt"])
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        if amp:
            scaler.load_state_dict(snap["scaler"])
        total = [torch.zeros_like(p) for _, p in params]
        my_bufs = None
        for q in range(ws):
            with torch.no_grad():     # rank 0's buffers, broadcast before every rank's forward
                for n, b in model.named_buffers():
                    b.copy_(snap["buffers"][n])
            for _, p in params:
                p.grad = None
            x, y = data[q][step]
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = torch.nn.functional.cross_entropy(model(x), y)
            scaler.scale(loss).backward()
            for t, (_, p) in zip(total, params):
                t += p.grad
            if q == rank:
                my_bufs = {n: b.detach().float().cpu().clone() for n, b in model.named_buffers()}
        for t, (_, p) in zip(total, params):
            p.grad = t / ws
        grads = {n: (p.grad / scaler.get_scale() if amp else p.grad).detach().float().cpu() for n, p in params}
        scaler.step(opt)
        scaler.update()
        out.append({"params": {n: p.detach().float().cpu() for n, p in params}, "buffers": my_bufs,
                    "grads": grads, "scale": float(scaler.get_scale()) if amp else 1.0,
                    "tracker": float(scaler._get_growth_tracker()) if amp else 0.0})
    return out


def _worker(rank, ws, port, out_dir, extra, amp, steps, inf_step, mode):
    try:
        import torch.distributed as dist

        from distributed_pytorch_training_amd.utils.env import setup_miopen_env

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws),
                          RANK=str(rank), LOCAL_RANK="0")
        # a private MIOpen find-db seeded from the shipped one: the solutions MIOpen picks for the
        # native run and the emulation must not depend on what earlier tests wrote to the shared
        # user db (seen: the AMP case 0.0 grad error alone, 35 % after the full GPU suite)
        os.environ.pop("MIOPEN_USER_DB_PATH", None)
        setup_miopen_env(scratch=os.path.join(out_dir, f"miopen{rank}"))
        if mode == "emulate":
            # keep MIOpen's reduced-precision fp32 solver families (Winograd, FFT) out of both the
            # engine under test and the emulation, so the semantics check does not see which of
            # them immediate mode picked for each run (round 2: 5e-3 fp32 gradient drift from
            # that alone).  (ATen's own kernels are no way out: with MIOpen off the BN bias
            # gradients of this net move by 1e-2 for 1e-9 parameter perturbations.)
            os.environ.update(MIOPEN_DEBUG_CONV_WINOGRAD="0", MIOPEN_DEBUG_CONV_FFT="0")
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        torch.backends.cudnn.deterministic = True     # MIOpen: deterministic algorithms
        native = _run_native(rank, ws, dev, extra, amp, steps, inf_step, record=(mode == "emulate"))
        if mode == "emulate":
            # rank 0's pre-step states (the broadcast source) drive both ranks' emulations
            torch.save(native["snaps"], os.path.join(out_dir, f"snaps{rank}.pt"))
            dist.barrier()
            snaps0 = torch.load(os.path.join(out_dir, "snaps0.pt"), weights_only=False)
            ref = _emulate(ws, rank, dev, amp, steps, inf_step, snaps0)
        elif mode == "local":
            ref = _run_native(rank, 1, dev, extra, amp, steps, inf_step)
        else:
            ref = None
        torch.save({"native": native, "ref": ref}, os.path.join(out_dir, f"r{rank}.pt"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
            f.write(traceback.format_exc())
        raise


def _spawn(tmp_path, extra, amp=True, steps=STEPS, inf_step=INF_STEP, mode="emulate", timeout=150):
    import torch.multiprocessing as mp

    ctx = mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), extra, amp, steps, inf_step, mode),
                             nprocs=2, start_method="spawn", join=False)
    deadline = time.time() + timeout
    try:
        while not ctx.join(timeout=2):
            if time.time() > deadline:
                raise TimeoutError("multi-rank GPU workers did not finish")
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
    errs = [p.read_text() for p in tmp_path.glob("err*.txt")]
    assert not errs, errs
    return [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(2)]


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def _rel_l2(a: dict, b: dict, base: dict = None):
    """||a - b|| / ||b - base|| over ALL tensors flattened together."""
    da = torch.cat([(a[n] - (base[n] if base else 0)).reshape(-1) for n in b])
    db = torch.cat([(b[n] - (base[n] if base else 0)).reshape(-1) for n in b])
    return float((da - db).norm() / db.norm().clamp_min(1e-30))


MIOPEN = ["--no-fused-bn", "--no-native-conv"]   # plain torch layers: the emulation's kernels


@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
def test_world_size_2_matches_ddp_semantics(cuda, tmp_path, amp):
    """3 steps (AMP: rank 1's step-2 batch carries an inf) against the one-process emulation of
    the reference's DDP, each step emulated from the state the native step started from; both
    run the same MIOpen kernels, so each step matches to rounding."""
    res = _spawn(tmp_path, MIOPEN, amp=amp, inf_step=INF_STEP if amp else -1, mode="emulate")
    for r in range(2):
        nat, ref = res[r]["native"], res[r]["ref"]
        assert nat["comm_ops"] > 0 and nat["buckets"] >= 2
        for step, (sn, em) in enumerate(zip(nat["snaps"], ref)):
            skipped = amp and step == INF_STEP
            before = {n: v.float() for n, v in sn["params"].items()}
            after = {n: v.float() for n, v in sn["after_params"].items()}
            bufs = {n: v.float() for n, v in sn["after_buffers"].items() if v.numel() > 1}
            ebufs = {n: v for n, v in em["buffers"].items() if v.numel() > 1}
            # the rank whose batch carries the inf ends that forward with non-finite running
            # statistics on both sides (rank 0's broadcast repairs them before the next forward)
            for n in bufs:
                assert torch.equal(bufs[n].isfinite(), ebufs[n].isfinite()), (n, step)
            b_err = _rel_l2({n: v.nan_to_num(0.0, 0.0, 0.0) for n, v in bufs.items()},
                            {n: v.nan_to_num(0.0, 0.0, 0.0) for n, v in ebufs.items()})
            tag = f"{'amp' if amp else 'fp32'} rank {r} step {step}"
            if skipped:
                # the inf on rank 1 skips the step on both ranks: parameters unchanged, scale backed off
                assert all(torch.equal(after[n], before[n]) for n in before), tag
                assert all(torch.equal(em["params"][n], before[n]) for n in before), tag
                d_err = g_err = 0.0
            else:
                d_err = _rel_l2(after, em["params"], before)
                g_err = _rel_l2(sn["grads"], em["grads"])
            print(f"{tag}: rel-L2 dparam {d_err:.2e} grad {g_err:.2e} buffers {b_err:.2e} "
                  f"scale {sn['after_scale']}/{em['scale']} tracker {sn['after_tracker']}/{em['tracker']}")
            worst = [] if skipped else sorted(((_rel(sn["grads"][n], g), n) for n, g in em["grads"].items()),
                                              reverse=True)[:4]
            # identical kernels on both sides: only the fused optimizer's rounding differs
            assert d_err < 1e-4 and g_err < 1e-4 and b_err < 1e-4, (tag, d_err, g_err, b_err, worst)
            assert sn["after_scale"] == em["scale"] and sn["after_tracker"] == em["tracker"], tag
            for n, b in em["buffers"].items():
                if b.numel() == 1:
                    assert torch.equal(sn["after_buffers"][n].float(), b), (tag, n)   # num_batches_tracked
        if amp:
            # the inf on rank 1 at step 2 skipped that step on both ranks: scale backed off once
            assert nat["scale"] == 32768.0 and nat["tracker"] == 1.0, (nat["scale"], nat["tracker"])
    for n in res[0]["native"]["params"]:
        assert torch.equal(res[0]["native"]["params"][n], res[1]["native"]["params"][n]), n


def _bf16(t):
    return t.to(torch.bfloat16).float()


# (variant, flags): the FULL native engine (MFMA convs, fused BN, weight shadows, steal mode)
LOCAL_CASES = [
    ("native_fp32_wire", []),
    # the asynchronous bridge: collectives enqueued on the comm stream (HIP host functions), the
    # autograd thread never blocks - same sums required
    ("native_fp32_wire_async", ["--comm", "host-async"]),
    ("native_bf16_wire", ["--grad-dtype", "bf16"]),
    ("miopen_bf16_wire", MIOPEN + ["--grad-dtype", "bf16"]),
]


GRAPH_STEPS = 6      # 3 eager warmup steps, the capture, then replays: the last step is a replay


@pytest.mark.parametrize("variant,extra", LOCAL_CASES, ids=[c[0] for c in LOCAL_CASES])
def test_world_size_2_reduces_local_gradients_exactly(cuda, tmp_path, variant, extra):
    """One step of the full native engine at world size 2 vs each rank's own local (world size
    1) step from the same weights: the reduced arena must be exactly the sum of the two local
    loss-scaled gradients (fp32 wire), or bf16(bf16(a) + bf16(b)) (bf16 wire: pack, bf16
    collective, unpack).  Exercises every line of the multi-rank data path on the hardware."""
    res = _spawn(tmp_path, extra, amp=True, steps=1, inf_step=-1, mode="local")
    a = res[0]["ref"]["raw_grads"]
    b = res[1]["ref"]["raw_grads"]
    bf16_wire = "--grad-dtype" in extra
    worst = 0.0
    for r in range(2):
        got = res[r]["native"]["raw_grads"]
        for n in a:
            want = _bf16(_bf16(a[n]) + _bf16(b[n])) if bf16_wire else a[n] + b[n]
            err = _rel(got[n], want)
            worst = max(worst, err)
            assert err < 1e-6, (variant, r, n, err)
    print(f"{variant}: worst per-tensor relative error vs local sum {worst:.2e}")
    for n in res[0]["native"]["params"]:
        assert torch.equal(res[0]["native"]["params"][n], res[1]["native"]["params"][n]), n


def test_world_size_2_graph_replay_reduces_local_gradients_exactly(cuda, tmp_path):
    """the captured step at world size 2 (``--cuda-graph`` over ``--comm
    host-async``: the bucket all-reduces and the rank-0 buffer broadcasts become graph host
    nodes, csrc/host_comm.cpp) must reduce to exactly the sum of the two ranks' local gradients
    on its REPLAYED steps.  lr = 0 keeps the parameters at rank 0's initial weights on every step,
    so the last (replayed) step's local world-size-1 gradients are a fixed function of that
    step's batches - the same for the replaying 2-rank job and each rank's eager local run."""
    res = _spawn(tmp_path, ["--comm", "host-async", "--cuda-graph", "--lr", "0"], amp=True,
                 steps=GRAPH_STEPS, inf_step=-1, mode="local", timeout=240)
    a = res[0]["ref"]["raw_grads"]
    b = res[1]["ref"]["raw_grads"]
    for r in range(2):
        nat = res[r]["native"]
        assert nat["replays"] == GRAPH_STEPS - 3, nat["replays"]   # the capture call replays too
        for n in a:
            err = _rel(nat["raw_grads"][n], a[n] + b[n])
            assert err < 1e-6, (r, n, err)
    for n in res[0]["native"]["params"]:
        assert torch.equal(res[0]["native"]["params"][n], res[1]["native"]["params"][n]), n


def test_world_size_2_native_engine_skips_inf_step_on_every_rank(cuda, tmp_path):
    """Full native engine, 3 steps, inf in rank 1's step-2 batch: the comm-stream check must
    flag it on BOTH ranks (the scale backs off once, parameters stay finite and identical)."""
    res = _spawn(tmp_path, [], amp=True, inf_step=INF_STEP, mode="none")
    for r in range(2):
        nat = res[r]["native"]
        assert nat["scale"] == 32768.0 and nat["tracker"] == 1.0, (nat["scale"], nat["tracker"])
        assert all(torch.isfinite(p).all() for p in nat["params"].values())
    for n in res[0]["native"]["params"]:
        assert torch.equal(res[0]["native"]["params"][n], res[1]["native"]["params"][n]), n
