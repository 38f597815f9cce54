"""NativeDDP (C++ reducer) vs torch DDP, world_size 2 on gloo/CPU (BASELINE config 1 plumbing)."""
import copy
import os
import socket
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, case, out_dir):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                          LOCAL_RANK=str(rank))
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        torch.manual_seed(1234 + rank)           # ranks start DIFFERENT: DDP must broadcast rank 0
        res = CASES[case](rank, ws)
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
            f.write(traceback.format_exc())
        raise


def _run(case, tmp_path, ws=2):
    port = _free_port()
    mp.start_processes(_worker, args=(ws, port, case, str(tmp_path)), nprocs=ws, start_method="spawn")
    errs = [p.read_text() for p in tmp_path.glob("err*.txt")]
    assert not errs, errs
    return [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(ws)]


def _model():
    from distributed_pytorch_training_amd.models import build_model
    return build_model("resnet18", 10)


def _data(rank, step, n=8):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def case_parity(rank, ws, grad_dtype="fp32", rebuild=True, cap=1.0):
    from distributed_pytorch_training_amd.optim import FusedSGD
    from distributed_pytorch_training_amd.parallel.ddp import NativeDDP

    base = _model()
    ref = torch.nn.parallel.DistributedDataParallel(copy.deepcopy(base))
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    mod = copy.deepcopy(base)
    order = list(mod.parameters())
    nat = NativeDDP(mod, rank=rank, world_size=ws, bucket_cap_mb=cap, first_bucket_mb=0.25,
                    grad_dtype=grad_dtype, rebuild_buckets=rebuild)
    opt = FusedSGD(nat.arena, lr=0.1, momentum=0.9, weight_decay=5e-4, params_in_order=order)
    crit = torch.nn.CrossEntropyLoss()
    grads = []
    for step in range(3):
        x, y = _data(rank, step)
        ref_opt.zero_grad(set_to_none=True)
        crit(ref(x), y).backward()
        crit(nat(x), y).backward()
        ref_grads = [p.grad.clone() for p in ref.module.parameters()]
        pos = {id(p): i for i, p in enumerate(nat.arena.params)}
        ours = nat.averaged_grads()
        nat_grads = [ours[pos[id(p)]].clone() for p in order]
        grads.append(max(float((a - b).abs().max()) for a, b in zip(ref_grads, nat_grads)))
        ref_opt.step()
        nat.maybe_rebuild_buckets(opt)
        opt.step(None, host_factor=nat.grad_factor)
    params = max(float((p - q).abs().max()) for p, q in zip(ref.module.parameters(), order))
    bufs = max(float((a.float() - b.float()).abs().max()) for a, b in zip(ref.module.buffers(), mod.buffers()))
    flat = torch.cat([p.detach().reshape(-1) for p in order])
    return {"grad_err": grads, "param_err": params, "buf_err": bufs, "flat": flat,
            "buckets": nat.plan.num_buckets, "rebuilt": nat._rebuilt}


def case_bf16(rank, ws):
    return case_parity(rank, ws, grad_dtype="bf16")


def case_norebuild(rank, ws):
    return case_parity(rank, ws, rebuild=False, cap=25.0)


def case_no_sync(rank, ws):
    """Gradient accumulation: no_sync micro-batch + synced micro-batch == torch DDP no_sync."""
    from distributed_pytorch_training_amd.parallel.ddp import NativeDDP

    base = _model()
    ref = torch.nn.parallel.DistributedDataParallel(copy.deepcopy(base))
    mod = copy.deepcopy(base)
    nat = NativeDDP(mod, rank=rank, world_size=ws)
    crit = torch.nn.CrossEntropyLoss()
    x1, y1 = _data(rank, 7)
    x2, y2 = _data(rank, 8)
    with ref.no_sync():
        crit(ref(x1), y1).backward()
    crit(ref(x2), y2).backward()
    with nat.no_sync():
        crit(nat(x1), y1).backward()
    crit(nat(x2), y2).backward()
    pos = {id(p): i for i, p in enumerate(nat.arena.params)}
    ours = nat.averaged_grads()
    err = max(float((p.grad - ours[pos[id(q)]]).abs().max())
              for p, q in zip(ref.module.parameters(), mod.parameters()))
    return {"err": err}


def case_amp_inf(rank, ws):
    """A non-finite gradient on ONE rank must make EVERY rank skip the step (global found_inf)."""
    from distributed_pytorch_training_amd.amp import DeviceGradScaler
    from distributed_pytorch_training_amd.optim import FusedSGD
    from distributed_pytorch_training_amd.parallel.ddp import NativeDDP

    mod = _model()
    scaler = DeviceGradScaler("cpu", init_scale=1024.0)
    nat = NativeDDP(mod, rank=rank, world_size=ws, found_inf=scaler.found_inf, scale=scaler.scale_tensor,
                    check_inf=True)
    opt = FusedSGD(nat.arena, lr=0.1, momentum=0.9)
    x, y = _data(rank, 3)
    if rank == 1:
        x[0, 0, 0, 0] = float("inf")
    before = nat.arena.param_flat.clone()
    loss = torch.nn.functional.cross_entropy(nat(x), y)
    scaler.scale(loss).backward()
    found = float(scaler.found_inf)
    opt.step(scaler, host_factor=nat.grad_factor, grads_checked=nat.grads_checked)
    return {"found": found, "unchanged": bool(torch.equal(before, nat.arena.param_flat)),
            "scale": scaler.get_scale()}


CASES = {"parity": case_parity, "bf16": case_bf16, "norebuild": case_norebuild, "no_sync": case_no_sync,
         "amp_inf": case_amp_inf}


@pytest.mark.parametrize("case", ["parity", "norebuild"])
def test_native_ddp_matches_torch_ddp(case, tmp_path):
    r0, r1 = _run(case, tmp_path)
    for r in (r0, r1):
        assert max(r["grad_err"]) < 1e-5, r["grad_err"]
        assert r["param_err"] < 1e-5
        assert r["buf_err"] < 1e-5      # BN running stats follow rank 0 (broadcast_buffers)
    assert torch.equal(r0["flat"], r1["flat"])  # replicas bit-identical
    if case == "parity":
        assert r0["rebuilt"] and r0["buckets"] > 3


def test_bf16_wire_close_to_fp32(tmp_path):
    r0, r1 = _run("bf16", tmp_path)
    assert r0["grad_err"][0] < 2e-2, r0["grad_err"]
    assert torch.equal(r0["flat"], r1["flat"])


def test_no_sync_accumulation(tmp_path):
    for r in _run("no_sync", tmp_path):
        assert r["err"] < 1e-5


def test_global_found_inf_skips_every_rank(tmp_path):
    for r in _run("amp_inf", tmp_path):
        assert r["found"] == 1.0 and r["unchanged"] and r["scale"] == 512.0
