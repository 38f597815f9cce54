"""Teacher-forced bf16 numerics of the headline configuration (VERDICT r4 next #3a).

ResNet-50 (1000 classes), channels_last, one training step per teacher-forced state S_k: the same
fp32 master weights, BatchNorm buffers and batch go into three engines

* ``ref``    - stock torch modules in fp32 (the reference's default precision,
               reference train_ddp.py:210-214): the numerical truth;
* ``stock``  - the same torch modules under ``torch.autocast(bfloat16)`` (stock PyTorch-ROCm's bf16 AMP);
* ``native`` - the framework's bf16 step (``Trainer`` ``--impl native --amp --amp-dtype bf16``:
               MFMA conv kernels, fused BatchNorm, weight shadows, device loss scaler, fused SGD).

Per step and per parameter group (stage x {conv, bn, fc}) it reports the relative L2 error of each
bf16 engine's gradient against ``ref``'s, and of the whole SGD update (momentum state zeroed in
every engine, so update = -lr (g + wd p)).  The run then continues from ``ref``'s updated state
(teacher forcing), so every step measures one step's numerics from a shared state.

    python bench/bf16_teacher.py --steps 5 --batch 64 --image-size 112
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def group_of(name: str) -> str:
    stage = name.split(".")[0]
    if stage == "fc":
        return "fc"
    kind = "bn" if (".bn" in "." + name or "downsample.1" in name) else "conv"
    return f"{stage}.{kind}"


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def grouped(named: dict) -> dict:
    out = {}
    for n, t in named.items():
        out.setdefault(group_of(n), []).append(t.reshape(-1).double())
    return {g: torch.cat(v) for g, v in out.items()}


def pretrain(model, steps: int, batch: int, image_size: int, lr: float, dev, log=print):
    """fp32 SGD on the learnable prototypes task (data/loader.py): at random init a ResNet-50's
    gradient is chaotic - ReLU-mask flips from ANY rounding difference cascade through 50 BN
    layers, so bf16 and fp32 gradients are nearly orthogonal in both engines (rel-L2 1.2-1.3,
    profiles/bf16_teacher_r5.md) and the comparison has no power.  A briefly trained network is
    out of that regime."""
    from distributed_pytorch_training_amd.data import SyntheticLoader
    if steps <= 0:
        return
    loader = SyntheticLoader(batch * steps, batch, image_size, 10, dev, channels_last=True, seed=7,
                             task="prototypes", noise=2.0)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    model.train()
    for i, (x, y) in enumerate(loader):
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        if (i + 1) % 50 == 0:
            log(json.dumps({"pretrain_step": i + 1, "loss": round(float(loss), 4)}))


def run(steps: int = 5, batch: int = 64, image_size: int = 112, seed: int = 0, lr: float = 0.1,
        wd: float = 5e-4, log=print, pretrain_steps: int = 0, pretrain_lr: float = 0.05,
        task: str = "random") -> dict:
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.graph import step_state
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    dev = torch.device("cuda:0")
    cl = torch.channels_last
    torch.manual_seed(seed)
    ref = build_model("resnet50", 1000, dev, image_size=image_size, channels_last=True).float()
    stock = build_model("resnet50", 1000, dev, image_size=image_size, channels_last=True).float()
    nat_model = build_model("resnet50", 1000, dev, image_size=image_size, channels_last=True)
    args = parse_args(["--model", "resnet50", "--dataset", "synthetic", "--batch-size", str(batch),
                       "--image-size", str(image_size), "--num-classes", "1000", "--amp", "--amp-dtype", "bf16",
                       "--channels-last", "--no-cuda-graph", "--lr", str(lr), "--momentum", "0.9",
                       "--weight-decay", str(wd)])
    tr = Trainer(nat_model, args, 0, 1, dev, log=lambda s: None)
    pnames = [n for n, _ in ref.named_parameters()]
    pretrain(ref, pretrain_steps, batch, image_size, pretrain_lr, dev, log)
    g = torch.Generator(device=dev).manual_seed(1000 + seed)
    protos = None
    if task == "prototypes":
        from distributed_pytorch_training_amd.data.loader import class_prototypes
        protos = class_prototypes(10, image_size, dev)
    rows = []
    for k in range(steps):
        state = {n: t.detach().clone() for n, t in ref.state_dict().items()}
        if protos is None:
            x = torch.randn(batch, 3, image_size, image_size, device=dev, generator=g).contiguous(memory_format=cl)
            y = torch.randint(0, 1000, (batch,), device=dev, generator=g)
        else:
            y = torch.randint(0, 10, (batch,), device=dev, generator=g)
            x = (protos.index_select(0, y) + 2.0 * torch.randn(batch, 3, image_size, image_size, device=dev,
                                                             generator=g)).contiguous(memory_format=cl)

        # fp32 reference and stock bf16 autocast: plain autograd gradients
        grads = {}
        for name, model, amp in (("ref", ref, False), ("stock", stock, True)):
            model.load_state_dict(state)
            model.train()
            model.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = F.cross_entropy(model(x), y)
            loss.backward()
            grads[name] = {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}

        # native: load S_k into the arena (params are views of it), zero the optimizer state
        tr.module.load_state_dict(state)
        tr.sync_weights()
        st = step_state(tr)
        with torch.no_grad():
            for key, t in st.items():
                if key.startswith("opt"):
                    t.zero_()
            tr.optimizer._step.zero_() if isinstance(tr.optimizer._step, torch.Tensor) else None
        if not isinstance(tr.optimizer._step, torch.Tensor):
            tr.optimizer._step = 0
        scale = float(tr.scaler.scale_tensor.item()) if tr.amp else 1.0
        p_before = {n: p.detach().clone() for n, p in tr.module.named_parameters()}
        tr.train_step(x, y)
        torch.cuda.synchronize()
        found_inf = float(tr.scaler.found_inf.item()) if tr.amp else 0.0
        pos = {id(p): i for i, p in enumerate(tr.ddp.arena.params)}
        ag = tr.ddp.averaged_grads()
        grads["native"] = {n: (ag[pos[id(p)]] / scale).float().clone() for n, p in tr.module.named_parameters()}
        upd_native = {n: (p.detach() - p_before[n]) for n, p in tr.module.named_parameters()}

        # reference update: fresh SGD (first step: buf = d), same hyper-parameters
        upd = {}
        for name in ("ref", "stock"):
            upd[name] = {n: -lr * (grads[name][n] + wd * state[n].float()) for n in pnames}
        upd["native"] = upd_native

        row = {"step": k, "scale": scale, "found_inf": found_inf, "grad": {}, "update": {}, "cos": {}}
        gref = grouped(grads["ref"])
        for eng in ("stock", "native"):
            ge = grouped(grads[eng])
            row["grad"][eng] = {gname: rel(ge[gname], gref[gname]) for gname in gref}
            row["grad"][eng]["all"] = rel(torch.cat([ge[n] for n in gref]), torch.cat([gref[n] for n in gref]))
            fa = torch.cat([ge[n] for n in gref])
            fr = torch.cat([gref[n] for n in gref])
            row["cos"][eng] = float((fa @ fr) / (fa.norm() * fr.norm()).clamp_min(1e-30))
            row["update"][eng] = rel(torch.cat([upd[eng][n].reshape(-1).double() for n in pnames]),
                                     torch.cat([upd["ref"][n].reshape(-1).double() for n in pnames]))
        rows.append(row)
        log(json.dumps(row))

        # teacher forcing: advance the reference state with its own fp32 update
        with torch.no_grad():
            for n, p in ref.named_parameters():
                p.copy_(state[n] + upd["ref"][n])
    tr.close()
    return summarize(rows)


def summarize(rows) -> dict:
    groups = list(rows[0]["grad"]["stock"].keys())
    mean = lambda eng, gname: sum(r["grad"][eng][gname] for r in rows) / len(rows)
    table = {gname: {"stock": mean("stock", gname), "native": mean("native", gname)} for gname in groups}
    for gname in table:
        table[gname]["ratio"] = table[gname]["native"] / max(table[gname]["stock"], 1e-30)
    upd = {eng: sum(r["update"][eng] for r in rows) / len(rows) for eng in ("stock", "native")}
    cos = {eng: sum(r["cos"][eng] for r in rows) / len(rows) for eng in ("stock", "native")}
    return {"steps": len(rows), "groups": table, "update": upd, "cos": cos, "rows": rows}


def markdown(res: dict) -> str:
    lines = ["| parameter group | stock bf16 rel-L2 vs fp32 | native bf16 rel-L2 vs fp32 | native / stock |",
             "|---|---|---|---|"]
    for gname, v in res["groups"].items():
        lines.append(f"| {gname} | {v['stock']:.4g} | {v['native']:.4g} | {v['ratio']:.3f} |")
    u = res["update"]
    lines.append(f"| **SGD update** | {u['stock']:.4g} | {u['native']:.4g} | {u['native'] / max(u['stock'], 1e-30):.3f} |")
    c = res.get("cos")
    if c:
        lines.append(f"| gradient cosine vs fp32 | {c['stock']:.4f} | {c['native']:.4f} | |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--image-size", type=int, default=112)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pretrain-steps", type=int, default=0)
    ap.add_argument("--task", default="random", choices=["random", "prototypes"])
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env
    setup_miopen_env()
    torch.cuda.set_device(0)
    res = run(a.steps, a.batch, a.image_size, a.seed, pretrain_steps=a.pretrain_steps, task=a.task)
    print(markdown(res))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
