"""Weight-gradient GEMM (dW = dY^T X, K = tokens) on MI355X: plain mm vs split-K batched GEMM
with fp32 partial outputs, for the ViT-B/16 shapes (T = 128*197)."""
import json
import sys

import torch


def t_ms(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = torch.device("cuda:0")
    T = 128 * 197
    out = []
    for n_out, n_in in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, n_in, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * T * n_out * n_in
        ref = dy.t() @ x
        row = {"shape": [n_out, n_in, T], "mm_ms": t_ms(lambda: dy.t() @ x)}
        try:
            row["mm_f32out_ms"] = t_ms(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception as e:  # noqa: BLE001
            row["mm_f32out_err"] = str(e)[:120]
        for S in (2, 4, 8, 16):
            if T % S:
                continue
            a = dy.view(S, T // S, n_out).transpose(1, 2)
            b = x.view(S, T // S, n_in)
            try:
                f = lambda: torch.bmm(a, b, out_dtype=torch.float32).sum(0)
                row[f"splitk{S}_f32_ms"] = t_ms(f)
                err = (f().to(torch.bfloat16).float() - ref.float()).abs().max().item()
                row[f"splitk{S}_maxerr_vs_mm"] = err
            except Exception as e:  # noqa: BLE001
                row[f"splitk{S}_err"] = str(e)[:120]
            row[f"splitk{S}_bf16_ms"] = t_ms(lambda: torch.bmm(a, b).float().sum(0))
        row["mm_tflops"] = flops / row["mm_ms"] / 1e9
        out.append(row)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
