import torch, sys
sys.path.insert(0, ".")
from distributed_pytorch_training_amd import ops
C = ops.native()
for dt in (torch.float32, torch.bfloat16):
    x = torch.arange(1*8*4*4, dtype=torch.float32, device="cuda").reshape(1, 8, 4, 4).to(dt).contiguous(memory_format=torch.channels_last)
    y, idx = C.maxpool_fwd(x, 3, 2, 1)
    torch.cuda.synchronize()
    ref = torch.nn.functional.max_pool2d(x, 3, 2, 1)
    print(dt, "ours", y[0, 0].tolist(), "ref", ref[0, 0].tolist(), "idx", idx[0, 0].tolist(), flush=True)
    print("equal", torch.equal(y, ref), flush=True)
