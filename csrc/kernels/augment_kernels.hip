// On-device CIFAR augmentation (gfx950).
//
// Replaces the reference's CPU pipeline (DataLoader workers running torchvision
// RandomCrop(32, padding=4) -> RandomHorizontalFlip -> ToTensor -> Normalize, reference
// train_ddp.py:91-101) with one gather kernel over a uint8 dataset that
// stays resident in HBM (CIFAR-10 train = 150 MiB, nothing next to 288 GB):
//   out[b, c, y, x] = (img[idx[b], c, y+dy-pad, xs] / 255 - mean[c]) / std[c]
//   xs = flip[b] ? (W-1-x)+dx-pad : x+dx-pad;  out-of-range source pixels are the zero pad
// (torchvision pads uint8 zeros *before* ToTensor/Normalize, so a pad pixel normalises to
// -mean/std, reproduced exactly).  Evaluation uses dy = dx = pad, flip = 0.
// One thread per output pixel handles all channels; the output is fp32 or bf16, NCHW or
// NHWC (channels_last feeds MIOpen's NHWC kernels with no layout transform).
#include "common.h"
#include "kernels.h"

namespace dpt {

template <bool BF16, bool NHWC>
__global__ __launch_bounds__(kBlock) void augment_kernel(const uint8_t* __restrict__ data,
                                                         const int64_t* __restrict__ idx,
                                                         const int32_t* __restrict__ offs,
                                                         const uint8_t* __restrict__ flips, void* out,
                                                         int64_t B, int C, int H, int W, int pad,
                                                         AugNorm norm) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t total = B * H * W;
  if (t >= total) return;
  const int x = (int)(t % W);
  const int y = (int)((t / W) % H);
  const int64_t b = t / ((int64_t)H * W);
  const int dy = offs ? offs[2 * b] : pad;
  const int dx = offs ? offs[2 * b + 1] : pad;
  const bool fl = flips ? flips[b] != 0 : false;
  const int sy = y + dy - pad;
  const int sx = (fl ? (W - 1 - x) : x) + dx - pad;
  const bool inside = sy >= 0 && sy < H && sx >= 0 && sx < W;
  const uint8_t* img = data + idx[b] * (int64_t)C * H * W;
  for (int c = 0; c < C; ++c) {
    float v = inside ? (float)img[((int64_t)c * H + sy) * W + sx] : 0.0f;
    v = (v * (1.0f / 255.0f) - norm.mean[c]) * norm.inv_std[c];
    int64_t o = NHWC ? ((b * H + y) * W + x) * C + c : ((b * C + c) * H + y) * W + x;
    if (BF16) static_cast<uint16_t*>(out)[o] = f32_to_bf16(v);
    else static_cast<float*>(out)[o] = v;
  }
}

void launch_augment(const uint8_t* data, const int64_t* idx, const int32_t* offs,
                    const uint8_t* flips, void* out, bool out_bf16, bool nhwc, int64_t B, int C,
                    int H, int W, int pad, AugNorm norm, hipStream_t s) {
  int64_t total = B * H * W;
  if (total == 0) return;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock)), block(kBlock);
  if (out_bf16) {
    if (nhwc) hipLaunchKernelGGL((augment_kernel<true, true>), grid, block, 0, s, data, idx, offs, flips, out, B, C, H, W, pad, norm);
    else hipLaunchKernelGGL((augment_kernel<true, false>), grid, block, 0, s, data, idx, offs, flips, out, B, C, H, W, pad, norm);
  } else {
    if (nhwc) hipLaunchKernelGGL((augment_kernel<false, true>), grid, block, 0, s, data, idx, offs, flips, out, B, C, H, W, pad, norm);
    else hipLaunchKernelGGL((augment_kernel<false, false>), grid, block, 0, s, data, idx, offs, flips, out, B, C, H, W, pad, norm);
  }
}

}  // namespace dpt
