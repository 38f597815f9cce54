// Channels-last max-pool with window-local argmax (gfx950).
//
// ResNet's stem pool (3x3, stride 2, pad 1 on a [B,112,112,64] bf16 activation) runs in
// ATen as max_pool_forward_nhwc + max_pool_backward_nhwc; the backward alone took 0.62 ms
// of a 33 ms ResNet-50 step on MI355X (profiles/).  Here:
//   forward : one thread per (output pixel, 8-channel group): 9 x 16-byte window loads,
//             max + argmax per channel (NaN wins, first max wins ties, like ATen), 16-byte
//             store of the result and an 8-byte store of the eight window-local argmaxes
//             (uint8 0..K*K-1 instead of ATen's int64 flat indices: 8x less index traffic);
//   backward: gather, no atomics - one thread per (input pixel, 8-channel group) visits the
//             <= ceil(K/S)^2 windows covering it and sums the gradients of those whose argmax
//             points at it; every input gradient element is written exactly once.
// Note: an earlier forward with a loop-carried "first in-bounds element" flag returned the
// first window element instead of the max for the fp32 instantiation on gfx950 (bf16 was
// right); the analytic clipped window seeded with -inf below is what tests/test_bn_gpu.py
// verifies for every dtype.
#include "common.h"
#include "kernels.h"

namespace dpt {

__device__ __forceinline__ void pool_load8(int dtype, const void* p, int64_t i, float f[8]) {
  if (dtype == 0) {
    const float4* q = reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    float4 a = q[0], b = q[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    return;
  }
  uint4 w = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
  uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = dtype == 1 ? bf16_to_f32(u[k] & 0xffff) : f16_to_f32(u[k] & 0xffff);
    f[2 * k + 1] = dtype == 1 ? bf16_to_f32(u[k] >> 16) : f16_to_f32(u[k] >> 16);
  }
}

__device__ __forceinline__ uint16_t pool_to16(int dtype, float v) {
  return dtype == 1 ? f32_to_bf16(v) : __builtin_bit_cast(uint16_t, (_Float16)v);
}

__device__ __forceinline__ void pool_store8(int dtype, void* p, int64_t i, const float f[8]) {
  if (dtype == 0) {
    float4* q = reinterpret_cast<float4*>(static_cast<float*>(p) + i);
    q[0] = make_float4(f[0], f[1], f[2], f[3]);
    q[1] = make_float4(f[4], f[5], f[6], f[7]);
    return;
  }
  uint4 w;
  w.x = (uint32_t)pool_to16(dtype, f[0]) | ((uint32_t)pool_to16(dtype, f[1]) << 16);
  w.y = (uint32_t)pool_to16(dtype, f[2]) | ((uint32_t)pool_to16(dtype, f[3]) << 16);
  w.z = (uint32_t)pool_to16(dtype, f[4]) | ((uint32_t)pool_to16(dtype, f[5]) << 16);
  w.w = (uint32_t)pool_to16(dtype, f[6]) | ((uint32_t)pool_to16(dtype, f[7]) << 16);
  *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) = w;
}

template <int DT>
__global__ __launch_bounds__(kBlock) void maxpool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int64_t B, int H, int W,
                                                             int C, int Ho, int Wo, int K, int S, int P) {
  const int cg8 = C >> 3;
  const int64_t total = B * Ho * Wo * cg8;
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % cg8);
  int64_t pix = t / cg8;
  const int ox = (int)(pix % Wo);
  pix /= Wo;
  const int oy = (int)(pix % Ho);
  const int64_t b = pix / Ho;
  // Window clipped to the image; the first in-bounds position seeds the argmax (ATen keeps
  // it when every value is -inf), the running max starts at -inf.
  const int ky0 = max(0, P - oy * S), ky1 = min(K, H + P - oy * S);
  const int kx0 = max(0, P - ox * S), kx1 = min(K, W + P - ox * S);
  float best[8];
  int arg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { best[k] = -__builtin_inff(); arg[k] = ky0 * K + kx0; }
  for (int ky = ky0; ky < ky1; ++ky) {
    const int iy = oy * S - P + ky;
    for (int kx = kx0; kx < kx1; ++kx) {
      const int ix = ox * S - P + kx;
      float v[8];
      pool_load8(DT, x, ((b * H + iy) * W + ix) * C + cg * 8, v);
      const int pos = ky * K + kx;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        // strictly greater (first max wins), and a NaN wins unless one is already held
        const bool take = (v[k] > best[k]) || (v[k] != v[k] && best[k] == best[k]);
        best[k] = take ? v[k] : best[k];
        arg[k] = take ? pos : arg[k];
      }
    }
  }
  const int64_t o = ((b * Ho + oy) * Wo + ox) * C + cg * 8;
  pool_store8(DT, y, o, best);
  uint2 packed;
  packed.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
  packed.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + o) = packed;
}

template <int DT>
__global__ __launch_bounds__(kBlock) void maxpool_bwd_kernel(const void* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx,
                                                             void* __restrict__ dx, int64_t B, int H, int W,
                                                             int C, int Ho, int Wo, int K, int S, int P) {
  const int cg8 = C >> 3;
  const int64_t total = B * H * W * cg8;
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % cg8);
  int64_t pix = t / cg8;
  const int ix = (int)(pix % W);
  pix /= W;
  const int iy = (int)(pix % H);
  const int64_t b = pix / H;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // windows oy with oy*S - P <= iy <= oy*S - P + K - 1
  const int oy0 = max(0, (iy + P - K + S) / S), oy1 = min(Ho - 1, (iy + P) / S);
  const int ox0 = max(0, (ix + P - K + S) / S), ox1 = min(Wo - 1, (ix + P) / S);
  for (int oy = oy0; oy <= oy1; ++oy) {
    const int ky = iy - (oy * S - P);
    if (ky < 0 || ky >= K) continue;
    for (int ox = ox0; ox <= ox1; ++ox) {
      const int kx = ix - (ox * S - P);
      if (kx < 0 || kx >= K) continue;
      const uint8_t pos = (uint8_t)(ky * K + kx);
      const int64_t o = ((b * Ho + oy) * Wo + ox) * C + cg * 8;
      const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
      float g[8];
      pool_load8(DT, dy, o, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint8_t a = (uint8_t)(((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xff);
        if (a == pos) acc[k] += g[k];
      }
    }
  }
  pool_store8(DT, dx, ((b * H + iy) * W + ix) * C + cg * 8, acc);
}

void launch_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* idx, int64_t B, int H, int W, int C, int Ho,
                        int Wo, int K, int S, int P, hipStream_t s) {
  const int64_t total = B * Ho * Wo * (C / 8);
  if (total == 0) return;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock)), block(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(maxpool_fwd_kernel<0>, grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
    case 1: hipLaunchKernelGGL(maxpool_fwd_kernel<1>, grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
    default: hipLaunchKernelGGL(maxpool_fwd_kernel<2>, grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
  }
}

void launch_maxpool_bwd(int dtype, const void* dy, const uint8_t* idx, void* dx, int64_t B, int H, int W, int C,
                        int Ho, int Wo, int K, int S, int P, hipStream_t s) {
  const int64_t total = B * H * W * (C / 8);
  if (total == 0) return;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock)), block(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(maxpool_bwd_kernel<0>, grid, block, 0, s, dy, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
    case 1: hipLaunchKernelGGL(maxpool_bwd_kernel<1>, grid, block, 0, s, dy, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
    default: hipLaunchKernelGGL(maxpool_bwd_kernel<2>, grid, block, 0, s, dy, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
  }
}

}  // namespace dpt
