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
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

typedef float pf32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 pbf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 pf16x2 __attribute__((ext_vector_type(2)));


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

// Index math: the pixel decomposition is done in 32 bits (IDX = uint32_t) whenever the
// element count fits - 64-bit integer division is a ~100-instruction software sequence on
// CDNA and made both kernels ALU-bound (ResNet-50 stem at batch 256: 25.7M threads).
template <int DT, typename IDX>
__global__ __launch_bounds__(kBlock) void maxpool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int64_t B, int H, int W,
                                                             int C, int Ho, int Wo, int K, int S, int P) {
  const IDX cg8 = (IDX)(C >> 3);
  const IDX total = (IDX)(B * Ho * Wo * cg8);
  const IDX t = (IDX)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % cg8);
  IDX pix = t / cg8;
  const int ox = (int)(pix % (IDX)Wo);
  pix /= (IDX)Wo;
  const int oy = (int)(pix % (IDX)Ho);
  const int64_t b = (int64_t)(pix / (IDX)Ho);
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
        const bool take = !(v[k] <= best[k]) && (best[k] == best[k]);
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

// dy2 (optional): a second output gradient summed in while gathering - the pool output fed
// two consumers (ResNet's stem pool: layer1's conv path and its downsample), see ops/pool.py.
template <int DT, typename IDX>
__global__ __launch_bounds__(kBlock) void maxpool_bwd_kernel(const void* __restrict__ dy,
                                                             const void* __restrict__ dy2,
                                                             const uint8_t* __restrict__ idx,
                                                             void* __restrict__ dx, int64_t B, int H, int W,
                                                             int C, int Ho, int Wo, int K, int S, int P) {
  const IDX cg8 = (IDX)(C >> 3);
  const IDX total = (IDX)(B * H * W * cg8);
  const IDX t = (IDX)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const int cg = (int)(t % cg8);
  IDX pix = t / cg8;
  const int ix = (int)(pix % (IDX)W);
  pix /= (IDX)W;
  const int iy = (int)(pix % (IDX)H);
  const int64_t b = (int64_t)(pix / (IDX)H);
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
      float g[8], g2[8];
      pool_load8(DT, dy, o, g);
      if (dy2 != nullptr) {
        pool_load8(DT, dy2, o, g2);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] += g2[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint8_t a = (uint8_t)(((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xff);
        if (a == pos) acc[k] += g[k];
      }
    }
  }
  pool_store8(DT, dx, ((b * H + iy) * W + ix) * C + cg * 8, acc);
}

// 3x3 forward with the window fully unrolled: all nine 16-byte loads are issued before the
// max scan (the general kernel's runtime-bounded loop waits for each load in turn).  Out-of-
// image taps load a clamped in-bounds address and are skipped by the scan, which visits the
// taps in the same (ky, kx) order - identical max / argmax / NaN semantics.
// AFF: the pool input is relu(x*a + b) of a BatchNorm whose apply pass is folded in here (the
// ResNet stem): every loaded element goes through the apply's exact arithmetic and rounding
// (fma, NaN-propagating ReLU, round to the storage type) before the max, so values, argmax
// and tie-breaking equal pooling the materialised BN output - which is never written.
template <int DT, bool AFF = false>
__global__ __launch_bounds__(kBlock) void maxpool3_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                              uint8_t* __restrict__ idx, int H, int W, int C, int Ho,
                                                              int Wo, int S, int P, uint32_t total,
                                                              const float* __restrict__ coef = nullptr) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const uint32_t cg8 = (uint32_t)C >> 3;
  const int cg = (int)(t % cg8);
  uint32_t pix = t / cg8;
  const int ox = (int)(pix % (uint32_t)Wo);
  pix /= (uint32_t)Wo;
  const int oy = (int)(pix % (uint32_t)Ho);
  const int64_t b = (int64_t)(pix / (uint32_t)Ho);
  const int ky0 = max(0, P - oy * S), ky1 = min(3, H + P - oy * S);
  const int kx0 = max(0, P - ox * S), kx1 = min(3, W + P - ox * S);
  float v[9][8];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = min(max(oy * S - P + ky, 0), H - 1);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = min(max(ox * S - P + kx, 0), W - 1);
      pool_load8(DT, x, ((b * H + iy) * W + ix) * C + cg * 8, v[ky * 3 + kx]);
    }
  }
  if (AFF) {
    float ca[8], cb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { ca[k] = coef[cg * 8 + k]; cb[k] = coef[C + cg * 8 + k]; }
#pragma unroll
    for (int q = 0; q < 9; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float o = __builtin_fmaf(v[q][k], ca[k], cb[k]);
        o = o < 0.0f ? 0.0f : o;
        if (DT == 1) o = bf16_to_f32(f32_to_bf16(o));
        else if (DT == 2) o = f16_to_f32(pool_to16(2, o));
        v[q][k] = o;
      }
  }
  float best[8];
  int arg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { best[k] = -__builtin_inff(); arg[k] = ky0 * 3 + kx0; }
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const bool in = ky >= ky0 && ky < ky1 && kx >= kx0 && kx < kx1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float vv = v[ky * 3 + kx][k];
        const bool take = in && !(vv <= best[k]) && (best[k] == best[k]);  // > or NaN-over-number
        best[k] = take ? vv : best[k];
        arg[k] = take ? ky * 3 + kx : arg[k];
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

// 3x3 / stride 2 / pad 1 forward (the ResNet stem): one thread per 2x2 OUTPUT block x 8
// channels.  The four windows of output rows {2a, 2a+1} x cols {2b, 2b+1} cover input rows
// 4a-1..4a+3 and cols 4b-1..4b+3: 25 loads (and, with AFF, 25 BN+ReLU transforms) serve four
// outputs instead of 36.  Rows are streamed top to bottom and each tap updates the windows
// that contain it in window-local (ky, kx) order, so max / argmax / tie / NaN semantics are
// the per-output kernel's exactly.  AFF rounding uses the hardware round-to-nearest-even
// converts (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32) - the same values as f32_to_bf16.
template <int DT, bool AFF>
__global__ __launch_bounds__(kBlock) void maxpool3s2_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                                uint8_t* __restrict__ idx, int H, int W, int C, int Ho,
                                                                int Wo, uint32_t total,
                                                                const float* __restrict__ coef) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const uint32_t cg8 = (uint32_t)C >> 3;
  const int cg = (int)(t % cg8);
  uint32_t pix = t / cg8;
  const uint32_t Wo2 = ((uint32_t)Wo + 1) >> 1, Ho2 = ((uint32_t)Ho + 1) >> 1;
  const int bx = (int)(pix % Wo2);
  pix /= Wo2;
  const int by = (int)(pix % Ho2);
  const int64_t b = (int64_t)(pix / Ho2);
  const int y0 = 4 * by - 1, x0 = 4 * bx - 1;
  float ca[8], cb[8];
  if (AFF) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { ca[k] = coef[cg * 8 + k]; cb[k] = coef[C + cg * 8 + k]; }
  }
  float best[4][8];
  int arg[4][8];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    // first in-image tap of window w (the scan's argmax seed, as in the per-output kernel)
    const int wy = y0 + 2 * (w >> 1), wx = x0 + 2 * (w & 1);
    const int a0 = (wy < 0 ? 1 : 0) * 3 + (wx < 0 ? 1 : 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[w][k] = -__builtin_inff(); arg[w][k] = a0; }
  }
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const int iy = y0 + r;
    const bool yin = iy >= 0 && iy < H;
    const int cy = min(max(iy, 0), H - 1);
    float v[5][8];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const int cx = min(max(x0 + c, 0), W - 1);
      pool_load8(DT, x, ((b * H + cy) * W + cx) * C + cg * 8, v[c]);
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      if (AFF) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          pf32x2 o;
          o[0] = __builtin_fmaf(v[c][k], ca[k], cb[k]);
          o[1] = __builtin_fmaf(v[c][k + 1], ca[k + 1], cb[k + 1]);
          o[0] = o[0] < 0.0f ? 0.0f : o[0];
          o[1] = o[1] < 0.0f ? 0.0f : o[1];
          if (DT == 1) {
            const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(o, pbf16x2));
            o[0] = __uint_as_float(u << 16);
            o[1] = __uint_as_float(u & 0xffff0000u);
          } else if (DT == 2) {
            const pf16x2 h = __builtin_convertvector(o, pf16x2);
            o[0] = (float)h[0];
            o[1] = (float)h[1];
          }
          v[c][k] = o[0];
          v[c][k + 1] = o[1];
        }
      }
      const int ix = x0 + c;
      const bool in = yin && ix >= 0 && ix < W;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int ky = r - 2 * (w >> 1), kx = c - 2 * (w & 1);
        if (ky < 0 || ky > 2 || kx < 0 || kx > 2) continue;  // resolved at compile time
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // vv > best, or vv NaN while best is not: !(vv <= best) && best == best (2 compares)
          const float vv = v[c][k];
          const bool take = in && !(vv <= best[w][k]) && (best[w][k] == best[w][k]);
          best[w][k] = take ? vv : best[w][k];
          arg[w][k] = take ? ky * 3 + kx : arg[w][k];
        }
      }
    }
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int oy = 2 * by + (w >> 1), ox = 2 * bx + (w & 1);
    if (oy >= Ho || ox >= Wo) continue;
    const int64_t o = ((b * Ho + oy) * Wo + ox) * C + cg * 8;
    pool_store8(DT, y, o, best[w]);
    uint2 packed;
    packed.x = (uint32_t)arg[w][0] | ((uint32_t)arg[w][1] << 8) | ((uint32_t)arg[w][2] << 16) | ((uint32_t)arg[w][3] << 24);
    packed.y = (uint32_t)arg[w][4] | ((uint32_t)arg[w][5] << 8) | ((uint32_t)arg[w][6] << 16) | ((uint32_t)arg[w][7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = packed;
  }
}

// 3x3 / stride 2 / pad 1 (ResNet stem) backward: one thread per 2x2 input block (rows 2a,
// 2a+1, cols 2b, 2b+1) x 8 channels.  Window oy covers rows 2oy-1..2oy+1, so the block's four
// pixels are covered exactly by windows {a, a+1} x {b, b+1}: each is read once per block (vs
// 2.25 window reads per pixel, data-dependent trip counts and branches in the general gather)
// and the window-local argmax decides which pixel receives its gradient.
// BNS: the pool input was relu(bn(x)) (ResNet's stem BatchNorm+ReLU): also sum that BN's
// backward statistics s1 = sum dz, s2 = sum dz*(x - mean), dz = dx * (fma(x, a, b) > 0), per
// block into [C][gridDim.x] partials (C = 8 * groups, kBlock % (C / 8) == 0) - the BN backward
// then skips its statistics pass over the two largest tensors of the network.
template <int DT, bool BNS = false>
__global__ __launch_bounds__(kBlock) void maxpool3s2_bwd_kernel(const void* __restrict__ dy,
                                                                const void* __restrict__ dy2,
                                                                const uint8_t* __restrict__ idx,
                                                                void* __restrict__ dx, int H, int W, int C, int Ho,
                                                                int Wo, int Ha, int Wa, uint32_t total,
                                                                const void* __restrict__ bnx = nullptr,
                                                                const float* __restrict__ bn_mean = nullptr,
                                                                const float* __restrict__ bn_coef = nullptr,
                                                                float* __restrict__ bp1 = nullptr,
                                                                float* __restrict__ bp2 = nullptr) {
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  // grid-stride (BNS launches at most kPoolBnBlocks blocks: one partial per block and channel;
  // the stride is a multiple of kBlock, so a lane's channel group never changes)
  for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < total; t += gridDim.x * kBlock) {
  const uint32_t cg8 = (uint32_t)C >> 3;
  const int cg = (int)(t % cg8);
  uint32_t q = t / cg8;
  const int b = (int)(q % (uint32_t)Wa);
  q /= (uint32_t)Wa;
  const int a = (int)(q % (uint32_t)Ha);
  const int64_t n = (int64_t)(q / (uint32_t)Ha);
  float acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[i][k] = 0.f;
#pragma unroll
  for (int dyw = 0; dyw < 2; ++dyw) {
#pragma unroll
    for (int dxw = 0; dxw < 2; ++dxw) {
      const int oy = a + dyw, ox = b + dxw;
      if (oy >= Ho || ox >= Wo) continue;
      const int64_t o = ((n * Ho + oy) * Wo + ox) * C + cg * 8;
      const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
      float g[8];
      pool_load8(DT, dy, o, g);
      if (dy2 != nullptr) {
        float g2[8];
        pool_load8(DT, dy2, o, g2);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] += g2[k];
      }
      // pixel (2a + py, 2b + px) sits at window position ((py + 1 - 2*dyw) * 3 + (px + 1 - 2*dxw))
#pragma unroll
      for (int py = 0; py < 2; ++py) {
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const int ky = py + 1 - 2 * dyw, kx = px + 1 - 2 * dxw;
          if (ky < 0 || kx < 0) continue;  // compile-time after unrolling
          const uint32_t pos = (uint32_t)(ky * 3 + kx);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t am = ((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xffu;
            acc[py * 2 + px][k] += am == pos ? g[k] : 0.f;
          }
        }
      }
    }
  }
  float bm[8], ba[8], bb[8], xq[4][8];
  if (BNS) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bm[k] = bn_mean[cg * 8 + k];
      ba[k] = bn_coef[cg * 8 + k];
      bb[k] = bn_coef[C + cg * 8 + k];
    }
    // BN inputs of the block's four pixels, loaded before any store (the compiler cannot move
    // loads above stores it cannot prove disjoint)
#pragma unroll
    for (int py = 0; py < 2; ++py)
#pragma unroll
      for (int px = 0; px < 2; ++px) {
        const int iy = min(2 * a + py, H - 1), ix = min(2 * b + px, W - 1);
        pool_load8(DT, bnx, ((n * H + iy) * W + ix) * C + cg * 8, xq[py * 2 + px]);
      }
  }
#pragma unroll
  for (int py = 0; py < 2; ++py) {
    const int iy = 2 * a + py;
    if (iy >= H) continue;
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      const int ix = 2 * b + px;
      if (ix >= W) continue;
      const int64_t off = ((n * H + iy) * W + ix) * C + cg * 8;
      pool_store8(DT, dx, off, acc[py * 2 + px]);
      if (BNS) {
        // statistics from the values the BN backward will read (rounded to the storage type)
        float g[8];
        const float* xv = xq[py * 2 + px];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          g[k] = acc[py * 2 + px][k];
          if (DT != 0) g[k] = DT == 1 ? bf16_to_f32(f32_to_bf16(g[k])) : f16_to_f32(pool_to16(2, g[k]));
          const float dz = __builtin_fmaf(xv[k], ba[k], bb[k]) > 0.0f ? g[k] : 0.0f;
          s1[k] += dz;
          s2[k] = __builtin_fmaf(dz, xv[k] - bm[k], s2[k]);
        }
      }
    }
  }
  }  // grid-stride loop
  if (BNS) {
    // threads of one channel group: t % (C/8) equal -> lanes l, l + C/8, ... then the 4 waves
    __shared__ float red[2][kBlock / 64][64 * 8];
    const int cg8 = C >> 3, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      for (int off = cg8; off < 64; off <<= 1) {
        s1[k] += __shfl_xor(s1[k], off, 64);
        s2[k] += __shfl_xor(s2[k], off, 64);
      }
    if (lane < cg8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[0][wave][lane * 8 + k] = s1[k];
        red[1][wave][lane * 8 + k] = s2[k];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += kBlock) {
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) { a1 += red[0][w][c]; a2 += red[1][w][c]; }
      bp1[(int64_t)c * gridDim.x + blockIdx.x] = a1;
      bp2[(int64_t)c * gridDim.x + blockIdx.x] = a2;
    }
  }
}

template <typename IDX>
static void maxpool_fwd_dispatch(int dtype, dim3 grid, const void* x, void* y, uint8_t* idx, int64_t B, int H, int W,
                                 int C, int Ho, int Wo, int K, int S, int P, hipStream_t s) {
  const dim3 block(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL((maxpool_fwd_kernel<0, IDX>), grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
    case 1: hipLaunchKernelGGL((maxpool_fwd_kernel<1, IDX>), grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
    default: hipLaunchKernelGGL((maxpool_fwd_kernel<2, IDX>), grid, block, 0, s, x, y, idx, B, H, W, C, Ho, Wo, K, S, P); break;
  }
}

template <typename IDX>
static void maxpool_bwd_dispatch(int dtype, dim3 grid, const void* dy, const void* dy2, const uint8_t* idx, void* dx,
                                 int64_t B, int H, int W, int C, int Ho, int Wo, int K, int S, int P, hipStream_t s) {
  const dim3 block(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL((maxpool_bwd_kernel<0, IDX>), grid, block, 0, s, dy, dy2, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
    case 1: hipLaunchKernelGGL((maxpool_bwd_kernel<1, IDX>), grid, block, 0, s, dy, dy2, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
    default: hipLaunchKernelGGL((maxpool_bwd_kernel<2, IDX>), grid, block, 0, s, dy, dy2, idx, dx, B, H, W, C, Ho, Wo, K, S, P); break;
  }
}

void launch_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* idx, int64_t B, int H, int W, int C, int Ho,
                        int Wo, int K, int S, int P, hipStream_t s, const float* coef) {
  const int64_t total = B * Ho * Wo * (C / 8);
  if (total == 0) return;
  const dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
  const int64_t total2 = B * ((Ho + 1) / 2) * ((Wo + 1) / 2) * (C / 8);
  if (K == 3 && S == 2 && P == 1 && total2 + kBlock < (int64_t(1) << 32)) {  // 2x2-block kernel
    const dim3 grid2((unsigned)((total2 + kBlock - 1) / kBlock)), block(kBlock);
    const uint32_t t2 = (uint32_t)total2;
    if (coef != nullptr) {
      switch (dtype) {
        case 0: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<0, true>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
        case 1: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<1, true>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
        default: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<2, true>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
      }
    } else {
      switch (dtype) {
        case 0: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<0, false>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
        case 1: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<1, false>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
        default: hipLaunchKernelGGL((maxpool3s2_fwd_kernel<2, false>), grid2, block, 0, s, x, y, idx, H, W, C, Ho, Wo, t2, coef); break;
      }
    }
    return;
  }
  if (K == 3 && total + kBlock < (int64_t(1) << 32)) {
    const dim3 block(kBlock);
    if (coef != nullptr) {
      switch (dtype) {
        case 0: hipLaunchKernelGGL((maxpool3_fwd_kernel<0, true>), grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total, coef); break;
        case 1: hipLaunchKernelGGL((maxpool3_fwd_kernel<1, true>), grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total, coef); break;
        default: hipLaunchKernelGGL((maxpool3_fwd_kernel<2, true>), grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total, coef); break;
      }
      return;
    }
    switch (dtype) {
      case 0: hipLaunchKernelGGL(maxpool3_fwd_kernel<0>, grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total); break;
      case 1: hipLaunchKernelGGL(maxpool3_fwd_kernel<1>, grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total); break;
      default: hipLaunchKernelGGL(maxpool3_fwd_kernel<2>, grid, block, 0, s, x, y, idx, H, W, C, Ho, Wo, S, P, (uint32_t)total); break;
    }
    return;
  }
  if (coef != nullptr) throw std::runtime_error("maxpool_fwd: the folded BatchNorm apply needs a 3x3 window");
  if (total + kBlock < (int64_t(1) << 32)) maxpool_fwd_dispatch<uint32_t>(dtype, grid, x, y, idx, B, H, W, C, Ho, Wo, K, S, P, s);
  else maxpool_fwd_dispatch<uint64_t>(dtype, grid, x, y, idx, B, H, W, C, Ho, Wo, K, S, P, s);
}

// Blocks of the statistics-summing 3x3/s2 max-pool backward: capped, because every block ends
// with C scattered partial stores per array ([C][blocks], the layout the finalize reads) and the
// finalize reads them all - ResNet-50's stem at batch 256 had 25,088 blocks (DPT_POOL_BN_BLOCKS;
// in-step rocprofv3: uncapped 268 us, 4096 blocks 241, 2048 237, 1024 234, and the stem's BN
// finalize drops from ~21 us to a few, profiles/pool_bn_blocks_r2.txt).
constexpr int kPoolBnBlocks = 1024;

int maxpool_bwd_bn_chunks(int64_t B, int H, int W, int C) {
  const int64_t total2 = B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  return (int)std::min<int64_t>((total2 + kBlock - 1) / kBlock, kPoolBnBlocks);
}

void launch_maxpool_bwd(int dtype, const void* dy, const void* dy2, const uint8_t* idx, void* dx, int64_t B, int H,
                        int W, int C, int Ho, int Wo, int K, int S, int P, hipStream_t s, const void* bnx,
                        const float* bn_mean, const float* bn_coef, float* bp1, float* bp2) {
  const int64_t total = B * H * W * (C / 8);
  if (total == 0) return;
  const int Ha = (H + 1) / 2, Wa = (W + 1) / 2;
  const int64_t total2 = B * Ha * Wa * (C / 8);
  if (K == 3 && S == 2 && P == 1 && Ho == Ha && Wo == Wa && total2 + kBlock < (int64_t(1) << 32)) {
    dim3 g2((unsigned)((total2 + kBlock - 1) / kBlock)), block(kBlock);
    if (bnx != nullptr) {
      g2.x = (unsigned)maxpool_bwd_bn_chunks(B, H, W, C);  // grid-stride; t + stride stays < 2^32
      if (total2 + (int64_t)g2.x * kBlock >= (int64_t(1) << 32))
        throw std::runtime_error("maxpool_bwd: too many elements for the fused statistics path");
      switch (dtype) {
        case 0: hipLaunchKernelGGL((maxpool3s2_bwd_kernel<0, true>), g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2, bnx, bn_mean, bn_coef, bp1, bp2); break;
        case 1: hipLaunchKernelGGL((maxpool3s2_bwd_kernel<1, true>), g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2, bnx, bn_mean, bn_coef, bp1, bp2); break;
        default: hipLaunchKernelGGL((maxpool3s2_bwd_kernel<2, true>), g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2, bnx, bn_mean, bn_coef, bp1, bp2); break;
      }
      return;
    }
    switch (dtype) {
      case 0: hipLaunchKernelGGL(maxpool3s2_bwd_kernel<0>, g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2); break;
      case 1: hipLaunchKernelGGL(maxpool3s2_bwd_kernel<1>, g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2); break;
      default: hipLaunchKernelGGL(maxpool3s2_bwd_kernel<2>, g2, block, 0, s, dy, dy2, idx, dx, H, W, C, Ho, Wo, Ha, Wa, (uint32_t)total2); break;
    }
    return;
  }
  const dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
  if (total + kBlock < (int64_t(1) << 32)) maxpool_bwd_dispatch<uint32_t>(dtype, grid, dy, dy2, idx, dx, B, H, W, C, Ho, Wo, K, S, P, s);
  else maxpool_bwd_dispatch<uint64_t>(dtype, grid, dy, dy2, idx, dx, B, H, W, C, Ho, Wo, K, S, P, s);
}

// Global average pool backward, channels-last: dx[n, p, c] = g[n, c] * inv (every pixel p of
// image n).  ATen's mean backward expands g and copies the strided view into channels_last
// with a non-vectorised kernel (81 us for ResNet-50's [256, 2048, 7, 7] at batch 256); here
// each thread writes 16-byte rows.
template <int DT, int GT>
__global__ __launch_bounds__(kBlock) void gap_bwd_kernel(const void* __restrict__ g, void* __restrict__ dx,
                                                         uint32_t HW, uint32_t C, uint32_t total, float inv) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const uint32_t cg8 = C >> 3;
  const uint32_t cg = t % cg8, n = t / cg8 / HW;
  float v[8];
  pool_load8(GT, g, (int64_t)n * C + cg * 8, v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= inv;
  pool_store8(DT, dx, (int64_t)t * 8, v);
}

// Global-average-pool backward of a block-tail output y = relu(bn(x) + res) (the network's last
// residual block): dz = (g[n, c] / HW) * (y > 0) - the tail's masked gradient, stored in the
// storage type - plus that BatchNorm's backward statistics s1 = sum dz, s2 = sum dz*(x - mean)
// summed from the stored values, per block of `rpb` rows into [C][gridDim.x] partials.  The
// BN backward then applies from the partials (no statistics pass over dy, y and x, no separate
// broadcast pass).  C/8 threads per row, kBlock % (C/8) == 0.
template <int DT, int GT>
__global__ __launch_bounds__(kBlock) void gap_bwd_bnr_kernel(const void* __restrict__ g, void* __restrict__ dz,
                                                             const void* __restrict__ y, const void* __restrict__ x,
                                                             const float* __restrict__ mean, int64_t M, uint32_t HW,
                                                             int C, int rpb, float inv, float* __restrict__ p1,
                                                             float* __restrict__ p2) {
  __shared__ float red[2][kBlock * 8];
  const int tpr = C >> 3, rpp = kBlock / tpr;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { mu[k] = mean[cg * 8 + k]; s1[k] = 0.f; s2[k] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = r0 + rpb < M ? r0 + rpb : M;
  for (int64_t r = r0 + rr; r < r1; r += rpp) {
    const int64_t n = r / HW, off = r * C + cg * 8;
    float gv[8], yv[8], xv[8], o[8];
    pool_load8(GT, g, n * C + cg * 8, gv);
    pool_load8(DT, y, off, yv);
    pool_load8(DT, x, off, xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = yv[k] > 0.0f ? gv[k] * inv : 0.0f;
    pool_store8(DT, dz, off, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // statistics from the stored (rounded) values: what the BN backward apply reads
      const float d = DT == 0 ? o[k] : DT == 1 ? bf16_to_f32(f32_to_bf16(o[k])) : f16_to_f32(pool_to16(2, o[k]));
      s1[k] += d;
      s2[k] = __builtin_fmaf(d, xv[k] - mu[k], s2[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][rr * C + cg * 8 + k] = s1[k];
    red[1][rr * C + cg * 8 + k] = s2[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float a1 = 0.f, a2 = 0.f;
    for (int j = 0; j < rpp; ++j) { a1 += red[0][j * C + c]; a2 += red[1][j * C + c]; }
    p1[(int64_t)c * gridDim.x + blockIdx.x] = a1;
    p2[(int64_t)c * gridDim.x + blockIdx.x] = a2;
  }
}

int gap_bwd_bnr_chunks(int64_t M, int64_t C) {
  const int rpp = kBlock / (int)(C / 8);
  // ~one block per CU: each block ends with C scattered stores per partial array into the
  // [C][blocks] layout the finalize reads, which at C = 2048 costs more than the extra rows per
  // block - ResNet-50's tail, 7x7x2048 x 256 images: 1024 blocks 62 us, 256 blocks 42 us, 128
  // blocks 62 us (profiles/gap_bwd_bnr_blocks_r2.txt)
  constexpr int target = 256;
  int64_t rpb = (M + target - 1) / target;
  rpb = (rpb + rpp - 1) / rpp * rpp;
  return (int)((M + rpb - 1) / rpb);
}

void launch_gap_bwd_bnr(int dtype, int gdtype, const void* g, void* dz, const void* y, const void* x,
                        const float* mean, int64_t N, int64_t HW, int64_t C, float* p1, float* p2, hipStream_t s) {
  const int64_t M = N * HW;
  const int chunks = gap_bwd_bnr_chunks(M, C);
  const int rpb = (int)((M + chunks - 1) / chunks);
  const dim3 grid((unsigned)chunks), block(kBlock);
  const float inv = 1.0f / (float)HW;
#define DPT_GAPB(D, G) hipLaunchKernelGGL((gap_bwd_bnr_kernel<D, G>), grid, block, 0, s, g, dz, y, x, mean, M, (uint32_t)HW, (int)C, rpb, inv, p1, p2)
  if (gdtype == 0) {
    if (dtype == 0) DPT_GAPB(0, 0); else if (dtype == 1) DPT_GAPB(1, 0); else DPT_GAPB(2, 0);
  } else if (gdtype == 1) {
    if (dtype == 0) DPT_GAPB(0, 1); else if (dtype == 1) DPT_GAPB(1, 1); else DPT_GAPB(2, 1);
  } else {
    if (dtype == 0) DPT_GAPB(0, 2); else if (dtype == 1) DPT_GAPB(1, 2); else DPT_GAPB(2, 2);
  }
#undef DPT_GAPB
}

void launch_gap_bwd(int dtype, int gdtype, const void* g, void* dx, int64_t N, int64_t HW, int64_t C, hipStream_t s) {
  const int64_t total = N * HW * (C / 8);
  if (total == 0) return;
  const dim3 grid((unsigned)((total + kBlock - 1) / kBlock)), block(kBlock);
  const float inv = 1.0f / (float)HW;
#define DPT_GAP(D, G) hipLaunchKernelGGL((gap_bwd_kernel<D, G>), grid, block, 0, s, g, dx, (uint32_t)HW, (uint32_t)C, (uint32_t)total, inv)
  if (gdtype == 0) {
    if (dtype == 0) DPT_GAP(0, 0); else if (dtype == 1) DPT_GAP(1, 0); else DPT_GAP(2, 0);
  } else if (gdtype == 1) {
    if (dtype == 0) DPT_GAP(0, 1); else if (dtype == 1) DPT_GAP(1, 1); else DPT_GAP(2, 1);
  } else {
    if (dtype == 0) DPT_GAP(0, 2); else if (dtype == 1) DPT_GAP(1, 2); else DPT_GAP(2, 2);
  }
#undef DPT_GAP
}

}  // namespace dpt
