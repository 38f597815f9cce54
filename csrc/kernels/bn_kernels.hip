// Fused channels-last BatchNorm (+ReLU) (+residual add) for training on gfx950.
//
// Why: on MI355X a ResNet-50 bf16 step (batch 256, channels_last) spends 37% of its kernel
// time in MIOpen's BatchNorm kernels and another ~15% in the ReLU / threshold-backward /
// residual-add elementwise kernels around them (profiles/resnet50_miopen_bn_breakdown.md) - all
// HBM-bound passes over the same activations.  These kernels fuse them:
//
//   forward  (train): stats     read x                      -> per-chunk (sum, sumsq) partials
//                     finalize  partials -> mean, invstd, a = g*invstd, b = beta - mean*a,
//                               running stats (momentum, unbiased var), num_batches_tracked++
//                     apply     y = relu(x*a + b [+ r])      read x [, r], write y
//   backward:         stats     dz = (dy [+ dy2]) * (y > 0);  s1 = sum dz, s2 = sum dz*(x - mean)
//                               [residual blocks: store dz - it IS the residual-path gradient]
//                     finalize  dgamma = s2*invstd, dbeta = s1, dx coefficients k1,k2,k3
//                     apply     dx = k1*dz + k2*(x - mean) + k3   (dz recomputed or read back)
//
// Layout: a channels_last activation is a row-major [M = N*H*W, C] matrix.  Threads are
// "channel-stationary": with 256 threads and C/8 threads per row, each thread owns one
// 8-channel group (one 16-byte vector of bf16) for every row it visits, so per-channel
// coefficients live in registers and every global access is a full 16-byte vector.
// Requires C % 8 == 0 and (C/8) | 256, i.e. C in {8, 16, ..., 2048} (every ResNet width);
// the Python layer falls back to the unfused path otherwise.
//
// Reductions are deterministic two-level: fixed row chunks -> fp32 partials [C][chunks]
// -> fp64 per-channel sums in a finalize kernel (one wave per 2 channels).  No atomics.
#include <cstdlib>

#include "carry.h"
#include "common.h"
#include "kernels.h"

namespace dpt {

// ---- 8-element vector I/O for the three activation dtypes ----------------------------------
struct BF16 {
  using raw = uint16_t;
  __device__ static void load8(const void* p, int64_t i, float f[8]) {
    uint4 w = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = bf16_to_f32(u[k] & 0xffff);
      f[2 * k + 1] = bf16_to_f32(u[k] >> 16);
    }
  }
  __device__ static void store8(void* p, int64_t i, const float f[8]) {
    uint4 w;
    w.x = (uint32_t)f32_to_bf16(f[0]) | ((uint32_t)f32_to_bf16(f[1]) << 16);
    w.y = (uint32_t)f32_to_bf16(f[2]) | ((uint32_t)f32_to_bf16(f[3]) << 16);
    w.z = (uint32_t)f32_to_bf16(f[4]) | ((uint32_t)f32_to_bf16(f[5]) << 16);
    w.w = (uint32_t)f32_to_bf16(f[6]) | ((uint32_t)f32_to_bf16(f[7]) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) = w;
  }
  // y > 0 test straight on the bits (sign clear, not +0, not NaN): no conversion needed.
  __device__ static bool pos16(uint32_t h) { return !(h & 0x8000u) && (h & 0x7fffu) && (h & 0x7fffu) <= 0x7f80u; }
  // store8 that also returns the ReLU mask of the STORED (rounded) values, bit k = channel k
  __device__ static uint32_t store8m(void* p, int64_t i, const float f[8]) {
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = f32_to_bf16(f[k]);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) =
        make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) m |= (pos16(h[k]) ? 1u : 0u) << k;
    return m;
  }
  __device__ static void pos8(const void* p, int64_t i, bool m[8]) {
    uint4 w = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t lo = u[k] & 0xffff, hi = u[k] >> 16;
      m[2 * k] = !(lo & 0x8000) && (lo & 0x7fff) && (lo & 0x7fff) <= 0x7f80;
      m[2 * k + 1] = !(hi & 0x8000) && (hi & 0x7fff) && (hi & 0x7fff) <= 0x7f80;
    }
  }
};

struct F16 {
  __device__ static void load8(const void* p, int64_t i, float f[8]) {
    uint4 w = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
    uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = f16_to_f32(u[k] & 0xffff);
      f[2 * k + 1] = f16_to_f32(u[k] >> 16);
    }
  }
  __device__ static uint16_t to16(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
  __device__ static void store8(void* p, int64_t i, const float f[8]) {
    uint4 w;
    w.x = (uint32_t)to16(f[0]) | ((uint32_t)to16(f[1]) << 16);
    w.y = (uint32_t)to16(f[2]) | ((uint32_t)to16(f[3]) << 16);
    w.z = (uint32_t)to16(f[4]) | ((uint32_t)to16(f[5]) << 16);
    w.w = (uint32_t)to16(f[6]) | ((uint32_t)to16(f[7]) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + i) = w;
  }
  __device__ static uint32_t store8m(void* p, int64_t i, const float f[8]) {
    store8(p, i, f);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) m |= ((float)__builtin_bit_cast(_Float16, to16(f[k])) > 0.0f ? 1u : 0u) << k;
    return m;
  }
  __device__ static void pos8(const void* p, int64_t i, bool m[8]) {
    float f[8];
    load8(p, i, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = f[k] > 0.0f;
  }
};

struct F32 {
  __device__ static void load8(const void* p, int64_t i, float f[8]) {
    const float4* q = reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    float4 a = q[0], b = q[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  __device__ static void store8(void* p, int64_t i, const float f[8]) {
    float4* q = reinterpret_cast<float4*>(static_cast<float*>(p) + i);
    q[0] = make_float4(f[0], f[1], f[2], f[3]);
    q[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  __device__ static uint32_t store8m(void* p, int64_t i, const float f[8]) {
    store8(p, i, f);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) m |= (f[k] > 0.0f ? 1u : 0u) << k;
    return m;
  }
  __device__ static void pos8(const void* p, int64_t i, bool m[8]) {
    float f[8];
    load8(p, i, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = f[k] > 0.0f;
  }
};

// ---- forward statistics: per-chunk partial sum / sum of squares --------------------------------
template <typename IO>
__global__ __launch_bounds__(kBlock) void bn_fwd_stats_kernel(const void* __restrict__ x, int64_t M, int C,
                                                              int64_t rows_per_chunk, int chunks,
                                                              float* __restrict__ psum,
                                                              float* __restrict__ psq) {
  __shared__ float lds[2 * kBlock * 8];
  const int tpr = C >> 3, rpi = kBlock / tpr;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  const int64_t row0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t row1 = min(row0 + rows_per_chunk, M);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t r = row0 + rr;
  for (; r + 3 * rpi < row1; r += 4 * rpi) {  // four 16-byte rows in flight per thread
    float a[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) IO::load8(x, (r + u * rpi) * C + cg * 8, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += a[u][k];
        q[k] += a[u][k] * a[u][k];
      }
  }
  for (; r < row1; r += rpi) {
    float a[8];
    IO::load8(x, r * C + cg * 8, a);
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] += a[k]; q[k] += a[k] * a[k]; }
  }
  float* ls = lds;
  float* lq = lds + kBlock * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ls[rr * C + cg * 8 + k] = s[k];
    lq[rr * C + cg * 8 + k] = q[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float ts = 0.f, tq = 0.f;
    for (int j = 0; j < rpi; ++j) { ts += ls[j * C + c]; tq += lq[j * C + c]; }
    psum[(int64_t)c * chunks + blockIdx.x] = ts;
    psq[(int64_t)c * chunks + blockIdx.x] = tq;
  }
}

__global__ __launch_bounds__(kBlock) void bn_fwd_finalize_kernel(
    const float* __restrict__ psum, const float* __restrict__ psq, int chunks, int C, int64_t M,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* run_mean, float* run_var, int64_t* num_batches, float* save_mean, float* save_invstd,
    float* coef_a, float* coef_b) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 8 + wave * 2 + (lane >> 5);
  const int part = lane & 31;
  if (blockIdx.x == 0 && threadIdx.x == 0 && num_batches) num_batches[0] += 1;
  if (c >= C) return;
  double s, q;
  half_wave_sum2(psum, psq, c, chunks, part, s, q);
  if (part != 0) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.0f, bt = beta ? beta[c] : 0.0f;
  const float a = g * invstd;
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  coef_a[c] = a;
  coef_b[c] = bt - (float)mean * a;
  if (run_mean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.0f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

// Same finalize for MANY partials per channel (the conv epilogue writes one per 128 rows: up
// to ~6k at ResNet-50's 56x56 layers): one 256-thread block per channel, fp64 block reduce.
// Wave-reduced fp64 sums of two contiguous fp32 rows of `chunks` partials (one block per
// channel): 8 loads of each row in flight per thread - the finalize is a latency chain of
// chunks / (kBlock * U) dependent round trips, not a bandwidth problem.

template <int NT>
__global__ __launch_bounds__(NT) void bn_fwd_finalize_wide_kernel(
    const float* __restrict__ psum, const float* __restrict__ psq, int chunks, int C, int64_t M,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* run_mean, float* run_var, int64_t* num_batches, float* save_mean, float* save_invstd,
    float* coef_a, float* coef_b) {
  __shared__ double red[2][NT / 64];
  const int c = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (c == 0 && threadIdx.x == 0 && num_batches) num_batches[0] += 1;
  double s, q;
  block_row_sum2<NT>(psum + (int64_t)c * chunks, psq + (int64_t)c * chunks, chunks, s, q);
  if (lane == 0) { red[0][wave] = s; red[1][wave] = q; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s = 0.0;
  q = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) { s += red[0][w]; q += red[1][w]; }
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.0f, bt = beta ? beta[c] : 0.0f;
  const float a = g * invstd;
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  coef_a[c] = a;
  coef_b[c] = bt - (float)mean * a;
  if (run_mean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.0f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

// ---- forward apply: y = relu(x*a + b [+ r]) --------------------------------------------------
// AFF: the residual is itself a BatchNorm input (a residual block's downsample branch): y =
// relu(x*a + b + r*a2 + b2) - the downsample BN's output is never materialised.
template <typename IO, bool RELU, bool RES, bool AFF = false>
__global__ __launch_bounds__(kBlock) void bn_fwd_apply_kernel(const void* __restrict__ x,
                                                              const void* __restrict__ res,
                                                              void* __restrict__ y,
                                                              const float* __restrict__ coef_a,
                                                              const float* __restrict__ coef_b,
                                                              int64_t M, int C, int rev,
                                                              const float* __restrict__ coef_a2 = nullptr,
                                                              const float* __restrict__ coef_b2 = nullptr,
                                                              uint8_t* __restrict__ mask = nullptr) {
  const int tpr = C >> 3, rpi = kBlock / tpr;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  float a[8], b[8], a2[8], b2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = coef_a[cg * 8 + k];
    b[k] = coef_b[cg * 8 + k];
    a2[k] = AFF ? coef_a2[cg * 8 + k] : 0.f;
    b2[k] = AFF ? coef_b2[cg * 8 + k] : 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * rpi;
  for (int64_t rf = (int64_t)blockIdx.x * rpi + rr; rf < M; rf += 2 * stride) {
    const bool two = rf + stride < M;
    // rev: walk the rows last-to-first so the first blocks re-read what the stats pass
    // touched last (still resident in the 256 MB Infinity Cache / L2)
    const int64_t r = rev ? M - 1 - rf : rf;
    const int64_t r2 = rev ? r - stride : r + stride;
    float v0[8], v1[8], q0[8], q1[8];
    IO::load8(x, r * C + cg * 8, v0);
    if (two) IO::load8(x, r2 * C + cg * 8, v1);
    if (RES) {
      IO::load8(res, r * C + cg * 8, q0);
      if (two) IO::load8(res, r2 * C + cg * 8, q1);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o0 = __builtin_fmaf(v0[k], a[k], b[k]);  // bwd mask-from-x recomputes exactly this
      float o1 = __builtin_fmaf(v1[k], a[k], b[k]);
      if (RES && AFF) {
        o0 += __builtin_fmaf(q0[k], a2[k], b2[k]);
        o1 += __builtin_fmaf(q1[k], a2[k], b2[k]);
      } else if (RES) {
        o0 += q0[k];
        o1 += q1[k];
      }
      if (RELU) {  // NaN-propagating like torch.relu (a NaN must still reach the AMP check)
        o0 = o0 < 0.0f ? 0.0f : o0;
        o1 = o1 < 0.0f ? 0.0f : o1;
      }
      v0[k] = o0;
      v1[k] = o1;
    }
    if (RELU && RES && mask != nullptr) {
      // block tail: also the 1-bit ReLU mask [M][C/8] the consuming conv's backward-data
      // epilogue reads instead of y (ops/bn.py) - 1/16 of y's bytes
      mask[r * tpr + cg] = (uint8_t)IO::store8m(y, r * C + cg * 8, v0);
      if (two) mask[r2 * tpr + cg] = (uint8_t)IO::store8m(y, r2 * C + cg * 8, v1);
    } else {
      IO::store8(y, r * C + cg * 8, v0);
      if (two) IO::store8(y, r2 * C + cg * 8, v1);
    }
  }
}

// ReLU mask of one 8-channel vector: from the saved output (y > 0) or, MX, recomputed from
// the BN input with the forward's own coefficients (fma(x, a, b) > 0 - the exact value the
// forward apply clamped), which saves reading y in both backward passes.
template <typename IO, bool MX>
__device__ __forceinline__ void relu_mask8(const void* y, int64_t off, const float xv[8], const float a[8],
                                           const float b[8], bool m[8]) {
  if (MX) {
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = __builtin_fmaf(xv[k], a[k], b[k]) > 0.0f;
  } else {
    IO::pos8(y, off, m);
  }
}

// ---- backward statistics: s1 = sum dz, s2 = sum dz*(x-mean), dz = (dy [+ dy2]) * (y > 0) ------
// TWO: the output had two consumers (conv path + identity path of the next residual block,
// see ops/bn.py "pair" outputs); their gradients arrive separately and are summed here
// instead of in an autograd add kernel.  WDZ: also store dz (it is the residual-path
// gradient dres, and the apply pass then reads dz instead of dy, dy2 and y).  MX: ReLU mask
// recomputed from x and the forward coefficients coef = [a | b] (non-residual BN+ReLU).
template <typename IO, bool RELU, bool TWO, bool WDZ, int UNR, bool MX>
__global__ __launch_bounds__(kBlock) void bn_bwd_stats_kernel(const void* __restrict__ dy,
                                                              const void* __restrict__ dy2,
                                                              const void* __restrict__ y,
                                                              const void* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ coef, int64_t M,
                                                              int C, int64_t rows_per_chunk, int chunks,
                                                              float* __restrict__ p1,
                                                              float* __restrict__ p2,
                                                              void* __restrict__ dz_out) {
  __shared__ float lds[2 * kBlock * 8];
  const int tpr = C >> 3, rpi = kBlock / tpr;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  float mu[8], fa[8], fb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[cg * 8 + k];
    fa[k] = MX ? coef[cg * 8 + k] : 0.f;
    fb[k] = MX ? coef[C + cg * 8 + k] : 0.f;
  }
  const int64_t row0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t row1 = min(row0 + rows_per_chunk, M);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t r = row0 + rr;
  for (; r + (UNR - 1) * rpi < row1; r += UNR * rpi) {  // UNR rows x (3 or 4) tensors in flight
    float g[UNR][8], g2[UNR][8], xv[UNR][8];
    bool m[UNR][8];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t off = (r + u * rpi) * C + cg * 8;
      IO::load8(dy, off, g[u]);
      if (TWO) IO::load8(dy2, off, g2[u]);
      IO::load8(x, off, xv[u]);
      if (RELU && !MX) IO::pos8(y, off, m[u]);
    }
    if (RELU && MX) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) relu_mask8<IO, true>(y, 0, xv[u], fa, fb, m[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float gk = TWO ? g[u][k] + g2[u][k] : g[u][k];
        float dz = (!RELU || m[u][k]) ? gk : 0.0f;
        g[u][k] = dz;
        s[k] += dz;
        q[k] += dz * (xv[u][k] - mu[k]);
      }
      if (WDZ) IO::store8(dz_out, (r + u * rpi) * C + cg * 8, g[u]);
    }
  }
  for (; r < row1; r += rpi) {
    const int64_t off = r * C + cg * 8;
    float g[8], g2[8], xv[8];
    bool m[8];
    IO::load8(dy, off, g);
    if (TWO) IO::load8(dy2, off, g2);
    IO::load8(x, off, xv);
    if (RELU) relu_mask8<IO, MX>(y, off, xv, fa, fb, m);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gk = TWO ? g[k] + g2[k] : g[k];
      float dz = (!RELU || m[k]) ? gk : 0.0f;
      g[k] = dz;
      s[k] += dz;
      q[k] += dz * (xv[k] - mu[k]);
    }
    if (WDZ) IO::store8(dz_out, off, g);
  }
  float* ls = lds;
  float* lq = lds + kBlock * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ls[rr * C + cg * 8 + k] = s[k];
    lq[rr * C + cg * 8 + k] = q[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float ts = 0.f, tq = 0.f;
    for (int j = 0; j < rpi; ++j) { ts += ls[j * C + c]; tq += lq[j * C + c]; }
    p1[(int64_t)c * chunks + blockIdx.x] = ts;
    p2[(int64_t)c * chunks + blockIdx.x] = tq;
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void bn_bwd_finalize_kernel(BnBwdFin f) {
  __shared__ double red[2 * (NT / 64)];
  bn_bwd_finalize_block<NT>(f, (int)blockIdx.x, red);
}

// Two BatchNorms' finalizes in one launch (a block tail with its downsample BN folded in)
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize2_kernel(BnBwdFin f, BnBwdFin h) {
  __shared__ double red[2 * (kBlock / 64)];
  if ((int)blockIdx.x < f.blocks) bn_bwd_finalize_block(f, (int)blockIdx.x, red);
  else bn_bwd_finalize_block(h, (int)blockIdx.x - f.blocks, red);
}

BnBwdFin make_bn_bwd_fin(const float* p1, const float* p2, int chunks, int C, int64_t M, const float* gamma,
                         const float* invstd, float* dgamma, float* dbeta, float* k1, float* k2, float* k3,
                         int wide) {
  BnBwdFin f;
  f.p1 = p1; f.p2 = p2; f.chunks = chunks; f.C = C; f.M = M; f.gamma = gamma; f.invstd = invstd;
  f.dgamma = dgamma; f.dbeta = dbeta; f.k1 = k1; f.k2 = k2; f.k3 = k3;
  f.wide = wide < 0 ? bn_bwd_fin_wide(chunks) : wide;
  f.blocks = bn_bwd_fin_blocks(C, f.wide);
  return f;
}

// Wide finalizes (one block per channel, thousands of partials) run 256-thread blocks too: 512
// and 1024 measured 0.3-0.5 % slower in the step (docs/DESIGN.md §9).
// Measurement only (bench/ab_step.py arm bn_set_skip_finalize:1): skip every BatchNorm finalize
// launch - WRONG values (stale coefficients), the upper bound of what folding the finalizes into
// neighbouring kernels could save.  Never set in training.
static int g_bn_skip_finalize = 0;
void bn_set_skip_finalize(int on) { g_bn_skip_finalize = on; }

static void launch_bn_bwd_fin(const BnBwdFin& f, hipStream_t s) {
  if (g_bn_skip_finalize) return;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<kBlock>, dim3((unsigned)f.blocks), dim3(kBlock), 0, s, f);
}

// dx = k1*dz + k2*(x - mean) + k3, dz = dy*(y>0) recomputed (RELU; mask from x if MX) or
// read back (FROM_DZ).
template <typename IO, bool RELU, bool FROM_DZ, bool MX>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(const void* __restrict__ dy,
                                                              const void* __restrict__ y,
                                                              const void* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ coef,
                                                              const float* __restrict__ k1,
                                                              const float* __restrict__ k2,
                                                              const float* __restrict__ k3, void* dx,
                                                              int64_t M, int C, int rev, ReduceCarry rc) {
  if (rc.blocks) {  // carried backward-weight reduce (carry.h): the grid's last rc.blocks blocks
    const int napply = (int)gridDim.x - rc.blocks;
    if ((int)blockIdx.x >= napply) {
      __shared__ float4 red[kBlock];
      carry_reduce(rc, (int)blockIdx.x - napply, red);
      return;
    }
  }
  const int tpr = C >> 3, rpi = kBlock / tpr;
  // grid-stride over the apply blocks only (carry blocks excluded)
  const int apply_grid = (int)gridDim.x - rc.blocks;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  float mu[8], c1[8], c2[8], c3[8], fa[8], fb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[cg * 8 + k];
    c1[k] = k1[cg * 8 + k];
    c2[k] = k2[cg * 8 + k];
    c3[k] = k3[cg * 8 + k];
    fa[k] = MX ? coef[cg * 8 + k] : 0.f;
    fb[k] = MX ? coef[C + cg * 8 + k] : 0.f;
  }
  const int64_t stride = (int64_t)apply_grid * rpi;
  for (int64_t rf = (int64_t)blockIdx.x * rpi + rr; rf < M; rf += stride) {
    const int64_t r = rev ? M - 1 - rf : rf;  // see bn_fwd_apply_kernel
    float g[8], xv[8], o[8];
    bool m[8];
    IO::load8(dy, r * C + cg * 8, g);
    IO::load8(x, r * C + cg * 8, xv);
    if (RELU && !FROM_DZ) relu_mask8<IO, MX>(y, r * C + cg * 8, xv, fa, fb, m);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float dz = (FROM_DZ || !RELU || m[k]) ? g[k] : 0.0f;
      o[k] = c1[k] * dz + c2[k] * (xv[k] - mu[k]) + c3[k];
    }
    IO::store8(dx, r * C + cg * 8, o);
  }
}

// Block tail with a downsample branch (ops/bn.py _BN2AddReLUPair): one pass over dz writes both
// BatchNorms' input gradients, dx = k1*dz + k2*(x - mean) + k3 and dx2 = j1*dz + j2*(x2 - mean2) + j3.
template <typename IO>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply2_kernel(const void* __restrict__ dz,
                                                               const void* __restrict__ x,
                                                               const void* __restrict__ x2,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ mean2,
                                                               const float* __restrict__ k,
                                                               const float* __restrict__ j, void* dx, void* dx2,
                                                               int64_t M, int C, int rev) {
  const int tpr = C >> 3, rpi = kBlock / tpr;
  const int cg = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  float mu[8], mu2[8], c1[8], c2[8], c3[8], e1[8], e2[8], e3[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = cg * 8 + q;
    mu[q] = mean[c];
    mu2[q] = mean2[c];
    c1[q] = k[c]; c2[q] = k[C + c]; c3[q] = k[2 * C + c];
    e1[q] = j[c]; e2[q] = j[C + c]; e3[q] = j[2 * C + c];
  }
  const int64_t stride = (int64_t)gridDim.x * rpi;
  for (int64_t rf = (int64_t)blockIdx.x * rpi + rr; rf < M; rf += stride) {
    const int64_t r = rev ? M - 1 - rf : rf;
    const int64_t off = r * C + cg * 8;
    float g[8], xv[8], x2v[8], o[8], o2[8];
    IO::load8(dz, off, g);
    IO::load8(x, off, xv);
    IO::load8(x2, off, x2v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = c1[q] * g[q] + c2[q] * (xv[q] - mu[q]) + c3[q];
      o2[q] = e1[q] * g[q] + e2[q] * (x2v[q] - mu2[q]) + e3[q];
    }
    IO::store8(dx, off, o);
    IO::store8(dx2, off, o2);
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
bool bn_supported(int64_t C) {
  return C >= 8 && C % 8 == 0 && C <= 8 * kBlock && kBlock % (C / 8) == 0;
}

// Geometry constants, measured on MI355X at the ResNet-50 shapes (bench/bn_micro.py,
// profiles/bn_kernel_knob_sweep.txt): statistics blocks per channel group, rows in flight in
// the backward statistics pass, forward / backward apply grid caps (one 2-row iteration per
// thread forward), and apply passes walking rows last-to-first (the rows the producing kernel
// wrote last are still in the caches).
constexpr int kBnMaxChunks = 512;
constexpr int kBnBwdUnroll = 2;
constexpr int kBnApplyMax = 32768;
constexpr int kBnBwdApplyMax = 4 * kMaxBlocks;
constexpr int kBnReverse = 1;

BnGeometry bn_geometry(int64_t M, int64_t C) {
  BnGeometry g;
  const int64_t rpi = kBlock / (C / 8);
  // Enough chunks to fill the chip (<= 1024 blocks of 256 threads, 4 per CU), >= 64 rows
  // each so the fp32 partials stay a few percent of the activation bytes and the finalize
  // sweep stays short; rows_per_chunk is a multiple of rpi.
  int64_t rows = (M + kBnMaxChunks - 1) / kBnMaxChunks;
  if (rows < 64) rows = 64;
  rows = (rows + rpi - 1) / rpi * rpi;
  g.rows_per_chunk = rows;
  g.chunks = (int)((M + rows - 1) / rows);
  if (g.chunks < 1) g.chunks = 1;
  int64_t apply = (M + rpi * 2 - 1) / (rpi * 2);
  g.apply_blocks = (int)(apply < 1 ? 1 : (apply > kBnApplyMax ? kBnApplyMax : apply));
  return g;
}

template <typename IO>
static void fwd_apply_dispatch(bool relu, bool res, const void* x, const void* r, void* y, const float* a,
                               const float* b, int64_t M, int C, int blocks, hipStream_t s, uint8_t* mask = nullptr) {
  dim3 gr(blocks), bl(kBlock);
  const int rev = kBnReverse;
  if (relu && res)
    hipLaunchKernelGGL((bn_fwd_apply_kernel<IO, true, true>), gr, bl, 0, s, x, r, y, a, b, M, C, rev, nullptr, nullptr,
                       mask);
  else if (relu) hipLaunchKernelGGL((bn_fwd_apply_kernel<IO, true, false>), gr, bl, 0, s, x, r, y, a, b, M, C, rev);
  else if (res) hipLaunchKernelGGL((bn_fwd_apply_kernel<IO, false, true>), gr, bl, 0, s, x, r, y, a, b, M, C, rev);
  else hipLaunchKernelGGL((bn_fwd_apply_kernel<IO, false, false>), gr, bl, 0, s, x, r, y, a, b, M, C, rev);
}

void launch_bn_fwd_train(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                         const float* gamma, const float* beta, float eps, float momentum, float* run_mean,
                         float* run_var, int64_t* num_batches, float* save_mean, float* save_invstd,
                         float* save_coef, float* workspace, bool relu, hipStream_t s, uint8_t* mask) {
  BnGeometry g = bn_geometry(M, C);
  float* psum = workspace;
  float* psq = psum + (int64_t)C * g.chunks;
  float* ca = save_coef ? save_coef : psq + (int64_t)C * g.chunks;
  float* cb = ca + C;
  dim3 bl(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(bn_fwd_stats_kernel<F32>, dim3(g.chunks), bl, 0, s, x, M, (int)C, g.rows_per_chunk, g.chunks, psum, psq); break;
    case 1: hipLaunchKernelGGL(bn_fwd_stats_kernel<BF16>, dim3(g.chunks), bl, 0, s, x, M, (int)C, g.rows_per_chunk, g.chunks, psum, psq); break;
    default: hipLaunchKernelGGL(bn_fwd_stats_kernel<F16>, dim3(g.chunks), bl, 0, s, x, M, (int)C, g.rows_per_chunk, g.chunks, psum, psq); break;
  }
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((unsigned)((C + 7) / 8)), bl, 0, s, psum, psq, g.chunks, (int)C, M,
                     gamma, beta, eps, momentum, run_mean, run_var, num_batches, save_mean, save_invstd, ca, cb);
  if (y == nullptr) return;  // statistics only (the apply is fused elsewhere)
  switch (dtype) {
    case 0: fwd_apply_dispatch<F32>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
    case 1: fwd_apply_dispatch<BF16>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
    default: fwd_apply_dispatch<F16>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
  }
}

// BN forward whose statistics were already summed by the producing convolution's epilogue
// (conv_kernels.hip): psum/psq are [C][chunks] partials -> finalize -> apply.
void launch_bn_fwd_from_partials(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                                 const float* psum, const float* psq, int chunks, const float* gamma,
                                 const float* beta, float eps, float momentum, float* run_mean, float* run_var,
                                 int64_t* num_batches, float* save_mean, float* save_invstd, float* save_coef,
                                 bool relu, hipStream_t s, uint8_t* mask) {
  BnGeometry g = bn_geometry(M, C);
  float* ca = save_coef;
  float* cb = ca + C;
  if (g_bn_skip_finalize) {
  } else if (chunks > 256) {
#define DPT_FWD_FIN(NT)                                                                                        \
  hipLaunchKernelGGL(bn_fwd_finalize_wide_kernel<NT>, dim3((unsigned)C), dim3(NT), 0, s, psum, psq, chunks, (int)C, \
                     M, gamma, beta, eps, momentum, run_mean, run_var, num_batches, save_mean, save_invstd, ca, cb)
    // tens of thousands of partials per channel (the ResNet stem's conv epilogue: 25,088 at
    // batch 256, 64 channels = 64 blocks): 1024 threads, 4x the loads in flight of this
    // latency-bound sweep
    if (chunks > 8192) DPT_FWD_FIN(1024);
    else DPT_FWD_FIN(kBlock);
#undef DPT_FWD_FIN
  } else
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((unsigned)((C + 7) / 8)), dim3(kBlock), 0, s, psum, psq, chunks,
                       (int)C, M, gamma, beta, eps, momentum, run_mean, run_var, num_batches, save_mean, save_invstd,
                       ca, cb);
  if (y == nullptr) return;  // statistics only (the apply is fused elsewhere)
  switch (dtype) {
    case 0: fwd_apply_dispatch<F32>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
    case 1: fwd_apply_dispatch<BF16>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
    default: fwd_apply_dispatch<F16>(relu, res != nullptr, x, res, y, ca, cb, M, (int)C, g.apply_blocks, s, mask); break;
  }
}

void launch_bn_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                     const float* coef_a, const float* coef_b, bool relu, hipStream_t s) {
  BnGeometry g = bn_geometry(M, C);
  switch (dtype) {
    case 0: fwd_apply_dispatch<F32>(relu, res != nullptr, x, res, y, coef_a, coef_b, M, (int)C, g.apply_blocks, s); break;
    case 1: fwd_apply_dispatch<BF16>(relu, res != nullptr, x, res, y, coef_a, coef_b, M, (int)C, g.apply_blocks, s); break;
    default: fwd_apply_dispatch<F16>(relu, res != nullptr, x, res, y, coef_a, coef_b, M, (int)C, g.apply_blocks, s); break;
  }
}

template <typename IO, int UNR>
static void bwd_stats_dispatch(bool relu, const void* dy, const void* dy2, const void* y, const void* x,
                               const float* mean, const float* coef, int64_t M, int C, const BnGeometry& g,
                               float* p1, float* p2, void* dz, hipStream_t s) {
  dim3 bl(kBlock), gs(g.chunks);
  const int64_t rpc = g.rows_per_chunk;
#define DPT_BN_STATS(R, T, W, MXV) \
  hipLaunchKernelGGL((bn_bwd_stats_kernel<IO, R, T, W, UNR, MXV>), gs, bl, 0, s, dy, dy2, y, x, mean, coef, M, C, \
                     rpc, g.chunks, p1, p2, dz)
  if (dz != nullptr) {  // dz written by the stats pass, read back by the apply pass
    if (relu && dy2) DPT_BN_STATS(true, true, true, false);
    else if (relu) DPT_BN_STATS(true, false, true, false);
    else if (dy2) DPT_BN_STATS(false, true, true, false);
    else DPT_BN_STATS(false, false, true, false);
  } else {
    if (relu && coef) DPT_BN_STATS(true, false, false, true);
    else if (relu) DPT_BN_STATS(true, false, false, false);
    else DPT_BN_STATS(false, false, false, false);
  }
#undef DPT_BN_STATS
}

template <typename IO>
static void bwd_dispatch(bool relu, const void* dy, const void* dy2, const void* y, const void* x,
                         const float* mean, const float* coef, int64_t M, int C, const BnGeometry& g, float* p1,
                         float* p2, const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                         float* k1, float* k2, float* k3, void* dx, void* dz, hipStream_t s) {
  dim3 bl(kBlock);
  bwd_stats_dispatch<IO, kBnBwdUnroll>(relu, dy, dy2, y, x, mean, coef, M, C, g, p1, p2, dz, s);
  launch_bn_bwd_fin(make_bn_bwd_fin(p1, p2, g.chunks, C, M, gamma, invstd, dgamma, dbeta, k1, k2, k3, 0), s);
  dim3 ga(g.apply_blocks * 2 > kBnBwdApplyMax ? kBnBwdApplyMax : g.apply_blocks * 2);
  if (dz != nullptr) hipLaunchKernelGGL((bn_bwd_apply_kernel<IO, false, true, false>), ga, bl, 0, s, dz, y, x, mean, coef, k1, k2, k3, dx, M, C, kBnReverse, ReduceCarry{});
  else if (relu && coef) hipLaunchKernelGGL((bn_bwd_apply_kernel<IO, true, false, true>), ga, bl, 0, s, dy, y, x, mean, coef, k1, k2, k3, dx, M, C, kBnReverse, ReduceCarry{});
  else if (relu) hipLaunchKernelGGL((bn_bwd_apply_kernel<IO, true, false, false>), ga, bl, 0, s, dy, y, x, mean, coef, k1, k2, k3, dx, M, C, kBnReverse, ReduceCarry{});
  else hipLaunchKernelGGL((bn_bwd_apply_kernel<IO, false, false, false>), ga, bl, 0, s, dy, y, x, mean, coef, k1, k2, k3, dx, M, C, kBnReverse, ReduceCarry{});
}

// dz: if non-null, receives dz = (dy [+ dy2]) * relu_mask (the residual-path gradient);
// required when dy2 is given.  coef: the forward's [a | b] (2C floats); when given (and no dz),
// the ReLU mask is recomputed from x and y is not read.
void launch_bn_bwd(int dtype, const void* dy, const void* dy2, const void* y, const void* x, int64_t M,
                   int64_t C, const float* gamma, const float* mean, const float* invstd, const float* coef,
                   float* dgamma, float* dbeta, void* dx, void* dz, float* workspace, bool relu, hipStream_t s) {
  BnGeometry g = bn_geometry(M, C);
  float* p1 = workspace;
  float* p2 = p1 + (int64_t)C * g.chunks;
  float* k1 = p2 + (int64_t)C * g.chunks;
  float* k2 = k1 + C;
  float* k3 = k2 + C;
  switch (dtype) {
    case 0: bwd_dispatch<F32>(relu, dy, dy2, y, x, mean, dz ? nullptr : coef, M, (int)C, g, p1, p2, gamma, invstd, dgamma, dbeta, k1, k2, k3, dx, dz, s); break;
    case 1: bwd_dispatch<BF16>(relu, dy, dy2, y, x, mean, dz ? nullptr : coef, M, (int)C, g, p1, p2, gamma, invstd, dgamma, dbeta, k1, k2, k3, dx, dz, s); break;
    default: bwd_dispatch<F16>(relu, dy, dy2, y, x, mean, dz ? nullptr : coef, M, (int)C, g, p1, p2, gamma, invstd, dgamma, dbeta, k1, k2, k3, dx, dz, s); break;
  }
}

// Backward finalize over MANY [C][chunks] partials (the dgrad epilogue of the consuming conv
// writes one per 128 rows): one 256-thread block per channel, fp64 block reduce.

// BN+ReLU backward whose statistics (s1 = sum dz, s2 = sum dz*(x - mean), dz = dy * relu mask)
// were summed by the dgrad epilogue of the conv that consumed this BN's output: [C][chunks]
// partials -> finalize -> apply (mask recomputed from x and the forward coefficients).
void launch_bn_bwd_apply_pre(int dtype, const void* dy, const void* x, int64_t M, int64_t C, const float* mean,
                             const float* coef, const float* kbuf, void* dx, hipStream_t s, bool from_dz) {
  BnGeometry g = bn_geometry(M, C);
  const float* k1 = kbuf;
  const float* k2 = k1 + C;
  const float* k3 = k2 + C;
  dim3 bl(kBlock);
  ReduceCarry rc;
  const int ga = (g.apply_blocks * 2 > kBnBwdApplyMax ? kBnBwdApplyMax : g.apply_blocks * 2) +
                 take_attached_reduce(rc);
  if (from_dz) {  // dy is already the masked gradient dz (block-tail BN, ops/conv.py BNR)
    switch (dtype) {
      case 0: hipLaunchKernelGGL((bn_bwd_apply_kernel<F32, false, true, false>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
      case 1: hipLaunchKernelGGL((bn_bwd_apply_kernel<BF16, false, true, false>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
      default: hipLaunchKernelGGL((bn_bwd_apply_kernel<F16, false, true, false>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
    }
    return;
  }
  switch (dtype) {
    case 0: hipLaunchKernelGGL((bn_bwd_apply_kernel<F32, true, false, true>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
    case 1: hipLaunchKernelGGL((bn_bwd_apply_kernel<BF16, true, false, true>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
    default: hipLaunchKernelGGL((bn_bwd_apply_kernel<F16, true, false, true>), dim3(ga), bl, 0, s, dy, nullptr, x, mean, coef, k1, k2, k3, dx, M, (int)C, kBnReverse, rc); break;
  }
}

void launch_bn_bwd_from_partials(int dtype, const void* dy, const void* x, int64_t M, int64_t C, const float* gamma,
                                 const float* mean, const float* invstd, const float* coef, const float* p1,
                                 const float* p2, int chunks, float* dgamma, float* dbeta, void* dx, float* kbuf,
                                 hipStream_t s, bool from_dz) {
  BnGeometry g = bn_geometry(M, C);
  float* k1 = kbuf;
  float* k2 = k1 + C;
  float* k3 = k2 + C;
  dim3 bl(kBlock);
  launch_bn_bwd_fin(make_bn_bwd_fin(p1, p2, chunks, (int)C, M, gamma, invstd, dgamma, dbeta, k1, k2, k3, -1), s);
  launch_bn_bwd_apply_pre(dtype, dy, x, M, C, mean, coef, kbuf, dx, s, from_dz);
}

void launch_bn_apply_aff(int dtype, const void* x, const void* x2, void* y, int64_t M, int64_t C, const float* a,
                         const float* b, const float* a2, const float* b2, hipStream_t s, uint8_t* mask) {
  BnGeometry g = bn_geometry(M, C);
  dim3 gr(g.apply_blocks), bl(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL((bn_fwd_apply_kernel<F32, true, true, true>), gr, bl, 0, s, x, x2, y, a, b, M, (int)C, kBnReverse, a2, b2, mask); break;
    case 1: hipLaunchKernelGGL((bn_fwd_apply_kernel<BF16, true, true, true>), gr, bl, 0, s, x, x2, y, a, b, M, (int)C, kBnReverse, a2, b2, mask); break;
    default: hipLaunchKernelGGL((bn_fwd_apply_kernel<F16, true, true, true>), gr, bl, 0, s, x, x2, y, a, b, M, (int)C, kBnReverse, a2, b2, mask); break;
  }
}

// Two BatchNorms fed the same (masked) output gradient dz: the block tail (input x, statistics
// s1 = sum dz, s2 = sum dz*(x - mean)) and its downsample branch (input x2, s1 and s3 = sum
// dz*(x2 - mean2)), partials [C][chunks] from the consuming conv's dgrad epilogue.
void launch_bn2_bwd_from_partials(int dtype, const void* dz, const void* x, const void* x2, int64_t M, int64_t C,
                                  const float* gamma, const float* mean, const float* invstd, const float* gamma2,
                                  const float* mean2, const float* invstd2, const float* p1, const float* p2,
                                  const float* p3, int chunks, float* dgamma, float* dbeta, float* dgamma2,
                                  float* dbeta2, void* dx, void* dx2, float* kbuf, hipStream_t s) {
  BnGeometry g = bn_geometry(M, C);
  float* k = kbuf;          // [3C] tail
  float* j = kbuf + 3 * C;  // [3C] downsample
  dim3 bl(kBlock);
  const BnBwdFin f1 = make_bn_bwd_fin(p1, p2, chunks, (int)C, M, gamma, invstd, dgamma, dbeta, k, k + C, k + 2 * C, -1);
  const BnBwdFin f2 =
      make_bn_bwd_fin(p1, p3, chunks, (int)C, M, gamma2, invstd2, dgamma2, dbeta2, j, j + C, j + 2 * C, -1);
  if (!g_bn_skip_finalize)
    hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3((unsigned)(f1.blocks + f2.blocks)), dim3(kBlock), 0, s, f1, f2);
  dim3 ga(g.apply_blocks * 2 > kBnBwdApplyMax ? kBnBwdApplyMax : g.apply_blocks * 2);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(bn_bwd_apply2_kernel<F32>, ga, bl, 0, s, dz, x, x2, mean, mean2, k, j, dx, dx2, M, (int)C, kBnReverse); break;
    case 1: hipLaunchKernelGGL(bn_bwd_apply2_kernel<BF16>, ga, bl, 0, s, dz, x, x2, mean, mean2, k, j, dx, dx2, M, (int)C, kBnReverse); break;
    default: hipLaunchKernelGGL(bn_bwd_apply2_kernel<F16>, ga, bl, 0, s, dz, x, x2, mean, mean2, k, j, dx, dx2, M, (int)C, kBnReverse); break;
  }
}

int64_t bn_workspace_floats(int64_t M, int64_t C) {
  BnGeometry g = bn_geometry(M, C);
  return 2 * (int64_t)C * g.chunks + 3 * C;
}

}  // namespace dpt
