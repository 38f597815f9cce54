// Work carried in the tail of another kernel's grid ("carry" blocks).
//
// A few kernels of a training step are tiny, latency-bound and sit between two big ones in the
// same stream: the split-K reduce of a backward-weight and the BatchNorm backward finalize
// (~6 us each, mostly launch and ramp, 100+ per ResNet-50 step).  Their inputs are complete
// before the NEXT big kernel of the stream starts, so that kernel can run them: its launch
// appends the carried work's blocks to its grid, and the carry blocks (the highest block ids,
// dispatched last) run as the big kernel's tail drains.  Stream order is all the
// synchronisation needed - nothing crosses blocks of one grid.
//
//   ReduceCarry  sum of a backward-weight's split-K partials -> dw (carried by the conv's
//                backward-data launch, or by the BatchNorm backward apply)
//   BnBwdFin     BatchNorm backward finalize: partials (s1, s2) -> dgamma, dbeta and the dx
//                coefficients k1, k2, k3 (carried by the conv's backward-weight launch)
#pragma once

#include "common.h"

namespace dpt {

struct ReduceCarry {
  const float4* part = nullptr;  // [splits][n4] float4 partials
  void* out = nullptr;           // n4 float4 -> kind 0 f32 / 1 bf16 / 2 f16
  int64_t n4 = 0;
  int splits = 0, kind = 0;
  int blocks = 0;  // carry blocks appended to the carrier's grid (0: none)
  int ph = 1;      // phases per block (splits >= 16: 16, >= 4: 4, else 1)
};

// out[v] = sum_s part[s][v] for the float4s v of block `bid`: PH phases per block split the S
// loop, `red` (kBlock float4s of LDS) combines them.
template <int PH>
__device__ __forceinline__ void wgrad_reduce_body(const float4* __restrict__ part, int64_t n4, int S,
                                                  void* __restrict__ out, int out_kind, int bid, float4* red) {
  constexpr int OUT = kBlock / PH;
  const int o = threadIdx.x % OUT, ph = threadIdx.x / OUT;
  const int64_t v = (int64_t)bid * OUT + o;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (v < n4) {
    int q = ph;
    for (; q + 3 * PH < S; q += 4 * PH) {
      const float4 b0 = part[(int64_t)q * n4 + v], b1 = part[(int64_t)(q + PH) * n4 + v];
      const float4 b2 = part[(int64_t)(q + 2 * PH) * n4 + v], b3 = part[(int64_t)(q + 3 * PH) * n4 + v];
      a.x += (b0.x + b1.x) + (b2.x + b3.x);
      a.y += (b0.y + b1.y) + (b2.y + b3.y);
      a.z += (b0.z + b1.z) + (b2.z + b3.z);
      a.w += (b0.w + b1.w) + (b2.w + b3.w);
    }
    for (; q < S; q += PH) {
      const float4 b = part[(int64_t)q * n4 + v];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  red[threadIdx.x] = a;
  __syncthreads();
  if (ph != 0 || v >= n4) return;
#pragma unroll
  for (int k = 1; k < PH; ++k) {
    const float4 b = red[k * OUT + o];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  if (out_kind == 0) {
    static_cast<float4*>(out)[v] = a;
  } else if (out_kind == 2) {  // fp16
    const _Float16 h[4] = {(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w};
    uint2 w;
    w.x = (uint32_t)__builtin_bit_cast(uint16_t, h[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[1]) << 16);
    w.y = (uint32_t)__builtin_bit_cast(uint16_t, h[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[3]) << 16);
    static_cast<uint2*>(out)[v] = w;
  } else {
    uint2 w;
    w.x = (uint32_t)f32_to_bf16(a.x) | ((uint32_t)f32_to_bf16(a.y) << 16);
    w.y = (uint32_t)f32_to_bf16(a.z) | ((uint32_t)f32_to_bf16(a.w) << 16);
    static_cast<uint2*>(out)[v] = w;
  }
}

__device__ __forceinline__ void carry_reduce(const ReduceCarry& r, int bid, void* lds) {
  float4* red = static_cast<float4*>(lds);
  if (r.ph == 16) wgrad_reduce_body<16>(r.part, r.n4, r.splits, r.out, r.kind, bid, red);
  else if (r.ph == 4) wgrad_reduce_body<4>(r.part, r.n4, r.splits, r.out, r.kind, bid, red);
  else wgrad_reduce_body<1>(r.part, r.n4, r.splits, r.out, r.kind, bid, red);
}

// Sum `chunks` partials of channel c with 32 lanes (one half-wave) in fp64.  Eight
// independent loads in flight per lane: the partials are L2-resident, so this loop is
// latency-bound, not bandwidth-bound.
__device__ __forceinline__ void half_wave_sum2(const float* p1, const float* p2, int64_t c, int chunks,
                                               int part, double& s1, double& s2) {
  constexpr int U = 8;
  double a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { a[u] = 0.0; b[u] = 0.0; }
  const float* q1 = p1 + c * chunks;
  const float* q2 = p2 + c * chunks;
  int k = part;
  for (; k + 32 * (U - 1) < chunks; k += 32 * U) {
    float x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { x[u] = q1[k + 32 * u]; y[u] = q2[k + 32 * u]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { a[u] += (double)x[u]; b[u] += (double)y[u]; }
  }
  for (; k < chunks; k += 32) { a[0] += (double)q1[k]; b[0] += (double)q2[k]; }
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) { s1 += a[u]; s2 += b[u]; }
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
}

// Sum one row of `chunks` partials with a whole block in fp64 (8 loads of each row in flight
// per thread; 16 measured slower: 21 -> 25 us for the stem's 25,088 partials per channel, 6.4 ->
// 7.2 us averaged over the step's wide finalizes); the result is reduced within each wave (lane 0
// of every wave holds its wave's sum).
template <int NT = kBlock>
__device__ __forceinline__ void block_row_sum2(const float* __restrict__ q1, const float* __restrict__ q2,
                                               int chunks, double& s, double& q) {
  constexpr int U = 8;
  double a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { a[u] = 0.0; b[u] = 0.0; }
  int k = threadIdx.x;
  for (; k + (U - 1) * NT < chunks; k += U * NT) {
    float x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { x[u] = q1[k + u * NT]; y[u] = q2[k + u * NT]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { a[u] += (double)x[u]; b[u] += (double)y[u]; }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int kk = k + u * NT;
    if (kk < chunks) { a[u] += (double)q1[kk]; b[u] += (double)q2[kk]; }
  }
  s = 0.0;
  q = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) { s += a[u]; q += b[u]; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    q += __shfl_xor(q, off, 64);
  }
}

// BatchNorm backward finalize: s1 = sum dz, s2 = sum dz*(x - mean) from [C][chunks] partials ->
// dgamma = s2*invstd, dbeta = s1, dx = k1*dz + k2*(x - mean) + k3 with k1 = gamma*invstd,
// k2 = -k1*invstd^2*s2/M, k3 = -k1*s1/M (fp64 sums).  wide: one block per channel (many
// partials), else one half-wave per channel (8 channels per block).
struct BnBwdFin {
  const float* p1 = nullptr;
  const float* p2 = nullptr;
  int chunks = 0, C = 0;
  int64_t M = 0;
  const float* gamma = nullptr;  // nullptr: 1
  const float* invstd = nullptr;
  float* dgamma = nullptr;  // optional
  float* dbeta = nullptr;   // optional
  float* k1 = nullptr;
  float* k2 = nullptr;
  float* k3 = nullptr;
  int wide = 0;
  int blocks = 0;  // carry blocks (0: none)
};

__host__ __device__ inline int bn_bwd_fin_wide(int chunks) { return chunks > 256 ? 1 : 0; }
// (bn_kernels.hip) wide < 0: by chunk count
BnBwdFin make_bn_bwd_fin(const float* p1, const float* p2, int chunks, int C, int64_t M, const float* gamma,
                         const float* invstd, float* dgamma, float* dbeta, float* k1, float* k2, float* k3,
                         int wide);
__host__ __device__ inline int bn_bwd_fin_blocks(int C, int wide) { return wide ? C : (C + 7) / 8; }

__device__ __forceinline__ void bn_bwd_fin_store(const BnBwdFin& f, int64_t c, double s1, double s2) {
  const double is = (double)f.invstd[c];
  const double g = f.gamma ? (double)f.gamma[c] : 1.0;
  if (f.dgamma) f.dgamma[c] = (float)(s2 * is);
  if (f.dbeta) f.dbeta[c] = (float)s1;
  const double a = g * is;
  f.k1[c] = (float)a;
  f.k2[c] = (float)(-a * is * is * s2 / (double)f.M);
  f.k3[c] = (float)(-a * s1 / (double)f.M);
}

// Block `bid` of the finalize (NT threads - wide only, kBlock otherwise; lds: >= NT bytes).
template <int NT = kBlock>
__device__ __forceinline__ void bn_bwd_finalize_block(const BnBwdFin& f, int bid, void* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (f.wide) {
    double* red = static_cast<double*>(lds);  // [2][NT / 64]
    const int c = bid;
    double s1, s2;
    block_row_sum2<NT>(f.p1 + (int64_t)c * f.chunks, f.p2 + (int64_t)c * f.chunks, f.chunks, s1, s2);
    if (lane == 0) { red[wave] = s1; red[NT / 64 + wave] = s2; }
    __syncthreads();
    if (threadIdx.x != 0) return;
    s1 = 0.0;
    s2 = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) { s1 += red[w]; s2 += red[NT / 64 + w]; }
    bn_bwd_fin_store(f, c, s1, s2);
  } else if constexpr (NT == kBlock) {
    const int64_t c = (int64_t)bid * 8 + wave * 2 + (lane >> 5);
    const int part = lane & 31;
    if (c >= f.C) return;
    double s1, s2;
    half_wave_sum2(f.p1, f.p2, c, f.chunks, part, s1, s2);
    if (part != 0) return;
    bn_bwd_fin_store(f, c, s1, s2);
  }
}

}  // namespace dpt
