// Fused transformer-block elementwise kernels (ViT-B/16 under bf16 autocast) for gfx950.
//
// Why: in a stock ViT-B/16 step on MI355X (batch 128, bf16 autocast) about a third of the
// kernel time is not GEMM or attention but the HBM passes around them
// (profiles/vit_b16_breakdown.md): fp32 LayerNorm forward/backward + gamma/beta partial
// reductions, autocast casts of the LayerNorm outputs, fp32 residual adds (and their
// gradient accumulations), GELU forward/backward and bias-gradient column sums.  The
// encoder's residual stream is fp32 (the class-token concat promotes it); the GEMM
// operands are bf16.  These kernels collapse each block boundary into one pass:
//
//   ln_fwd     s = x + a + bias (fp32, a = the branch GEMM output WITHOUT its bias, bf16)
//              h = LayerNorm(s) * gamma + beta, written directly as bf16 (the next GEMM's
//              operand: no separate cast), per-row mean / rstd saved
//   ln_bwd     gx = gs + LN_backward(gh)  (fp32: the residual-stream gradient, in one pass),
//              ga = bf16(gx) (the branch GEMM's output gradient), and per-block partial
//              column sums of gh*xhat, gh, gx  ->  dgamma, dbeta, dbias (the branch bias)
//   gelu_fwd   h = gelu(u + bias) (exact erf GELU, nn.GELU's default), u = fc1 output w/o bias
//   gelu_bwd   gu = gh * gelu'(u + bias) and partial column sums of gu -> dbias
//   colsum     deterministic second-level reduction of the [n, D] partials
//
// Layout: activations are row-major [T = tokens, D]; D must be a multiple of 256
// (768 for ViT-B, 1024 ViT-L, 1280 ViT-H) for the LayerNorm kernels: one wave per row,
// each lane owning D/256 float4 column groups (coalesced 1 KiB per wave access), the row
// held in registers so mean and variance are exact two-pass values.  GELU kernels need
// F % 8 == 0 (16-byte vectors of 8 bf16).
#include <cmath>

#include "gelu.h"
#include "common.h"
#include "kernels.h"

namespace dpt {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// 16-bit activation codec: KIND 1 = bf16, 2 = fp16.
template <int KIND>
__device__ __forceinline__ float h2f(uint32_t h) {
  if (KIND == 1) return bf16_to_f32((uint16_t)h);
  return f16_to_f32((uint16_t)h);
}
template <int KIND>
__device__ __forceinline__ uint32_t f2h(float f) {
  if (KIND == 1) return f32_to_bf16(f);
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}
template <int KIND>
__device__ __forceinline__ void load4h(const uint16_t* p, float v[4]) {
  uint2 w = *reinterpret_cast<const uint2*>(p);
  v[0] = h2f<KIND>(w.x & 0xffff);
  v[1] = h2f<KIND>(w.x >> 16);
  v[2] = h2f<KIND>(w.y & 0xffff);
  v[3] = h2f<KIND>(w.y >> 16);
}
template <int KIND>
__device__ __forceinline__ void store4h(uint16_t* p, const float v[4]) {
  uint2 w;
  w.x = f2h<KIND>(v[0]) | (f2h<KIND>(v[1]) << 16);
  w.y = f2h<KIND>(v[2]) | (f2h<KIND>(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = w;
}
template <int KIND>
__device__ __forceinline__ void load8h(const uint16_t* p, float v[8]) {
  uint4 w = *reinterpret_cast<const uint4*>(p);
  uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = h2f<KIND>(u[k] & 0xffff);
    v[2 * k + 1] = h2f<KIND>(u[k] >> 16);
  }
}
template <int KIND>
__device__ __forceinline__ void store8h(uint16_t* p, const float v[8]) {
  uint4 w;
  w.x = f2h<KIND>(v[0]) | (f2h<KIND>(v[1]) << 16);
  w.y = f2h<KIND>(v[2]) | (f2h<KIND>(v[3]) << 16);
  w.z = f2h<KIND>(v[4]) | (f2h<KIND>(v[5]) << 16);
  w.w = f2h<KIND>(v[6]) | (f2h<KIND>(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = w;
}

// A per-column parameter (bias) of kind 0 fp32 / 1 bf16 / 2 fp16; nullptr reads as 0.
__device__ __forceinline__ float load_param(const void* p, int kind, int64_t i) {
  if (p == nullptr) return 0.f;
  if (kind == 0) return static_cast<const float*>(p)[i];
  const uint16_t h = static_cast<const uint16_t*>(p)[i];
  return kind == 1 ? bf16_to_f32(h) : f16_to_f32(h);
}

// ---- LayerNorm forward (+ residual add + branch bias) ----------------------------------------
// gamma / beta / bias are re-read per row (L1/L2 hits) instead of living in 36 registers per lane:
// 64 VGPRs instead of 82 puts 8 waves on a SIMD (the whole 2,048-block grid resident at once)
// instead of 5 (1,280 blocks, then a 60 %-full second round).
__device__ __forceinline__ void load4_param(const void* p, int kind, int64_t c0, float v[4]) {
  if (p == nullptr) {
    v[0] = v[1] = v[2] = v[3] = 0.f;
  } else if (kind == 0) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + c0);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else if (kind == 1) {
    load4h<1>(static_cast<const uint16_t*>(p) + c0, v);
  } else {
    load4h<2>(static_cast<const uint16_t*>(p) + c0, v);
  }
}

template <int VPL, int KIND, bool ADD>
__global__ __launch_bounds__(kBlock, 8) void ln_fwd_kernel(const float* __restrict__ x,
                                                        const uint16_t* __restrict__ a,
                                                        const void* __restrict__ bias, int bias_kind,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        float* __restrict__ s_out, uint16_t* __restrict__ h_out,
                                                        float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int64_t T, float eps) {
  constexpr int D = VPL * 256;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < T; row += (int64_t)gridDim.x * 4) {
    const int64_t base = row * D;
    float v[VPL][4];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const float4 q = *reinterpret_cast<const float4*>(x + base + (i * 64 + lane) * 4);
      v[i][0] = q.x; v[i][1] = q.y; v[i][2] = q.z; v[i][3] = q.w;
    }
    if (ADD) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float w[4], bs[4];
        load4h<KIND>(a + base + (i * 64 + lane) * 4, w);
        load4_param(bias, bias_kind, (i * 64 + lane) * 4, bs);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] += w[j] + bs[j];
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += v[i][j];
    const float mean = wave_sum(sum) * (1.f / D);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        sq += d * d;
      }
    const float rstd = rsqrtf(wave_sum(sq) * (1.f / D) + eps);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c0 = (i * 64 + lane) * 4;
      const int64_t off = base + c0;
      if (ADD) *reinterpret_cast<float4*>(s_out + off) = make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
      float gm[4] = {1.f, 1.f, 1.f, 1.f}, bt[4] = {0.f, 0.f, 0.f, 0.f};
      if (gamma) load4_param(gamma, 0, c0, gm);
      if (beta) load4_param(beta, 0, c0, bt);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gm[j] + bt[j];
      store4h<KIND>(h_out + off, o);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// ---- LayerNorm backward (+ residual-gradient add, branch-gradient cast, param partials) -----
template <int VPL>
__device__ __forceinline__ void block_colsum_store(float (&acc)[VPL][4], float* red, float* out, int lane,
                                                   int wave) {
  constexpr int D = VPL * 256;
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wave * D + (i * 64 + lane) * 4 + j] = acc[i][j];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += kBlock) out[c] = (red[c] + red[D + c]) + (red[2 * D + c] + red[3 * D + c]);
  __syncthreads();
}

template <int VPL, int KIND, bool HAS_GS, bool WRITE_GA>
__global__ __launch_bounds__(kBlock) void ln_bwd_kernel(const float* __restrict__ gs,
                                                        const uint16_t* __restrict__ gh,
                                                        const float* __restrict__ s,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma, float* __restrict__ gx,
                                                        uint16_t* __restrict__ ga, float* __restrict__ part,
                                                        int64_t T, int64_t rows_per_block) {
  constexpr int D = VPL * 256;
  __shared__ float red[4 * D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm[VPL][4], ag[VPL][4], ab[VPL][4], ax[VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      gm[i][j] = gamma ? gamma[(i * 64 + lane) * 4 + j] : 1.f;
      ag[i][j] = ab[i][j] = ax[i][j] = 0.f;
    }
  const int64_t row0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t row1 = min(row0 + rows_per_block, T);
  for (int64_t row = row0 + wave; row < row1; row += 4) {
    const int64_t base = row * D;
    const float mu = mean[row], rs = rstd[row];
    float xh[VPL][4], g[VPL][4], d[VPL][4];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int64_t off = base + (i * 64 + lane) * 4;
      const float4 q = *reinterpret_cast<const float4*>(s + off);
      xh[i][0] = q.x; xh[i][1] = q.y; xh[i][2] = q.z; xh[i][3] = q.w;
      load4h<KIND>(gh + off, d[i]);
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[i][j] = (xh[i][j] - mu) * rs;
        g[i][j] = d[i][j] * gm[i][j];
        s1 += g[i][j];
        s2 += g[i][j] * xh[i][j];
        ag[i][j] += d[i][j] * xh[i][j];
        ab[i][j] += d[i][j];
      }
    const float c1 = wave_sum(s1) * (1.f / D), c2 = wave_sum(s2) * (1.f / D);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int64_t off = base + (i * 64 + lane) * 4;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] - c1 - xh[i][j] * c2);
      if (HAS_GS) {
        const float4 q = *reinterpret_cast<const float4*>(gs + off);
        o[0] += q.x; o[1] += q.y; o[2] += q.z; o[3] += q.w;
      }
      *reinterpret_cast<float4*>(gx + off) = make_float4(o[0], o[1], o[2], o[3]);
      if (WRITE_GA) store4h<KIND>(ga + off, o);
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[i][j] += o[j];
    }
  }
  // part layout: [3][gridDim.x][D] = dgamma, dbeta, dbias partials
  const int64_t nb = gridDim.x;
  block_colsum_store<VPL>(ag, red, part + (0 * nb + blockIdx.x) * D, lane, wave);
  block_colsum_store<VPL>(ab, red, part + (1 * nb + blockIdx.x) * D, lane, wave);
  if (WRITE_GA) block_colsum_store<VPL>(ax, red, part + (2 * nb + blockIdx.x) * D, lane, wave);
}

// ---- bias + exact (erf) GELU ------------------------------------------------------------------
// erf_and_gauss / gelu_f / gelu_grad: gelu.h (shared with the conv DGELU epilogue)

// Column-stationary layout for both GELU passes: grid (ceil(F/8 / 128), chunks) of 128-thread
// blocks; a thread owns one 8-column group (its 8 bias values stay in registers) and walks a
// chunk of rows with 4 rows (8 x 16-byte accesses) in flight.
constexpr int kGeluRows = 4;

template <int KIND>
__global__ __launch_bounds__(128) void gelu_fwd_kernel(const uint16_t* __restrict__ u,
                                                       const void* __restrict__ bias, int bias_kind,
                                                       uint16_t* __restrict__ h, int64_t T, int F,
                                                       int64_t rows_per_chunk) {
  const int cg = blockIdx.x * 128 + threadIdx.x;
  if (cg * 8 >= F) return;
  float b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) b[k] = load_param(bias, bias_kind, cg * 8 + k);
  const int64_t row0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t row1 = min(row0 + rows_per_chunk, T);
  int64_t r = row0;
  for (; r + kGeluRows <= row1; r += kGeluRows) {
    float z[kGeluRows][8];
#pragma unroll
    for (int q = 0; q < kGeluRows; ++q) load8h<KIND>(u + (r + q) * F + cg * 8, z[q]);
#pragma unroll
    for (int q = 0; q < kGeluRows; ++q) {
#pragma unroll
      for (int k = 0; k < 8; ++k) z[q][k] = gelu_f(z[q][k] + b[k]);
      store8h<KIND>(h + (r + q) * F + cg * 8, z[q]);
    }
  }
  for (; r < row1; ++r) {
    float z[8];
    load8h<KIND>(u + r * F + cg * 8, z);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = gelu_f(z[k] + b[k]);
    store8h<KIND>(h + r * F + cg * 8, z);
  }
}

// GELU = false: plain column sums of gh (a Linear's bias gradient), nothing written but part.
template <int KIND, bool GELU>
__global__ __launch_bounds__(128) void gelu_bwd_kernel(const uint16_t* __restrict__ gh,
                                                       const uint16_t* __restrict__ u,
                                                       const void* __restrict__ bias, int bias_kind,
                                                       uint16_t* __restrict__ gu, float* __restrict__ part,
                                                       int64_t T, int F, int64_t rows_per_chunk) {
  const int cg = blockIdx.x * 128 + threadIdx.x;
  if (cg * 8 >= F) return;
  float b[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    b[k] = load_param(bias, bias_kind, cg * 8 + k);
    acc[k] = 0.f;
  }
  const int64_t row0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t row1 = min(row0 + rows_per_chunk, T);
  int64_t r = row0;
  for (; r + kGeluRows <= row1; r += kGeluRows) {
    float g[kGeluRows][8], z[kGeluRows][8];
#pragma unroll
    for (int q = 0; q < kGeluRows; ++q) {
      load8h<KIND>(gh + (r + q) * F + cg * 8, g[q]);
      if (GELU) load8h<KIND>(u + (r + q) * F + cg * 8, z[q]);
    }
#pragma unroll
    for (int q = 0; q < kGeluRows; ++q) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (GELU) g[q][k] *= gelu_grad(z[q][k] + b[k]);
        acc[k] += g[q][k];
      }
      if (GELU) store8h<KIND>(gu + (r + q) * F + cg * 8, g[q]);
    }
  }
  for (; r < row1; ++r) {
    float g[8], z[8];
    load8h<KIND>(gh + r * F + cg * 8, g);
    if (GELU) load8h<KIND>(u + r * F + cg * 8, z);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (GELU) g[k] *= gelu_grad(z[k] + b[k]);
      acc[k] += g[k];
    }
    if (GELU) store8h<KIND>(gu + r * F + cg * 8, g);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[(int64_t)blockIdx.y * F + cg * 8 + k] = acc[k];
}

// ---- 16-bit strided row copy (attention head split/merge) ------------------------------------
// dst[i0,i1,i2,i3,:L] = src[i0,i1,i2,i3,:L]; the L-element rows are contiguous in both, every
// row start is 16-byte aligned (host-checked); one 16-byte vector per thread iteration.
struct Rows4 {
  int n[4];
  int64_t ss[4], ds[4];
};

__global__ __launch_bounds__(kBlock) void rows_copy16_kernel(const uint16_t* __restrict__ src,
                                                             uint16_t* __restrict__ dst, Rows4 g, int L) {
  const int vpr = L >> 3;
  const int64_t total = (int64_t)g.n[0] * g.n[1] * g.n[2] * g.n[3] * vpr;
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < total; v += (int64_t)gridDim.x * kBlock) {
    unsigned row = (unsigned)(v / vpr);
    const int k = (int)(v - (int64_t)row * vpr);
    const unsigned i3 = row % (unsigned)g.n[3];
    row /= (unsigned)g.n[3];
    const unsigned i2 = row % (unsigned)g.n[2];
    row /= (unsigned)g.n[2];
    const unsigned i1 = row % (unsigned)g.n[1];
    const unsigned i0 = row / (unsigned)g.n[1];
    const int64_t so = i0 * g.ss[0] + i1 * g.ss[1] + i2 * g.ss[2] + i3 * g.ss[3] + k * 8;
    const int64_t d0 = i0 * g.ds[0] + i1 * g.ds[1] + i2 * g.ds[2] + i3 * g.ds[3] + k * 8;
    *reinterpret_cast<uint4*>(dst + d0) = *reinterpret_cast<const uint4*>(src + so);
  }
}

// ---- deterministic column sums of [n, D] partials -> out (kind 0 f32 / 1 bf16 / 2 f16) -----
// grid (ceil(D/64), sets), 1024 threads: 16 waves split the n rows (4 loads in flight each),
// lane = column; fp64 accumulation, fixed combine order.  Set s reads part + s*set_stride.
struct ColsumOut {
  void* out[3];
  int kind[3];
};

__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int64_t n, int64_t D,
                                                      int64_t set_stride, ColsumOut o) {
  __shared__ double red[16][64];
  void* out = o.out[blockIdx.y];
  if (out == nullptr) return;  // whole block: uniform
  const float* p = part + blockIdx.y * set_stride;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  double acc = 0.0;
  if (c < D) {
    int64_t r = wave;
    for (; r + 48 < n; r += 64) {
      const float a0 = p[r * D + c], a1 = p[(r + 16) * D + c];
      const float a2 = p[(r + 32) * D + c], a3 = p[(r + 48) * D + c];
      acc += ((double)a0 + (double)a1) + ((double)a2 + (double)a3);
    }
    for (; r < n; r += 16) acc += (double)p[r * D + c];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < D) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    const float v = (float)t;
    const int kind = o.kind[blockIdx.y];
    if (kind == 0) static_cast<float*>(out)[c] = v;
    else if (kind == 1) static_cast<uint16_t*>(out)[c] = f32_to_bf16(v);
    else static_cast<uint16_t*>(out)[c] = __builtin_bit_cast(uint16_t, (_Float16)v);
  }
}

static void launch_colsum(const float* part, int64_t n, int64_t D, int sets, void* o0, int k0, void* o1, int k1,
                          void* o2, int k2, hipStream_t s) {
  ColsumOut o;
  o.out[0] = o0; o.out[1] = o1; o.out[2] = o2;
  o.kind[0] = k0; o.kind[1] = k1; o.kind[2] = k2;
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)sets), dim3(1024), 0, s, part, n, D,
                     n * D, o);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
bool ln_supported(int64_t D) { return D % 256 == 0 && D >= 256 && D <= 2048; }

static int ln_grid(int64_t T) {
  int64_t g = (T + 3) / 4;
  return (int)(g < 1 ? 1 : (g > kMaxBlocks ? kMaxBlocks : g));
}

template <int VPL, int KIND>
static void ln_fwd_vpl(const float* x, const uint16_t* a, const void* bias, int bias_kind, const float* gamma,
                       const float* beta, float* s_out, uint16_t* h_out, float* mean, float* rstd, int64_t T,
                       float eps, hipStream_t st) {
  dim3 gr(ln_grid(T)), bl(kBlock);
  if (a) hipLaunchKernelGGL((ln_fwd_kernel<VPL, KIND, true>), gr, bl, 0, st, x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps);
  else hipLaunchKernelGGL((ln_fwd_kernel<VPL, KIND, false>), gr, bl, 0, st, x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps);
}

template <int KIND>
static void ln_fwd_kind(int64_t D, const float* x, const uint16_t* a, const void* bias, int bias_kind,
                        const float* gamma, const float* beta, float* s_out, uint16_t* h_out, float* mean,
                        float* rstd, int64_t T, float eps, hipStream_t st) {
  switch (D / 256) {
    case 1: ln_fwd_vpl<1, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 2: ln_fwd_vpl<2, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 3: ln_fwd_vpl<3, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 4: ln_fwd_vpl<4, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 5: ln_fwd_vpl<5, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 6: ln_fwd_vpl<6, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    case 7: ln_fwd_vpl<7, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
    default: ln_fwd_vpl<8, KIND>(x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, st); break;
  }
}

void launch_ln_fwd(int kind, const float* x, const uint16_t* a, const void* bias, int bias_kind, const float* gamma,
                   const float* beta, float* s_out, uint16_t* h_out, float* mean, float* rstd, int64_t T, int64_t D,
                   float eps, hipStream_t s) {
  if (kind == 1) ln_fwd_kind<1>(D, x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, s);
  else ln_fwd_kind<2>(D, x, a, bias, bias_kind, gamma, beta, s_out, h_out, mean, rstd, T, eps, s);
}

int ln_bwd_blocks(int64_t T) {
  // >= 16 rows per block (4 per wave) so the [3][blocks][D] partials stay small next to the
  // activations, <= 1024 blocks (16 waves per CU) for latency hiding.
  int64_t b = T / 16;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

template <int VPL, int KIND>
static void ln_bwd_vpl(const float* gs, const uint16_t* gh, const float* sv, const float* mean, const float* rstd,
                       const float* gamma, float* gx, uint16_t* ga, float* part, int64_t T, hipStream_t st) {
  const int nb = ln_bwd_blocks(T);
  const int64_t rpb = (T + nb - 1) / nb;
  dim3 gr(nb), bl(kBlock);
  if (gs && ga) hipLaunchKernelGGL((ln_bwd_kernel<VPL, KIND, true, true>), gr, bl, 0, st, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, rpb);
  else if (gs) hipLaunchKernelGGL((ln_bwd_kernel<VPL, KIND, true, false>), gr, bl, 0, st, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, rpb);
  else if (ga) hipLaunchKernelGGL((ln_bwd_kernel<VPL, KIND, false, true>), gr, bl, 0, st, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, rpb);
  else hipLaunchKernelGGL((ln_bwd_kernel<VPL, KIND, false, false>), gr, bl, 0, st, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, rpb);
}

template <int KIND>
static void ln_bwd_kind(int64_t D, const float* gs, const uint16_t* gh, const float* sv, const float* mean,
                        const float* rstd, const float* gamma, float* gx, uint16_t* ga, float* part, int64_t T,
                        hipStream_t st) {
  switch (D / 256) {
    case 1: ln_bwd_vpl<1, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 2: ln_bwd_vpl<2, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 3: ln_bwd_vpl<3, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 4: ln_bwd_vpl<4, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 5: ln_bwd_vpl<5, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 6: ln_bwd_vpl<6, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    case 7: ln_bwd_vpl<7, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
    default: ln_bwd_vpl<8, KIND>(gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, st); break;
  }
}

void launch_ln_bwd(int kind, const float* gs, const uint16_t* gh, const float* sv, const float* mean,
                   const float* rstd, const float* gamma, float* gx, uint16_t* ga, float* part, float* dgamma,
                   float* dbeta, void* dbias, int dbias_kind, int64_t T, int64_t D, hipStream_t s) {
  if (kind == 1) ln_bwd_kind<1>(D, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, s);
  else ln_bwd_kind<2>(D, gs, gh, sv, mean, rstd, gamma, gx, ga, part, T, s);
  const int64_t nb = ln_bwd_blocks(T);
  void* db = (dbias && ga) ? dbias : nullptr;
  if (dgamma || dbeta || db)
    launch_colsum(part, nb, D, db ? 3 : 2, dgamma, 0, dbeta, 0, db, dbias_kind, s);
}

// 2-wave blocks per CU of the GELU passes (bench/gelu_ab.py, ViT-B/16's [25216, 3072] at batch
// 128): the forward 73 -> 58 us going 6 -> 12 per CU (more 16-byte rows in flight), the backward
// best at 8 (105 vs 113 us; its per-chunk column-sum partials grow with the chunk count).
// A/B knob: vit_set_gelu_blocks_per_cu (0 = these defaults).
constexpr int kGeluFwdBlocksPerCu = 12, kGeluBwdBlocksPerCu = 8;
static int g_gelu_blocks_per_cu = 0;
void vit_set_gelu_blocks_per_cu(int n) { g_gelu_blocks_per_cu = n > 0 ? n : 0; }

static int gelu_chunks(int64_t T, int64_t F, int blocks_per_cu) {
  const int64_t colblocks = (F / 8 + 127) / 128;
  const int per_cu = g_gelu_blocks_per_cu > 0 ? g_gelu_blocks_per_cu : blocks_per_cu;
  int64_t c = (256 * (int64_t)per_cu) / (colblocks > 0 ? colblocks : 1);
  if (c > T / 8) c = T / 8;
  return (int)(c < 1 ? 1 : c);
}

int gelu_bwd_chunks(int64_t T, int64_t F) {
  // (F/8/128 column blocks) x chunks of 2-wave blocks
  const int64_t colblocks = (F / 8 + 127) / 128;
  int64_t c = (256 * (int64_t)(g_gelu_blocks_per_cu > 0 ? g_gelu_blocks_per_cu : kGeluBwdBlocksPerCu)) /
              (colblocks > 0 ? colblocks : 1);
  if (c > T / 8) c = T / 8;
  return (int)(c < 1 ? 1 : c);
}

void launch_gelu_fwd(int kind, const uint16_t* u, const void* bias, int bias_kind, uint16_t* h, int64_t T, int64_t F,
                     hipStream_t s) {
  const int chunks = gelu_chunks(T, F, kGeluFwdBlocksPerCu);
  const int64_t rpc = (T + chunks - 1) / chunks;
  dim3 gr((unsigned)((F / 8 + 127) / 128), (unsigned)chunks), bl(128);
  if (kind == 1) hipLaunchKernelGGL(gelu_fwd_kernel<1>, gr, bl, 0, s, u, bias, bias_kind, h, T, (int)F, rpc);
  else hipLaunchKernelGGL(gelu_fwd_kernel<2>, gr, bl, 0, s, u, bias, bias_kind, h, T, (int)F, rpc);
}

void launch_gelu_bwd(int kind, const uint16_t* gh, const uint16_t* u, const void* bias, int bias_kind, uint16_t* gu,
                     float* part, void* dbias, int dbias_kind, int64_t T, int64_t F, hipStream_t s) {
  const int chunks = gelu_bwd_chunks(T, F);
  const int64_t rpc = (T + chunks - 1) / chunks;
  dim3 gr((unsigned)((F / 8 + 127) / 128), (unsigned)chunks), bl(128);
  if (kind == 1) hipLaunchKernelGGL((gelu_bwd_kernel<1, true>), gr, bl, 0, s, gh, u, bias, bias_kind, gu, part, T, (int)F, rpc);
  else hipLaunchKernelGGL((gelu_bwd_kernel<2, true>), gr, bl, 0, s, gh, u, bias, bias_kind, gu, part, T, (int)F, rpc);
  if (dbias) launch_colsum(part, chunks, F, 1, dbias, dbias_kind, nullptr, 0, nullptr, 0, s);
}

void launch_bias_grad16(int kind, const uint16_t* gy, float* part, void* dbias, int dbias_kind, int64_t T, int64_t F,
                        hipStream_t s) {
  const int chunks = gelu_bwd_chunks(T, F);
  const int64_t rpc = (T + chunks - 1) / chunks;
  dim3 gr((unsigned)((F / 8 + 127) / 128), (unsigned)chunks), bl(128);
  if (kind == 1) hipLaunchKernelGGL((gelu_bwd_kernel<1, false>), gr, bl, 0, s, gy, nullptr, nullptr, 0, nullptr, part, T, (int)F, rpc);
  else hipLaunchKernelGGL((gelu_bwd_kernel<2, false>), gr, bl, 0, s, gy, nullptr, nullptr, 0, nullptr, part, T, (int)F, rpc);
  launch_colsum(part, chunks, F, 1, dbias, dbias_kind, nullptr, 0, nullptr, 0, s);
}

// out[i] = sum_s part[s][i]  (split-K partials -> the weight gradient, fp32 or 16-bit)
__global__ __launch_bounds__(kBlock) void sum_partials_kernel(const float4* __restrict__ part, int64_t n4, int S,
                                                              void* __restrict__ out, int out_kind) {
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n4; v += (int64_t)gridDim.x * kBlock) {
    float4 a = part[v];
    for (int q = 1; q < S; ++q) {
      const float4 b = part[q * n4 + v];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (out_kind == 0) {
      static_cast<float4*>(out)[v] = a;
    } else {
      const float f[4] = {a.x, a.y, a.z, a.w};
      if (out_kind == 1) store4h<1>(static_cast<uint16_t*>(out) + v * 4, f);
      else store4h<2>(static_cast<uint16_t*>(out) + v * 4, f);
    }
  }
}

void launch_colsum_rows(const float* part, int64_t n, int64_t D, void* out, int out_kind, hipStream_t s) {
  launch_colsum(part, n, D, 1, out, out_kind, nullptr, 0, nullptr, 0, s);
}

void launch_sum_partials(const float* part, int64_t n, int S, void* out, int out_kind, hipStream_t s) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(sum_partials_kernel, dim3(grid_for(n4, 2)), dim3(kBlock), 0, s,
                     reinterpret_cast<const float4*>(part), n4, S, out, out_kind);
}

void launch_rows_copy16(const uint16_t* src, uint16_t* dst, const int n[4], const int64_t ss[4], const int64_t ds[4],
                        int L, hipStream_t s) {
  Rows4 g;
  for (int i = 0; i < 4; ++i) {
    g.n[i] = n[i];
    g.ss[i] = ss[i];
    g.ds[i] = ds[i];
  }
  const int64_t total = (int64_t)n[0] * n[1] * n[2] * n[3] * (L / 8);
  if (total == 0) return;
  hipLaunchKernelGGL(rows_copy16_kernel, dim3(grid_for(total, 2)), dim3(kBlock), 0, s, src, dst, g, L);
}

}  // namespace dpt
