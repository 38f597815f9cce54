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
template <int VPL, int KIND, bool ADD>
__global__ __launch_bounds__(kBlock) void ln_fwd_kernel(const float* __restrict__ x,
                                                        const uint16_t* __restrict__ a,
                                                        const void* __restrict__ bias, int bias_kind,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        float* __restrict__ s_out, uint16_t* __restrict__ h_out,
                                                        float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int64_t T, float eps) {
  constexpr int D = VPL * 256;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm[VPL][4], bt[VPL][4], bs[VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = (i * 64 + lane) * 4 + j;
      gm[i][j] = gamma ? gamma[c] : 1.f;
      bt[i][j] = beta ? beta[c] : 0.f;
      bs[i][j] = ADD ? load_param(bias, bias_kind, c) : 0.f;
    }
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
        float w[4];
        load4h<KIND>(a + base + (i * 64 + lane) * 4, w);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] += w[j] + bs[i][j];
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
      const int64_t off = base + (i * 64 + lane) * 4;
      if (ADD) *reinterpret_cast<float4*>(s_out + off) = make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gm[i][j] + bt[i][j];
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

// ---- bias + exact GELU ----------------------------------------------------------------------
__device__ __forceinline__ float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float z) {
  const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
  const float pdf = expf(-0.5f * z * z) * 0.39894228040143268f;
  return cdf + z * pdf;
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void gelu_fwd_kernel(const uint16_t* __restrict__ u,
                                                          const void* __restrict__ bias, int bias_kind,
                                                          uint16_t* __restrict__ h, int64_t n8, int F) {
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n8; v += (int64_t)gridDim.x * kBlock) {
    const int c0 = (int)((v * 8) % F);
    float z[8];
    load8h<KIND>(u + v * 8, z);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = gelu_f(z[k] + load_param(bias, bias_kind, c0 + k));
    store8h<KIND>(h + v * 8, z);
  }
}

// grid (ceil(F/8 / 128), chunks); 128-thread blocks; thread = one 8-column group over a row chunk
template <int KIND>
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
  for (; r + 1 < row1; r += 2) {  // two rows in flight
    float g0[8], z0[8], g1[8], z1[8];
    const int64_t o0 = r * F + cg * 8, o1 = o0 + F;
    load8h<KIND>(gh + o0, g0);
    load8h<KIND>(u + o0, z0);
    load8h<KIND>(gh + o1, g1);
    load8h<KIND>(u + o1, z1);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g0[k] *= gelu_grad(z0[k] + b[k]);
      g1[k] *= gelu_grad(z1[k] + b[k]);
      acc[k] += g0[k] + g1[k];
    }
    store8h<KIND>(gu + o0, g0);
    store8h<KIND>(gu + o1, g1);
  }
  if (r < row1) {
    float g0[8], z0[8];
    const int64_t o0 = r * F + cg * 8;
    load8h<KIND>(gh + o0, g0);
    load8h<KIND>(u + o0, z0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g0[k] *= gelu_grad(z0[k] + b[k]);
      acc[k] += g0[k];
    }
    store8h<KIND>(gu + o0, g0);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[(int64_t)blockIdx.y * F + cg * 8 + k] = acc[k];
}

// ---- deterministic column sums of [n, D] partials -> out (kind 0 f32 / 1 bf16 / 2 f16) -----
// grid (ceil(D/64)), 256 threads: 4 waves split the n rows, lane = column; fp64 accumulation.
__global__ __launch_bounds__(kBlock) void colsum_kernel(const float* __restrict__ part, int64_t n, int64_t D,
                                                        void* __restrict__ out, int out_kind) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  double acc = 0.0;
  if (c < D) {
    int64_t r = wave;
    for (; r + 12 < n; r += 16) {
      const float a0 = part[r * D + c], a1 = part[(r + 4) * D + c];
      const float a2 = part[(r + 8) * D + c], a3 = part[(r + 12) * D + c];
      acc += ((double)a0 + (double)a1) + ((double)a2 + (double)a3);
    }
    for (; r < n; r += 4) acc += (double)part[r * D + c];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < D) {
    const float v = (float)((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]));
    if (out_kind == 0) static_cast<float*>(out)[c] = v;
    else if (out_kind == 1) static_cast<uint16_t*>(out)[c] = f32_to_bf16(v);
    else static_cast<uint16_t*>(out)[c] = __builtin_bit_cast(uint16_t, (_Float16)v);
  }
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
  dim3 gr((unsigned)((D + 63) / 64)), bl(kBlock);
  if (dgamma) hipLaunchKernelGGL(colsum_kernel, gr, bl, 0, s, part, nb, D, (void*)dgamma, 0);
  if (dbeta) hipLaunchKernelGGL(colsum_kernel, gr, bl, 0, s, part + nb * D, nb, D, (void*)dbeta, 0);
  if (dbias && ga) hipLaunchKernelGGL(colsum_kernel, gr, bl, 0, s, part + 2 * nb * D, nb, D, dbias, dbias_kind);
}

void launch_gelu_fwd(int kind, const uint16_t* u, const void* bias, int bias_kind, uint16_t* h, int64_t T, int64_t F,
                     hipStream_t s) {
  const int64_t n8 = T * F / 8;
  dim3 gr(grid_for(n8, 2)), bl(kBlock);
  if (kind == 1) hipLaunchKernelGGL(gelu_fwd_kernel<1>, gr, bl, 0, s, u, bias, bias_kind, h, n8, (int)F);
  else hipLaunchKernelGGL(gelu_fwd_kernel<2>, gr, bl, 0, s, u, bias, bias_kind, h, n8, (int)F);
}

int gelu_bwd_chunks(int64_t T, int64_t F) {
  // ~12 waves per CU in total: (F/8/128 column blocks) x chunks of 2-wave blocks.
  const int64_t colblocks = (F / 8 + 127) / 128;
  int64_t c = (256 * 6) / (colblocks > 0 ? colblocks : 1);
  if (c > T / 8) c = T / 8;
  return (int)(c < 1 ? 1 : c);
}

void launch_gelu_bwd(int kind, const uint16_t* gh, const uint16_t* u, const void* bias, int bias_kind, uint16_t* gu,
                     float* part, void* dbias, int dbias_kind, int64_t T, int64_t F, hipStream_t s) {
  const int chunks = gelu_bwd_chunks(T, F);
  const int64_t rpc = (T + chunks - 1) / chunks;
  dim3 gr((unsigned)((F / 8 + 127) / 128), (unsigned)chunks), bl(128);
  if (kind == 1) hipLaunchKernelGGL(gelu_bwd_kernel<1>, gr, bl, 0, s, gh, u, bias, bias_kind, gu, part, T, (int)F, rpc);
  else hipLaunchKernelGGL(gelu_bwd_kernel<2>, gr, bl, 0, s, gh, u, bias, bias_kind, gu, part, T, (int)F, rpc);
  if (dbias) hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((F + 63) / 64)), dim3(kBlock), 0, s, part, (int64_t)chunks, F,
                                dbias, dbias_kind);
}

}  // namespace dpt
