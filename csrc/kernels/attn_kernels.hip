// Fused multi-head self-attention (forward + backward) for short sequences on gfx950 MFMA.
//
// ViT-B/16 runs 197 tokens x 12 heads x 64 dims per image.  A whole head fits on chip (K and V
// are 197 x 64 bf16 = 25 KB each), so one workgroup owns one (image, head): no online-softmax
// rescaling, no split-K atomics, and Q/K/V are read straight out of the QKV projection's
// [B, S, 3, H, 64] output (no head split / merge copies) and the context is written straight
// into the out-projection's [B, S, H*64] input.
//
// Every product is a v_mfma_f32_32x32x16_bf16; the softmax stays in the accumulator registers
// and is fed to the next product as an operand without leaving them (mfma.h acc_frag, the
// "accumulator tile as the next MFMA's operand" idiom: scores are computed transposed,
// keys x queries, so a query's keys are that lane's registers).  Per 32-query wave:
//   forward   S^T = K Q^T  ->  P^T = softmax over keys (registers + one xor-32 shuffle)
//             O^T = V^T P^T  (V^T fragments by ds_read_b64_tr_b16 in P^T's k order)
//             saves lse2 = log2-sum-exp of scaled scores per query
//   backward  D = rowsum(dO * O); phase 1 (wave = 32 keys): S, dP = dO V^T, P, dS = P (dP - D),
//             dV += P^T dO, dK += dS^T Q (P / dS reused as A operands);  phase 2 (wave = 32
//             queries): S^T, dP^T, dS^T, dQ^T += K^T dS^T.
// Padding keys (>= S) are masked to probability 0; padding queries are never stored and get
// lse2 = +inf in the backward, so they contribute nothing to dK / dV.
#include <cmath>

#include "common.h"
#include "kernels.h"
#include "mfma.h"

namespace dpt {

namespace attn {
constexpr int D = 64;     // head dim
constexpr int RB = 128;   // LDS row bytes (64 bf16)
}  // namespace attn

// 2^x on the transcendental unit (v_exp_f32) without the denormal-range fix-up libm's exp2f adds
// (compare, scale, ldexp, select: 4 more VALU per score).  It differs only where 2^x < 2^-126,
// probabilities that vanish in the bf16 operands anyway; forward and backward use the same one,
// so the recomputed P matches the forward's.
__device__ __forceinline__ float attn_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Stage rows [0, S) of a [S, ld]-strided bf16 matrix's 64-column slice into an LDS image of
// SP rows (rows >= S zero).
__device__ __forceinline__ void attn_stage(unsigned char* img, const uint16_t* src, int64_t ld, int S, int SP,
                                           int tid, int nthreads) {
  for (int c = tid; c < SP * 8; c += nthreads) {
    const int row = c >> 3, ch = c & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < S) v = *reinterpret_cast<const uint4*>(src + (int64_t)row * ld + ch * 8);
    *reinterpret_cast<uint4*>(img + row * attn::RB + wg_slot<attn::RB>(row, ch) * 16) = v;
  }
}

template <int NT>
__global__ __launch_bounds__(NT * 64) void attn_fwd_kernel(const uint16_t* __restrict__ qkv,
                                                           uint16_t* __restrict__ ctx, float* __restrict__ lse2,
                                                           int S, int H, float scale_log2) {
  using namespace attn;
  constexpr int SP = NT * 32, NTH = NT * 64;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * SP * RB];
  unsigned char* kimg = lds;
  unsigned char* vimg = lds + SP * RB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / H, hh = bh - b * H;
  const int64_t ld = 3LL * H * D;
  const uint16_t* base = qkv + (int64_t)b * S * ld;
  attn_stage(kimg, base + (int64_t)(H + hh) * D, ld, S, SP, tid, NTH);
  attn_stage(vimg, base + (int64_t)(2 * H + hh) * D, ld, S, SP, tid, NTH);

  const int r = lane & 31, h = lane >> 5;
  const int q = w * 32 + r;
  bf16x8_t qf[4];  // B operand of S^T = K Q^T: Q[q][16s + 8h .. +7]
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < S) v = *reinterpret_cast<const uint4*>(base + (int64_t)q * ld + hh * D + 16 * s + 8 * h);
    qf[s] = __builtin_bit_cast(bf16x8_t, v);
  }
  __syncthreads();

  f32x16_t sc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
    for (int e = 0; e < 16; ++e) sc[kt][e] = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) sc[kt] = mfma32(row_frag<RB>(kimg, kt * 32 + r, 2 * s + h), qf[s], sc[kt]);
  }
  // softmax over keys (this lane's registers + the other lane half)
  // padding keys exist only in the last tile(s): the per-element mask is a wave-uniform branch
  // away everywhere else (it was 2 of the ~10 VALU per score)
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    if ((kt + 1) * 32 > S) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (key >= S) sc[kt][e] = -INFINITY;
      }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) m = fmaxf(m, sc[kt][e]);
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float ms = m * scale_log2;
  float l = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float pv = attn_exp2(__builtin_fmaf(sc[kt][e], scale_log2, -ms));
      sc[kt][e] = pv;
      l += pv;
    }
  l += __shfl_xor(l, 32, 64);

  f32x16_t o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[dt][e] = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t pf = acc_frag(sc[kt], s2);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        o[dt] = mfma32(tr_frag<RB, true>(vimg, kt * 32 + 16 * s2, dt * 32, lane), pf, o[dt]);
    }
  if (q < S) {
    const float inv = 1.0f / l;
    uint16_t* out = ctx + ((int64_t)b * S + q) * H * D + hh * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // rows d = 32dt + 8g + 4h + 0..3 (registers 4g..4g+3)
        const f32x2_t v0 = {o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv};
        const f32x2_t v1 = {o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv};
        uint2 pk;
        pk.x = __builtin_bit_cast(uint32_t, __builtin_convertvector(v0, bf16x2_t));
        pk.y = __builtin_bit_cast(uint32_t, __builtin_convertvector(v1, bf16x2_t));
        *reinterpret_cast<uint2*>(out + dt * 32 + 8 * g + 4 * h) = pk;
      }
    if (h == 0) lse2[(int64_t)bh * SP + q] = ms + log2f(l);
  }
}

// PHASE 0: both phases in one workgroup (four LDS images, one workgroup per CU); 1: dK / dV only
// (Q and dO images); 2: dQ only (K and V images) - two launches at half the LDS each, so two
// workgroups share a CU (attn_set_bwd_split; phase 1 reads K / V rows and phase 2 Q / dO rows as
// register fragments straight from global memory)
#ifndef DPT_ATTN_P1_WAVES  // min waves per SIMD of the split phase-1 kernel (4 = two workgroups per CU)
#define DPT_ATTN_P1_WAVES 2
#endif
template <int NT, int PHASE = 0>
__global__ __launch_bounds__(NT * 64, PHASE == 1 ? DPT_ATTN_P1_WAVES : PHASE == 2 ? 4 : 1) void attn_bwd_kernel(const uint16_t* __restrict__ qkv,
                                                                        const uint16_t* __restrict__ out,
                                                                        const uint16_t* __restrict__ dout,
                                                                        const float* __restrict__ lse2,
                                                                        uint16_t* __restrict__ dqkv, int S, int H,
                                                                        float scale_log2, float scale) {
  using namespace attn;
  constexpr int SP = NT * 32, NTH = NT * 64;
  constexpr int NIMG = PHASE ? 2 : 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[NIMG * SP * RB + 2 * SP * 4];
  // phase-1 images: Q, dO; phase-2 images: K, V (PHASE 0: all four)
  unsigned char* qimg = lds;
  unsigned char* oimg = lds + SP * RB;  // dO
  unsigned char* kimg = lds + (PHASE == 2 ? 0 : 2) * SP * RB;
  unsigned char* vimg = lds + (PHASE == 2 ? 1 : 3) * SP * RB;
  float* ls = reinterpret_cast<float*>(lds + NIMG * SP * RB);
  float* dd = ls + SP;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / H, hh = bh - b * H;
  const int64_t ld = 3LL * H * D, ldo = (int64_t)H * D;
  const uint16_t* base = qkv + (int64_t)b * S * ld;
  const uint16_t* obase = dout + (int64_t)b * S * ldo + hh * D;
  if (PHASE != 2) {
    attn_stage(qimg, base + (int64_t)hh * D, ld, S, SP, tid, NTH);
    attn_stage(oimg, obase, ldo, S, SP, tid, NTH);
  }
  if (PHASE != 1) {
    attn_stage(kimg, base + (int64_t)(H + hh) * D, ld, S, SP, tid, NTH);
    attn_stage(vimg, base + (int64_t)(2 * H + hh) * D, ld, S, SP, tid, NTH);
  }
  // row fragment (16 B) of a [S, ld] bf16 matrix straight from global memory (rows >= S: zero)
  auto gfrag = [&](const uint16_t* src, int64_t ldm, int row, int ch) -> bf16x8_t {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < S) v = *reinterpret_cast<const uint4*>(src + (int64_t)row * ldm + ch * 8);
    return __builtin_bit_cast(bf16x8_t, v);
  };
  for (int t = tid; t < SP; t += NTH) {  // D[q] = sum_d dO * O (fp32), lse2 (+inf for padding)
    float acc = 0.f;
    if (t < S) {
      const uint16_t* po = out + ((int64_t)b * S + t) * ldo + hh * D;
      const uint16_t* pd = dout + ((int64_t)b * S + t) * ldo + hh * D;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint4 a = *reinterpret_cast<const uint4*>(po + c * 8);
        const uint4 g = *reinterpret_cast<const uint4*>(pd + c * 8);
        const uint32_t ua[4] = {a.x, a.y, a.z, a.w}, ug[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc = __builtin_fmaf(bf16_to_f32(ua[k] & 0xffff), bf16_to_f32(ug[k] & 0xffff), acc);
          acc = __builtin_fmaf(bf16_to_f32(ua[k] >> 16), bf16_to_f32(ug[k] >> 16), acc);
        }
      }
    }
    dd[t] = acc;
    ls[t] = t < S ? lse2[(int64_t)bh * SP + t] : INFINITY;
  }
  __syncthreads();
  const int r = lane & 31, h = lane >> 5;

  // ---- phase 1: this wave's 32 keys against every query tile -> dK, dV ----
  if (PHASE != 2) {
    const int k0 = w * 32, key = k0 + r;
    f32x16_t dv[2], dk[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) { dv[dt][e] = 0.f; dk[dt][e] = 0.f; }
    bf16x8_t kf[4], vf[4];  // B operands: K[key][d], V[key][d] rows
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (PHASE == 1) {
        kf[s] = gfrag(base + (int64_t)(H + hh) * D, ld, key, 2 * s + h);
        vf[s] = gfrag(base + (int64_t)(2 * H + hh) * D, ld, key, 2 * s + h);
      } else {
        kf[s] = row_frag<RB>(kimg, key, 2 * s + h);
        vf[s] = row_frag<RB>(vimg, key, 2 * s + h);
      }
    }
    for (int qt = 0; qt < NT; ++qt) {
      f32x16_t sc, dp;
#pragma unroll
      for (int e = 0; e < 16; ++e) { sc[e] = 0.f; dp[e] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc = mfma32(row_frag<RB>(qimg, qt * 32 + r, 2 * s + h), kf[s], sc);   // S = Q K^T
        dp = mfma32(row_frag<RB>(oimg, qt * 32 + r, 2 * s + h), vf[s], dp);   // dP = dO V^T
      }
      // rows = queries, column = this lane's key: rows (e & 3) of group e >> 2 are 4 consecutive
      // queries, so their lse2 / D values come in one 16-byte LDS read each (8 reads, not 32)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int q4 = qt * 32 + 8 * e4 + 4 * h;
        const float4 l4 = *reinterpret_cast<const float4*>(ls + q4);
        const float4 d4 = *reinterpret_cast<const float4*>(dd + q4);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int e = 4 * e4 + j;
          const float pv = key < S ? attn_exp2(__builtin_fmaf(sc[e], scale_log2, -lv[j])) : 0.f;
          sc[e] = pv;
          dp[e] = pv * (dp[e] - dv4[j]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8_t pa = acc_frag(sc, s2), da = acc_frag(dp, s2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32(pa, tr_frag<RB, true>(oimg, qt * 32 + 16 * s2, dt * 32, lane), dv[dt]);  // P^T dO
          dk[dt] = mfma32(da, tr_frag<RB, true>(qimg, qt * 32 + 16 * s2, dt * 32, lane), dk[dt]);  // dS^T Q
        }
      }
    }
    // rows = keys (registers), column = d (lane)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kk = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (kk < S) {
          uint16_t* row = dqkv + ((int64_t)b * S + kk) * ld;
          row[(int64_t)(H + hh) * D + dt * 32 + r] = f32_to_bf16(dk[dt][e] * scale);
          row[(int64_t)(2 * H + hh) * D + dt * 32 + r] = f32_to_bf16(dv[dt][e]);
        }
      }
  }

  // ---- phase 2: this wave's 32 queries against every key tile -> dQ ----
  if (PHASE != 1) {
    const int q = w * 32 + r;
    bf16x8_t qf[4], of[4];  // B operands of S^T = K Q^T and dP^T = V dO^T
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (PHASE == 2) {
        qf[s] = gfrag(base + (int64_t)hh * D, ld, q, 2 * s + h);
        of[s] = gfrag(obase, ldo, q, 2 * s + h);
      } else {
        qf[s] = row_frag<RB>(qimg, q, 2 * s + h);
        of[s] = row_frag<RB>(oimg, q, 2 * s + h);
      }
    }
    const float lq = ls[q], dq0 = dd[q];
    f32x16_t dq[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) dq[dt][e] = 0.f;
    for (int kt = 0; kt < NT; ++kt) {
      f32x16_t st, dpt;
#pragma unroll
      for (int e = 0; e < 16; ++e) { st[e] = 0.f; dpt[e] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(row_frag<RB>(kimg, kt * 32 + r, 2 * s + h), qf[s], st);
        dpt = mfma32(row_frag<RB>(vimg, kt * 32 + r, 2 * s + h), of[s], dpt);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {  // rows = keys, column = this lane's query
        const int key = kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const float pv = key < S ? attn_exp2(__builtin_fmaf(st[e], scale_log2, -lq)) : 0.f;
        st[e] = pv * (dpt[e] - dq0);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8_t df = acc_frag(st, s2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          dq[dt] = mfma32(tr_frag<RB, true>(kimg, kt * 32 + 16 * s2, dt * 32, lane), df, dq[dt]);  // K^T dS^T
      }
    }
    if (q < S) {
      uint16_t* row = dqkv + ((int64_t)b * S + q) * ld + (int64_t)hh * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x2_t v0 = {dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale};
          const f32x2_t v1 = {dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale};
          uint2 pk;
          pk.x = __builtin_bit_cast(uint32_t, __builtin_convertvector(v0, bf16x2_t));
          pk.y = __builtin_bit_cast(uint32_t, __builtin_convertvector(v1, bf16x2_t));
          *reinterpret_cast<uint2*>(row + dt * 32 + 8 * g + 4 * h) = pk;
        }
    }
  }
}

bool attn_supported(int S, int Dh) { return Dh == attn::D && S >= 1 && S <= 256; }

int attn_lse_stride(int S) { return (S + 31) / 32 * 32; }

#define DPT_ATTN_DISPATCH(NTV, KERNEL, ...)                                                              \
  switch (NTV) {                                                                                         \
    case 1: hipLaunchKernelGGL(KERNEL<1>, grid, dim3(64), 0, st, __VA_ARGS__); break;                    \
    case 2: hipLaunchKernelGGL(KERNEL<2>, grid, dim3(128), 0, st, __VA_ARGS__); break;                   \
    case 3: hipLaunchKernelGGL(KERNEL<3>, grid, dim3(192), 0, st, __VA_ARGS__); break;                   \
    case 4: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(256), 0, st, __VA_ARGS__); break;                   \
    case 5: hipLaunchKernelGGL(KERNEL<5>, grid, dim3(320), 0, st, __VA_ARGS__); break;                   \
    case 6: hipLaunchKernelGGL(KERNEL<6>, grid, dim3(384), 0, st, __VA_ARGS__); break;                   \
    case 7: hipLaunchKernelGGL(KERNEL<7>, grid, dim3(448), 0, st, __VA_ARGS__); break;                   \
    default: hipLaunchKernelGGL(KERNEL<8>, grid, dim3(512), 0, st, __VA_ARGS__); break;                  \
  }

void launch_attn_fwd(const uint16_t* qkv, uint16_t* ctx, float* lse2, int B, int S, int H, float scale,
                     hipStream_t st) {
  const int nt = (S + 31) / 32;
  const dim3 grid((unsigned)(B * H));
  const float sl2 = scale * 1.4426950408889634f;
  DPT_ATTN_DISPATCH(nt, attn_fwd_kernel, qkv, ctx, lse2, S, H, sl2)
}

// Split by default for 7 query / key tiles (ViT-B/16, 197 tokens): 214-224 -> 194-202 us per
// call at batch 128 x 12 heads, bitwise identical (bench/attn_bwd_ab.py).  The phase-2 kernel
// holds two workgroups per CU (128 VGPRs); phase 1 stays at 168 VGPRs (at 128 it spills: 262 us).
static int g_attn_bwd_split = 1;
void attn_set_bwd_split(int on) { g_attn_bwd_split = on; }

void launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse2,
                     uint16_t* dqkv, int B, int S, int H, float scale, hipStream_t st) {
  const int nt = (S + 31) / 32;
  const dim3 grid((unsigned)(B * H));
  const float sl2 = scale * 1.4426950408889634f;
  if (g_attn_bwd_split && nt == 7) {  // ViT-B/16 (197 tokens)
    hipLaunchKernelGGL((attn_bwd_kernel<7, 1>), grid, dim3(448), 0, st, qkv, out, dout, lse2, dqkv, S, H, sl2, scale);
    hipLaunchKernelGGL((attn_bwd_kernel<7, 2>), grid, dim3(448), 0, st, qkv, out, dout, lse2, dqkv, S, H, sl2, scale);
    return;
  }
  DPT_ATTN_DISPATCH(nt, attn_bwd_kernel, qkv, out, dout, lse2, dqkv, S, H, sl2, scale)
}

#undef DPT_ATTN_DISPATCH

}  // namespace dpt
