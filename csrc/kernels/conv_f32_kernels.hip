// Channels-last fp32 convolutions on the gfx950 fp32 matrix cores (v_mfma_f32_32x32x2_f32).
//
// Why: the reference's default precision is fp32 (train_ddp.py:210-214).  Its convolutions ran
// on MIOpen, whose fp32 NHWC solvers are a mix of ASM implicit GEMMs that split K with atomics
// (forward non-deterministic at 1e-6: ReLU-mask flips, profiles/replay_noise_r5.md), CK grouped
// solvers that are wrong under hipGraph replay (profiles/graph_replay_miopen_r4.md) and naive
// kernels - and fp32 ResNet-50 reached 39 TFLOP/s, a quarter of the 157 TFLOP/s fp32 MFMA peak.
// These kernels compute exact fp32 (one rounding per product, a k-ordered fma chain: the MFMA's
// numerics, cdna_hip_programming.md "FP32-input MFMA"), deterministically (split-K partials are
// summed by a separate kernel in a fixed order, never with atomics), and replay-safe.
//
// GEMM views (channels_last activations are row-major [pixels, channels]; K-steps of 32 floats
// = one 128-byte LDS row, the geometry of the bf16 kernels in conv_kernels.hip):
//   forward   y[m, co] = sum_k A[m, k] W[co, k],  m = (n, ho, wo), k = (r*S + s)*C + c,
//             A[m, k] = x[n, ho*st - pad + r, wo*st - pad + s, c]      (0 in the padding)
//   dgrad     dx[m, c] = sum_k A[m, k] Wt[c, k],  m = (n, h, w), k = (r*S + s)*Co + co,
//             A[m, k] = dy[n, (h + pad - r)/st, (w + pad - s)/st, co]  (0 unless divisible/in range)
//             Wt[c][r][s][co] = w[co][r][s][c] (transposed by the caller: weights are small)
//   wgrad     dW[co, j] = sum_q dy[q, co] X[q, j],  q = (n, ho, wo), j = (r*S + s)*C + c,
//             X[q, j] = x[n, ho*st - pad + r, wo*st - pad + s, c];  both operands are K-major
//             (rows = pixels), staged as [32 q][128] images and read one float per lane.
//
// Tiles: 128 x 128 outputs x 32 K per step, 256 threads = 4 waves of 64 x 64 (2 x 2 MFMA tiles of
// 32 x 32).  Operands go global -> LDS directly (buffer_load ... lds, zero padding = out-of-range
// offset), one stage (32 KiB: 4 resident blocks per CU overlap each other's loads with MFMAs - an
// fp32 K-step is 64 MFMAs x 64 cycles per wave, so 8 B/clk/CU of operand traffic suffices).
// Split-K over blocks when the tile grid is small; the partial tiles are reduced by
// conv_f32_reduce_kernel (fixed summation order).
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace dpt {
namespace cf32 {

constexpr int BM = 128, BN = 128, BK = 32;  // BK floats = 128 B per LDS row
constexpr int kThreads = 256;
constexpr int kRowBytes = BK * 4;
constexpr uint32_t kOOB = 0xFFFFFF00u;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ void glds16(const __amdgpu_buffer_rsrc_t& rs, unsigned char* lds_base, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_base, 16, off, 0, 0, 0);
}

}  // namespace cf32

struct ConvF32Args {
  const float* a;  // forward: x [N,H,W,C]; dgrad: dy [N,Ho,Wo,Co]
  const float* b;  // forward: w [Co][R*S*C]; dgrad: wt [C][R*S*Co]
  float* out;      // [splits][M][ncols]
  int N, H, W, C, Ho, Wo, Co, R, S, stride, pad;
  int ca;          // channels of the A source (forward C, dgrad Co)
  int ncols;       // forward Co, dgrad C
  int64_t M;       // forward N*Ho*Wo, dgrad N*H*W
  int K;           // R*S*ca
  int m_tiles, n_tiles, splits, kps;
  uint32_t a_bytes, b_bytes;
};

// DGRAD = false: forward; true: backward-data (transposed-conv gather of dy).
template <bool DGRAD>
__global__ __launch_bounds__(cf32::kThreads, 2) void conv_f32_mk_kernel(ConvF32Args p) {
  using namespace cf32;
  constexpr int STAGE = (BM + BN) * kRowBytes;  // 32 KiB
  __shared__ __attribute__((aligned(16))) unsigned char lds[STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = p.m_tiles * p.n_tiles;
  const int bid0 = xcd_remap(blockIdx.x, tiles * p.splits);
  const int sp = bid0 % p.splits, bid = bid0 / p.splits;
  const int mt = bid / p.n_tiles, nt = bid % p.n_tiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  // output-row geometry: forward rows are (n, ho, wo) of y, dgrad rows (n, h, w) of dx
  const int Hm = DGRAD ? p.H : p.Ho, Wm = DGRAD ? p.W : p.Wo;
  const int Hs = DGRAD ? p.Ho : p.H, Ws = DGRAD ? p.Wo : p.W;  // A source image

  // per-lane A rows (4 glds instructions per wave, 8 rows each) and B rows
  int rn[4], ry[4], rx[4], arow[4], achunk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    arow[i] = row;
    achunk[i] = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t m = m0 + row;
    if (m < p.M) {
      const int64_t hw = (int64_t)Hm * Wm;
      rn[i] = (int)(m / hw);
      const int rem = (int)(m - (int64_t)rn[i] * hw);
      ry[i] = rem / Wm;
      rx[i] = rem - ry[i] * Wm;
    } else {
      rn[i] = -1;
      ry[i] = rx[i] = 0;
    }
  }
  int bofs[4];
  bool bok[4];
  int bchunk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    bchunk[i] = (lane & 7) ^ ((row >> 1) & 7);
    const int j = n0 + row;
    bok[i] = j < p.ncols;
    bofs[i] = bok[i] ? j * p.K : 0;
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, (int)p.b_bytes, 0x00020000);

  const int nk = (p.K + BK - 1) / BK;
  const int ks0 = sp * p.kps;
  const int ks1 = min(nk, ks0 + p.kps);

  // ca % 32 == 0 (every ResNet conv but the stem): a K-step is 32 channels of ONE tap, so the
  // tap and channel block are wave-uniform (scalar) and a row's source offset is its base plus
  // a per-step constant; only the bounds (and, strided dgrad, the parity) are per row.
  const bool wide = p.ca % BK == 0;
  const int cpk = p.ca / BK;
  auto stage = [&](int ks) {
    unsigned char* a = lds;
    unsigned char* b = lds + BM * kRowBytes;
    if (wide) {
      const int tap = ks / cpk, cb = ks - tap * cpk;
      const int r = tap / p.S, s = tap - r * p.S;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t off = kOOB;
        if (rn[i] >= 0) {
          int ys, xs;
          bool ok;
          if (DGRAD) {
            const int t = ry[i] + p.pad - r, u = rx[i] + p.pad - s;
            if (p.stride == 1) {
              ys = t; xs = u; ok = true;
            } else {
              ok = t >= 0 && u >= 0 &&
                   (p.stride == 2 ? ((t | u) & 1) == 0 : (t % p.stride) == 0 && (u % p.stride) == 0);
              ys = p.stride == 2 ? t >> 1 : t / p.stride;
              xs = p.stride == 2 ? u >> 1 : u / p.stride;
            }
          } else {
            ys = ry[i] * p.stride - p.pad + r;
            xs = rx[i] * p.stride - p.pad + s;
            ok = true;
          }
          ok = ok && (unsigned)ys < (unsigned)Hs && (unsigned)xs < (unsigned)Ws;
          if (ok) off = (uint32_t)((((int64_t)rn[i] * Hs + ys) * Ws + xs) * p.ca + cb * BK + achunk[i] * 4) * 4u;
        }
        cf32::glds16(ra, a + (wid * 4 + i) * 1024, off);
      }
    } else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = ks * BK + achunk[i] * 4;  // 4 channels of one tap (ca % 4 == 0)
      uint32_t off = kOOB;
      if (rn[i] >= 0 && k < p.K) {
        const int tap = k / p.ca, c = k - tap * p.ca;
        const int r = tap / p.S, s = tap - r * p.S;
        int ys, xs;
        bool ok;
        if (DGRAD) {
          const int t = ry[i] + p.pad - r, u = rx[i] + p.pad - s;
          ok = t >= 0 && u >= 0 && (t % p.stride) == 0 && (u % p.stride) == 0;
          ys = t / p.stride;
          xs = u / p.stride;
        } else {
          ys = ry[i] * p.stride - p.pad + r;
          xs = rx[i] * p.stride - p.pad + s;
          ok = true;
        }
        ok = ok && (unsigned)ys < (unsigned)Hs && (unsigned)xs < (unsigned)Ws;
        if (ok) off = (uint32_t)((((int64_t)rn[i] * Hs + ys) * Ws + xs) * p.ca + c) * 4u;
      }
      cf32::glds16(ra, a + (wid * 4 + i) * 1024, off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = ks * BK + bchunk[i] * 4;
      const uint32_t off = (bok[i] && k < p.K) ? (uint32_t)(bofs[i] + k) * 4u : kOOB;
      cf32::glds16(rb, b + (wid * 4 + i) * 1024, off);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  for (int ks = ks0; ks < ks1; ++ks) {
    stage(ks);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned char* a = lds;
    const unsigned char* b = lds + BM * kRowBytes;
    // lane (lr, lh) supplies K index 16*lh + t to MFMA t: its 16 floats are chunks 4lh..4lh+3
    float4 fa[2][4], fb[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wm * 64 + i * 32 + lr;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        fa[i][q] = *reinterpret_cast<const float4*>(a + row * kRowBytes + cf32::swz(row, 4 * lh + q) * 16);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 64 + j * 32 + lr;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        fb[j][q] = *reinterpret_cast<const float4*>(b + row * kRowBytes + cf32::swz(row, 4 * lh + q) * 16);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][q][e], fb[j][q][e], acc[i][j], 0, 0, 0);
    __syncthreads();
  }

  // accumulator map: column = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  float* out = p.out + (int64_t)sp * p.M * p.ncols;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + lr;
      if (col >= p.ncols) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (m < p.M) out[m * p.ncols + col] = acc[i][j][e];
      }
    }
}

struct ConvF32WArgs {
  const float* dy;  // [Q = N*Ho*Wo][Co]
  const float* x;   // [N,H,W,C]
  float* out;       // [splits][Co][R*S*C]
  int N, H, W, C, Ho, Wo, Co, R, S, stride, pad;
  int J;            // R*S*C
  int64_t Q;
  int m_tiles, n_tiles, splits, kps;
  uint32_t dy_bytes, x_bytes;
};

// dW = dy^T X over pixel K-steps of 32; both operands staged as [32 pixels][128] float images
// (512-byte rows, two rows per 1 KiB glds instruction) and read one float per lane and MFMA
// (ds_read_b32: 32 consecutive floats of one row per 32-lane half - conflict-free).
__global__ __launch_bounds__(cf32::kThreads, 2) void conv_f32_wgrad_kernel(ConvF32WArgs p) {
  using namespace cf32;
  constexpr int IMG = BK * BM * 4;  // 16 KiB per operand
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = p.m_tiles * p.n_tiles;
  const int bid0 = xcd_remap(blockIdx.x, tiles * p.splits);
  const int sp = bid0 % p.splits, bid = bid0 / p.splits;
  const int mt = bid / p.n_tiles, nt = bid % p.n_tiles;
  const int i0 = mt * BM, j0 = nt * BN;
  const int chunk = lane & 31;
  // A: channels i0 + chunk*4 .. +3 of dy rows; B: column j0 + chunk*4 = (tap, c) of x, fixed per lane
  const int ai = i0 + chunk * 4;
  const bool aok = ai < p.Co;
  const int bj = j0 + chunk * 4;
  const bool bok = bj < p.J;
  int br = 0, bs = 0, bc = 0;
  if (bok) {
    const int tap = bj / p.C;
    bc = bj - tap * p.C;
    br = tap / p.S;
    bs = tap - br * p.S;
  }
  const int64_t nq = (p.Q + BK - 1) / BK;
  const int64_t ks0 = (int64_t)sp * p.kps;
  const int64_t ks1 = min(nq, ks0 + p.kps);
  // this lane's 4 pixel rows of a K-step (one per glds instruction): row = (wid*4 + i)*2 + lane/32
  int64_t q[4];
  int qn[4], qh[4], qw[4];
  const int HoWo = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    q[i] = ks0 * BK + (wid * 4 + i) * 2 + (lane >> 5);
    const int64_t qq = q[i] < p.Q ? q[i] : 0;
    qn[i] = (int)(qq / HoWo);
    const int rem = (int)(qq - (int64_t)qn[i] * HoWo);
    qh[i] = rem / p.Wo;
    qw[i] = rem - qh[i] * p.Wo;
  }
  const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, (int)p.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)p.x_bytes, 0x00020000);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  for (int64_t ks = ks0; ks < ks1; ++ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool qok = q[i] < p.Q;
      const uint32_t aoff = (qok && aok) ? (uint32_t)(q[i] * p.Co + ai) * 4u : kOOB;
      cf32::glds16(rdy, lds + (wid * 4 + i) * 1024, aoff);
      uint32_t xoff = kOOB;
      if (qok && bok) {
        const int hi = qh[i] * p.stride - p.pad + br, wi = qw[i] * p.stride - p.pad + bs;
        if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
          xoff = (uint32_t)((((int64_t)qn[i] * p.H + hi) * p.W + wi) * p.C + bc) * 4u;
      }
      cf32::glds16(rx, lds + IMG + (wid * 4 + i) * 1024, xoff);
      // advance this row by one K-step (32 pixels)
      q[i] += BK;
      qw[i] += BK;
      while (qw[i] >= p.Wo) {
        qw[i] -= p.Wo;
        if (++qh[i] >= p.Ho) {
          qh[i] = 0;
          ++qn[i];
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* A = reinterpret_cast<const float*>(lds);
    const float* B = reinterpret_cast<const float*>(lds + IMG);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int krow = t + 16 * lh;
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = A[krow * BM + wm * 64 + i * 32 + lr];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = B[krow * BN + wn * 64 + j * 32 + lr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  float* out = p.out + (int64_t)sp * p.Co * p.J;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = j0 + wn * 64 + j * 32 + lr;
      if (col >= p.J) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = i0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (row < p.Co) out[(int64_t)row * p.J + col] = acc[i][j][e];
      }
    }
}

// out[e] = sum over s of part[s][e] in split order (deterministic); n4 float4s per split.
__global__ __launch_bounds__(kBlock) void conv_f32_reduce_kernel(const float4* __restrict__ part, int64_t n4,
                                                                 int splits, float4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 a = part[i];
    for (int s = 1; s < splits; ++s) {
      const float4 b = part[(int64_t)s * n4 + i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    out[i] = a;
  }
}

namespace {

// split-K so that a small tile grid still fills the chip (>= 16 K-steps per split, at most
// `target` blocks): every extra split costs a partial tile written and read back by the reduce
// (measured on ResNet-50: a 1024-block target moved ~28 GB/step through conv_f32_reduce_kernel)
void choose_splits(int tiles, int64_t nk, int target, int* splits, int* kps) {
  int sp = 1;
  if (tiles < target && nk >= 32) {
    sp = (int)std::min<int64_t>(nk / 16, (target + tiles - 1) / tiles);
    sp = std::max(sp, 1);
  }
  int64_t k = (nk + sp - 1) / sp;
  sp = (int)((nk + k - 1) / k);
  *splits = sp;
  *kps = (int)k;
}

void check_bytes(int64_t bytes, const char* what) {
  if (bytes >= (int64_t)1 << 31) throw std::invalid_argument(std::string("conv_f32: ") + what + " exceeds 2 GiB");
}

}  // namespace

int64_t conv_f32_workspace(int64_t M, int ncols, int K, int* splits_out) {
  const int tiles = (int)((M + cf32::BM - 1) / cf32::BM) * ((ncols + cf32::BN - 1) / cf32::BN);
  int sp, kps;
  choose_splits(tiles, (K + cf32::BK - 1) / cf32::BK, 512, &sp, &kps);
  if (splits_out) *splits_out = sp;
  return sp > 1 ? (int64_t)sp * M * ncols : 0;
}

void launch_conv_f32(const float* a, const float* b, float* out, float* ws, bool dgrad, int N, int H, int W, int C,
                     int Ho, int Wo, int Co, int R, int S, int stride, int pad, hipStream_t st) {
  ConvF32Args p{};
  p.a = a;
  p.b = b;
  p.N = N; p.H = H; p.W = W; p.C = C; p.Ho = Ho; p.Wo = Wo; p.Co = Co; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad;
  p.ca = dgrad ? Co : C;
  p.ncols = dgrad ? C : Co;
  p.M = dgrad ? (int64_t)N * H * W : (int64_t)N * Ho * Wo;
  p.K = R * S * p.ca;
  if (p.ca % 4 != 0) throw std::invalid_argument("conv_f32: channels of the gathered operand must be a multiple of 4");
  const int64_t a_bytes = dgrad ? (int64_t)N * Ho * Wo * Co * 4 : (int64_t)N * H * W * C * 4;
  const int64_t b_bytes = (int64_t)p.ncols * p.K * 4;
  check_bytes(a_bytes, "input");
  check_bytes(b_bytes, "weight");
  p.a_bytes = (uint32_t)a_bytes;
  p.b_bytes = (uint32_t)b_bytes;
  p.m_tiles = (int)((p.M + cf32::BM - 1) / cf32::BM);
  p.n_tiles = (p.ncols + cf32::BN - 1) / cf32::BN;
  choose_splits(p.m_tiles * p.n_tiles, (p.K + cf32::BK - 1) / cf32::BK, 512, &p.splits, &p.kps);
  if (p.splits > 1 && ws == nullptr) throw std::invalid_argument("conv_f32: split-K needs a workspace");
  p.out = p.splits > 1 ? ws : out;
  const dim3 grid(p.m_tiles * p.n_tiles * p.splits);
  if (dgrad) conv_f32_mk_kernel<true><<<grid, cf32::kThreads, 0, st>>>(p);
  else conv_f32_mk_kernel<false><<<grid, cf32::kThreads, 0, st>>>(p);
  if (p.splits > 1) {
    const int64_t n4 = p.M * p.ncols / 4;
    conv_f32_reduce_kernel<<<grid_for(n4, 2), kBlock, 0, st>>>(reinterpret_cast<const float4*>(ws), n4, p.splits,
                                                              reinterpret_cast<float4*>(out));
  }
}

int64_t conv_f32_wgrad_workspace(int N, int Ho, int Wo, int Co, int J) {
  const int tiles = ((Co + cf32::BM - 1) / cf32::BM) * ((J + cf32::BN - 1) / cf32::BN);
  int sp, kps;
  choose_splits(tiles, ((int64_t)N * Ho * Wo + cf32::BK - 1) / cf32::BK, 512, &sp, &kps);
  return sp > 1 ? (int64_t)sp * Co * J : 0;
}

void launch_conv_f32_wgrad(const float* dy, const float* x, float* dw, float* ws, int N, int H, int W, int C,
                           int Ho, int Wo, int Co, int R, int S, int stride, int pad, hipStream_t st) {
  ConvF32WArgs p{};
  p.dy = dy;
  p.x = x;
  p.N = N; p.H = H; p.W = W; p.C = C; p.Ho = Ho; p.Wo = Wo; p.Co = Co; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad;
  p.J = R * S * C;
  p.Q = (int64_t)N * Ho * Wo;
  if (C % 4 != 0 || Co % 4 != 0) throw std::invalid_argument("conv_f32_wgrad: channels must be multiples of 4");
  const int64_t dy_bytes = p.Q * Co * 4, x_bytes = (int64_t)N * H * W * C * 4;
  check_bytes(dy_bytes, "grad_output");
  check_bytes(x_bytes, "input");
  p.dy_bytes = (uint32_t)dy_bytes;
  p.x_bytes = (uint32_t)x_bytes;
  p.m_tiles = (Co + cf32::BM - 1) / cf32::BM;
  p.n_tiles = (p.J + cf32::BN - 1) / cf32::BN;
  choose_splits(p.m_tiles * p.n_tiles, (p.Q + cf32::BK - 1) / cf32::BK, 512, &p.splits, &p.kps);
  if (p.splits > 1 && ws == nullptr) throw std::invalid_argument("conv_f32_wgrad: split-K needs a workspace");
  p.out = p.splits > 1 ? ws : dw;
  const dim3 grid(p.m_tiles * p.n_tiles * p.splits);
  conv_f32_wgrad_kernel<<<grid, cf32::kThreads, 0, st>>>(p);
  if (p.splits > 1) {
    const int64_t n4 = (int64_t)Co * p.J / 4;
    conv_f32_reduce_kernel<<<grid_for(n4, 2), kBlock, 0, st>>>(reinterpret_cast<const float4*>(ws), n4, p.splits,
                                                              reinterpret_cast<float4*>(dw));
  }
}

}  // namespace dpt
