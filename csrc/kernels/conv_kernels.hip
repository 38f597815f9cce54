// Channels-last bf16 convolutions as implicit GEMMs on the gfx950 matrix cores.
//
// Why: in a ResNet-50 bf16 step on MI355X the MIOpen/CK convolutions run at ~430 TFLOP/s
// averaged over forward, backward-data and backward-weight (17% of the 2.5 PF dense peak),
// and every conv output is re-read by a separate BatchNorm statistics pass.  Owning the conv
// lets the epilogue emit the BatchNorm partial sums (sum, sum of squares per output channel)
// while the tile is still on chip, so the BN statistics pass disappears.
//
// GEMM view (channels_last activations are row-major [pixels, channels]):
//   forward   y[m, co]  = sum_{r,s,ci} x[pix(m) + (r,s), ci] * w[co, r, s, ci]
//             M = N*Ho*Wo, N = Cout, K = R*S*Cin; A rows gathered per (r, s) tap (zero padding
//             = rows outside the image), B = the KRSC weight itself (K-contiguous rows).
//   dgrad     (stride 1) the same kernel on dy with the flipped/transposed weight
//             wt[ci, r', s', co] = w[co, R-1-r', S-1-s', ci] and pad' = R-1-pad.
//
// Tile: 128 (pixels) x BN (channels) x 64 (K), 256 threads = 4 waves, each wave a 32*MI x 64
// sub-tile of v_mfma_f32_32x32x16_bf16 accumulators.  Operands are register-staged into a
// double-buffered LDS image with 128-byte rows whose 16-byte chunks are XOR-swizzled by
// (row>>1)&7, so the 16 rows one ds_read_b128 quarter-wave touches land on distinct banks.
// One barrier per K-step: tile t+1's global loads are in flight while tile t is multiplied.
// Epilogue: accumulators -> bf16 -> LDS (row-padded image) -> coalesced 16-byte row stores;
// the optional BN statistics are summed from the bf16-rounded values (exactly what a BN
// pass over y would read) and written as per-M-tile partials [Cout][m_tiles], the layout
// bn_fwd_finalize_kernel consumes.
//
// Blocks are numbered so the BN-tiles of one M-tile (which share the same A rows) are
// consecutive and land on the same XCD (bijective XCD remap, cdna_hip_programming.md T1).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <stdexcept>

#include "carry.h"
#include "gelu.h"
#include "common.h"
#include "kernels.h"
#include "mfma.h"

namespace dpt {


#ifndef DPT_WGRAD_WAVES  // backward-weight occupancy target (waves per SIMD) for the 4-wave tiles
#define DPT_WGRAD_WAVES 4
#endif
#ifndef DPT_CONV_HALF_EPI
#define DPT_CONV_HALF_EPI 0
#endif

namespace conv {

constexpr int BM = 128;
constexpr int BK = 64;
constexpr int kThreads = 256;
constexpr int kRowBytes = BK * 2;  // 128 B per staged row

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Bijective XCD remap: consecutive logical ids share an XCD (MI355X: 8 XCDs, dispatch is
// round-robin over them by hardware block id).
__device__ __forceinline__ int opaque_v(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace conv

// 16-bit element type of a conv (F16 = false: bf16, true: fp16).  Operands travel as raw 16-bit
// data (glds, LDS, fragments); only the MFMA and the fp32 <-> 16-bit conversions differ.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

template <bool F16>
__device__ __forceinline__ f32x16_t cmfma(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// two fp32 -> a packed 16-bit pair (round to nearest even: v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32)
template <bool F16>
__device__ __forceinline__ uint32_t cpack(f32x2_t v) {
  if constexpr (F16) return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
  else return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
// element h (0: low half, 1: high half) of a packed 16-bit pair as fp32
template <bool F16>
__device__ __forceinline__ float cunpack(uint32_t u, int h) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, (uint16_t)(h ? (u >> 16) : (u & 0xffffu)));
  else return __uint_as_float(h ? (u & 0xffff0000u) : (u << 16));
}

// Stream-K workspace (one per device and stream, conv_sk_workspace): a contributing segment's
// fp32 partial tile [G][float4 slot][thread], a published flag per block (set with an agent-scope
// store after the sc1 payload drained; reset by the consuming block, so every launch starts from
// zeros - hipGraph replays included), and a give-up counter of the bounded spin.
struct ConvSk {
  float* part = nullptr;
  unsigned* flags = nullptr;
  unsigned* err = nullptr;
  int G = 0;
  uint32_t part_bytes = 0;
};

struct ConvFwdArgs {
  const uint16_t* x;  // [N, H, W, C]
  const uint16_t* w;  // [Cout, R, S, C]
  uint16_t* y;        // [N, Ho, Wo, Cout]
  float* psum;        // optional BN partials [Cout][m_tiles]
  float* psq;
  int N, H, W, C, Ho, Wo, Cout, R, S, stride, pad;
  int64_t M;
  int m_tiles, n_tiles;  // m_tiles: 128-row tiles (the BN-partials layout)
  int mt256;             // 256-row tiles when BM = 256
  // BNB epilogue: the BatchNorm whose ReLU output was this conv's input
  const uint16_t* bnx;   // BN input x [M, Cout] (same layout as y)
  const float* bn_mean;  // [Cout]
  const float* bn_coef;  // [2*Cout] = [a | b]
  float* bp1;            // partials [Cout][m_tiles]
  float* bp2;
  // BNR epilogue: that BatchNorm was a block tail relu(bn(x) + res) whose output also fed the
  // next block's identity path
  const uint16_t* bny;    // its output y (ReLU mask)
  const uint16_t* bnres;  // the identity-path gradient (added before the mask)
  // the same ReLU mask as 1 bit per element, [M][Cout/8] bytes written by the tail's forward
  // apply (bn_kernels.hip): read instead of bny when set - 1/16 of y's bytes
  const uint8_t* bnmask = nullptr;
  // DGELU: the Linear's bias in the operands' 16-bit type (read instead of bn_mean when set)
  const uint16_t* bias16 = nullptr;
  // BNR with a downsample branch: the block's identity path was BN2(x2) (folded into the tail,
  // ops/bn.py _BN2AddReLUPair): also sum s3 = sum dz*(x2 - mean2) for that BatchNorm
  const uint16_t* bnx2;
  const float* bn_mean2;
  float* bp3;
  // BKN tap map: GEMM tap (r, s) reads weight tap (tr0 + trs*r, ts0 + tss*s) of the Rw x Sw
  // weight (stride-1 backward-data: the flip R-1-r; strided backward-data: one parity class)
  int Rw, Sw, tr0, trs, ts0, tss;
  // REMAP epilogue: GEMM output row (n, a, b) lands on row (n*oH + 2a + oph)*oW + 2b + opw
  int oH, oW, oph, opw;
  // BNB partials: column mt + bp_off of a [Cout][bp_ld] array (the strided backward-data's
  // parity classes write consecutive column ranges of one array)
  int bp_ld, bp_off;
  int f16;  // fp16 element type (bf16 otherwise)
  // split-K (small grids): block (tile, split) reduces K-steps [split*kps, +kps) into an fp32
  // partial tile of part [splits][M][Cout]; conv_split_epilogue_kernel sums the splits and runs
  // the epilogue (16-bit rounding, BN statistics, BNB/BNR) the unsplit kernel would have run
  float* part;
  int splits, kps;
  // Carried backward-weight reduce (carry.h): the last red.blocks blocks of the grid sum the
  // split-K partials of a backward-weight launched just before (the same conv's) instead of
  // computing a conv tile (AttachWgradReduce, kernels.h).  red.blocks = 0: none.
  ReduceCarry red;
  // Stream-K (conv_fwd_kernel<..., SK = true>): the first sk.G blocks split the tiles' K-steps
  // evenly; a tile shared by several blocks is finished by the block holding its last K-step
  // (see conv_fwd_kernel).  sk.G = 0: off.
  ConvSk sk;
};


template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// K-major operands (rows of the LDS image = k) use the transposing reads and the swizzle of
// mfma.h: wg_frag is its natural-k-order tr_frag.
template <int RB>
__device__ __forceinline__ bf16x8_t wg_frag(const unsigned char* img, int krow0, int col0, int lane) {
  return tr_frag<RB, false>(img, krow0, col0, lane);
}

// 16 zero bytes: the global source of glds lanes whose A row falls in the zero padding.
__device__ __attribute__((aligned(64))) uint4 g_conv_zero16[4];

// STAGES: LDS buffers of the K loop (2 = tile t+1 streams in while tile t is multiplied; 1 =
// half the LDS, twice the resident blocks - for K <= 2 steps, where there is nothing to
// overlap inside a block).  LDSEPI: stage the output tile through LDS for 16-byte row
// stores; otherwise each lane stores its accumulator column straight from registers.
// BKN: the B operand is the ORIGINAL weight w[co][r][s][ci] read as [k = co][n = ci] with the
// taps flipped - the backward-data GEMM without materialising a transposed weight copy - staged
// as K-major rows and taken with transposing LDS reads.
// BMT: block rows (128, or 256 = 4 MFMA row tiles per wave for more reuse per LDS byte).
// STATS: emit the BN partial sums (compiled out otherwise).
// BNB (backward-data of a conv whose input is relu(bn(x)), LDS epilogue only): while storing
// the input gradient dz, also sum that BatchNorm's backward statistics s1 = sum dz*mask,
// s2 = sum dz*mask*(x - mean) with mask = fma(x, a, b) > 0 recomputed from the BN input x and
// the forward coefficients - the BN backward then skips its statistics pass (ops/conv.py).
// BNR (with BNB): the BatchNorm was a residual-block tail y = relu(bn(x) + res) whose output
// fed this conv AND the next block's identity path: the stored gradient is the block tail's
// whole masked gradient dz = (g + g_identity) * (y > 0) - the tail's residual-path gradient
// and the input of its backward apply - and s1/s2 are summed from it.  Replaces the
// tail's backward-statistics pass (4 reads + 1 write of a 4C-channel tensor) by 3 reads here.
// REMAP (LDS epilogue): output rows scattered to one stride-2 parity class of a larger image
// (strided backward-data); ZSIB: also write zeros to the other three positions of each 2x2
// cell (1x1 / stride-2 backward-data, whose other classes receive no gradient).
// BNR2 (with BNR): the downsample-branch statistic s3 too (p.bnx2 / bn_mean2 / bp3).
// F16: fp16 operands and outputs (bf16 otherwise).
// NT: threads per block - 256 (4 waves, 2 blocks per CU) or 512 (8 waves, 2 per SIMD, one
// 256-row block per CU: twice the MFMA work per staged byte, the large-tile regime of
// cdna_hip_programming.md §5 where the 2-stage glds pipeline is MFMA-bound rather than
// L2-bound).
// HALO (3x3 / stride 1 / pad 1 with Ho = H, Wo = W, C % 64 == 0, 1 stage, 128 rows, not split):
// the K loop runs tap row r, channel block cb, then the three taps s of that row.  The 128 output
// rows of a tile are consecutive flattened pixels, so for tap (r, s) they read the consecutive
// input pixels m0 + (r-1)*W + (s-1) + row: ONE 136-row halo strip per (r, cb) serves all three s
// (the MFMA reads LDS row row + s), and each fragment row that falls in the zero padding (an
// image border, where the flattened index wraps into the neighbouring row or image) is zeroed
// in registers.  A operand bytes per three K-steps: 17 KiB instead of 48 KiB - the 128 x 128
// tile is bound by what one CU can pull from L2 into LDS (docs/DESIGN.md 7.1).
template <int BMT, int BN, int STAGES, bool LDSEPI, bool BKN, bool STATS = true, bool BNB = false,
          bool BNR = false, bool REMAP = false, bool ZSIB = false, bool BNR2 = false, bool F16 = false,
          int NT = conv::kThreads, bool SPLIT = false, bool HALO = false, int HB = 1, bool SK = false,
          bool DGELU = false, bool BREG = false>
__global__ __launch_bounds__(NT, (SK || BREG) ? 4 : 2) void conv_fwd_kernel(ConvFwdArgs p) {
  using namespace conv;
  constexpr int BM = BMT;
  constexpr int NW = NT / 64;         // waves
  // BREG: the B operand (weights) never touches LDS - every wave loads its own 32 output
  // channels' fragments straight from L2 into VGPRs (one 16-byte buffer load per lane and
  // k-slice, refilled right after the MFMAs that consumed it), and the LDS holds only A, double
  // buffered: the next A tile (1x1: the next K-step; HALO: the next halo strip, one per three
  // taps) streams in while this one is multiplied, in the same LDS as the single-stage tile's A + B
  constexpr int WCOL = BREG ? 32 : 64;  // output channels per wave
  constexpr int WN = BN / WCOL;       // waves along N
  constexpr int WM = NW / WN;         // waves along M
  constexpr int MI = BM / (WM * 32);  // 32-row MFMA tiles per wave
  constexpr int NI = WCOL / 32;       // 32-col MFMA tiles per wave
  static_assert(WM * WN == NW && MI >= 1 && MI * WM * 32 == BM, "conv_fwd_kernel: bad wave tiling");
  constexpr int A_PER_T = BM * 8 / NT;  // glds instructions per wave per K-step (A)
  constexpr int B_PER_T = BN * 8 / NT;  // (B)
  static_assert(!HALO || (BMT == 128 && STAGES == 1 && !BKN && !SPLIT && NT == conv::kThreads), "HALO config");
  static_assert(!SK || (STAGES == 1 && !HALO && !SPLIT && LDSEPI && !BNR2 && NT == conv::kThreads), "SK config");
  // DGELU (with BNB, a Linear's backward-data: ViT's fc2): the output is gu = g * gelu'(u + b)
  // with u = bnx (the fc1 GEMM output before its bias) and b = bn_mean (fp32 bias); bp1 gets the
  // per-tile column sums of gu (fc1's bias gradient), bp2 is not written
  static_assert(!DGELU || (BNB && !BNR && !STATS && !REMAP && LDSEPI && !SK), "DGELU config");
  static_assert(!BREG || (BMT == 128 && STAGES == 1 && LDSEPI && !BKN && !SPLIT && !SK && HB == 1 &&
                          NT == conv::kThreads && (BN == 128 || BN == 64)), "BREG config");
  constexpr int HROWS = 136;  // halo strip rows: 128 + 2, rounded up to whole 8-row glds instructions
  // HB (HALO): B taps staged per load phase - 1: one per K-step; 3: all three taps of the row
  // with the halo strip, one wait per three K-steps (more LDS: fewer resident blocks)
  static_assert(HB == 1 || (HALO && HB == 3), "HB");
  constexpr int A_BYTES = (HALO ? HROWS : BM) * kRowBytes, B_BYTES = BN * kRowBytes;
  constexpr int STAGE = A_BYTES + (BREG ? 0 : HB * B_BYTES);
  constexpr int NSTAGE = BREG ? 2 : STAGES;  // LDS operand buffers
  constexpr int C_STRIDE = BN * 2 + 16;  // epilogue image row stride (bytes), padded
  constexpr int RED = 2 * WM * BN * 4;   // BN-statistics cross-wave scratch
  // HALO: one zeroed 128-byte row after the K-loop buffers - a fragment row in the padding
  // reads it instead of being zeroed in registers (4 v_cndmask per fragment and K-step)
  constexpr int ZROW = NSTAGE * STAGE;
  constexpr int LDS_MAIN = NSTAGE * STAGE + (HALO ? kRowBytes : 0);
  // HALF: the 128-row, 4-wave LDS epilogue stages its output image 64 rows at a time, so the
  // epilogue (17 KiB + statistics scratch) fits under the 32 KiB K-loop buffer of a 128 x 128
  // tile: 5 resident blocks per CU instead of 4 (36 KiB), i.e. 25 % more bytes in flight for a
  // K loop that is latency-bound on its L2 -> LDS loads (profiles/conv_pmc_r2.md)
  constexpr bool HALF = DPT_CONV_HALF_EPI && LDSEPI && BM == 128 && NT == conv::kThreads && MI * 32 <= 64 && !BNB &&
                        !SPLIT;
  constexpr int EROWS = HALF ? 64 : BM;  // rows of the epilogue image
  constexpr int LDS_EPI = (LDSEPI ? EROWS * C_STRIDE : 0) + RED;
  constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS];
  if constexpr (NT == conv::kThreads) {
    if (p.red.blocks) {  // carried backward-weight reduce blocks (ConvFwdArgs::red)
      const int nconv = (int)gridDim.x - p.red.blocks;
      if ((int)blockIdx.x >= nconv) {
        carry_reduce(p.red, (int)blockIdx.x - nconv, lds);
        return;
      }
    }
  }

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles = (BM == 256 ? p.mt256 : p.m_tiles) * p.n_tiles;
  const int nk_all = (int)((int64_t)p.R * p.S * p.C / BK);

  // One output tile's K-steps [ks0, ks1) and its epilogue.  sk_role (stream-K only): 0 the whole
  // tile; 1 a leading part of it - publish the partial accumulators in slot sk_slot and stop; 2 its
  // trailing part - first add the partials of blocks sk_c0, sk_c0 + 8, .., sk_c1 (lower ids, one XCD).
  auto tile_body = [&](const int mt, const int nt, const int sp, const int ks0, const int ks1, const int sk_role,
                       const int sk_slot, const int sk_c0, const int sk_c1) {
  // stream-K runs this body in a loop: recompute the lane-dependent values per tile (an opaque
  // copy of the thread id), or the compiler hoists every per-lane address out of the loop and
  // keeps them live across the K loop (~100 more VGPRs: half the resident blocks)
  const int tid = SK ? conv::opaque_v((int)threadIdx.x) : (int)threadIdx.x, lane = tid & 63;
  const int wid = SK ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  // ---- per-lane A rows, pixel coordinates fixed for the whole K loop ----
  // One glds wave instruction fills 8 whole LDS rows lane-linearly: lane L of wave w owns
  // LDS slot L&7 of row (A_PER_T*w + i)*8 + L/8 and loads the chunk the swizzle puts there
  // (slot ^ ((row>>1)&7): the XOR is its own inverse).
  // Narrow inputs (C = 16/32): one 64-wide K-step spans 64/C consecutive taps along s, i.e.
  // consecutive input pixels, so a lane's 16-byte chunk sits at sub-tap (chunk*8)/C and the
  // address is unchanged (pixel stride = C elements); only its bounds check moves.
  // 32-bit element offsets and buffer loads into LDS (conv_check_offsets on the host): the
  // descriptors hold the base addresses in SGPRs, the zero padding is the range check (offset
  // kOOB), so a lane keeps 6 offsets instead of 6 64-bit pointers (fewer VGPRs: no spills at 5
  // waves per SIMD) and selects nothing but an offset.
  int hi0[A_PER_T], wi0[A_PER_T], aoff[A_PER_T];
  const int64_t HoWo = (int64_t)p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int arow = (wid * A_PER_T + i) * 8 + (lane >> 3);
    const int achunk = (lane & 7) ^ ((arow >> 1) & 7);
    const int64_t m = m0 + arow;
    if (m < p.M) {
      const int64_t n = m / HoWo;
      const int rem = (int)(m - n * HoWo);
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      hi0[i] = ho * p.stride - p.pad;
      wi0[i] = wo * p.stride - p.pad + (p.C < BK ? achunk * 8 / p.C : 0);
      aoff[i] = (int)(((n * p.H + hi0[i]) * (int64_t)p.W + wo * p.stride - p.pad) * p.C + achunk * 8);
    } else {
      hi0[i] = -(1 << 28);  // never in bounds
      wi0[i] = 0;
      aoff[i] = 0;
    }
  }
  const int64_t Kg = (int64_t)p.R * p.S * p.C;
  int woff[B_PER_T];
  constexpr int RBK = BN * 2;              // BKN image row bytes (BK rows of BN channels)
  constexpr int KN_RPI = 1024 / RBK;       // rows per glds instruction
#pragma unroll
  for (int i = 0; i < B_PER_T; ++i) {
    if (BKN) {
      // row k of the [BK][BN] image = output channel co of the original weight (this lane
      // fills chunk wg_slot(row, lane % chunks) of it)
      const int krow = (wid * B_PER_T + i) * KN_RPI + lane / (RBK / 16);
      const int kchunk = wg_slot<RBK>(krow, lane % (RBK / 16));
      woff[i] = krow * p.Rw * p.Sw * p.Cout + n0 + kchunk * 8;
    } else {
      const int brow = (wid * B_PER_T + i) * 8 + (lane >> 3);
      const int bchunk = (lane & 7) ^ ((brow >> 1) & 7);
      woff[i] = (int)((n0 + brow) * Kg) + bchunk * 8;
    }
  }
  constexpr uint32_t kOOB = 0xFFFFFF00u;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, 0, (int)((uint32_t)p.N * (uint32_t)(p.H * p.W * p.C) * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, (int)((uint32_t)(BKN ? p.Rw * p.Sw : p.R * p.S) * (uint32_t)(p.C * p.Cout) * 2u), 0x00020000);

  const int cblocks = p.C >= BK ? p.C / BK : 1;
  const int tps = p.C >= BK ? 1 : BK / p.C;  // taps per K-step (narrow inputs)

  // global -> LDS directly (no staging registers); wave-uniform LDS base per 1 KiB.
  auto stage = [&](int ks, int buf) {
    const int rs = (ks / cblocks) * tps, cb = ks - (ks / cblocks) * cblocks;
    const int r = rs / p.S, s = rs - r * p.S;
    const int koff = (r * p.W + s) * p.C + cb * BK;
    unsigned char* a = lds + buf * STAGE;
    unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int hi = hi0[i] + r, wi = wi0[i] + s;
      const bool ok = ((unsigned)hi < (unsigned)p.H) & ((unsigned)wi < (unsigned)p.W);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(a + (wid * A_PER_T + i) * 1024),
                                               16, ok ? (uint32_t)(aoff[i] + koff) * 2u : kOOB, 0, 0, 0);
    }
    // BKN: rows co = cb*BK + krow, mapped tap (tr0 + trs*r, ts0 + tss*s)
    const int wk = BKN ? (cb * BK * p.Rw * p.Sw + (p.tr0 + p.trs * r) * p.Sw + (p.ts0 + p.tss * s)) * p.Cout
                       : ks * BK;  // k = (r*S + s)*C + c: K-step ks is [64ks, 64ks+64)
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(b + (wid * B_PER_T + i) * 1024),
                                               16, (uint32_t)(woff[i] + wk) * 2u, 0, 0, 0);
  };

  f32x16_t acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  auto mma = [&](int buf) {
    const unsigned char* a = lds + buf * STAGE;
    const unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = kk * 2 + lh;
      bf16x8_t fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * (MI * 32) + i * 32 + lr;
        fa[i] = *reinterpret_cast<const bf16x8_t*>(a + row * kRowBytes + conv::swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (BKN) {
          fb[j] = wg_frag<RBK>(b, kk * 16, wn * WCOL + j * 32, lane);
        } else {
          const int row = wn * WCOL + j * 32 + lr;
          fb[j] = *reinterpret_cast<const bf16x8_t*>(b + row * kRowBytes + conv::swz(row, ch) * 16);
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = cmfma<F16>(fa[i], fb[j], acc[i][j]);
    }
  };

  if constexpr (BREG) {
    static_assert(NI == 1 && WM * MI * 32 == BM, "BREG: one 32-column B fragment per wave and k-slice");
    typedef unsigned breg_u32x4 __attribute__((ext_vector_type(4)));
    // this lane's B column is output channel n0 + wn*32 + lr; its 8 k of k-slice kk are the
    // K-step's elements [16kk + 8lh, +8): 16 contiguous bytes of the KRSC weight row
    const uint32_t bvoff = (uint32_t)((int64_t)(n0 + wn * WCOL + lr) * Kg + 8 * lh) * 2u;
    auto load_b = [&](int kbase, int kk) -> bf16x8_t {  // kbase: first k of the K-step (uniform)
      const breg_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, bvoff + (uint32_t)kk * 32u,
                                                                 (uint32_t)kbase * 2u, 0);
      return __builtin_bit_cast(bf16x8_t, v);
    };
    bf16x8_t fb[BK / 16];
    if constexpr (HALO) {
      int fho[MI], fwo[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int64_t m = m0 + wm * (MI * 32) + i * 32 + lr;
        if (m < p.M) {
          const int rem = (int)(m % HoWo);
          fho[i] = rem / p.Wo;
          fwo[i] = rem - fho[i] * p.Wo;
        } else {
          fho[i] = -(1 << 28);
          fwo[i] = 0;
        }
      }
      if (tid < kRowBytes / 16) *reinterpret_cast<uint4*>(lds + ZROW + tid * 16) = uint4{0u, 0u, 0u, 0u};
      const int64_t npix = (int64_t)p.N * p.H * p.W;
      auto stage_halo = [&](int r, int cb, int buf) {
        const int64_t q0 = m0 + (int64_t)(r - 1) * p.W - 1;
        unsigned char* hb = lds + buf * STAGE;
        for (int gi = wid; gi < HROWS / 8; gi += NW) {
          const int j = gi * 8 + (lane >> 3);
          const int chunk = (lane & 7) ^ ((j >> 1) & 7);
          const int64_t q = q0 + j;
          const bool ok = q >= 0 && q < npix;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rx, (__attribute__((address_space(3))) void*)(hb + gi * 1024), 16,
              ok ? (uint32_t)((int)q * p.C + cb * BK + chunk * 8) * 2u : kOOB, 0, 0, 0);
        }
      };
      auto kb = [&](int r, int sx, int cb) { return (r * 3 + sx) * p.C + cb * BK; };
      // tap (r, sx) of the strip in `buf` with the B fragments in fb; kn >= 0: refill fb with
      // the K-step at k = kn, one k-slice at a time right after its MFMAs
      auto mma_h = [&](int buf, int r, int sx, int kn) {
        const unsigned char* hb = lds + buf * STAGE;
        int abase[MI];
        const int hrow0 = wm * (MI * 32) + lr + sx;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bool ok = ((unsigned)(fho[i] + r - 1) < (unsigned)p.H) & ((unsigned)(fwo[i] + sx - 1) < (unsigned)p.W);
          abase[i] = ok ? buf * STAGE + (hrow0 + i * 32) * kRowBytes : ZROW;
        }
        (void)hb;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
          const int coff = conv::swz(hrow0, kk * 2 + lh) * 16;
          bf16x8_t fa[MI];
#pragma unroll
          for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(lds + (abase[i] | coff));
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][0] = cmfma<F16>(fa[i], fb[kk], acc[i][0]);
          if (kn >= 0) fb[kk] = load_b(kn, kk);
        }
      };
      const int T = 3 * cblocks;
      stage_halo(0, 0, 0);
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) fb[kk] = load_b(kb(0, 0, 0), kk);
      for (int t = 0; t < T; ++t) {
        const int r = t / cblocks, cb = t - r * cblocks, buf = t & 1;
        const int rn = (t + 1) / cblocks, cbn = (t + 1) - rn * cblocks;
        vmcnt_wait<0>();   // this strip and tap 0's B fragments
        __syncthreads();   // every wave's part of the strip is in; strip t-1's buffer is free
        mma_h(buf, r, 0, kb(r, 1, cb));
        vmcnt_wait<0>();   // tap 1's B fragments
        mma_h(buf, r, 1, kb(r, 2, cb));
        if (t + 1 < T) stage_halo(rn, cbn, buf ^ 1);  // lands while tap 2 is multiplied
        // tap 2's B fragments were issued before the strip: wait for them only
        if (t + 1 < T) {
          if (wid < (HROWS / 8) % NW) vmcnt_wait<(HROWS / 8 + NW - 1) / NW>();
          else vmcnt_wait<(HROWS / 8) / NW>();
        } else {
          vmcnt_wait<0>();
        }
        mma_h(buf, r, 2, t + 1 < T ? kb(rn, 0, cbn) : -1);
      }
      __syncthreads();  // the epilogue reuses the LDS
    } else {
      auto stage_a = [&](int ks, int buf) {
        const int rs = (ks / cblocks) * tps, cb = ks - (ks / cblocks) * cblocks;
        const int r = rs / p.S, s = rs - r * p.S;
        const int koff = (r * p.W + s) * p.C + cb * BK;
        unsigned char* a = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
          const int hi = hi0[i] + r, wi = wi0[i] + s;
          const bool ok = ((unsigned)hi < (unsigned)p.H) & ((unsigned)wi < (unsigned)p.W);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(a + (wid * A_PER_T + i) * 1024),
                                                   16, ok ? (uint32_t)(aoff[i] + koff) * 2u : kOOB, 0, 0, 0);
        }
      };
      auto mma_r = [&](int buf, int kn) {
        const unsigned char* a = lds + buf * STAGE;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
          const int ch = kk * 2 + lh;
          bf16x8_t fa[MI];
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int row = wm * (MI * 32) + i * 32 + lr;
            fa[i] = *reinterpret_cast<const bf16x8_t*>(a + row * kRowBytes + conv::swz(row, ch) * 16);
          }
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][0] = cmfma<F16>(fa[i], fb[kk], acc[i][0]);
          if (kn >= 0) fb[kk] = load_b(kn, kk);
        }
      };
      stage_a(ks0, 0);
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) fb[kk] = load_b(ks0 * BK, kk);
      for (int ks = ks0; ks < ks1; ++ks) {
        const int cur = (ks - ks0) & 1;
        vmcnt_wait<0>();   // A tile ks (LDS) and its B fragments (VGPRs)
        __syncthreads();   // every wave's part of A is in; the other buffer is free
        const bool more = ks + 1 < ks1;
        if (more) stage_a(ks + 1, cur ^ 1);
        mma_r(cur, more ? (ks + 1) * BK : -1);
      }
      __syncthreads();  // the epilogue reuses the LDS
    }
  } else if constexpr (HALO) {
    // per-lane fragment rows: output pixel coordinates, fixed for the whole loop
    int fho[MI], fwo[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * (MI * 32) + i * 32 + lr;
      if (m < p.M) {
        const int rem = (int)(m % HoWo);
        fho[i] = rem / p.Wo;
        fwo[i] = rem - fho[i] * p.Wo;
      } else {
        fho[i] = -(1 << 28);  // never valid
        fwo[i] = 0;
      }
    }
    if (tid < kRowBytes / 16) *reinterpret_cast<uint4*>(lds + ZROW + tid * 16) = uint4{0u, 0u, 0u, 0u};
    const int64_t npix = (int64_t)p.N * p.H * p.W;
    const unsigned char* hb = lds;            // halo strip [HROWS][128 B]
    unsigned char* bb = lds + A_BYTES;        // B [BN][128 B]
    auto stage_b = [&](int r, int sx, int cb) {
      const int wk = (r * 3 + sx) * p.C + cb * BK;
      unsigned char* bd = bb + (HB == 3 ? sx * B_BYTES : 0);
#pragma unroll
      for (int i = 0; i < B_PER_T; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bd + (wid * B_PER_T + i) * 1024),
                                                 16, (uint32_t)(woff[i] + wk) * 2u, 0, 0, 0);
    };
    auto stage_halo = [&](int r, int cb) {
      const int64_t q0 = m0 + (int64_t)(r - 1) * p.W - 1;  // input pixel of halo row 0
      for (int gi = wid; gi < HROWS / 8; gi += NW) {      // 17 instructions over the 4 waves
        const int j = gi * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ ((j >> 1) & 7);
        const int64_t q = q0 + j;
        const bool ok = q >= 0 && q < npix;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(hb + gi * 1024), 16,
            ok ? (uint32_t)((int)q * p.C + cb * BK + chunk * 8) * 2u : kOOB, 0, 0, 0);
      }
    };
    auto mma_h = [&](int r, int sx) {
      // row base per fragment (the zero row for padding); the swizzle term (hrow >> 1) & 7 is
      // the same for every i (rows 32 apart), so one chunk offset per kk serves all of them
      int abase[MI];
      const int hrow0 = wm * (MI * 32) + lr + sx;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bool ok = ((unsigned)(fho[i] + r - 1) < (unsigned)p.H) & ((unsigned)(fwo[i] + sx - 1) < (unsigned)p.W);
        abase[i] = ok ? (hrow0 + i * 32) * kRowBytes : ZROW;
      }
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        const int coff = conv::swz(hrow0, kk * 2 + lh) * 16;
        bf16x8_t fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(hb + (abase[i] | coff));
        const int ch = kk * 2 + lh;
        const unsigned char* bs = bb + (HB == 3 ? sx * B_BYTES : 0);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int row = wn * WCOL + j * 32 + lr;
          fb[j] = *reinterpret_cast<const bf16x8_t*>(bs + row * kRowBytes + conv::swz(row, ch) * 16);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = cmfma<F16>(fa[i], fb[j], acc[i][j]);
      }
    };
    for (int r = 0; r < 3; ++r) {
      for (int cb = 0; cb < cblocks; ++cb) {
        if constexpr (HB == 3) {
          stage_halo(r, cb);
#pragma unroll
          for (int sx = 0; sx < 3; ++sx) stage_b(r, sx, cb);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
#pragma unroll 1
          for (int sx = 0; sx < 3; ++sx) mma_h(r, sx);
          __syncthreads();
        } else {
#pragma unroll 1
          for (int sx = 0; sx < 3; ++sx) {
            if (sx == 0) stage_halo(r, cb);
            stage_b(r, sx, cb);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            mma_h(r, sx);
            __syncthreads();
          }
        }
      }
    }
  } else if constexpr (STAGES >= 3) {
    // Deep pipeline (cdna_hip_programming.md §5 "Pipelining across barriers"): STAGES-1 K-tiles
    // stay in flight across ONE raw s_barrier per K-step.  Iteration i waits (counted vmcnt)
    // until this wave's loads of tile i have landed, the barrier makes every wave's tile-i
    // loads visible AND proves every wave finished reading tile i-1, whose buffer then receives
    // tile i+STAGES-1 while tile i is multiplied.  No vmcnt(0) / __syncthreads inside the loop
    // (its fence would drain the in-flight tiles); all LDS lives in the one `lds` array.
    constexpr int PER = A_PER_T + B_PER_T;  // glds per wave per K-tile
    static_assert(STAGES <= 4, "pipeline depth");
    const int nk = ks1 - ks0;
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < nk) stage(ks0 + t, t);
    int buf = 0;
    for (int i = 0; i < nk; ++i) {
      const int ahead = min(STAGES - 2, nk - 1 - i);  // later tiles already issued
      if (ahead >= 2) vmcnt_wait<2 * PER>();
      else if (ahead == 1) vmcnt_wait<PER>();
      else vmcnt_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (i + STAGES - 1 < nk) {
        const int nb = buf == 0 ? STAGES - 1 : buf - 1;  // buffer of tile i-1 == (i+STAGES-1) % STAGES
        stage(ks0 + i + STAGES - 1, nb);
      }
      mma(buf);
      buf = buf + 1 == STAGES ? 0 : buf + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the epilogue reuses the LDS
  } else if (STAGES == 2) {
    stage(ks0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = ks0; ks < ks1; ++ks) {
      const int cur = (ks - ks0) & 1;
      if (ks + 1 < ks1) stage(ks + 1, cur ^ 1);
      mma(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    for (int ks = ks0; ks < ks1; ++ks) {
      stage(ks, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      mma(0);
      __syncthreads();
    }
  }
  if constexpr (SPLIT) {
    // fp32 partial tile straight from the accumulators: 32 lanes = 32 consecutive channels
    const int lr2 = lane & 31, lh2 = lane >> 5;
    float* out = p.part + (int64_t)sp * p.M * p.Cout;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * WCOL + j * 32 + lr2;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t m = m0 + wm * (MI * 32) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh2;
          if (m < p.M) out[m * p.Cout + col] = acc[i][j][e];
        }
      }
    return;
  }

  if constexpr (SK) {
    // float4 q of thread tid in slot b: ((b * ACC4 + q) * NT + tid) - coalesced per float4
    constexpr int ACC4 = MI * NI * 4;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) unsigned gu32;
    // one VGPR offset per thread and slot; the float4 index q rides in the SGPR offset
    const __amdgpu_buffer_rsrc_t rp =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.sk.part, 0, (int)p.sk.part_bytes, 0x00020000);
    // a consumer that gave up on a contributor poisons its tile with NaN: the step's non-finite
    // check then sees it, and the trainer fails loudly on the give-up counter (conv_sk_errors) at
    // its host touch points - a late publish can leave a flag set for a later launch
    __shared__ int sk_gave_up;
    if (sk_role == 2) {
      // consume: wave 0 polls each contributor's flag (relaxed, with sleeps, bounded), resets it for
      // the next launch, ONE agent-scope acquire, then every wave reads the partials
      if (wid == 0) {
        int gave_up = 0;
        for (int b = sk_c0; b <= sk_c1; b += 8) {
          unsigned spins = 0;
          while (__hip_atomic_load((gu32*)(p.sk.flags + b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 20)) {  // ~1 s: a contributor that never publishes - give up, count it
              if (lane == 0) __hip_atomic_fetch_add((gu32*)p.sk.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              gave_up = 1;
              break;
            }
          }
          if (lane == 0) __hip_atomic_store((gu32*)(p.sk.flags + b), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) sk_gave_up = gave_up;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (sk_gave_up) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = __builtin_nanf("");
      }
    }
    if (sk_role != 0) {
      // one pass over the accumulators, a float4 at a time, for both roles (keeps them in place:
      // separate store and load-add passes need ~30 more VGPRs, below 4 waves per SIMD).
      // role 1 publishes its slot (cdna_hip_programming.md Guideline 16, R1: write-through sc1
      // payload, every storing wave drains, the block barrier, ONE agent-scope flag store);
      // role 2 adds the contributors' slots in a fixed order (deterministic for a given grid)
      const bool pub = sk_role == 1;
      const int bfirst = pub ? sk_slot : sk_c0, blast = pub ? sk_slot : sk_c1;
      for (int b = bfirst; b <= blast; b += 8) {
        const int voff = (int)((((uint32_t)b * ACC4) * NT + tid) * 16u);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const int soff = ((i * NI + j) * 4 + e4) * NT * 16;
              if (pub) {
                const u32x4 v = {__float_as_uint(acc[i][j][4 * e4]), __float_as_uint(acc[i][j][4 * e4 + 1]),
                                 __float_as_uint(acc[i][j][4 * e4 + 2]), __float_as_uint(acc[i][j][4 * e4 + 3])};
                __builtin_amdgcn_raw_buffer_store_b128(v, rp, voff, soff, 16);
              } else {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rp, voff, soff, 0);
                acc[i][j][4 * e4] += __uint_as_float(v.x);
                acc[i][j][4 * e4 + 1] += __uint_as_float(v.y);
                acc[i][j][4 * e4 + 2] += __uint_as_float(v.z);
                acc[i][j][4 * e4 + 3] += __uint_as_float(v.w);
              }
            }
      }
      if (pub) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
          __hip_atomic_store((gu32*)(p.sk.flags + sk_slot), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
  }

  // ---- epilogue: 16-bit rounding, BN partial sums, stores ----
  // accumulator map (32x32x16): column = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5); pairs of
  // rows are rounded together by v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32
  const bool stats = STATS && p.psum != nullptr;
  float cs[NI], cq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { cs[j] = 0.f; cq[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wn * WCOL + j * 32 + lr;
      const int rbase = wm * (MI * 32) + i * 32 + 4 * lh;
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const int r0 = rbase + (e & 3) + 8 * (e >> 2);
        const f32x2_t v = {acc[i][j][e], acc[i][j][e + 1]};
        const uint32_t u = cpack<F16>(v);
        const uint16_t h0 = (uint16_t)u, h1 = (uint16_t)(u >> 16);
        if (LDSEPI) {
          if (!HALF) {
            *reinterpret_cast<uint16_t*>(lds + r0 * C_STRIDE + col * 2) = h0;
            *reinterpret_cast<uint16_t*>(lds + (r0 + 1) * C_STRIDE + col * 2) = h1;
          }
        } else {
          if (m0 + r0 < p.M) p.y[(m0 + r0) * p.Cout + n0 + col] = h0;
          if (m0 + r0 + 1 < p.M) p.y[(m0 + r0 + 1) * p.Cout + n0 + col] = h1;
        }
        if (STATS) {
          // rows past M hold exact zeros (their A rows were zero-filled): no effect on the sums
          const float f0 = cunpack<F16>(u, 0), f1 = cunpack<F16>(u, 1);
          cs[j] += f0 + f1;
          cq[j] = __builtin_fmaf(f0, f0, __builtin_fmaf(f1, f1, cq[j]));
        }
      }
    }
  float* red = reinterpret_cast<float*>(lds + (LDSEPI ? EROWS * C_STRIDE : 0));  // [2][WM][BN]
  if (stats) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
      if (lh == 0) {
        const int col = wn * WCOL + j * 32 + lr;
        red[wm * BN + col] = cs[j];
        red[WM * BN + wm * BN + col] = cq[j];
      }
    }
  }
  if (!LDSEPI && !stats) return;
  __syncthreads();
  if (stats && tid < BN) {
    // partials are per 128-row sub-tile (the layout is independent of BM): waves whose rows
    // fall in the same sub-tile are combined
    constexpr int SUB = BM / 128, WPS = WM / SUB;  // sub-tiles per block, waves per sub-tile
#pragma unroll
    for (int st = 0; st < SUB; ++st) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = st * WPS; w < (st + 1) * WPS; ++w) { s += red[w * BN + tid]; q += red[WM * BN + w * BN + tid]; }
      const int sub = mt * SUB + st;
      if ((int64_t)sub * 128 < p.M) {
        p.psum[(int64_t)(n0 + tid) * p.m_tiles + sub] = s;
        p.psq[(int64_t)(n0 + tid) * p.m_tiles + sub] = q;
      }
    }
  }
  if (LDSEPI) {
    constexpr int CPR = BN / 8;          // 16-byte chunks per output row
    constexpr int RPP = NT / CPR;  // rows per pass
    constexpr int NPASS = EROWS / RPP;
    // global operands of the BN epilogues are loaded a group of passes at a time, before any
    // store of the group (the output may alias nothing, but the compiler cannot know that)
    constexpr int GRP = NPASS < 4 ? NPASS : 4;
    const int oc = tid % CPR, orow = tid / CPR;
    float ba[8], bb[8], bm[8], s1[8], s2[8], bm2[8], s3[8];
    constexpr bool two = BNR && BNR2;
    if (BNB) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = n0 + oc * 8 + k;
        ba[k] = (BNR || DGELU) ? 0.f : p.bn_coef[c];
        bb[k] = (BNR || DGELU) ? 0.f : p.bn_coef[p.Cout + c];
        bm[k] = (DGELU && p.bias16 != nullptr) ? cunpack<F16>((uint32_t)p.bias16[c], 0) : p.bn_mean[c];
        bm2[k] = two ? p.bn_mean2[c] : 0.f;
        s1[k] = 0.f;
        s2[k] = 0.f;
        s3[k] = 0.f;
      }
    }
    // destination row of GEMM row m (REMAP: its pixel in one parity class of the larger image)
    auto grow = [&](int64_t m) -> int64_t {
      if (!REMAP) return m;
      const uint32_t mm = (uint32_t)m, hw = (uint32_t)HoWo;
      const uint32_t img = mm / hw, rem = mm - img * hw;
      const int a = (int)(rem / (uint32_t)p.Wo), b = (int)(rem - (uint32_t)a * (uint32_t)p.Wo);
      return ((int64_t)img * p.oH + 2 * a + p.oph) * p.oW + 2 * b + p.opw;
    };
    for (int half = 0; half < (HALF ? 2 : 1); ++half) {
    if (HALF) {
      // this half's 64 rows: the waves that own them round their accumulators into the image
      if (half) __syncthreads();  // every thread is done reading the first half
      if ((wm * MI * 32) / 64 == half) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int col = wn * WCOL + j * 32 + lr;
            const int rbase = wm * (MI * 32) + i * 32 + 4 * lh - half * 64;
#pragma unroll
            for (int e = 0; e < 16; e += 2) {
              const int r0 = rbase + (e & 3) + 8 * (e >> 2);
              const f32x2_t v = {acc[i][j][e], acc[i][j][e + 1]};
              const uint32_t u = cpack<F16>(v);
              *reinterpret_cast<uint16_t*>(lds + r0 * C_STRIDE + col * 2) = (uint16_t)u;
              *reinterpret_cast<uint16_t*>(lds + (r0 + 1) * C_STRIDE + col * 2) = (uint16_t)(u >> 16);
            }
          }
      }
      __syncthreads();
    }
    const int64_t mh = m0 + half * EROWS;  // first global row of the image
#pragma unroll
    for (int g0 = 0; g0 < NPASS; g0 += GRP) {
      uint4 xv[GRP], yv[GRP], rv[GRP], x2v[GRP];
      uint32_t mv[GRP];
      if (BNB) {
#pragma unroll
        for (int q = 0; q < GRP; ++q) {
          const int64_t m = mh + (g0 + q) * RPP + orow;
          const int64_t off = grow(m < p.M ? m : 0) * p.Cout + n0 + oc * 8;
          xv[q] = *reinterpret_cast<const uint4*>(p.bnx + off);
          if (BNR) {
            if (p.bnmask != nullptr) {
              mv[q] = p.bnmask[off >> 3];
              yv[q] = make_uint4(0u, 0u, 0u, 0u);
            } else {
              mv[q] = 0u;
              yv[q] = *reinterpret_cast<const uint4*>(p.bny + off);
            }
            rv[q] = *reinterpret_cast<const uint4*>(p.bnres + off);
            if (two) x2v[q] = *reinterpret_cast<const uint4*>(p.bnx2 + off);
            else x2v[q] = make_uint4(0u, 0u, 0u, 0u);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < GRP; ++q) {
        const int row = (g0 + q) * RPP + orow;
        const int64_t m = mh + row;
        if (m < p.M) {
          uint4 v = *reinterpret_cast<const uint4*>(lds + row * C_STRIDE + oc * 16);
          if (BNB) {
            const uint32_t gu[4] = {v.x, v.y, v.z, v.w};
            const uint32_t xu[4] = {xv[q].x, xv[q].y, xv[q].z, xv[q].w};
            const uint32_t yu[4] = {yv[q].x, yv[q].y, yv[q].z, yv[q].w};
            const uint32_t ru[4] = {rv[q].x, rv[q].y, rv[q].z, rv[q].w};
            const uint32_t x2u[4] = {x2v[q].x, x2v[q].y, x2v[q].z, x2v[q].w};
            uint32_t du[4];
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) {
              float dzp[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int k = 2 * k2 + h;
                const float g = cunpack<F16>(gu[k2], h);
                const float x = cunpack<F16>(xu[k2], h);
                float dz;
                if (DGELU) {
                  dz = g * gelu_grad(x + bm[k]);
                } else if (BNR) {
                  const bool pos = p.bnmask != nullptr ? ((mv[q] >> k) & 1u) != 0u : cunpack<F16>(yu[k2], h) > 0.0f;
                  const float rr = cunpack<F16>(ru[k2], h);
                  dz = pos ? g + rr : 0.0f;
                } else {
                  dz = __builtin_fmaf(x, ba[k], bb[k]) > 0.0f ? g : 0.0f;
                }
                dzp[h] = dz;
                s1[k] += dz;
                if (!DGELU) s2[k] = __builtin_fmaf(dz, x - bm[k], s2[k]);
                if (two) {
                  const float x2 = cunpack<F16>(x2u[k2], h);
                  s3[k] = __builtin_fmaf(dz, x2 - bm2[k], s3[k]);
                }
              }
              if (BNR || DGELU) {
                const f32x2_t d2 = {dzp[0], dzp[1]};
                du[k2] = cpack<F16>(d2);
              }
            }
            if (BNR || DGELU) v = make_uint4(du[0], du[1], du[2], du[3]);
          }
          if (REMAP) {
            const int64_t gr = grow(m);
            const int oy = (int)((gr / p.oW) % p.oH), ox = (int)(gr % p.oW);
            uint16_t* orow = p.y + gr * p.Cout + n0 + oc * 8;
            *reinterpret_cast<uint4*>(orow) = v;
            if (ZSIB) {
              const uint4 z = make_uint4(0u, 0u, 0u, 0u);
              const int64_t rs = (int64_t)p.oW * p.Cout;
              if (ox + 1 < p.oW) *reinterpret_cast<uint4*>(orow + p.Cout) = z;
              if (oy + 1 < p.oH) {
                *reinterpret_cast<uint4*>(orow + rs) = z;
                if (ox + 1 < p.oW) *reinterpret_cast<uint4*>(orow + rs + p.Cout) = z;
              }
            }
          } else {
            *reinterpret_cast<uint4*>(p.y + m * p.Cout + n0 + oc * 8) = v;
          }
        }
      }
    }
    }  // half
    if (BNB) {
      // threads sharing a channel group: orow = tid / CPR -> lanes l, l+CPR, ... of a wave, then
      // the NW waves through LDS (the epilogue image is no longer read: reuse its space)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int off = CPR; off < 64; off <<= 1) {
          s1[k] += __shfl_xor(s1[k], off, 64);
          if (!DGELU) s2[k] += __shfl_xor(s2[k], off, 64);
          if (two) s3[k] += __shfl_xor(s3[k], off, 64);
        }
      }
      __syncthreads();
      constexpr int NS3 = two ? 3 : 2;
      float* bred = reinterpret_cast<float*>(lds);  // [NW waves][NS3][BN]
      if (lane < CPR) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          bred[(wid * NS3) * BN + oc * 8 + k] = s1[k];
          bred[(wid * NS3 + 1) * BN + oc * 8 + k] = s2[k];
          if (two) bred[(wid * NS3 + 2) * BN + oc * 8 + k] = s3[k];
        }
      }
      __syncthreads();
      if (tid < BN) {
        float a = 0.f, b = 0.f, c3 = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          a += bred[(w * NS3) * BN + tid];
          b += bred[(w * NS3 + 1) * BN + tid];
          if (two) c3 += bred[(w * NS3 + 2) * BN + tid];
        }
        // partials stay one column per 128-row sub-tile whatever BM is: a 256-row block
        // writes its sum in its first column and zero in the second
        constexpr int SUBB = BM / 128;
        // DGELU: [m_tiles][Cout] rows (the bias gradient is then one sum_partials pass)
        const int64_t pc = DGELU ? (int64_t)mt * p.Cout + n0 + tid
                                 : (int64_t)(n0 + tid) * p.bp_ld + p.bp_off + (int64_t)mt * SUBB;
        p.bp1[pc] = a;
        if (!DGELU) p.bp2[pc] = b;
        if (two) p.bp3[pc] = c3;
        if (SUBB == 2 && ((int64_t)mt * 2 + 1) * 128 < p.M) {
          p.bp1[pc + 1] = 0.f;
          if (!DGELU) p.bp2[pc + 1] = 0.f;
          if (two) p.bp3[pc + 1] = 0.f;
        }
      }
    }
  }
  };  // tile_body

  if constexpr (SK) {
    // Stream-K, per XCD: the tiles are cut into 8 contiguous groups (consecutive tiles share A
    // rows: one L2) and group x = blockIdx & 7 is spread over its G/8 blocks x, x+8, x+16, ...
    // (the dispatcher deals consecutive block ids round-robin over the XCDs).  Block i of a group
    // owns iterations [I*i/g, I*(i+1)/g) of the group's tile-major (tile, K-step) space: its whole
    // tiles first, then its last segment (stopping inside a tile: publish the partial), then its
    // first segment (starting inside a tile: finish it with the partials of the group's lower
    // blocks).  Every wait points at a lower block id, and lower ids never wait on higher ones,
    // so the grid drains whatever the residency.
    const uint32_t g = (uint32_t)p.sk.G >> 3, nk = (uint32_t)nk_all;
    const uint32_t x = blockIdx.x & 7, i = blockIdx.x >> 3;
    const uint32_t t_lo = (uint32_t)tiles * x / 8, t_hi = (uint32_t)tiles * (x + 1) / 8;
    const uint32_t I = (t_hi - t_lo) * nk;  // I * g < 2^32 (conv_sk_blocks)
    const uint32_t s0 = I * i / g, s1 = I * (i + 1) / g;
    // segments in run order: those after the first (whole tiles, then the last), then the first
    const uint32_t f1 = min(s1, (s0 / nk + 1) * nk);
    const uint32_t nseg = s1 > s0 ? 1u + (s1 > f1 ? (s1 - 1) / nk - f1 / nk + 1 : 0u) : 0u;
    for (uint32_t q = 0; q < nseg; ++q) {
      const uint32_t b0 = q + 1 == nseg ? s0 : f1 + q * nk;  // f1 is a tile boundary when s1 > f1
      const uint32_t tl = b0 / nk;
      const uint32_t b1 = min(s1, (tl + 1) * nk);
      const int k0 = (int)(b0 - tl * nk), k1 = (int)(b1 - tl * nk);
      int role = 0, c0 = 0, c1 = -1;
      if (k0 > 0 && k1 == nk_all) {
        role = 2;
        const uint32_t it0 = tl * nk;  // contributors: the blocks of the group holding [it0, b0)
        uint32_t c = it0 * g / I;
        while (c + 1 < i && I * (c + 1) / g <= it0) ++c;
        while (c > 0 && I * c / g > it0) --c;
        c0 = (int)(x + 8 * c);
        c1 = (int)blockIdx.x - 8;
      } else if (k1 < nk_all) {
        role = 1;
      }
      if (q > 0) __syncthreads();  // the previous tile's epilogue is done with the LDS
      const int t = (int)(t_lo + tl);
      tile_body(t / p.n_tiles, t % p.n_tiles, 0, k0, k1, role, (int)blockIdx.x, c0, c1);
    }
  } else {
    const int nsplit = SPLIT ? p.splits : 1;
    const int bid0 = conv::xcd_remap(blockIdx.x, tiles * nsplit);
    // split-K: the splits of one tile are consecutive ids (one XCD, shared A/B rows in its L2)
    const int sp = SPLIT ? bid0 % nsplit : 0;
    const int bid = SPLIT ? bid0 / nsplit : bid0;
    const int ks0 = SPLIT ? sp * p.kps : 0;
    const int ks1 = SPLIT ? min(nk_all, ks0 + p.kps) : nk_all;
    tile_body(bid / p.n_tiles, bid % p.n_tiles, sp, ks0, ks1, 0, 0, 0, -1);
  }
}

// ---- split-K epilogue: sum the fp32 partial tiles, then the conv epilogue --------------------
// One block per (16-row slab, 64-channel group), 256 threads = 8 channel groups x 16 rows x 2
// split halves (each half sums every other split; LDS joins them) - small-grid convs have few
// rows, so the slab is kept short to spread the split sums over many blocks.  Identical
// per-element math to conv_fwd_kernel's LDS epilogue (16-bit rounding of the sum, BN
// statistics from the rounded values; BNB: s1 = sum dz, s2 = sum dz*(x - mean) with the BN+ReLU
// mask; BNR: dz = (g + res) * (y > 0) is what is stored; BNR2: s3 = sum dz*(x2 - mean2)).
// Statistics partials: one column per 16-row slab, [C][ceil(M/16)] (conv_split_cols).
constexpr int kSplitRows = 16;
template <bool STATS, bool BNB, bool BNR, bool BNR2, bool REMAP, bool ZSIB, bool F16>
__global__ __launch_bounds__(256) void conv_split_epilogue_kernel(ConvFwdArgs p) {
  const int rb = blockIdx.x, cgb = blockIdx.y, cols = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int oc = tid & 7, orow = (tid >> 3) & 15, half = tid >> 7;
  const int c0 = cgb * 64 + oc * 8;
  const int64_t MC = p.M * p.Cout;
  const int64_t m = (int64_t)rb * kSplitRows + orow;
  const bool live = m < p.M;
  const int64_t poff = (live ? m : 0) * p.Cout + c0;  // partials: GEMM row
  // destination row (REMAP: the GEMM row's pixel in one stride-2 parity class of dx)
  int64_t grow = live ? m : 0;
  int oy = 0, ox = 0;
  if (REMAP) {
    const int64_t hw = (int64_t)p.Ho * p.Wo, img = grow / hw, rem = grow - img * hw;
    const int a = (int)(rem / p.Wo), b = (int)(rem - (int64_t)a * p.Wo);
    oy = 2 * a + p.oph;
    ox = 2 * b + p.opw;
    grow = (img * p.oH + oy) * p.oW + ox;
  }
  const int64_t off = grow * p.Cout + c0;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = 0.f;
  if (live) {
    for (int sp = half; sp < p.splits; sp += 2) {
      const float4* q = reinterpret_cast<const float4*>(p.part + sp * MC + poff);
      const float4 a = q[0], b = q[1];
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
  }
  __shared__ float join[128][9];
  __shared__ float red[2][3][64];
  if (half == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) join[tid & 127][k] = v[k];
  }
  __syncthreads();
  constexpr bool two = BNR && BNR2;
  float q0[8], q1[8], q2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q0[k] = q1[k] = q2[k] = 0.f;
  if (half == 0 && live) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += join[tid][k];
    uint32_t u[4];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) u[k2] = cpack<F16>(f32x2_t{v[2 * k2], v[2 * k2 + 1]});
    if (BNB) {
      const uint4 xv = *reinterpret_cast<const uint4*>(p.bnx + off);
      uint4 yv = make_uint4(0u, 0u, 0u, 0u), rv = yv, x2v = yv;
      uint32_t mv = 0u;
      if (BNR) {
        if (p.bnmask != nullptr) mv = p.bnmask[off >> 3];
        else yv = *reinterpret_cast<const uint4*>(p.bny + off);
        rv = *reinterpret_cast<const uint4*>(p.bnres + off);
        if (two) x2v = *reinterpret_cast<const uint4*>(p.bnx2 + off);
      }
      const uint32_t xu[4] = {xv.x, xv.y, xv.z, xv.w}, yu[4] = {yv.x, yv.y, yv.z, yv.w};
      const uint32_t ru[4] = {rv.x, rv.y, rv.z, rv.w}, x2u[4] = {x2v.x, x2v.y, x2v.z, x2v.w};
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        float dzp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * k2 + h, c = c0 + k;
          const float g = cunpack<F16>(u[k2], h);
          const float x = cunpack<F16>(xu[k2], h);
          float dz;
          if (BNR) {
            const bool pos = p.bnmask != nullptr ? ((mv >> k) & 1u) != 0u : cunpack<F16>(yu[k2], h) > 0.0f;
            dz = pos ? g + cunpack<F16>(ru[k2], h) : 0.0f;
          } else {
            dz = __builtin_fmaf(x, p.bn_coef[c], p.bn_coef[p.Cout + c]) > 0.0f ? g : 0.0f;
          }
          dzp[h] = dz;
          q0[k] = dz;
          q1[k] = dz * (x - p.bn_mean[c]);
          if (two) q2[k] = dz * (cunpack<F16>(x2u[k2], h) - p.bn_mean2[c]);
        }
        if (BNR) u[k2] = cpack<F16>(f32x2_t{dzp[0], dzp[1]});
      }
    }
    if (STATS) {
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float f = cunpack<F16>(u[k2], h);
          q0[2 * k2 + h] = f;
          q1[2 * k2 + h] = f * f;
        }
    }
    *reinterpret_cast<uint4*>(p.y + off) = make_uint4(u[0], u[1], u[2], u[3]);
    if (ZSIB) {  // the three other positions of the 2x2 cell get no gradient (1x1 / stride 2)
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      const int64_t rs = (int64_t)p.oW * p.Cout;
      if (ox + 1 < p.oW) *reinterpret_cast<uint4*>(p.y + off + p.Cout) = z;
      if (oy + 1 < p.oH) {
        *reinterpret_cast<uint4*>(p.y + off + rs) = z;
        if (ox + 1 < p.oW) *reinterpret_cast<uint4*>(p.y + off + rs + p.Cout) = z;
      }
    }
  }
  if (!STATS && !BNB) return;
  // the 16 rows of a channel group: lanes l, l+8, ..., l+56 of waves 0 and 1
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      q0[k] += __shfl_xor(q0[k], o, 64);
      q1[k] += __shfl_xor(q1[k], o, 64);
      if (two) q2[k] += __shfl_xor(q2[k], o, 64);
    }
  }
  if (wid < 2 && lane < 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[wid][0][oc * 8 + k] = q0[k];
      red[wid][1][oc * 8 + k] = q1[k];
      if (two) red[wid][2][oc * 8 + k] = q2[k];
    }
  }
  __syncthreads();
  if (tid < 64) {
    const float a = red[0][0][tid] + red[1][0][tid], b = red[0][1][tid] + red[1][1][tid];
    const int64_t c = (int64_t)cgb * 64 + tid;
    if (STATS) {
      p.psum[c * cols + rb] = a;
      p.psq[c * cols + rb] = b;
    } else {
      const int64_t pc = c * p.bp_ld + p.bp_off + rb;
      p.bp1[pc] = a;
      p.bp2[pc] = b;
      if (two) p.bp3[pc] = red[0][2][tid] + red[1][2][tid];
    }
  }
}

// ---- forward, software-pipelined: BK = 32 stages, NS-deep LDS ring, counted vmcnt -------------
//
// PMC on the 1-stage kernel (3x3 256->256 @14x14, batch 256) showed 30% MFMA busy with 36% of
// wave cycles parked in s_waitcnt/barrier: each block waits a full HBM round trip per K-step.
// Here a block keeps NS-1 K-tiles in flight: tile t+NS-1 is issued (global_load_lds) right
// after the barrier that retires tile t, the barrier is a raw s_barrier (no vmcnt(0) fence),
// and the wait before it is counted - vmcnt(G * tiles still allowed in flight), G = glds
// instructions per wave per tile (cdna_hip_programming.md "Pipelining across barriers").
// LDS rows are 64 B (32 bf16); 16-byte chunks are XOR-swizzled by (row>>2)&3 so the 16 rows a
// ds_read_b128 quarter-wave touches (4 per 256-B bank row) land on distinct banks.
// Epilogue: pairs of accumulators are rounded with v_cvt_pk_bf16_f32 and written to a padded
// LDS image, then stored as 16-byte rows; BN statistics (STATS) from the rounded values.
template <int BN, int NS, bool STATS>
__global__ __launch_bounds__(conv::kThreads, 2) void conv_fwd_pipe_kernel(ConvFwdArgs p) {
  using namespace conv;
  constexpr int BM = 128, BKP = 32, RB = BKP * 2;  // 64-byte LDS rows
  constexpr int WN = BN / 64, WM = 4 / WN, MI = BM / (WM * 32), NI = 2;
  constexpr int A_G = BM * RB / 1024 / 4, B_G = BN * RB / 1024 / 4;  // glds per wave per stage
  constexpr int G = A_G + B_G;
  constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB;
  constexpr int C_STRIDE = BN * 2 + 16;
  constexpr int RED = 2 * WM * BN * 4;
  constexpr int LDS_MAIN = NS * STAGE, LDS_EPI = BM * C_STRIDE + RED;
  constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  static_assert(NS >= 2 && NS <= 4, "pipeline depth 2..4");
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int bid = conv::xcd_remap(blockIdx.x, p.m_tiles * p.n_tiles);
  const int mt = bid / p.n_tiles, nt = bid % p.n_tiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  // glds lane-linear fill: one wave instruction = 16 rows of 64 B; lane L -> row base + L/4,
  // slot L&3, loading the chunk the swizzle puts in that slot.
  int hi0[A_G], wi0[A_G];
  int64_t abase[A_G];
  const int64_t HoWo = (int64_t)p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int row = (wid * A_G + i) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const int64_t m = m0 + row;
    if (m < p.M) {
      const int64_t n = m / HoWo;
      const int rem = (int)(m - n * HoWo);
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      hi0[i] = ho * p.stride - p.pad;
      wi0[i] = wo * p.stride - p.pad;
      abase[i] = ((n * p.H + hi0[i]) * (int64_t)p.W + wi0[i]) * p.C + chunk * 8;
    } else {
      hi0[i] = -(1 << 28);
      wi0[i] = 0;
      abase[i] = 0;
    }
  }
  const int64_t Kg = (int64_t)p.R * p.S * p.C;
  const uint16_t* wrow[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int row = (wid * B_G + i) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    wrow[i] = p.w + (int64_t)(n0 + row) * Kg + chunk * 8;
  }
  const int cblocks = p.C / BKP;
  const int nk = p.R * p.S * cblocks;

  auto stage = [&](int ks, int buf) {
    const int rs = ks / cblocks, cb = ks - rs * cblocks;
    const int r = rs / p.S, s = rs - r * p.S;
    const int64_t koff = ((int64_t)r * p.W + s) * p.C + cb * BKP;
    unsigned char* a = lds + buf * STAGE;
    unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const int hi = hi0[i] + r, wi = wi0[i] + s;
      const bool ok = (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
      const void* src = ok ? (const void*)(p.x + abase[i] + koff) : (const void*)g_conv_zero16;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(a + (wid * A_G + i) * 1024),
                                       16, 0, 0);
    }
    const int64_t wk = (int64_t)rs * p.C + cb * BKP;
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(wrow[i] + wk),
                                       (__attribute__((address_space(3))) void*)(b + (wid * B_G + i) * 1024),
                                       16, 0, 0);
  };

  f32x16_t acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int lr = lane & 31, lh = lane >> 5;
  // fragment byte offsets inside a stage (loop-invariant)
  int aoff[2][MI], boff[2][NI];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 2 + lh;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * (MI * 32) + i * 32 + lr;
      aoff[kk][i] = row * RB + ((ch ^ ((row >> 2) & 3)) << 4);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * 64 + j * 32 + lr;
      boff[kk][j] = A_BYTES + row * RB + ((ch ^ ((row >> 2) & 3)) << 4);
    }
  }

#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) stage(t, t);
  for (int ks = 0; ks < nk; ++ks) {
    const int ahead = min(NS - 2, nk - 1 - ks);  // tiles allowed to stay in flight
    if (ahead >= 2) vmcnt_wait<2 * G>();
    else if (ahead == 1) vmcnt_wait<G>();
    else vmcnt_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (ks + NS - 1 < nk) stage(ks + NS - 1, (ks + NS - 1) % NS);
    const unsigned char* base = lds + (ks % NS) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(base + aoff[kk][i]);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(base + boff[kk][j]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue ----
  float cs[NI], cq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { cs[j] = 0.f; cq[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      unsigned char* colp = lds + (wn * 64 + j * 32 + lr) * 2 + (wm * (MI * 32) + i * 32 + 4 * lh) * C_STRIDE;
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const f32x2_t v = {acc[i][j][e], acc[i][j][e + 1]};
        const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
        const int r0 = (e & 3) + 8 * (e >> 2);  // rows r0, r0+1 of this lane's column
        *reinterpret_cast<uint16_t*>(colp + r0 * C_STRIDE) = (uint16_t)u;
        *reinterpret_cast<uint16_t*>(colp + (r0 + 1) * C_STRIDE) = (uint16_t)(u >> 16);
        if (STATS) {
          const float f0 = __uint_as_float(u << 16), f1 = __uint_as_float(u & 0xffff0000u);
          cs[j] += f0 + f1;
          cq[j] = __builtin_fmaf(f0, f0, __builtin_fmaf(f1, f1, cq[j]));
        }
      }
    }
  float* red = reinterpret_cast<float*>(lds + BM * C_STRIDE);  // [2][WM][BN]
  if (STATS) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
      if (lh == 0) {
        const int col = wn * 64 + j * 32 + lr;
        red[wm * BN + col] = cs[j];
        red[WM * BN + wm * BN + col] = cq[j];
      }
    }
  }
  __syncthreads();
  if (STATS && tid < BN) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) { s += red[w * BN + tid]; q += red[WM * BN + w * BN + tid]; }
    p.psum[(int64_t)(n0 + tid) * p.m_tiles + mt] = s;
    p.psq[(int64_t)(n0 + tid) * p.m_tiles + mt] = q;
  }
  constexpr int CPR = BN / 8, RPP = kThreads / CPR;
  const int oc = tid % CPR, orow = tid / CPR;
#pragma unroll
  for (int r0 = 0; r0 < BM; r0 += RPP) {
    const int row = r0 + orow;
    const int64_t m = m0 + row;
    if (m < p.M) {
      const uint4 v = *reinterpret_cast<const uint4*>(lds + row * C_STRIDE + oc * 16);
      *reinterpret_cast<uint4*>(p.y + m * p.Cout + n0 + oc * 8) = v;
    }
  }
}

// ---- backward-weight: dW[co, (r,s,ci)] = sum_m dy[m, co] * x[pix(m) + (r,s), ci] -------------
//
// The reduction runs over pixels, the ROW index of both channels_last operands, so both are
// staged into LDS exactly as they sit in memory ([pixel][channel] rows, filled by glds) and
// the MFMA fragments (8 consecutive pixels of one channel per lane) are taken with the gfx950
// transposing read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).  Row chunks are
// XOR-swizzled (256-B rows: ch ^ ((row&3)<<2 | (row>>2)&3); 128-B rows: ch ^ ((row>>1)&1)<<2
// | (row>>2)&3) so the 4 rows x 32 columns one 32-lane half reads hit 64 distinct banks.
// Output tiles: BMW output channels x BNW input channels of one tap (r,s); the pixel range is
// split over `splits` blocks per tile (split-K), each writing an fp32 partial
// [split][Cout][R*S*Cin] summed by conv_wgrad_reduce_kernel (deterministic, no atomics).
struct FastDiv {  // n / d for 0 <= n < 2^31 via a 32-bit multiply-high
  uint32_t d, mul, shr;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

struct ConvWgradArgs {
  const uint16_t* dy;  // [N, Ho, Wo, Cout]
  const uint16_t* x;   // [N, H, W, C]
  float* part;         // [splits][Cout][R*S*C]
  int N, H, W, C, Ho, Wo, Cout, R, S, stride, pad;
  int M;               // N*Ho*Wo (< 2^31)
  int co_tiles, n_tiles, splits, steps_per_split;
  FastDiv div_wo, div_howo;
  int direct;          // 1x1, stride 1, pad 0: x row = dy row
  // K-step advance of a lane's x row by BKP = 64 pixels, 64 = A*Ho*Wo + B*Wo + Cq (host-side):
  // wi += dw_step (wrap: -wwrap, hi += stride), hi += dh_step (wrap: -hwrap); the element
  // offset moves by dp_w / dp_wwrap / dp_h / dp_hwrap alongside (image carries folded in)
  int dw_step, wwrap, dh_step, hwrap;
  int dp_w, dp_wwrap, dp_h, dp_hwrap;
  int f16;             // fp16 operands (bf16 otherwise)
  // conv_wgrad_halo_kernel: padded pixel count N*H*(W+2) and divisors by W+2 and H
  int Mp = 0;
  FastDiv div_wp{}, div_h{};
};

// NT = 256: 2 x 2 waves; NT = 512 (256 x 256 tiles): 2 x 4 waves of 128 x 64 - twice the MFMA
// work per staged byte, one block per CU.
// DIR: the 1x1 / stride-1 / pad-0 case (p.direct) as a compile-time path - the x row of a K-step
// is its dy row, so a lane keeps one offset per load and no bounds state (rows past M and the
// taps past R*S of a narrow tile read the descriptor's zero fill or land in columns that are
// not stored): 44 fewer VALU per K-step, 120 VGPRs instead of 128 + spills, 1-7 % per call
// (profiles/wgrad_direct_ab_r3.md; asking the freed registers for 5 waves/SIMD spills the
// fragment addresses into the K loop: 2x slower).
template <int BMW, int BNW, int STAGES, bool F16 = false, int NT = conv::kThreads, bool DIR = false>
__global__ __launch_bounds__(NT, (NT == conv::kThreads && BNW <= 128) ? DPT_WGRAD_WAVES : 2) void conv_wgrad_kernel(ConvWgradArgs p) {
  using namespace conv;
  constexpr int NW = NT / 64;
  constexpr int WNW = NT == 512 ? 4 : 2, WMW = NW / WNW;  // waves along N / M
  constexpr int BKP = 64;                   // pixels per K-step
  constexpr int RBA = BMW * 2, RBB = BNW * 2;  // LDS row bytes (dy image, x image)
  constexpr int A_BYTES = BKP * RBA, B_BYTES = BKP * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / NW;  // glds instructions per wave per tile
  constexpr int B_INSTR = B_BYTES / 1024 / NW;
  constexpr int A_RPI = 1024 / RBA, B_RPI = 1024 / RBB;  // rows per glds instruction
  constexpr int WTM = BMW / WMW, WTN = BNW / WNW;  // wave tile
  constexpr int MI = WTM / 32, NI = WTN / 32;
  static_assert(MI >= 1 && NI >= 1 && A_INSTR >= 1 && B_INSTR >= 1, "conv_wgrad_kernel: bad tiling");
  __shared__ __attribute__((aligned(16))) unsigned char lds[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WNW, wn = wid % WNW;
  const int tiles = p.co_tiles * p.n_tiles;
  const int bid = conv::xcd_remap(blockIdx.x, tiles * p.splits);
  const int sp = bid / tiles, tile = bid - sp * tiles;
  const int ct = tile / p.n_tiles, nt = tile - ct * p.n_tiles;
  const int co0 = ct * BMW;
  // n-tile = K range [nt*BNW, nt*BNW + BNW) of k = (r*S + s)*C + c; narrow inputs (C < BNW)
  // cover BNW/C consecutive taps along s per tile (consecutive input pixels)
  const int cblocks = p.C >= BNW ? p.C / BNW : 1;
  const int tps = p.C >= BNW ? 1 : BNW / p.C;
  const int rs = (nt / cblocks) * tps, cb = nt - (nt / cblocks) * cblocks;
  const int r = rs / p.S, s = rs - r * p.S;
  const int ci0 = cb * BNW;
  const int k0 = sp * p.steps_per_split;
  const int k1 = min(k0 + p.steps_per_split, (p.M + BKP - 1) / BKP);

  // per-lane glds rows/chunks (lane-linear images, source-side swizzle)
  int arow[A_INSTR], achk[A_INSTR], brow[B_INSTR], bchk[B_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    arow[i] = (wid * A_INSTR + i) * A_RPI + lane / (RBA / 16);
    achk[i] = wg_slot<RBA>(arow[i], lane % (RBA / 16));
  }
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    brow[i] = (wid * B_INSTR + i) * B_RPI + lane / (RBB / 16);
    bchk[i] = wg_slot<RBB>(brow[i], lane % (RBB / 16));
  }

  // Per-lane row state, set up once and advanced by one K-step per stage() call (stage() runs
  // for ks = k0, k0+1, ... in order): the K loop does no divisions and no multiplies - the
  // 64-bit address multiplies of a per-step recompute were the largest VALU cost of this loop.
  // 32-bit offsets (launch_conv_wgrad checks the tensor sizes).
  int aoff[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) aoff[i] = (k0 * BKP + arow[i]) * p.Cout + co0 + achk[i] * 8;
  // Narrow inputs (C < BNW): the tile holds tps consecutive taps t = rs + sub, sub = this
  // chunk's (chunk*8)/C, anywhere in the R x S window (a tile may span tap rows - the 16-tap
  // 4x4 stem in one 256-column tile - and the last tile may run past R*S: ragged, those taps
  // read zeros and are not stored).  A lane's chunk is fixed, so its tap offset (bdr, bds)
  // from the block's base tap (r, s) and its address delta are constants.
  const int bm0 = k0 * BKP + brow[0];  // rows of one lane differ by compile-time constants
  int bh[B_INSTR], bw[B_INSTR], bdr[B_INSTR], bds[B_INSTR], boff[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int m = k0 * BKP + brow[i];
    int delta = bchk[i] * 8;
    bdr[i] = 0; bds[i] = 0;
    if (tps > 1) {
      const int sub = bchk[i] * 8 / p.C, t = rs + sub;
      if (t < p.R * p.S) {
        const int tr = t / p.S, ts = t - tr * p.S;
        bdr[i] = tr - r; bds[i] = ts - s;
      } else {
        bdr[i] = -(1 << 28);  // past the last tap: never in bounds
      }
      delta = (bdr[i] * p.W + bds[i]) * p.C + (bchk[i] * 8 - sub * p.C);
      if (t >= p.R * p.S) delta = 0;
    }
    if (DIR || p.direct) {
      bh[i] = 0; bw[i] = 0;
      boff[i] = m * p.C + ci0 + delta;
    } else {
      const int n = m / (p.Ho * p.Wo), rem = m - n * (p.Ho * p.Wo);
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      bh[i] = ho * p.stride - p.pad + r;
      bw[i] = wo * p.stride - p.pad + s;
      boff[i] = ((n * p.H + bh[i]) * p.W + bw[i]) * p.C + ci0 + delta;
    }
  }
  int bm = bm0;
  const int wlim = p.Wo * p.stride - p.pad + s;  // wo >= Wo
  const int hlim = p.Ho * p.stride - p.pad + r;  // ho >= Ho
  const int adelta = BKP * p.Cout;
  const int dp_step = p.dp_w + p.dp_h, hstep1 = p.dh_step + p.stride;

  // Buffer loads into LDS: the descriptors' range check zero-fills rows past the end (dy:
  // m >= M) and the zero-padding taps (x: offset kOOB), so no address selects are needed.
  constexpr uint32_t kOOB = 0xFFFFFF00u;  // >= any num_records here, and offset + 16 does not wrap
  const __amdgpu_buffer_rsrc_t rdy =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, (int)((uint32_t)p.M * (uint32_t)p.Cout * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, 0, (int)((uint32_t)p.N * (uint32_t)(p.H * p.W * p.C) * 2u), 0x00020000);

  auto stage = [&](int /*ks*/, int buf) {
    unsigned char* a = lds + buf * STAGE;
    unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy, (__attribute__((address_space(3))) void*)(a + (wid * A_INSTR + i) * 1024),
                                               16, (uint32_t)aoff[i] * 2u, 0, 0, 0);
      aoff[i] += adelta;
    }
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) {
      if constexpr (DIR) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(b + (wid * B_INSTR + i) * 1024),
                                                 16, (uint32_t)boff[i] * 2u, 0, 0, 0);
        boff[i] += dp_step;
        continue;
      }
      // bitwise, not short-circuit: no exec-mask branches around the select
      const bool ok = (bm + (brow[i] - brow[0]) < p.M) &
                      ((p.direct != 0) | (((unsigned)(bh[i] + bdr[i]) < (unsigned)p.H) &
                                          ((unsigned)(bw[i] + bds[i]) < (unsigned)p.W)));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(b + (wid * B_INSTR + i) * 1024),
                                               16, ok ? (uint32_t)boff[i] * 2u : kOOB, 0, 0, 0);
      boff[i] += dp_step;
      if (!p.direct) {  // "c ? v + k : v" forms: one add + one v_cndmask each
        bw[i] += p.dw_step;
        const bool cw = bw[i] >= wlim;
        bw[i] = cw ? bw[i] - p.wwrap : bw[i];
        bh[i] = cw ? bh[i] + hstep1 : bh[i] + p.dh_step;
        boff[i] = cw ? boff[i] + p.dp_wwrap : boff[i];
        const bool ch = bh[i] >= hlim;
        bh[i] = ch ? bh[i] - p.hwrap : bh[i];
        boff[i] = ch ? boff[i] + p.dp_hwrap : boff[i];
      }
    }
    bm += BKP;
  };

  f32x16_t acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  auto mma = [&](int buf) {
    const unsigned char* a = lds + buf * STAGE;
    const unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BKP / 16; ++kk) {
      bf16x8_t fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = wg_frag<RBA>(a, kk * 16, wm * WTM + i * 32, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = wg_frag<RBB>(b, kk * 16, wn * WTN + j * 32, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = cmfma<F16>(fa[i], fb[j], acc[i][j]);
    }
  };
  if (STAGES == 2) {
    if (k0 < k1) {
      stage(k0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int ks = k0; ks < k1; ++ks) {
        const int cur = (ks - k0) & 1;
        if (ks + 1 < k1) stage(ks + 1, cur ^ 1);
        mma(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    for (int ks = k0; ks < k1; ++ks) {
      stage(ks, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      mma(0);
      __syncthreads();
    }
  }
  // fp32 partial tile: rows = output channels, columns = (r, s, ci) of this tap
  const int64_t Kg = (int64_t)p.R * p.S * p.C;
  float* out = p.part + (int64_t)sp * p.Cout * Kg + (int64_t)nt * BNW;
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wn * WTN + j * 32 + lr;
      if ((int64_t)nt * BNW + col >= Kg) continue;  // ragged last tile: taps past R*S
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = co0 + wm * WTM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        out[(int64_t)row * Kg + col] = acc[i][j][e];
      }
    }
}

// ---- backward-weight HALO: the three taps (r, 0..2) of a 3x3 / stride-1 / pad-1 conv ---------
//
// conv_wgrad_kernel stages a dy tile and an x tile per tap: 9 dy + 9 x tiles per 64 pixels.
// Here the K loop runs over PADDED output pixels p = (n*H + ho)*(W+2) + wo, wo in [0, W+2):
// the two dummy columns per image row have dy = 0, and the input pixel of tap (r, s) is the
// padded input index q = p + (r-1)*(W+2) + s whose columns 0 and W+1 are the zero padding -
// an image row never wraps into the next.  So one strip of 68 consecutive padded x rows serves
// all three taps of tap row r (tap s = the strip read s rows further down), and one dy tile
// serves all three: 1 dy + 1 strip per 64 pixels and 3 taps.  dy rows whose tap row
// ho + r - 1 leaves the image are zero-filled (kOOB), which also kills the strip rows read from
// the neighbouring image rows.  Tile: 64 output channels x BNW input channels x 3 taps; 2 x 2
// waves of 32 x BNW/2 x 3 (BNW = 128: 6 accumulators, 2 waves per SIMD; BNW = 64: 3, 4 waves
// per SIMD - the one that pays, see wgrad_halo_mode).  Costs (W+2)/W more MFMA work (7 % at
// W = 28, 29 % at W = 7) for ~2.9x fewer staged bytes.
template <int BNW, int STAGES, bool F16>
__global__ __launch_bounds__(conv::kThreads, BNW == 64 ? 4 : 2) void conv_wgrad_halo_kernel(ConvWgradArgs p) {
  using namespace conv;
  constexpr int NW = 4, BKP = 64;
  constexpr int RBA = 128, RBB = BNW * 2;  // dy rows: 64 channels, x rows: BNW channels
  constexpr int B_RPI = 1024 / RBB;        // strip rows per glds instruction (4 or 8)
  constexpr int HROWS = (BKP + 2 + B_RPI - 1) / B_RPI * B_RPI;  // 68 or 72
  constexpr int NI = BNW / 64;             // 32-column accumulators per wave and tap
  constexpr int A_BYTES = BKP * RBA, B_BYTES = HROWS * RBB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / NW, A_RPI = 1024 / RBA;  // 2 per wave, 8 rows each
  constexpr int B_GI = B_BYTES / 1024;                              // 17 or 9 per block
  constexpr int B_PW = (B_GI + NW - 1) / NW;
  __shared__ __attribute__((aligned(16))) unsigned char lds[STAGES * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = p.co_tiles * p.n_tiles;
  const int bid = conv::xcd_remap(blockIdx.x, tiles * p.splits);
  const int sp = bid / tiles, tile = bid - sp * tiles;
  const int ct = tile / p.n_tiles, nt = tile - ct * p.n_tiles;
  const int cblocks = p.C / BNW;
  const int r = nt / cblocks, cb = nt - r * cblocks;
  const int co0 = ct * 64, ci0 = cb * BNW;
  const int k0 = sp * p.steps_per_split;
  const int k1 = min(k0 + p.steps_per_split, (p.Mp + BKP - 1) / BKP);
  const int Wp = p.W + 2, NH = p.N * p.H;

  int arow[A_INSTR], achk[A_INSTR], brow[B_PW], bchk[B_PW];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    arow[i] = (wid * A_INSTR + i) * A_RPI + lane / (RBA / 16);
    achk[i] = wg_slot<RBA>(arow[i], lane % (RBA / 16));
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    brow[i] = (wid + i * NW) * B_RPI + lane / (RBB / 16);
    bchk[i] = wg_slot<RBB>(brow[i], lane % (RBB / 16));
  }
  constexpr uint32_t kOOB = 0xFFFFFF00u;
  const __amdgpu_buffer_rsrc_t rdy =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, (int)((uint32_t)p.M * (uint32_t)p.Cout * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, 0, (int)((uint32_t)p.N * (uint32_t)(p.H * p.W * p.C) * 2u), 0x00020000);
  const int qbase = (r - 1) * Wp;  // strip row j of K-step ks = padded input ks*64 + qbase + j

  auto stage = [&](int ks, int buf) {
    unsigned char* a = lds + buf * STAGE;
    unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const int pp = ks * BKP + arow[i];
      const int R = (int)fdiv((uint32_t)pp, p.div_wp), wo = pp - R * Wp;
      const int ho = R - (int)fdiv((uint32_t)R, p.div_h) * p.H;
      const bool ok = (pp < p.Mp) & (wo < p.W) & ((unsigned)(ho + r - 1) < (unsigned)p.H);
      const uint32_t off = (((uint32_t)R * p.W + wo) * p.Cout + co0 + achk[i] * 8) * 2u;  // used when ok
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy, (__attribute__((address_space(3))) void*)(a + (wid * A_INSTR + i) * 1024),
                                               16, ok ? off : kOOB, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      if (wid + i * NW < B_GI) {  // wave-uniform
        const int q = ks * BKP + qbase + brow[i];
        const int qc = max(q, 0);
        const int R = (int)fdiv((uint32_t)qc, p.div_wp), c = qc - R * Wp;
        const bool ok = (q >= 0) & (R < NH) & (c >= 1) & (c <= p.W);
        const uint32_t off = (((uint32_t)R * p.W + c - 1) * p.C + ci0 + bchk[i] * 8) * 2u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(b + (wid + i * NW) * 1024),
                                                 16, ok ? off : kOOB, 0, 0, 0);
      }
    }
  };

  f32x16_t acc[3][NI];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[s][j][e] = 0.f;

  auto mma = [&](int buf) {
    const unsigned char* a = lds + buf * STAGE;
    const unsigned char* b = a + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BKP / 16; ++kk) {
      const bf16x8_t fa = wg_frag<RBA>(a, kk * 16, wm * 32, lane);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        bf16x8_t fb[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = wg_frag<RBB>(b, kk * 16 + s, wn * (BNW / 2) + j * 32, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[s][j] = cmfma<F16>(fa, fb[j], acc[s][j]);
      }
    }
  };
  if (STAGES == 2) {
    if (k0 < k1) {
      stage(k0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int ks = k0; ks < k1; ++ks) {
        const int cur = (ks - k0) & 1;
        if (ks + 1 < k1) stage(ks + 1, cur ^ 1);
        mma(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    for (int ks = k0; ks < k1; ++ks) {
      stage(ks, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      mma(0);
      __syncthreads();
    }
  }
  const int64_t Kg = (int64_t)9 * p.C;
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    float* out = p.part + (int64_t)sp * p.Cout * Kg + (int64_t)(r * 3 + s) * p.C + ci0;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wn * (BNW / 2) + j * 32 + lr;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = co0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        out[(int64_t)row * Kg + col] = acc[s][j][e];
      }
    }
  }
}

// out[i] = sum_s part[s][i]: PH phases per block split the S loop, LDS combines them.
template <int PH>
__global__ __launch_bounds__(kBlock) void conv_wgrad_reduce_kernel(const float4* __restrict__ part, int64_t n4,
                                                                   int S, void* __restrict__ out, int out_kind) {
  __shared__ float4 red[kBlock];
  wgrad_reduce_body<PH>(part, n4, S, out, out_kind, (int)blockIdx.x, red);
}

// ---- narrow-input convs (the 3-channel stem): explicit im2col -> the 1x1 MFMA GEMM ---------------
// a[m, k] (bf16, k padded to Kp, a multiple of 64) = x[pix(m) + tap(k)] for k < R*S*C, else 0;
// k = (r*S + s)*C + c matches the KRSC weight flattened to [Cout, R*S*C].  x is fp32 or bf16
// channels_last (the loader's dtype: the autocast cast of the input disappears with it).
template <typename T>
__global__ __launch_bounds__(kBlock) void im2col_kernel(const T* __restrict__ x, uint16_t* __restrict__ a,
                                                         int64_t M, int H, int W, int C, int Ho, int Wo, int R,
                                                         int S, int stride, int pad, int Kp) {
  const int cpr = Kp / 8;
  const int64_t n_items = M * cpr;
  const int K = R * S * C;
  for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < n_items; it += (int64_t)gridDim.x * kBlock) {
    const int64_t m = it / cpr;
    const int ch = (int)(it - m * cpr);
    const int64_t n = m / ((int64_t)Ho * Wo);
    const int rem = (int)(m - n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    uint32_t packed[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint16_t v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = ch * 8 + j + u;
        float f = 0.f;
        if (k < K) {
          const int tap = k / C, c = k - tap * C;
          const int r = tap / S, s = tap - r * S;
          const int hi = ho * stride - pad + r, wi = wo * stride - pad + s;
          if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W) {
            const T raw = x[((n * H + hi) * (int64_t)W + wi) * C + c];
            if constexpr (sizeof(T) == 4) f = (float)raw;
            else f = bf16_to_f32((uint16_t)raw);
          }
        }
        v[u] = f32_to_bf16(f);
      }
      packed[j / 2] = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
    }
    *reinterpret_cast<uint4*>(a + m * Kp + ch * 8) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  }
}

// ---- space-to-depth (2x2) stem input ---------------------------------------------------------
// A 7x7/2 conv on [H, W, 3] is a 4x4/1 conv on the 2x2 space-to-depth image [H/2, W/2, 12]
// (channels padded to 16, weight taps re-indexed as r = 2r' + a - 1, s = 2s' + b - 1): K = 256,
// every 64-wide K-step four consecutive pixels of one row - the narrow-input path of the
// implicit-GEMM kernels.  One thread per output pixel: 4 input pixels in, 32 bytes out.
template <typename T>
__global__ __launch_bounds__(kBlock) void space_to_depth2_kernel(const T* __restrict__ x, uint16_t* __restrict__ a,
                                                                 int64_t npix, int H, int W, int C, int out_f16) {
  const int H2 = H / 2, W2 = W / 2;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < npix; t += (int64_t)gridDim.x * kBlock) {
    const int64_t n = t / ((int64_t)H2 * W2);
    const int rem = (int)(t - n * H2 * W2);
    const int i = rem / W2, j = rem - i * W2;
    uint32_t pk[8];
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
      const T* src = x + ((n * H + 2 * i + (ab >> 1)) * (int64_t)W + 2 * j + (ab & 1)) * C;
      float f[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f[c] = 0.f;
        if (c < C) {
          if constexpr (sizeof(T) == 4) f[c] = (float)src[c];
          else f[c] = bf16_to_f32((uint16_t)src[c]);
        }
      }
      const f32x2_t v0 = {f[0], f[1]}, v1 = {f[2], f[3]};
      pk[2 * ab] = out_f16 ? cpack<true>(v0) : cpack<false>(v0);
      pk[2 * ab + 1] = out_f16 ? cpack<true>(v1) : cpack<false>(v1);
    }
    uint4* dst = reinterpret_cast<uint4*>(a + t * 16);
    dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    dst[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
  }
}

// The 3-channel fp32 image (the ResNet input) two output pixels per thread: the 4 x 2 input
// pixels are two rows of 48 contiguous, 16-byte-aligned bytes - 6 float4 loads and 4 16-byte
// stores per thread instead of 24 scalar loads (69 us -> memory-bound on ResNet-50's 154 MB).
template <bool F16>
__global__ __launch_bounds__(kBlock) void space_to_depth2_c3_kernel(const float* __restrict__ x, uint16_t* __restrict__ a,
                                                                    int64_t n2, int H, int W) {
  const int H2 = H / 2, Q = W / 4;  // Q pixel pairs per output row
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < n2; t += (int64_t)gridDim.x * kBlock) {
    const int64_t n = t / ((int64_t)H2 * Q);
    const int rem = (int)(t - n * H2 * Q);
    const int i = rem / Q, q = rem - i * Q;
    float v[2][12];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float4* src = reinterpret_cast<const float4*>(x + ((n * H + 2 * i + r) * (int64_t)W + 4 * q) * 3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float4 f = src[k];
        v[r][4 * k] = f.x; v[r][4 * k + 1] = f.y; v[r][4 * k + 2] = f.z; v[r][4 * k + 3] = f.w;
      }
    }
    // output pixel p (= 2q + p) gathers input pixels (2i + r, 4q + 2p + b): channel (r*2 + b)*4 + c
    uint32_t pk[2][8];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const int r = ab >> 1, b = ab & 1, base = (2 * p + b) * 3;
        const f32x2_t v0 = {v[r][base], v[r][base + 1]}, v1 = {v[r][base + 2], 0.f};
        pk[p][2 * ab] = cpack<F16>(v0);
        pk[p][2 * ab + 1] = cpack<F16>(v1);
      }
    uint4* dst = reinterpret_cast<uint4*>(a + (t * 2) * 16);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      dst[2 * p] = make_uint4(pk[p][0], pk[p][1], pk[p][2], pk[p][3]);
      dst[2 * p + 1] = make_uint4(pk[p][4], pk[p][5], pk[p][6], pk[p][7]);
    }
  }
}

void launch_space_to_depth2(const void* x, bool x_bf16, uint16_t* a, int N, int H, int W, int C, hipStream_t st,
                            bool out_f16) {
  if (!x_bf16 && C == 3 && W % 4 == 0 && H % 2 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0) {
    const int64_t n2 = (int64_t)N * (H / 2) * (W / 4);
    const dim3 grid((unsigned)grid_for(n2, 1));
    if (out_f16)
      hipLaunchKernelGGL(space_to_depth2_c3_kernel<true>, grid, dim3(kBlock), 0, st, static_cast<const float*>(x), a, n2,
                         H, W);
    else
      hipLaunchKernelGGL(space_to_depth2_c3_kernel<false>, grid, dim3(kBlock), 0, st, static_cast<const float*>(x), a,
                         n2, H, W);
    return;
  }
  const int64_t npix = (int64_t)N * (H / 2) * (W / 2);
  const dim3 grid((unsigned)grid_for(npix, 2));
  if (x_bf16)
    hipLaunchKernelGGL(space_to_depth2_kernel<uint16_t>, grid, dim3(kBlock), 0, st, static_cast<const uint16_t*>(x), a,
                       npix, H, W, C, out_f16 ? 1 : 0);
  else
    hipLaunchKernelGGL(space_to_depth2_kernel<float>, grid, dim3(kBlock), 0, st, static_cast<const float*>(x), a, npix,
                       H, W, C, out_f16 ? 1 : 0);
}

void launch_im2col(const void* x, bool x_bf16, uint16_t* a, int N, int H, int W, int C, int R, int S, int stride,
                   int pad, int Kp, hipStream_t st) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  const int64_t items = M * (Kp / 8);
  const dim3 grid((unsigned)grid_for(items, 4));
  if (x_bf16)
    hipLaunchKernelGGL(im2col_kernel<uint16_t>, grid, dim3(kBlock), 0, st, static_cast<const uint16_t*>(x), a, M, H,
                       W, C, Ho, Wo, R, S, stride, pad, Kp);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, grid, dim3(kBlock), 0, st, static_cast<const float*>(x), a, M, H, W, C,
                       Ho, Wo, R, S, stride, pad, Kp);
}

// wt[ci, r', s', co] = w[co, R-1-r', S-1-s', ci]: the backward-data operand of a stride-1 conv.
__global__ __launch_bounds__(kBlock) void conv_wt_flip_kernel(const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ wt, int Cout, int R,
                                                              int S, int C) {
  const int64_t n = (int64_t)Cout * R * S * C;
  for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < n; o += (int64_t)gridDim.x * kBlock) {
    // o indexes wt = [C][R][S][Cout]
    const int co = (int)(o % Cout);
    int64_t t = o / Cout;
    const int s = (int)(t % S);
    t /= S;
    const int r = (int)(t % R);
    const int ci = (int)(t / R);
    wt[o] = w[(((int64_t)co * R + (R - 1 - r)) * S + (S - 1 - s)) * C + ci];
  }
}

// Every conv weight of a step flipped in ONE launch (ops/conv.py flip cache): blocks are dealt
// to the descriptors in order; each thread writes 8 consecutive co of one (ci, r', s') row
// (16-byte store) gathered from w[co][R-1-r'][S-1-s'][ci].  32-bit index math.
__global__ __launch_bounds__(kBlock) void conv_wt_flip_multi_kernel(WtFlipBatch b) {
  int i = 0;
  while (i + 1 < b.count && (int)blockIdx.x >= b.blk0[i + 1]) ++i;
  const int Cout = b.Cout[i], R = b.R[i], S = b.S[i], C = b.C[i];
  const uint32_t rows8 = (uint32_t)C * R * S * (Cout / 8);
  const uint32_t t = (uint32_t)(blockIdx.x - b.blk0[i]) * kBlock + threadIdx.x;
  if (t >= rows8) return;
  const uint32_t cog = t % (uint32_t)(Cout / 8);
  uint32_t q = t / (uint32_t)(Cout / 8);
  const int s = (int)(q % (uint32_t)S);
  q /= (uint32_t)S;
  const int r = (int)(q % (uint32_t)R);
  const int ci = (int)(q / (uint32_t)R);
  const uint16_t* w = b.w[i];
  const uint32_t cstride = (uint32_t)R * S * C;
  const uint32_t base = ((uint32_t)(R - 1 - r) * S + (S - 1 - s)) * C + ci + cog * 8 * cstride;
  uint16_t v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = w[base + k * cstride];
  uint4 o;
  o.x = v[0] | ((uint32_t)v[1] << 16);
  o.y = v[2] | ((uint32_t)v[3] << 16);
  o.z = v[4] | ((uint32_t)v[5] << 16);
  o.w = v[6] | ((uint32_t)v[7] << 16);
  *reinterpret_cast<uint4*>(b.wt[i] + (int64_t)t * 8) = o;
}

// Same flip as 64 x 64 tiles through LDS (every weight with C % 64 == 0 and Cout % 64 == 0, i.e.
// every stride-1 conv of the ResNets): per tap (r, s) the weight is a [Cout][C] matrix with
// contiguous ci rows and the flipped copy its transpose with contiguous co rows, so both sides
// move whole 128-byte row segments (the gather above reads 2 bytes per lane per row: 72 us for
// ResNet-50's 23.5 M weights, ~1.3 TB/s).  One block per (weight, tap, 64-co tile, 64-ci tile).
__global__ __launch_bounds__(kBlock) void conv_wt_flip_tiled_kernel(WtFlipBatch b) {
  __shared__ uint16_t tile[64][64 + 2];  // +2: the column reads of the store phase spread over banks
  int i = 0;
  while (i + 1 < b.count && (int)blockIdx.x >= b.blk0[i + 1]) ++i;
  const int Cout = b.Cout[i], R = b.R[i], S = b.S[i], C = b.C[i];
  const int cit = C / 64, cot = Cout / 64;
  int q = (int)blockIdx.x - b.blk0[i];
  const int ct = q % cit;
  q /= cit;
  const int ot = q % cot;
  const int rs = q / cot;  // tap r*S + s of the original weight
  const int r = rs / S, s = rs - r * S;
  const uint16_t* w = b.w[i];
  uint16_t* wt = b.wt[i];
  const int tid = threadIdx.x;
  // load: 64 co rows x 8 chunks of 8 ci (16 B), 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = tid + k * kBlock, row = e >> 3, ch = e & 7;
    const int co = ot * 64 + row;
    const uint4 v = *reinterpret_cast<const uint4*>(w + ((int64_t)co * R * S + rs) * C + ct * 64 + ch * 8);
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[row][ch * 8 + 2 * j] = (uint16_t)u[j];
      tile[row][ch * 8 + 2 * j + 1] = (uint16_t)(u[j] >> 16);
    }
  }
  __syncthreads();
  // store: 64 ci rows x 8 chunks of 8 co of wt[ci][R-1-r][S-1-s][co]
  const int rsf = (R - 1 - r) * S + (S - 1 - s);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = tid + k * kBlock, row = e >> 3, ch = e & 7;
    const int ci = ct * 64 + row;
    uint32_t u[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      u[j] = (uint32_t)tile[ch * 8 + 2 * j][row] | ((uint32_t)tile[ch * 8 + 2 * j + 1][row] << 16);
    *reinterpret_cast<uint4*>(wt + ((int64_t)ci * R * S + rsf) * Cout + ot * 64 + ch * 8) =
        make_uint4(u[0], u[1], u[2], u[3]);
  }
}

void launch_conv_wt_flip_multi(WtFlipBatch b, hipStream_t s) {
  bool tiled = true;
  for (int i = 0; i < b.count; ++i) tiled = tiled && b.C[i] % 64 == 0 && b.Cout[i] % 64 == 0;
  int blocks = 0;
  for (int i = 0; i < b.count; ++i) {
    b.blk0[i] = blocks;
    if (tiled) {
      blocks += (b.C[i] / 64) * (b.Cout[i] / 64) * b.R[i] * b.S[i];
    } else {
      const int64_t rows8 = (int64_t)b.C[i] * b.R[i] * b.S[i] * (b.Cout[i] / 8);
      blocks += (int)((rows8 + kBlock - 1) / kBlock);
    }
  }
  if (blocks == 0) return;
  if (tiled) hipLaunchKernelGGL(conv_wt_flip_tiled_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, b);
  else hipLaunchKernelGGL(conv_wt_flip_multi_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, b);
}

bool conv_supported(int C, int Cout) { return C % 64 == 0 && Cout % 64 == 0; }

// Narrow inputs (C = 16 or 32) need the taps of one K-step to be consecutive along s.
bool conv_supported_narrow(int C, int Cout, int S) {
  return (C == 16 || C == 32) && Cout % 64 == 0 && S % (64 / C) == 0;
}

int conv_m_tiles(int64_t M) { return (int)((M + conv::BM - 1) / conv::BM); }
int conv_split_cols(int64_t M) { return (int)((M + 15) / 16); }

// Kernel variant: 0 = default (1-stage + LDS epilogue), 5/6 = 256-row blocks (register / LDS
// epilogue), 1 = 2-stage + LDS epilogue, 2 = 2-stage +
// register epilogue, 3 = 1-stage + register epilogue, 4 = 1-stage + LDS epilogue.
// The backward-weight kernel takes 1-2 -> 2 stages, 0/3-4 -> 1 stage.
// conv_set_variant switches at run time (A/B tests, benchmarks; the bindings' conv_set_variant).
static int g_conv_variant = 0;
static int conv_variant() { return g_conv_variant; }
// forward / backward-data tile variant: codes >= 20 select backward-weight tiles only
static int fwd_variant() { return g_conv_variant >= 20 ? 0 : g_conv_variant; }
void conv_set_variant(int v) { g_conv_variant = v; }

// Production choice of the 8-wave 256-row tiles (variant 0): deep reductions onto narrow
// outputs, where the 128 x 128 tile re-reads A from L2 once per 128 output channels and the
// per-CU L2 -> LDS rate caps it (profiles/conv_variants_*.md, ResNet-50 batch 256):
//   N = 256, K >= 1024, M >= 32768          -> 9  (256 x 256): 3x3 256->256 @14x14 709 -> 896 TF
//   N = 512, K >= 2048, M <= 16384          -> 10 (256 x 128): 3x3 512->512 @7x7 714 -> 802 TF
// Off by default: in the ResNet-50 training step (stats / BNB / BNR epilogues, L2 shared with
// the neighbouring kernels) the per-shape wins did not show (11680/11521 vs 11659/11534 img/s,
// same-box A/B).  conv_set_big(1) turns it on.
static int g_conv_big = 0;
// conv_set_big(2 / 3): the deep one-tap convs (K >= 1024 / >= 512, N a multiple of 256) on the
// 8-wave 128 x 256 tile with the 3-stage pipelined K loop (variant 13): their grids are 392-784
// 128 x 128 tiles of 16-32 K-steps, latency-bound at ~3 resident blocks per CU
// (profiles/step_pmc_r5.md); in isolation v13 was 5-17 % faster there (profiles/conv_variants_r3_pipe3.md).
static int conv_big_auto(int64_t M, int N, int64_t K, int taps) {
  if (!g_conv_big) return 0;
  if (g_conv_big >= 2) {
    const int64_t kmin = g_conv_big == 2 ? 1024 : 512;
    return (taps == 1 && K >= kmin && N % 256 == 0) ? 13 : 0;
  }
  if (N == 256 && K >= 1024 && M >= 32768) return 9;
  if (N == 512 && K >= 2048 && M <= 16384) return 10;
  return 0;
}
void conv_set_big(int on) { g_conv_big = on; }


// Launch one conv_fwd_kernel instantiation in the element type of a.f16 (fp16 is instantiated
// for the production 128-row, 1-stage, LDS-epilogue variants only).
// conv_fwd_kernel addresses both operands with 32-bit byte offsets through buffer descriptors
// (num_records < 2^32, padding reads at offset 0xFFFFFF00).
static void conv_check_offsets(const ConvFwdArgs& a, bool bkn) {
  const int64_t xb = (int64_t)a.N * a.H * a.W * a.C * 2;
  const int64_t wb = (int64_t)(bkn ? a.Rw * a.Sw : a.R * a.S) * a.C * a.Cout * 2;
  if (xb >= 0xFFFFFF00ll || wb >= 0x7FFFFFFFll)
    throw std::runtime_error("conv: operand tensors beyond 2^31 elements are not supported");
}

// ---- piggybacked backward-weight reduce (AttachWgradReduce, kernels.h) -------------------------
static thread_local WgradReduce* g_attached_reduce = nullptr;

static int reduce_phases(int splits) { return splits >= 16 ? 16 : splits >= 4 ? 4 : 1; }

void launch_wgrad_reduce(const WgradReduce& r, hipStream_t st) {
  const float4* part = reinterpret_cast<const float4*>(r.part);
  const int ph = reduce_phases(r.splits), out_per_block = kBlock / ph;
  const dim3 grid((unsigned)((r.n4 + out_per_block - 1) / out_per_block)), block(kBlock);
  if (ph == 16) hipLaunchKernelGGL(conv_wgrad_reduce_kernel<16>, grid, block, 0, st, part, r.n4, r.splits, r.out, r.kind);
  else if (ph == 4) hipLaunchKernelGGL(conv_wgrad_reduce_kernel<4>, grid, block, 0, st, part, r.n4, r.splits, r.out, r.kind);
  else hipLaunchKernelGGL(conv_wgrad_reduce_kernel<1>, grid, block, 0, st, part, r.n4, r.splits, r.out, r.kind);
}

AttachWgradReduce::AttachWgradReduce(WgradReduce* r, hipStream_t s) : r_(r), s_(s) {
  if (g_attached_reduce != nullptr) throw std::runtime_error("AttachWgradReduce: a reduce is already attached");
  g_attached_reduce = (r != nullptr && !r->consumed) ? r : nullptr;
}

AttachWgradReduce::~AttachWgradReduce() {
  g_attached_reduce = nullptr;
  if (r_ != nullptr && !r_->consumed) {
    launch_wgrad_reduce(*r_, s_);
    r_->consumed = true;
  }
}

// The attached reduce (if any) moves into `rc`: returns the blocks to append to the grid.
int take_attached_reduce(ReduceCarry& rc) {
  WgradReduce* r = g_attached_reduce;
  if (r == nullptr || r->consumed) return 0;
  r->consumed = true;
  g_attached_reduce = nullptr;
  rc.part = reinterpret_cast<const float4*>(r->part);
  rc.out = r->out;
  rc.n4 = r->n4;
  rc.splits = r->splits;
  rc.kind = r->kind;
  rc.ph = reduce_phases(r->splits);
  rc.blocks = (int)((r->n4 + kBlock / rc.ph - 1) / (kBlock / rc.ph));
  return rc.blocks;
}
static int take_attached_reduce(ConvFwdArgs& a) { return take_attached_reduce(a.red); }

// 3x3 / stride 1 / pad 1 convs (and their backward-data) take the HALO K loop (conv_fwd_kernel).
// conv_set_halo: 0 = per-tap loop (A/B), 1 = auto (default): all three B taps per load phase
// (HB = 3) when the tile grid is at most 512 tiles (two blocks per CU) - there the grid, not LDS,
// limits the resident blocks and one wait per three K-steps wins (3x3 512->512 @7x7: 0.075 ->
// 0.064 ms; a 1024-tile cut-off measured slower) - else one B tap per phase (HB = 1; HB = 3
// everywhere lost 1.2 % in the step), 2 / 3 = force HB
static int g_conv_halo = 1;
// B operand straight into VGPRs (conv_fwd_kernel BREG): bit 0 = 3x3 HALO convs, bit 1 = the
// other single-stage 128-row convs (1x1, strided, stem); conv_set_breg (A/B)
static int g_conv_breg = 0;
void conv_set_breg(int mode) { g_conv_breg = mode; }
int conv_get_breg() { return g_conv_breg; }
static int halo_hb(const ConvFwdArgs& a, int bn) {
  if (g_conv_halo == 2) return 1;
  if (g_conv_halo == 3) return 3;
  return (int64_t)a.m_tiles * (a.Cout / bn) <= 512 ? 3 : 1;
}
static bool halo_ok(const ConvFwdArgs& a) {
  return g_conv_halo && a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.C % 64 == 0 && a.Ho == a.H &&
         a.Wo == a.W;
}
void conv_set_halo(int on) { g_conv_halo = on; }

// ---- stream-K (conv_fwd_kernel<..., SK = true>) --------------------------------------------------
// Grids whose 128 x BN tiles do not divide evenly over the 256 CUs lose the idle part of the last
// round: 784 tiles of a ResNet-50 layer3 1x1 conv are 3 rounds on 240 CUs and 4 on 16, and the K loop
// is bound by each CU's L2 -> LDS bandwidth, so the step takes 4 tile-times where 3.06 would do
// (profiles/wave_efficiency_r5.md).  Stream-K spreads the (tile, K-step) iterations evenly over
// 256 x k blocks; a tile cut between blocks costs one fp32 partial tile written and read back.
// conv_set_streamk: 0 = off, 1 = auto (per-CU tile balance below kSkEff), 2 = every eligible grid.
static int g_conv_sk = 0;
static double kSkEff = 0.9;
void conv_set_streamk(int mode, double eff) {
  g_conv_sk = mode;
  if (eff > 0) kSkEff = eff;
}
int conv_get_streamk() { return g_conv_sk; }

namespace {
struct SkWorkspace {
  float* part = nullptr;
  unsigned* flags = nullptr;  // kSkMaxBlocks publish flags, then the give-up counter
  bool failed = false;
};
constexpr int kSkMaxBlocks = 256 * 6;
constexpr size_t kSkPartBytes = 64ull << 20;  // 1024 blocks x 64 KiB (128 x 128 fp32 tile)
std::mutex g_sk_mu;
SkWorkspace g_sk_ws[64];
}  // namespace

// The device's stream-K workspace, allocated (and the flags zeroed) on first use outside a graph
// capture; nullptr while capturing before that (the launch then runs the data-parallel grid).
// One workspace per device: the engine issues its convolutions on one stream at a time.
static SkWorkspace* sk_workspace(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_sk_mu);
  SkWorkspace& w = g_sk_ws[dev];
  if (w.part != nullptr) return &w;
  if (w.failed) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (s != nullptr && hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) return nullptr;
  void* part = nullptr;
  void* flags = nullptr;
  if (hipMalloc(&part, kSkPartBytes) != hipSuccess || hipMalloc(&flags, (kSkMaxBlocks + 64) * sizeof(unsigned)) != hipSuccess ||
      hipMemset(flags, 0, (kSkMaxBlocks + 64) * sizeof(unsigned)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    if (part) (void)hipFree(part);
    if (flags) (void)hipFree(flags);
    (void)hipGetLastError();
    w.failed = true;
    return nullptr;
  }
  w.part = static_cast<float*>(part);
  w.flags = static_cast<unsigned*>(flags);
  return &w;
}

void conv_sk_prepare() { (void)sk_workspace(nullptr); }

unsigned conv_sk_errors() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || g_sk_ws[dev].flags == nullptr) return 0;
  unsigned e = 0;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&e, g_sk_ws[dev].flags + kSkMaxBlocks, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
    throw std::runtime_error("conv_sk_errors: device read failed");
  return e;
}

// Blocks of the stream-K grid for this conv (0: run the data-parallel grid).  bpc = resident
// blocks per CU of the variant (LDS-limited: 4 at BN = 128, 6 at BN = 64).
int conv_sk_blocks(int64_t tiles, int nk, int bn, int mode) {
  if (mode == 0 || nk < 2 || tiles < 256) return 0;
  const double per_cu = (double)tiles / 256.0;
  const double eff = per_cu / std::ceil(per_cu);
  if (mode == 1 && eff >= kSkEff) return 0;
  const int bpc = bn == 128 ? 4 : 6;
  const int k = std::min<int>(bpc, (int)std::ceil(per_cu));
  const int G = 256 * k;
  // every block of every XCD group must hold at least one K-step (an empty block never publishes)
  if ((tiles / 8) * nk < G / 8 + 1) return 0;
  if ((tiles / 8 + 1) * (int64_t)nk * (G / 8) >= (1ll << 32)) return 0;  // 32-bit partition math
  return G;
}

template <int BMT, int BN, int STAGES, bool LDSEPI, bool BKN, bool STATS = true, bool BNB = false,
          bool BNR = false, bool REMAP = false, bool ZSIB = false, bool BNR2 = false, int NT = conv::kThreads>
static void fwd_launch(dim3 grid, dim3 /*block*/, hipStream_t s, const ConvFwdArgs& a0) {
  const dim3 block(NT);
  ConvFwdArgs a = a0;
  if constexpr (NT == conv::kThreads) grid.x += (unsigned)take_attached_reduce(a);
  conv_check_offsets(a, BKN);
  if constexpr (BMT == 128 && STAGES == 1 && LDSEPI && !BKN && !REMAP && NT == conv::kThreads) {
    // B operand in registers (conv_set_breg: bit 0 the 3x3 HALO convs, bit 1 the others)
    const bool halo = halo_ok(a);
    if ((g_conv_breg & (halo ? 1 : 2)) && a.n_tiles * BN == a.Cout) {
      if (halo) {
        if (a.f16)
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, true,
                                              conv::kThreads, false, true, 1, false, false, true>), grid, block, 0, s, a);
        else
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, false,
                                              conv::kThreads, false, true, 1, false, false, true>), grid, block, 0, s, a);
      } else {
        if (a.f16)
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, true,
                                              conv::kThreads, false, false, 1, false, false, true>), grid, block, 0, s, a);
        else
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, false,
                                              conv::kThreads, false, false, 1, false, false, true>), grid, block, 0, s, a);
      }
      return;
    }
    if (halo) {
      if (halo_hb(a, BN) == 3) {  // all three B taps with the halo strip
        if (a.f16)
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, true,
                                              conv::kThreads, false, true, 3>), grid, block, 0, s, a);
        else
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, false,
                                              conv::kThreads, false, true, 3>), grid, block, 0, s, a);
        return;
      }
      if (a.f16)
        hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, true,
                                            conv::kThreads, false, true>), grid, block, 0, s, a);
      else
        hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, false, STATS, BNB, BNR, false, ZSIB, BNR2, false,
                                            conv::kThreads, false, true>), grid, block, 0, s, a);
      return;
    }
  }
  if constexpr (BMT == 128 && STAGES == 1 && LDSEPI && NT == conv::kThreads) {
    // (not with BNR2: that epilogue spills at the 128-VGPR bound of 4 waves per SIMD)
    if constexpr (!BNR2) {
      if (g_conv_sk && !a.f16) {
        const int64_t tiles = (int64_t)a.m_tiles * a.n_tiles;
        const int G = conv_sk_blocks(tiles, (int)((int64_t)a.R * a.S * a.C / conv::BK), BN, g_conv_sk);
        SkWorkspace* ws = G > 0 ? sk_workspace(s) : nullptr;
        if (ws != nullptr && (size_t)G * (BN == 128 ? 65536u : 32768u) <= kSkPartBytes && G <= kSkMaxBlocks &&
            a.n_tiles * BN == a.Cout) {
          a.sk.part = ws->part;
          a.sk.flags = ws->flags;
          a.sk.err = ws->flags + kSkMaxBlocks;
          a.sk.G = G;
          a.sk.part_bytes = (uint32_t)kSkPartBytes;
          const dim3 sgrid((unsigned)(G + a.red.blocks));
          hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, 1, true, BKN, STATS, BNB, BNR, REMAP, ZSIB, BNR2, false,
                                              conv::kThreads, false, false, 1, true>),
                             sgrid, block, 0, s, a);
          return;
        }
      }
    }
    if (a.f16) {
      hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, STAGES, LDSEPI, BKN, STATS, BNB, BNR, REMAP, ZSIB, BNR2, true>),
                         grid, block, 0, s, a);
      return;
    }
  } else {
    if (a.f16) throw std::runtime_error("conv: fp16 runs the default kernel variant only");
  }
  hipLaunchKernelGGL((conv_fwd_kernel<BMT, BN, STAGES, LDSEPI, BKN, STATS, BNB, BNR, REMAP, ZSIB, BNR2, false, NT>),
                     grid, block, 0, s, a);
}

// ---- split-K for small grids ------------------------------------------------------------------
// A conv whose 128 x BN tile grid is far below one block per CU (ResNet-18 on 32x32 images:
// layer4 is 4 tiles at batch 128, each a 72-step K loop) is latency-bound on the K loop: split
// the K-steps over blocks (fp32 partials, summed by conv_split_epilogue_kernel).  Target ~2
// blocks per CU, at least 2 K-steps per split.  conv_set_splitk(0) disables it (A/B).
// 0 = never split, 1 = auto (the policy below), 2 = the in-graph policy everywhere (tests that
// compare eager with replayed steps); conv_set_splitk
static int g_splitk = 1;
static int splitk_mode() { return g_splitk; }
void conv_set_splitk(int mode) { g_splitk = mode; }
int conv_get_splitk() { return g_splitk; }

int conv_fwd_splits(int64_t M, int Cout, int64_t K, int* kps_out, hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const bool capturing = s != nullptr && hipStreamIsCapturing(s, &cs) == hipSuccess &&
                         cs == hipStreamCaptureStatusActive;
  return conv_fwd_splits_for(M, Cout, K, capturing, kps_out);
}

// Thresholds of the policy below: split grids of fewer than kSplitTiles tiles (eagerly: at most
// kSplitEager tiles with >= 24 K-steps) to about kSplitTarget blocks (512 / 1024 targets
// measured -1 % / -5 %, docs/DESIGN.md §7.2).
static int kSplitTiles = 160, kSplitEager = 32, kSplitTarget = 512, kSplitEagerMinK = 24;
// A/B knob (bench/ab_step.py): the thresholds above; a value <= 0 keeps the current one
void conv_set_splitk_policy(int tiles, int eager_tiles, int eager_min_k, int target) {
  if (tiles > 0) kSplitTiles = tiles;
  if (eager_tiles > 0) kSplitEager = eager_tiles;
  if (eager_min_k > 0) kSplitEagerMinK = eager_min_k;
  if (target > 0) kSplitTarget = target;
}

int conv_fwd_splits_for(int64_t M, int Cout, int64_t K, bool graph, int* kps_out) {
  const int n_tiles = Cout % 128 == 0 ? Cout / 128 : Cout / 64;
  const int64_t tiles = (int64_t)conv_m_tiles(M) * n_tiles;
  const int nk = (int)(K / conv::BK);
  if (kps_out) *kps_out = nk;
  const int mode = splitk_mode();
  if (mode == 0 || tiles >= kSplitTiles || nk < 4) return 1;
  // Eager launches are host-bound at these sizes: the extra epilogue launch only pays where the
  // single-block K loop is long (tens of microseconds); inside a hipGraph capture it always does.
  if (!graph && mode == 1 && (tiles > kSplitEager || nk < kSplitEagerMinK)) return 1;
  const int want = (int)((kSplitTarget + tiles - 1) / tiles);
  const int kps = std::max(2, (nk + want - 1) / want);
  const int splits = (nk + kps - 1) / kps;
  if (splits <= 1) return 1;
  if (kps_out) *kps_out = kps;
  return splits;
}

template <int BN, bool STATS, bool BNB, bool BNR, bool BNR2, bool BKN = false, bool REMAP = false, bool ZSIB = false>
static void split_launch(const ConvFwdArgs& a, hipStream_t s) {
  ConvFwdArgs am = a;  // the main kernel takes an attached backward-weight reduce, the epilogue not
  const dim3 grid((unsigned)(a.m_tiles * a.n_tiles * a.splits + take_attached_reduce(am))), block(conv::kThreads);
  conv_check_offsets(a, BKN);
  // the main loop's epilogue flags do not matter (SPLIT returns before it): one instantiation
  if (a.f16)
    hipLaunchKernelGGL((conv_fwd_kernel<128, BN, 1, true, BKN, false, false, false, false, false, false, true,
                                        conv::kThreads, true>), grid, block, 0, s, am);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<128, BN, 1, true, BKN, false, false, false, false, false, false, false,
                                        conv::kThreads, true>), grid, block, 0, s, am);
  const dim3 egrid((unsigned)((a.M + kSplitRows - 1) / kSplitRows), (unsigned)(a.Cout / 64));
  if (a.f16)
    hipLaunchKernelGGL((conv_split_epilogue_kernel<STATS, BNB, BNR, BNR2, REMAP, ZSIB, true>), egrid, dim3(256), 0, s,
                       a);
  else
    hipLaunchKernelGGL((conv_split_epilogue_kernel<STATS, BNB, BNR, BNR2, REMAP, ZSIB, false>), egrid, dim3(256), 0, s,
                       a);
}

// Launch the split-K path when the plan asks for it and a workspace was provided.  BNB
// statistics go to columns [bp_off, bp_off + ceil(M/16)) of the [C][bp_ld] partial arrays.
static bool maybe_split(ConvFwdArgs& a, float* ws, bool stats, bool bnb, bool bnr, bool bnr2, hipStream_t s,
                        bool bkn = false, bool remap = false, bool zsib = false) {
  if (ws == nullptr) return false;
  int kps = 0;
  const int splits = conv_fwd_splits(a.M, a.Cout, (int64_t)a.R * a.S * a.C, &kps, s);
  if (splits <= 1) return false;
  a.part = ws;
  a.splits = splits;
  a.kps = kps;
  a.n_tiles = a.Cout % 128 == 0 ? a.Cout / 128 : a.Cout / 64;
  const bool wide = a.Cout % 128 == 0;
#define DPT_SPLIT(...)                                      \
  do {                                                      \
    if (wide) split_launch<128, __VA_ARGS__>(a, s);         \
    else split_launch<64, __VA_ARGS__>(a, s);               \
  } while (0)
  if (remap) {
    if (bnb) DPT_SPLIT(false, true, false, false, true, true, false);
    else if (zsib) DPT_SPLIT(false, false, false, false, true, true, true);
    else DPT_SPLIT(false, false, false, false, true, true, false);
  } else if (stats) {
    DPT_SPLIT(true, false, false, false);
  } else if (bnb && bnr && bnr2) {
    DPT_SPLIT(false, true, true, true);
  } else if (bnb && bnr) {
    DPT_SPLIT(false, true, true, false);
  } else if (bnb) {
    DPT_SPLIT(false, true, false, false);
  } else {
    DPT_SPLIT(false, false, false, false);
  }
#undef DPT_SPLIT
  (void)bkn;
  return true;
}

template <int BMW, int BNW, int STAGES>
static void wgrad_launch(dim3 grid, dim3 block, hipStream_t s, const ConvWgradArgs& a) {
  if constexpr (STAGES == 1) {
    if (a.direct && !a.f16) {
      hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, STAGES, false, conv::kThreads, true>), grid, block, 0, s, a);
      return;
    }
    if (a.f16) {
      hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, STAGES, true>), grid, block, 0, s, a);
      return;
    }
  } else {
    if (a.f16) throw std::runtime_error("conv_wgrad: fp16 runs the default kernel variant only");
  }
  hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, STAGES, false>), grid, block, 0, s, a);
}

template <int BN>
static void conv_fwd_dispatch(int variant, bool bkn, ConvFwdArgs a, hipStream_t s) {
  if (a.f16) variant = 4;
  if (variant == 0) variant = 4;  // measured best at every ResNet-50 shape but two (profiles/conv_*.md)
  const dim3 block(conv::kThreads);
  const int mt128 = a.m_tiles;
  if (variant >= 5 && !bkn) {  // 256-row blocks (4 row tiles per wave)
    a.mt256 = (mt128 + 1) / 2;  // m_tiles stays the 128-row count: the BN-partials layout
    const dim3 grid((unsigned)(a.mt256 * a.n_tiles));
    if (variant == 5) fwd_launch<256, BN, 1, false, false>(grid, block, s, a);
    else fwd_launch<256, BN, 1, true, false>(grid, block, s, a);
    return;
  }
  const dim3 grid((unsigned)(a.m_tiles * a.n_tiles));
  const int nk32 = a.R * a.S * (a.C / 32);
  if (!bkn && (variant == 7 || variant == 8 || variant == 14)) {
    const bool st = a.psum != nullptr;
    if (variant == 14) {  // 2-stage BK = 32 ring: the same 32 KiB of operand LDS as the 1-stage tile
      if (st) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 2, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 2, false>), grid, block, 0, s, a);
    } else if (variant == 7) {
      if (st) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 3, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 3, false>), grid, block, 0, s, a);
    } else {
      if (st) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 4, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN, 4, false>), grid, block, 0, s, a);
    }
    return;
  }
  (void)nk32;
  if (bkn) {
    fwd_launch<128, BN, 1, true, true>(grid, block, s, a);
    return;
  }
  switch (variant) {
    case 2: fwd_launch<128, BN, 2, false, false>(grid, block, s, a); break;
    case 3: fwd_launch<128, BN, 1, false, false>(grid, block, s, a); break;
    case 4:
      if (a.psum) fwd_launch<128, BN, 1, true, false, true>(grid, block, s, a);
      else fwd_launch<128, BN, 1, true, false, false>(grid, block, s, a);
      break;
    default: fwd_launch<128, BN, 2, true, false>(grid, block, s, a); break;
  }
}

// 8-wave (512-thread) variants: 9 = 256x256 tile, 10 = 256x128, 11 = 128x256 (2 stages);
// 12 = 256x128, 13 = 128x256 with the 3-stage pipelined K loop (two K-tiles in flight across
// one raw barrier per step).  Returns false when the shape does not fit the variant's N tile.
static int big_bn(int v) { return (v == 10 || v == 12) ? 128 : 256; }
static int big_bm(int v) { return (v == 11 || v == 13) ? 128 : 256; }
static bool conv_fwd_big(int v, ConvFwdArgs& a, hipStream_t s) {
  const int bn = big_bn(v), bm = big_bm(v);
  if (a.Cout % bn) return false;
  a.n_tiles = a.Cout / bn;
  a.mt256 = (int)((a.M + 255) / 256);
  const int mt = bm == 256 ? a.mt256 : a.m_tiles;
  const dim3 grid((unsigned)(mt * a.n_tiles)), block(512);
  const bool st = a.psum != nullptr;
  if (v == 12) {
    if (st) fwd_launch<256, 128, 3, true, false, true, false, false, false, false, false, 512>(grid, block, s, a);
    else fwd_launch<256, 128, 3, true, false, false, false, false, false, false, false, 512>(grid, block, s, a);
  } else if (v == 13) {
    if (st) fwd_launch<128, 256, 3, true, false, true, false, false, false, false, false, 512>(grid, block, s, a);
    else fwd_launch<128, 256, 3, true, false, false, false, false, false, false, false, 512>(grid, block, s, a);
  } else if (v == 9) {
    if (st) fwd_launch<256, 256, 2, true, false, true, false, false, false, false, false, 512>(grid, block, s, a);
    else fwd_launch<256, 256, 2, true, false, false, false, false, false, false, false, 512>(grid, block, s, a);
  } else if (v == 10) {
    if (st) fwd_launch<256, 128, 2, true, false, true, false, false, false, false, false, 512>(grid, block, s, a);
    else fwd_launch<256, 128, 2, true, false, false, false, false, false, false, false, 512>(grid, block, s, a);
  } else {
    if (st) fwd_launch<128, 256, 2, true, false, true, false, false, false, false, false, 512>(grid, block, s, a);
    else fwd_launch<128, 256, 2, true, false, false, false, false, false, false, false, 512>(grid, block, s, a);
  }
  return true;
}

// Per-shape forward tile policy (variant 0 only; bits, conv_set_fwd_shape_policy):
//   1: expanding 1x1 convs with the BN-statistics epilogue (C <= 128, Cout >= 2C) -> 256-row
//      blocks with the LDS epilogue (variant 6): the statistics partials are summed over 256
//      rows per block instead of 128 (64->256 @56: 0.155 -> 0.130 ms with statistics, MIOpen
//      0.106 without; bench/conv_variant_sweep.py, profiles/conv_variant_sweep_r4.md);
//   2: the 3x3 stride-2 256->256 conv (K = 2304, M >= 32768) -> the 8-wave 256x256 tile (variant
//      9): 0.081 -> 0.069 ms, 1.05-1.08x MIOpen.
//   16: the s2d stem's 4x4 conv (C = 16) on the 2-stage K loop (variant 1).
//   4 / 8: 1x1 stride-1 convs with the statistics epilogue on grids under 1,024 tiles (the deep
//      reducing convs at 14x14 / 7x7, latency-bound with ~3 resident blocks per CU:
//      profiles/step_pmc_r5.md) -> the BK = 32 pipelined K loop, 2 stages (variant 14, 4 blocks
//      per CU) / 3 stages (variant 7).
static int g_fwd_shape_policy = 0;
void conv_set_fwd_shape_policy(int bits) { g_fwd_shape_policy = bits; }
static int fwd_shape_variant(const ConvFwdArgs& a, bool stats) {
  if (a.f16) return 0;
  if ((g_fwd_shape_policy & 1) && stats && a.R == 1 && a.S == 1 && a.stride == 1 && a.C <= 128 &&
      a.Cout >= 2 * a.C)
    return 6;
  if ((g_fwd_shape_policy & 2) && a.R == 3 && a.stride == 2 && a.Cout == 256 && a.C == 256 && a.M >= 32768)
    return 9;
  if ((g_fwd_shape_policy & 12) && stats && a.R == 1 && a.S == 1 && a.stride == 1 && a.C % 32 == 0 &&
      (int64_t)a.m_tiles * a.n_tiles < 1024)
    return (g_fwd_shape_policy & 4) ? 14 : 7;
  // 16: the 16-channel space-to-depth stem (4 K-steps, 6 resident blocks per CU, latency-bound)
  // on the double-buffered K loop (variant 1)
  if ((g_fwd_shape_policy & 16) && a.C == 16) return 1;
  return 0;
}

static void conv_fwd_impl(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int C, int Cout,
                          int R, int S, int stride, int pad, float* psum, float* psq, bool bkn, hipStream_t s,
                          int Ho = 0, int Wo = 0, bool f16 = false, float* ws = nullptr) {
  ConvFwdArgs a;
  a.part = nullptr; a.splits = 1; a.kps = 0;
  a.f16 = f16 ? 1 : 0;
  a.x = x; a.w = w; a.y = y; a.psum = psum; a.psq = psq;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  // explicit output size: asymmetric padding (pad on top/left only, e.g. the space-to-depth stem)
  a.Ho = Ho > 0 ? Ho : (H + 2 * pad - R) / stride + 1;
  a.Wo = Wo > 0 ? Wo : (W + 2 * pad - S) / stride + 1;
  a.M = (int64_t)N * a.Ho * a.Wo;
  a.m_tiles = conv_m_tiles(a.M);
  a.Rw = R; a.Sw = S; a.tr0 = R - 1; a.trs = -1; a.ts0 = S - 1; a.tss = -1;  // BKN: flipped taps
  const bool wide = Cout % 128 == 0;
  a.n_tiles = Cout / (wide ? 128 : 64);
  a.mt256 = 0;
  int v = fwd_variant();
  if (!bkn && maybe_split(a, ws, psum != nullptr, false, false, false, s)) return;
  if (!bkn && v == 0) v = fwd_shape_variant(a, psum != nullptr);
  if (!bkn && !a.f16) {
    const int vb = (v >= 9 && v <= 13) ? v : v == 0 ? conv_big_auto(a.M, Cout, (int64_t)R * S * C, R * S) : 0;
    if (vb && conv_fwd_big(vb, a, s)) return;
  }
  if (wide) conv_fwd_dispatch<128>(v, bkn, a, s);
  else conv_fwd_dispatch<64>(v, bkn, a, s);
}

// Stride-1 backward-data through a flipped/transposed weight wt [C][R][S][Cout] (the forward
// kernel on dy), whose epilogue also sums the backward statistics of the BatchNorm+ReLU that
// produced the conv's input (BNB epilogue).  bnx/dx: [N, Ho, Wo, C].
void launch_conv_dgrad_bnstats(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, int N, int Ho, int Wo, int Cout,
                               int C, int R, int S, int pad, const uint16_t* bnx, const float* bn_mean,
                               const float* bn_coef, float* bp1, float* bp2, hipStream_t s,
                               const uint16_t* bny, const uint16_t* bnres, const uint16_t* bnx2,
                               const float* bn_mean2, float* bp3, bool f16, float* ws, const uint8_t* bnmask) {
  ConvFwdArgs a;
  a.part = nullptr; a.splits = 1; a.kps = 0;
  a.f16 = f16 ? 1 : 0;
  a.x = dy; a.w = wt; a.y = dx; a.psum = nullptr; a.psq = nullptr;
  a.N = N; a.H = Ho; a.W = Wo; a.C = Cout; a.Cout = C; a.R = R; a.S = S; a.stride = 1; a.pad = R - 1 - pad;
  a.Ho = Ho + 2 * a.pad - R + 1;
  a.Wo = Wo + 2 * a.pad - S + 1;
  a.M = (int64_t)N * a.Ho * a.Wo;
  a.m_tiles = conv_m_tiles(a.M);
  a.mt256 = 0;
  a.bnx = bnx; a.bn_mean = bn_mean; a.bn_coef = bn_coef; a.bp1 = bp1; a.bp2 = bp2;
  a.bny = bny; a.bnres = bnres; a.bnmask = bnmask;
  a.bnx2 = bnx2; a.bn_mean2 = bn_mean2; a.bp3 = bp3;
  a.bp_ld = a.m_tiles; a.bp_off = 0;
  const bool res = bny != nullptr;
  const dim3 block(conv::kThreads);
  {
    const int64_t keep_ld = a.bp_ld;
    a.bp_ld = conv_split_cols(a.M);  // split: one partial column per 16-row slab
    if (maybe_split(a, ws, false, true, res, res && bnx2 != nullptr, s)) return;
    a.bp_ld = keep_ld;
  }
  const bool two = res && bnx2 != nullptr;
  const int cv = fwd_variant();
  if (!f16 && (cv == 0 || (cv >= 9 && cv <= 13))) {
    // 8-wave tiles (conv_big_auto, or a forced variant): N = C, K = Cout*R*S
    const int vb = cv ? cv : conv_big_auto(a.M, C, (int64_t)Cout * R * S, R * S);
    if (vb && C % big_bn(vb) == 0) {
      const int bn = big_bn(vb), bm = big_bm(vb);
      a.n_tiles = C / bn;
      a.mt256 = (int)((a.M + 255) / 256);
      const dim3 g((unsigned)((bm == 256 ? a.mt256 : a.m_tiles) * a.n_tiles));
      if (vb == 12) {
        if (two) fwd_launch<256, 128, 3, true, false, false, true, true, false, false, true, 512>(g, block, s, a);
        else if (res) fwd_launch<256, 128, 3, true, false, false, true, true, false, false, false, 512>(g, block, s, a);
        else fwd_launch<256, 128, 3, true, false, false, true, false, false, false, false, 512>(g, block, s, a);
      } else if (vb == 13) {
        if (two) fwd_launch<128, 256, 3, true, false, false, true, true, false, false, true, 512>(g, block, s, a);
        else if (res) fwd_launch<128, 256, 3, true, false, false, true, true, false, false, false, 512>(g, block, s, a);
        else fwd_launch<128, 256, 3, true, false, false, true, false, false, false, false, 512>(g, block, s, a);
      } else if (vb == 9) {
        if (two) fwd_launch<256, 256, 2, true, false, false, true, true, false, false, true, 512>(g, block, s, a);
        else if (res) fwd_launch<256, 256, 2, true, false, false, true, true, false, false, false, 512>(g, block, s, a);
        else fwd_launch<256, 256, 2, true, false, false, true, false, false, false, false, 512>(g, block, s, a);
      } else if (vb == 10) {
        if (two) fwd_launch<256, 128, 2, true, false, false, true, true, false, false, true, 512>(g, block, s, a);
        else if (res) fwd_launch<256, 128, 2, true, false, false, true, true, false, false, false, 512>(g, block, s, a);
        else fwd_launch<256, 128, 2, true, false, false, true, false, false, false, false, 512>(g, block, s, a);
      } else {
        a.n_tiles = 0;  // unsupported forced variant for this pass: fall through to the default
      }
      if (a.n_tiles) return;
    }
  }
  a.n_tiles = C % 128 == 0 ? C / 128 : C / 64;
  const dim3 grid((unsigned)(a.m_tiles * a.n_tiles));
  if (C % 128 == 0) {
    if (two) fwd_launch<128, 128, 1, true, false, false, true, true, false, false, true>(grid, block, s, a);
    else if (res) fwd_launch<128, 128, 1, true, false, false, true, true>(grid, block, s, a);
    else fwd_launch<128, 128, 1, true, false, false, true>(grid, block, s, a);
  } else {
    if (two) fwd_launch<128, 64, 1, true, false, false, true, true, false, false, true>(grid, block, s, a);
    else if (res) fwd_launch<128, 64, 1, true, false, false, true, true>(grid, block, s, a);
    else fwd_launch<128, 64, 1, true, false, false, true>(grid, block, s, a);
  }
}

// A Linear's backward-data with the exact-GELU backward of its input fused into the epilogue
// (ViT's fc2 -> GELU -> fc1 chain): gu[t, i] = (sum_o dy[t, o] wt[i, o]) * gelu'(u[t, i] + bias[i])
// and bp1[i][mt] = the column sums of gu over 128-row tile mt (the bias gradient's partials).
// dy [T, n_out], wt [n_in, n_out] (the weight transposed), u / gu [T, n_in] 16-bit, bias fp32.
void launch_linear_dgrad_dgelu(const uint16_t* dy, const uint16_t* wt, const uint16_t* u, const float* bias,
                               const uint16_t* bias16, uint16_t* gu, float* bp1, int64_t T, int n_out, int n_in,
                               bool f16, hipStream_t s) {
  if (n_in % 128 != 0 || n_out % 64 != 0) throw std::runtime_error("linear_dgrad_dgelu: n_in % 128, n_out % 64");
  ConvFwdArgs a;
  a.part = nullptr; a.splits = 1; a.kps = 0;
  a.f16 = f16 ? 1 : 0;
  a.x = dy; a.w = wt; a.y = gu; a.psum = nullptr; a.psq = nullptr;
  a.N = 1; a.H = 1; a.W = (int)T; a.C = n_out; a.Cout = n_in; a.R = 1; a.S = 1; a.stride = 1; a.pad = 0;
  a.Ho = 1; a.Wo = (int)T;
  a.M = T;
  a.m_tiles = conv_m_tiles(a.M);
  a.mt256 = 0;
  a.n_tiles = n_in / 128;
  a.bnx = u; a.bn_mean = bias; a.bias16 = bias16; a.bn_coef = nullptr; a.bp1 = bp1; a.bp2 = nullptr;
  a.bny = nullptr; a.bnres = nullptr; a.bnmask = nullptr; a.bnx2 = nullptr; a.bn_mean2 = nullptr; a.bp3 = nullptr;
  a.bp_ld = a.m_tiles; a.bp_off = 0;
  conv_check_offsets(a, false);
  const dim3 grid((unsigned)(a.m_tiles * a.n_tiles)), block(conv::kThreads);
  if (f16)
    hipLaunchKernelGGL((conv_fwd_kernel<128, 128, 1, true, false, false, true, false, false, false, false, true,
                                        conv::kThreads, false, false, 1, false, true>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<128, 128, 1, true, false, false, true, false, false, false, false, false,
                                        conv::kThreads, false, false, 1, false, true>), grid, block, 0, s, a);
}

int linear_dgrad_dgelu_tiles(int64_t T) { return conv_m_tiles(T); }

void launch_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int C, int Cout,
                     int R, int S, int stride, int pad, float* psum, float* psq, hipStream_t s, int Ho, int Wo,
                     bool f16, float* ws) {
  conv_fwd_impl(x, w, y, N, H, W, C, Cout, R, S, stride, pad, psum, psq, false, s, Ho, Wo, f16, ws);
}

// Stride-1 backward-data: dx[N,H,W,C] = conv(dy, flip(w)^T, pad' = R-1-pad) with the flip and
// transpose done by the B-operand addressing (no weight copy).
void launch_conv_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int N, int Ho, int Wo, int Cout, int C,
                       int R, int S, int pad, hipStream_t s, bool f16) {
  conv_fwd_impl(dy, w, dx, N, Ho, Wo, Cout, C, R, S, 1, R - 1 - pad, nullptr, nullptr, true, s, 0, 0, f16);
}

// Strided backward-data (stride 2, any R/S/pad) straight from the KRSC weight w [Cout,R,S,C]:
// dx [N,H,W,C] splits into the four parity classes (h % 2, w % 2).  Class (ph, pw) is a
// stride-1, top/left-unpadded conv of dy [N,Ho,Wo,Cout] with the taps r = r0 + 2j (r = h + pad
// - 2i, r = ph + pad mod 2), taken in decreasing r so the dy row index increases with the GEMM
// tap; its output rows land on (2a + ph, 2b + pw) (REMAP epilogue).  A class with no taps
// (e.g. the odd classes of a 1x1 / stride-2 conv) gets zeros from the class-(0,0) launch (ZSIB)
// - every dx element is written exactly once, no memset pass.
// Parity-class geometry of the stride-2 backward-data (one stride-1 conv per non-empty class).
struct S2Class {
  int ph, pw, Rc, Sc, pad, Ha, Wa, tr0, ts0;
  bool zsib;
};
static int s2_classes(int H, int W, int R, int S, int pad, S2Class* out) {
  int J[2], r0[2], Js[2], s0[2], D[2];
  for (int ph = 0; ph < 2; ++ph) {
    r0[ph] = ((ph + pad) % 2 + 2) % 2;
    J[ph] = r0[ph] < R ? (R - 1 - r0[ph]) / 2 + 1 : 0;
    D[ph] = (ph + pad - r0[ph]) / 2;  // dy row of tap r0 for a = 0
    s0[ph] = r0[ph];
    Js[ph] = s0[ph] < S ? (S - 1 - s0[ph]) / 2 + 1 : 0;
  }
  const bool zsib = J[1] == 0 && Js[1] == 0 && J[0] > 0 && Js[0] > 0;
  int n = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      const int Ha = (H - ph + 1) / 2, Wa = (W - pw + 1) / 2;
      if (Ha <= 0 || Wa <= 0 || J[ph] == 0 || Js[pw] == 0) continue;
      // GEMM tap jj (0..J-1) reads dy row a + D - (J-1) + jj, weight tap r0 + 2*(J-1-jj)
      const int pad_c = J[ph] - 1 - D[ph];
      if (Js[pw] - 1 - D[pw] != pad_c) throw std::runtime_error("conv_dgrad_s2: unequal class paddings");
      out[n++] = S2Class{ph, pw, J[ph], Js[pw], pad_c, Ha, Wa, r0[ph] + 2 * (J[ph] - 1), s0[pw] + 2 * (Js[pw] - 1),
                         zsib && ph == 0 && pw == 0};
    }
  return n;
}

ConvS2Plan conv_dgrad_s2_plan(int N, int H, int W, int C, int Cout, int R, int S, int pad, hipStream_t s) {
  S2Class cl[4];
  const int n = s2_classes(H, W, R, S, pad, cl);
  ConvS2Plan pl{0, 0};
  for (int i = 0; i < n; ++i) {
    const int64_t M = (int64_t)N * cl[i].Ha * cl[i].Wa;
    const int splits = conv_fwd_splits(M, C, (int64_t)cl[i].Rc * cl[i].Sc * Cout, nullptr, s);
    pl.chunks += splits > 1 ? conv_split_cols(M) : conv_m_tiles(M);
    if (splits > 1) pl.ws_floats = std::max(pl.ws_floats, (int64_t)splits * M * C);
  }
  return pl;
}

int conv_dgrad_s2_chunks(int N, int H, int W, int R, int S, int pad) {
  S2Class cl[4];
  const int n = s2_classes(H, W, R, S, pad, cl);
  int chunks = 0;
  for (int i = 0; i < n; ++i) chunks += conv_m_tiles((int64_t)N * cl[i].Ha * cl[i].Wa);
  return chunks;
}

void launch_conv_dgrad_s2(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int N, int Ho, int Wo, int Cout,
                          int C, int R, int S, int pad, int H, int W, hipStream_t s, const uint16_t* bnx,
                          const float* bn_mean, const float* bn_coef, float* bp1, float* bp2, bool f16, float* ws) {
  const bool bnb = bnx != nullptr;
  // with a workspace the classes may split (the caller sized ws and bp_ld by conv_dgrad_s2_plan)
  const int bp_ld = bnb ? (ws ? conv_dgrad_s2_plan(N, H, W, C, Cout, R, S, pad, s).chunks
                              : conv_dgrad_s2_chunks(N, H, W, R, S, pad))
                        : 0;
  int bp_off = 0;
  S2Class cl[4];
  const int ncl = s2_classes(H, W, R, S, pad, cl);
  for (int ci = 0; ci < ncl; ++ci) {
    const S2Class& k = cl[ci];
    ConvFwdArgs a;
    a.part = nullptr; a.splits = 1; a.kps = 0;
    a.f16 = f16 ? 1 : 0;
    a.x = dy; a.w = w; a.y = dx; a.psum = nullptr; a.psq = nullptr;
    a.N = N; a.H = Ho; a.W = Wo; a.C = Cout; a.Cout = C; a.R = k.Rc; a.S = k.Sc; a.stride = 1;
    a.pad = k.pad;
    a.Ho = k.Ha; a.Wo = k.Wa;
    a.M = (int64_t)N * k.Ha * k.Wa;
    a.m_tiles = conv_m_tiles(a.M);
    a.mt256 = 0;
    a.Rw = R; a.Sw = S;
    a.tr0 = k.tr0; a.trs = -2;
    a.ts0 = k.ts0; a.tss = -2;
    a.oH = H; a.oW = W; a.oph = k.ph; a.opw = k.pw;
    a.bnx = bnx; a.bny = nullptr; a.bnres = nullptr; a.bn_mean = bn_mean; a.bn_coef = bn_coef;
    a.bnx2 = nullptr; a.bn_mean2 = nullptr; a.bp3 = nullptr;
    a.bp1 = bp1; a.bp2 = bp2; a.bp_ld = bp_ld; a.bp_off = bp_off;
    const bool z = k.zsib;
    // zero classes (ZSIB) only arise for 1x1 kernels, whose input is never a fused BN+ReLU output
    // in the models here: BNB and ZSIB are not combined
    if (bnb && z) throw std::runtime_error("conv_dgrad_s2: BN statistics with zero-filled classes unsupported");
    if (maybe_split(a, ws, false, bnb, false, false, s, true, true, z)) {
      bp_off += conv_split_cols(a.M);
      continue;
    }
    bp_off += a.m_tiles;
    const dim3 block(conv::kThreads);
    a.n_tiles = C % 128 == 0 ? C / 128 : C / 64;
    const dim3 grid((unsigned)(a.m_tiles * a.n_tiles));
    if (bnb) {
      if (C % 128 == 0) fwd_launch<128, 128, 1, true, true, false, true, false, true, false>(grid, block, s, a);
      else fwd_launch<128, 64, 1, true, true, false, true, false, true, false>(grid, block, s, a);
      continue;
    }
    if (C % 128 == 0) {
      if (z) fwd_launch<128, 128, 1, true, true, false, false, false, true, true>(grid, block, s, a);
      else fwd_launch<128, 128, 1, true, true, false, false, false, true, false>(grid, block, s, a);
    } else {
      if (z) fwd_launch<128, 64, 1, true, true, false, false, false, true, true>(grid, block, s, a);
      else fwd_launch<128, 64, 1, true, true, false, false, false, true, false>(grid, block, s, a);
    }
  }
}

// conv_wgrad_halo_kernel modes: 0 off, 1 / 2: 128-channel strips, 3 / 4: 64-channel strips
// (even: double-buffered), 5 auto (default; conv_set_wgrad_halo for A/B): mode 3 for 64-channel inputs,
// where the per-tap kernel's two-tap tiles waste 1/9 of their MFMA work on a ragged last tile
// (64x56x56 -> 64: 0.118 -> 0.085-0.095 ms); the per-tap kernel elsewhere (the halo's W+2
// padding costs 7-29 % more MFMA work and measured level or slower at 128-512 channels,
// profiles/wgrad_halo_r2.md)
static int g_wgrad_halo = 5;
static int wgrad_halo_mode(int C = 0) {
  if (g_wgrad_halo == 5) return C == 64 ? 3 : 0;
  if (g_wgrad_halo == 6) return C == 64 ? 4 : 0;  // A/B: the double-buffered strip on the same convs
  return g_wgrad_halo;
}
void conv_set_wgrad_halo(int on) { g_wgrad_halo = on; }

static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) { f.mul = 0; f.shr = 0; return f; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;  // l = ceil(log2 d) >= 1
  // mul = ceil(2^(31+l) / d) < 2^32; q = mulhi(n, mul) >> (l-1) is exact for n < 2^31
  // (error term n * (mul - 2^(31+l)/d) / 2^(31+l) < 1/d).
  f.mul = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
  f.shr = l - 1;
  return f;
}

// Block target of the split-K backward-weight plan.  Measured per ResNet-50 shape at batch 256
// (bench/wgrad_target_sweep.py, profiles/wgrad_target_sweep_r3.md): 1x1 / stride-1 convs (one
// tap, streaming both operands once) want ~512 blocks - fewer fp32 partial tiles to write and
// reduce; convs with taps or a stride want more blocks to hide their K loop, 768 on the long
// (>= 3136 K-step) reductions and 640 on the shorter ones.  Step total 3.65 -> 3.49 ms.
// conv_set_wgrad_target(n > 0): n blocks for every shape (the sweep); 0: this policy.
static int g_wgrad_target = 0;
void conv_set_wgrad_target(int blocks) { g_wgrad_target = blocks; }
// backward-weight K loop depth (A/B, conv_set_wgrad_stages): 0 = the single-stage tile (4 blocks
// per CU); 1 = the double-buffered tile (2 blocks per CU) for grids of at most one wave at 2
// blocks per CU - there residency is set by the grid, not by LDS, so the deeper pipeline costs
// no resident block; 2 = double-buffered everywhere
static int g_wgrad_stages = 0;
void conv_set_wgrad_stages(int mode) { g_wgrad_stages = mode; }
static int wgrad_target(int R, int S, int stride, int steps) {
  if (g_wgrad_target > 0) return g_wgrad_target;
  if (R * S == 1 && stride == 1) return 512;
  return steps >= 3136 ? 768 : 640;
}

ConvWgradPlan conv_wgrad_plan(int N, int H, int W, int C, int Cout, int R, int S, int stride, int pad, int Ho,
                              int Wo, int target_blocks) {
  ConvWgradPlan pl;
  pl.Ho = Ho > 0 ? Ho : (H + 2 * pad - R) / stride + 1;
  pl.Wo = Wo > 0 ? Wo : (W + 2 * pad - S) / stride + 1;
  const int64_t M = (int64_t)N * pl.Ho * pl.Wo;
  const int hmode = wgrad_halo_mode(C);
  if (hmode && R == 3 && S == 3 && stride == 1 && pad == 1 && pl.Ho == H && pl.Wo == W &&
      C % (hmode >= 3 ? 64 : 128) == 0 && Cout % 64 == 0 && (int64_t)N * H * (W + 2) + 128 < (1ll << 31)) {
    // conv_wgrad_halo_kernel: 64 x BNW x 3-tap tiles over N*H*(W+2) padded pixels (modes 1/2:
    // BNW = 128, 2 blocks per CU; 3/4: BNW = 64, 4 per CU; even modes double-buffer)
    pl.halo = hmode;
    pl.bmw = 64;
    pl.bnw = pl.halo >= 3 ? 64 : 128;
    const int tiles = (Cout / 64) * 3 * (C / pl.bnw);
    const int steps = (int)(((int64_t)N * H * (W + 2) + 63) / 64);
    const int target = g_wgrad_target > 0 ? g_wgrad_target : pl.bnw == 128 ? 512 : 768;
    int splits = (target + tiles - 1) / tiles;
    const int min_steps = (int64_t)tiles * (steps / 32) >= 512 ? 32 : 2;
    splits = std::max(1, std::min(splits, steps / min_steps));
    pl.steps_per_split = (steps + splits - 1) / splits;
    pl.splits = (steps + pl.steps_per_split - 1) / pl.steps_per_split;
    pl.part_floats = pl.splits > 1 ? (int64_t)pl.splits * Cout * 9 * C : 0;
    return pl;
  }
  pl.bmw = Cout % 128 == 0 ? 128 : 64;
  // column tile: 128 input channels of one tap; 64-channel inputs take two taps per tile (a
  // ragged last tile for odd tap counts: 3x3 -> 5 tiles, 1/9 of the MFMA work wasted, twice
  // the MFMA work per staged dy tile); the 16-channel space-to-depth stem takes all 16 taps of
  // its 4x4 window in one 256-column tile (dy staged once instead of four times)
  pl.bnw = C % 128 == 0 ? 128 : (C == 64 && R * S > 1) ? 128 : (C == 16 && R * S * C >= 256 && pl.bmw == 64) ? 256 : 64;
  // variant 20 (A/B, bench/wgrad_variants.py): 8-wave 256 x 256 tiles where both channel counts
  // allow them.  Its own code: 10-13 select forward/dgrad tile variants (conv_fwd_big).
  if (conv_variant() == 20 && Cout % 256 == 0 && C % 256 == 0) pl.bmw = pl.bnw = 256;
  const int tiles = (Cout / pl.bmw) * ((R * S * C + pl.bnw - 1) / pl.bnw);
  const int steps = (int)((M + 63) / 64);
  // ~768 blocks (3 per CU) and at least 32 K-steps per split: a split's fp32 partial tile
  // (BMW x BNW x 4 B, written once and read once by the reduce) then costs < 1/8 of the
  // operand bytes it streams.  Small problems that cannot fill the chip that way (ResNet-18 on
  // 32x32 images: 2-128 K-steps) are K-loop-latency-bound instead: down to 2 K-steps per split.
  int splits = ((target_blocks > 0 ? target_blocks : wgrad_target(R, S, stride, steps)) + tiles - 1) / tiles;
  const int min_steps = (int64_t)tiles * (steps / 32) >= 512 ? 32 : 2;
  splits = std::max(1, std::min(splits, steps / min_steps));
  pl.steps_per_split = (steps + splits - 1) / splits;
  pl.splits = (steps + pl.steps_per_split - 1) / pl.steps_per_split;
  pl.part_floats = pl.splits > 1 ? (int64_t)pl.splits * Cout * R * S * C : 0;
  return pl;
}

void launch_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* part, void* dw, int dw_kind, int N, int H,
                       int W, int C, int Cout, int R, int S, int stride, int pad, const ConvWgradPlan& pl,
                       hipStream_t st, bool f16, WgradReduce* defer) {
  ConvWgradArgs a;
  a.f16 = f16 ? 1 : 0;
  const bool direct_out = pl.splits == 1 && dw_kind == 0;  // fp32 result written in place
  if (defer != nullptr) defer->consumed = true;              // nothing pending unless set below
  a.dy = dy; a.x = x; a.part = direct_out ? static_cast<float*>(dw) : part;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  a.Ho = pl.Ho; a.Wo = pl.Wo;
  a.M = N * pl.Ho * pl.Wo;
  a.co_tiles = Cout / pl.bmw;
  a.n_tiles = (R * S * C + pl.bnw - 1) / pl.bnw;
  a.splits = pl.splits;
  a.steps_per_split = pl.steps_per_split;
  a.div_wo = make_fastdiv((uint32_t)pl.Wo);
  a.div_howo = make_fastdiv((uint32_t)(pl.Ho * pl.Wo));
  a.direct = (R == 1 && S == 1 && stride == 1 && pad == 0) ? 1 : 0;
  // the kernel's 32-bit element offsets (rows up to one K-step past the end are addressed,
  // never loaded)
  if (((int64_t)a.M + 64) * Cout >= (1ll << 31) || ((int64_t)N + 1) * H * W * C >= (1ll << 31))
    throw std::runtime_error("conv_wgrad: activation tensors beyond 2^31 elements are not supported");
  {
    const int howo = pl.Ho * pl.Wo, q = 64 / howo, rem = 64 % howo, bq = rem / pl.Wo, cq = rem % pl.Wo;
    a.dw_step = cq * stride; a.wwrap = pl.Wo * stride;
    a.dh_step = bq * stride; a.hwrap = pl.Ho * stride;
    if (a.direct) {
      a.dp_w = 64 * C; a.dp_wwrap = a.dp_h = a.dp_hwrap = 0;
    } else {
      a.dp_w = (cq * stride + q * H * W) * C;
      a.dp_wwrap = (stride * W - pl.Wo * stride) * C;
      a.dp_h = bq * stride * W * C;
      a.dp_hwrap = (H * W - pl.Ho * stride * W) * C;
    }
  }
  if (pl.halo) {
    a.co_tiles = Cout / 64;
    a.n_tiles = 3 * (C / pl.bnw);
    a.Mp = N * H * (W + 2);
    a.div_wp = make_fastdiv((uint32_t)(W + 2));
    a.div_h = make_fastdiv((uint32_t)H);
  }
  dim3 grid((unsigned)(a.co_tiles * a.n_tiles * a.splits)), block(conv::kThreads);
  const int v = a.f16 ? 0 : fwd_variant();
  if (pl.halo) {
#define DPT_WH(BNW, ST)                                                                      \
  do {                                                                                       \
    if (a.f16) hipLaunchKernelGGL((conv_wgrad_halo_kernel<BNW, ST, true>), grid, block, 0, st, a);  \
    else hipLaunchKernelGGL((conv_wgrad_halo_kernel<BNW, ST, false>), grid, block, 0, st, a);       \
  } while (0)
    switch (pl.halo) {
      case 2: DPT_WH(128, 2); break;
      case 3: DPT_WH(64, 1); break;
      case 4: DPT_WH(64, 2); break;
      default: DPT_WH(128, 1); break;
    }
#undef DPT_WH
  } else if (pl.bmw == 256 && pl.bnw == 64) {
    wgrad_launch<256, 64, 1>(grid, block, st, a);
  } else if (pl.bmw == 256) {  // conv_wgrad_plan chose the 8-wave 256 x 256 tile
    if (a.f16) throw std::runtime_error("conv_wgrad: the 256 x 256 variant is bf16 only");
    hipLaunchKernelGGL((conv_wgrad_kernel<256, 256, 2, false, 512>), grid, dim3(512), 0, st, a);
  } else if ((v == 1 || v == 2 || (!a.f16 && (g_wgrad_stages == 2 ||
                                             (g_wgrad_stages == 1 && grid.x <= 2u * 256u)))) && pl.bnw <= 128) {
    if (pl.bmw == 128 && pl.bnw == 128) wgrad_launch<128, 128, 2>(grid, block, st, a);
    else if (pl.bmw == 128) wgrad_launch<128, 64, 2>(grid, block, st, a);
    else if (pl.bnw == 128) wgrad_launch<64, 128, 2>(grid, block, st, a);
    else wgrad_launch<64, 64, 2>(grid, block, st, a);
  } else {
    if (pl.bmw == 128 && pl.bnw == 128) wgrad_launch<128, 128, 1>(grid, block, st, a);
    else if (pl.bmw == 128) wgrad_launch<128, 64, 1>(grid, block, st, a);
    else if (pl.bnw == 256) wgrad_launch<64, 256, 1>(grid, block, st, a);
    else if (pl.bnw == 128) wgrad_launch<64, 128, 1>(grid, block, st, a);
    else wgrad_launch<64, 64, 1>(grid, block, st, a);
  }
  if (direct_out) return;
  const WgradReduce r{part, dw, (int64_t)Cout * R * S * C / 4, pl.splits, dw_kind, false};
  if (defer != nullptr) *defer = r;
  else launch_wgrad_reduce(r, st);
}

void launch_conv_wt_flip(const uint16_t* w, uint16_t* wt, int Cout, int R, int S, int C, hipStream_t s) {
  const int64_t n = (int64_t)Cout * R * S * C;
  hipLaunchKernelGGL(conv_wt_flip_kernel, dim3((unsigned)grid_for(n, 4)), dim3(kBlock), 0, s, w, wt, Cout, R, S, C);
}

}  // namespace dpt
