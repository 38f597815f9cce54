// gfx950 matrix-core helpers shared by the MFMA kernels (conv_kernels.hip, attn_kernels.hip).
//
// v_mfma_f32_32x32x16_bf16 operand maps (cdna_hip_programming.md §3): lane l (r = l&31,
// h = l>>5) holds A[row r][k = 8h..8h+7] and B[k = 8h..8h+7][col r]; the accumulator holds
// column l&31, rows (e&3) + 8*(e>>2) + 4h for e = 0..15.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpt {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---- LDS images with rows of RB bytes (RB = 128: 64 bf16, RB = 256: 128 bf16, RB = 512) -------
// 16-byte chunk ch of row `row` is stored at slot wg_slot(row, ch).  The XOR makes both read
// kinds conflict-free: ds_read_b128 of one chunk from 16 consecutive rows (A/B operands with
// rows = M/N) and ds_read_b64_tr_b16 of 4 consecutive rows x 32 columns per 32-lane half
// (operands with rows = K).  The XOR is an involution: a lane-linear glds fill loads, for the
// slot it writes, chunk wg_slot(row, slot).
template <int RB>
__device__ __forceinline__ int wg_slot(int row, int ch) {
  // RB = 512 (256 bf16): the same low-4-bit XOR - each row starts on bank 0, and the 4 rows one
  // transposing read touches land on 4 distinct 64-byte bank groups
  if (RB == 256 || RB == 512) return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  return ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}

// Row-operand fragment: row `row`, k-chunk `ch` (8 elements) -> one ds_read_b128.
template <int RB>
__device__ __forceinline__ bf16x8_t row_frag(const unsigned char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8_t*>(img + row * RB + wg_slot<RB>(row, ch) * 16);
}

// K-major fragment (rows of the image = k): 8 k-rows of this lane's column (col0 + lane&31)
// from two ds_read_b64_tr_b16.  PERM = false: rows krow0 + 8h + 0..7 (natural k order);
// PERM = true: rows krow0 + 4h + {0..3} and krow0 + 8 + 4h + {0..3} - the k order of an
// accumulator tile reused as the other operand (element j of half h = row 8(j>>2) + 4h + (j&3)).
template <int RB, bool PERM = false>
__device__ __forceinline__ bf16x8_t tr_frag(const unsigned char* img, int krow0, int col0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int colb = col0 + 16 * (g & 1) + 4 * pp;  // this lane's 4 columns (address role)
  const int ch = colb >> 3, sub = (colb & 7) * 2;
  const int r1 = PERM ? krow0 + 4 * (g >> 1) + q : krow0 + 8 * (g >> 1) + q;
  const int r2 = PERM ? r1 + 8 : r1 + 4;
  typedef __attribute__((address_space(3))) i16x4_t lds_v4;
  const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + r1 * RB + wg_slot<RB>(r1, ch) * 16 + sub));
  const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + r2 * RB + wg_slot<RB>(r2, ch) * 16 + sub));
  i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// Accumulator registers 8s..8s+7 as a bf16 operand fragment for k-step s (PERM k order).
__device__ __forceinline__ bf16x8_t acc_frag(const f32x16_t& x, int s) {
  bf16x8_t f;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2_t v = {x[8 * s + j], x[8 * s + j + 1]};
    const bf16x2_t h = __builtin_convertvector(v, bf16x2_t);
    f[j] = h[0];
    f[j + 1] = h[1];
  }
  return f;
}

}  // namespace dpt
