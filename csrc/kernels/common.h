// Shared device helpers for the gfx950 kernel library.
//
// Every hot kernel here is HBM-bound streaming over *flat* buffers (the parameter /
// gradient / optimizer-state arenas laid out by parallel/flat.py), so the recipe is the
// same everywhere (cdna_hip_programming.md Appendix B "Element-wise", Guidelines 11/13):
//   * 16 B per lane per access (float4 / 8 x bf16), wave64, 256-thread blocks;
//   * grid capped at 256 CUs x 8 blocks and grid-strided, UNROLL independent float4s in
//     flight per thread so each CU keeps enough bytes outstanding to cover HBM latency;
//   * flags/scalars (loss scale, found_inf, step) are read from device memory, never
//     synchronised to the host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpt {

constexpr int kBlock = 256;         // 4 waves of 64
constexpr int kMaxBlocks = 256 * 8; // 256 CUs x 8 resident blocks

__host__ inline int grid_for(int64_t n_vec, int unroll) {
  int64_t per_block = (int64_t)kBlock * unroll;
  int64_t g = (n_vec + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxBlocks) g = kMaxBlocks;
  return (int)g;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// Round-to-nearest-even f32 -> bf16 (NaN stays a NaN): the plain cast is the hardware
// v_cvt_pk_bf16_f32 on gfx950 - one instruction instead of the integer rounding sequence and
// its exec-masked NaN branch (MI355X_MICROARCH.md, Correctness boundaries).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  _Float16 v = __builtin_bit_cast(_Float16, h);
  return (float)v;
}

__device__ __forceinline__ bool finite4(float4 v) {
  return __builtin_isfinite(v.x) & __builtin_isfinite(v.y) &
         __builtin_isfinite(v.z) & __builtin_isfinite(v.w);
}

// Combined gradient multiplier: host_factor (e.g. 1/world_size) / loss_scale.
__device__ __forceinline__ float grad_factor(const float* scale, float host_factor) {
  return scale ? host_factor / scale[0] : host_factor;
}

}  // namespace dpt
