// Gradient-bucket kernels that run on the reducer's communication stream (gfx950).
//
// The reference's DDP reducer copies every gradient into its bucket pre-divided by the
// world size and copies it back after the all-reduce (SURVEY.md §2.5 K11/K13,
// reducer.hpp:279,327,499).  Here gradients already live inside the bucket (autograd
// accumulates into views of the flat arena), the 1/world_size factor moves into the
// optimizer, and the only per-bucket work after the RCCL all-reduce is:
//   * fp32 wire: nothing but the non-finite check (`grad_check`, optim_kernels.hip), which
//     runs on the comm stream behind the all-reduce and so overlaps the rest of backward;
//   * bf16 wire (--grad-dtype bf16, gradient compression): `pack_bf16` before the
//     all-reduce (8 B read + 2 B... per element: read f32, write bf16) and `unpack_bf16`
//     after it (read bf16, write f32, OR the non-finite flag in the same pass).
#include "common.h"
#include "kernels.h"

namespace dpt {

// 8 elements per lane: two float4 loads -> one 16-byte bf16x8 store.
__global__ __launch_bounds__(kBlock) void pack_bf16_kernel(const float4* __restrict__ src,
                                                           uint4* __restrict__ dst, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += stride) {
    float4 a = src[2 * i], b = src[2 * i + 1];
    uint4 o;
    o.x = (uint32_t)f32_to_bf16(a.x) | ((uint32_t)f32_to_bf16(a.y) << 16);
    o.y = (uint32_t)f32_to_bf16(a.z) | ((uint32_t)f32_to_bf16(a.w) << 16);
    o.z = (uint32_t)f32_to_bf16(b.x) | ((uint32_t)f32_to_bf16(b.y) << 16);
    o.w = (uint32_t)f32_to_bf16(b.z) | ((uint32_t)f32_to_bf16(b.w) << 16);
    dst[i] = o;
  }
}

__global__ __launch_bounds__(kBlock) void unpack_bf16_kernel(const uint4* __restrict__ src,
                                                             float4* __restrict__ dst, int64_t n8,
                                                             const float* scale, float host_factor,
                                                             float* found_inf) {
  const float f = found_inf ? grad_factor(scale, host_factor) : 1.0f;
  int bad = 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += stride) {
    uint4 w = src[i];
    float4 a = make_float4(bf16_to_f32(w.x & 0xffff), bf16_to_f32(w.x >> 16),
                           bf16_to_f32(w.y & 0xffff), bf16_to_f32(w.y >> 16));
    float4 b = make_float4(bf16_to_f32(w.z & 0xffff), bf16_to_f32(w.z >> 16),
                           bf16_to_f32(w.w & 0xffff), bf16_to_f32(w.w >> 16));
    if (found_inf) {
      bad |= !finite4(make_float4(a.x * f, a.y * f, a.z * f, a.w * f));
      bad |= !finite4(make_float4(b.x * f, b.y * f, b.z * f, b.w * f));
    }
    dst[2 * i] = a;
    dst[2 * i + 1] = b;
  }
  if (found_inf && __syncthreads_or(bad) && threadIdx.x == 0) found_inf[0] = 1.0f;
}

void launch_pack_bf16(const float* src, uint16_t* dst, int64_t n, hipStream_t s) {
  int64_t n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(pack_bf16_kernel, dim3(grid_for(n8, 1)), dim3(kBlock), 0, s,
                     reinterpret_cast<const float4*>(src), reinterpret_cast<uint4*>(dst), n8);
}

void launch_unpack_bf16(const uint16_t* src, float* dst, int64_t n, const float* scale,
                        float host_factor, float* found_inf, hipStream_t s) {
  int64_t n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(unpack_bf16_kernel, dim3(grid_for(n8, 1)), dim3(kBlock), 0, s,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<float4*>(dst), n8, scale,
                     host_factor, found_inf);
}

// Test-only: one wave busy-waits `ticks` of the constant-rate wall clock, then exits.  The
// watchdog GPU tests enqueue it on the communicator stream ahead of a collective to model a
// peer that never arrives.  Bounded twice: by the clock and by an iteration cap, so every
// wave exits even if the clock read misbehaved.
__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks, uint64_t max_iters) {
  const uint64_t t0 = wall_clock64();
  for (uint64_t it = 0; it < max_iters; ++it) {
    if (wall_clock64() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(100);
  }
}

void launch_spin(double ms, hipStream_t s) {
  int dev = 0, khz = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  const uint64_t ticks = (uint64_t)(ms * (double)khz);
  // s_sleep 100 ~ 6400 cycles >= ~2 us at any shader clock: 4x the needed count is plenty
  const uint64_t max_iters = (uint64_t)(ms * 1000.0) * 4 + 1000;
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks, max_iters);
}

}  // namespace dpt
