// Multi-tensor gradient gather into the flat bucket arena (gfx950).
//
// Autograd's AccumulateGrad either adds each parameter's gradient into an existing .grad
// (one small elementwise launch per parameter: 161 launches, ~0.8 ms of a ResNet-50 step on
// MI355X) or, when .grad is undefined, simply *steals* the freshly computed gradient tensor
// (no kernel).  The reducer lets it steal, then moves a whole bucket's gradients into the
// contiguous arena with ONE launch: blockIdx.y selects the tensor, blockIdx.x strides over its
// 16-byte vectors (scalar tail for sizes that are not a multiple of 4).  ACCUMULATE adds into
// the arena instead of overwriting it (gradient-accumulation micro-batches).  Sources may be
// fp32, or bf16/fp16 (weight gradients of the bf16 weight shadows, converted to fp32 here, in
// the same pass that moves them - autocast would have run a separate cast-back kernel).
#include "common.h"
#include "kernels.h"

namespace dpt {

__device__ __forceinline__ float half_bits_to_f32(uint16_t h, int kind) {
  return kind == 1 ? bf16_to_f32(h) : f16_to_f32(h);
}

template <bool ACCUMULATE>
__global__ __launch_bounds__(kBlock) void gather_kernel(GatherBatch batch) {
  const int t = blockIdx.y;
  if (t >= batch.count) return;
  const int kind = batch.kind[t];
  float* __restrict__ dst = batch.dst[t];
  const int64_t n = batch.numel[t];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (kind == 0) {
    const float* __restrict__ src = static_cast<const float*>(batch.src[t]);
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    const int64_t nvec = vec ? n / 4 : 0;
    for (int64_t i = tid; i < nvec; i += stride) {
      float4 v = reinterpret_cast<const float4*>(src)[i];
      if (ACCUMULATE) {
        float4 d = reinterpret_cast<float4*>(dst)[i];
        v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
      }
      reinterpret_cast<float4*>(dst)[i] = v;
    }
    for (int64_t i = nvec * 4 + tid; i < n; i += stride) {
      float v = src[i];
      dst[i] = ACCUMULATE ? dst[i] + v : v;
    }
    return;
  }
  const uint16_t* __restrict__ src = static_cast<const uint16_t*>(batch.src[t]);
  const bool vec = (reinterpret_cast<uintptr_t>(src) & 7) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  const int64_t nvec = vec ? n / 4 : 0;
  for (int64_t i = tid; i < nvec; i += stride) {
    const uint2 w = reinterpret_cast<const uint2*>(src)[i];
    float4 v = make_float4(half_bits_to_f32(w.x & 0xffff, kind), half_bits_to_f32(w.x >> 16, kind),
                           half_bits_to_f32(w.y & 0xffff, kind), half_bits_to_f32(w.y >> 16, kind));
    if (ACCUMULATE) {
      float4 d = reinterpret_cast<float4*>(dst)[i];
      v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
    }
    reinterpret_cast<float4*>(dst)[i] = v;
  }
  for (int64_t i = nvec * 4 + tid; i < n; i += stride) {
    float v = half_bits_to_f32(src[i], kind);
    dst[i] = ACCUMULATE ? dst[i] + v : v;
  }
}

void launch_gather(const GatherBatch& batch, bool accumulate, hipStream_t s) {
  if (batch.count <= 0) return;
  int64_t maxn = 0;
  for (int i = 0; i < batch.count; ++i) maxn = batch.numel[i] > maxn ? batch.numel[i] : maxn;
  // Enough x-blocks that the largest tensor gets ~4 vectors per thread; tensors are
  // independent rows of the grid, so small ones finish early and free their CUs.
  int64_t gx = (maxn / 4 + (int64_t)kBlock * 4 - 1) / ((int64_t)kBlock * 4);
  if (gx < 1) gx = 1;
  if (gx > 1024) gx = 1024;
  dim3 grid((unsigned)gx, (unsigned)batch.count), block(kBlock);
  if (accumulate) hipLaunchKernelGGL(gather_kernel<true>, grid, block, 0, s, batch);
  else hipLaunchKernelGGL(gather_kernel<false>, grid, block, 0, s, batch);
}

}  // namespace dpt
