// Device-side training metrics (gfx950).
//
// The reference syncs the host twice per step to accumulate metrics
// (`loss.item()` and `preds.eq(targets).sum().item()`, reference train_ddp.py:217-220;
// SURVEY.md §2.5 K17).  This kernel folds argmax + compare + count + loss*batch into one
// launch that accumulates into a device float64 triple {loss_sum, correct, total}; the host
// reads it only at print_freq boundaries and at epoch end.
//
// One wave64 per logits row: lanes stride the class dimension, then a 6-step xor-shuffle
// reduction picks (max, lowest index) with NaN ranked above every number (torch.max
// propagates NaN).  Lane 0 of each wave adds its hit into LDS; one float64 atomic per block.
#include "common.h"
#include "kernels.h"

namespace dpt {

template <typename Load>
__global__ __launch_bounds__(kBlock) void metrics_kernel(const void* __restrict__ logits, int64_t rows,
                                                         int64_t cols, int64_t ld,
                                                         const int64_t* __restrict__ targets,
                                                         const float* __restrict__ loss,
                                                         double* __restrict__ acc, Load load) {
  __shared__ int hits[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * (kBlock / 64) + wave;
  int hit = 0;
  if (row < rows) {
    float best = -__builtin_inff();
    int64_t bidx = cols;  // sentinel: larger than any index
    bool best_nan = false;
    for (int64_t c = lane; c < cols; c += 64) {
      float v = load(logits, row * ld + c);
      bool vn = v != v;
      bool better = best_nan ? false : (vn || v > best || bidx == cols);
      if (better) { best = v; bidx = c; best_nan = vn; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      float ob = __shfl_xor(best, off, 64);
      int64_t oi = __shfl_xor(bidx, off, 64);
      bool on = __shfl_xor((int)best_nan, off, 64) != 0;
      bool take;
      if (oi == cols) take = false;
      else if (bidx == cols) take = true;
      else if (best_nan != on) take = on;
      else if (on || ob == best) take = oi < bidx;
      else take = ob > best;
      if (take) { best = ob; bidx = oi; best_nan = on; }
    }
    hit = (bidx == targets[row]) ? 1 : 0;
  }
  if (lane == 0) hits[wave] = hit;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += hits[w];
    if (s) atomicAdd(&acc[1], (double)s);
    if (blockIdx.x == 0) {
      if (loss) atomicAdd(&acc[0], (double)loss[0] * (double)rows);
      atomicAdd(&acc[2], (double)rows);
    }
  }
}

struct LoadF32 {
  __device__ float operator()(const void* p, int64_t i) const { return static_cast<const float*>(p)[i]; }
};
struct LoadBF16 {
  __device__ float operator()(const void* p, int64_t i) const {
    return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  }
};
struct LoadF16 {
  __device__ float operator()(const void* p, int64_t i) const {
    return f16_to_f32(static_cast<const uint16_t*>(p)[i]);
  }
};

void launch_metrics(const void* logits, int dtype, int64_t rows, int64_t cols, int64_t ld,
                    const int64_t* targets, const float* loss, double* acc, hipStream_t s) {
  if (rows == 0) return;
  dim3 grid((unsigned)((rows + (kBlock / 64) - 1) / (kBlock / 64))), block(kBlock);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(metrics_kernel<LoadF32>, grid, block, 0, s, logits, rows, cols, ld, targets, loss, acc, LoadF32{}); break;
    case 1: hipLaunchKernelGGL(metrics_kernel<LoadBF16>, grid, block, 0, s, logits, rows, cols, ld, targets, loss, acc, LoadBF16{}); break;
    default: hipLaunchKernelGGL(metrics_kernel<LoadF16>, grid, block, 0, s, logits, rows, cols, ld, targets, loss, acc, LoadF16{}); break;
  }
}

}  // namespace dpt
