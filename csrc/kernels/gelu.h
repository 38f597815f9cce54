// Exact (erf) GELU and its derivative for the epilogues that apply them (vit_kernels.hip's GELU
// passes, conv_kernels.hip's DGELU backward-data epilogue): one definition, so the fused and the
// stand-alone paths compute the same values.
#pragma once

#include <hip/hip_runtime.h>

namespace dpt {

// erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output rounding of
// 3.9e-3 relative): branch-free, one exp + one reciprocal, and the exp(-z^2/2) it computes is
// exactly the Gaussian density the backward needs.  ocml's erff costs ~50 instructions with
// data-dependent branches; this is ~15, which moves the GELU passes back to the HBM bound.
__device__ __forceinline__ float erf_and_gauss(float z, float& g) {  // erf(z/sqrt2), exp(-z^2/2)
  const float x = fabsf(z) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * x);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f +
                                                                                   t * 1.061405429f))));
  g = __expf(-x * x);
  return copysignf(1.f - p * g, z);
}
__device__ __forceinline__ float gelu_f(float z) {
  float g;
  return 0.5f * z * (1.f + erf_and_gauss(z, g));
}
__device__ __forceinline__ float gelu_grad(float z) {
  float g;
  const float cdf = 0.5f * (1.f + erf_and_gauss(z, g));
  return cdf + z * g * 0.39894228040143268f;
}

}  // namespace dpt
