// Fused, loss-scale-aware optimizer kernels over flat fp32 arenas (gfx950).
//
// Replaces, for one flat arena, what the reference's step runs as separate passes
// (SURVEY.md §2.5 K13-K16): the AMP unscale (`_amp_foreach_non_finite_check_and_unscale_`),
// the host sync on found_inf (torch/amp/grad_scaler.py:356), four foreach SGD passes
// (torch/optim/sgd.py:424-476), `_amp_update_scale_`, and the next step's zero_grad.
//
//   grad_check   : found_inf |= !isfinite(g * factor)          (read g)          4 B/param
//   sgd_step     : d = g*factor + wd*p; buf = mu*buf + (1-damp)*d | d (first);
//                  p -= lr * (nesterov ? d + mu*buf : buf); g = 0
//                  (read p,g,buf; write p,buf,g)                               24 B/param
//   adam_step    : torch.optim.Adam/AdamW math, bias correction from a device step count
//                  (read p,g,m,v; write p,m,v,g)                               32 B/param
//   optim_tail   : 1 thread: GradScaler growth/backoff, step += !found_inf, found_inf = 0
//
// `factor` = host_factor / loss_scale with loss_scale read from device memory, so the
// whole sequence runs with zero host synchronisation and is hipGraph-capturable.
// When found_inf is set the update is skipped (GradScaler semantics: optimizer.step() is
// not called) but gradients are still zeroed, matching zero_grad() before the next step.
#include "common.h"
#include "kernels.h"

namespace dpt {

// 16-bit shadow of 4 updated parameters (bf16 kind 1, fp16 kind 2): one 8-byte store.
__device__ __forceinline__ void store_shadow4(uint16_t* shadow, int kind, int64_t i, float4 v) {
  auto cv = [kind](float f) -> uint32_t {
    return kind == 1 ? (uint32_t)f32_to_bf16(f) : (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);
  };
  uint2 w;
  w.x = cv(v.x) | (cv(v.y) << 16);
  w.y = cv(v.z) | (cv(v.w) << 16);
  reinterpret_cast<uint2*>(shadow)[i] = w;
}

template <int UNROLL>
__global__ __launch_bounds__(kBlock) void grad_check_kernel(const float4* __restrict__ g,
                                                            int64_t nvec, const float* scale,
                                                            float host_factor, float* found_inf) {
  const float f = grad_factor(scale, host_factor);
  int bad = 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock * UNROLL;
  for (int64_t base = (int64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec; base += stride) {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t i = base + (int64_t)u * kBlock;
      v[u] = i < nvec ? g[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float4 s = make_float4(v[u].x * f, v[u].y * f, v[u].z * f, v[u].w * f);
      bad |= !finite4(s);
    }
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) found_inf[0] = 1.0f;
}

template <int UNROLL, bool MOMENTUM, bool NESTEROV>
__global__ __launch_bounds__(kBlock) void sgd_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                     float4* __restrict__ buf, int64_t nvec, float lr,
                                                     float momentum, float one_m_damp, float wd,
                                                     const float* scale, float host_factor,
                                                     const float* found_inf, const float* step,
                                                     int zero_grad, uint16_t* __restrict__ shadow,
                                                     int shadow_kind) {
  const bool skip = found_inf != nullptr && found_inf[0] != 0.0f;
  const int64_t stride = (int64_t)gridDim.x * kBlock * UNROLL;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (skip) {
    if (!zero_grad) return;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec; base += stride)
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        int64_t i = base + (int64_t)u * kBlock;
        if (i < nvec) g[i] = z;
      }
    return;
  }
  const float f = grad_factor(scale, host_factor);
  const bool first = MOMENTUM && (step == nullptr || step[0] == 0.0f);
  for (int64_t base = (int64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec; base += stride) {
    float4 pv[UNROLL], gv[UNROLL], bv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t i = base + (int64_t)u * kBlock;
      if (i < nvec) {
        pv[u] = p[i];
        gv[u] = g[i];
        if (MOMENTUM && !first) bv[u] = buf[i];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t i = base + (int64_t)u * kBlock;
      if (i >= nvec) continue;
      float* pp = reinterpret_cast<float*>(&pv[u]);
      float* gg = reinterpret_cast<float*>(&gv[u]);
      float* bb = reinterpret_cast<float*>(&bv[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d = gg[k] * f + wd * pp[k];
        if (MOMENTUM) {
          bb[k] = first ? d : momentum * bb[k] + one_m_damp * d;
          d = NESTEROV ? d + momentum * bb[k] : bb[k];
        }
        pp[k] = pp[k] - lr * d;
      }
      p[i] = pv[u];
      if (shadow) store_shadow4(shadow, shadow_kind, i, pv[u]);
      if (MOMENTUM) buf[i] = bv[u];
      if (zero_grad) g[i] = z;
    }
  }
}

// Scalar coefficients are formed in double (on the host, or in-kernel for the step-dependent
// bias corrections) and rounded once, as torch does with its Python-float hyper-parameters:
// 1 - 0.999f in fp32 is 1.3e-5 away from fp32(0.001).
struct AdamCoef {
  float lr, beta1, beta2, one_m_beta1, one_m_beta2, eps, wd, decay;
  double beta1_d, beta2_d;
};

template <int UNROLL, bool ADAMW>
__global__ __launch_bounds__(kBlock) void adam_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                      float4* __restrict__ m, float4* __restrict__ v,
                                                      int64_t nvec, AdamCoef co, const float* scale,
                                                      float host_factor, const float* found_inf,
                                                      const float* step, int zero_grad,
                                                      uint16_t* __restrict__ shadow, int shadow_kind) {
  const bool skip = found_inf != nullptr && found_inf[0] != 0.0f;
  const int64_t stride = (int64_t)gridDim.x * kBlock * UNROLL;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (skip) {
    if (!zero_grad) return;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec; base += stride)
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        int64_t i = base + (int64_t)u * kBlock;
        if (i < nvec) g[i] = z;
      }
    return;
  }
  const float f = grad_factor(scale, host_factor);
  const double t = (double)(step ? step[0] : 0.0f) + 1.0;
  const float bc2_sqrt = (float)sqrt(1.0 - pow(co.beta2_d, t));
  const float step_size = (float)((double)co.lr / (1.0 - pow(co.beta1_d, t)));
  const float beta2 = co.beta2, one_m_beta1 = co.one_m_beta1, one_m_beta2 = co.one_m_beta2;
  const float eps = co.eps, wd = co.wd, decay = co.decay;
  for (int64_t base = (int64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec; base += stride) {
    float4 pv[UNROLL], gv[UNROLL], mv[UNROLL], vv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t i = base + (int64_t)u * kBlock;
      if (i < nvec) { pv[u] = p[i]; gv[u] = g[i]; mv[u] = m[i]; vv[u] = v[i]; }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t i = base + (int64_t)u * kBlock;
      if (i >= nvec) continue;
      float* pp = reinterpret_cast<float*>(&pv[u]);
      float* gg = reinterpret_cast<float*>(&gv[u]);
      float* mm = reinterpret_cast<float*>(&mv[u]);
      float* vq = reinterpret_cast<float*>(&vv[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gr = gg[k] * f;
        if (ADAMW) pp[k] *= decay;
        else gr += wd * pp[k];
        mm[k] = mm[k] + one_m_beta1 * (gr - mm[k]);          // m.lerp_(g, 1-beta1)
        vq[k] = beta2 * vq[k] + one_m_beta2 * gr * gr;
        float denom = sqrtf(vq[k]) / bc2_sqrt + eps;
        pp[k] = pp[k] - step_size * (mm[k] / denom);
      }
      p[i] = pv[u]; m[i] = mv[u]; v[i] = vv[u];
      if (shadow) store_shadow4(shadow, shadow_kind, i, pv[u]);
      if (zero_grad) g[i] = z;
    }
  }
}

__global__ void optim_tail_kernel(float* scale, int* growth_tracker, float* found_inf, float* step,
                                  float growth_factor, float backoff_factor, int growth_interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool inf = found_inf[0] != 0.0f;
  if (scale != nullptr) {
    if (inf) {
      scale[0] *= backoff_factor;
      growth_tracker[0] = 0;
    } else {
      int successful = growth_tracker[0] + 1;
      if (successful == growth_interval) {
        float ns = scale[0] * growth_factor;
        if (__builtin_isfinite(ns)) scale[0] = ns;
        growth_tracker[0] = 0;
      } else {
        growth_tracker[0] = successful;
      }
    }
  }
  if (step != nullptr && !inf) step[0] += 1.0f;
  found_inf[0] = 0.0f;
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
constexpr int kUnroll = 2;

void launch_grad_check(const float* g, int64_t n, const float* scale, float host_factor,
                       float* found_inf, hipStream_t s) {
  int64_t nvec = n / 4;
  if (nvec == 0) return;
  hipLaunchKernelGGL((grad_check_kernel<4>), dim3(grid_for(nvec, 4)), dim3(kBlock), 0, s,
                     reinterpret_cast<const float4*>(g), nvec, scale, host_factor, found_inf);
}

void launch_sgd(float* p, float* g, float* buf, int64_t n, float lr, float momentum,
                float dampening, float wd, bool nesterov, const float* scale, float host_factor,
                const float* found_inf, const float* step, bool zero_grad, uint16_t* shadow,
                int shadow_kind, hipStream_t s) {
  const float one_m_damp = (float)(1.0 - (double)dampening);  // formed in double, as torch does
  int64_t nvec = n / 4;
  if (nvec == 0) return;
  dim3 grid(grid_for(nvec, kUnroll)), block(kBlock);
  auto P = reinterpret_cast<float4*>(p);
  auto G = reinterpret_cast<float4*>(g);
  auto B = reinterpret_cast<float4*>(buf);
  if (momentum == 0.0f) {
    hipLaunchKernelGGL((sgd_kernel<kUnroll, false, false>), grid, block, 0, s, P, G, B, nvec, lr,
                       momentum, one_m_damp, wd, scale, host_factor, found_inf, step, (int)zero_grad, shadow, shadow_kind);
  } else if (nesterov) {
    hipLaunchKernelGGL((sgd_kernel<kUnroll, true, true>), grid, block, 0, s, P, G, B, nvec, lr,
                       momentum, one_m_damp, wd, scale, host_factor, found_inf, step, (int)zero_grad, shadow, shadow_kind);
  } else {
    hipLaunchKernelGGL((sgd_kernel<kUnroll, true, false>), grid, block, 0, s, P, G, B, nvec, lr,
                       momentum, one_m_damp, wd, scale, host_factor, found_inf, step, (int)zero_grad, shadow, shadow_kind);
  }
}

void launch_adam(float* p, float* g, float* m, float* v, int64_t n, double lr, double beta1,
                 double beta2, double eps, double wd, bool adamw, const float* scale, float host_factor,
                 const float* found_inf, const float* step, bool zero_grad, uint16_t* shadow,
                 int shadow_kind, hipStream_t s) {
  int64_t nvec = n / 4;
  if (nvec == 0) return;
  dim3 grid(grid_for(nvec, kUnroll)), block(kBlock);
  auto P = reinterpret_cast<float4*>(p);
  auto G = reinterpret_cast<float4*>(g);
  auto M = reinterpret_cast<float4*>(m);
  auto V = reinterpret_cast<float4*>(v);
  AdamCoef co;
  co.lr = (float)lr;
  co.beta1 = (float)beta1;
  co.beta2 = (float)beta2;
  co.one_m_beta1 = (float)(1.0 - beta1);
  co.one_m_beta2 = (float)(1.0 - beta2);
  co.eps = (float)eps;
  co.wd = (float)wd;
  co.decay = adamw ? (float)(1.0 - lr * wd) : 1.0f;
  co.beta1_d = beta1;
  co.beta2_d = beta2;
  if (adamw)
    hipLaunchKernelGGL((adam_kernel<kUnroll, true>), grid, block, 0, s, P, G, M, V, nvec, co, scale,
                       host_factor, found_inf, step, (int)zero_grad, shadow, shadow_kind);
  else
    hipLaunchKernelGGL((adam_kernel<kUnroll, false>), grid, block, 0, s, P, G, M, V, nvec, co, scale,
                       host_factor, found_inf, step, (int)zero_grad, shadow, shadow_kind);
}

void launch_optim_tail(float* scale, int* growth_tracker, float* found_inf, float* step,
                       float growth_factor, float backoff_factor, int growth_interval,
                       hipStream_t s) {
  hipLaunchKernelGGL(optim_tail_kernel, dim3(1), dim3(64), 0, s, scale, growth_tracker, found_inf,
                     step, growth_factor, backoff_factor, growth_interval);
}

}  // namespace dpt
