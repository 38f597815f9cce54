// Python bindings of the native runtime: kernel launchers (tensor-checked), the RCCL
// communicator and the C++ reducer.  Kernels launch on the caller's current HIP stream.
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "kernels/kernels.h"
#include "host_comm.h"
#include "pg_comm.h"
#include "rccl_comm.h"
#include "watchdog.h"
#include "reducer.h"

namespace py = pybind11;
using at::Tensor;

namespace {

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

dpt::WireType wire_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return dpt::WireType::kF32;
    case at::kBFloat16: return dpt::WireType::kBF16;
    case at::kHalf: return dpt::WireType::kF16;
    case at::kLong: return dpt::WireType::kI64;
    default: TORCH_CHECK(false, "unsupported collective dtype ", t.scalar_type());
  }
  return dpt::WireType::kF32;
}

void check_flat_f32(const Tensor& t, const char* name, int64_t align = 4) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor (HIP kernel path)");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() % align == 0, name, " numel must be a multiple of ", align);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

const float* opt_f32(const c10::optional<Tensor>& t, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= 1, name,
              " must be a float32 GPU tensor");
  return t->data_ptr<float>();
}

void grad_check(Tensor g, c10::optional<Tensor> scale, double host_factor, Tensor found_inf) {
  check_flat_f32(g, "grad");
  check_flat_f32(found_inf, "found_inf", 1);
  c10::hip::HIPGuard guard(g.device().index());
  dpt::launch_grad_check(g.data_ptr<float>(), g.numel(), opt_f32(scale, "scale"), (float)host_factor,
                         found_inf.data_ptr<float>(), cur_stream(g));
}

// Optional 16-bit parameter shadow (bf16 / fp16, same length as the arena).
std::pair<uint16_t*, int> shadow_arg(const c10::optional<Tensor>& sh, int64_t n) {
  if (!sh.has_value() || !sh->defined()) return {nullptr, 0};
  TORCH_CHECK(sh->is_cuda() && sh->is_contiguous() && sh->numel() == n &&
                  (sh->scalar_type() == at::kBFloat16 || sh->scalar_type() == at::kHalf),
              "shadow must be a contiguous bf16/fp16 GPU tensor of the arena's size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(sh->data_ptr()) % 8 == 0, "shadow must be 8-byte aligned");
  return {reinterpret_cast<uint16_t*>(sh->data_ptr()), sh->scalar_type() == at::kBFloat16 ? 1 : 2};
}

void sgd_step(Tensor p, Tensor g, Tensor buf, double lr, double momentum, double dampening,
              double wd, bool nesterov, c10::optional<Tensor> scale, double host_factor,
              c10::optional<Tensor> found_inf, c10::optional<Tensor> step, bool zero_grad,
              c10::optional<Tensor> shadow) {
  check_flat_f32(p, "param");
  check_flat_f32(g, "grad");
  TORCH_CHECK(g.numel() == p.numel(), "grad/param size mismatch");
  if (momentum != 0.0) {
    check_flat_f32(buf, "momentum_buffer");
    TORCH_CHECK(buf.numel() == p.numel(), "momentum buffer size mismatch");
  }
  auto [sp, sk] = shadow_arg(shadow, p.numel());
  c10::hip::HIPGuard guard(p.device().index());
  dpt::launch_sgd(p.data_ptr<float>(), g.data_ptr<float>(),
                  momentum != 0.0 ? buf.data_ptr<float>() : nullptr, p.numel(), (float)lr,
                  (float)momentum, (float)dampening, (float)wd, nesterov, opt_f32(scale, "scale"),
                  (float)host_factor, opt_f32(found_inf, "found_inf"), opt_f32(step, "step"),
                  zero_grad, sp, sk, cur_stream(p));
}

void adam_step(Tensor p, Tensor g, Tensor m, Tensor v, double lr, double beta1, double beta2,
               double eps, double wd, bool adamw, c10::optional<Tensor> scale, double host_factor,
               c10::optional<Tensor> found_inf, c10::optional<Tensor> step, bool zero_grad,
               c10::optional<Tensor> shadow) {
  check_flat_f32(p, "param");
  check_flat_f32(g, "grad");
  check_flat_f32(m, "exp_avg");
  check_flat_f32(v, "exp_avg_sq");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(),
              "adam arena size mismatch");
  auto [sp, sk] = shadow_arg(shadow, p.numel());
  c10::hip::HIPGuard guard(p.device().index());
  dpt::launch_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                   p.numel(), lr, beta1, beta2, eps, wd, adamw,
                   opt_f32(scale, "scale"), (float)host_factor, opt_f32(found_inf, "found_inf"),
                   opt_f32(step, "step"), zero_grad, sp, sk, cur_stream(p));
}

void optim_tail(c10::optional<Tensor> scale, c10::optional<Tensor> growth_tracker, Tensor found_inf,
                c10::optional<Tensor> step, double growth_factor, double backoff_factor,
                int64_t growth_interval) {
  check_flat_f32(found_inf, "found_inf", 1);
  int* gt = nullptr;
  if (growth_tracker.has_value() && growth_tracker->defined()) {
    TORCH_CHECK(growth_tracker->is_cuda() && growth_tracker->scalar_type() == at::kInt,
                "growth_tracker must be an int32 GPU tensor");
    gt = growth_tracker->data_ptr<int>();
  }
  float* sc = const_cast<float*>(opt_f32(scale, "scale"));
  TORCH_CHECK(sc == nullptr || gt != nullptr, "scale needs a growth_tracker");
  c10::hip::HIPGuard guard(found_inf.device().index());
  dpt::launch_optim_tail(sc, gt, found_inf.data_ptr<float>(), const_cast<float*>(opt_f32(step, "step")),
                         (float)growth_factor, (float)backoff_factor, (int)growth_interval,
                         cur_stream(found_inf));
}

void pack_bf16(Tensor src, Tensor dst) {
  check_flat_f32(src, "src", 8);
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kBFloat16 && dst.is_contiguous() &&
                  dst.numel() == src.numel(), "dst must be a contiguous bf16 GPU tensor of src's size");
  c10::hip::HIPGuard guard(src.device().index());
  dpt::launch_pack_bf16(src.data_ptr<float>(), reinterpret_cast<uint16_t*>(dst.data_ptr()), src.numel(),
                        cur_stream(src));
}

void unpack_bf16(Tensor src, Tensor dst, c10::optional<Tensor> scale, double host_factor,
                 c10::optional<Tensor> found_inf) {
  check_flat_f32(dst, "dst", 8);
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kBFloat16 && src.is_contiguous() &&
                  dst.numel() == src.numel(), "src must be a contiguous bf16 GPU tensor of dst's size");
  c10::hip::HIPGuard guard(dst.device().index());
  dpt::launch_unpack_bf16(reinterpret_cast<const uint16_t*>(src.data_ptr()), dst.data_ptr<float>(),
                          dst.numel(), opt_f32(scale, "scale"), (float)host_factor,
                          const_cast<float*>(opt_f32(found_inf, "found_inf")), cur_stream(dst));
}

void accumulate_metrics(Tensor logits, Tensor targets, c10::optional<Tensor> loss, Tensor acc) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2, "logits must be a 2-D GPU tensor");
  TORCH_CHECK(logits.stride(1) == 1, "logits rows must be contiguous");
  TORCH_CHECK(targets.is_cuda() && targets.scalar_type() == at::kLong && targets.is_contiguous() &&
                  targets.numel() == logits.size(0), "targets must be contiguous int64 [rows]");
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kDouble && acc.numel() >= 3 && acc.is_contiguous(),
              "acc must be a float64 GPU tensor with >= 3 elements");
  int dt;
  switch (logits.scalar_type()) {
    case at::kFloat: dt = 0; break;
    case at::kBFloat16: dt = 1; break;
    case at::kHalf: dt = 2; break;
    default: TORCH_CHECK(false, "logits dtype must be f32/bf16/f16");
  }
  const float* lp = nullptr;
  Tensor lf;
  if (loss.has_value() && loss->defined()) {
    lf = loss->detach().to(at::kFloat).reshape({1});
    lp = lf.data_ptr<float>();
  }
  c10::hip::HIPGuard guard(logits.device().index());
  dpt::launch_metrics(logits.data_ptr(), dt, logits.size(0), logits.size(1), logits.stride(0),
                      targets.data_ptr<int64_t>(), lp, acc.data_ptr<double>(), cur_stream(logits));
}

void augment(Tensor data, Tensor idx, c10::optional<Tensor> offs, c10::optional<Tensor> flips, Tensor out,
             bool nhwc, int64_t pad, std::vector<double> mean, std::vector<double> std) {
  TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 4 && data.is_contiguous(),
              "data must be contiguous uint8 [N,C,H,W] on the GPU");
  const int64_t C = data.size(1), H = data.size(2), W = data.size(3), B = idx.numel();
  TORCH_CHECK(C <= 4 && (int64_t)mean.size() == C && (int64_t)std.size() == C, "mean/std must have C<=4 entries");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.is_contiguous(), "idx must be int64 GPU");
  const int32_t* op = nullptr;
  const uint8_t* fp = nullptr;
  if (offs.has_value() && offs->defined()) {
    TORCH_CHECK(offs->is_cuda() && offs->scalar_type() == at::kInt && offs->is_contiguous() && offs->numel() == 2 * B,
                "offs must be int32 [B,2]");
    op = offs->data_ptr<int32_t>();
  }
  if (flips.has_value() && flips->defined()) {
    TORCH_CHECK(flips->is_cuda() && flips->scalar_type() == at::kByte && flips->numel() == B, "flips must be uint8 [B]");
    fp = flips->data_ptr<uint8_t>();
  }
  TORCH_CHECK(out.is_cuda() && out.numel() == B * C * H * W, "out size mismatch");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out must be f32/bf16");
  if (nhwc) {
    TORCH_CHECK(out.is_contiguous(at::MemoryFormat::ChannelsLast), "out must be channels_last");
  } else {
    TORCH_CHECK(out.is_contiguous(), "out must be contiguous NCHW");
  }
  dpt::AugNorm n{};
  for (int c = 0; c < C; ++c) { n.mean[c] = (float)mean[c]; n.inv_std[c] = (float)(1.0 / std[c]); }
  c10::hip::HIPGuard guard(data.device().index());
  dpt::launch_augment(data.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(), op, fp, out.data_ptr(),
                      out.scalar_type() == at::kBFloat16, nhwc, B, (int)C, (int)H, (int)W, (int)pad, n,
                      cur_stream(data));
}

int bn_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "fused BN supports f32/bf16/f16 activations");
  }
  return 0;
}

// Activation as a row-major [M, C] view: 4-D channels_last or 2-D contiguous.
std::pair<int64_t, int64_t> bn_rows(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last");
    return {t.size(0) * t.size(2) * t.size(3), t.size(1)};
  }
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), name, " must be 4-D channels_last or 2-D contiguous");
  return {t.size(0), t.size(1)};
}

float* f32_param(const c10::optional<Tensor>& t, int64_t C, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
              name, " must be a contiguous float32 GPU tensor of C elements");
  return t->data_ptr<float>();
}

// ---- channels_last bf16 / fp16 implicit-GEMM convolutions --------------------------------
void check_cl_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf) && t.dim() == 4, name,
              " must be a 4-d bf16/fp16 GPU tensor");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
bool is_f16(const Tensor& t) { return t.scalar_type() == at::kHalf; }

// split-K scratch for a conv with a small tile grid (undefined when it runs unsplit)
Tensor splitk_ws(const Tensor& like, int64_t M, int Cout, int64_t K) {
  const int splits = dpt::conv_fwd_splits(M, Cout, K, nullptr, cur_stream(like));
  if (splits <= 1) return Tensor();
  return at::empty({(int64_t)splits * M * Cout}, like.options().dtype(at::kFloat));
}
// columns of a conv's BN partials: one per 128-row tile, or per 16-row slab when split-K runs
int64_t partial_cols(const Tensor& ws, int64_t M) {
  return ws.defined() ? dpt::conv_split_cols(M) : dpt::conv_m_tiles(M);
}
void same_16(const Tensor& a, const Tensor& b, const char* op) {
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), op, ": operands must share one 16-bit dtype (bf16 or fp16)");
}

// A backward-weight whose split-K reduce has not run yet (conv_wgrad_deferred): it keeps the
// partials alive until a backward-data launch takes the reduce into its grid's tail
// (dpt::AttachWgradReduce) or conv_reduce_flush launches it on its own.
struct PendingReduce {
  Tensor part, dw;
  dpt::WgradReduce r{};
  bool done() const { return r.consumed; }
};
using PendingReducePtr = std::shared_ptr<PendingReduce>;

// Scoped attach of an optional pending reduce to the conv launches of one binding call.
struct MaybeAttach {
  std::unique_ptr<dpt::AttachWgradReduce> g;
  MaybeAttach(const PendingReducePtr& p, hipStream_t s) {
    if (p && !p->r.consumed) g = std::make_unique<dpt::AttachWgradReduce>(&p->r, s);
  }
};

// Returns {y, psum, psq} (psum/psq empty unless want_stats): y = conv2d(x, w, stride, pad).
// out_h/out_w > 0: explicit output size, no larger than the symmetric-padding one (the extra
// padding rows/columns at the bottom/right are dropped: asymmetric padding).
std::vector<Tensor> conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, bool want_stats, int64_t out_h,
                             int64_t out_w) {
  check_cl_bf16(x, "x");
  check_cl_bf16(w, "w");
  same_16(x, w, "conv_fwd");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Cout = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_fwd: channel mismatch");
  TORCH_CHECK(dpt::conv_supported(C, Cout) || dpt::conv_supported_narrow(C, Cout, S),
              "conv_fwd: needs C % 64 == 0 (or C in {16, 32} with S % (64/C) == 0) and Cout % 64 == 0");
  TORCH_CHECK(stride >= 1 && pad >= 0, "conv_fwd: bad stride/pad");
  const int Hs = (H + 2 * pad - R) / stride + 1, Ws = (W + 2 * pad - S) / stride + 1;
  const int Ho = out_h > 0 ? out_h : Hs, Wo = out_w > 0 ? out_w : Ws;
  TORCH_CHECK(Ho > 0 && Wo > 0 && Ho <= Hs && Wo <= Ws, "conv_fwd: bad output size");
  auto y = at::empty({N, Cout, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  Tensor ws = splitk_ws(x, (int64_t)N * Ho * Wo, Cout, (int64_t)R * S * C);
  Tensor ps, pq;
  if (want_stats) {
    const int64_t mt = partial_cols(ws, (int64_t)N * Ho * Wo);
    ps = at::empty({Cout, mt}, x.options().dtype(at::kFloat));
    pq = at::empty({Cout, mt}, x.options().dtype(at::kFloat));
  }
  dpt::launch_conv_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()), N, H, W, C, Cout, R, S, (int)stride, (int)pad,
                       want_stats ? ps.data_ptr<float>() : nullptr, want_stats ? pq.data_ptr<float>() : nullptr,
                       cur_stream(x), Ho, Wo, is_f16(x), ws.defined() ? ws.data_ptr<float>() : nullptr);
  return {y, ps, pq};
}

// dx = conv2d backward-data for a stride-1 conv (flip/transpose folded into the kernel's
// weight addressing).
Tensor conv_dgrad(Tensor dy, Tensor w, int64_t pad) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(w, "w");
  same_16(dy, w, "conv_dgrad");
  const int Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(dy.size(1) == Cout, "conv_dgrad: channel mismatch");
  TORCH_CHECK(dpt::conv_supported(Cout, C), "conv_dgrad: needs C % 64 == 0 and Cout % 64 == 0");
  TORCH_CHECK(R - 1 - pad >= 0 && S == R, "conv_dgrad: needs square kernel and pad <= R-1");
  const int N = dy.size(0), Ho = dy.size(2), Wo = dy.size(3);
  // stride 1: H = Ho + R - 1 - 2*pad
  auto dx = at::empty({N, C, Ho + R - 1 - 2 * (int)pad, Wo + S - 1 - 2 * (int)pad},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(dy.device().index());
  dpt::launch_conv_dgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                         reinterpret_cast<uint16_t*>(dx.data_ptr()), N, Ho, Wo, Cout, C, R, S, (int)pad, cur_stream(dy),
                         is_f16(dy));
  return dx;
}

// Optional 1-bit ReLU mask output of a block tail's forward apply: uint8 [M, C/8] on x's device.
static uint8_t* relu_mask_ptr(const c10::optional<Tensor>& m, int64_t M, int64_t C, const Tensor& x, const char* who) {
  if (!m.has_value() || !m->defined()) return nullptr;
  TORCH_CHECK(m->device() == x.device() && m->scalar_type() == at::kByte && m->is_contiguous() && m->dim() == 2 &&
                  m->size(0) == M && m->size(1) == C / 8,
              who, ": mask_out must be a contiguous uint8 [M, C/8] tensor on x's device");
  return m->data_ptr<uint8_t>();
}

// Stride-1 backward-data whose epilogue also sums the backward statistics of the BatchNorm+ReLU
// that produced the conv's input (bn_x: that BN's input, same shape as dx; coef = [a | b]).
// Returns {dx, p1, p2} with p1/p2 [C, m_tiles] for bn_bwd_partials.
// With bn_y / bn_res (block-tail BN+add+ReLU whose output also fed the identity path): dx is
// the tail's whole masked gradient (dx + bn_res) * (bn_y > 0) and p1/p2 are summed from it.
std::vector<Tensor> conv_dgrad_bnstats(Tensor dy, Tensor w, int64_t pad, Tensor bn_x, Tensor bn_mean,
                                       c10::optional<Tensor> bn_coef,
                                       c10::optional<Tensor> bn_y, c10::optional<Tensor> bn_res,
                                       c10::optional<Tensor> w_flipped, c10::optional<Tensor> bn_x2,
                                       c10::optional<Tensor> bn_mean2, PendingReducePtr wgrad_reduce,
                                       c10::optional<Tensor> bn_mask) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(w, "w");
  check_cl_bf16(bn_x, "bn_x");
  same_16(dy, w, "conv_dgrad_bnstats");
  same_16(dy, bn_x, "conv_dgrad_bnstats");
  const int Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(dy.size(1) == Cout && dpt::conv_supported(Cout, C), "conv_dgrad_bnstats: bad shapes");
  TORCH_CHECK(R - 1 - pad >= 0 && S == R, "conv_dgrad_bnstats: needs square kernel and pad <= R-1");
  const int N = dy.size(0), Ho = dy.size(2), Wo = dy.size(3);
  const int H = Ho + R - 1 - 2 * (int)pad, W = Wo + S - 1 - 2 * (int)pad;
  TORCH_CHECK(bn_x.size(0) == N && bn_x.size(1) == C && bn_x.size(2) == H && bn_x.size(3) == W,
              "conv_dgrad_bnstats: bn_x must match the conv input");
  const bool res = bn_y.has_value() && bn_y->defined();
  TORCH_CHECK(res == (bn_res.has_value() && bn_res->defined()), "conv_dgrad_bnstats: bn_y and bn_res go together");
  TORCH_CHECK(res || (bn_coef.has_value() && bn_coef->defined()), "conv_dgrad_bnstats: bn_coef needed without bn_y");
  if (res) {
    check_cl_bf16(*bn_y, "bn_y");
    check_cl_bf16(*bn_res, "bn_res");
    same_16(dy, *bn_y, "conv_dgrad_bnstats");
    same_16(dy, *bn_res, "conv_dgrad_bnstats");
    TORCH_CHECK(bn_y->sizes() == bn_x.sizes() && bn_res->sizes() == bn_x.sizes(),
                "conv_dgrad_bnstats: bn_y / bn_res must match bn_x");
  }
  const bool pre = w_flipped.has_value() && w_flipped->defined();
  if (pre) {
    check_cl_bf16(*w_flipped, "w_flipped");
    same_16(dy, *w_flipped, "conv_dgrad_bnstats");
    TORCH_CHECK(w_flipped->size(0) == C && w_flipped->size(1) == Cout && w_flipped->size(2) == R &&
                    w_flipped->size(3) == S, "conv_dgrad_bnstats: w_flipped must be [C, Cout, R, S]");
  }
  auto wt = pre ? *w_flipped : at::empty({C, Cout, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(dy.device().index());
  Tensor ws = splitk_ws(dy, (int64_t)N * H * W, C, (int64_t)R * S * Cout);
  const int64_t mt = partial_cols(ws, (int64_t)N * H * W);
  auto p1 = at::empty({C, mt}, dy.options().dtype(at::kFloat));
  auto p2 = at::empty({C, mt}, dy.options().dtype(at::kFloat));
  const bool two = bn_x2.has_value() && bn_x2->defined();
  if (two) {
    TORCH_CHECK(res, "conv_dgrad_bnstats: bn_x2 needs bn_y / bn_res");
    check_cl_bf16(*bn_x2, "bn_x2");
    same_16(dy, *bn_x2, "conv_dgrad_bnstats");
    TORCH_CHECK(bn_x2->sizes() == bn_x.sizes(), "conv_dgrad_bnstats: bn_x2 must match bn_x");
  }
  auto p3 = at::empty({two ? C : 0, two ? mt : 0}, dy.options().dtype(at::kFloat));
  // the tail's 1-bit ReLU mask (bn_fwd_train mask_out): read instead of bn_y
  const uint8_t* mp = nullptr;
  if (bn_mask.has_value() && bn_mask->defined()) {
    TORCH_CHECK(res, "conv_dgrad_bnstats: bn_mask needs bn_y / bn_res");
    mp = relu_mask_ptr(bn_mask, (int64_t)N * H * W, C, dy, "conv_dgrad_bnstats");
  }
  auto st = cur_stream(dy);
  if (!pre)
    dpt::launch_conv_wt_flip(reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(wt.data_ptr()),
                             Cout, R, S, C, st);
  MaybeAttach att(wgrad_reduce, st);
  dpt::launch_conv_dgrad_bnstats(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                 reinterpret_cast<const uint16_t*>(wt.data_ptr()), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                 N, Ho, Wo, Cout, C, R, S, (int)pad, reinterpret_cast<const uint16_t*>(bn_x.data_ptr()),
                                 f32_param(bn_mean, C, "bn_mean"), f32_param(bn_coef, 2 * C, "bn_coef"),
                                 p1.data_ptr<float>(), p2.data_ptr<float>(), st,
                                 res ? reinterpret_cast<const uint16_t*>(bn_y->data_ptr()) : nullptr,
                                 res ? reinterpret_cast<const uint16_t*>(bn_res->data_ptr()) : nullptr,
                                 two ? reinterpret_cast<const uint16_t*>(bn_x2->data_ptr()) : nullptr,
                                 two ? f32_param(bn_mean2, C, "bn_mean2") : nullptr,
                                 two ? p3.data_ptr<float>() : nullptr, is_f16(dy),
                                 ws.defined() ? ws.data_ptr<float>() : nullptr, mp);
  return {dx, p1, p2, p3};
}

// Stride-2 backward-data: dx [N, C, H, W] (channels_last) of y = conv2d(x, w, stride 2, pad).
std::vector<Tensor> conv_dgrad_s2(Tensor dy, Tensor w, int64_t pad, int64_t H, int64_t W, c10::optional<Tensor> bn_x,
                                  c10::optional<Tensor> bn_mean, c10::optional<Tensor> bn_coef,
                                  PendingReducePtr wgrad_reduce) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(w, "w");
  same_16(dy, w, "conv_dgrad_s2");
  const int Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(dy.size(1) == Cout && dpt::conv_supported(Cout, C), "conv_dgrad_s2: needs C, Cout % 64 == 0");
  const int N = dy.size(0), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(Ho == (H + 2 * pad - R) / 2 + 1 && Wo == (W + 2 * pad - S) / 2 + 1, "conv_dgrad_s2: geometry mismatch");
  TORCH_CHECK((int64_t)N * H * W < (int64_t(1) << 31), "conv_dgrad_s2: too many pixels");
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool bnb = bn_x.has_value() && bn_x->defined();
  c10::hip::HIPGuard guard(dy.device().index());
  const dpt::ConvS2Plan plan = dpt::conv_dgrad_s2_plan(N, (int)H, (int)W, C, Cout, R, S, (int)pad, cur_stream(dy));
  Tensor ws;
  if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, dy.options().dtype(at::kFloat));
  Tensor p1, p2;
  if (bnb) {
    check_cl_bf16(*bn_x, "bn_x");
    same_16(dy, *bn_x, "conv_dgrad_s2");
    TORCH_CHECK(bn_x->sizes() == dx.sizes(), "conv_dgrad_s2: bn_x must match the conv input");
    p1 = at::empty({C, plan.chunks}, dy.options().dtype(at::kFloat));
    p2 = at::empty({C, plan.chunks}, dy.options().dtype(at::kFloat));
  }
  MaybeAttach att(wgrad_reduce, cur_stream(dy));
  dpt::launch_conv_dgrad_s2(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                            reinterpret_cast<uint16_t*>(dx.data_ptr()), N, Ho, Wo, Cout, C, R, S, (int)pad, (int)H, (int)W,
                            cur_stream(dy), bnb ? reinterpret_cast<const uint16_t*>(bn_x->data_ptr()) : nullptr,
                            bnb ? f32_param(bn_mean, C, "bn_mean") : nullptr,
                            bnb ? f32_param(bn_coef, 2 * C, "bn_coef") : nullptr,
                            bnb ? p1.data_ptr<float>() : nullptr, bnb ? p2.data_ptr<float>() : nullptr, is_f16(dy),
                            ws.defined() ? ws.data_ptr<float>() : nullptr);
  if (!bnb) return {dx};
  return {dx, p1, p2};
}

// Flip/transpose many KRSC weights [Cout, C, R, S] (channels_last) into [C, Cout, R, S]
// (channels_last, taps flipped) in one launch.
std::vector<Tensor> conv_wt_flip_multi(std::vector<Tensor> ws) {
  std::vector<Tensor> out;
  out.reserve(ws.size());
  if (ws.empty()) return out;
  c10::hip::HIPGuard guard(ws[0].device().index());
  auto st = cur_stream(ws[0]);
  dpt::WtFlipBatch b;
  b.count = 0;
  for (size_t i = 0; i < ws.size(); ++i) {
    const Tensor& w = ws[i];
    check_cl_bf16(w, "w");
    const int Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
    TORCH_CHECK(Cout % 8 == 0 && (int64_t)Cout * C * R * S < (int64_t(1) << 31), "conv_wt_flip_multi: bad weight");
    auto wt = at::empty({C, Cout, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
    out.push_back(wt);
    const int k = b.count++;
    b.w[k] = reinterpret_cast<const uint16_t*>(w.data_ptr());
    b.wt[k] = reinterpret_cast<uint16_t*>(wt.data_ptr());
    b.Cout[k] = Cout; b.R[k] = R; b.S[k] = S; b.C[k] = C;
    if (b.count == dpt::kWtFlipMax || i + 1 == ws.size()) {
      dpt::launch_conv_wt_flip_multi(b, st);
      b.count = 0;
    }
  }
  return out;
}

// Stride-1 backward-data through an already flipped/transposed weight (conv_wt_flip_multi).
Tensor conv_dgrad_preflipped(Tensor dy, Tensor wt, int64_t pad, PendingReducePtr wgrad_reduce) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(wt, "w_flipped");
  same_16(dy, wt, "conv_dgrad_preflipped");
  const int C = wt.size(0), Cout = wt.size(1), R = wt.size(2), S = wt.size(3);
  TORCH_CHECK(dy.size(1) == Cout && dpt::conv_supported(Cout, C), "conv_dgrad_preflipped: bad shapes");
  TORCH_CHECK(R - 1 - pad >= 0 && S == R, "conv_dgrad_preflipped: needs square kernel and pad <= R-1");
  const int N = dy.size(0), Ho = dy.size(2), Wo = dy.size(3);
  auto dx = at::empty({N, C, Ho + R - 1 - 2 * (int)pad, Wo + S - 1 - 2 * (int)pad},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(dy.device().index());
  Tensor ws = splitk_ws(dy, dx.size(0) * dx.size(2) * dx.size(3), C, (int64_t)R * S * Cout);
  MaybeAttach att(wgrad_reduce, cur_stream(dy));
  dpt::launch_conv_fwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(wt.data_ptr()),
                       reinterpret_cast<uint16_t*>(dx.data_ptr()), N, Ho, Wo, Cout, C, R, S, 1, (int)(R - 1 - pad),
                       nullptr, nullptr, cur_stream(dy), 0, 0, is_f16(dy), ws.defined() ? ws.data_ptr<float>() : nullptr);
  return dx;
}

// Same through an explicitly flipped/transposed weight copy (returned too): the reference
// path the tests compare the folded addressing against.
std::vector<Tensor> conv_dgrad_flip(Tensor dy, Tensor w, int64_t pad, PendingReducePtr wgrad_reduce) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(w, "w");
  same_16(dy, w, "conv_dgrad_flip");
  const int Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(dy.size(1) == Cout, "conv_dgrad: channel mismatch");
  TORCH_CHECK(dpt::conv_supported(Cout, C), "conv_dgrad: needs C % 64 == 0 and Cout % 64 == 0");
  TORCH_CHECK(R - 1 - pad >= 0 && S == R, "conv_dgrad: needs square kernel and pad <= R-1");
  auto wt = at::empty({C, Cout, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(dy.device().index());
  auto st = cur_stream(dy);
  dpt::launch_conv_wt_flip(reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(wt.data_ptr()),
                           Cout, R, S, C, st);
  const int N = dy.size(0), Ho = dy.size(2), Wo = dy.size(3);
  auto dx = at::empty({N, C, Ho + R - 1 - 2 * (int)pad, Wo + S - 1 - 2 * (int)pad},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor ws = splitk_ws(dy, dx.size(0) * dx.size(2) * dx.size(3), C, (int64_t)R * S * Cout);
  MaybeAttach att(wgrad_reduce, st);
  dpt::launch_conv_fwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(wt.data_ptr()),
                       reinterpret_cast<uint16_t*>(dx.data_ptr()), N, Ho, Wo, Cout, C, R, S, 1, (int)(R - 1 - pad),
                       nullptr, nullptr, st, 0, 0, is_f16(dy), ws.defined() ? ws.data_ptr<float>() : nullptr);
  return {dx, wt};
}

// dw = conv2d backward-weight (fp32 or bf16 output, KRSC = channels_last [Cout, C, R, S]).
// pending != nullptr: a split-K reduce is left for a backward-data launch (conv_wgrad_deferred).
Tensor conv_wgrad_impl(Tensor dy, Tensor x, std::vector<int64_t> wshape, int64_t stride, int64_t pad, bool fp32_out,
                       PendingReduce* pending, int64_t target_blocks = 0) {
  check_cl_bf16(dy, "grad_output");
  check_cl_bf16(x, "x");
  same_16(dy, x, "conv_wgrad");
  TORCH_CHECK(wshape.size() == 4, "conv_wgrad: weight shape must be [Cout, C, R, S]");
  const int Cout = wshape[0], C = wshape[1], R = wshape[2], S = wshape[3];
  const int N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.size(1) == C && dy.size(1) == Cout && dy.size(0) == N, "conv_wgrad: shape mismatch");
  TORCH_CHECK(dpt::conv_supported(C, Cout) || dpt::conv_supported_narrow(C, Cout, S),
              "conv_wgrad: needs C % 64 == 0 (or C in {16, 32} with S % (64/C) == 0) and Cout % 64 == 0");
  const int Hs = (H + 2 * pad - R) / stride + 1, Ws = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dy.size(2) >= 1 && dy.size(2) <= Hs && dy.size(3) >= 1 && dy.size(3) <= Ws,
              "conv_wgrad: grad_output spatial mismatch");
  // the output size comes from dy (covers asymmetric padding)
  auto pl = dpt::conv_wgrad_plan(N, H, W, C, Cout, R, S, (int)stride, (int)pad, (int)dy.size(2), (int)dy.size(3),
                                 (int)target_blocks);
  TORCH_CHECK((int64_t)N * pl.Ho * pl.Wo < (1ll << 31), "conv_wgrad: too many pixels");
  auto dw = at::empty({Cout, C, R, S}, x.options().dtype(fp32_out ? at::kFloat : x.scalar_type())
                                          .memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t pf = pl.splits == 1 && !fp32_out ? (int64_t)Cout * C * R * S : pl.part_floats;
  auto part = at::empty({std::max<int64_t>(pf, 4)}, x.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_conv_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                         part.data_ptr<float>(), dw.data_ptr(), fp32_out ? 0 : (is_f16(x) ? 2 : 1), N, H, W, C, Cout, R,
                         S, (int)stride, (int)pad, pl, cur_stream(x), is_f16(x), pending ? &pending->r : nullptr);
  if (pending) {
    pending->part = part;
    pending->dw = dw;
  }
  return dw;
}

Tensor conv_wgrad(Tensor dy, Tensor x, std::vector<int64_t> wshape, int64_t stride, int64_t pad, bool fp32_out,
                  int64_t target_blocks) {
  return conv_wgrad_impl(dy, x, wshape, stride, pad, fp32_out, nullptr, target_blocks);
}

// (dw, pending): the backward-weight kernel is launched, its split-K reduce (if the plan needs
// one) is not - pass `pending` to the conv's backward-data binding (wgrad_reduce=) to run it in
// that launch's tail, or conv_reduce_flush it.  pending is None when nothing is left to do.
py::tuple conv_wgrad_deferred(Tensor dy, Tensor x, std::vector<int64_t> wshape, int64_t stride, int64_t pad) {
  auto p = std::make_shared<PendingReduce>();
  Tensor dw = conv_wgrad_impl(dy, x, wshape, stride, pad, false, p.get());
  if (p->r.consumed) return py::make_tuple(dw, py::none());
  return py::make_tuple(dw, p);
}

void conv_reduce_flush(PendingReducePtr p) {
  if (!p || p->r.consumed) return;
  c10::hip::HIPGuard guard(p->part.device().index());
  dpt::launch_wgrad_reduce(p->r, cur_stream(p->part));
  p->r.consumed = true;
}

// a = im2col(x) as a channels_last [N, Kp, Ho, Wo] bf16 tensor (x: channels_last fp32/bf16)
// ---- fp32 convolutions (conv_f32_kernels.hip) ---------------------------------------------
void check_cl_f32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 4, name, ": expected a 4-D CUDA fp32 tensor");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, ": expected channels_last memory");
}

Tensor conv_f32_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad) {
  check_cl_f32(x, "x");
  check_cl_f32(w, "w");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Co = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_f32_fwd: channel mismatch");
  TORCH_CHECK(C % 4 == 0 && Co % 4 == 0, "conv_f32_fwd: channels must be multiples of 4");
  TORCH_CHECK(stride >= 1 && pad >= 0, "conv_f32_fwd: bad stride/pad");
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "conv_f32_fwd: empty output");
  auto y = at::empty({N, Co, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t wsn = dpt::conv_f32_workspace((int64_t)N * Ho * Wo, Co, R * S * C);
  Tensor ws = wsn > 0 ? at::empty({wsn}, x.options()) : Tensor();
  dpt::launch_conv_f32(x.data_ptr<float>(), w.data_ptr<float>(), y.data_ptr<float>(),
                       ws.defined() ? ws.data_ptr<float>() : nullptr, false, N, H, W, C, Ho, Wo, Co, R, S,
                       (int)stride, (int)pad, cur_stream(x));
  return y;
}

// dx of a conv with input H x W: the transposed-conv gather of dy against the weight
// transposed to [C][R][S][Co] (a copy of the small weight tensor).
Tensor conv_f32_dgrad(Tensor dy, Tensor w, int64_t stride, int64_t pad, int64_t H, int64_t W) {
  check_cl_f32(dy, "grad_output");
  check_cl_f32(w, "w");
  const int N = dy.size(0), Co = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  const int C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(0) == Co, "conv_f32_dgrad: channel mismatch");
  TORCH_CHECK(C % 4 == 0 && Co % 4 == 0, "conv_f32_dgrad: channels must be multiples of 4");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == Ho && (W + 2 * pad - S) / stride + 1 == Wo,
              "conv_f32_dgrad: input size does not match grad_output");
  Tensor wt = w.permute({1, 2, 3, 0}).contiguous();  // logical [C, R, S, Co] from memory [Co][R][S][C]
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(dy.device().index());
  const int64_t wsn = dpt::conv_f32_workspace((int64_t)N * H * W, C, R * S * Co);
  Tensor ws = wsn > 0 ? at::empty({wsn}, dy.options()) : Tensor();
  dpt::launch_conv_f32(dy.data_ptr<float>(), wt.data_ptr<float>(), dx.data_ptr<float>(),
                       ws.defined() ? ws.data_ptr<float>() : nullptr, true, N, (int)H, (int)W, C, Ho, Wo, Co, R, S,
                       (int)stride, (int)pad, cur_stream(dy));
  return dx;
}

Tensor conv_f32_wgrad(Tensor dy, Tensor x, std::vector<int64_t> wshape, int64_t stride, int64_t pad) {
  check_cl_f32(dy, "grad_output");
  check_cl_f32(x, "x");
  TORCH_CHECK(wshape.size() == 4, "conv_f32_wgrad: weight shape must be [Co, C, R, S]");
  const int Co = wshape[0], C = wshape[1], R = wshape[2], S = wshape[3];
  const int N = x.size(0), H = x.size(2), W = x.size(3), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(x.size(1) == C && dy.size(1) == Co && dy.size(0) == N, "conv_f32_wgrad: shape mismatch");
  TORCH_CHECK(C % 4 == 0 && Co % 4 == 0, "conv_f32_wgrad: channels must be multiples of 4");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == Ho && (W + 2 * pad - S) / stride + 1 == Wo,
              "conv_f32_wgrad: input size does not match grad_output");
  auto dw = at::empty({Co, C, R, S}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t wsn = dpt::conv_f32_wgrad_workspace(N, Ho, Wo, Co, R * S * C);
  Tensor ws = wsn > 0 ? at::empty({wsn}, x.options()) : Tensor();
  dpt::launch_conv_f32_wgrad(dy.data_ptr<float>(), x.data_ptr<float>(), dw.data_ptr<float>(),
                             ws.defined() ? ws.data_ptr<float>() : nullptr, N, H, W, C, Ho, Wo, Co, R, S,
                             (int)stride, (int)pad, cur_stream(x));
  return dw;
}

Tensor im2col(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Kp) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "im2col: x must be a 4-d fp32/bf16 GPU tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "im2col: x must be channels_last");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(Kp % 64 == 0 && Kp >= R * S * C, "im2col: Kp must be a multiple of 64 covering R*S*C");
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  auto a = at::empty({N, Kp, Ho, Wo}, x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_im2col(x.data_ptr(), x.scalar_type() == at::kBFloat16, reinterpret_cast<uint16_t*>(a.data_ptr()), N, H,
                     W, C, (int)R, (int)S, (int)stride, (int)pad, (int)Kp, cur_stream(x));
  return a;
}

// ---- fused self-attention (ViT) ---------------------------------------------------------------
void check_bf16_contig(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), name,
              " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

// qkv [B, S, 3*H*64] -> {ctx [B, S, H*64], lse2 [B*H, stride]}
std::vector<Tensor> attn_fwd(Tensor qkv, int64_t heads, double scale) {
  check_bf16_contig(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * heads * 64, "attn_fwd: qkv must be [B, S, 3*H*64]");
  const int B = qkv.size(0), S = qkv.size(1), H = heads;
  TORCH_CHECK(dpt::attn_supported(S, 64), "attn_fwd: needs S <= 256 and head dim 64");
  auto ctx = at::empty({B, S, H * 64}, qkv.options());
  auto lse = at::empty({(int64_t)B * H, dpt::attn_lse_stride(S)}, qkv.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(qkv.device().index());
  dpt::launch_attn_fwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()), reinterpret_cast<uint16_t*>(ctx.data_ptr()),
                       lse.data_ptr<float>(), B, S, H, (float)scale, cur_stream(qkv));
  return {ctx, lse};
}

Tensor attn_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, int64_t heads, double scale) {
  check_bf16_contig(qkv, "qkv");
  check_bf16_contig(out, "out");
  check_bf16_contig(dout, "grad_output");
  const int B = qkv.size(0), S = qkv.size(1), H = heads;
  TORCH_CHECK(out.sizes() == dout.sizes() && out.dim() == 3 && out.size(0) == B && out.size(1) == S &&
                  out.size(2) == H * 64 && qkv.size(2) == 3 * H * 64, "attn_bwd: shape mismatch");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.numel() == (int64_t)B * H * dpt::attn_lse_stride(S), "attn_bwd: bad lse");
  auto dqkv = at::empty_like(qkv);
  c10::hip::HIPGuard guard(qkv.device().index());
  dpt::launch_attn_bwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()), reinterpret_cast<const uint16_t*>(out.data_ptr()),
                       reinterpret_cast<const uint16_t*>(dout.data_ptr()), lse.data_ptr<float>(),
                       reinterpret_cast<uint16_t*>(dqkv.data_ptr()), B, S, H, (float)scale, cur_stream(qkv));
  return dqkv;
}

// 2x2 space-to-depth of a channels_last [N, C<=4, H, W] fp32/bf16 image -> channels_last bf16
// [N, 16, H/2, W/2] (channel (a*2 + b)*4 + c)
Tensor space_to_depth2(Tensor x, bool out_f16) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "space_to_depth2: x must be a 4-d fp32/bf16 GPU tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "space_to_depth2: x must be channels_last");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C <= 4 && H % 2 == 0 && W % 2 == 0, "space_to_depth2: needs C <= 4 and even H, W");
  auto a = at::empty({N, 16, H / 2, W / 2},
                     x.options().dtype(out_f16 ? at::kHalf : at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_space_to_depth2(x.data_ptr(), x.scalar_type() == at::kBFloat16, reinterpret_cast<uint16_t*>(a.data_ptr()),
                              N, H, W, C, cur_stream(x), out_f16);
  return a;
}

std::vector<Tensor> bn_fwd_train(Tensor x, c10::optional<Tensor> residual, c10::optional<Tensor> weight,
                                 c10::optional<Tensor> bias, c10::optional<Tensor> running_mean,
                                 c10::optional<Tensor> running_var, c10::optional<Tensor> num_batches,
                                 double momentum, double eps, bool relu, c10::optional<Tensor> psum,
                                 c10::optional<Tensor> psq, bool apply, c10::optional<Tensor> mask_out) {
  auto [M, C] = bn_rows(x, "x");
  TORCH_CHECK(dpt::bn_supported(C), "fused BN: unsupported channel count ", C);
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual mismatch");
    bn_rows(*residual, "residual");
    rp = residual->data_ptr();
  }
  int64_t* nb = nullptr;
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->is_cuda() && num_batches->scalar_type() == at::kLong, "num_batches must be int64 GPU");
    nb = num_batches->data_ptr<int64_t>();
  }
  // apply = false: statistics, running-stat update and coefficients only (y is empty)
  auto y = apply ? at::empty_like(x) : at::empty({0}, x.options());
  void* yp = apply ? y.data_ptr() : nullptr;
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto coef = at::empty({2 * C}, fopt);  // [a | b]: y = relu(x*a + b [+ r]); lets bn_bwd skip reading y
  uint8_t* mp = relu_mask_ptr(mask_out, M, C, x, "bn_fwd_train");
  TORCH_CHECK(mp == nullptr || (relu && rp != nullptr && apply), "bn_fwd_train: mask_out needs relu + residual");
  c10::hip::HIPGuard guard(x.device().index());
  if (psum.has_value() && psum->defined()) {
    // statistics summed by the producing conv's epilogue: [C][chunks] fp32 partials
    TORCH_CHECK(psq.has_value() && psq->defined(), "bn_fwd_train: psum without psq");
    TORCH_CHECK(psum->is_cuda() && psum->scalar_type() == at::kFloat && psum->dim() == 2 && psum->size(0) == C &&
                    psum->is_contiguous() && psq->sizes() == psum->sizes() && psq->is_contiguous(),
                "bn_fwd_train: partials must be contiguous fp32 [C, chunks]");
    dpt::launch_bn_fwd_from_partials(bn_dtype(x), x.data_ptr(), rp, yp, M, C, psum->data_ptr<float>(),
                                     psq->data_ptr<float>(), (int)psum->size(1), f32_param(weight, C, "weight"),
                                     f32_param(bias, C, "bias"), (float)eps, (float)momentum,
                                     f32_param(running_mean, C, "running_mean"),
                                     f32_param(running_var, C, "running_var"), nb, mean.data_ptr<float>(),
                                     invstd.data_ptr<float>(), coef.data_ptr<float>(), relu, cur_stream(x), mp);
    return {y, mean, invstd, coef};
  }
  auto ws = at::empty({dpt::bn_workspace_floats(M, C)}, fopt);
  dpt::launch_bn_fwd_train(bn_dtype(x), x.data_ptr(), rp, yp, M, C, f32_param(weight, C, "weight"),
                           f32_param(bias, C, "bias"), (float)eps, (float)momentum,
                           f32_param(running_mean, C, "running_mean"), f32_param(running_var, C, "running_var"), nb,
                           mean.data_ptr<float>(), invstd.data_ptr<float>(), coef.data_ptr<float>(),
                           ws.data_ptr<float>(), relu, cur_stream(x), mp);
  return {y, mean, invstd, coef};
}

// y = relu(x*a + b + x2*a2 + b2), coef = [a | b], coef2 = [a2 | b2] (bn_fwd_train coefficients)
Tensor bn_apply_aff(Tensor x, Tensor x2, Tensor coef, Tensor coef2, c10::optional<Tensor> mask_out) {
  auto [M, C] = bn_rows(x, "x");
  TORCH_CHECK(dpt::bn_supported(C), "fused BN: unsupported channel count ", C);
  TORCH_CHECK(x2.sizes() == x.sizes() && x2.scalar_type() == x.scalar_type(), "bn_apply_aff: x2 mismatch");
  bn_rows(x2, "x2");
  const float* a = f32_param(coef, 2 * C, "coef");
  const float* a2 = f32_param(coef2, 2 * C, "coef2");
  auto y = at::empty_like(x);
  c10::hip::HIPGuard guard(x.device().index());
  uint8_t* mp = relu_mask_ptr(mask_out, M, C, x, "bn_apply_aff");
  dpt::launch_bn_apply_aff(bn_dtype(x), x.data_ptr(), x2.data_ptr(), y.data_ptr(), M, C, a, a + C, a2, a2 + C,
                           cur_stream(x), mp);
  return y;
}

// Backward of bn_apply_aff + ReLU from dgrad-epilogue partials (dz already masked): {dx, dx2,
// dgamma, dbeta, dgamma2, dbeta2}.
std::vector<Tensor> bn2_bwd_partials(Tensor dz, Tensor x, Tensor x2, c10::optional<Tensor> weight,
                                     c10::optional<Tensor> weight2, Tensor mean, Tensor invstd, Tensor mean2,
                                     Tensor invstd2, Tensor p1, Tensor p2, Tensor p3, bool want_dparams) {
  auto [M, C] = bn_rows(x, "x");
  TORCH_CHECK(dz.sizes() == x.sizes() && x2.sizes() == x.sizes() && dz.scalar_type() == x.scalar_type() &&
                  x2.scalar_type() == x.scalar_type(), "bn2_bwd_partials: shape/dtype mismatch");
  bn_rows(dz, "dz");
  bn_rows(x2, "x2");
  for (const Tensor* t : {&p1, &p2, &p3})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(0) == C &&
                    t->is_contiguous() && t->sizes() == p1.sizes(), "bn2_bwd_partials: partials must be fp32 [C, chunks]");
  auto fopt = x.options().dtype(at::kFloat);
  auto dx = at::empty_like(x), dx2 = at::empty_like(x2);
  Tensor dg = want_dparams ? at::empty({C}, fopt) : Tensor(), db = want_dparams ? at::empty({C}, fopt) : Tensor();
  Tensor dg2 = want_dparams ? at::empty({C}, fopt) : Tensor(), db2 = want_dparams ? at::empty({C}, fopt) : Tensor();
  auto kbuf = at::empty({6 * C}, fopt);
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_bn2_bwd_from_partials(
      bn_dtype(x), dz.data_ptr(), x.data_ptr(), x2.data_ptr(), M, C, f32_param(weight, C, "weight"),
      f32_param(mean, C, "mean"), f32_param(invstd, C, "invstd"), f32_param(weight2, C, "weight2"),
      f32_param(mean2, C, "mean2"), f32_param(invstd2, C, "invstd2"), p1.data_ptr<float>(), p2.data_ptr<float>(),
      p3.data_ptr<float>(), (int)p1.size(1), want_dparams ? dg.data_ptr<float>() : nullptr,
      want_dparams ? db.data_ptr<float>() : nullptr, want_dparams ? dg2.data_ptr<float>() : nullptr,
      want_dparams ? db2.data_ptr<float>() : nullptr, dx.data_ptr(), dx2.data_ptr(), kbuf.data_ptr<float>(),
      cur_stream(x));
  return {dx, dx2, dg, db, dg2, db2};
}

Tensor bn_apply(Tensor x, c10::optional<Tensor> residual, Tensor a, Tensor b, bool relu) {
  auto [M, C] = bn_rows(x, "x");
  TORCH_CHECK(dpt::bn_supported(C), "fused BN: unsupported channel count ", C);
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual mismatch");
    bn_rows(*residual, "residual");
    rp = residual->data_ptr();
  }
  auto y = at::empty_like(x);
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_bn_apply(bn_dtype(x), x.data_ptr(), rp, y.data_ptr(), M, C, f32_param(a, C, "a"),
                       f32_param(b, C, "b"), relu, cur_stream(x));
  return y;
}

// Returns {dx, dgamma, dbeta, dz}.  dy2: gradient of the second (aliased) output, if the
// forward exposed one.  dz (= the residual-path gradient) is materialised when want_dz or
// dy2 is given.
// coef: the forward's [a | b]; with ReLU and no residual-path output, the mask is recomputed
// from x (y may then be None).
std::vector<Tensor> bn_bwd(Tensor dy, c10::optional<Tensor> dy2, c10::optional<Tensor> y, Tensor x,
                           c10::optional<Tensor> weight, Tensor mean, Tensor invstd, bool relu, bool want_dz,
                           bool want_dparams, c10::optional<Tensor> coef) {
  auto [M, C] = bn_rows(x, "x");
  auto [Md, Cd] = bn_rows(dy, "grad_output");
  TORCH_CHECK(M == Md && C == Cd && dy.scalar_type() == x.scalar_type(), "grad_output mismatch");
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    auto [M2, C2] = bn_rows(*dy2, "grad_output2");
    TORCH_CHECK(M2 == M && C2 == C && dy2->scalar_type() == x.scalar_type(), "grad_output2 mismatch");
    d2 = dy2->data_ptr();
  }
  const bool make_dz = want_dz || d2 != nullptr;
  const float* cp = nullptr;
  if (relu && !make_dz && coef.has_value() && coef->defined()) cp = f32_param(*coef, 2 * C, "coef");
  const void* yp = nullptr;
  if (relu && cp == nullptr) {
    TORCH_CHECK(y.has_value() && y->defined(), "relu backward needs the saved output (or coef)");
    bn_rows(*y, "y");
    yp = y->data_ptr();
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto dx = at::empty_like(x);
  Tensor dz = make_dz ? at::empty_like(x) : Tensor();
  Tensor dg = want_dparams ? at::empty({C}, fopt) : Tensor();
  Tensor db = want_dparams ? at::empty({C}, fopt) : Tensor();
  auto ws = at::empty({dpt::bn_workspace_floats(M, C)}, fopt);
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_bn_bwd(bn_dtype(x), dy.data_ptr(), d2, yp, x.data_ptr(), M, C, f32_param(weight, C, "weight"),
                     f32_param(mean, C, "mean"), f32_param(invstd, C, "invstd"), cp,
                     want_dparams ? dg.data_ptr<float>() : nullptr, want_dparams ? db.data_ptr<float>() : nullptr,
                     dx.data_ptr(), make_dz ? dz.data_ptr() : nullptr, ws.data_ptr<float>(), relu, cur_stream(x));
  return {dx, dg, db, dz};
}

// BN+ReLU backward from statistics partials summed by the consuming conv's dgrad epilogue:
// {dx, dgamma, dbeta}; the ReLU mask is recomputed from x and coef.
std::vector<Tensor> bn_bwd_partials(Tensor dy, Tensor x, c10::optional<Tensor> weight, Tensor mean, Tensor invstd,
                                    c10::optional<Tensor> coef, Tensor p1, Tensor p2, bool want_dparams, bool from_dz) {
  auto [M, C] = bn_rows(x, "x");
  auto [Md, Cd] = bn_rows(dy, "grad_output");
  TORCH_CHECK(M == Md && C == Cd && dy.scalar_type() == x.scalar_type(), "grad_output mismatch");
  TORCH_CHECK(p1.is_cuda() && p1.scalar_type() == at::kFloat && p1.dim() == 2 && p1.size(0) == C &&
                  p1.is_contiguous() && p2.sizes() == p1.sizes() && p2.is_contiguous(),
              "bn_bwd_partials: partials must be contiguous fp32 [C, chunks]");
  TORCH_CHECK(from_dz || (coef.has_value() && coef->defined()), "bn_bwd_partials: coef needed unless from_dz");
  auto fopt = x.options().dtype(at::kFloat);
  auto dx = at::empty_like(x);
  Tensor dg = want_dparams ? at::empty({C}, fopt) : Tensor();
  Tensor db = want_dparams ? at::empty({C}, fopt) : Tensor();
  auto kbuf = at::empty({3 * C}, fopt);
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_bn_bwd_from_partials(bn_dtype(x), dy.data_ptr(), x.data_ptr(), M, C, f32_param(weight, C, "weight"),
                                   f32_param(mean, C, "mean"), f32_param(invstd, C, "invstd"),
                                   f32_param(coef, 2 * C, "coef"), p1.data_ptr<float>(), p2.data_ptr<float>(),
                                   (int)p1.size(1), want_dparams ? dg.data_ptr<float>() : nullptr,
                                   want_dparams ? db.data_ptr<float>() : nullptr, dx.data_ptr(), kbuf.data_ptr<float>(),
                                   cur_stream(x), from_dz);
  return {dx, dg, db};
}

std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t stride, int64_t pad, c10::optional<Tensor> bn_coef) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool: x must be a 4-D channels_last GPU tensor");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(!(bn_coef.has_value() && bn_coef->defined()) || k == 3, "maxpool: the folded BN needs a 3x3 window");
  TORCH_CHECK(C % 8 == 0 && k >= 1 && k * k <= 255 && stride >= 1 && pad >= 0 && pad <= k / 2, "maxpool: bad config");
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  auto y = at::empty({B, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({B, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_maxpool_fwd(bn_dtype(x), x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), B, (int)H, (int)W,
                          (int)C, (int)Ho, (int)Wo, (int)k, (int)stride, (int)pad, cur_stream(x),
                          bn_coef.has_value() && bn_coef->defined() ? f32_param(bn_coef, 2 * C, "bn_coef") : nullptr);
  
  return {y, idx};
}

std::vector<Tensor> maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t stride, int64_t pad,
                                c10::optional<Tensor> dy2, c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mean,
                                c10::optional<Tensor> bn_coef) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_bwd: grad must be channels_last");
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == at::kByte &&
                  idx.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_bwd: idx mismatch");
  const int64_t B = dy.size(0), C = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && Ho == (H + 2 * pad - k) / stride + 1 && Wo == (W + 2 * pad - k) / stride + 1,
              "maxpool_bwd: geometry mismatch");
  const bool two = dy2.has_value() && dy2->defined();
  if (two)
    TORCH_CHECK(dy2->sizes() == dy.sizes() && dy2->scalar_type() == dy.scalar_type() &&
                    dy2->is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_bwd: dy2 must match grad_output");
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool bns = bn_x.has_value() && bn_x->defined();
  Tensor p1, p2;
  if (bns) {
    TORCH_CHECK(k == 3 && stride == 2 && pad == 1, "maxpool_bwd: BN statistics only for the 3x3/2/1 pool");
    TORCH_CHECK(C <= 512 && (C & (C - 1)) == 0, "maxpool_bwd: BN statistics need a power-of-two C <= 512");
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_x->scalar_type() == dy.scalar_type() &&
                    bn_x->is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool_bwd: bn_x must match dx");
    const int chunks = dpt::maxpool_bwd_bn_chunks(B, (int)H, (int)W, (int)C);
    p1 = at::empty({C, chunks}, dy.options().dtype(at::kFloat));
    p2 = at::empty({C, chunks}, dy.options().dtype(at::kFloat));
  }
  c10::hip::HIPGuard guard(dy.device().index());
  dpt::launch_maxpool_bwd(bn_dtype(dy), dy.data_ptr(), two ? dy2->data_ptr() : nullptr, idx.data_ptr<uint8_t>(),
                          dx.data_ptr(), B, (int)H, (int)W,
                          (int)C, (int)Ho, (int)Wo, (int)k, (int)stride, (int)pad, cur_stream(dy), bns ? bn_x->data_ptr() : nullptr,
                          bns ? f32_param(bn_mean, C, "bn_mean") : nullptr, bns ? f32_param(bn_coef, 2 * C, "bn_coef") : nullptr,
                          bns ? p1.data_ptr<float>() : nullptr, bns ? p2.data_ptr<float>() : nullptr);
  if (bns) return {dx, p1, p2};
  
  return {dx};
}

// dx = broadcast of g [N, C] / (H*W) over an [N, C, H, W] channels_last tensor of dtype like_dtype
// {dz, p1, p2}: global-average-pool backward through a block tail y = relu(bn(x) + res):
// dz = g/(H*W) * (y > 0) (y's dtype) and the tail BN's backward statistics partials.
std::vector<Tensor> gap_bwd_bnr(Tensor g, Tensor y, Tensor x, Tensor mean) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous(), "gap_bwd_bnr: g must be a contiguous [N, C]");
  auto [M, C] = bn_rows(y, "y");
  auto [Mx, Cx] = bn_rows(x, "x");
  TORCH_CHECK(M == Mx && C == Cx && x.scalar_type() == y.scalar_type() && g.size(1) == C && g.size(0) == y.size(0),
              "gap_bwd_bnr: shape mismatch");
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "gap_bwd_bnr: needs C/8 | 256");
  const int64_t N = y.size(0), HW = y.size(2) * y.size(3);
  auto dz = at::empty_like(y);
  const int chunks = dpt::gap_bwd_bnr_chunks(M, C);
  auto p1 = at::empty({C, chunks}, y.options().dtype(at::kFloat));
  auto p2 = at::empty({C, chunks}, y.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(y.device().index());
  dpt::launch_gap_bwd_bnr(bn_dtype(y), bn_dtype(g), g.data_ptr(), dz.data_ptr(), y.data_ptr(), x.data_ptr(),
                          f32_param(mean, C, "mean"), N, HW, C, p1.data_ptr<float>(), p2.data_ptr<float>(),
                          cur_stream(y));
  return {dz, p1, p2};
}

Tensor gap_bwd(Tensor g, int64_t H, int64_t W, at::ScalarType dtype) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && g.size(1) % 8 == 0, "gap_bwd: g must be [N, C], C % 8 == 0");
  TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16 || dtype == at::kHalf, "gap_bwd: dtype");
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(N * H * W * (C / 8) < (int64_t(1) << 32) - 256, "gap_bwd: too large");
  auto dx = at::empty({N, C, H, W}, g.options().dtype(dtype).memory_format(at::MemoryFormat::ChannelsLast));
  c10::hip::HIPGuard guard(g.device().index());
  dpt::launch_gap_bwd(bn_dtype(dx), bn_dtype(g), g.data_ptr(), dx.data_ptr(), N, H * W, C, cur_stream(g));
  return dx;
}

// ---- ViT block kernels (vit_kernels.hip) -----------------------------------------------------
int act16_kind(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(t.scalar_type() == at::kHalf, name, " must be bf16 or fp16");
  return 2;
}

// A per-column parameter of any float dtype (the fp32 master or its 16-bit shadow).
int param_kind(const Tensor& t, int64_t D, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == D, name, " must be a contiguous GPU tensor of ", D,
              " elements");
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, name, " must be f32/bf16/f16");
  }
  return 0;
}

at::ScalarType kind_dtype(int kind) { return kind == 1 ? at::kBFloat16 : at::kHalf; }

// s = x + a + bias (only when a is given), h = LayerNorm(s) (16-bit), per-row mean / rstd.
std::vector<Tensor> ln_fwd(Tensor x, c10::optional<Tensor> a, c10::optional<Tensor> bias,
                           c10::optional<Tensor> gamma, c10::optional<Tensor> beta, double eps, int64_t out_kind) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "ln: x must be contiguous fp32 GPU");
  const int64_t D = x.size(-1), T = x.numel() / D;
  TORCH_CHECK(dpt::ln_supported(D), "ln: width must be a multiple of 256 in [256, 2048], got ", D);
  const bool add = a.has_value() && a->defined();
  int kind = (int)out_kind;
  const void* bp = nullptr;
  int bk = 0;
  if (add) {
    kind = act16_kind(*a, "ln: a");
    TORCH_CHECK(a->sizes() == x.sizes(), "ln: a must match x");
    if (bias.has_value() && bias->defined()) {
      bk = param_kind(*bias, D, "ln: bias");
      bp = bias->data_ptr();
    }
  }
  TORCH_CHECK(kind == 1 || kind == 2, "ln: output kind must be 1 (bf16) or 2 (fp16)");
  Tensor sv = add ? at::empty_like(x) : Tensor();
  auto h = at::empty(x.sizes(), x.options().dtype(kind_dtype(kind)));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({T}, fopt), rstd = at::empty({T}, fopt);
  c10::hip::HIPGuard guard(x.device().index());
  dpt::launch_ln_fwd(kind, x.data_ptr<float>(), add ? static_cast<const uint16_t*>(a->data_ptr()) : nullptr, bp, bk,
                     f32_param(gamma, D, "gamma"), f32_param(beta, D, "beta"), add ? sv.data_ptr<float>() : nullptr,
                     static_cast<uint16_t*>(h.data_ptr()), mean.data_ptr<float>(), rstd.data_ptr<float>(), T, D,
                     (float)eps, cur_stream(x));
  return {sv, h, mean, rstd};
}

// Returns {gx, ga, dgamma, dbeta, dbias}: gx = gs + LN_bwd(gh) (fp32); with want_ga also
// ga = 16-bit(gx) and, if bias_like is given, dbias = column sums of gx in bias_like's dtype.
std::vector<Tensor> ln_bwd(c10::optional<Tensor> gs, Tensor gh, Tensor sv, Tensor mean, Tensor rstd,
                           c10::optional<Tensor> gamma, bool want_ga, c10::optional<Tensor> bias_like,
                           bool want_dparams) {
  TORCH_CHECK(sv.is_cuda() && sv.scalar_type() == at::kFloat && sv.is_contiguous(), "ln_bwd: s must be fp32");
  const int64_t D = sv.size(-1), T = sv.numel() / D;
  TORCH_CHECK(dpt::ln_supported(D), "ln_bwd: unsupported width ", D);
  const int kind = act16_kind(gh, "ln_bwd: grad_h");
  TORCH_CHECK(gh.sizes() == sv.sizes(), "ln_bwd: grad_h must match s");
  TORCH_CHECK(mean.numel() == T && rstd.numel() == T, "ln_bwd: mean/rstd must have one entry per row");
  const float* gsp = nullptr;
  if (gs.has_value() && gs->defined()) {
    TORCH_CHECK(gs->scalar_type() == at::kFloat && gs->is_contiguous() && gs->sizes() == sv.sizes(),
                "ln_bwd: grad_s must be contiguous fp32 like s");
    gsp = gs->data_ptr<float>();
  }
  auto fopt = sv.options().dtype(at::kFloat);
  auto gx = at::empty_like(sv);
  Tensor ga = want_ga ? at::empty(sv.sizes(), sv.options().dtype(kind_dtype(kind))) : Tensor();
  Tensor dg = want_dparams ? at::empty({D}, fopt) : Tensor();
  Tensor db = want_dparams ? at::empty({D}, fopt) : Tensor();
  Tensor dbias;
  int dbk = 0;
  if (want_ga && bias_like.has_value() && bias_like->defined()) {
    dbk = param_kind(*bias_like, D, "ln_bwd: bias");
    dbias = at::empty({D}, sv.options().dtype(bias_like->scalar_type()));
  }
  auto part = at::empty({3 * (int64_t)dpt::ln_bwd_blocks(T) * D}, fopt);
  c10::hip::HIPGuard guard(sv.device().index());
  dpt::launch_ln_bwd(kind, gsp, static_cast<const uint16_t*>(gh.data_ptr()), sv.data_ptr<float>(),
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), f32_param(gamma, D, "gamma"), gx.data_ptr<float>(),
                     want_ga ? static_cast<uint16_t*>(ga.data_ptr()) : nullptr, part.data_ptr<float>(),
                     want_dparams ? dg.data_ptr<float>() : nullptr, want_dparams ? db.data_ptr<float>() : nullptr,
                     dbias.defined() ? dbias.data_ptr() : nullptr, dbk, T, D, cur_stream(sv));
  return {gx, ga, dg, db, dbias};
}

Tensor gelu_fwd(Tensor u, c10::optional<Tensor> bias) {
  const int kind = act16_kind(u, "gelu: u");
  const int64_t F = u.size(-1), T = u.numel() / F;
  TORCH_CHECK(F % 8 == 0, "gelu: width must be a multiple of 8");
  const void* bp = nullptr;
  int bk = 0;
  if (bias.has_value() && bias->defined()) {
    bk = param_kind(*bias, F, "gelu: bias");
    bp = bias->data_ptr();
  }
  auto h = at::empty_like(u);
  c10::hip::HIPGuard guard(u.device().index());
  dpt::launch_gelu_fwd(kind, static_cast<const uint16_t*>(u.data_ptr()), bp, bk, static_cast<uint16_t*>(h.data_ptr()),
                       T, F, cur_stream(u));
  return h;
}

// Returns {gu, dbias}: gu = gh * gelu'(u + bias); dbias = column sums of gu (bias dtype).
std::vector<Tensor> gelu_bwd(Tensor gh, Tensor u, c10::optional<Tensor> bias, bool want_dbias) {
  const int kind = act16_kind(u, "gelu_bwd: u");
  TORCH_CHECK(act16_kind(gh, "gelu_bwd: grad") == kind && gh.sizes() == u.sizes(), "gelu_bwd: grad must match u");
  const int64_t F = u.size(-1), T = u.numel() / F;
  TORCH_CHECK(F % 8 == 0, "gelu_bwd: width must be a multiple of 8");
  const void* bp = nullptr;
  int bk = 0;
  if (bias.has_value() && bias->defined()) {
    bk = param_kind(*bias, F, "gelu_bwd: bias");
    bp = bias->data_ptr();
  }
  auto gu = at::empty_like(u);
  Tensor db = (want_dbias && bp) ? at::empty({F}, u.options().dtype(bias->scalar_type())) : Tensor();
  auto part = at::empty({(int64_t)dpt::gelu_bwd_chunks(T, F) * F}, u.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(u.device().index());
  dpt::launch_gelu_bwd(kind, static_cast<const uint16_t*>(gh.data_ptr()), static_cast<const uint16_t*>(u.data_ptr()),
                       bp, bk, static_cast<uint16_t*>(gu.data_ptr()), part.data_ptr<float>(),
                       db.defined() ? db.data_ptr() : nullptr, bk, T, F, cur_stream(u));
  return {gu, db};
}

// A Linear's backward-data with the GELU backward fused (conv_fwd_kernel DGELU epilogue):
// gu = (dy @ wt^T) * gelu'(u + bias) and part [n_in][tiles] (the column sums of gu per 128-row
// tile, [tiles][n_in]: bias gradient = part.sum(0)).  dy [T, n_out], wt [n_in, n_out] (the weight transposed),
// u [T, n_in] 16-bit and contiguous; bias [n_in] fp32 or u's dtype.
std::vector<Tensor> linear_dgrad_dgelu(Tensor dy, Tensor wt, Tensor u, Tensor bias) {
  const int kind = act16_kind(u, "linear_dgrad_dgelu: u");
  TORCH_CHECK(act16_kind(dy, "linear_dgrad_dgelu: grad") == kind && act16_kind(wt, "linear_dgrad_dgelu: wt") == kind,
              "linear_dgrad_dgelu: grad, wt and u must share one 16-bit dtype");
  TORCH_CHECK(dy.dim() == 2 && wt.dim() == 2 && u.dim() == 2 && dy.is_contiguous() && wt.is_contiguous() &&
                  u.is_contiguous(), "linear_dgrad_dgelu: contiguous 2-D operands");
  const int64_t T = dy.size(0), n_out = dy.size(1), n_in = wt.size(0);
  TORCH_CHECK(wt.size(1) == n_out && u.size(0) == T && u.size(1) == n_in, "linear_dgrad_dgelu: shape mismatch");
  TORCH_CHECK(n_in % 128 == 0 && n_out % 64 == 0, "linear_dgrad_dgelu: n_in % 128 == 0 and n_out % 64 == 0");
  const bool b16 = bias.scalar_type() == u.scalar_type();
  TORCH_CHECK((b16 || bias.scalar_type() == at::kFloat) && bias.is_contiguous() && bias.numel() == n_in &&
                  bias.is_cuda(), "linear_dgrad_dgelu: fp32 or u-typed bias of n_in elements on the device");
  TORCH_CHECK(T * n_out < (1ll << 31) && T * n_in < (1ll << 31), "linear_dgrad_dgelu: too many elements");
  auto gu = at::empty_like(u);
  auto part = at::empty({(int64_t)dpt::linear_dgrad_dgelu_tiles(T), n_in}, u.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(u.device().index());
  dpt::launch_linear_dgrad_dgelu(static_cast<const uint16_t*>(dy.data_ptr()), static_cast<const uint16_t*>(wt.data_ptr()),
                                 static_cast<const uint16_t*>(u.data_ptr()),
                                 b16 ? nullptr : bias.data_ptr<float>(),
                                 b16 ? static_cast<const uint16_t*>(bias.data_ptr()) : nullptr,
                                 static_cast<uint16_t*>(gu.data_ptr()), part.data_ptr<float>(), T, (int)n_out,
                                 (int)n_in, kind == 2, cur_stream(u));
  return {gu, part};
}

// Column sums of a 16-bit [.., F] gradient (a Linear's bias gradient) in out_dtype's kind.
Tensor bias_grad16(Tensor gy, int64_t out_kind) {
  const int kind = act16_kind(gy, "bias_grad16: grad");
  const int64_t F = gy.size(-1), T = gy.numel() / F;
  TORCH_CHECK(F % 8 == 0 && (out_kind >= 0 && out_kind <= 2), "bias_grad16: F % 8 == 0, kind 0..2");
  auto db = at::empty({F}, gy.options().dtype(out_kind == 0 ? at::kFloat : kind_dtype((int)out_kind)));
  auto part = at::empty({(int64_t)dpt::gelu_bwd_chunks(T, F) * F}, gy.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(gy.device().index());
  dpt::launch_bias_grad16(kind, static_cast<const uint16_t*>(gy.data_ptr()), part.data_ptr<float>(), db.data_ptr(),
                          (int)out_kind, T, F, cur_stream(gy));
  return db;
}

// Sum of split-K partials [S, ...] (fp32) into a new tensor of out_kind (0 f32, 1 bf16, 2 f16).
Tensor sum_partials(Tensor part, int64_t out_kind) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() >= 2,
              "sum_partials: contiguous fp32 [S, ...]");
  const int64_t S = part.size(0), n = part.numel() / S;
  TORCH_CHECK(n % 4 == 0 && out_kind >= 0 && out_kind <= 2, "sum_partials: n % 4 == 0, kind 0..2");
  auto out = at::empty(part.sizes().slice(1),
                       part.options().dtype(out_kind == 0 ? at::kFloat : kind_dtype((int)out_kind)));
  c10::hip::HIPGuard guard(part.device().index());
  dpt::launch_sum_partials(part.data_ptr<float>(), n, (int)S, out.data_ptr(), (int)out_kind, cur_stream(part));
  return out;
}

// Column sums of a [n, D] fp32 partials array (many rows: 16 waves per 64 columns) into out_kind.
Tensor colsum_rows(Tensor part, int64_t out_kind) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 2,
              "colsum_rows: contiguous fp32 [n, D]");
  TORCH_CHECK(out_kind >= 0 && out_kind <= 2, "colsum_rows: kind 0..2");
  auto out = at::empty({part.size(1)}, part.options().dtype(out_kind == 0 ? at::kFloat : kind_dtype((int)out_kind)));
  c10::hip::HIPGuard guard(part.device().index());
  dpt::launch_colsum_rows(part.data_ptr<float>(), part.size(0), part.size(1), out.data_ptr(), (int)out_kind,
                          cur_stream(part));
  return out;
}

// dst.copy_(src) for same-shape 16-bit tensors of <= 5 dims whose last dim is contiguous in
// both (e.g. attention heads [b,h,s,dh] <-> [b,s,h,dh]): one vectorised strided-row kernel.
void copy_rows16(Tensor src, Tensor dst) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.device() == dst.device(), "copy_rows16: GPU tensors");
  TORCH_CHECK(src.scalar_type() == dst.scalar_type() && src.element_size() == 2, "copy_rows16: same 16-bit dtype");
  TORCH_CHECK(src.sizes() == dst.sizes() && src.dim() >= 1 && src.dim() <= 5, "copy_rows16: same shape, <= 5 dims");
  const int nd = (int)src.dim();
  const int64_t L = src.size(nd - 1);
  TORCH_CHECK(src.stride(nd - 1) == 1 && dst.stride(nd - 1) == 1 && L % 8 == 0, "copy_rows16: rows must be contiguous, L % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "copy_rows16: 16-byte aligned data");
  int n[4] = {1, 1, 1, 1};
  int64_t ss[4] = {0, 0, 0, 0}, ds[4] = {0, 0, 0, 0};
  for (int d = 0; d < nd - 1; ++d) {
    const int slot = 4 - (nd - 1) + d;
    TORCH_CHECK(src.size(d) < (1LL << 31), "copy_rows16: dim too large");
    TORCH_CHECK(src.stride(d) % 8 == 0 && dst.stride(d) % 8 == 0, "copy_rows16: row starts must be 16-byte aligned");
    n[slot] = (int)src.size(d);
    ss[slot] = src.stride(d);
    ds[slot] = dst.stride(d);
  }
  TORCH_CHECK((int64_t)n[0] * n[1] * n[2] * n[3] < (1LL << 32), "copy_rows16: too many rows");
  c10::hip::HIPGuard guard(src.device().index());
  dpt::launch_rows_copy16(static_cast<const uint16_t*>(src.data_ptr()), static_cast<uint16_t*>(dst.data_ptr()), n, ss,
                          ds, (int)L, cur_stream(src));
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native runtime: gfx950 kernels, RCCL communicator, C++ gradient reducer";
  m.def("grad_check", &grad_check, py::arg("grad"), py::arg("scale"), py::arg("host_factor"), py::arg("found_inf"));
  m.def("sgd_step", &sgd_step, py::arg("param"), py::arg("grad"), py::arg("momentum_buffer"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"), py::arg("scale"),
        py::arg("host_factor"), py::arg("found_inf"), py::arg("step"), py::arg("zero_grad"),
        py::arg("shadow") = py::none());
  m.def("adam_step", &adam_step, py::arg("param"), py::arg("grad"), py::arg("exp_avg"), py::arg("exp_avg_sq"),
        py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("adamw"),
        py::arg("scale"), py::arg("host_factor"), py::arg("found_inf"), py::arg("step"), py::arg("zero_grad"),
        py::arg("shadow") = py::none());
  m.def("optim_tail", &optim_tail, py::arg("scale"), py::arg("growth_tracker"), py::arg("found_inf"),
        py::arg("step"), py::arg("growth_factor"), py::arg("backoff_factor"), py::arg("growth_interval"));
  m.def("pack_bf16", &pack_bf16);
  m.def("unpack_bf16", &unpack_bf16);
  m.def("accumulate_metrics", &accumulate_metrics, py::arg("logits"), py::arg("targets"), py::arg("loss"), py::arg("acc"));
  m.def("augment", &augment, py::arg("data"), py::arg("idx"), py::arg("offs"), py::arg("flips"), py::arg("out"),
        py::arg("nhwc"), py::arg("pad"), py::arg("mean"), py::arg("std"));
  m.def("bn_supported", [](int64_t C) { return dpt::bn_supported(C); });
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("residual"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches"), py::arg("momentum"), py::arg("eps"),
        py::arg("relu"), py::arg("psum") = py::none(), py::arg("psq") = py::none(), py::arg("apply") = true,
        py::arg("mask_out") = py::none());
  m.def("bn_apply", &bn_apply, py::arg("x"), py::arg("residual"), py::arg("a"), py::arg("b"), py::arg("relu"));
  m.def("bn_apply_aff", &bn_apply_aff, py::arg("x"), py::arg("x2"), py::arg("coef"), py::arg("coef2"),
        py::arg("mask_out") = py::none());
  m.def("bn2_bwd_partials", &bn2_bwd_partials, py::arg("dz"), py::arg("x"), py::arg("x2"), py::arg("weight"),
        py::arg("weight2"), py::arg("mean"), py::arg("invstd"), py::arg("mean2"), py::arg("invstd2"), py::arg("p1"),
        py::arg("p2"), py::arg("p3"), py::arg("want_dparams"));
  m.def("bn_bwd", &bn_bwd, py::arg("grad_output"), py::arg("grad_output2"), py::arg("y"), py::arg("x"),
        py::arg("weight"), py::arg("mean"), py::arg("invstd"), py::arg("relu"), py::arg("want_dz"),
        py::arg("want_dparams"), py::arg("coef") = py::none());
  m.def("ln_supported", &dpt::ln_supported, py::arg("D"));
  m.def("ln_fwd", &ln_fwd, py::arg("x"), py::arg("a"), py::arg("bias"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("out_kind") = 1);
  m.def("ln_bwd", &ln_bwd, py::arg("grad_s"), py::arg("grad_h"), py::arg("s"), py::arg("mean"), py::arg("rstd"),
        py::arg("gamma"), py::arg("want_ga"), py::arg("bias_like"), py::arg("want_dparams"));
  m.def("gelu_fwd", &gelu_fwd, py::arg("u"), py::arg("bias"));
  m.def("gelu_bwd", &gelu_bwd, py::arg("grad"), py::arg("u"), py::arg("bias"), py::arg("want_dbias"));
  m.def("linear_dgrad_dgelu", &linear_dgrad_dgelu, py::arg("grad"), py::arg("wt"), py::arg("u"), py::arg("bias"));
  m.def("vit_set_gelu_blocks_per_cu", &dpt::vit_set_gelu_blocks_per_cu, py::arg("n"));
  m.def("copy_rows16", &copy_rows16, py::arg("src"), py::arg("dst"));
  m.def("bias_grad16", &bias_grad16, py::arg("grad"), py::arg("out_kind"));
  m.def("sum_partials", &sum_partials, py::arg("part"), py::arg("out_kind"));
  m.def("colsum_rows", &colsum_rows, py::arg("part"), py::arg("out_kind"));
  m.def("maxpool_fwd", &maxpool_fwd, py::arg("x"), py::arg("k"), py::arg("stride"), py::arg("pad"),
        py::arg("bn_coef") = py::none());
  m.def("gap_bwd", &gap_bwd, py::arg("g"), py::arg("H"), py::arg("W"), py::arg("dtype"));
  m.def("gap_bwd_bnr", &gap_bwd_bnr, py::arg("g"), py::arg("y"), py::arg("x"), py::arg("mean"));
  m.def("maxpool_bwd", &maxpool_bwd, py::arg("grad_output"), py::arg("idx"), py::arg("H"), py::arg("W"),
        py::arg("k"), py::arg("stride"), py::arg("pad"), py::arg("grad_output2") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_mean") = py::none(), py::arg("bn_coef") = py::none());
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("want_stats"),
        py::arg("out_h") = 0, py::arg("out_w") = 0);
  m.def("space_to_depth2", &space_to_depth2, py::arg("x"), py::arg("out_f16") = false);
  m.def("conv_wgrad", &conv_wgrad, py::arg("grad_output"), py::arg("x"), py::arg("weight_shape"), py::arg("stride"),
        py::arg("pad"), py::arg("fp32_out"), py::arg("target_blocks") = 0);
  m.def("conv_f32_fwd", &conv_f32_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"));
  m.def("conv_f32_dgrad", &conv_f32_dgrad, py::arg("grad_output"), py::arg("w"), py::arg("stride"), py::arg("pad"),
        py::arg("H"), py::arg("W"));
  m.def("conv_f32_wgrad", &conv_f32_wgrad, py::arg("grad_output"), py::arg("x"), py::arg("weight_shape"),
        py::arg("stride"), py::arg("pad"));
  m.def("im2col", &im2col, py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("Kp"));
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("heads"), py::arg("scale"));
  m.def("attn_set_bwd_split", &dpt::attn_set_bwd_split, py::arg("on"));
  m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("out"), py::arg("grad_output"), py::arg("lse"),
        py::arg("heads"), py::arg("scale"));
  m.def("conv_set_variant", &dpt::conv_set_variant, py::arg("variant"));
  m.def("bn_set_skip_finalize", &dpt::bn_set_skip_finalize, py::arg("on"),
        "measurement only: skip every BatchNorm finalize launch (wrong values; timing upper bound)");
  m.def("conv_set_splitk_policy", &dpt::conv_set_splitk_policy, py::arg("tiles"), py::arg("eager_tiles"),
        py::arg("eager_min_k"), py::arg("target"), "split-K thresholds (A/B knob; <= 0 keeps a value)");
  m.def("conv_set_big", &dpt::conv_set_big, py::arg("on"));
  m.def("conv_set_halo", &dpt::conv_set_halo, py::arg("on"));
  m.def("conv_set_breg", &dpt::conv_set_breg, py::arg("mode"));
  m.def("conv_set_wgrad_stages", &dpt::conv_set_wgrad_stages, py::arg("mode"));
  m.def("conv_get_breg", &dpt::conv_get_breg);
  m.def("conv_set_streamk", &dpt::conv_set_streamk, py::arg("mode"), py::arg("eff") = 0.0);
  m.def("conv_get_streamk", &dpt::conv_get_streamk);
  m.def("conv_sk_prepare", &dpt::conv_sk_prepare);
  m.def("conv_sk_errors", &dpt::conv_sk_errors);
  m.def("conv_sk_blocks", &dpt::conv_sk_blocks, py::arg("tiles"), py::arg("nk"), py::arg("bn"), py::arg("mode"));
  m.def("conv_set_wgrad_target", &dpt::conv_set_wgrad_target, py::arg("blocks"));
  m.def("conv_set_wgrad_halo", &dpt::conv_set_wgrad_halo, py::arg("mode"));
  m.def("conv_fwd_splits", [](int64_t M, int Cout, int64_t K, bool graph) {
          return dpt::conv_fwd_splits_for(M, Cout, K, graph);
        }, py::arg("M"), py::arg("Cout"), py::arg("K"), py::arg("graph") = false);
  m.def("conv_set_splitk", &dpt::conv_set_splitk, py::arg("mode"));
  m.def("conv_get_splitk", &dpt::conv_get_splitk);
  m.def("conv_set_fwd_shape_policy", &dpt::conv_set_fwd_shape_policy, py::arg("bits"));
  m.def("conv_dgrad", &conv_dgrad, py::arg("grad_output"), py::arg("w"), py::arg("pad"));
  m.def("conv_dgrad_bnstats", &conv_dgrad_bnstats, py::arg("grad_output"), py::arg("w"), py::arg("pad"),
        py::arg("bn_x"), py::arg("bn_mean"), py::arg("bn_coef"), py::arg("bn_y") = py::none(),
        py::arg("bn_res") = py::none(), py::arg("w_flipped") = py::none(), py::arg("bn_x2") = py::none(),
        py::arg("bn_mean2") = py::none(), py::arg("wgrad_reduce") = nullptr, py::arg("bn_mask") = py::none());
  m.def("conv_wt_flip_multi", &conv_wt_flip_multi, py::arg("ws"));
  m.def("conv_dgrad_preflipped", &conv_dgrad_preflipped, py::arg("grad_output"), py::arg("w_flipped"), py::arg("pad"),
        py::arg("wgrad_reduce") = nullptr);
  m.def("bn_bwd_partials", &bn_bwd_partials, py::arg("grad_output"), py::arg("x"), py::arg("weight"), py::arg("mean"),
        py::arg("invstd"), py::arg("coef"), py::arg("p1"), py::arg("p2"), py::arg("want_dparams"),
        py::arg("from_dz") = false);
  m.def("conv_dgrad_s2", &conv_dgrad_s2, py::arg("grad_output"), py::arg("w"), py::arg("pad"), py::arg("H"),
        py::arg("W"), py::arg("bn_x") = py::none(), py::arg("bn_mean") = py::none(), py::arg("bn_coef") = py::none(),
        py::arg("wgrad_reduce") = nullptr);
  m.def("conv_dgrad_flip", &conv_dgrad_flip, py::arg("grad_output"), py::arg("w"), py::arg("pad"),
        py::arg("wgrad_reduce") = nullptr);
  py::class_<PendingReduce, PendingReducePtr>(m, "PendingWgradReduce")
      .def_property_readonly("done", &PendingReduce::done)
      .def_property_readonly("splits", [](const PendingReduce& p) { return p.r.splits; });
  m.def("conv_wgrad_deferred", &conv_wgrad_deferred, py::arg("grad_output"), py::arg("x"), py::arg("weight_shape"),
        py::arg("stride"), py::arg("pad"));
  m.def("conv_reduce_flush", &conv_reduce_flush, py::arg("pending"));
  m.def("rccl_version", []() { return std::string(dpt::rccl_version_string()); });

  // Collective seam (comm.h): RcclComm (production) and HostBridgeComm (ranks sharing a GPU)
  py::class_<dpt::Collective, std::shared_ptr<dpt::Collective>>(m, "Collective")
      .def("all_reduce", [](dpt::Collective& c, Tensor t, bool on_current_stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce needs a contiguous GPU tensor");
             c10::hip::HIPGuard guard(t.device().index());
             hipStream_t s = cur_stream(t);
             c.all_reduce(t.data_ptr(), (size_t)t.numel(), wire_of(t), on_current_stream ? s : c.stream());
           }, py::arg("tensor"), py::arg("on_current_stream") = true)
      .def("broadcast", [](dpt::Collective& c, Tensor t, int root) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "broadcast needs a contiguous GPU tensor");
             c10::hip::HIPGuard guard(t.device().index());
             c.broadcast(t.data_ptr(), (size_t)t.numel(), wire_of(t), root, cur_stream(t));
           }, py::arg("tensor"), py::arg("root") = 0)
      .def("abort", &dpt::Collective::abort)
      .def("destroy", &dpt::Collective::destroy)
      .def("check", &dpt::Collective::check)
      .def_property_readonly("kind", &dpt::Collective::kind)
      .def_property_readonly("ops", &dpt::Collective::ops)
      .def_property_readonly("sequence_hash", &dpt::Collective::sequence_hash)
      .def_property_readonly("rank", &dpt::Collective::rank)
      .def_property_readonly("world_size", &dpt::Collective::world_size)
      .def_property_readonly("device", &dpt::Collective::device)
      .def("track", [](dpt::Collective& c) {
             c10::hip::HIPGuard guard(c.device());
             c.track(c10::hip::getCurrentHIPStream(c.device()).stream());
           }, "hand the watchdog a completion marker for the work enqueued on the current stream")
      .def("_test_spin", [](dpt::Collective& c, double ms, bool on_current_stream) {
             TORCH_CHECK(ms >= 0 && ms <= 20000, "spin: 0..20000 ms");
             c10::hip::HIPGuard guard(c.device());
             dpt::launch_spin(ms, on_current_stream ? c10::hip::getCurrentHIPStream(c.device()).stream()
                                                    : c.stream());
           }, py::arg("ms"), py::arg("on_current_stream") = false,
           "test hook: enqueue a wall-clock busy-wait on the communicator (or current) stream");

  py::class_<dpt::RcclComm, dpt::Collective, std::shared_ptr<dpt::RcclComm>>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int, int, int, double>(), py::arg("unique_id"), py::arg("rank"),
           py::arg("world_size"), py::arg("device"), py::arg("min_ctas") = 0, py::arg("max_ctas") = 0,
           py::arg("init_timeout_s") = 0.0,
           // a peer's RCCL init may need this process's other threads; never hold the GIL there
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("min_ctas", &dpt::RcclComm::min_ctas)
      .def_property_readonly("max_ctas", &dpt::RcclComm::max_ctas)
      .def_property_readonly("handle", &dpt::RcclComm::handle)
      .def("inject_async_error", &dpt::RcclComm::inject_async_error, py::arg("message"))
      .def_static("new_unique_id", []() { return py::bytes(dpt::RcclComm::new_unique_id()); })
      .def("enable_watchdog", &dpt::RcclComm::enable_watchdog, py::arg("timeout_s"), py::arg("poll_s") = 0.5,
           py::arg("exit_grace_s") = 30.0)
      .def_property_readonly("watchdog_tripped", &dpt::RcclComm::watchdog_tripped)
      .def_property_readonly("watchdog_outstanding", &dpt::RcclComm::watchdog_outstanding)
      .def_property_readonly("watchdog_tracked", &dpt::RcclComm::watchdog_tracked)
      .def("async_error", &dpt::RcclComm::async_error);

  py::class_<dpt::HostBridgeComm, dpt::Collective, std::shared_ptr<dpt::HostBridgeComm>>(m, "HostBridgeComm")
      .def(py::init([](py::object ar, py::object bc, int rank, int ws, int dev, bool async_mode, py::object pg) {
             c10::intrusive_ptr<c10d::ProcessGroup> p;
             if (!pg.is_none()) p = pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
             return std::make_shared<dpt::HostBridgeComm>(std::move(ar), std::move(bc), rank, ws, dev, async_mode,
                                                          std::move(p));
           }),
           py::arg("all_reduce_fn"), py::arg("broadcast_fn"), py::arg("rank"), py::arg("world_size"),
           py::arg("device"), py::arg("async_mode") = false, py::arg("process_group") = py::none())
      // the async bridge drives a torch.distributed group from C++: check the Python object casts
      .def_static("_process_group_size", [](py::object pg) {
             return pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>()->getSize();
           })
      .def_property_readonly("async_mode", &dpt::HostBridgeComm::async_mode)
      .def_property_readonly("completed", &dpt::HostBridgeComm::completed)
      .def("release_graph_resources", &dpt::HostBridgeComm::release_graph_resources);

  // the Collective contract over a torch c10d group on device memory (RCCL through
  // ProcessGroupNCCL): the framework communicator's fallback and A/B arm (csrc/pg_comm.h)
  py::class_<dpt::ProcessGroupComm, dpt::Collective, std::shared_ptr<dpt::ProcessGroupComm>>(m, "ProcessGroupComm")
      .def(py::init([](py::object pg, int dev) {
             return std::make_shared<dpt::ProcessGroupComm>(pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>(), dev);
           }),
           py::arg("process_group"), py::arg("device"))
      .def_property_readonly("backend", &dpt::ProcessGroupComm::backend);

  // Watchdog decision logic with an explicit clock (unit-tested with a fake clock)
  py::class_<dpt::WatchdogCore>(m, "WatchdogCore")
      .def(py::init<double>(), py::arg("timeout_s"))
      .def("enqueue", &dpt::WatchdogCore::enqueue, py::arg("seq"), py::arg("now"))
      .def("poll", [](dpt::WatchdogCore& w, double now, py::function done, const std::string& aerr) {
             std::vector<uint64_t> completed;
             std::string trip = w.poll(now, [&](uint64_t s) { return done(s).cast<bool>(); }, aerr, &completed);
             return py::make_tuple(trip, completed);
           }, py::arg("now"), py::arg("done"), py::arg("async_error") = std::string())
      .def_property_readonly("tripped", &dpt::WatchdogCore::tripped)
      .def_property_readonly("reason", &dpt::WatchdogCore::reason)
      .def_property_readonly("outstanding", &dpt::WatchdogCore::outstanding)
      .def("oldest_age", &dpt::WatchdogCore::oldest_age, py::arg("now"));

  py::class_<dpt::Reducer, std::shared_ptr<dpt::Reducer>>(m, "Reducer")
      .def(py::init<std::vector<Tensor>, std::vector<Tensor>, Tensor, std::vector<int64_t>, std::vector<int64_t>,
                    std::vector<int64_t>, std::shared_ptr<dpt::Collective>, py::object, int, Tensor, Tensor, Tensor,
                    double, bool, bool, bool>(),
           py::arg("params"), py::arg("grad_views"), py::arg("flat_grad"), py::arg("bucket_offsets"),
           py::arg("bucket_numels"), py::arg("param_bucket"), py::arg("comm"), py::arg("py_allreduce"),
           py::arg("wire"), py::arg("wire_buf"), py::arg("found_inf"), py::arg("scale"), py::arg("host_factor"),
           py::arg("check_inf"), py::arg("profile"), py::arg("steal_grads") = false)
      .def("prepare_for_backward", &dpt::Reducer::prepare_for_backward)
      .def("mark_ready", &dpt::Reducer::mark_ready)
      .def("finalize", &dpt::Reducer::finalize)
      .def("set_require_sync", &dpt::Reducer::set_require_sync)
      .def("set_check_inf", &dpt::Reducer::set_check_inf)
      .def("set_accumulate", &dpt::Reducer::set_accumulate)
      .def("set_debug", &dpt::Reducer::set_debug)
      .def_property_readonly("require_sync", &dpt::Reducer::require_sync)
      .def("ready_order", &dpt::Reducer::ready_order)
      .def_property_readonly("num_buckets", &dpt::Reducer::num_buckets)
      .def_property_readonly("backward_count", &dpt::Reducer::backward_count)
      .def("bucket_times_ms", &dpt::Reducer::bucket_times_ms, py::arg("slot") = -1)
      .def("step_times_ms", &dpt::Reducer::step_times_ms, py::arg("slot") = -1)
      .def("bucket_start_ms", &dpt::Reducer::bucket_start_ms, py::arg("slot") = -1)
      .def("set_profile_slots", &dpt::Reducer::set_profile_slots, py::arg("n"))
      .def_property_readonly("profile_slots", &dpt::Reducer::profile_slots)
      .def_property_readonly("last_slot", &dpt::Reducer::last_slot)
      .def("remove_hooks", &dpt::Reducer::remove_hooks);
}
