// Host-side launchers of the gfx950 kernel library.  Raw pointers + hipStream_t only: the
// .hip translation units never include torch headers (bindings.cpp does the tensor checks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpt {

struct AugNorm {
  float mean[4];
  float inv_std[4];
};

// optim_kernels.hip
void launch_grad_check(const float* g, int64_t n, const float* scale, float host_factor,
                       float* found_inf, hipStream_t s);
// shadow (optional): a 16-bit copy of the updated parameters (bf16: kind 1, fp16: kind 2)
// written in the same pass - the weights the convolutions read under autocast.
void launch_sgd(float* p, float* g, float* buf, int64_t n, float lr, float momentum,
                float dampening, float wd, bool nesterov, const float* scale, float host_factor,
                const float* found_inf, const float* step, bool zero_grad, uint16_t* shadow,
                int shadow_kind, hipStream_t s);
void launch_adam(float* p, float* g, float* m, float* v, int64_t n, double lr, double beta1,
                 double beta2, double eps, double wd, bool adamw, const float* scale, float host_factor,
                 const float* found_inf, const float* step, bool zero_grad, uint16_t* shadow,
                 int shadow_kind, hipStream_t s);
void launch_optim_tail(float* scale, int* growth_tracker, float* found_inf, float* step,
                       float growth_factor, float backoff_factor, int growth_interval,
                       hipStream_t s);

// comm_kernels.hip
void launch_pack_bf16(const float* src, uint16_t* dst, int64_t n, hipStream_t s);
void launch_unpack_bf16(const uint16_t* src, float* dst, int64_t n, const float* scale,
                        float host_factor, float* found_inf, hipStream_t s);
// test-only: a 1-wave kernel that busy-waits `ms` milliseconds of wall clock
void launch_spin(double ms, hipStream_t s);

// metrics_kernels.hip  (dtype: 0 f32, 1 bf16, 2 f16)
void launch_metrics(const void* logits, int dtype, int64_t rows, int64_t cols, int64_t ld,
                    const int64_t* targets, const float* loss, double* acc, hipStream_t s);

// augment_kernels.hip
void launch_augment(const uint8_t* data, const int64_t* idx, const int32_t* offs,
                    const uint8_t* flips, void* out, bool out_bf16, bool nhwc, int64_t B, int C,
                    int H, int W, int pad, AugNorm norm, hipStream_t s);

// bn_kernels.hip  (dtype: 0 f32, 1 bf16, 2 f16; activations channels_last = row-major [M, C])
struct BnGeometry {
  int64_t rows_per_chunk;
  int chunks;
  int apply_blocks;
};
bool bn_supported(int64_t C);
BnGeometry bn_geometry(int64_t M, int64_t C);
int64_t bn_workspace_floats(int64_t M, int64_t C);
void launch_bn_fwd_train(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                         const float* gamma, const float* beta, float eps, float momentum, float* run_mean,
                         float* run_var, int64_t* num_batches, float* save_mean, float* save_invstd,
                         float* save_coef, float* workspace, bool relu, hipStream_t s, uint8_t* mask = nullptr);
// mask (relu + residual only, else ignored): also write the 1-bit ReLU mask of y, [M][C/8] bytes,
// bit k of byte (m, g) = y[m, 8g + k] > 0 after rounding to y's dtype
void launch_bn_fwd_from_partials(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                                 const float* psum, const float* psq, int chunks, const float* gamma,
                                 const float* beta, float eps, float momentum, float* run_mean, float* run_var,
                                 int64_t* num_batches, float* save_mean, float* save_invstd, float* save_coef,
                                 bool relu, hipStream_t s, uint8_t* mask = nullptr);
void launch_bn_bwd_from_partials(int dtype, const void* dy, const void* x, int64_t M, int64_t C, const float* gamma,
                                 const float* mean, const float* invstd, const float* coef, const float* p1,
                                 const float* p2, int chunks, float* dgamma, float* dbeta, void* dx, float* kbuf,
                                 hipStream_t s, bool from_dz = false);
// y = relu(x*a + b + x2*a2 + b2) (block tail with its downsample BatchNorm folded in)
void launch_bn_apply_aff(int dtype, const void* x, const void* x2, void* y, int64_t M, int64_t C, const float* a,
                         const float* b, const float* a2, const float* b2, hipStream_t s, uint8_t* mask = nullptr);
// backward of that: finalize both BNs from dgrad-epilogue partials (p1 shared), one apply pass
// writing dx and dx2; kbuf: 6C floats
void launch_bn2_bwd_from_partials(int dtype, const void* dz, const void* x, const void* x2, int64_t M, int64_t C,
                                  const float* gamma, const float* mean, const float* invstd, const float* gamma2,
                                  const float* mean2, const float* invstd2, const float* p1, const float* p2,
                                  const float* p3, int chunks, float* dgamma, float* dbeta, float* dgamma2,
                                  float* dbeta2, void* dx, void* dx2, float* kbuf, hipStream_t s);
void bn_set_skip_finalize(int on);  // measurement only (bench/ab_step.py): skip BN finalize launches
void launch_bn_apply(int dtype, const void* x, const void* res, void* y, int64_t M, int64_t C,
                     const float* coef_a, const float* coef_b, bool relu, hipStream_t s);
void launch_bn_bwd(int dtype, const void* dy, const void* dy2, const void* y, const void* x, int64_t M,
                   int64_t C, const float* gamma, const float* mean, const float* invstd, const float* coef,
                   float* dgamma, float* dbeta, void* dx, void* dz, float* workspace, bool relu, hipStream_t s);

// pool_kernels.hip  (channels_last [B,H,W,C], C % 8 == 0; idx = window-local uint8 argmax)
// coef (optional, 3x3 windows): [a | b] of a BatchNorm+ReLU folded into the pool's loads
void launch_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* idx, int64_t B, int H, int W, int C, int Ho,
                        int Wo, int K, int S, int P, hipStream_t s, const float* coef = nullptr);
// global-average-pool backward: dx [N, HW, C] (dtype) = g [N, C] (gdtype) / HW
void launch_gap_bwd(int dtype, int gdtype, const void* g, void* dx, int64_t N, int64_t HW, int64_t C, hipStream_t s);
// gap_bwd of a block-tail output y (mask) whose BN input is x: dz = g/HW * (y > 0) and that BN's
// backward statistics partials p1/p2 [C][gap_bwd_bnr_chunks(N*HW, C)]; C/8 must divide 256.
int gap_bwd_bnr_chunks(int64_t M, int64_t C);
void launch_gap_bwd_bnr(int dtype, int gdtype, const void* g, void* dz, const void* y, const void* x,
                        const float* mean, int64_t N, int64_t HW, int64_t C, float* p1, float* p2, hipStream_t s);
// dy2: optional second output gradient, summed in (pool output with two consumers)
// bnx/bn_mean/bn_coef (3x3/2/1 pools only): the input was relu(bn(bnx)); also write that BN's
// backward-statistics partials [C][maxpool_bwd_bn_chunks(...)] to bp1/bp2
void launch_maxpool_bwd(int dtype, const void* dy, const void* dy2, const uint8_t* idx, void* dx, int64_t B, int H,
                        int W, int C, int Ho, int Wo, int K, int S, int P, hipStream_t s, const void* bnx = nullptr,
                        const float* bn_mean = nullptr, const float* bn_coef = nullptr, float* bp1 = nullptr,
                        float* bp2 = nullptr);
int maxpool_bwd_bn_chunks(int64_t B, int H, int W, int C);

// gather_kernels.hip: up to kGatherMax tensors per launch (kernel-argument struct)
constexpr int kGatherMax = 48;
struct GatherBatch {
  const void* src[kGatherMax];
  float* dst[kGatherMax];
  int64_t numel[kGatherMax];
  int8_t kind[kGatherMax];  // source dtype: 0 f32, 1 bf16, 2 f16
  int count;
};
void launch_gather(const GatherBatch& batch, bool accumulate, hipStream_t s);

// vit_kernels.hip  (kind: 1 bf16, 2 fp16 for the 16-bit activations; param kinds 0 f32 / 1 bf16 /
// 2 fp16; rows are tokens, LayerNorm width D % 256 == 0, GELU width F % 8 == 0)
bool ln_supported(int64_t D);
int ln_bwd_blocks(int64_t T);
int gelu_bwd_chunks(int64_t T, int64_t F);
void vit_set_gelu_blocks_per_cu(int n);  // A/B: 2-wave blocks per CU of the GELU passes (default 6)
void launch_ln_fwd(int kind, const float* x, const uint16_t* a, const void* bias, int bias_kind, const float* gamma,
                   const float* beta, float* s_out, uint16_t* h_out, float* mean, float* rstd, int64_t T, int64_t D,
                   float eps, hipStream_t s);
// part: 3 * ln_bwd_blocks(T) * D floats of scratch
void launch_ln_bwd(int kind, const float* gs, const uint16_t* gh, const float* sv, const float* mean,
                   const float* rstd, const float* gamma, float* gx, uint16_t* ga, float* part, float* dgamma,
                   float* dbeta, void* dbias, int dbias_kind, int64_t T, int64_t D, hipStream_t s);
void launch_gelu_fwd(int kind, const uint16_t* u, const void* bias, int bias_kind, uint16_t* h, int64_t T, int64_t F,
                     hipStream_t s);
// part: gelu_bwd_chunks(T, F) * F floats of scratch
void launch_gelu_bwd(int kind, const uint16_t* gh, const uint16_t* u, const void* bias, int bias_kind, uint16_t* gu,
                     float* part, void* dbias, int dbias_kind, int64_t T, int64_t F, hipStream_t s);
// dbias = column sums of gy [T, F] (F % 8 == 0); part: gelu_bwd_chunks(T, F) * F floats
void launch_bias_grad16(int kind, const uint16_t* gy, float* part, void* dbias, int dbias_kind, int64_t T, int64_t F,
                        hipStream_t s);
// out[i] = sum over S of part[s][i], n % 4 == 0; out kind 0 f32 / 1 bf16 / 2 f16
void launch_sum_partials(const float* part, int64_t n, int S, void* out, int out_kind, hipStream_t s);
// out[c] = sum_r part[r][c] over an [n][D] fp32 array (fp64 accumulation, fixed order), out of kind
// 0 f32 / 1 bf16 / 2 f16: many short rows (sum_partials walks S serially per column)
void launch_colsum_rows(const float* part, int64_t n, int64_t D, void* out, int out_kind, hipStream_t s);
// dst[i0..i3, :L] = src[i0..i3, :L] (16-bit elements, strides in elements, L % 8 == 0, rows 16-B aligned)
void launch_rows_copy16(const uint16_t* src, uint16_t* dst, const int n[4], const int64_t ss[4], const int64_t ds[4],
                        int L, hipStream_t s);

// conv_kernels.hip: channels_last bf16 implicit-GEMM convolutions (MFMA).  x [N,H,W,C],
// w [Cout,R,S,C], y [N,Ho,Wo,Cout]; C % 64 == 0, Cout % 64 == 0.  psum/psq (optional): BN
// partial sums of y per (channel, M-tile), layout [Cout][conv_m_tiles(M)].
bool conv_supported(int C, int Cout);
bool conv_supported_narrow(int C, int Cout, int S);  // C = 16/32 with S % (64/C) == 0 (fwd, wgrad)
int conv_m_tiles(int64_t M);
void conv_set_variant(int v);
void conv_set_big(int on);  // 8-wave 256-row tiles where conv_big_auto picks them (default off)
void conv_set_wgrad_stages(int mode);  // backward-weight 2-stage K loop: 1 = one-wave grids, 2 = all (A/B)
void conv_set_breg(int mode);  // B operand in VGPRs: bit 0 HALO 3x3, bit 1 other convs (A/B)
int conv_get_breg();
void conv_set_halo(int on);  // 3x3 / stride-1 halo K loop (default on, DPT_CONV_HALO)
// stream-K conv_fwd_kernel grids (0 off, 1 auto below the per-CU balance eff, 2 every eligible
// grid; eff <= 0 keeps the threshold), workspace preallocation, and the bounded-spin give-up count
// Linear backward-data with the exact-GELU backward fused (conv_fwd_kernel DGELU epilogue):
// gu = (dy wt^T) * gelu'(u + bias), bp1 [linear_dgrad_dgelu_tiles(T)][n_in] column-sum partials;
// the bias is fp32 (bias) or the operands' 16-bit type (bias16, used when non-null)
void launch_linear_dgrad_dgelu(const uint16_t* dy, const uint16_t* wt, const uint16_t* u, const float* bias,
                               const uint16_t* bias16, uint16_t* gu, float* bp1, int64_t T, int n_out, int n_in,
                               bool f16, hipStream_t s);
int linear_dgrad_dgelu_tiles(int64_t T);
void conv_set_streamk(int mode, double eff);
int conv_get_streamk();
void conv_sk_prepare();
unsigned conv_sk_errors();
int conv_sk_blocks(int64_t tiles, int nk, int bn, int mode);
void conv_set_wgrad_target(int blocks);  // split-K backward-weight block target (0 = policy)
// Ho/Wo > 0: explicit output size (padding applied on top/left only beyond what it needs)
// ws: split-K workspace of conv_fwd_splits(M, Cout, R*S*C) * M * Cout floats when that is > 1
// (nullptr: never split).  Small tile grids split the K loop over blocks (fp32 partials).
// (s: the launch stream - inside a hipGraph capture small grids always split, eagerly only
// the very latency-bound ones); split-K writes BN partials with conv_split_cols(M) columns
int conv_fwd_splits(int64_t M, int Cout, int64_t K, int* kps = nullptr, hipStream_t s = nullptr);
int conv_fwd_splits_for(int64_t M, int Cout, int64_t K, bool graph, int* kps = nullptr);
int conv_split_cols(int64_t M);
void conv_set_splitk_policy(int tiles, int eager_tiles, int eager_min_k, int target);  // A/B knob
void conv_set_splitk(int mode);  // 0 off / 1 auto (default, DPT_CONV_SPLITK) / 2 in-graph policy always
int conv_get_splitk();
void conv_set_fwd_shape_policy(int bits);  // per-shape forward tiles (conv_kernels.hip)
void launch_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int C, int Cout,
                     int R, int S, int stride, int pad, float* psum, float* psq, hipStream_t s, int Ho = 0,
                     int Wo = 0, bool f16 = false, float* ws = nullptr);
// f16: fp16 operands/outputs throughout (bf16 otherwise) - every conv launcher below takes it.
// backward-weight: dw [Cout,R,S,C] (kind 0 f32 / 1 bf16 / 2 f16) = sum over pixels of dy x x-shifted;
// part: plan.part_floats floats of split-K scratch.  C % 64 == 0, Cout % 64 == 0.
struct ConvWgradPlan {
  int Ho, Wo, bmw, bnw, splits, steps_per_split;
  int64_t part_floats;
  int halo = 0;  // 3x3 / stride-1: the three taps of a tap row share one x strip (conv_wgrad_halo_kernel)
};
void conv_set_wgrad_halo(int mode);  // 0 off, 1-4 forced, 5 auto (default, DPT_WGRAD_HALO)
// target_blocks > 0: the split-K block target for this call (ViT's long-K linears want 768,
// profiles/vit_wgrad_ab_r5.md); 0: the shape policy (wgrad_target) or conv_set_wgrad_target
ConvWgradPlan conv_wgrad_plan(int N, int H, int W, int C, int Cout, int R, int S, int stride, int pad, int Ho = 0,
                              int Wo = 0, int target_blocks = 0);
// The split-K reduce of a backward-weight (partials [splits][n4 float4s] -> out, kind as dw_kind).
struct WgradReduce {
  const float* part;
  void* out;
  int64_t n4;
  int splits, kind;
  bool consumed;
};
void launch_wgrad_reduce(const WgradReduce& r, hipStream_t s);
// defer != nullptr: the reduce is not launched but described in *defer (consumed = false) when
// the plan needs one, for a conv backward-data launch to run in its tail (AttachWgradReduce).
void launch_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* part, void* dw, int dw_kind, int N, int H,
                       int W, int C, int Cout, int R, int S, int stride, int pad, const ConvWgradPlan& plan,
                       hipStream_t s, bool f16 = false, WgradReduce* defer = nullptr);
// BatchNorm backward apply with precomputed kbuf (a finalize run before it):
// dx = k1*dz + k2*(x - mean) + k3, dz = dy * relu-mask(fma(x, coef_a, coef_b) > 0), or dz = dy
// when from_dz.  Takes an attached backward-weight reduce into its grid (AttachWgradReduce).
void launch_bn_bwd_apply_pre(int dtype, const void* dy, const void* x, int64_t M, int64_t C, const float* mean,
                             const float* coef, const float* kbuf, void* dx, hipStream_t s, bool from_dz);
struct ReduceCarry;
// The reduce attached by a live AttachWgradReduce (if any) is described in rc and marked
// consumed; returns the carry blocks to append to the launching kernel's grid (0: none).
int take_attached_reduce(ReduceCarry& rc);
// Scoped hand-over of a deferred backward-weight reduce (host thread-local, one binding call):
// while the guard lives, the next 256-thread conv_fwd_kernel launch on this thread (forward,
// backward-data, split-K main kernel) appends the reduce's blocks to its grid and marks it
// consumed; the destructor launches it standalone on `s` if nothing did.  Saves the reduce's
// own launch and ramp (53 per ResNet-50 step): its blocks fill the conv's tail.
class AttachWgradReduce {
 public:
  AttachWgradReduce(WgradReduce* r, hipStream_t s);
  ~AttachWgradReduce();
  AttachWgradReduce(const AttachWgradReduce&) = delete;
  AttachWgradReduce& operator=(const AttachWgradReduce&) = delete;

 private:
  WgradReduce* r_;
  hipStream_t s_;
};
// stride-1 backward-data (flipped weight wt [C,R,S,Cout]) + the backward statistics of the
// BatchNorm+ReLU (input bnx, mean, coef [a|b]) that produced the conv's input: bp1/bp2 [C][m_tiles]
void launch_conv_dgrad_bnstats(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, int N, int Ho, int Wo, int Cout,
                               int C, int R, int S, int pad, const uint16_t* bnx, const float* bn_mean,
                               const float* bn_coef, float* bp1, float* bp2, hipStream_t s,
                               const uint16_t* bny = nullptr, const uint16_t* bnres = nullptr,
                               const uint16_t* bnx2 = nullptr, const float* bn_mean2 = nullptr,
                               float* bp3 = nullptr, bool f16 = false, float* ws = nullptr,
                               const uint8_t* bnmask = nullptr);
// many weights flipped/transposed (wt[ci][R-1-r][S-1-s][co] = w[co][r][s][ci]) in one launch
constexpr int kWtFlipMax = 64;
struct WtFlipBatch {
  const uint16_t* w[kWtFlipMax];
  uint16_t* wt[kWtFlipMax];
  int Cout[kWtFlipMax], R[kWtFlipMax], S[kWtFlipMax], C[kWtFlipMax];
  int blk0[kWtFlipMax];
  int count;
};
void launch_conv_wt_flip_multi(WtFlipBatch b, hipStream_t s);
// stride-2 backward-data straight from the KRSC weight w [Cout,R,S,C]: dy [N,Ho,Wo,Cout] -> dx [N,H,W,C]
struct ConvS2Plan {
  int chunks;          // BN-partial columns over all parity classes
  int64_t ws_floats;   // split-K workspace (0: no class splits)
};
ConvS2Plan conv_dgrad_s2_plan(int N, int H, int W, int C, int Cout, int R, int S, int pad, hipStream_t s);
void launch_conv_dgrad_s2(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int N, int Ho, int Wo, int Cout,
                          int C, int R, int S, int pad, int H, int W, hipStream_t s, const uint16_t* bnx = nullptr,
                          const float* bn_mean = nullptr, const float* bn_coef = nullptr, float* bp1 = nullptr,
                          float* bp2 = nullptr, bool f16 = false, float* ws = nullptr);
// [C][chunks] partial columns the BN-statistics variant of launch_conv_dgrad_s2 writes
int conv_dgrad_s2_chunks(int N, int H, int W, int R, int S, int pad);
// stride-1 backward-data straight from the KRSC weight w [Cout,R,S,C]: dy [N,Ho,Wo,Cout] -> dx [N,Ho,Wo,C]
void launch_conv_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int N, int Ho, int Wo, int Cout, int C,
                       int R, int S, int pad, hipStream_t s, bool f16 = false);
// space-to-depth stem input: x [N,H,W,C] fp32/bf16 (channels_last, H, W even, C <= 4) ->
// a [N, H/2, W/2, 16] bf16 with channel (a*2 + b)*4 + c = x[2i + a][2j + b][c] (zero for c >= C)
void launch_space_to_depth2(const void* x, bool x_bf16, uint16_t* a, int N, int H, int W, int C, hipStream_t s,
                            bool out_f16 = false);
// im2col for narrow-input convs: a [N*Ho*Wo, Kp] bf16 (k = (r*S+s)*C + c, zero past R*S*C)
void launch_im2col(const void* x, bool x_bf16, uint16_t* a, int N, int H, int W, int C, int R, int S, int stride,
                   int pad, int Kp, hipStream_t s);
// wt[ci, r, s, co] = w[co, R-1-r, S-1-s, ci]
void launch_conv_wt_flip(const uint16_t* w, uint16_t* wt, int Cout, int R, int S, int C, hipStream_t s);

// attn_kernels.hip: fused self-attention for short sequences (S <= 256, head dim 64).
// qkv [B, S, 3, H, 64] bf16 (the QKV projection output), ctx/out/dout [B, S, H*64] bf16,
// lse2 [B*H][attn_lse_stride(S)] fp32 (log2-sum-exp of the scaled scores), dqkv like qkv.
bool attn_supported(int S, int Dh);
int attn_lse_stride(int S);
void attn_set_bwd_split(int on);  // attention backward as two phase kernels (A/B)
void launch_attn_fwd(const uint16_t* qkv, uint16_t* ctx, float* lse2, int B, int S, int H, float scale,
                     hipStream_t s);
void launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse2,
                     uint16_t* dqkv, int B, int S, int H, float scale, hipStream_t s);

// conv_f32_kernels.hip: channels_last fp32 convolutions on v_mfma_f32_32x32x2_f32 (exact fp32,
// deterministic split-K).  dgrad = true: a is dy [N,Ho,Wo,Co], b the transposed weight
// [C][R][S][Co], out dx [N,H,W,C]; otherwise a is x, b the weight [Co][R][S][C], out y.
// ws: conv_f32_workspace(...) floats when that is > 0 (split-K partial tiles).
int64_t conv_f32_workspace(int64_t M, int ncols, int K, int* splits = nullptr);
void launch_conv_f32(const float* a, const float* b, float* out, float* ws, bool dgrad, int N, int H, int W, int C,
                     int Ho, int Wo, int Co, int R, int S, int stride, int pad, hipStream_t st);
int64_t conv_f32_wgrad_workspace(int N, int Ho, int Wo, int Co, int J);
void launch_conv_f32_wgrad(const float* dy, const float* x, float* dw, float* ws, int N, int H, int W, int C,
                           int Ho, int Wo, int Co, int R, int S, int stride, int pad, hipStream_t st);
}  // namespace dpt
