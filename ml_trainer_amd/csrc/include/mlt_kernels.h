// Host-visible launcher interface of the gfx950 kernels (csrc/kernels/*.hip).
// Pure HIP types only: the torch glue lives in csrc/bindings.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mlt_optim.h"

namespace mlt {

// ----------------------------------------------------------------------------
// Flat optimizers (optim.hip)
// ----------------------------------------------------------------------------
// lr = lr_ptr ? lr_ptr[lr_index_ptr ? (*lr_index_ptr - 1) : 0] : h.lr
// t  = step_ptr ? *step_ptr : t_host           (1-based step count)
void launch_flat_optim(float* p, const float* g, float* s1, float* s2, int64_t n, const OptHyper& h,
                       const float* lr_ptr, const int64_t* lr_index_ptr, const int64_t* step_ptr, float t_host,
                       uint16_t* shadow_bf16, const float* coef_ptr, hipStream_t stream,
                       const unsigned* skip = nullptr);  // skip: no update while *skip != 0
void launch_sq_norm(const float* x, int64_t n, float* out, hipStream_t stream);
void launch_clip_coef(const float* sq, float max_norm, float* coef, float* total_norm, hipStream_t stream);
void launch_cast_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t stream);
// dst[C][R] = src[R][C], bf16 (transpose.hip)
void launch_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, hipStream_t stream);

// ----------------------------------------------------------------------------
// LeNet-5 (reference src/model.py:7-24) fused forward/backward (lenet.hip)
// ----------------------------------------------------------------------------
enum LeNetCfg : int { LENET_DEFAULT = 0, LENET_TINY = 1 };
enum LeNetMode : int {
  LENET_FWD = 1,        // conv1 -> logits
  LENET_CE = 2,         // softmax-CE loss + dlogits + loss/accuracy accumulation
  LENET_BWD = 4,        // dlogits -> all parameter gradients
  LENET_OPT = 8,        // fused optimizer update inside the weight-gradient kernel (single process only)
  LENET_REDUCE = 16,    // (kept for API compatibility: the conv1 reduction always happens inside K5)
  LENET_TRACE = 256,    // fused kernel: block 0 stores per-phase clock64() stamps into slab1 (K5 skipped)
  LENET_SKIP_CONV1 = 512, LENET_SKIP_CONV2 = 1024, LENET_SKIP_FC = 2048,  // K5 roles skipped (profiling)
  LENET_K4WG = 4096,    // internal: K4 wrote the conv wgrad slabs, K5 only reduces them
  LENET_FROM_P1 = 8192, // internal: the per-sample kernel starts from p1 (conv2 -> fc chain) and stops there
  LENET_STATS_DEFER = 16384,  // internal: CE writes per-sample loss / hit to cestat; K4 sums them in sample order
  // timing probes of the bf16 per-sample kernel (wrong numerics: profiling only; env MLT_LENET_PROBE)
  LENET_PROBE_NOF1T = 1 << 17,  // role A skips the fc1 dgrad (transposed) weight fetch
  LENET_PROBE_NOF1W = 1 << 18,  // role B skips the fc1 forward weight fetch
  LENET_PROBE_NOF2 = 1 << 19,   // fc2 forward + dgrad weight fetches skipped
};

struct LeNetPtrs {
  const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4, *w5, *b5;  // params (fp32)
  float *gw1, *gb1, *gw2, *gb2, *gw3, *gb3, *gw4, *gb4, *gw5, *gb5;  // grads (fp32)
  float *x, *p1, *p2, *h1, *h2, *logits, *dlogits, *dh2, *dh1, *dflat, *g1, *slab1;
  uint8_t *i1, *i2;
  int64_t* targets;          // [B] class ids (written by conv1 in the augment path)
  const int64_t* dtargets;   // dataset targets [N] (augment path)
  double* stats;             // [2]: sum over batches of batch-mean loss, of batch accuracy
  unsigned* counters;        // [>= C1+1] zero-initialised arrival counters (K5 last-arriver reductions)
  uint8_t* stage;            // [B][3072] raw uint8 images of the next step (nullptr: no staging)
  int64_t* stage_meta;       // [B][4] (perm position, dataset row, target, 0) of each staged image; -1 = empty
  double* cestat;            // [B][2] per-sample (loss / B, hit / B) for the fixed-order stats sum (or nullptr)
  // bf16 MFMA engine (lenet_mfma.hip)
  uint8_t* stage2;           // [B][3072] raw uint8 images of the next step (staged by the per-sample kernel)
  int64_t* meta2;            // [B][4] (global step, perm position, dataset row, target) of each; -1 = empty
  int64_t* metaN;            // [B][4] (global step, perm position, perm entry, 0): lookup one step further
  int64_t* stepinfo;         // [4] (step, step in epoch, lr bits) of the running step, for the wgrad kernel
  uint16_t* shadow;          // bf16 copy of the flat fp32 parameters (fc weights are read from it)
  uint16_t* wimg;            // bf16 conv-weight MFMA fragment image (lenet_mfma_wimg_elems())
  float* trace;              // LENET_TRACE phase stamps (8-byte slots) or nullptr
  // next-step inputs prepared by the batch-reduction kernel's prep blocks (nullptr: off): the
  // augmented bf16 pixels [B][1024] x (c0, c1 | c2, 0) of the sample each block will compute next,
  // tagged pmeta[B][4] = (global step, perm position, target, 0); -1 = empty
  uint8_t* prep;
  int64_t* pmeta;
};

struct LeNetAug {
  const uint8_t* data;  // [N,32,32,3] HWC uint8; nullptr -> ptrs.x is the (normalised) input
  int64_t step_host, sie_host;  // used instead of ctrl[0], ctrl[1] when ctrl == nullptr
  const int32_t* perm;  // epoch sample order
  int64_t* ctrl;        // ctrl[0]: global step (1-based after the step), ctrl[1]: step in epoch
  int64_t n;            // dataset rows
  int64_t perm_len;
  uint64_t seed;
  int pad;              // RandomCrop padding (0 = no crop)
  int flip;             // RandomHorizontalFlip(p=0.5)
  int batch_stride;     // samples per step (offset into perm = ctrl[1]*batch_stride)
  float mean[3], std[3];
  float ascale[3], ashift[3];  // normalisation as one fma (bf16 engine): u * ascale + ashift
};

struct LeNetOpt {
  float *p, *g, *s1, *s2;  // whole flat buffers (params / grads / state)
  int64_t n;
  OptHyper h;
  const float* lr_ptr;     // device lr (table indexed by ctrl[1]-1 when lr_table)
  int lr_table;
  // flat-buffer offsets of the 10 LeNet tensors (w1,b1,w2,b2,w3,b3,w4,b4,w5,b5)
  int64_t off[10];
};

void launch_lenet(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                  hipStream_t stream);
// BERT classifier head (head.hip): classifier layer of num_labels outputs on the VALU
void launch_head_cls_fwd(const float* pooled, int B, int h, const float* wc, const float* bc, int L, float* logits,
                         hipStream_t st);
void launch_head_cls_bwd(const float* dlogits, const float* pooled, const float* wc, int B, int h, int L,
                         uint16_t* dpre, float* dwc, float* dbc, bool accumulate, hipStream_t st);
// bf16 MFMA training step (lenet_mfma.hip): 2 launches per step (per-sample chain + batch
// reductions / optimizer). Needs stage2 / meta2 / stepinfo / shadow, and slab1 >= B * slab floats.
void launch_lenet_mfma(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                       hipStream_t stream);
int lenet_mfma_slab_floats(int cfg);
int lenet_mfma_kw_blocks(int cfg);  // grid of the batch-reduction / optimizer kernel
// data-parallel bf16 step: optimizer update from the all-reduced gradient + bf16 shadow + fragment
// images in one launch (skip: nonzero vetoes the update)
void launch_lenet_mfma_apply(int cfg, const LeNetPtrs& P, const LeNetOpt& O, const unsigned* skip, hipStream_t stream);
// data-parallel bf16 step in TWO launches (as at W = 1): the per-sample kernel, then the batch
// reductions + xGMI exchange + rank-ordered sum + update of every gradient element in one launch
// (struct XgmiFused; throws if X.G < lenet_mfma_kw_blocks(cfg) or X.W outside 1..8)
struct XgmiFused;
void launch_lenet_mfma_dp(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                          const XgmiFused& X, hipStream_t stream);
int lenet_mfma_wimg_elems();
bool lenet_mfma_trace_build();  // LENET_TRACE stamps compiled in (MLT_LENET_TRACE_BUILD)
// batch reductions (+ the exchange when X) into O.g only, no update (transport self-test / timing)
void launch_lenet_mfma_reduce(int cfg, int B, const LeNetPtrs& P, const LeNetOpt& O, const XgmiFused* X,
                              hipStream_t stream);
int64_t lenet_mfma_xch_granules(int cfg);  // granules per parity the fused exchange needs
// shadow + wimg from the fp32 masters (O.p)
void launch_lenet_mfma_pack(int cfg, const LeNetPtrs& P, const LeNetOpt& O, hipStream_t stream);
void set_lenet_variant(int v);  // 0 default (4 launches), 1 fully fused per-sample chain, 2 split conv2 / fc
int get_lenet_variant();

// Standalone GPU augmentation (RandomCrop(32,pad) + HFlip + ToTensor + Normalize) for the
// generic (non-LeNet) device data path: out [B,3,32,32] fp32.
void launch_cifar_augment(const LeNetAug& A, int B, float* out, int64_t* targets_out, const int64_t* dtargets,
                          hipStream_t stream);

// ----------------------------------------------------------------------------
// Losses / metrics (losses.hip)
// ----------------------------------------------------------------------------
// acc[2] (zeroed by caller): {sum of row losses, number of valid rows}; loss[0] = mean.
void launch_ce_fwd(const void* logits, bool bf16, const int64_t* tgt, int64_t B, int C, float* dl, float* acc,
                   float* correct, float* loss, int64_t ignore_index, float label_smoothing, hipStream_t st);
void launch_ce_bwd(const float* dl, const float* gout, const float* acc, int64_t n, void* out, bool bf16,
                   hipStream_t st);
void launch_accuracy(const void* logits, bool bf16, const int64_t* tgt, int64_t B, int C, float* out,
                     hipStream_t st);
// Regression / NLL criteria and mcrmse (fp32). `part` holds loss_partials_needed() floats;
// out/stats[2] = {mean loss, denominator}; g is the unscaled elementwise gradient.
int loss_partials_needed();
void launch_pointwise_loss_fwd(const float* p, const float* t, int64_t n, int mode, float* g, float* part,
                               float* out, hipStream_t st);
void launch_nll_fwd(const float* logp, const int64_t* tgt, int64_t B, int C, int64_t ignore_index, float* part,
                    float* out, hipStream_t st);
void launch_loss_scale_grad(const float* g, const float* gout, const float* stats, int64_t n, float* out,
                            hipStream_t st);
void launch_nll_bwd(const int64_t* tgt, int64_t B, int C, int64_t ignore_index, const float* gout,
                    const float* stats, float* out, hipStream_t st);
void launch_mcrmse(const float* p, const float* t, int64_t B, int C, float* col, float* out, hipStream_t st);

// ----------------------------------------------------------------------------
// bf16 MFMA GEMM (gemm.hip): C[M,N] = alpha * op(A) . op(B) (+bias) (+epilogue)
//   a_mn: A stored [K][M] (else [M][K]);  b_mn: B stored [K][N] (else [N][K])
//   mode: 0 none, 1 GELU (pre-activation written to aux), 2 dGELU (multiply by gelu'(aux))
// ----------------------------------------------------------------------------
// Kernel choice per shape: cfg 0 = 128x128 register-staged kernel (any K % 8 == 0), cfg 1..4 =
// 256x256 / 256x128 / 128x256 / 256x192 global_load_lds kernels (K % 64 == 0) with split-K
// (deterministic in-launch slab reduction; needs ws_floats of fp32 workspace from the caller;
// tile counters come from an internal self-resetting pool when cnt == nullptr).
struct GemmPlan {
  int cfg;
  int splits;
  int ksteps;  // K-steps (of 64) per split
  int64_t ws_floats;
  int64_t cnt_ints;
  int ext = 0;  // split-K partials summed by a separate grid-wide reduce launch (else: last-arriver in-kernel)
};
GemmPlan plan_gemm_bf16(int a_mn, int b_mn, int M, int N, int K, int force_cfg, int force_splits,
                        int accumulate = 0);
void set_gemm_split_mode(int mode);  // -1 planner, 0 in-kernel last-arriver, 1 external reduce
void set_gemm_w4q8(int on);          // gemm_f8_q GELU: 1 4-wave kernel, 0 ping-pong, -1 env
void launch_gemm_bf16(const GemmPlan& plan, int a_mn, int b_mn, bool out_f32, const uint16_t* A, const uint16_t* B,
                      void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const float* bias,
                      const uint16_t* aux, int64_t ldaux, const uint16_t* res, int64_t ldres, float alpha, int mode,
                      int accumulate, float* ws, unsigned* cnt, hipStream_t st, float* colpart = nullptr);
// fp8 GEMM (gemm_tile.hip): A [M][K], B [N][K] both k-contiguous fp8 (fmt 0 = e4m3, 1 = e5m2),
// K % 128 == 0; alpha *= inv_scale_a[0] * inv_scale_b[0] (device scalars, delayed scaling).
GemmPlan plan_gemm_f8(int M, int N, int K, int force_cfg, int force_splits);
void launch_gemm_f8(const GemmPlan& plan, int fmt_a, int fmt_b, bool out_f32, const uint8_t* A, const uint8_t* B,
                    void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const float* inv_scale_a,
                    const float* inv_scale_b, const float* bias, const uint16_t* aux, int64_t ldaux,
                    const uint16_t* res, int64_t ldres, float alpha, int mode, int accumulate, float* ws,
                    unsigned* cnt, hipStream_t st);
// fp8 GEMM with a quantising epilogue (gemm_pp_kernel, OutT = uint8_t): Y = fp8(act(A.B^T*ia*ib
// + bias) * out_scale) [M,N] and Y^T [N,M] (mode 0 none, 1 GELU writing the bf16 pre-activation
// to aux, 2 dGELU reading it), amax of act(..) into out_amax, optional [M/64, N] column partials.
// M % 256 == 0, N % 256 == 0, K % 128 == 0; fmt_a e4m3 or e5m2, fmt_b e4m3.
void launch_gemm_f8_q(int fmt_a, int fmt_b, const uint8_t* A, const uint8_t* B, uint8_t* Y, uint8_t* Yt, int M, int N,
                      int K, int64_t lda, int64_t ldb, int64_t ldy, int64_t ldyt, const float* inv_scale_a,
                      const float* inv_scale_b, const float* bias, const uint16_t* aux, int64_t ldaux, int mode,
                      int out_fmt, const float* out_scale, float* out_amax, float* colpart, hipStream_t st);
// fp8 quantisation (fp8.hip); every amax argument points at kAmaxSlots slots spaced
// kAmaxStride floats apart (kAmaxSlots * kAmaxStride floats per tensor)
constexpr int kAmaxSlots = 64, kAmaxStride = 32;
void launch_cast_fp8(const void* x, bool x_f32, uint8_t* y, int64_t n, const float* scale, float* amax, int fmt,
                     hipStream_t st);
void launch_amax(const void* x, bool x_f32, int64_t n, float* amax, hipStream_t st);
void launch_cast_transpose_fp8(const float* w, uint8_t* y, uint8_t* yt, int R, int C, const float* scale, float* amax,
                               int fmt, hipStream_t st);
bool cast_transpose_fp8_wide_ok(const void* x, const void* y, const void* yt, int R, int C);
void launch_cast_transpose_fp8_bf16(const uint16_t* x, uint8_t* y, uint8_t* yt, int R, int C, const float* scale,
                                    float* amax, int fmt, hipStream_t st, float* colpart = nullptr);
void launch_fp8_update_scale(float* hist, int H, int n, float* amax, float* scale, float* inv_scale, const float* fmax,
                             int margin, int64_t step, hipStream_t st);

// one-shot xGMI all-reduce (allreduce.hip): peer region pointers indexed by rank
constexpr int kXgmiMaxRanks = 8;
struct XgmiPeers {
  float* data[kXgmiMaxRanks];
  uint64_t* flags[kXgmiMaxRanks];
  // two-shot (reduce-scatter + all-gather by remote pushes): per-rank [2][W][slot] staging of the
  // scattered slices (t1) and of the reduced slices (t2), each with its own [2][G][W] flags
  float* t1[kXgmiMaxRanks];
  float* t2[kXgmiMaxRanks];
  uint64_t* f1[kXgmiMaxRanks];
  uint64_t* f2[kXgmiMaxRanks];
};
// optional fused flat-optimizer update of the reduced slice (same semantics as
// launch_flat_optim with lr / step from device memory)
struct XgmiPostOpt {
  float *p, *s1, *s2;
  OptHyper h;
  const float* lr_ptr;
  const int64_t* lr_index_ptr;
  const int64_t* step_ptr;
};
// fault (tests only): 1 = this rank never publishes the slices b with b % (2 W) == rank, so on every
// rank those slices time out while the others reduce (the "late / partial peer" case)
void launch_xgmi_allreduce(float* grad, int64_t n, const XgmiPeers& P, int rank, int W, int64_t cap, int blocks,
                           uint64_t* seqs, float scale, unsigned* err, long long timeout_ticks,
                           const XgmiPostOpt* post, hipStream_t st, int fault = 0);
// The fused bf16 LeNet data-parallel step's view of the transport (lenet_mfma.hip, lenet_mwx):
// every gradient element the batch-reduction kernel produces is published as an 8-byte granule
// {fp32 value, low 32 bits of the block's launch counter} into its rank's granule array (parity
// p = seq & 1), written and read with single 8-byte system-scope accesses; a consumer lane polls the
// W - 1 peers' granules of ITS elements until their tags match, sums in rank order and applies the
// update in the same launch -- no flags, no barriers, one round trip. W = 1 is the loopback.
struct XgmiFused {
  uint64_t* gran[kXgmiMaxRanks];   // per-rank [2][cap] granules (indexed by flat parameter offset),
                                   // followed (gran + 2 cap) by the two-phase exchange's [2][cap] granules
                                   // of the REDUCED values of the 64-granule chunks the rank owns
                                   // (chunk c: rank c % W)
  uint64_t* seqs;                  // [G] per-block launch counters (this rank)
  unsigned* err;                   // sticky error word (host-mapped: the host polls it)
  unsigned* derr;                  // its device copy (what the kernel reads)
  int64_t cap;
  long long timeout;               // ticks of the 100 MHz constant clock
  int rank, W, G, fault;
  int two;                         // 1: two-phase exchange (reduce-scatter into owners, owners publish)
};
// two-shot variant: slot = floats per [rank] slot of t1 / t2 (>= ceil(n / W) rounded up to 4)
void launch_xgmi_allreduce_2shot(float* grad, int64_t n, const XgmiPeers& P, int rank, int W, int64_t slot,
                                 int blocks, uint64_t* seqs, float scale, unsigned* err, long long timeout_ticks,
                                 const XgmiPostOpt* post, hipStream_t st, int fault = 0);

int64_t colsum_ws_floats(int M, int N);
void launch_colsum_bf16(const uint16_t* X, int M, int N, int64_t ldx, float* out, int accumulate, float* ws,
                        hipStream_t st);
// out_k[c] (+)= sum_r part[r * ld + k * seg + c], c < W, k = 0..W/seg-1 (<= 3 segments; bit k of accmask =
// accumulate into out_k); fixed-order (deterministic)
struct SegOut {
  float* p[3];
};
void launch_reduce_rows(const float* part, int R, int64_t ld, int W, int seg, SegOut outs, int accmask, hipStream_t st);

// ----------------------------------------------------------------------------
// LayerNorm / embeddings (layernorm.hip), attention (attention.hip)
// ----------------------------------------------------------------------------
void launch_ln_fwd(const uint16_t* X, const float* gamma, const float* beta, uint16_t* Y, float* mean, float* rstd,
                   int64_t rows, int D, float eps, hipStream_t st);
int ln_bwd_partial_blocks(int64_t rows);
void launch_ln_bwd(const uint16_t* DY, const uint16_t* X, const float* gamma, const float* mean, const float* rstd,
                   uint16_t* DX, float* part, float* dgamma, float* dbeta, int64_t rows, int D, int accumulate,
                   const uint16_t* DRES, float* dxsum, int dxsum_acc, hipStream_t st);
// LayerNorm backward that also quantises dx (the next fp8 GEMM's dY): e5m2 Y8 [rows, D] + YT8
// [D, rows] with scale *qscale, amax into qamax's slots; dxsum required. false: shape not covered
int ln_bwd_q8_partial_blocks(int64_t rows);
bool launch_ln_bwd_q8(const uint16_t* DY, const uint16_t* X, const float* gamma, const float* mean, const float* rstd,
                      uint16_t* DX, float* part, float* dgamma, float* dbeta, int64_t rows, int D, int accumulate,
                      float* dxsum, int dxsum_acc, uint8_t* Y8, uint8_t* YT8, const float* qscale, float* qamax,
                      hipStream_t st);
void launch_embed_fwd(const int64_t* ids, const int64_t* tt, const uint16_t* Ww, const uint16_t* Wp,
                      const uint16_t* Wt, uint16_t* out, int64_t rows, int S, int D, int64_t vocab, int ntype,
                      hipStream_t st);
// sid / perm: the token ids sorted stably and the sorting permutation (deterministic, atomic-free
// word-table scatter); part: S x 2D floats of per-position token-type partial sums
void launch_embed_bwd(const int64_t* sid, const int64_t* perm, const int64_t* tt, const uint16_t* DX, float* gw,
                      float* gp, float* gt, float* part, int64_t rows, int S, int D, int64_t vocab, int ntype,
                      hipStream_t st);
void launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, const int* lens, int B, int S, int H,
                     float scale, hipStream_t st);
// colpart_q [B * ceil(S/64)][D] and colpart_kv [B * ceil(S/64)][2D] (or nullptr): bias-gradient
// column partials of dQ and dK|dV; returns whether they were written (ring kernels) and the
// number of partial rows in rows_q / rows_kv
// q8 (fp8 training, y != nullptr): instead of the bf16 dQKV, the backward kernels write its e5m2
// copy y [B*S][3D] and transpose yt [3D][B*S] -- each value the bf16 one rounded first, then scaled
// by *scale and quantised exactly as fp8_cast_transpose would -- and record amax(|dQKV|) into the
// kAmaxSlots sub-slots at amax (the ring kernels only; S % 16 == 0)
struct AttnQ8 {
  uint8_t* y = nullptr;
  uint8_t* yt = nullptr;
  const float* scale = nullptr;
  float* amax = nullptr;
  int64_t ldt = 0;  // yt row stride (B * S)
};
bool launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, float* delta,
                     const int* lens, uint16_t* dqkv, int B, int S, int H, float scale, hipStream_t st,
                     float* colpart_q = nullptr, float* colpart_kv = nullptr, int* rows_q = nullptr,
                     int* rows_kv = nullptr, const AttnQ8& q8 = AttnQ8{});

}  // namespace mlt
