// LeNet-5 bf16 MFMA training step -- host entry points (the kernels: lenet_mfma.inc). The one-launch
// step's per-world-size instantiations live in lenet_mfma_1l_w*.hip (parallel compilation).
#include "lenet_mfma.inc"

namespace mlt {

bool lenet_mfma_onelaunch_ok(int cfg, int B, int W) {
  const int U = cfg == LENET_TINY ? lm::upd_grid<lm::DmTiny>() : lm::upd_grid<lm::DmDefault>();
  return B >= 1 && U + B <= lm::kOneLaunchMaxGrid && lm::onelaunch_world(W);
}
void launch_lenet_mfma_onelaunch(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                                 unsigned long long* sync, const XgmiFused* X, hipStream_t stream) {
  if (B <= 0) return;
  switch (X ? X->W : 0) {
    case 0: lm::run1_w0(cfg, mode, B, P, A, O, sync, X, stream); break;
    case 1: lm::run1_w1(cfg, mode, B, P, A, O, sync, X, stream); break;
    case 2: lm::run1_w2(cfg, mode, B, P, A, O, sync, X, stream); break;
    case 4: lm::run1_w4(cfg, mode, B, P, A, O, sync, X, stream); break;
    case 8: lm::run1_w8(cfg, mode, B, P, A, O, sync, X, stream); break;
    default: throw std::runtime_error("lenet one-launch step: world size not in {1, 2, 4, 8}");
  }
}
void launch_lenet_mfma_flush(int cfg, int B, const LeNetPtrs& P, const LeNetOpt& O, const XgmiFused* X,
                             hipStream_t stream, bool opt) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::flush<lm::DmTiny>(B, P, O, X, stream, opt);
  else
    lm::flush<lm::DmDefault>(B, P, O, X, stream, opt);
}
int64_t lenet_mfma_xch_granules(int cfg) {
  return cfg == LENET_TINY ? lm::xch_granules<lm::DmTiny>() : lm::xch_granules<lm::DmDefault>();
}

void launch_lenet_mfma_dp(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                          const XgmiFused& X, hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::run_dp<lm::DmTiny>(mode, B, P, A, O, X, stream);
  else
    lm::run_dp<lm::DmDefault>(mode, B, P, A, O, X, stream);
}

int lenet_mfma_slab_floats(int cfg) { return cfg == LENET_TINY ? lm::DmTiny::SLABN : lm::DmDefault::SLABN; }
int lenet_mfma_wimg_elems() { return lm::kWimgTot; }
int lenet_mfma_kw_blocks(int cfg) {
  return cfg == LENET_TINY ? lm::mw_conv_blocks<lm::DmTiny>() + lm::mw_fc_blocks<lm::DmTiny>() + 1
                           : lm::mw_conv_blocks<lm::DmDefault>() + lm::mw_fc_blocks<lm::DmDefault>() + 1;
}

void launch_lenet_mfma_apply(int cfg, const LeNetPtrs& P, const LeNetOpt& O, const unsigned* skip, hipStream_t stream) {
  if (O.n <= 0) return;
  const dim3 grid((unsigned)((O.n + 255) / 256));
  if (cfg == LENET_TINY)
    hipLaunchKernelGGL(lm::lenet_mapply<lm::DmTiny>, grid, dim3(256), 0, stream, P, O, skip);
  else
    hipLaunchKernelGGL(lm::lenet_mapply<lm::DmDefault>, grid, dim3(256), 0, stream, P, O, skip);
}

void launch_lenet_mfma_pack(int cfg, const LeNetPtrs& P, const LeNetOpt& O, hipStream_t stream) {
  if (cfg == LENET_TINY)
    lm::pack<lm::DmTiny>(P, O, stream);
  else
    lm::pack<lm::DmDefault>(P, O, stream);
}

void launch_lenet_mfma(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                       hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::run<lm::DmTiny>(mode, B, P, A, O, stream);
  else
    lm::run<lm::DmDefault>(mode, B, P, A, O, stream);
}

}  // namespace mlt
