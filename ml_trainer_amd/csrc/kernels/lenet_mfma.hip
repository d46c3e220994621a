// LeNet-5 bf16 MFMA training step -- host entry points (the kernels: lenet_mfma.inc).
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
void launch_ms(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, hipStream_t st) {
  const float inv_B = 1.f / (float)B;
  if (cfg == LENET_TINY)
    hipLaunchKernelGGL(lenet_ms<DmTiny>, dim3(B), dim3(kT), 0, st, P.stage2, P.meta2, A.ctrl, P.wimg, P.metaN, mode,
                       inv_B, P, A, O, B);
  else
    hipLaunchKernelGGL(lenet_ms<DmDefault>, dim3(B), dim3(kT), 0, st, P.stage2, P.meta2, A.ctrl, P.wimg, P.metaN, mode,
                       inv_B, P, A, O, B);
}
}  // namespace lm

void launch_lenet_mfma_reduce(int cfg, int B, const LeNetPtrs& P, const LeNetOpt& O, const XgmiFused* X,
                              hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::reduce_only<lm::DmTiny>(cfg, B, P, O, X, stream);
  else
    lm::reduce_only<lm::DmDefault>(cfg, B, P, O, X, stream);
}
int lenet_mfma_slab_floats(int cfg) { return cfg == LENET_TINY ? lm::DmTiny::SLABN : lm::DmDefault::SLABN; }
int lenet_mfma_wimg_elems() { return lm::kWimgTot; }
bool lenet_mfma_trace_build() { return lm::kTraceBuild; }
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
