// LeNet-5 bf16 MFMA training step, data-parallel entry points. The batch-reduction kernels with the
// fused xGMI exchange (lenet_mwx<D, W>, W = 1 .. 8 and the two-phase forms) are instantiated one world
// size per translation unit (lenet_mfma_dpw<W>.hip) so that they compile in parallel.
#include "lenet_mfma.inc"

namespace mlt {

int64_t lenet_mfma_xch_granules(int cfg) {
  return cfg == LENET_TINY ? lm::xch_granules<lm::DmTiny>() : lm::xch_granules<lm::DmDefault>();
}

void launch_lenet_mfma_dp(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                          const XgmiFused& X, hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::run_dp<lm::DmTiny>(cfg, mode, B, P, A, O, X, stream);
  else
    lm::run_dp<lm::DmDefault>(cfg, mode, B, P, A, O, X, stream);
}

}  // namespace mlt
