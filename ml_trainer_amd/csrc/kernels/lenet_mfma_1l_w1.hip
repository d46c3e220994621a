// One-launch bf16 LeNet step, xGMI exchange over 1 rank (loopback): one translation unit per world
// size so that the instantiations compile in parallel (kernels: lenet_mfma.inc).
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
void run1_w1(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, unsigned long long* sync,
             const XgmiFused* X, hipStream_t st) {
  if (cfg == LENET_TINY)
    run1<DmTiny, 1>(mode, B, P, A, O, sync, X, st);
  else
    run1<DmDefault, 1>(mode, B, P, A, O, sync, X, st);
}
}  // namespace lm
}  // namespace mlt
