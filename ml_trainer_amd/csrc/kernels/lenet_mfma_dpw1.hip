// lenet_mwx<D, 1> (+ its two-phase form where one exists): one world size per translation unit
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
MLT_DEF_MWX(1)
}  // namespace lm
}  // namespace mlt
