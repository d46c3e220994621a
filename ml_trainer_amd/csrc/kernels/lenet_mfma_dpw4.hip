// lenet_mwx<D, 4> (+ its two-phase form where one exists): one world size per translation unit
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
MLT_DEF_MWX(4)
}  // namespace lm
}  // namespace mlt
