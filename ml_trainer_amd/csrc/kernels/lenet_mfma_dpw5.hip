// lenet_mwx<D, 5> (+ its two-phase form where one exists): one world size per translation unit
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
MLT_DEF_MWX(5)
}  // namespace lm
}  // namespace mlt
