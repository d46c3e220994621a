// lenet_mwx<D, 8> (+ its two-phase form where one exists): one world size per translation unit
#include "lenet_mfma.inc"

namespace mlt {
namespace lm {
MLT_DEF_MWX(8)
}  // namespace lm
}  // namespace mlt
