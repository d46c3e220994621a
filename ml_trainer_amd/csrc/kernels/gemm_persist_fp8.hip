// fp8 (OCP e4m3 / e5m2, MX-scaled MFMA) instantiations of the persistent GEMM (gemm_persist.hip),
// compiled as their own translation unit so the two halves build in parallel.
#define MLT_PERSIST_FP8 1
#include "gemm_persist.hip"
