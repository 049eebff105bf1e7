// Large-M LDS-dequant GEMM kernels of type-set 1 (see qgemm_impl.h); one TU per set.
#include "qgemm_impl.h"

namespace nls_gemm {
int launch_lds_k1(int wm, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  return launch_lds_kset<1>(wm, sl, ntiles, ks, ws, a, st);
}
}  // namespace nls_gemm
