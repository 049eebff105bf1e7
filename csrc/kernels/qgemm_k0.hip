// Large-M LDS-dequant GEMM kernels of type-set 0 (see qgemm_impl.h); one TU per set.
#include "qgemm_impl.h"

namespace nls_gemm {
int launch_lds_k0(int wm, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  return launch_lds_kset<0>(wm, sl, ntiles, ks, ws, a, st);
}
}  // namespace nls_gemm
