// Quantised GEMV/GEMM kernels of type-set 2 (see qgemv_impl.h); one TU per set so the
// instantiations compile in parallel.
#include "qgemv_impl.h"

namespace nls_gemv {
int launch_k2(int mode, int waves, int rt, int mt, const SegList& sl, int tiles, int ks, float* ws,
               const GemvArgs& a, hipStream_t st, int nmb) {
  return launch_kset<2>(mode, waves, rt, mt, sl, tiles, ks, ws, a, st, nmb);
}
}  // namespace nls_gemv
