// Quantised GEMV/GEMM kernels of type-set 3 (the ggml 32-value affine blocks Q4_0 / Q4_1 / Q5_0 / Q5_1 as
// QT_Q51, with Q6_K and Q8_0; see qgemv_impl.h); one TU per set so the instantiations compile in parallel.
#include "qgemv_impl.h"

namespace nls_gemv {
int launch_k3(int mode, int waves, int rt, int mt, const SegList& sl, int tiles, int ks, float* ws,
               const GemvArgs& a, hipStream_t st, int nmb) {
  return launch_kset<3>(mode, waves, rt, mt, sl, tiles, ks, ws, a, st, nmb);
}
}  // namespace nls_gemv
