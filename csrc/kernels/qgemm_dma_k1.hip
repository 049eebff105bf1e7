// LDS-DMA GEMM kernels (mode 3) of type-set 1 (see qgemm_dma.h); one TU per set.
#include "qgemm_dma.h"

namespace nls_dma {
int launch_dma_k1(int mt, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  return launch_dma_kset<1>(mt, sl, ntiles, ks, ws, a, st);
}
}  // namespace nls_dma
