// Speed-of-light probes of the mode-8 dense GEMM (csrc/kernels/hgemm8.hip) outside the library: the
// kernel is compiled with -DH8_PROBE=<bits> (no MFMA / no DMA / no vmcnt waits) and timed on the
// Llama-3-8B gate|up shape over rotating weight copies (weights stream from HBM as in decode).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DH8_PROBE=1 tools/hg8_probe.hip -o /tmp/p1
//   ./p1 [M=512] [bn=224] [rows=28672] [K=4096] [epi=3] [ks=1] [type=1]
// type 1 = the f16 mode-8 kernel (bn 256/224/128), 10 = the f16 mode-10 kernel (256 x 256 tiles);
// 12 / 14 = Q4_K / Q6_K tile-blocks through mode 9
// (bn 256/128; -DH9_PROBE=<bits> selects its probe), any byte pattern (timing only)
#include "../csrc/kernels/hgemm8.hip"
#include "../csrc/kernels/qgemm9.hip"
#include "../csrc/kernels/hgemm10.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 512;
  const int bn = argc > 2 ? atoi(argv[2]) : 224;
  const int rows = argc > 3 ? atoi(argv[3]) : 28672;
  const int K = argc > 4 ? atoi(argv[4]) : 4096;
  const int epi = argc > 5 ? atoi(argv[5]) : nls_gemv::EPI_SWIGLU;
  const int ks = argc > 6 ? atoi(argv[6]) : 1;
  const int qt = argc > 7 ? atoi(argv[7]) : 1;
  const int q9w = argc > 8 ? atoi(argv[8]) : 4;   // mode-9 waves (4 | 8)
  if (rows % bn || K % 32 || M <= 0) { printf("bad shape\n"); return 1; }
  const size_t wbytes = (qt == 1 || qt == 10) ? (size_t)rows * K * 2
                                : (size_t)(rows / 16) * (K / 256) * (qt == 12 ? 2304 : 3360);
  const int ncopy = (int)std::max<size_t>(1, ((size_t)1 << 30) / wbytes + 1);
  std::vector<void*> W(ncopy);
  for (auto& p : W) { CK(hipMalloc(&p, wbytes)); CK(hipMemset(p, 0x11, wbytes)); }
  void *x, *y;
  CK(hipMalloc(&x, (size_t)M * K * 2));
  CK(hipMemset(x, 0x22, (size_t)M * K * 2));
  CK(hipMalloc(&y, (size_t)M * rows * 4));
  void* ws = nullptr;
  if (ks > 1) CK(hipMalloc(&ws, (size_t)ks * M * rows * 4));
  nls_gemv::SegList sl{};
  sl.nseg = 1;
  sl.s[0].type = qt == 10 ? QT_F16 : qt;
  sl.s[0].rows = rows;
  sl.s[0].K = K;
  nls_gemv::GemvArgs a{};
  a.x = (const act_t*)x;
  a.ldx = K;
  a.y = y;
  a.ldy = epi == nls_gemv::EPI_SWIGLU ? rows / 2 : rows;
  a.M = M;
  a.epi = epi;
  a.alpha = 1.f;
  a.mtot = M;
  a.pad = rows;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto run = [&](int i) {
    sl.s[0].w = (const uint8_t*)W[i % ncopy];
    const int rc = qt == 10 ? nls_hg10::launch_dense10(sl, rows / 256, ks, (float*)ws, a, st)
                 : qt == 1 ? nls_hg8::launch_dense8(bn, sl, rows / bn, ks, (float*)ws, a, st)
                           : nls_q9::launch_q9(0, q9w, bn / 16 / q9w, sl, rows / bn, ks, (float*)ws, a, st);
    if (rc) { printf("launch failed\n"); exit(1); }
  };
  for (int i = 0; i < 3 * ncopy; ++i) run(i);
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < 20; ++i) run(i);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1e3f / 20);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[ts.size() / 2];
  printf("probe=%d/%d type=%d M=%d bn=%d rows=%d K=%d epi=%d ks=%d: %.2f us  %.1f TFLOP/s  %.0f GB/s weights\n",
         H8_PROBE, H9_PROBE, qt, M, bn, rows, K, epi, ks, us, 2.0 * M * rows * K / us / 1e6, wbytes / us / 1e3);
  return 0;
}
