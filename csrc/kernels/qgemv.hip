// Dispatcher of the quantised GEMV / GEMM (kernels: qgemv_impl.h, instantiated per type-set in
// qgemv_k{0,1,2}.hip).
#include "qgemm_impl.h"
#include "qgemm_dma.h"

using namespace nls_gemv;

namespace nls_hgemm {
int launch_dense(int wm, int bn, int waves, int nst, const SegList& sl, int ntiles, int ks, float* ws,
                 const GemvArgs& a, hipStream_t st);
}
namespace nls_hg10 {
int launch_dense10(int bn, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st);
}
namespace nls_q9 {
int launch_q9(int kset, int waves, int rt, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a,
              hipStream_t st, int bm);
}


extern "C" {

// Host-side segment descriptor (plain C layout for ctypes).
struct NlsSeg {
  const void* w;
  const int* xmap;
  const int* ymap;
  const int* mcount;
  int type, rows, K, ycol;
};

// Optional fused operands of a launch (plain C layout for ctypes; every pointer may be null).
struct NlsFuse {
  const float* xf; long ldxf; const float* nw; float eps;                    // input RMSNorm (path A)
  const int* pos; const int* slot; const float* cs; const float* bias;      // EPI_ROPE
  void* q_out; long ldq; void* kc; void* vc; int Hq, Hkv, D, pad0;
  void* hout; long ldh; const float* onw; int* cnt;                          // residual add + RMSNorm
  float* ssq_out; const float* ssq_in; int ldss, nss_in;                     // split RMSNorm (GemvArgs)
  const int* sel; int sel_slots, sel_base, pad1;                             // device-selected segments
  const void* wr; int E, topk, renorm, rcap;                                 // MoE route after the norm (onw)
  float* rlogits; float* topw; int* counts; int* xrows; int* yrows; int* rsel;
};

// mode 0: path A (waves split K, LDS reduce; mapped rows / MoE capable)
// mode 1: path B (waves split rows, LDS-staged activations, optional split-K `ks` with workspace
//         `ws` of ks*M*sum(rows) floats).
// mode 2: large-M LDS-dequant GEMM (qgemm_impl.h; K-quant types only): 8 waves, `rt` = WM (4: 256-row
//         activation blocks, 2: 128-row), optional split-K as mode 1.
// mode 3: large-M LDS-DMA GEMM (qgemm_dma.h; Q4_K/Q5_K/Q6_K only): 4 waves, `rt` = activation
//         tiles per block (16: 256 rows, 8: 128 rows; 6 / 4: 96 / 64 rows at two workgroups per CU, the MoE
//         expert blocks), mapped rows, optional split-K as mode 1.
// mode 4: large-M dense f16 GEMM (hgemm.hip): every segment is type F16 with `w` = a ROW-MAJOR
//         [rows][K] f16 matrix (not the tiled layout); 8 waves, `rt` = WM (4: 256-row activation
//         blocks, 2: 128-row), optional split-K as mode 1.
// mode 5: mode 4 with 256-row weight tiles (twice the MFMA work per fetched activation byte).
// mode 6: mode 4 at 128-row activation blocks (rt 2) with 2-deep rings: two workgroups per CU.
// mode 10: dense f16 GEMM, 256 x 256 tiles, 4 phases per 64-deep K-tile with the two wave groups staggered
//         by one barrier (hgemm10.hip); the mode-8 operands and epilogues, optional split-K.
// (Modes 11-13 -- mode 10 on raw K-quant tiles, mode 9 at 64-row blocks, stream-K -- lost every measured shape in
//  round 5 and were removed from the build; profiles/streamk_r05.txt, profiles/qgemm11_r05.txt.)
// mode 9: quantised GEMM on the raw tile-blocks (qgemm9.hip; Q4_K/Q5_K/Q6_K/Q8_0/Q51): 256-row activation
//         blocks x 16*waves*rt weight rows ((waves, rt) = (4, 2) | (8, 2) | (8, 1)), the mode-8
//         epilogues, optional split-K.
// Returns 0 on success, a hipError_t, or -1 on bad arguments.
static int qgemv_impl(const NlsSeg* segs, int nseg, const void* x, long ldx, void* y, long ldy, int M,
                      float alpha, int epi, void* argmax, int waves, int rt, int mode, int ks, void* ws,
                      void* stream, const NlsFuse* fz) {
  static const NlsFuse none{};
  if (!fz) fz = &none;
  const float* xf = fz->xf;
  if (xf && (M > 16 || !fz->nw || (mode != 0 && !(mode == 1 && fz->ssq_in)))) return -1;
  if (fz->ssq_in && (!xf || fz->nss_in < 1 || fz->nss_in > fz->ldss)) return -1;
  if (fz->ssq_out) {      // producer of a split RMSNorm: path A residual add, whole tiles of tokens
    const int ncols = ((M + 15) / 16) * 16;
    if (mode != 0 || epi != EPI_ADD_F32 || nseg != 1 || segs[0].xmap || segs[0].ymap || segs[0].mcount || argmax ||
        fz->onw || M > 32 || (waves * 64) % ncols || fz->ldss < (segs[0].rows + 16 * rt - 1) / (16 * rt))
      return -1;
  }
  if (epi == EPI_ROPE) {   // fused RoPE / KV append: path A or a dense GEMM without split-K; plain rows,
                           // contiguous Q|K|V segments
    if (!(mode == 0 || ((mode == 4 || mode == 5 || mode == 10) && ks <= 1)) || argmax ||
        !fz->pos || !fz->slot ||
        !fz->cs || !fz->q_out || !fz->kc || !fz->vc || fz->D < 2 || fz->D % 2 || fz->Hq < 1 || fz->Hkv < 1)
      return -1;
    int c = 0;
    for (int i = 0; i < nseg; ++i) {
      if (segs[i].xmap || segs[i].ymap || segs[i].mcount || segs[i].rows % 16 || segs[i].ycol != c) return -1;
      c += segs[i].rows;
    }
    if (c != (fz->Hq + 2 * fz->Hkv) * fz->D) return -1;
  }
  if (fz->onw && (mode != 0 || epi != EPI_ADD_F32 || nseg != 1 || segs[0].ycol || segs[0].xmap || segs[0].ymap ||
                  segs[0].mcount || !fz->cnt || !fz->hout || segs[0].rows % 4 || argmax))
    return -1;
  if (fz->wr && (!fz->onw || M > 4 || fz->E < 1 || fz->E > 64 || fz->topk < 1 || fz->topk > fz->E || fz->topk > 8 ||
                 !fz->rlogits || !fz->topw || !fz->counts || !fz->xrows || !fz->yrows || segs[0].rows % 4))
    return -1;
  if (fz->sel) {           // path A over routed experts only: identical segment shapes
    if (mode != 0 || fz->sel_slots < 1 || fz->sel_slots > 256 || argmax) return -1;
    for (int i = 1; i < nseg; ++i)
      if (segs[i].rows != segs[0].rows || segs[i].K != segs[0].K) return -1;
  }
  if (nseg < 1 || nseg > 8 || M < 1 ||
      (waves != 4 && waves != 8 && !(waves == 16 && mode >= 4) && !(waves == 7 && mode == 1 && rt == 1 && M == 1)))
    return -1;
  if (mode < 0 || mode > 10 || mode == 7 || mode == 8 || (mode == 6 && (waves != 8 || rt != 2))) return -1;
  if (mode == 10) {            // rt 1: 256-row weight tiles, rt 2: 128-row
    if (waves != 8 || (rt != 1 && rt != 2) || fz->xf || fz->onw || ldx % 8 ||
        ((epi == EPI_F32 || epi == EPI_ADD_F32 || epi == EPI_ACT) && ldy % 4))
      return -1;
    for (int i = 0; i < nseg; ++i)
      if (segs[i].type != QT_F16 || segs[i].xmap || segs[i].ymap || segs[i].mcount || segs[i].ycol % 4) return -1;
  } else if (mode == 9) {
    if (!((waves == 4 && rt == 2) || (waves == 8 && (rt == 2 || rt == 1))) || fz->xf || fz->onw || epi == EPI_ROPE || ldx % 8 ||
        ((epi == EPI_F32 || epi == EPI_ADD_F32 || epi == EPI_ACT) && ldy % 4))
      return -1;
    for (int i = 0; i < nseg; ++i)
      if (segs[i].xmap || segs[i].ymap || segs[i].mcount || segs[i].ycol % 4) return -1;
  } else if (mode >= 4 && mode <= 6) {
    if ((waves != 8 && waves != 16) || (rt != 2 && rt != 4) || fz->xf || fz->onw || (epi == EPI_ROPE && mode == 6))
      return -1;
    for (int i = 0; i < nseg; ++i)
      if (segs[i].type != QT_F16) return -1;
  } else if (mode == 3) {
    if (waves != 4 || (rt != 4 && rt != 6 && rt != 8 && rt != 16)) return -1;
  } else if (mode == 2 ? (waves != 8 || (rt != 1 && rt != 2 && rt != 4)) : (rt != 1 && rt != 2)) {
    return -1;
  }
  if (M > 64 && mode == 0) return -1;   // large M: path B / LDS GEMM
  if (mode != 0 && ks > 1 && !ws) return -1;
  if (epi == EPI_SLABS && (mode == 0 || ks < 2)) return -1;   // slabs exist only with split-K
  // mapped split-K (MoE down projection at many tokens): slabs indexed by the y row, one reduce
  bool mks = (mode >= 1 && mode <= 5) && ks > 1 && epi == EPI_F32 && !argmax;
  for (int i = 0; i < nseg && mks; ++i)
    mks = segs[i].ymap && segs[i].ycol == 0 && segs[i].rows == segs[0].rows;
  SegList sl{};
  int tiles = 0, cols = 0;
  const int tile_rows = mode == 10 ? 256 / rt : mode == 9 ? 16 * waves * rt : (mode == 5 ? 256 : (mode >= 2 ? 128 : (mode == 1 ? waves : 1) * rt * 16));
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].K % 256 || segs[i].rows < 1) return -1;
    if (epi == EPI_SWIGLU && segs[i].rows % 16) return -1;
    // mapped rows (MoE): path A, or path B / the LDS-dequant / LDS-DMA / dense GEMMs (modes 1-5) without
    // arg-max; split-K only as "mapped split-K" (every segment an expert writing the same output
    // columns of its own y rows, f32 store)
    if ((segs[i].xmap || segs[i].ymap || segs[i].mcount) && mode != 0 &&
        (!(mode >= 1 && mode <= 5) || argmax || epi == EPI_SLABS || (ks > 1 && !mks)))
      return -1;
    sl.s[i].w = (const uint8_t*)segs[i].w;
    sl.s[i].xmap = segs[i].xmap;
    sl.s[i].ymap = segs[i].ymap;
    sl.s[i].mcount = segs[i].mcount;
    sl.s[i].type = segs[i].type;
    sl.s[i].rows = segs[i].rows;
    sl.s[i].K = segs[i].K;
    sl.s[i].ycol = segs[i].ycol;
    sl.s[i].tile_begin = tiles;
    sl.s[i].tile_begin_col = cols;
    tiles += (segs[i].rows + tile_rows - 1) / tile_rows;
    cols += segs[i].rows;
  }
  sl.nseg = nseg;
  // pick the kernel type-set that covers every segment (Q6_K is in sets 0, 1 and 3; Q8_0 in 1 and 3)
  bool q4k = false, q5k = false, q8 = false, q51 = false, flt = false, bad = false;
  for (int i = 0; i < nseg; ++i) {
    const int t = segs[i].type;
    if (t == QT_Q4_K) q4k = true;
    else if (t == QT_Q5_K) q5k = true;
    else if (t == QT_Q8_0) q8 = true;
    else if (t == QT_Q51) q51 = true;
    else if (t == QT_F16 || t == QT_BF16 || t == QT_F32) flt = true;
    else if (t != QT_Q6_K) bad = true;
  }
  if (bad || (flt && (q4k || q5k || q8 || q51)) || (q4k && (q5k || q8 || q51)) || (q51 && q5k)) return -1;
  const int kset = flt ? 2 : (q51 ? 3 : (q4k ? 0 : ((q5k || q8) ? 1 : 0)));
  GemvArgs a{};
  a.x = (const act_t*)x;
  a.ldx = ldx;
  a.y = y;
  a.ldy = ldy;
  a.M = M;
  a.epi = epi;
  a.alpha = alpha;
  a.pad = mks ? segs[0].rows : cols;      // split-K slab width
  a.argmax = (unsigned long long*)argmax;
  a.m0 = 0;
  a.mtot = M;
  a.xf = xf;
  a.ldxf = fz->ldxf;
  a.nw = fz->nw;
  a.eps = fz->eps;
  a.pos = fz->pos;
  a.slot = fz->slot;
  a.cs = fz->cs;
  a.bias = fz->bias;
  a.q_out = (__bf16*)fz->q_out;
  a.ldq = fz->ldq;
  a.kc = (__bf16*)fz->kc;
  a.vc = (__bf16*)fz->vc;
  a.Hq = fz->Hq;
  a.Hkv = fz->Hkv;
  a.D = fz->D;
  a.hout = (act_t*)fz->hout;
  a.ldh = fz->ldh;
  a.onw = fz->onw;
  a.cnt = fz->cnt;
  a.sel = fz->sel;
  a.sel_base = fz->sel_base;
  a.sel_tiles = (segs[0].rows + tile_rows - 1) / tile_rows;
  if (fz->sel) tiles = fz->sel_slots * a.sel_tiles;
  a.wr = (const act_t*)fz->wr;
  a.E = fz->E;
  a.topk = fz->topk;
  a.renorm = fz->renorm;
  a.rcap = fz->rcap;
  a.rlogits = fz->rlogits;
  a.topw = fz->topw;
  a.counts = fz->counts;
  a.xrows = fz->xrows;
  a.yrows = fz->yrows;
  a.rsel = fz->rsel;
  a.ssq_out = fz->ssq_out;
  a.ssq_in = fz->ssq_in;
  a.ldss = fz->ldss;
  a.nss_in = fz->nss_in;
  const int mt = M > 64 ? 8 : (M + 15) / 16;
  const int nmb = M > 64 ? (M + 127) / 128 : 1;
  hipStream_t st = (hipStream_t)stream;
  auto launch = kset == 0 ? launch_k0 : (kset == 1 ? launch_k1 : (kset == 2 ? launch_k2 : launch_k3));
  if (mode >= 2 && mode <= 3 && kset >= 2) return -1;   // tiled float / Q51 weights: paths A and B only
  if (mode == 9 && kset == 2) return -1;   // mode 9: quantised formats only
  if (mode == 3)
    for (int i = 0; i < nseg; ++i)
      if (segs[i].type == QT_Q8_0) return -1;   // raw Q8_0 tiles do not fit the DMA LDS budget
  if (mode != 0) {
    if (ks < 1) ks = 1;
    int rc;
    if (mode == 10)
      rc = nls_hg10::launch_dense10(256 / rt, sl, tiles, ks, (float*)ws, a, st);
    else if (mode == 9)
      rc = nls_q9::launch_q9(kset, waves, rt, sl, tiles, ks, (float*)ws, a, st, 256);
    else if (mode >= 4)
      rc = nls_hgemm::launch_dense(rt, mode == 5 ? 256 : 128, waves, mode == 6 ? 2 : 3, sl, tiles, ks, (float*)ws, a,
                                   st);
    else if (mode == 3)
      rc = (kset == 0 ? nls_dma::launch_dma_k0 : nls_dma::launch_dma_k1)(rt, sl, tiles, ks, (float*)ws, a, st);
    else if (mode == 2)
      rc = (kset == 0 ? nls_gemm::launch_lds_k0 : nls_gemm::launch_lds_k1)(rt, sl, tiles, ks, (float*)ws, a, st);
    else
      rc = launch(1, waves, rt, mt, sl, tiles, ks, (float*)ws, a, st, nmb);
    if (rc || ks == 1 || epi == EPI_SLABS) return rc;
    RedList rl{};
    if (mks) {            // slabs [ks][M y rows][rows]: one shared output segment
      rl.s[0] = RedSeg{0, segs[0].rows, 0, 0};
      rl.nseg = 1;
      dim3 grid((segs[0].rows + 255) / 256, M);
      hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, (const float*)ws, ks, M, segs[0].rows, rl, a);
      return (int)hipGetLastError();
    }
    for (int i = 0; i < nseg; ++i) rl.s[i] = RedSeg{sl.s[i].tile_begin_col, sl.s[i].rows, sl.s[i].ycol, 0};
    rl.nseg = nseg;
    const int nout = epi == EPI_SWIGLU ? cols / 2 : cols;
    dim3 grid((nout + 255) / 256, M);
    hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, (const float*)ws, ks, M, cols, rl, a);
    return (int)hipGetLastError();
  }
  return launch(0, waves, rt, mt, sl, tiles, 1, nullptr, a, st, 1);
}

int nls_qgemv(const NlsSeg* segs, int nseg, const void* x, long ldx, void* y, long ldy, int M,
              float alpha, int epi, void* argmax, int waves, int rt, int mode, int ks, void* ws,
              void* stream) {
  return qgemv_impl(segs, nseg, x, ldx, y, ldy, M, alpha, epi, argmax, waves, rt, mode, ks, ws, stream, nullptr);
}

// Path A with the input RMSNorm fused into the activation staging: x rows = f16(rmsnorm(xf) * nw).
int nls_qgemv_norm(const NlsSeg* segs, int nseg, const float* xf, long ldxf, const float* nw, float eps, void* y,
                   long ldy, int M, float alpha, int epi, void* argmax, int waves, int rt, void* stream) {
  NlsFuse fz{};
  fz.xf = xf;
  fz.ldxf = ldxf;
  fz.nw = nw;
  fz.eps = eps;
  return qgemv_impl(segs, nseg, xf, 0, y, ldy, M, alpha, epi, argmax, waves, rt, 0, 1, nullptr, stream, &fz);
}

// Any launch with fused operands (input norm, RoPE/KV-append epilogue, residual + output norm).
int nls_qgemv_ex(const NlsSeg* segs, int nseg, const void* x, long ldx, void* y, long ldy, int M, float alpha,
                 int epi, void* argmax, int waves, int rt, int mode, int ks, void* ws, void* stream,
                 const NlsFuse* fz) {
  return qgemv_impl(segs, nseg, fz && fz->xf ? (const void*)fz->xf : x, ldx, y, ldy, M, alpha, epi, argmax, waves,
                    rt, mode, ks, ws, stream, fz);
}

int nls_fuse_size() { return (int)sizeof(NlsFuse); }

}  // extern "C"
