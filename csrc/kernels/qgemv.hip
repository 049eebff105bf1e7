// Quantised GEMV / skinny GEMM for decode (M <= 64 activation rows), gfx950.
//
//   y[m, n] = alpha * sum_k x[m, k] * W[n, k]      (W in GGUF block formats)
//
// Design (SURVEY.md §2F "gemv_q*"): decode is HBM-bound on the weight stream,
// so every weight byte is read exactly once, straight into VGPRs (no LDS round
// trip, non-temporal loads), dequantised in registers to bf16 and fed to
// v_mfma_f32_16x16x32_bf16 as the B operand (16 weight rows per tile). The
// activation rows (batch, padded to 16) are the A operand, so batch 1..16 costs
// the same MFMA issue as batch 1 and the weight dequant is amortised over the
// whole batch. A workgroup owns RT*16 output rows; its WAVES waves split K and
// reduce through LDS, so no atomics and bit-reproducible results.
//
// One launch may cover several weight matrices ("segments": fused Q|K|V with
// per-matrix quant types, or the experts of an MoE layer) and applies a fused
// epilogue: plain store, residual add (y += alpha*acc), SwiGLU on interleaved
// gate/up rows, and a fused greedy arg-max (packed u64 atomicMax per row).
#include "common.h"

namespace {

enum Epi : int { EPI_F32 = 0, EPI_BF16 = 1, EPI_ADD_F32 = 2, EPI_SWIGLU_BF16 = 3 };

struct Seg {
  const uint8_t* w;
  const int* xmap;     // optional: segment-local batch row -> x row (-1: none)
  const int* ymap;     // optional: segment-local batch row -> y row
  const int* mcount;   // optional: device count of valid rows (tiles skip when 0)
  int type, rows, K, tile_begin, ycol, pad;
};
struct SegList { Seg s[8]; int nseg; int pad[3]; };

struct GemvArgs {
  const __bf16* x; long ldx;
  void* y; long ldy;
  int M;               // rows of x / y (or max rows per segment when mapped)
  int epi;
  float alpha;
  int pad;
  unsigned long long* argmax;   // optional [M] packed (ordered value << 32 | ~idx)
};

DEVI unsigned long long argmax_key(float v, int idx) {
  uint32_t u = __builtin_bit_cast(uint32_t, v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xFFFFFFFFu - (uint32_t)idx);
}

DEVI float silu(float g) { return g / (1.f + __expf(-g)); }

template <int T, int WAVES, int RT, int MT>
DEVI void gemv_tile(const Seg& S, int row0, const GemvArgs& a, float* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const WDesc W{S.w, S.rows, S.K};
  const int nb = S.K >> 8;
  const int sb0 = (nb * wave) / WAVES, sb1 = (nb * (wave + 1)) / WAVES;

  int mcount = a.M;
  if (S.mcount) mcount = min(*S.mcount, a.M);

  // activation row pointers for this lane (A operand row = batch row r of tile mt)
  const __bf16* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int m = mt * 16 + r;
    int src = m;
    if (S.xmap) src = (m < mcount) ? S.xmap[m] : -1;
    xr[mt] = src >= 0 ? a.x + (size_t)src * a.ldx : nullptr;
  }
  int rowc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) rowc[rt] = min(row0 + rt * 16 + r, S.rows - 1);

  f32x4 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef typename RawOf<T>::type Raw;
  Raw cur[RT];
  if (sb0 < sb1) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) cur[rt] = load_raw<T, true>(W, rowc[rt], sb0, g);
  }
  const bf16x8 zero8 = {};
  for (int sb = sb0; sb < sb1; ++sb) {
    Raw nxt[RT];
    if (sb + 1 < sb1) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) nxt[rt] = load_raw<T, true>(W, rowc[rt], sb + 1, g);
    }
    bf16x8 wf[RT][8];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) dequant<T>(cur[rt], g, wf[rt]);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int ko = sb * 256 + xoff<T>(t, g);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 xa = xr[mt] ? *reinterpret_cast<const bf16x8*>(xr[mt] + ko) : zero8;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          acc[rt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, wf[rt][t], acc[rt][mt], 0, 0, 0);
      }
    }
    if (sb + 1 < sb1) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) cur[rt] = nxt[rt];
    }
  }

  // ---- cross-wave reduction through LDS -------------------------------------
  // red: [WAVES][RT][MT][4][64] ; tile: [RT*16 rows][MT*16 batch]
  float* red = lds;
  float* tile = lds + WAVES * RT * MT * 256;
  constexpr int NE = RT * MT * 256;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        red[(((wave * RT + rt) * MT + mt) * 4 + c) * 64 + lane] = acc[rt][mt][c];
  __syncthreads();
  for (int e = threadIdx.x; e < NE; e += WAVES * 64) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += red[w * NE + e];
    const int ln = e & 63, c = (e >> 6) & 3, mt = (e >> 8) % MT, rt = (e >> 8) / MT;
    const int rr = rt * 16 + (ln & 15);
    const int bb = mt * 16 + 4 * (ln >> 4) + c;
    tile[rr * (MT * 16) + bb] = s * a.alpha;
  }
  __syncthreads();

  // ---- epilogue ----------------------------------------------------------------
  const int ncols = MT * 16;
  if (a.epi == EPI_SWIGLU_BF16) {
    // tile rows [16i, 16i+8) = gate, [16i+8, 16i+16) = up of outputs (row0/2 + 8i + j)
    for (int e = threadIdx.x; e < RT * 8 * ncols; e += WAVES * 64) {
      const int bb = e % ncols, j = e / ncols, rt = j >> 3, jj = j & 7;
      if (bb >= mcount) continue;
      const int grow = row0 + rt * 16 + jj;
      if (grow >= S.rows) continue;
      const float gv = tile[(rt * 16 + jj) * ncols + bb];
      const float uv = tile[(rt * 16 + 8 + jj) * ncols + bb];
      const int yrow = S.ymap ? S.ymap[bb] : bb;
      const int n = S.ycol + (row0 >> 1) + rt * 8 + jj;
      reinterpret_cast<__bf16*>(a.y)[(size_t)yrow * a.ldy + n] = (__bf16)(silu(gv) * uv);
    }
    return;
  }
  for (int e = threadIdx.x; e < RT * 16 * ncols; e += WAVES * 64) {
    const int bb = e % ncols, rr = e / ncols;
    const int row = row0 + rr;
    if (bb >= mcount || row >= S.rows) continue;
    const float v = tile[rr * ncols + bb];
    const int yrow = S.ymap ? S.ymap[bb] : bb;
    const size_t off = (size_t)yrow * a.ldy + S.ycol + row;
    if (a.epi == EPI_F32) reinterpret_cast<float*>(a.y)[off] = v;
    else if (a.epi == EPI_ADD_F32) reinterpret_cast<float*>(a.y)[off] += v;
    else reinterpret_cast<__bf16*>(a.y)[off] = (__bf16)v;
  }
  if (a.argmax) {
    for (int bb = threadIdx.x; bb < min(mcount, ncols); bb += WAVES * 64) {
      unsigned long long best = 0;
      for (int rr = 0; rr < RT * 16; ++rr) {
        const int row = row0 + rr;
        if (row >= S.rows) break;
        unsigned long long k = argmax_key(tile[rr * ncols + bb], S.ycol + row);
        best = k > best ? k : best;
      }
      atomicMax(a.argmax + bb, best);
    }
  }
}

template <int WAVES, int RT, int MT>
__global__ __launch_bounds__(WAVES * 64) void qgemv_kernel(SegList segs, GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tile = blockIdx.x;
  Seg S = segs.s[0];
#pragma unroll
  for (int i = 1; i < 8; ++i)
    if (i < segs.nseg && tile >= segs.s[i].tile_begin) S = segs.s[i];
  if (S.mcount && *S.mcount <= 0) return;     // MoE expert with no routed tokens
  const int row0 = (tile - S.tile_begin) * RT * 16;
  switch (S.type) {
    case QT_Q4_K: gemv_tile<QT_Q4_K, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_Q5_K: gemv_tile<QT_Q5_K, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_Q6_K: gemv_tile<QT_Q6_K, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_Q8_0: gemv_tile<QT_Q8_0, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_F16: gemv_tile<QT_F16, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_BF16: gemv_tile<QT_BF16, WAVES, RT, MT>(S, row0, a, lds); break;
    case QT_F32: gemv_tile<QT_F32, WAVES, RT, MT>(S, row0, a, lds); break;
    default: break;
  }
}

template <int WAVES, int RT, int MT>
int launch_t(const SegList& sl, int ntiles, const GemvArgs& a, hipStream_t st) {
  const size_t lds = (size_t)(WAVES + 1) * RT * MT * 256 * sizeof(float);
  hipLaunchKernelGGL((qgemv_kernel<WAVES, RT, MT>), dim3(ntiles), dim3(WAVES * 64), lds, st, sl, a);
  return (int)hipGetLastError();
}

template <int WAVES, int RT>
int launch_mt(int mt, const SegList& sl, int nt, const GemvArgs& a, hipStream_t st) {
  switch (mt) {
    case 1: return launch_t<WAVES, RT, 1>(sl, nt, a, st);
    case 2: return launch_t<WAVES, RT, 2>(sl, nt, a, st);
    case 3: return launch_t<WAVES, RT, 3>(sl, nt, a, st);
    case 4: return launch_t<WAVES, RT, 4>(sl, nt, a, st);
  }
  return -1;
}

}  // namespace

extern "C" {

// Host-side segment descriptor (plain C layout for ctypes).
struct NlsSeg {
  const void* w;
  const int* xmap;
  const int* ymap;
  const int* mcount;
  int type, rows, K, ycol;
};

// Returns 0 on success, a hipError_t otherwise, -1 on bad arguments.
int nls_qgemv(const NlsSeg* segs, int nseg, const void* x, long ldx, void* y, long ldy, int M,
              float alpha, int epi, void* argmax, int waves, int rt, void* stream) {
  if (nseg < 1 || nseg > 8 || M < 1 || M > 64 || (rt != 1 && rt != 2) || (waves != 4 && waves != 8))
    return -1;
  SegList sl{};
  int tiles = 0;
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].K % 256 || segs[i].rows < 1) return -1;
    if (epi == EPI_SWIGLU_BF16 && segs[i].rows % 16) return -1;
    sl.s[i].w = (const uint8_t*)segs[i].w;
    sl.s[i].xmap = segs[i].xmap;
    sl.s[i].ymap = segs[i].ymap;
    sl.s[i].mcount = segs[i].mcount;
    sl.s[i].type = segs[i].type;
    sl.s[i].rows = segs[i].rows;
    sl.s[i].K = segs[i].K;
    sl.s[i].ycol = segs[i].ycol;
    sl.s[i].tile_begin = tiles;
    tiles += (segs[i].rows + rt * 16 - 1) / (rt * 16);
  }
  sl.nseg = nseg;
  GemvArgs a{(const __bf16*)x, ldx, y, ldy, M, epi, alpha, 0, (unsigned long long*)argmax};
  const int mt = (M + 15) / 16;
  hipStream_t st = (hipStream_t)stream;
  if (waves == 8) return rt == 1 ? launch_mt<8, 1>(mt, sl, tiles, a, st) : launch_mt<8, 2>(mt, sl, tiles, a, st);
  return rt == 1 ? launch_mt<4, 1>(mt, sl, tiles, a, st) : launch_mt<4, 2>(mt, sl, tiles, a, st);
}

}  // extern "C"
