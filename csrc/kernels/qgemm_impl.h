// Large-M quantised GEMM (prefill chunks, decode batches >= 128), gfx950.
//
//   y[m, n] = alpha * sum_k x[m, k] * W[n, k]      (W in GGUF K-quant blocks, x f16)
//
// Why a second GEMM (vs path B of qgemv_impl.h, where every wave dequantises its own weight
// rows into registers and re-reads the activation tile from LDS once per MFMA): at M >= 128
// that design is VALU- and LDS-bound (PMC on gate/up M=256: 6.7 VALU instructions per MFMA,
// 21 % MFMA busy). Here each workgroup DEQUANTISES ITS WEIGHT TILE ONCE INTO LDS and all
// eight waves share it:
//   * workgroup tile = 128 weight rows x BM activation rows (BM = 64*WM: 256 or 128),
//     8 waves as WM (M) x 8/WM (N), each wave a 64 x (128*WM/8) output tile of
//     v_mfma_f32_16x16x32_f16 accumulators (0.5-0.75 LDS reads per MFMA);
//   * K advances in quarters of a super-block (64 values): x quarter [BM][64] and the
//     dequantised W quarter [128][64] live in double-buffered, XOR-swizzled LDS
//     (16-B chunk c of row r stored at c ^ (r & 7): conflict-free ds_read_b128);
//   * wave w streams the raw blocks of tile-block w (16 rows) one super-block ahead and
//     dequantises ONE quarter per step with every lane busy (the v2 tile layouts of
//     common.h put each quarter's bytes in all 64 lanes) -- about one packed-f16 VALU
//     instruction per MFMA;
//   * one barrier per quarter: stage quarter j+1 (x registers -> LDS, dequant -> LDS) and
//     issue the global loads of quarter j+2, then the 32 MFMAs of quarter j.
// Grid: (tile, m-block, k-slice) with every m-block and k-slice of a weight tile on ONE XCD
// (dispatch puts workgroup i on XCD i % 8), so a weight tile is fetched once per XCD L2.
// Split-K (ks > 1) writes fp32 slabs reduced by the launcher's reduce kernels (fused with
// RoPE / residual+RMSNorm where the model uses them).
#pragma once
#include "qgemv_impl.h"

#ifndef NLS_GEMM_MFMA32
#define NLS_GEMM_MFMA32 0     // 1: 32x32x16 MFMA tiles (A/B variant, tools/gemm_ab.py)
#endif
#ifndef NLS_GEMM_SETPRIO
#define NLS_GEMM_SETPRIO 0    // 1: s_setprio(1) around each MFMA cluster (A/B variant)
#endif

namespace nls_gemm {
using namespace nls_gemv;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// NA = 16-row activation tiles each wave multiplies (1..4), chosen per m-block from its real row count:
// wave row wm owns activation tiles i*WM + wm (interleaved), so a block with few rows (MoE experts:
// ~64 routed rows in a 256-row block) spreads its MFMAs over every wave and skips the padding tiles
// instead of multiplying them (Mixtral B=256 gate/up: 4x fewer MFMAs), and stages only the rows used.
template <int T, int WM, int NA>
DEVI void lds_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, act_t* lds,
                   const int* xm, const int* ym) {
  constexpr int MTW = 4;                 // 16-row activation tiles per wave (at most)
  constexpr int WN = 8 / WM;
  constexpr int NTW = 8 / WN;            // 16-row weight tiles per wave
  constexpr int BM = WM * MTW * 16;
  constexpr int XS = BM * 64, WSZ = 128 * 64;    // f16 elements per buffer
  // 16-B x chunks staged per thread per quarter: 64-row groups up to the NA*WM tiles in use
  constexpr int NXU = (NA * WM * 16 + 63) / 64;
  static_assert(NA >= 1 && NA <= MTW && NXU * 512 <= BM * 8, "bad active-tile count");
  act_t* Xs = lds;                       // [2][BM][64]
  act_t* Ws = lds + 2 * XS;              // [2][128][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  const WDesc W{S.w, S.rows, S.K};
  const int nb = S.K >> 8;
  const int sb0 = (nb * kslice) / ks, sb1 = (nb * (kslice + 1)) / ks;
  const int sbl = max(sb1 - 1, sb0);
  const int M = a.M;
  const int drow = min(row0 + wave * 16 + r, S.rows - 1);   // this wave's dequant rows (clamped)

  // 32x32x16 MFMA tiles (variant): the wave's 64 x (128*WM/8) output as (MTW/2) x (NTW/2) 32x32
  // accumulators; blocks with a single 16-row weight tile per wave keep 16x16x32
  constexpr bool M32 = NLS_GEMM_MFMA32 && NTW >= 2 && NA == MTW;
  constexpr int MT2 = M32 ? MTW / 2 : 1, NT2 = M32 ? NTW / 2 : 1;
  f32x16 acc32[MT2][NT2];
  f32x4 acc[M32 ? 1 : NA][M32 ? 1 : NTW];
  if constexpr (M32) {
#pragma unroll
    for (int i = 0; i < MT2; ++i)
#pragma unroll
      for (int j = 0; j < NT2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[i][j][e] = 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int r32 = lane & 31, h32 = lane >> 5;

  // activation register ring: the quarter stored into LDS at step j was loaded XR steps earlier. vmcnt
  // retires loads in issue order, so the first x load issued after a raw-weight load bounds how long
  // that HBM load may take: XR = 4 gives it 5 quarter steps (XR = 1: 2). Four stages where registers
  // allow (<= 2 chunks per thread: every block of <= 128 rows, i.e. MoE experts and small batches).
  constexpr int XR = NXU <= 2 ? 4 : 1;
  u32x4 xr[XR][NXU];
  // the activation row each thread stages (fixed for the whole K loop); rows >= M only feed
  // outputs that are never stored: clamp, never branch. xm: MoE gather (block-local row -> x row)
  int xrow[NXU];
#pragma unroll
  for (int u = 0; u < NXU; ++u) {
    const int row = min((int)((threadIdx.x + 512 * u) >> 3), M - 1);
    xrow[u] = xm ? xm[row] : row;
  }
  auto load_x = [&](int st, int sb, int q) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NXU; ++u) {
      const int ch = (threadIdx.x + 512 * u) & 7;
      xr[st][u] = ld16(a.x + (size_t)xrow[u] * a.ldx + sb * 256 + q * 64 + ch * 8);
    }
  };
  auto store_x = [&](int st, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NXU; ++u) {
      const int idx = threadIdx.x + 512 * u, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<u32x4*>(Xs + buf * XS + row * 64 + ((ch ^ (row & 7)) << 3)) = xr[st][u];
    }
  };
  typedef typename RawOf<T>::type Raw;
  typedef typename ScOf<T>::type Sc;
  // One quarter step: dequantise W quarter `qn` of `rw` into buffer buf^1 and run the 32 MFMAs
  // of buffer buf. Program order = issue order wanted: both fragments' VALU first (independent
  // of the MFMAs, so the scheduler interleaves them into the MFMA stream), the K-step's LDS
  // reads before this step's W writes (the writes go to the other buffer).
  auto step_mma = [&](const Raw& rw, const Sc& sc, int qn, int buf) __attribute__((always_inline)) {
    const act_t* xb = Xs + buf * XS;
    const act_t* wb = Ws + buf * WSZ;
    act_t* wn_ = Ws + (buf ^ 1) * WSZ + (wave * 16 + r) * 64;
    f16x8 f[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) f[s] = frag_t<T>(rw, sc, 2 * qn + s);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int co = ((4 * s + g) ^ (r & 7)) << 3;
      if constexpr (M32) {
      // two K-steps of 16: lane half h32 reads 16-B chunk 4s + 2kk + h32 of its row (row & 7 == r32 & 7)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c2 = ((4 * s + 2 * kk + h32) ^ (r32 & 7)) << 3;
        f16x8 A[MT2], B[NT2];
#pragma unroll
        for (int i = 0; i < MT2; ++i)
          A[i] = *reinterpret_cast<const f16x8*>(xb + (wm * MTW * 16 + 32 * i + r32) * 64 + c2);
#pragma unroll
        for (int j = 0; j < NT2; ++j)
          B[j] = *reinterpret_cast<const f16x8*>(wb + (wn * NTW * 16 + 32 * j + r32) * 64 + c2);
        if (kk == 0) *reinterpret_cast<f16x8*>(wn_ + co) = f[s];
#if NLS_GEMM_SETPRIO
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int i = 0; i < MT2; ++i)
#pragma unroll
          for (int j = 0; j < NT2; ++j) acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[i], B[j], acc32[i][j], 0, 0, 0);
#if NLS_GEMM_SETPRIO
        __builtin_amdgcn_s_setprio(0);
#endif
      }
      } else {
      f16x8 A[NA], B[NTW];
#pragma unroll
      for (int i = 0; i < NA; ++i) A[i] = *reinterpret_cast<const f16x8*>(xb + ((i * WM + wm) * 16 + r) * 64 + co);
#pragma unroll
      for (int j = 0; j < NTW; ++j) B[j] = *reinterpret_cast<const f16x8*>(wb + (wn * NTW * 16 + 16 * j + r) * 64 + co);
      *reinterpret_cast<f16x8*>(wn_ + co) = f[s];
#if NLS_GEMM_SETPRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16(A[i], B[j], acc[i][j]);
#if NLS_GEMM_SETPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      }
    }
  };
  auto deq_w = [&](const Raw& rw, const Sc& sc, int q, int buf) __attribute__((always_inline)) {
    const int row = wave * 16 + r;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const f16x8 f = frag_t<T>(rw, sc, 2 * q + s);
      *reinterpret_cast<f16x8*>(Ws + buf * WSZ + row * 64 + (((4 * s + g) ^ (r & 7)) << 3)) = f;
    }
  };

  Raw rA, rB;
  Sc sA, sB;
  if (sb0 < sb1) {
    rA = load_raw<T, true>(W, drow, sb0, g);
    rB = load_raw<T, true>(W, drow, min(sb0 + 1, sbl), g);
    load_x(0, sb0, 0);
#pragma unroll
    for (int t = 1; t < XR; ++t) load_x(t, min(sb0 + t / 4, sbl), t % 4);   // quarters 1 .. XR-1
    prep_sc<T>(rA, g, sA);
    store_x(0, 0);
    deq_w(rA, sA, 0, 0);
    load_x(0, min(sb0 + XR / 4, sbl), XR % 4);                                // quarter XR
  }
  __syncthreads();
  // One quarter step qq (0..3) of super-block sb; jj = quarter index within the unrolled pair of
  // super-blocks (register stage (jj + 1) % XR holds quarter jj + 1). Buffer parity = quarter & 1.
  // Every load is unconditional (indices clamped): a conditional load breaks hipcc's vmcnt
  // bookkeeping (qgemv_impl.h). Each step: write the x registers of the next quarter into LDS,
  // re-issue that stage's load XR quarters ahead at once (sched_barrier: hipcc would otherwise sink
  // it to the end of the step), then the dequant of the next W quarter + this quarter's MFMAs.
  auto qstep = [&](Raw& rc, Sc& sc, Raw& rn, Sc& sn, int sb, int qq, int jj) __attribute__((always_inline)) {
    const int st = (jj + 1) % XR;
    store_x(st, (qq + 1) & 1);
    const int lq = qq + 1 + XR;
    load_x(st, min(sb + lq / 4, sbl), lq % 4);
    __builtin_amdgcn_sched_barrier(0);
    if (qq < 3) {
      step_mma(rc, sc, qq + 1, qq & 1);
      if (qq == 2) rc = load_raw<T, true>(W, drow, min(sb + 2, sbl), g);   // last use of rc: 2 super-blocks ahead
    } else {                                                               // quarter 0 of the next super-block
      prep_sc<T>(rn, g, sn);
      step_mma(rn, sn, 0, 1);
    }
    __syncthreads();
  };
  int sb = sb0;
  for (; sb + 1 < sb1; sb += 2) {
    qstep(rA, sA, rB, sB, sb, 0, 0);
    qstep(rA, sA, rB, sB, sb, 1, 1);
    qstep(rA, sA, rB, sB, sb, 2, 2);
    qstep(rA, sA, rB, sB, sb, 3, 3);
    qstep(rB, sB, rA, sA, sb + 1, 0, 4);
    qstep(rB, sB, rA, sA, sb + 1, 1, 5);
    qstep(rB, sB, rA, sA, sb + 1, 2, 6);
    qstep(rB, sB, rA, sA, sb + 1, 3, 7);
  }
  if (sb < sb1) {
    qstep(rA, sA, rB, sB, sb, 0, 0);
    qstep(rA, sA, rB, sB, sb, 1, 1);
    qstep(rA, sA, rB, sB, sb, 2, 2);
    qstep(rA, sA, rB, sB, sb, 3, 3);
  }

  // ---- epilogue from the accumulators ------------------------------------------------------------
  // 16x16 tiles: lane holds weight row rbase + 16j + r and activation rows 16(i*WM + wm) + 4g + e;
  // 32x32 tiles: weight row rbase + 32j + r32, activation rows mbase + 32i + (e&3) + 8(e>>2) + 4 h32
  const int rbase = row0 + wn * NTW * 16, mbase = wm * MTW * 16;
  constexpr int NJ = M32 ? NT2 : NTW, NI = M32 ? MT2 : NA, NE = M32 ? 16 : 4;
  constexpr int RED_LANES = M32 ? 32 : 16;       // lanes sharing an activation row (argmax reduction)
  auto wrow = [&](int j) { return M32 ? rbase + 32 * j + r32 : rbase + 16 * j + r; };
  auto arow = [&](int i, int e) {
    return M32 ? mbase + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h32 : (i * WM + wm) * 16 + 4 * g + e;
  };
  auto accv = [&](int i, int j, int e) -> float {
    if constexpr (M32) return acc32[i][j][e];
    else return acc[i][j][e];
  };
  if (ks > 1) {
    const int ntot = a.pad;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int row = wrow(j);
      if (row >= S.rows) continue;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int b = arow(i, e);
          if (b >= M) continue;
          if (ym)        // mapped split-K: slab row = the token's y row, columns shared by every expert
            ws[((size_t)kslice * a.mtot + ym[b]) * ntot + S.ycol + row] = accv(i, j, e);
          else
            ws[((size_t)kslice * a.mtot + a.m0 + b) * ntot + S.tile_begin_col + row] = accv(i, j, e);
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int row = wrow(j);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int b = arow(i, e);
        const float v = accv(i, j, e) * a.alpha;
        if (a.epi == EPI_SWIGLU) {
          // interleaved [g0..g7, u0..u7] per 16 weight rows: the partner row is lane ^ 8 (same b)
          const float u = __shfl_xor(v, 8, 64);
          if ((row & 8) == 0 && b < M && row < S.rows) {
            const int n = S.ycol + ((row & ~15) >> 1) + (row & 7);
            const int yb = ym ? ym[b] : b;
            reinterpret_cast<act_t*>(a.y)[(size_t)yb * a.ldy + n] = (act_t)(silu(v) * u);
          }
          continue;
        }
        if (b < M && row < S.rows) {
          const size_t off = (size_t)(ym ? ym[b] : b) * a.ldy + S.ycol + row;
          if (a.epi == EPI_F32) reinterpret_cast<float*>(a.y)[off] = v;
          else if (a.epi == EPI_ADD_F32) reinterpret_cast<float*>(a.y)[off] += v;
          else if (a.epi == EPI_ACT) reinterpret_cast<act_t*>(a.y)[off] = (act_t)v;
        }
      }
    }
  }
  if (a.argmax) {
    // greedy arg-max: max over the lane's weight rows, then the lanes sharing an activation row, then
    // the workgroup's waves through LDS (free after the main loop) -> ONE global atomic per
    // activation row per workgroup (vs one per 16 rows: 1M contended 64-bit atomics on the
    // 128K-row lm_head otherwise)
    unsigned long long* red = reinterpret_cast<unsigned long long*>(lds);
    __syncthreads();
    for (int idx = threadIdx.x; idx < BM; idx += 512) red[idx] = 0ull;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        unsigned long long k = 0ull;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = wrow(j);
          const unsigned long long kj = (row < S.rows) ? argmax_key(accv(i, j, e) * a.alpha, S.ycol + row) : 0ull;
          k = kj > k ? kj : k;
        }
#pragma unroll
        for (int o = 1; o < RED_LANES; o <<= 1) {
          const unsigned long long ok = __shfl_xor(k, o, 64);
          k = ok > k ? ok : k;
        }
        if ((lane & (RED_LANES - 1)) == 0) atomicMax(red + arow(i, e), k);
      }
    __syncthreads();
    for (int idx = threadIdx.x; idx < M; idx += 512) atomicMax(a.argmax + idx, red[idx]);
  }
}

template <int T, int WM>
DEVI void lds_tile_na(int na, const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, act_t* lds,
                      const int* xm, const int* ym) {
  switch (na) {
    case 1: lds_tile<T, WM, 1>(S, row0, kslice, ks, a, ws, lds, xm, ym); break;
    case 2: lds_tile<T, WM, 2>(S, row0, kslice, ks, a, ws, lds, xm, ym); break;
    case 3: lds_tile<T, WM, 3>(S, row0, kslice, ks, a, ws, lds, xm, ym); break;
    default: lds_tile<T, WM, 4>(S, row0, kslice, ks, a, ws, lds, xm, ym); break;
  }
}

template <int WM, int KSET>
__global__ __launch_bounds__(512) void qmm_lds_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                      int nmb) {
  extern __shared__ __attribute__((aligned(16))) act_t lds[];
  constexpr int BM = WM * 64;
  // (tile, m-block, k-slice) with all m-blocks and k-slices of a tile on one XCD
  const int i = blockIdx.x, xcd = i & 7, j = i >> 3;
  const int kslice = j % ks;
  const int mb = (j / ks) % nmb;
  const int tile = (j / ks / nmb) * 8 + xcd;
  if (tile >= ntiles) return;
  const int m0 = mb * BM;
  Seg S = segs.s[0];
#pragma unroll
  for (int s = 1; s < 8; ++s)
    if (s < segs.nseg && tile >= segs.s[s].tile_begin) S = segs.s[s];
  // MoE grouped GEMM: the expert's routed-row count lives on the device; m-blocks past it exit
  // before reading any weights (the grid is sized for the worst case, every token on one expert)
  const int mrows = S.mcount ? min(*S.mcount, a.M) : a.M;
  if (m0 >= mrows) return;
  const int* xm = S.xmap ? S.xmap + m0 : nullptr;
  const int* ym = S.ymap ? S.ymap + m0 : nullptr;
  a.m0 = m0;
  if (!xm) a.x += (size_t)m0 * a.ldx;
  const size_t esz = (a.epi == EPI_F32 || a.epi == EPI_ADD_F32 || a.epi == EPI_ARGMAX) ? 4 : 2;
  if (!ym) a.y = (char*)a.y + (size_t)m0 * a.ldy * esz;
  if (a.argmax) a.argmax += m0;
  a.M = min(BM, mrows - m0);
  const int row0 = (tile - S.tile_begin) * 128;
  // active 16-row tiles per wave (block-uniform): ceil(ceil(M / 16) / WM)
  const int na = NLS_GEMM_MFMA32 ? 4 : min(4, ((a.M + 15) / 16 + WM - 1) / WM);
  if constexpr (KSET == 0) {
    switch (S.type) {
      case QT_Q4_K: lds_tile_na<QT_Q4_K, WM>(na, S, row0, kslice, ks, a, ws, lds, xm, ym); break;
      case QT_Q6_K: lds_tile_na<QT_Q6_K, WM>(na, S, row0, kslice, ks, a, ws, lds, xm, ym); break;
      default: break;
    }
  } else {
    switch (S.type) {
      case QT_Q5_K: lds_tile_na<QT_Q5_K, WM>(na, S, row0, kslice, ks, a, ws, lds, xm, ym); break;
      case QT_Q6_K: lds_tile_na<QT_Q6_K, WM>(na, S, row0, kslice, ks, a, ws, lds, xm, ym); break;
      case QT_Q8_0: lds_tile_na<QT_Q8_0, WM>(na, S, row0, kslice, ks, a, ws, lds, xm, ym); break;
      default: break;
    }
  }
}

template <int WM, int KSET>
int launch_lds_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  constexpr int BM = WM * 64;
  const int nmb = (a.M + BM - 1) / BM;
  const size_t lds = (size_t)2 * (BM + 128) * 64 * sizeof(act_t);
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)qmm_lds_kernel<WM, KSET>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL((qmm_lds_kernel<WM, KSET>), dim3(grid), dim3(512), lds, st, sl, a, ks, ws, ntiles, nmb);
  return (int)hipGetLastError();
}

template <int KSET>
int launch_lds_kset(int wm, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  if (wm == 4) return launch_lds_t<4, KSET>(sl, ntiles, ks, ws, a, st);
  if (wm == 2) return launch_lds_t<2, KSET>(sl, ntiles, ks, ws, a, st);
  if (wm == 1) return launch_lds_t<1, KSET>(sl, ntiles, ks, ws, a, st);   // 64-row blocks (MoE experts)
  return -1;
}

int launch_lds_k0(int wm, const SegList&, int, int, float*, const GemvArgs&, hipStream_t);
int launch_lds_k1(int wm, const SegList&, int, int, float*, const GemvArgs&, hipStream_t);

}  // namespace nls_gemm
