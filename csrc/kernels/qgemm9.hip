// Quantised large-M GEMM on the weights' GGUF tile-blocks, "mode 9" of the qgemv dispatcher (gfx950).
//
//   y[m, n] (epilogue) alpha * sum_k x[m, k] * W[n, k]      x f16 [M, K], W K-quant tile-blocks (common.h)
//
// Why (the round-3 probes on the 8B gate|up at 512 rows, profiles/gemm_probes_r03.txt): the dense f16
// kernel of mode 8 takes 105 us, 99 us of it with the MFMAs switched off -- it is bound by what one CU
// pulls into LDS (~41 GB/s per CU at full load: 256 activation rows + 224 f16 weight rows per 32-deep
// K-step = 30 KiB). A 256 x 256 tile that streams the RAW Q4_K tile-blocks instead takes 16 + 4.5 KiB per
// K-step (Q6_K 16 + 6.6): 1.5x less intake for the same MFMA work; the dequantisation (the f16
// magic-number path of common.h, ~19 VALU per 8-value fragment) is 2 fragments per 32 MFMAs of a wave.
// Measured: 102 us on that shape, 70 us without MFMAs, 55 us with neither MFMAs nor DMA -- the
// activation fragment reads (16 ds_read_b128 per wave per K-step, 128 KiB per CU) and the per-stage
// barrier are now the floor; on par with hipBLASLt across the 8B shapes (0.86-1.07x), ahead of it on the
// down projection.
//
// Workgroup = 256 activation rows x 16*RT*NWV weight rows, NWV waves (8: two per SIMD, 4: one per SIMD with
// 512 registers); wave w owns weight rows 16*RT*w.. (RT 16-row tiles) against ALL 256 activation rows (16
// tiles of 16): RT fragments dequantised per K-step,
// 16 activation fragments read from LDS, 16*RT MFMAs (v_mfma_f32_16x16x32_f16, weights as the A
// operand: a lane ends with 4 consecutive output columns of one row -> 16-byte epilogue stores,
// SwiGLU's gate/up partner is lane ^ 32, as mode 8).
//   * activations: 32-deep stages [256][32] f16 (16 KiB) by LDS-DMA into an NS-deep ring (NS 5-7 by the
//     weight format's LDS share), chunks XOR-swizzled on the DMA source (conflict-free ds_read_b128);
//   * weights: the workgroup's 8*RT raw tile-blocks of ONE 256-deep super-block (Q4_K 2304 B each) in a
//     single LDS buffer: every wave pulls its RT blocks into registers at the super-block's first stage
//     (scales unpacked once), and the next super-block's blocks are DMA'd into the buffer one stage later
//     -- they land 7 stages before they are needed;
//   * one raw s_barrier per stage behind a COUNTED vmcnt (compile-time per stage position, the weight
//     DMA in flight included) certifies the NEXT stage, NS-3 stages stay in flight across it.
// Grid and split-K as modes 3 / 8: (tile, m-block, k-slice), all m-blocks and k-slices of a weight tile
// on ONE XCD (the tile's HBM bytes are fetched once per XCD L2).
#include "qgemm_dma.h"

// H9_PROBE builds speed-of-light variants (the round-3 probe harness): bit 0 = no MFMA (fragments still read), bit 1 = no
// DMA, bit 2 = no vmcnt waits, bit 3 = no dequantisation (raw bits as fragments). 0 in the library.
#ifndef H9_PROBE
#define H9_PROBE 0
#endif

namespace nls_q9 {
using namespace nls_gemv;
using nls_dma::glds16;
using nls_dma::lds_addr;

constexpr int LDS_MAX = 160 * 1024;

// NWV waves x RT weight tiles over BM activation rows (256; mode 12: 64, the MoE experts' routed rows):
// activation / raw-weight DMA instructions per wave per stage / super-block (NWV*RT tile-blocks), the ring depth
template <int T, int RT, int NWV, int BM = 256>
struct Geo {
  static constexpr int XS = BM * 64;                             // bytes of one activation stage [BM][32] f16
  static constexpr int XI = XS / 1024 / NWV;
  static_assert(XI >= 1 && XS % (1024 * NWV) == 0, "one stage must split evenly over the waves");
  static constexpr int TB = TileBytes<T>::v;
  static constexpr int NW = (RT * TB + 1023) / 1024;
  static constexpr int WL = NWV * NW * 1024;                     // weight buffer incl. pad lanes
  static constexpr int NS0 = (LDS_MAX - WL) / XS;
  static constexpr int NS = NS0 > 7 ? 7 : NS0;
  static constexpr int LDS = NS * XS + WL;
  static_assert(NS >= 4, "ring too shallow");
};

DEVI int swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

template <int N>
DEVI void wait_vm() {
  if constexpr (H9_PROBE & 4) return;
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
DEVI void wait_vm_lgkm0() {
  if constexpr (H9_PROBE & 4) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return;
  }
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(N) : "memory");
}

// one 16-row tile's raw super-block from its LDS copy (the global tile-block's byte layout)
template <int T>
DEVI typename RawOf<T>::type raw_lds(const uint8_t* b, int g, int r) {
  const int l = 16 * g + r;
  typename RawOf<T>::type x;
  if constexpr (T == QT_Q4_K) {
    x.hdr = ld16(b + 16 * r);
    x.p0 = ld16(b + 256 + 16 * l);
    x.p1 = ld16(b + 1280 + 16 * l);
  } else if constexpr (T == QT_Q5_K) {
    x.hdr = ld16(b + 16 * r);
    x.qh = ld8(b + 256 + 8 * l);
    x.p0 = ld16(b + 768 + 16 * l);
    x.p1 = ld16(b + 1792 + 16 * l);
  } else if constexpr (T == QT_Q51) {
    x.dd = ld16(b + 32 * r);
    x.mm = ld16(b + 32 * r + 16);
    x.qh = ld8(b + 512 + 8 * l);
    x.p0 = ld16(b + 1024 + 16 * l);
    x.p1 = ld16(b + 2048 + 16 * l);
  } else if constexpr (T == QT_Q6_K) {
    x.qa = ld16(b + 16 * l);
    x.qb = ld16(b + 1024 + 16 * l);
    x.qh = ld16(b + 2048 + 16 * l);
    x.sc = ld16(b + 3072 + 16 * r);
    x.d = *reinterpret_cast<const uint16_t*>(b + 3328 + 2 * r);
  } else {   // Q8_0
#pragma unroll
    for (int p = 0; p < 4; ++p) x.q[p] = ld16(b + 1024 * p + 16 * l);
    x.d = ld16(b + 4096 + 16 * r);
  }
  return x;
}

// DMA instructions allowed in flight at the barrier of the stage at super-block position P, which
// certifies the NEXT stage (8s + P + 1): the NS-3 stages issued after it, plus the next super-block's
// weights when they went out after it (issued at P = 1 behind stage 8s + NS)
template <int NS, int NW, int XI, int P>
struct Cnt {
  static constexpr int v = (NS - 3) * XI + ((P >= 2 && P <= NS - 1) ? NW : 0);
};

template <int T, int RT, int NWV, int BM = 256>
DEVI void q9_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds,
                  const int* xm = nullptr, const int* ym = nullptr) {
  typedef Geo<T, RT, NWV, BM> G;
  constexpr int NS = G::NS, NW = G::NW, TB = G::TB, XI = G::XI, XS = G::XS;
  constexpr int MT = BM / 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int nb = S.K >> 8;
  const int sb0 = (nb * kslice) / ks, sb1 = (nb * (kslice + 1)) / ks;
  const int nst = 8 * (sb1 - sb0);
  const int M = a.M;
  const int ntile = (S.rows + 15) >> 4;
  const int tile0 = row0 >> 4;
  uint8_t* Wl = lds + NS * XS;

  // ---- DMA sources. Activations: instruction i of wave w covers rows 16(XI w + i) .. +15, lane L ->
  // row + (L >> 2), physical chunk L & 3 <- logical chunk (L & 3) ^ swz(row)
  const int lc = (lane & 3) ^ swz(lane >> 2);
  const act_t* xsrc[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int row = min(16 * (XI * wave + i) + (lane >> 2), M - 1);   // rows >= M: clamped, never stored
    const int xr = xm ? xm[row] : row;                                 // mapped rows: the routed token's row
    xsrc[i] = a.x + (size_t)xr * a.ldx + (size_t)sb0 * 256 + lc * 8;
  }
  // raw weights: byte b of the packed buffer <- tile-block b / TB (clamped to the segment), byte b % TB;
  // the sources are recomputed per super-block (registers are the scarce resource here, not VALU)
  auto wsrc = [&](int i) __attribute__((always_inline)) {
    // the lane id through volatile asm: keeps the compiler from hoisting NW 64-bit pointers out of the
    // loop (they end up in scratch, and the reload's vmcnt(0) drains the whole DMA pipeline)
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    int b = ((NW * wave + i) << 10) + 16 * ln;
    if (b >= NWV * RT * TB) b = 0;                     // pad lanes: any valid source, lands in the pad
    const int lt = b / TB;
    const int t = min(tile0 + lt, ntile - 1);
    return S.w + ((size_t)t * nb + sb0) * TB + (b - lt * TB);
  };
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint32_t xdst = base + (uint32_t)(XI * wave) * 1024u;
  const uint32_t wdst = base + NS * XS + (uint32_t)(NW * wave) * 1024u;
  auto dma_x = [&](int j) __attribute__((always_inline)) {     // stage j (clamped) -> ring slot j % NS
    if constexpr (H9_PROBE & 2) return;
    const int jj = min(j, nst - 1);
    const uint32_t so = (uint32_t)(j % NS) * XS;
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + jj * 32, xdst + so + i * 1024);
  };
  auto dma_w = [&](int s) __attribute__((always_inline)) {     // super-block sb0 + s (clamped)
    if constexpr (H9_PROBE & 2) return;
    const size_t off = (size_t)min(s, sb1 - sb0 - 1) * TB;
#pragma unroll
    for (int i = 0; i < NW; ++i) glds16(wsrc(i) + off, wdst + i * 1024);
  };

  f32x4 acc[RT][MT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  typename RawOf<T>::type raw[RT];
  typename ScOf<T>::type sc[RT];
  const int fro = r * 64 + ((g ^ swz(r)) << 4);

  // activation fragments in groups of 4 (16 rows each): while a group's 4 RT MFMAs run, the next group's
  // 4 ds_read_b128 are in flight; group 0 of stage j+1 is requested at the end of stage j (its barrier
  // certified stage j+1), so no stage starts on an exposed LDS latency
  f16x8 XA[4], XB[4];
  auto rdg = [&](f16x8* X, int j, int grp) __attribute__((always_inline)) {
    const uint8_t* b = lds + (j % NS) * XS + fro + grp * 4096;
#pragma unroll
    for (int q = 0; q < 4; ++q) X[q] = *reinterpret_cast<const f16x8*>(b + q * 1024);
  };
  auto mmg = [&](const f16x8* wf, const f16x8* X, int grp) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if constexpr (H9_PROBE & 1) asm volatile("" ::"v"(wf[i]), "v"(X[q]));
        else acc[i][4 * grp + q] = mfma16(wf[i], X[q], acc[i][4 * grp + q]);
      }
  };
  // weight fragments are software-pipelined too: stage j's MFMA groups carry the dequantisation of stage
  // j+1's RT fragments (~19 VALU each) in their issue gaps -- two 4-cycle VALU fit beside each
  // 16-cycle MFMA (MI355X_MICROARCH.md 'vector-instruction ISSUE cost'), so the dequantisation is not
  // paid in front of the MFMAs by both waves of a SIMD at once
  f16x8 wf[RT], wn[RT];
  auto frag = [&](int i, int t) __attribute__((always_inline)) {
    if constexpr ((H9_PROBE & 8) && T == QT_Q4_K) return __builtin_bit_cast(f16x8, u32x4{raw[i].p0[t & 3], raw[i].p1[t & 3], 0u, 0u});
    else return frag_t<T>(raw[i], sc[i], t);
  };
  // group grp dequantises the next stage's fragments i = grp, grp + 4, ...
  auto fillw = [&](int grp, int pn) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < RT; ++i)
      if (i % 4 == grp) wn[i] = frag(i, pn);
  };
  // MFMA group `grp` with VALU work `fill` interleaved: one MFMA, then up to 3 VALU, ...
  auto mmv = [&](const f16x8* X, int grp, auto fill) __attribute__((always_inline)) {
    fill();
    mmg(wf, X, grp);
#pragma unroll
    for (int k = 0; k < 4 * RT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // one stage: 16 activation fragments (4 groups), 16 RT MFMAs; `pn` = the next stage's K-step
  auto stage = [&](int j, int pn) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
    rdg(XB, j, 1);
    __builtin_amdgcn_sched_barrier(0);
    mmv(XA, 0, [&]() __attribute__((always_inline)) { fillw(0, pn); });
    rdg(XA, j, 2);
    __builtin_amdgcn_sched_barrier(0);
    mmv(XB, 1, [&]() __attribute__((always_inline)) { fillw(1, pn); });
    rdg(XB, j, 3);
    __builtin_amdgcn_sched_barrier(0);
    mmv(XA, 2, [&]() __attribute__((always_inline)) { fillw(2, pn); });
    rdg(XA, j + 1, 0);                               // next stage's group 0 (a harmless re-read past the end)
    __builtin_amdgcn_sched_barrier(0);
    mmv(XB, 3, [&]() __attribute__((always_inline)) { fillw(3, pn); });
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int i = 0; i < RT; ++i) wf[i] = wn[i];
  };
  // BM 64 (one group of 4 activation tiles per stage): the stages alternate between XA and XB, each stage
  // requesting the next one's fragments before its MFMAs, and its MFMAs carry ALL the next stage's weight
  // dequantisation
  auto stage64 = [&](int j, int pn, auto ODD) __attribute__((always_inline)) {
    constexpr bool odd = decltype(ODD)::value;
    f16x8* cur = odd ? XB : XA;
    f16x8* nxt = odd ? XA : XB;
    __builtin_amdgcn_s_setprio(1);
    rdg(nxt, j + 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    mmv(cur, 0, [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < RT; ++i) wn[i] = frag(i, pn);
    });
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int i = 0; i < RT; ++i) wf[i] = wn[i];
  };

  if (nst > 0) {
    dma_w(0);
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) dma_x(s);
    wait_vm<(NS - 2) * XI>();                        // W(sb0) and stage 0 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < RT; ++i) raw[i] = raw_lds<T>(Wl + (RT * wave + i) * TB, g, r);
#pragma unroll
    for (int i = 0; i < RT; ++i) prep_sc<T>(raw[i], g, sc[i]);
#pragma unroll
    for (int i = 0; i < RT; ++i) wf[i] = frag(i, 0);
    rdg(XA, 0, 0);
    for (int s = 0; s < sb1 - sb0; ++s) {
      const int j0 = 8 * s;
      // stage j0+p: certify stage j0+p+1 (counted vmcnt + barrier), refill the slot of stage j0+p-1,
      // compute stage j0+p while dequantising stage j0+p+1's weight fragments. p = 1: every wave's raw
      // reads are done (lgkmcnt(0) before the barrier) -> the next super-block's weights go out; they
      // have landed by stage 7's barrier (issued behind stage j0+NS, NS <= 7), which is where the
      // registers switch to them (stage 7's own fragments were dequantised during stage 6)
      auto step = [&](auto P) __attribute__((always_inline)) {
        constexpr int p = decltype(P)::value;
        if constexpr (p == 1) wait_vm_lgkm0<Cnt<NS, NW, XI, p>::v>();
        else wait_vm<Cnt<NS, NW, XI, p>::v>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        dma_x(j0 + p + NS - 1);
        if constexpr (p == 1) dma_w(s + 1);
        if constexpr (p == 7) {
#pragma unroll
          for (int i = 0; i < RT; ++i) raw[i] = raw_lds<T>(Wl + (RT * wave + i) * TB, g, r);
#pragma unroll
          for (int i = 0; i < RT; ++i) prep_sc<T>(raw[i], g, sc[i]);
        }
        if constexpr (BM == 64)
          stage64(j0 + p, (p + 1) & 7, std::integral_constant<bool, (p & 1) != 0>{});
        else
          stage(j0 + p, (p + 1) & 7);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      step(std::integral_constant<int, 4>{});
      step(std::integral_constant<int, 5>{});
      step(std::integral_constant<int, 6>{});
      step(std::integral_constant<int, 7>{});
    }
  }
  wait_vm<0>();                                       // drain the clamped tail DMAs
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: lane holds weight rows nb0 + 16i + 4g + e and activation row 16m + r (mapped: output row
  // ym[16m + r]; mapped split-K slabs are indexed by the output row, one shared segment column range)
  const int g4 = 4 * g;
  const int nb0 = row0 + wave * RT * 16;
  auto yrow = [&](int mm) __attribute__((always_inline)) { return ym ? ym[mm] : mm; };
  if (ks > 1 || a.epi == EPI_SLABS) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const int n = nb0 + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int mm = 16 * m + r;
        if (mm >= M) continue;
        const size_t srow = ym ? (size_t)ym[mm] : (size_t)(a.m0 + mm);
        const int scol = ym ? n : S.tile_begin_col + n;
        *reinterpret_cast<f32x4*>(ws + ((size_t)kslice * a.mtot + srow) * a.pad + scol) = acc[i][m];
      }
    }
    return;
  }
  const float al = a.alpha;
  if (a.epi == EPI_SWIGLU) {
    // interleaved [g0..g7 | u0..u7] per 16 weight rows: lanes 0-31 hold gate rows, lanes 32-63 the up rows
#pragma unroll
    for (int i = 0; i < RT; ++i) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4 u;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = __shfl_xor(acc[i][m][e] * al, 32, 64);
        const int n16 = nb0 + 16 * i, mm = 16 * m + r;
        if (lane < 32 && mm < M && n16 < S.rows) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          h4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (_Float16)(silu(acc[i][m][e] * al) * u[e]);
          *reinterpret_cast<h4*>(reinterpret_cast<act_t*>(a.y) + (size_t)yrow(mm) * a.ldy + S.ycol + (n16 >> 1) + g4) = o;
        }
      }
    }
    return;
  }
  if (a.epi != EPI_ARGMAX) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const int n = nb0 + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int mm = 16 * m + r;
        if (mm >= M) continue;
        const f32x4 v = acc[i][m] * al;
        if (a.epi == EPI_ACT) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<h4*>(reinterpret_cast<act_t*>(a.y) + (size_t)yrow(mm) * a.ldy + S.ycol + n) =
              h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
          f32x4* q = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.y) + (size_t)yrow(mm) * a.ldy + S.ycol + n);
          *q = a.epi == EPI_ADD_F32 ? *q + v : v;
        }
      }
    }
  }
  if (a.argmax) {
    // per activation row: max over the lane's rows, then the 4 lanes of the row (l ^ 16, l ^ 32)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      unsigned long long k = 0ull;
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = nb0 + 16 * i + g4 + e;
          const unsigned long long kk = n < S.rows ? argmax_key(acc[i][m][e] * al, S.ycol + n) : 0ull;
          k = kk > k ? kk : k;
        }
      unsigned long long o = __shfl_xor(k, 16, 64);
      k = o > k ? o : k;
      o = __shfl_xor(k, 32, 64);
      k = o > k ? o : k;
      const int mm = 16 * m + r;
      if (lane < 16 && mm < M) atomicMax(a.argmax + mm, k);
    }
  }
}

// the formats of one kernel type-set (dispatcher's kset: 0 = Q4_K/Q6_K, 1 = Q5_K/Q6_K/Q8_0,
// 3 = Q51/Q6_K/Q8_0) and the LDS they need
template <int KSET, int RT, int NWV, int BM>
constexpr int kset_lds() {
  return KSET == 0 ? (Geo<QT_Q4_K, RT, NWV, BM>::LDS > Geo<QT_Q6_K, RT, NWV, BM>::LDS ? Geo<QT_Q4_K, RT, NWV, BM>::LDS
                                                                                      : Geo<QT_Q6_K, RT, NWV, BM>::LDS)
                   : LDS_MAX;
}

// NWV = 8: two waves per SIMD (256 registers); NWV = 4: one wave per SIMD with up to 512 registers, so a
// wave holds 4 weight tiles x 16 activation tiles of accumulators (half the LDS reads per MFMA).
// BM = 64 (mode 12, the MoE experts' grouped GEMM): segments may be mapped -- each expert's routed rows are
// gathered through xmap and scattered through ymap, and m-blocks past the expert's device-side row count
// exit before reading any weights (the grid is sized for every token on one expert)
template <int KSET, int RT, int NWV, int BM>
__global__ __launch_bounds__(64 * NWV, 1) void qgemm9_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                          int nmb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t q9lds[];
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
  // mapped rows only at BM 64 (the dispatcher refuses them for mode 9): the 256-row build keeps mode 9's code
  const int mrows = (BM == 64 && S.mcount) ? min(*S.mcount, a.M) : a.M;
  if (m0 >= mrows) return;
  const int* xm = (BM == 64 && S.xmap) ? S.xmap + m0 : nullptr;
  const int* ym = (BM == 64 && S.ymap) ? S.ymap + m0 : nullptr;
  a.m0 = m0;
  if (!xm) a.x += (size_t)m0 * a.ldx;
  const size_t esz = (a.epi == EPI_F32 || a.epi == EPI_ADD_F32 || a.epi == EPI_ARGMAX) ? 4 : 2;
  if (!ym) a.y = (char*)a.y + (size_t)m0 * a.ldy * esz;
  if (a.argmax) a.argmax += m0;
  a.M = min(BM, mrows - m0);
  const int row0 = (tile - S.tile_begin) * 16 * RT * NWV;
  if constexpr (KSET == 0) {
    if (S.type == QT_Q4_K) q9_tile<QT_Q4_K, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
    else q9_tile<QT_Q6_K, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
  } else if constexpr (KSET == 1) {
    if (S.type == QT_Q5_K) q9_tile<QT_Q5_K, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
    else if (S.type == QT_Q8_0) q9_tile<QT_Q8_0, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
    else q9_tile<QT_Q6_K, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
  } else {
    if (S.type == QT_Q51) q9_tile<QT_Q51, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
    else if (S.type == QT_Q8_0) q9_tile<QT_Q8_0, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
    else q9_tile<QT_Q6_K, RT, NWV, BM>(S, row0, kslice, ks, a, ws, q9lds, xm, ym);
  }
}

template <int KSET, int RT, int NWV, int BM>
int launch_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  constexpr int lds = kset_lds<KSET, RT, NWV, BM>();
  const int nmb = (a.M + BM - 1) / BM;
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)qgemm9_kernel<KSET, RT, NWV, BM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds) != hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL((qgemm9_kernel<KSET, RT, NWV, BM>), dim3(grid), dim3(64 * NWV), lds, st, sl, a, ks, ws, ntiles,
                     nmb);
  return (int)hipGetLastError();
}

template <int KSET>
int launch_k(int waves, int rt, int bm, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a,
             hipStream_t st) {
  // bm 64 (the round-5 "mode 12" MoE variant, 2.6-3.1x slower than mode 2 on Mixtral's experts) is no longer
  // instantiated: the template keeps the geometry, the default build does not carry the code
  if (bm != 256) return -1;
  if (waves == 4 && rt == 2) return launch_t<KSET, 2, 4, 256>(sl, ntiles, ks, ws, a, st);
  if (waves == 8 && rt == 2) return launch_t<KSET, 2, 8, 256>(sl, ntiles, ks, ws, a, st);
  if (waves == 8 && rt == 1) return launch_t<KSET, 1, 8, 256>(sl, ntiles, ks, ws, a, st);
  return -1;
}

// waves x rt weight tiles of 16 rows per workgroup: (4, 2) | (8, 2) | (8, 1) (4 x 4 spills: 256 accumulators
// plus the pipelined fragments exceed 512 registers) over 256 activation rows; kset as the dispatcher's
int launch_q9(int kset, int waves, int rt, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a,
              hipStream_t st, int bm) {
  if (kset == 0) return launch_k<0>(waves, rt, bm, sl, ntiles, ks, ws, a, st);
  if (kset == 1) return launch_k<1>(waves, rt, bm, sl, ntiles, ks, ws, a, st);
  if (kset == 3) return launch_k<3>(waves, rt, bm, sl, ntiles, ks, ws, a, st);
  return -1;
}

}  // namespace nls_q9
