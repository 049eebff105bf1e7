// Large-M quantised GEMM, LDS-DMA edition ("mode 3"), gfx950.
//
//   y[m, n] = alpha * sum_k x[m, k] * W[n, k]      (W in GGUF K-quant blocks, x f16)
//
// Why (PMC of the mode-2 kernel, qgemm_impl.h, gate/up M=256): 32 % MFMA busy, 1/3 of the wave
// cycles parked at waits/barriers, 3.4 VALU per MFMA. Its activation tile travels
// global -> VGPR -> ds_write (32 KiB of ds_write per 64-deep quarter, more LDS-store cycles than the
// quarter's MFMA cycles) and the dequantised weights take another 16 KiB ds_write round.
// Here NOTHING is written to LDS through VGPRs:
//   * both operands arrive by LDS-DMA (`global_load_lds_dwordx4`, 1 KiB per wave-instruction,
//     issued as inline asm so hipcc neither counts nor drains them): the activation quarter
//     [BM][64] f16 into a 3-deep ring (XOR-swizzled by permuting the per-lane SOURCE chunk,
//     the DMA writes lane-linearly), and the RAW quantised tile-blocks of the workgroup's
//     128 weight rows once per 256-deep super-block;
//   * every wave owns 32 weight rows (RT = 2 16-row tiles) x all BM activation rows (MT = BM/16
//     tiles): it reads its raw blocks from LDS once per super-block, dequantises one K-step
//     fragment per tile in registers (v2 tile layout + f16 magic-number dequant, common.h)
//     and feeds it as the B operand of MT MFMAs -> 1 fragment dequant per MT MFMAs
//     (about 1 VALU per MFMA at BM = 256) and 0.5 ds_read_b128 per MFMA;
//   * one raw s_barrier per quarter with a COUNTED vmcnt: quarter j+2 (and the next
//     super-block's weights) stay in flight across it (cdna_hip_programming.md §5
//     "Pipelining across barriers", 3-buffer span).
// 4 waves (one per SIMD, registers up to 512), 1 workgroup per CU. Grid and split-K as mode 2:
// (tile, m-block, k-slice) with every m-block and k-slice of a weight tile on one XCD.
#pragma once
#include "qgemv_impl.h"

#ifndef NLS_DMA_NA
#define NLS_DMA_NA 1     // 0: 96-row blocks multiply every tile (A/B builds)
#endif

namespace nls_dma {
using namespace nls_gemv;

// LDS byte address of a pointer into the dynamic LDS array
DEVI uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// 16 B per lane global -> LDS (dst = wave-uniform `lds_dst` + 16 * lane). Inline asm: invisible to
// hipcc's waitcnt pass (no vmcnt(0) before every ds_read); completion is counted by hand.
DEVI void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
template <int N>
DEVI void wait_vm_lgkm0() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(N) : "memory");
}

// raw weight DMA instructions per wave per super-block (8 tile-blocks per workgroup, 4 waves)
template <int T> struct DmaW { static constexpr int n = (8 * TileBytes<T>::v + 4095) / 4096; };

// raw super-block of one 16-row tile, read from its LDS copy (same byte layout as the global
// tile-block: common.h)
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
  } else {   // Q6_K
    x.qa = ld16(b + 16 * l);
    x.qb = ld16(b + 1024 + 16 * l);
    x.qh = ld16(b + 2048 + 16 * l);
    x.sc = ld16(b + 3072 + 16 * r);
    x.d = *reinterpret_cast<const uint16_t*>(b + 3328 + 2 * r);
  }
  return x;
}

template <int T, int MT>
DEVI void dma_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds,
                   const int* xm, const int* ym) {
  constexpr int RT = 2;
  constexpr int BM = MT * 16;
  constexpr int XS = BM * 128;                  // bytes per activation quarter [BM][64] f16
  constexpr int NX = BM / 32;                   // x DMA instructions per wave per quarter (8 rows each)
  constexpr int NW = DmaW<T>::n;                // raw-W DMA instructions per wave per super-block
  constexpr int TB = TileBytes<T>::v;
  uint8_t* Xs = lds;                            // [3][BM][64] f16, 16-B chunk c of row r at c ^ (r & 7)
  uint8_t* Wl = lds + 3 * XS;                   // 8 raw tile-blocks, packed (4 * NW KiB)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int nb = S.K >> 8;
  const int sb0 = (nb * kslice) / ks, sb1 = (nb * (kslice + 1)) / ks;
  const int nq = 4 * (sb1 - sb0);               // quarters of this K slice
  const int M = a.M;
  const int ntile = (S.rows + 15) >> 4;         // 16-row tiles of the segment
  const int tile0 = row0 >> 4;

  // ---- per-lane DMA sources ----------------------------------------------------------------
  // x: instruction i of wave w covers rows 8*(NX*w + i) .. +8; lane -> row + (lane >> 3), physical
  // chunk lane & 7 <- logical chunk (lane & 7) ^ (row & 7). xm (MoE): block row -> gathered x row, so the
  // DMA gathers an expert's routed rows straight from the token activations
  const act_t* xsrc[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int row = 8 * (NX * wave + i) + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int lr = min(row, M - 1);                            // rows >= M: clamped, never stored
    xsrc[i] = a.x + (size_t)(xm ? xm[lr] : lr) * a.ldx + c * 8;
  }
  // raw W: LDS byte b of the packed region <- tile-block b / TB, byte b % TB (TB % 16 == 0)
  const uint8_t* wsrc[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    int b = ((NW * wave + i) << 10) + 16 * lane;
    if (b >= 8 * TB) b = 0;                     // pad lanes: any valid source, lands in the pad
    const int lt = b / TB;
    const int t = min(tile0 + lt, ntile - 1);
    wsrc[i] = S.w + (size_t)t * nb * TB + (b - lt * TB);
  }
  const uint32_t xl0 = __builtin_amdgcn_readfirstlane(lds_addr(Xs)) + (uint32_t)(NX * wave) * 1024u;
  const uint32_t wl0 = __builtin_amdgcn_readfirstlane(lds_addr(Wl)) + (uint32_t)(NW * wave) * 1024u;
  auto dma_x = [&](int j) __attribute__((always_inline)) {     // quarter j (clamped) -> ring slot j % 3
    const int jc = min(j, nq - 1);
    const int koff = (sb0 + (jc >> 2)) * 256 + (jc & 3) * 64;
    const uint32_t dst = xl0 + (uint32_t)(j % 3) * XS;
#pragma unroll
    for (int i = 0; i < NX; ++i) glds16(xsrc[i] + koff, dst + i * 1024);
  };
  auto dma_w = [&](int sb) __attribute__((always_inline)) {    // super-block sb (clamped)
    const size_t off = (size_t)min(sb, sb1 - 1) * TB;
#pragma unroll
    for (int i = 0; i < NW; ++i) glds16(wsrc[i] + off, wl0 + i * 1024);
  };

  f32x4 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef typename RawOf<T>::type Raw;
  typedef typename ScOf<T>::type Sc;
  Raw raw[RT];
  Sc sc[RT];

  // one quarter: 2 K-steps x (RT fragments, MT A reads, RT*MT MFMAs). Every A fragment of the
  // quarter is requested up front (2*MT ds_read_b128 in flight) and the weight fragments are
  // dequantised while they land, so the LDS latency is exposed once per quarter, not per MFMA
  // pair (hipcc otherwise issues one read, waits lgkmcnt(0), runs its RT MFMAs, and repeats).
  // NA (compile time) = the 16-row activation tiles actually multiplied: a 96-row MoE block holding <= 64 routed
  // rows skips the padding tiles' LDS reads and MFMAs (their accumulators stay 0 and are never stored)
  auto quarter = [&](int j, int q, auto nac) __attribute__((always_inline)) {
    constexpr int NA = decltype(nac)::value;
    const uint8_t* xb = Xs + (j % 3) * XS;
    f16x8 xa[2][NA];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < NA; ++mt) {
        const int row = mt * 16 + r, c = 4 * t + g;
        xa[t][mt] = *reinterpret_cast<const f16x8*>(xb + row * 128 + ((c ^ (row & 7)) << 4));
      }
    f16x8 wf[2][RT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) wf[t][rt] = frag_t<T>(raw[rt], sc[rt], 2 * q + t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < NA; ++mt)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][mt] = mfma16(xa[t][mt], wf[t][rt], acc[rt][mt]);
  };

  auto main_loop = [&](auto nac) __attribute__((always_inline)) {
    // prologue: W(sb0), X(0), X(1); wait for the first two groups
    dma_w(sb0);
    dma_x(0);
    dma_x(1);
    wait_vm_lgkm0<NX>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int s = sb0; s < sb1; ++s) {
      const int j0 = 4 * (s - sb0);
      // ---- q = 0: this super-block's raw weights -> registers, scales
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) raw[rt] = raw_lds<T>(Wl + (2 * wave + rt) * TB, g, r);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) prep_sc<T>(raw[rt], g, sc[rt]);
      dma_x(j0 + 2);
      quarter(j0, 0, nac);
      wait_vm_lgkm0<NX>();                      // X(j0+1) landed (X(j0+2) in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---- q = 1: every wave has its raw regs -> stream the next super-block's weights
      dma_x(j0 + 3);
      dma_w(s + 1);
      quarter(j0 + 1, 1, nac);
      wait_vm_lgkm0<NX + NW>();                 // X(j0+2) landed (X(j0+3), W(s+1) in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---- q = 2
      dma_x(j0 + 4);
      quarter(j0 + 2, 2, nac);
      wait_vm_lgkm0<NX + NW>();                 // X(j0+3) landed (W(s+1), X(j0+4) in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---- q = 3
      dma_x(j0 + 5);
      quarter(j0 + 3, 3, nac);
      wait_vm_lgkm0<NX>();                      // W(s+1), X(j0+4) landed (X(j0+5) in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  if (nq > 0) {
    if constexpr (MT == 6 && NLS_DMA_NA) {
      if (M <= 64) main_loop(std::integral_constant<int, 4>{});
      else main_loop(std::integral_constant<int, 6>{});
    } else {
      main_loop(std::integral_constant<int, MT>{});
    }
  }
  // drain the clamped tail DMAs before anything reuses LDS or the workgroup retires
  wait_vm_lgkm0<0>();
  __syncthreads();

  // ---- epilogue from the accumulators: lane holds weight row rbase + 16*rt + r and activation
  // rows 16*mt + 4g + e
  const int rbase = row0 + wave * 32;
  if (ks > 1) {
    const int ntot = a.pad;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = rbase + 16 * rt + r;
      if (row >= S.rows) continue;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = 16 * mt + 4 * g + e;
          if (b >= M) continue;
          if (ym)        // mapped split-K: slab row = the token's y row, columns shared by every expert
            ws[((size_t)kslice * a.mtot + ym[b]) * ntot + S.ycol + row] = acc[rt][mt][e];
          else
            ws[((size_t)kslice * a.mtot + a.m0 + b) * ntot + S.tile_begin_col + row] = acc[rt][mt][e];
        }
    }
    return;
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = rbase + 16 * rt + r;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int b = 16 * mt + 4 * g + e;
        const float v = acc[rt][mt][e] * a.alpha;
        if (a.epi == EPI_SWIGLU) {
          const float u = __shfl_xor(v, 8, 64);
          if (r < 8 && b < M && row < S.rows) {
            const int n = S.ycol + ((rbase + 16 * rt) >> 1) + r;
            reinterpret_cast<act_t*>(a.y)[(size_t)(ym ? ym[b] : b) * a.ldy + n] = (act_t)(silu(v) * u);
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
    // max over the lane's rows, the 16 lanes of a row group, then the 4 waves through LDS:
    // one global atomic per activation row per workgroup
    unsigned long long* red = reinterpret_cast<unsigned long long*>(lds);
    for (int idx = threadIdx.x; idx < BM; idx += 256) red[idx] = 0ull;
    __syncthreads();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned long long k = 0ull;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int row = rbase + 16 * rt + r;
          const unsigned long long kj = (row < S.rows) ? argmax_key(acc[rt][mt][e] * a.alpha, S.ycol + row) : 0ull;
          k = kj > k ? kj : k;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const unsigned long long ok = __shfl_xor(k, o, 64);
          k = ok > k ? ok : k;
        }
        if (r == 0) atomicMax(red + 16 * mt + 4 * g + e, k);
      }
    __syncthreads();
    for (int idx = threadIdx.x; idx < M; idx += 256) atomicMax(a.argmax + idx, red[idx]);
  }
}

// MT <= 6 (64 / 96-row blocks: MoE experts at ~64 routed rows) is built for TWO workgroups
// per CU (<= 256 VGPRs at 4 waves, 52 / 64 KiB of LDS): one workgroup's DMA waits and barriers hide behind the
// other's MFMAs, where the 128 / 256-row blocks own a CU each.
template <int MT, int KSET>
__global__ __launch_bounds__(256, MT <= 6 ? 2 : 1) void qmm_dma_kernel(SegList segs, GemvArgs a, int ks, float* ws,
                                                                        int ntiles, int nmb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
  constexpr int BM = MT * 16;
  const int i = blockIdx.x, xcd = i & 7, j = i >> 3;
  const int kslice = j % ks;
  const int mb = (j / ks) % nmb;
  const int tile = (j / ks / nmb) * 8 + xcd;
  if (tile >= ntiles) return;
  Seg S = segs.s[0];
#pragma unroll
  for (int s = 1; s < 8; ++s)
    if (s < segs.nseg && tile >= segs.s[s].tile_begin) S = segs.s[s];
  const int m0 = mb * BM;
  // MoE grouped GEMM: the expert's routed-row count lives on the device; m-blocks past it exit before any DMA
  // (the grid is sized for the worst case, every token on one expert)
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
  if constexpr (KSET == 0) {
    switch (S.type) {
      case QT_Q4_K: dma_tile<QT_Q4_K, MT>(S, row0, kslice, ks, a, ws, dlds, xm, ym); break;
      case QT_Q6_K: dma_tile<QT_Q6_K, MT>(S, row0, kslice, ks, a, ws, dlds, xm, ym); break;
      default: break;
    }
  } else {
    switch (S.type) {
      case QT_Q5_K: dma_tile<QT_Q5_K, MT>(S, row0, kslice, ks, a, ws, dlds, xm, ym); break;
      case QT_Q6_K: dma_tile<QT_Q6_K, MT>(S, row0, kslice, ks, a, ws, dlds, xm, ym); break;
      default: break;
    }
  }
}

// LDS: 3 activation quarters + the largest raw region of the set (Q6_K: 7 KiB per wave)
template <int MT>
constexpr size_t dma_lds_bytes() { return (size_t)3 * MT * 16 * 128 + 4 * 1024 * DmaW<QT_Q6_K>::n; }

template <int MT, int KSET>
int launch_dma_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  constexpr int BM = MT * 16;
  const int nmb = (a.M + BM - 1) / BM;
  const size_t lds = dma_lds_bytes<MT>();
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)qmm_dma_kernel<MT, KSET>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL((qmm_dma_kernel<MT, KSET>), dim3(grid), dim3(256), lds, st, sl, a, ks, ws, ntiles, nmb);
  return (int)hipGetLastError();
}

template <int KSET>
int launch_dma_kset(int mt, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  if (mt == 16) return launch_dma_t<16, KSET>(sl, ntiles, ks, ws, a, st);
  if (mt == 8) return launch_dma_t<8, KSET>(sl, ntiles, ks, ws, a, st);
  if (mt == 6) return launch_dma_t<6, KSET>(sl, ntiles, ks, ws, a, st);
  if (mt == 4) return launch_dma_t<4, KSET>(sl, ntiles, ks, ws, a, st);
  return -1;
}

int launch_dma_k0(int mt, const SegList&, int, int, float*, const GemvArgs&, hipStream_t);
int launch_dma_k1(int mt, const SegList&, int, int, float*, const GemvArgs&, hipStream_t);

}  // namespace nls_dma
