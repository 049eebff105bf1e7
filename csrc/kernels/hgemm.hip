// Dense f16 GEMM for large M ("modes 4 and 5" of the qgemv dispatcher), gfx950.
//
//   y[m, n] = alpha * sum_k x[m, k] * W[n, k]      (x f16 [M, K], W f16 [N, K] row-major)
//
// Why a dense path next to the K-quant GEMMs (modes 2/3): at decode batches >= 128 and in prefill
// the quantised GEMMs spend ~2.6 VALU instructions per MFMA on dequantisation and addressing
// (PMC, profiles/pmc_gemm_dense_vs_quant_M512.txt) and their 128-row weight tiles re-fetch the
// activation tile for every 128 output columns. An MI355X has 288 GB of HBM3E, so the engine keeps an
// f16 copy of every projection matrix next to its quantised tiles (Llama-3-8B: 15 GB) when that copy
// fits comfortably: the few-row GEMVs keep streaming the 4.5 GB of quantised tiles (HBM-bound), the
// large-M GEMMs read f16 and the main loop is DMA + MFMA only. The f16 copy is the dequant kernel's
// output (a single f16 rounding of d*sc*q - dmin*m, exactly what modes 2/3 feed their MFMAs), so
// the two paths agree up to accumulation order.
//
// Structure (cdna_hip_programming.md §5, "glds, 3 LDS buffers, counted vmcnt, raw s_barrier"):
//   * workgroup tile = BN weight rows (128: mode 4, 256: mode 5) x BM activation rows (BM = 64*WM:
//     256 or 128), 8 waves as WM (M) x 8/WM (N), each wave 64 activation rows x BN*WM/8 weight rows
//     of v_mfma_f32_16x16x32_f16 accumulators; the 256 x 256 tile does twice the MFMA work per
//     fetched activation byte of the 256 x 128 one;
//   * K advances in 64-wide steps; BOTH operands arrive by LDS-DMA (global_load_lds_dwordx4,
//     1 KiB per wave-instruction: 8 rows x 128 B) into rings (activations 3 deep; weights 3 deep, or
//     2 deep when 3 would pass the 160 KiB of LDS), XOR-swizzled by permuting the per-lane SOURCE
//     chunk (16-B chunk c of row r lands at c ^ (r & 7): conflict-free ds_read_b128);
//   * one raw s_barrier per K-step with a counted vmcnt: the next activation stage stays in flight
//     across it; nothing passes through VGPRs on its way into LDS.
// Measured (MI355X, 8B shapes, weights streamed from HBM; profiles/tune_dense_vs_quant_r02.txt):
// gate/up M=512 930 TFLOP/s (mode 2: 827), M=2048 1.02 PFLOP/s; B=512 decode 13.47 vs 14.01 ms/step.
// Grid, split-K slabs and epilogues are those of mode 2 (qgemm_impl.h): (tile, m-block, k-slice)
// with every m-block and k-slice of a weight tile on ONE XCD, so a weight tile is fetched from HBM
// once per XCD L2.
#include "qgemm_dma.h"

namespace nls_hgemm {
using namespace nls_gemv;
using nls_dma::glds16;
using nls_dma::lds_addr;
using nls_dma::wait_vm_lgkm0;

template <int WM, int BN, int NWV, int NST = 3>
struct HG {
  static constexpr int NT = 64 * NWV;         // threads per workgroup (8 or 16 waves)
  static constexpr int BM = 64 * WM;          // activation rows per workgroup
  static constexpr int WN = NWV / WM;         // waves along N
  static constexpr int NTW = BN / 16 / WN;    // 16-row weight tiles per wave
  static constexpr int MTW = 4;               // 16-row activation tiles per wave
  static constexpr int XS = BM * 128;         // bytes of one activation stage [BM][64] f16
  static constexpr int WSB = BN * 128;        // bytes of one weight stage [BN][64] f16
  static constexpr int NSX = NST;             // activation ring depth
  // weight ring depth (LDS budget); NST = 2: both rings 2 deep, small enough for 2 workgroups per CU
  static constexpr int NSW = NST == 2 ? 2 : ((NSX * XS + 3 * WSB <= 160 * 1024) ? 3 : 2);
  static constexpr int NX = BM / 8 / NWV;     // activation DMA instructions per wave per stage
  static constexpr int NW = BN / 8 / NWV;     // weight DMA instructions per wave per stage
  static_assert(NX >= 1 && NW >= 1 && NTW >= 1, "tile too small for the wave count");
  static constexpr size_t LDS = (size_t)NSX * XS + (size_t)NSW * WSB;
};

template <int WM, int BN, int NWV, int NST>
using HGAcc = f32x4[HG<WM, BN, NWV, NST>::MTW][HG<WM, BN, NWV, NST>::NTW];

// acc += the tile's product over K-steps [kt0, kt1) (64 columns each); LDS is free again on return
template <int WM, int BN, int NWV, int NST>
DEVI void hg_main(const Seg& S, int row0, int kt0, int kt1, const GemvArgs& a, uint8_t* lds, const int* xm,
                  HGAcc<WM, BN, NWV, NST>& acc) {
  typedef HG<WM, BN, NWV, NST> G;
  constexpr int MTW = G::MTW, NTW = G::NTW, NX = G::NX, NW = G::NW, WN = G::WN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  const int nq = kt1 - kt0;
  const int M = a.M;

  // ---- per-lane DMA sources: a DMA group is 8 rows starting at a multiple of 8, lane -> row
  // group_row + (lane >> 3), physical chunk lane & 7 <- logical chunk (lane & 7) ^ (lane >> 3)
  const int c = (lane & 7) ^ (lane >> 3);
  const act_t* xsrc[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    // rows >= M: clamped, never stored; xm: MoE gather (block-local row -> x row) on the DMA source
    const int row = min(8 * (NX * wave + i) + (lane >> 3), M - 1);
    xsrc[i] = a.x + (size_t)(xm ? xm[row] : row) * a.ldx + kt0 * 64 + c * 8;
  }
  const act_t* wsrc[NW];
  const act_t* Wd = reinterpret_cast<const act_t*>(S.w);
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int row = row0 + 8 * (NW * wave + i) + (lane >> 3);
    wsrc[i] = Wd + (size_t)min(row, S.rows - 1) * S.K + kt0 * 64 + c * 8;
  }
  uint8_t* const Wl = lds + G::NSX * G::XS;
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint32_t xl = base + (uint32_t)(NX * wave) * 1024u;
  const uint32_t wl = base + G::NSX * G::XS + (uint32_t)(NW * wave) * 1024u;
  auto dma_x = [&](int j) __attribute__((always_inline)) {    // K-step j (clamped) -> x slot j % NSX
    const int koff = min(j, nq - 1) * 64;
    const uint32_t so = (uint32_t)(j % G::NSX) * G::XS;
#pragma unroll
    for (int i = 0; i < NX; ++i) glds16(xsrc[i] + koff, xl + so + i * 1024);
  };
  auto dma_w = [&](int j) __attribute__((always_inline)) {    // K-step j (clamped) -> W slot j % NSW
    const int koff = min(j, nq - 1) * 64;
    const uint32_t so = (uint32_t)(j % G::NSW) * G::WSB;
#pragma unroll
    for (int i = 0; i < NW; ++i) glds16(wsrc[i] + koff, wl + so + i * 1024);
  };

  // one K-step (two 32-deep MFMA K-slices): each slice's fragments are requested together (the LDS
  // latency is exposed once per slice), then its MTW * NTW MFMAs
  auto step = [&](int j) __attribute__((always_inline)) {
    const uint8_t* xb = lds + (j % G::NSX) * G::XS;
    const uint8_t* wb = Wl + (j % G::NSW) * G::WSB;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int co = ((4 * t + g) ^ (r & 7)) << 4;
      f16x8 A[MTW], B[NTW];
#pragma unroll
      for (int i = 0; i < MTW; ++i) A[i] = *reinterpret_cast<const f16x8*>(xb + (wm * 64 + 16 * i + r) * 128 + co);
#pragma unroll
      for (int jj = 0; jj < NTW; ++jj)
        B[jj] = *reinterpret_cast<const f16x8*>(wb + (wn * NTW * 16 + 16 * jj + r) * 128 + co);
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int jj = 0; jj < NTW; ++jj) acc[i][jj] = mfma16(A[i], B[jj], acc[i][jj]);
    }
  };

  if (nq > 0) {
    if constexpr (G::NSW == 3) {
      // both rings 3 deep: steps j+1 and j+2 in flight while step j computes
      dma_w(0);
      dma_x(0);
      dma_w(1);
      dma_x(1);
      wait_vm_lgkm0<NX + NW>();                 // step 0 landed (step 1 in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int j = 0; j < nq; ++j) {
        dma_w(j + 2);                           // slots (j+2)%3 were last read in step j-1: retired
        dma_x(j + 2);
        step(j);
        wait_vm_lgkm0<NX + NW>();               // step j+1 landed (j+2 in flight)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    } else if constexpr (G::NSX == 2) {
      // both rings 2 deep (two workgroups per CU hide each other's load waits): step j+1 is issued at
      // the top of step j and fully waited for at its end
      dma_w(0);
      dma_x(0);
      wait_vm_lgkm0<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int j = 0; j < nq; ++j) {
        dma_w(j + 1);                           // slots (j+1)%2 were last read in step j-1: retired
        dma_x(j + 1);
        step(j);
        wait_vm_lgkm0<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    } else {
      // weights 2 deep (LDS budget), activations 3 deep: W(j+1) and X(j+2) are issued at the top
      // of step j; the wait at its end leaves only X(j+2) in flight
      dma_w(0);
      dma_x(0);
      dma_x(1);
      wait_vm_lgkm0<NX>();                      // W(0), X(0) landed (X(1) in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int j = 0; j < nq; ++j) {
        dma_w(j + 1);                           // W slot (j+1)%2 was last read in step j-1: retired
        dma_x(j + 2);
        step(j);
        wait_vm_lgkm0<NX>();                    // X(j+1), W(j+1) landed (X(j+2) in flight)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
  }
  wait_vm_lgkm0<0>();                           // drain the clamped tail DMAs before LDS reuse / exit
  __syncthreads();
}

// epilogue of a finished tile: split-K slab (ks > 1) or the launch's epilogue
template <int WM, int BN, int NWV, int NST>
DEVI void hg_epi(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds,
                 const int* ym, HGAcc<WM, BN, NWV, NST>& acc) {
  typedef HG<WM, BN, NWV, NST> G;
  constexpr int MTW = G::MTW, NTW = G::NTW, WN = G::WN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  const int M = a.M;
  // ---- lane holds weight rows rbase + 16j + r and activation rows 16i + 4g + e
  const int rbase = row0 + wn * NTW * 16, mbase = wm * 64;
  if (ks > 1) {
    const int ntot = a.pad;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int row = rbase + 16 * j + r;
      if (row >= S.rows) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = mbase + 16 * i + 4 * g + e;
          if (b >= M) continue;
          if (ym)        // mapped split-K: slab row = the token's y row, columns shared by every expert
            ws[((size_t)kslice * a.mtot + ym[b]) * ntot + S.ycol + row] = acc[i][j][e];
          else
            ws[((size_t)kslice * a.mtot + a.m0 + b) * ntot + S.tile_begin_col + row] = acc[i][j][e];
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int row = rbase + 16 * j + r;
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int b = mbase + 16 * i + 4 * g + e;
        const float v = acc[i][j][e] * a.alpha;
        if (a.epi == EPI_ROPE) {
          // RoPE pair (row, row ^ 1) = lanes r, r ^ 1 (same b)
          const float pv = __shfl_xor(v, 1, 64);
          if (b < M && row < S.rows) rope_store1(a, S.ycol + row, a.m0 + b, v, pv);
          continue;
        }
        if (a.epi == EPI_SWIGLU) {
          // interleaved [g0..g7, u0..u7] per 16 weight rows: the partner row is lane ^ 8 (same b)
          const float u = __shfl_xor(v, 8, 64);
          if (r < 8 && b < M && row < S.rows) {
            const int n = S.ycol + ((row & ~15) >> 1) + (row & 7);
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
    // max over the lane's weight rows, the 16 lanes of an activation row, then the waves through
    // LDS (free after the main loop): one global atomic per activation row per workgroup
    unsigned long long* red = reinterpret_cast<unsigned long long*>(lds);
    for (int idx = threadIdx.x; idx < G::BM; idx += G::NT) red[idx] = 0ull;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned long long k = 0ull;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int row = rbase + 16 * j + r;
          const unsigned long long kj = (row < S.rows) ? argmax_key(acc[i][j][e] * a.alpha, S.ycol + row) : 0ull;
          k = kj > k ? kj : k;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const unsigned long long ok = __shfl_xor(k, o, 64);
          k = ok > k ? ok : k;
        }
        if (r == 0) atomicMax(red + mbase + 16 * i + 4 * g + e, k);
      }
    __syncthreads();
    for (int idx = threadIdx.x; idx < M; idx += G::NT) atomicMax(a.argmax + idx, red[idx]);
  }
}

template <int WM, int BN, int NWV, int NST>
DEVI void hgemm_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds,
                     const int* xm, const int* ym) {
  typedef HG<WM, BN, NWV, NST> G;
  HGAcc<WM, BN, NWV, NST> acc;
#pragma unroll
  for (int i = 0; i < G::MTW; ++i)
#pragma unroll
    for (int j = 0; j < G::NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkt = S.K >> 6;
  hg_main<WM, BN, NWV, NST>(S, row0, (nkt * kslice) / ks, (nkt * (kslice + 1)) / ks, a, lds, xm, acc);
  hg_epi<WM, BN, NWV, NST>(S, row0, kslice, ks, a, ws, lds, ym, acc);
}

template <int WM, int BN, int NWV, int NST>
__global__ __launch_bounds__(64 * NWV, NST == 2 ? 2 : 1) void hgemm_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                       int nmb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t hlds[];
  constexpr int BM = HG<WM, BN, NWV, NST>::BM;
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
  // MoE grouped GEMM (as mode 2): the expert's routed-row count lives on the device; m-blocks past it
  // exit before issuing any DMA (the grid is sized for every routed row on one expert)
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
  hgemm_tile<WM, BN, NWV, NST>(S, (tile - S.tile_begin) * BN, kslice, ks, a, ws, hlds, xm, ym);
}

template <int WM, int BN, int NWV, int NST>
int launch_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  typedef HG<WM, BN, NWV, NST> G;
  const int nmb = (a.M + G::BM - 1) / G::BM;
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)hgemm_kernel<WM, BN, NWV, NST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)G::LDS) != hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL((hgemm_kernel<WM, BN, NWV, NST>), dim3(grid), dim3(G::NT), G::LDS, st, sl, a, ks, ws, ntiles, nmb);
  return (int)hipGetLastError();
}

// bn: weight rows per workgroup (128: 3-deep rings; 256: x 3-deep, W 2-deep, 160 KiB of LDS at
// wm 4); nst 2: 2-deep rings (64 KiB at wm 2, bn 128: two workgroups per CU); waves: 8 (2 per SIMD, 64 x 16*bn/128 accumulator tile per wave) or 16 (4 per SIMD, half
// the tile per wave: more waves to cover each other's LDS and barrier waits)
int launch_dense(int wm, int bn, int waves, int nst, const SegList& sl, int ntiles, int ks, float* ws,
                 const GemvArgs& a, hipStream_t st) {
#define NLS_HG(W, B, V, S) \
  if (wm == W && bn == B && waves == V && nst == S) return launch_t<W, B, V, S>(sl, ntiles, ks, ws, a, st);
  NLS_HG(4, 128, 8, 3) NLS_HG(2, 128, 8, 3) NLS_HG(4, 256, 8, 3) NLS_HG(2, 256, 8, 3)
  NLS_HG(4, 128, 16, 3) NLS_HG(2, 128, 16, 3) NLS_HG(4, 256, 16, 3) NLS_HG(2, 256, 16, 3)
  NLS_HG(2, 128, 8, 2)
#undef NLS_HG
  return -1;
}

}  // namespace nls_hgemm
