// Dense f16 GEMM, "mode 8" of the qgemv dispatcher (gfx950): the large-M projections on the weights'
// f16 copies, built to replace the vendor library (hipBLASLt) on every decode / prefill shape.
//
//   y[m, n] (epilogue) alpha * sum_k x[m, k] * W[n, k]      x f16 [M, K], W f16 [N, K] row-major
//
// Why a second dense kernel next to hgemm.hip (modes 4-6): that one stages 64-deep K-steps through
// rings sized by the 160 KiB LDS (two or three deep), so each K-step's DMA has at most one step of
// compute to hide behind, and it reads its operands as 16 x 16 fragments straight before the MFMAs
// that consume them. Here (cdna_hip_programming.md §5 "Pipelining across barriers", "3-buf span"):
//   * K advances in 32-deep STAGES through a 5-deep LDS ring (64-byte rows): 4 stages are in flight
//     while one is computed, so every LDS-DMA (`global_load_lds_dwordx4`, 1 KiB per wave instruction)
//     has ~3 stages of MFMA work to land behind; one raw s_barrier per stage with a COUNTED vmcnt
//     (2 stages stay in flight across it);
//   * the MFMA fragments are double-buffered in registers: right after the barrier that certifies
//     stage j+1 a wave requests stage j+1's fragments, then runs stage j's MFMAs on the fragments it
//     requested one stage earlier -- the LDS latency hides behind the MFMAs, not in front of them;
//   * workgroup = 256 activation rows x BN weight rows (BN 256, or 224 so that the 28672-row gate|up
//     of Llama-3-8B at 512 rows is EXACTLY 256 workgroups: one per CU, no tail wave), 8 waves as
//     4 (activations) x 2 (weights), each 64 x BN/2 of v_mfma_f32_16x16x32_f16 accumulators with the
//     WEIGHT rows as the A operand: a lane ends up with 4 consecutive output columns of one row, so
//     every epilogue stores 16 contiguous bytes, and SwiGLU's gate/up partner is lane ^ 32;
//   * 16-byte chunks are XOR-swizzled per 4-row group (chunk ^ {0,2,3,1}[(row >> 2) & 3]) on the DMA
//     SOURCE address (the DMA writes LDS lane-linearly): conflict-free ds_read_b128 for the
//     {0-3,12-15,20-27}... lane groups of the instruction (MI355X_MICROARCH.md §LDS);
//   * epilogues: f32 store / residual add / f16 SwiGLU / split-K slabs / fused arg-max keys, so the
//     library GEMM's separate SwiGLU / add passes are gone with it.
// Grid and split-K as hgemm.hip: (tile, m-block, k-slice) with every m-block and k-slice of a weight
// tile on ONE XCD (the tile is fetched from HBM once per XCD L2).
#include "qgemm_dma.h"

// tools/hg8_probe.hip builds speed-of-light variants: bit 0 = no MFMA (fragments still read),
// bit 1 = no DMA, bit 2 = no vmcnt waits (results wrong; timing only). 0 in the library.
#ifndef H8_PROBE
#define H8_PROBE 0
#endif

namespace nls_hg8 {
using namespace nls_gemv;
using nls_dma::glds16;
using nls_dma::lds_addr;

template <int BN>
struct Cfg {
  static constexpr int BM = 256;                  // activation rows per workgroup
  static constexpr int NT = BN / 32;              // 16-row weight tiles per wave (2 waves along N)
  static constexpr int MT = 4;                    // 16-row activation tiles per wave (4 waves along M)
  static constexpr int XB = BM * 64;              // bytes of one activation stage [256][32] f16
  static constexpr int WB = BN * 64;              // bytes of one weight stage [BN][32] f16
  static constexpr int SB = XB + WB;
  static constexpr int NS = 5;                    // ring depth (stages)
  static constexpr int XI = BM / 16 / 8;          // activation DMA instructions per wave per stage (2)
  static constexpr int WI = BN / 16;              // weight DMA instructions per stage, whole workgroup
  static constexpr size_t LDS = (size_t)NS * SB;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(BN % 32 == 0 && WI <= 16, "BN");
};

// 16-byte chunk swizzle of a 64-byte LDS row: physical chunk = logical ^ swz(row)
DEVI int swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

template <int N>
DEVI void wait_vm() {
  if constexpr (H8_PROBE & 4) return;
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int BN, int WCNT>
DEVI void h8_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds) {
  typedef Cfg<BN> C;
  constexpr int NT = C::NT, MT = C::MT, NS = C::NS;
  constexpr int PER = C::XI + WCNT;               // this wave's DMA instructions per stage
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int nst_all = S.K >> 5;
  const int s0 = (nst_all * kslice) / ks, s1 = (nst_all * (kslice + 1)) / ks;
  const int nst = s1 - s0;
  const int M = a.M;

  // ---- DMA sources. Instruction q of an operand covers rows 16q..16q+15: lane L -> row 16q + (L >> 2),
  // physical chunk L & 3 <- logical chunk (L & 3) ^ swz(row); swz(row) = swz(L >> 2) (16q is a multiple of 16)
  const int lc = (lane & 3) ^ swz(lane >> 2);
  const act_t* xsrc[C::XI];
#pragma unroll
  for (int i = 0; i < C::XI; ++i) {
    const int row = min(16 * (C::XI * wave + i) + (lane >> 2), M - 1);     // rows >= M: clamped, never stored
    xsrc[i] = a.x + (size_t)row * a.ldx + (size_t)s0 * 32 + lc * 8;
  }
  const act_t* Wd = reinterpret_cast<const act_t*>(S.w);
  const act_t* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = min(wave + 8 * i, C::WI - 1);
    const int row = min(row0 + 16 * q + (lane >> 2), S.rows - 1);
    wsrc[i] = Wd + (size_t)row * S.K + (size_t)s0 * 32 + lc * 8;
  }
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint32_t xdst = base + (uint32_t)(C::XI * wave) * 1024u;
  const uint32_t wdst = base + C::XB + (uint32_t)wave * 1024u;
  auto dma = [&](int j) __attribute__((always_inline)) {      // stage j (clamped) -> ring slot j % NS
    if constexpr (H8_PROBE & 2) return;
    const int jj = min(j, nst - 1);
    const uint32_t so = (uint32_t)(j % NS) * C::SB;
#pragma unroll
    for (int i = 0; i < C::XI; ++i) glds16(xsrc[i] + jj * 32, xdst + so + i * 1024);
#pragma unroll
    for (int i = 0; i < WCNT; ++i) glds16(wsrc[i] + jj * 32, wdst + so + i * 8192);
  };

  // ---- fragment reads: lane reads row (l & 15) of a 16-row tile, logical chunk l >> 4
  const int fro = (lane & 15) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4);
  const int aoff = C::XB + wn * NT * 16 * 64 + fro;           // weight fragments (A operand)
  const int boff = wm * MT * 16 * 64 + fro;                   // activation fragments (B operand)
  f16x8 FA0[NT], FB0[MT], FA1[NT], FB1[MT];
  auto rd = [&](f16x8* FA, f16x8* FB, int j) __attribute__((always_inline)) {
    const uint8_t* sb = lds + (j % NS) * C::SB;
#pragma unroll
    for (int t = 0; t < NT; ++t) FA[t] = *reinterpret_cast<const f16x8*>(sb + aoff + t * 1024);
#pragma unroll
    for (int t = 0; t < MT; ++t) FB[t] = *reinterpret_cast<const f16x8*>(sb + boff + t * 1024);
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const f16x8* FA, const f16x8* FB) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if constexpr (H8_PROBE & 1) asm volatile("" ::"v"(FA[i]), "v"(FB[j]));
        else acc[i][j] = mfma16(FA[i], FB[j], acc[i][j]);
      }
  };

  if (nst > 0) {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) dma(s);
    wait_vm<(NS - 2) * PER>();                                // stage 0 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd(FA0, FB0, 0);
    // iteration j: stage j+1 certified (counted vmcnt + barrier), DMA stage j+NS-1 into the slot of
    // stage j-1 (whose fragments every wave consumed before this barrier), request stage j+1's
    // fragments, then compute stage j from the fragments requested one iteration earlier
    int j = 0;
    for (; j + 1 < nst; j += 2) {
      wait_vm<(NS - 3) * PER>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      dma(j + NS - 1);
      rd(FA1, FB1, j + 1);
      __builtin_amdgcn_s_setprio(1);
      mma(FA0, FB0);
      __builtin_amdgcn_s_setprio(0);
      wait_vm<(NS - 3) * PER>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      dma(j + NS);
      rd(FA0, FB0, j + 2);                                    // (clamped slot: harmless past the end)
      __builtin_amdgcn_s_setprio(1);
      mma(FA1, FB1);
      __builtin_amdgcn_s_setprio(0);
    }
    if (j < nst) mma(FA0, FB0);
  }
  wait_vm<0>();                                                // drain the clamped tail DMAs
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: lane holds weight rows nb + 16i + 4(l >> 4) + e and activation row mb + 16j + (l & 15)
  const int g4 = 4 * (lane >> 4), r16 = lane & 15;
  const int nb = row0 + wn * NT * 16, mb = wm * MT * 16;
  if (ks > 1 || a.epi == EPI_SLABS) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int n = nb + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = mb + 16 * j + r16;
        if (m >= M) continue;
        *reinterpret_cast<f32x4*>(ws + ((size_t)kslice * a.mtot + a.m0 + m) * a.pad + S.tile_begin_col + n) = acc[i][j];
      }
    }
    return;
  }
  const float al = a.alpha;
  if (a.epi == EPI_SWIGLU) {
    // interleaved [g0..g7 | u0..u7] per 16 weight rows: lanes 0-31 hold gate rows 4(l>>4).., lanes 32-63
    // the up rows 8 higher -- the partner is lane ^ 32
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        f32x4 u;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = __shfl_xor(acc[i][j][e] * al, 32, 64);
        const int n16 = nb + 16 * i, m = mb + 16 * j + r16;
        if (lane < 32 && m < M && n16 < S.rows) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          h4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (_Float16)(silu(acc[i][j][e] * al) * u[e]);
          *reinterpret_cast<h4*>(reinterpret_cast<act_t*>(a.y) + (size_t)m * a.ldy + S.ycol + (n16 >> 1) + g4) = o;
        }
      }
    }
    return;
  }
  if (a.epi != EPI_ARGMAX) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int n = nb + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = mb + 16 * j + r16;
        if (m >= M) continue;
        const f32x4 v = acc[i][j] * al;
        if (a.epi == EPI_ACT) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<h4*>(reinterpret_cast<act_t*>(a.y) + (size_t)m * a.ldy + S.ycol + n) =
              h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
          f32x4* p = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.y) + (size_t)m * a.ldy + S.ycol + n);
          *p = a.epi == EPI_ADD_F32 ? *p + v : v;
        }
      }
    }
  }
  if (a.argmax) {
    // per activation row: max over the lane's rows, then the 4 lanes of the row (l ^ 16, l ^ 32);
    // one 64-bit atomic per row per wave
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      unsigned long long k = 0ull;
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = nb + 16 * i + g4 + e;
          const unsigned long long kk = n < S.rows ? argmax_key(acc[i][j][e] * al, S.ycol + n) : 0ull;
          k = kk > k ? kk : k;
        }
      unsigned long long o = __shfl_xor(k, 16, 64);
      k = o > k ? o : k;
      o = __shfl_xor(k, 32, 64);
      k = o > k ? o : k;
      const int m = mb + 16 * j + r16;
      if (lane < 16 && m < M) atomicMax(a.argmax + m, k);
    }
  }
}

template <int BN>
__global__ __launch_bounds__(512, 1) void hgemm8_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                          int nmb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t h8lds[];
  constexpr int BM = Cfg<BN>::BM;
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
  a.m0 = m0;
  a.x += (size_t)m0 * a.ldx;
  const size_t esz = (a.epi == EPI_F32 || a.epi == EPI_ADD_F32 || a.epi == EPI_ARGMAX) ? 4 : 2;
  a.y = (char*)a.y + (size_t)m0 * a.ldy * esz;
  if (a.argmax) a.argmax += m0;
  a.M = min(BM, a.M - m0);
  const int row0 = (tile - S.tile_begin) * BN;
  // weight DMA instructions per wave: WI over 8 waves (BN 224: waves 0-5 issue 2, waves 6-7 one)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (Cfg<BN>::WI == 16) {
    h8_tile<BN, 2>(S, row0, kslice, ks, a, ws, h8lds);
  } else if constexpr (Cfg<BN>::WI == 8) {
    h8_tile<BN, 1>(S, row0, kslice, ks, a, ws, h8lds);
  } else {
    if (wave + 8 < Cfg<BN>::WI) h8_tile<BN, 2>(S, row0, kslice, ks, a, ws, h8lds);
    else h8_tile<BN, 1>(S, row0, kslice, ks, a, ws, h8lds);
  }
}

template <int BN>
int launch_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  typedef Cfg<BN> C;
  const int nmb = (a.M + C::BM - 1) / C::BM;
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)hgemm8_kernel<BN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS) !=
        hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL((hgemm8_kernel<BN>), dim3(grid), dim3(512), C::LDS, st, sl, a, ks, ws, ntiles, nmb);
  return (int)hipGetLastError();
}

// bn: weight rows per workgroup (256 | 224 | 128)
int launch_dense8(int bn, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  if (bn == 256) return launch_t<256>(sl, ntiles, ks, ws, a, st);
  if (bn == 224) return launch_t<224>(sl, ntiles, ks, ws, a, st);
  if (bn == 128) return launch_t<128>(sl, ntiles, ks, ws, a, st);
  return -1;
}

}  // namespace nls_hg8
