// Dense f16 GEMM, "mode 10" of the qgemv dispatcher (gfx950): 256 x 256 tiles in 4 phases per 64-deep
// K-tile with the two wave groups staggered by one barrier (cdna_hip_programming.md "The 256^2 8-phase
// template": counted vmcnt, raw barriers, one LDS-DMA unit per phase, the per-phase interleave).
//
//   y[m, n] (epilogue) alpha * sum_k x[m, k] * W[n, k]      x f16 [M, K], W f16 [N, K] row-major
//
// Why (profiles/gemm_probes_r03.txt): mode 8's one-barrier-per-stage ring keeps all 8 waves in the same
// section at once -- every wave reads LDS and issues DMA together, then every wave runs MFMAs together,
// and with MFMAs off the kernel still takes 94 % of its time. Here:
//   * 8 waves = 2 groups (wr: 128 weight rows each) x 4 (wc: 64 activation rows each); a wave owns a
//     128 x 64 output block (8 x 4 accumulator tiles of v_mfma_f32_16x16x32_f16, weights as the A
//     operand so a lane ends with 4 consecutive output columns, as mode 8);
//   * a K-tile is 4 phases, each: [load section] ds_read the phase's fragments + issue one 16 KiB
//     LDS-DMA unit (2 global_load_lds_dwordx4 per lane) -> barrier -> lgkmcnt(0), 16 MFMAs at raised
//     priority -> vmcnt(6) -> barrier. Group 1 runs ONE barrier behind group 0, so on every SIMD (one wave
//     of each group) one wave's MFMAs overlap the other wave's LDS reads and DMA issue;
//   * fragment schedule per K-tile (quadrants of the wave's block): Q0 = weight rows 0-63 x act rows
//     0-31 (reads A(nq0) 8 + B(mh0) 4), Q1 = x act rows 32-63 (B(mh1) 4), Q2 = weight rows 64-127 (A(nq1)
//     8), Q3 = (nq1, mh0) from registers;
//   * the 64 KiB K-tile buffer is 4 units in the order they are needed -- U0 = A(nq0 of both groups),
//     U1 = B(mh0), U2 = B(mh1), U3 = A(nq1) -- and a unit is restaged as soon as its previous contents are
//     read (>= 2 phases, the WAR rule with a staggered group): U0(T) at phase Q2(T-2), U1(T) Q3(T-2),
//     U2(T) Q0(T-1), U3(T) Q1(T-1). Every unit is issued >= 5 phases before its first read and 3 units
//     stay in flight (vmcnt(6)), which the group stagger needs (a reader in group 0 is ordered only after
//     group 1's wait of the phase before);
//   * 2 K-tile buffers = 128 KiB of LDS, 1 workgroup per CU; 16-byte chunks XOR-swizzled per 4-row group
//     on the DMA source, as mode 8 (conflict-free ds_read_b128).
// Grid and split-K as mode 8: (tile, m-block, k-slice), every m-block and k-slice of a weight tile on one
// XCD. The epilogues are mode 8's (f32 / residual add / f16 / SwiGLU / split-K slabs / arg-max keys).
#include "qgemm_dma.h"

namespace nls_hg10 {
using namespace nls_gemv;
using nls_dma::glds16;
using nls_dma::lds_addr;

// BN = 256 (rt 1) or 128 (rt 2: narrow-N shapes get twice the workgroups -- Q|K|V, o at M = 512..2048): the
// weight half of a K-tile buffer and each wave's weight rows halve; the activation half, the phase schedule
// and the unit order stay, only the DMA instruction counts of the two weight units (and so the counted
// vmcnt of each phase) change.
constexpr int BM = 256;
constexpr int KT = 64;                       // K per tile
template <int BN>
struct H10 {
  static constexpr int AB = BN * KT * 2;     // weight half of a K-tile buffer (32 or 16 KiB)
  static constexpr int TB = AB + BM * KT * 2;
  static constexpr int LDS = 2 * TB;
  static constexpr int RTG = BN / 32;        // 16-row weight tiles per wave group (wr)
  static constexpr int NQH = RTG / 2;        // ... per quadrant half (nq)
  static constexpr int NA = BN / 128;        // DMA instructions per lane of a weight unit (B units: 2)
  // counted waits: the last three units issued stay in flight (units U0/U3 carry NA, U1/U2 two)
  static constexpr int VM_PRO = NA + 2;      // after the prologue: U0(1) U1(1)
  static constexpr int VM_Q0 = NA + 4;       // U0(T+1) U1(T+1) U2(T+1)
  static constexpr int VM_Q1 = NA + 4;       // U1(T+1) U2(T+1) U3(T+1)
  static constexpr int VM_Q2 = 2 * NA + 2;   // U2(T+1) U3(T+1) U0(T+2)
  static constexpr int VM_Q3 = 2 * NA + 2;   // U3(T+1) U0(T+2) U1(T+2)
};

DEVI int swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

template <int N>
DEVI void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// unit u's (row-tile, k-step) subtiles; a subtile = 16 rows x 32 k = 1 KiB at (rt * 2 + ks) * 1 KiB of
// its operand region. A units (0, 3): weight row-tiles; B units (1, 2): activation row-tiles.
template <int BN>
DEVI int unit_rt(int u, int idx) {           // idx: row-tile slot of the unit
  // BN 256: U0: A {0-3, 8-11}; U3: A {4-7, 12-15}. BN 128: U0: A {0-1, 4-5}; U3: A {2-3, 6-7}.
  // U1: B {0,1,4,5,8,9,12,13}; U2: B {2,3,6,7,10,11,14,15}
  constexpr int NQH = H10<BN>::NQH, RTG = H10<BN>::RTG;
  if (u == 0) return (idx % NQH) + RTG * (idx / NQH);
  if (u == 3) return NQH + (idx % NQH) + RTG * (idx / NQH);
  if (u == 1) return (idx & 1) + 4 * (idx >> 1);
  return 2 + (idx & 1) + 4 * (idx >> 1);
}

// ---- epilogue (mode 8's; shared by modes 10 and 11): lane holds weight rows nb + 16i + 4(l >> 4) + e, activation
// row mb + 16j + (l & 15)
template <int BN>
DEVI void h10_epilogue(const f32x4 (&acc)[2 * H10<BN>::NQH][4], const Seg& S, int row0, int kslice, int ks,
                       const GemvArgs& a, float* ws) {
  constexpr int NQH = H10<BN>::NQH;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int M = a.M;
  const int g4 = 4 * (lane >> 4), r16 = lane & 15;
  const int nb = row0 + wr * (BN / 2), mb = wc * 64;
  if (ks > 1 || a.epi == EPI_SLABS) {
#pragma unroll
    for (int i = 0; i < 2 * NQH; ++i) {
      const int n = nb + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mb + 16 * j + r16;
        if (m >= M) continue;
        *reinterpret_cast<f32x4*>(ws + ((size_t)kslice * a.mtot + a.m0 + m) * a.pad + S.tile_begin_col + n) = acc[i][j];
      }
    }
    return;
  }
  const float al = a.alpha;
  if (a.epi == EPI_ROPE) {
    // RoPE pairs (e, e + 1) of the lane's 4 consecutive weight rows: no cross-lane traffic
#pragma unroll
    for (int i = 0; i < 2 * NQH; ++i) {
      const int n = nb + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mb + 16 * j + r16;
        if (m >= M) continue;
        const f32x4 v = acc[i][j] * al;
        rope_store1(a, S.ycol + n, a.m0 + m, v[0], v[1]);
        rope_store1(a, S.ycol + n + 1, a.m0 + m, v[1], v[0]);
        rope_store1(a, S.ycol + n + 2, a.m0 + m, v[2], v[3]);
        rope_store1(a, S.ycol + n + 3, a.m0 + m, v[3], v[2]);
      }
    }
    return;
  }
  if (a.epi == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 2 * NQH; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
    for (int i = 0; i < 2 * NQH; ++i) {
      const int n = nb + 16 * i + g4;
      if (n >= S.rows) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned long long k = 0ull;
#pragma unroll
      for (int i = 0; i < 2 * NQH; ++i)
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
DEVI void h10_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, uint8_t* lds) {
  typedef H10<BN> C;
  constexpr int TB = C::TB, NQH = C::NQH, NA = C::NA;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nkt_all = S.K / KT;
  const int t0 = (nkt_all * kslice) / ks, t1 = (nkt_all * (kslice + 1)) / ks;
  const int nkt = t1 - t0;
  const int M = a.M;
  const act_t* Wd = reinterpret_cast<const act_t*>(S.w);

  // ---- DMA: unit u of K-tile T -> buffer T & 1. This wave issues subtiles idx = n * wave + j (j < n; n = 2,
  // or NA for a weight unit) of every unit: row-tile unit_rt(u, idx >> 1), k-step idx & 1. Lane L -> row
  // 16 rt + (L >> 2), physical chunk L & 3 <- logical chunk (L & 3) ^ swz(L >> 2).
  const int lc = (lane & 3) ^ swz(lane >> 2);
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  auto dma = [&](int u, int T) __attribute__((always_inline)) {
    const int Tc = t0 + min(T, nkt - 1);       // clamped: past the end re-stages the last tile (same bytes)
    const bool bu = u == 1 || u == 2;
    const uint32_t buf = base + (uint32_t)(T & 1) * TB + (bu ? (uint32_t)C::AB : 0u);
    const int n = bu ? 2 : NA;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j >= n) break;
      const int idx = n * wave + j;
      const int rt = unit_rt<BN>(u, idx >> 1), kstep = idx & 1;
      const act_t* src;
      if (u == 1 || u == 2) {
        const int row = min(16 * rt + (lane >> 2), M - 1);
        src = a.x + (size_t)row * a.ldx;
      } else {
        const int row = min(row0 + 16 * rt + (lane >> 2), S.rows - 1);
        src = Wd + (size_t)row * S.K;
      }
      glds16(src + (size_t)Tc * KT + kstep * 32 + lc * 8, buf + (uint32_t)(rt * 2 + kstep) * 1024u);
    }
  };

  // ---- fragments: lane reads row (l & 15) of a 16-row subtile, logical chunk l >> 4
  const int fro = (lane & 15) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4);
  f16x8 FA[NQH][2], FB0[2][2], FB1[2][2];
  auto rdA = [&](int T, int nq) __attribute__((always_inline)) {
    const uint8_t* p = lds + (T & 1) * TB + fro;
#pragma unroll
    for (int i = 0; i < NQH; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        FA[i][s] = *reinterpret_cast<const f16x8*>(p + ((wr * C::RTG + nq * NQH + i) * 2 + s) * 1024);
  };
  auto rdB = [&](f16x8 (&F)[2][2], int T, int mh) __attribute__((always_inline)) {
    const uint8_t* p = lds + (T & 1) * TB + C::AB + fro;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) F[i][s] = *reinterpret_cast<const f16x8*>(p + ((wc * 4 + mh * 2 + i) * 2 + s) * 1024);
  };
  f32x4 acc[2 * NQH][4];
#pragma unroll
  for (int i = 0; i < 2 * NQH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int nq, int mh, const f16x8 (&F)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NQH; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[nq * NQH + i][mh * 2 + j] = mfma16(FA[i][s], F[j][s], acc[nq * NQH + i][mh * 2 + j]);
  };
  auto bar = []() __attribute__((always_inline)) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if (nkt > 0) {
    // prologue: what the steady state would have issued before phase Q0(0): U0(0) U1(0) U2(0) U3(0) U0(1)
    // U1(1); K-tile 0 complete (2 units left in flight), then one barrier for all and group 1's stagger
    dma(0, 0);
    dma(1, 0);
    dma(2, 0);
    dma(3, 0);
    dma(0, 1);
    dma(1, 1);
    wait_vm<C::VM_PRO>();
    bar();
    if (wr == 1) bar();
    for (int T = 0; T < nkt; ++T) {
      // ---- Q0: (nq0, mh0); stage U2(T+1)
      rdA(T, 0);
      rdB(FB0, T, 0);
      dma(2, T + 1);
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      mma(0, 0, FB0);
      __builtin_amdgcn_s_setprio(0);
      wait_vm<C::VM_Q0>();
      bar();
      // ---- Q1: (nq0, mh1); stage U3(T+1)
      rdB(FB1, T, 1);
      dma(3, T + 1);
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      mma(0, 1, FB1);
      __builtin_amdgcn_s_setprio(0);
      wait_vm<C::VM_Q1>();
      bar();
      // ---- Q2: (nq1, mh1); stage U0(T+2)
      rdA(T, 1);
      dma(0, T + 2);
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      mma(1, 1, FB1);
      __builtin_amdgcn_s_setprio(0);
      wait_vm<C::VM_Q2>();
      bar();
      // ---- Q3: (nq1, mh0) from registers; stage U1(T+2)
      dma(1, T + 2);
      bar();
      __builtin_amdgcn_s_setprio(1);
      mma(1, 0, FB0);
      __builtin_amdgcn_s_setprio(0);
      wait_vm<C::VM_Q3>();
      bar();
    }
    if (wr == 0) bar();                         // barrier counts even again
  }
  wait_vm<0>();                                 // drain the clamped tail DMAs
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  h10_epilogue<BN>(acc, S, row0, kslice, ks, a, ws);
}

template <int BN>
__global__ __launch_bounds__(512, 1) void hgemm10_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                          int nmb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t h10lds[];
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
  const int row0 = (tile - S.tile_begin) * BN;       // (host tile counts use BN-row tiles)
  h10_tile<BN>(S, row0, kslice, ks, a, ws, h10lds);
}

template <int BN>
int launch_t(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  constexpr int LDS = H10<BN>::LDS;
  const int nmb = (a.M + BM - 1) / BM;
  const int grid = ((ntiles + 7) / 8) * 8 * nmb * ks;
  static bool attr = false;
  if (!attr) {   // > 64 KiB of dynamic LDS must be opted into
    if (hipFuncSetAttribute((const void*)hgemm10_kernel<BN>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS) !=
        hipSuccess)
      return -1;
    attr = true;
  }
  hipLaunchKernelGGL(hgemm10_kernel<BN>, dim3(grid), dim3(512), LDS, st, sl, a, ks, ws, ntiles, nmb);
  return (int)hipGetLastError();
}

// bn: weight rows per workgroup tile (256 or 128)
int launch_dense10(int bn, const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st) {
  if (bn == 256) return launch_t<256>(sl, ntiles, ks, ws, a, st);
  if (bn == 128) return launch_t<128>(sl, ntiles, ks, ws, a, st);
  return -1;
}


}  // namespace nls_hg10
