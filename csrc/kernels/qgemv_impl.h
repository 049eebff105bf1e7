// Quantised GEMV / skinny GEMM for decode (M <= 64 activation rows), gfx950.
//
//   y[m, n] = alpha * sum_k x[m, k] * W[n, k]      (W in GGUF block formats)
//
// Design (SURVEY.md §2F "gemv_q*"): decode is HBM-bound on the weight stream,
// so every weight byte is read exactly once, straight into VGPRs (no LDS round
// trip, non-temporal loads), dequantised in registers to f16 (magic-number dequant,
// common.h) and fed to v_mfma_f32_16x16x32_f16 as the B operand (16 weight rows per tile). The
// activation rows (batch, padded to 16) are the A operand, so batch 1..16 costs
// the same MFMA issue as batch 1 and the weight dequant is amortised over the
// whole batch. A workgroup owns RT*16 output rows; its WAVES waves split K and
// reduce through LDS, so no atomics and bit-reproducible results.
//
// One launch may cover several weight matrices ("segments": fused Q|K|V with
// per-matrix quant types, or the experts of an MoE layer) and applies a fused
// epilogue: plain store, residual add (y += alpha*acc), SwiGLU on interleaved
// gate/up rows, and a fused greedy arg-max (packed u64 atomicMax per row).
#pragma once
#include "common.h"
#include "moe_route.h"

namespace nls_gemv {


// EPI_SLABS: split-K partial slabs only (the caller fuses the reduce, e.g. with RMSNorm);
// EPI_ARGMAX: fused arg-max keys only, no logits stored (greedy decode)
// EPI_ROPE: the Q|K|V projection's rows leave the tile rotated (adjacent-pair RoPE, + optional bias)
//           straight into q (bf16) and the paged K/V cache: no fp32 qkv round trip, no RoPE launch
enum Epi : int { EPI_F32 = 0, EPI_ACT = 1, EPI_ADD_F32 = 2, EPI_SWIGLU = 3, EPI_SLABS = 4, EPI_ARGMAX = 5,
                 EPI_ROPE = 6 };

struct Seg {
  const uint8_t* w;
  const int* xmap;     // optional: segment-local batch row -> x row (-1: none)
  const int* ymap;     // optional: segment-local batch row -> y row
  const int* mcount;   // optional: device count of valid rows (tiles skip when 0)
  int type, rows, K, tile_begin, ycol, tile_begin_col;
};
struct SegList { Seg s[8]; int nseg; int pad[3]; };

struct GemvArgs {
  const act_t* x; long ldx;
  void* y; long ldy;
  int M;               // rows of x / y (or max rows per segment when mapped)
  int epi;
  float alpha;
  int pad;            // path B split-K: total raw output columns
  unsigned long long* argmax;   // optional [M] packed (ordered value << 32 | ~idx)
  int m0, mtot;       // large-M split-K: first activation row of this block, total rows (slab index)
  // optional fused input RMSNorm (path A, staged rows): x = f16(rmsnorm(xf[m]) * nw), xf f32
  const float* xf; long ldxf;
  const float* nw; float eps;
  // EPI_ROPE operands (see rope_kv_kernel in ops.hip for the cache layout)
  const int* pos; const int* slot; const float* cs; const float* bias;
  __bf16* q_out; long ldq; __bf16* kc; __bf16* vc; int Hq, Hkv, D;
  // EPI_ADD_F32 + onw: after the residual update the LAST workgroup to finish (agent-scope ticket
  // `cnt`, zero between launches) normalises the updated rows: hout = f16(rmsnorm(y) * onw)
  act_t* hout; long ldh; const float* onw; int* cnt;
  // RMSNorm split across a producer / consumer pair (no norm launch, no full-row reduction pass):
  // an EPI_ADD_F32 path-A launch writes, per token m, its workgroup's share of sum(x^2) over the
  // rows it updated to ssq_out[m * ldss + blockIdx.x]; a consumer with xf / nw sums the nss_in
  // shares of ssq_in (fixed order: deterministic) to get the row's inverse RMS.
  float* ssq_out; const float* ssq_in; int ldss, nss_in;
  // device-selected segments (MoE decode, few tokens): workgroup i serves segment sel[i / sel_tiles] -
  // sel_base (out of range or a repeat of an earlier slot: exit), tile i % sel_tiles of it -- only the
  // routed experts' tiles are launched instead of every expert's (most of which would exit at once)
  const int* sel; int sel_tiles, sel_base, pad1;
  // MoE decode (with onw): after the residual update + FFN RMSNorm the last workgroup also computes the router
  // logits hout . wr[e] (wr: the router's f16 copy [E][D]) and the top-k route (route_one) -- the separate
  // norm + router + route launch folded away. counts [E] are zeroed here first.
  const act_t* wr; int E, topk, renorm, rcap;
  float* rlogits; float* topw; int* counts; int* xrows; int* yrows; int* rsel;
};

// inv[m] = 1 / rms of rows m < M from producer partial sums of squares (see GemvArgs::ssq_in); one
// wave per row, lanes sum the shares in a fixed order; ends with a workgroup barrier
template <int NT>
DEVI void ssq_inv(const float* ssq, int ldss, int n, int M, int K, float eps, float* inv) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int m = wave; m < M; m += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < n; j += 64) s += ssq[(size_t)m * ldss + j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) inv[m] = rsqrtf(s / (float)K + eps);
  }
  __syncthreads();
}

// Workgroup ticket: true in exactly one workgroup, the last of `n` to arrive, after which every
// global store of the others is visible to it (cdna_hip_programming.md Guideline 16: each wave drains
// its stores, barrier, one lane releases at agent scope then bumps the counter; the last arriver
// acquires). The last arriver re-arms the counter for the next launch. `flag`: one LDS int.
DEVI bool last_arriver(int* cnt, int n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == n - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// rows [0, M) of y (f32, width D, stride ldy) -> hout = f16(rmsnorm(row) * w); one workgroup of NT threads
template <int NT>
DEVI void rows_rmsnorm(const float* y, long ldy, int M, int D, const float* w, float eps, act_t* hout, long ldh,
                       float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  typedef act_t act4 __attribute__((ext_vector_type(4)));
  for (int m = 0; m < M; ++m) {
    const float* yr = y + (size_t)m * ldy;
    float ss = 0.f;
    for (int i = threadIdx.x * 4; i < D; i += NT * 4) {
      const float4 v = *reinterpret_cast<const float4*>(yr + i);
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) tot += red[i];
    __syncthreads();
    const float inv = rsqrtf(tot / (float)D + eps);
    for (int i = threadIdx.x * 4; i < D; i += NT * 4) {
      const float4 v = *reinterpret_cast<const float4*>(yr + i);
      const float4 g = *reinterpret_cast<const float4*>(w + i);
      *reinterpret_cast<act4*>(hout + (size_t)m * ldh + i) =
          act4{(act_t)(v.x * inv * g.x), (act_t)(v.y * inv * g.y), (act_t)(v.z * inv * g.z), (act_t)(v.w * inv * g.w)};
    }
  }
}

// EPI_ROPE of the dense GEMMs (modes 4/5/10, split-K 1): Q|K|V column `col` of activation row `b` (global
// row) with value v and the value p of its RoPE partner column col ^ 1 (adjacent pairs, as path A): add the
// bias, rotate q / k, store bf16 into q or the paged K / V cache (slot < 0: padding row, no cache write)
DEVI void rope_store1(const GemvArgs& a, int col, int b, float v, float p) {
  const bool odd = col & 1;
  float x0 = odd ? p : v, x1 = odd ? v : p;
  if (a.bias) {
    x0 += a.bias[col & ~1];
    x1 += a.bias[col | 1];
  }
  const int h = col / a.D, dd = col - h * a.D;
  const long s = a.slot[b];
  float y = odd ? x1 : x0;
  __bf16* d = nullptr;
  if (h < a.Hq + a.Hkv) {
    const float2 c = reinterpret_cast<const float2*>(a.cs + (size_t)a.pos[b] * a.D)[dd >> 1];
    y = odd ? x0 * c.y + x1 * c.x : x0 * c.x - x1 * c.y;
    if (h < a.Hq) d = a.q_out + (size_t)b * a.ldq + col;
    else if (s >= 0) d = a.kc + ((size_t)s * a.Hkv + (h - a.Hq)) * a.D + dd;
  } else if (s >= 0) {
    d = a.vc + ((size_t)s * a.Hkv + (h - a.Hq - a.Hkv)) * a.D + dd;
  }
  if (d) *d = (__bf16)y;
}

// MoE route in the last workgroup (GemvArgs::wr): router logits of the M normalised rows hout (f16, as
// moe_norm_route_kernel multiplies them) against the f16 router copy, then one wave per token routes it.
// scratch: >= NT / 64 * 64 + 4 * 64 floats.
template <int NT>
DEVI void route_rows(const GemvArgs& a, int M, int D, float* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = NT / 64;
  float* red = scratch;                  // [NW][64]
  float* lg = scratch + NW * 64;         // [4][64]
  for (int e = threadIdx.x; e < a.E; e += NT) a.counts[e] = 0;
  __syncthreads();                       // (hout written above and the counts zeroed, visible to the workgroup)
  for (int t = 0; t < M; ++t) {
    const act_t* hr = a.hout + (size_t)t * a.ldh;
    for (int e = 0; e < a.E; ++e) {
      const act_t* wr = a.wr + (size_t)e * D;
      float acc = 0.f;
      for (int i = threadIdx.x * 4; i < D; i += NT * 4) {
        typedef act_t act4 __attribute__((ext_vector_type(4)));
        const act4 hv = *reinterpret_cast<const act4*>(hr + i);
        const act4 wv = *reinterpret_cast<const act4*>(wr + i);
        acc += (float)hv.x * (float)wv.x + (float)hv.y * (float)wv.y + (float)hv.z * (float)wv.z +
               (float)hv.w * (float)wv.w;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) red[wave * 64 + e] = acc;
    }
    __syncthreads();
    if (threadIdx.x < a.E) {
      float s2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s2 += red[w * 64 + threadIdx.x];
      lg[t * 64 + threadIdx.x] = s2;
      a.rlogits[(size_t)t * a.E + threadIdx.x] = s2;
    }
    __syncthreads();
  }
  if (wave < M) route_one(lg + wave * 64, wave, lane, a.E, a.topk, a.renorm, a.topw, a.counts, a.xrows, a.yrows,
                          a.rcap, a.rsel);
}

DEVI unsigned long long argmax_key(float v, int idx) {
  uint32_t u = __builtin_bit_cast(uint32_t, v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xFFFFFFFFu - (uint32_t)idx);
}

// x * sigmoid(x) with the hardware reciprocal (1 ulp; an IEEE divide is ~10 instructions per value in
// the GEMM epilogues). exp(-g) = inf for g << 0 gives g * 0 = -0.
DEVI float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }


// Batch-1 activation staging of the XL paths in two halves. xpre() issues every load of the row -- the
// f16 input row, or for a fused input RMSNorm the f32 residual row, the norm weights and the producer's
// sum-of-squares shares -- into registers BEFORE the weight prologue; xput() writes the (normalised)
// row to LDS after it. Loads retire in issue order (in-order vmcnt), so a staging load issued after the
// weight prologue makes the staging wait for the weights, and the loop-carried share / row reads of
// the general path cost several dependent L2 round trips on the critical path (why folding the norms
// into the GEMVs measured neutral in round 2). One row (batch-1 decode) only; false: general path.
struct XPre {
  static constexpr int NX = 8;      // 16-byte chunks per thread (fused norm: NX/2 of x, NX/2 of weights)
  u32x4 v[NX];
  float sh[2];
  int nj;
};

template <int NT>
DEVI bool xpre(XPre& p, const GemvArgs& a, int M, int K, int k0, int kn) {
  constexpr int NX = XPre::NX;
  const int tid = threadIdx.x;
  if (M != 1) return false;
  if (!a.xf) {
    const int nch = kn >> 3;
    if (nch > NX * NT) return false;
    p.nj = (nch + NT - 1) / NT;
#pragma unroll
    for (int j = 0; j < NX; ++j)
      if (j < p.nj) p.v[j] = ld16(a.x + k0 + min(tid + j * NT, nch - 1) * 8);
    return true;
  }
  const int nch = kn >> 2;
  if (nch > (NX / 2) * NT || (a.ssq_in ? a.nss_in > 2 * NT : kn != K)) return false;
  p.nj = (nch + NT - 1) / NT;
#pragma unroll
  for (int j = 0; j < NX / 2; ++j)
    if (j < p.nj) {
      const int c = min(tid + j * NT, nch - 1);
      p.v[j] = ld16(a.xf + k0 + c * 4);
      p.v[NX / 2 + j] = ld16(a.nw + k0 + c * 4);
    }
  if (a.ssq_in) {
#pragma unroll
    for (int i = 0; i < 2; ++i) p.sh[i] = a.ssq_in[min(tid + i * NT, a.nss_in - 1)];
  }
  return true;
}

// the second half: `off(k)` = LDS element offset of slice element k (a multiple of 4); red: NT/64 floats
template <int NT, typename Off>
DEVI void xput(const XPre& p, const GemvArgs& a, int K, int kn, act_t* xs, float* red, Off off) {
  constexpr int NX = XPre::NX;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (!a.xf) {
    const int nch = kn >> 3;
#pragma unroll
    for (int j = 0; j < NX; ++j)
      if (j < p.nj && tid + j * NT < nch) *reinterpret_cast<u32x4*>(xs + off((tid + j * NT) * 8)) = p.v[j];
    return;
  }
  const int nch = kn >> 2;
  float ss = 0.f;
  if (a.ssq_in) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ss += tid + i * NT < a.nss_in ? p.sh[i] : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < NX / 2; ++j)
      if (j < p.nj && tid + j * NT < nch) {
        const float4 v = __builtin_bit_cast(float4, p.v[j]);
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if (lane == 0) red[wave] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) tot += red[w];
  const float inv = rsqrtf(tot / (float)K + a.eps);
  typedef act_t act4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < NX / 2; ++j)
    if (j < p.nj && tid + j * NT < nch) {
      const float4 v = __builtin_bit_cast(float4, p.v[j]), w = __builtin_bit_cast(float4, p.v[NX / 2 + j]);
      *reinterpret_cast<act4*>(xs + off((tid + j * NT) * 4)) =
          act4{(act_t)(v.x * inv * w.x), (act_t)(v.y * inv * w.y), (act_t)(v.z * inv * w.z), (act_t)(v.w * inv * w.w)};
    }
}

// XL: the activation rows are first staged into LDS (batch <= a few rows, no row maps), so the
// main loop's x reads are ds_reads and the VMEM queue holds only the weight stream: its in-order
// vmcnt waits then never drain the DEPTH-deep weight prefetch (global x loads issued each step
// would: waiting for step s's x also waits for every older weight reload).
template <int T, int WAVES, int RT, int MT, bool XL = false>
DEVI void gemv_tile(const Seg& S, int row0, const GemvArgs& a, float* lds) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform
  const int r = lane & 15, g = lane >> 4;
  const WDesc W{S.w, S.rows, S.K};
  const int nb = S.K >> 8;
  const int sb0 = (nb * wave) / WAVES, sb1 = (nb * (wave + 1)) / WAVES;

  int mcount = a.M;
  if (S.mcount) mcount = min(*S.mcount, a.M);

  int rowc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) rowc[rt] = min(row0 + rt * 16 + r, S.rows - 1);

  f32x4 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Weight stream: two register buffers with FIXED roles (A: even, B: odd super-blocks), the
  // loop unrolled by two, so a buffer is reloaded (sb + 2) right after its dequant and no
  // register holding an in-flight load is ever copied (a copy would force vmcnt(0)).
  typedef typename RawOf<T>::type Raw;
  // Weight-stream depth: 4 super-blocks in flight per wave for the K-quants (<= 68 VGPRs of raw
  // blocks at RT = 1), 2 for the wide plain-float tiles. Decode at batch 1 is latency-bound on
  // this stream (each wave owns only K/WAVES of a 16-row tile).
  constexpr int DEPTH = (RT == 1 && sizeof(Raw) <= 80) ? 4 : 2;
  Raw wA[RT], wB[RT], wC[RT], wD[RT];
  // All weight loads are unconditional (super-block index clamped into [sb0, sb1)): a
  // conditional load breaks hipcc's vmcnt bookkeeping at the join and it falls back to
  // vmcnt(0). The clamped tail reloads hit L2 and are never consumed.
  const int sbl = max(sb1 - 1, sb0);
  XPre xp;
  bool xfast = false;
  if constexpr (XL) xfast = xpre<WAVES * 64>(xp, a, mcount, S.K, 0, S.K);
  if (sb0 < sb1) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) wA[rt] = load_raw<T, true>(W, rowc[rt], sb0, g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) wB[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 1, sbl), g);
    if constexpr (DEPTH == 4) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) wC[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 2, sbl), g);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) wD[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 3, sbl), g);
    }
  }
  // (the prologue weight loads above are issued BEFORE the activation rows are staged: at batch 1 the
  // x round trip -- and the fused RMSNorm's reduction -- then overlaps the first weight fetch instead of
  // preceding it on the critical path)
  // Activation rows (A operand row = batch row r of tile mt). Padded / unmapped rows load a
  // valid row (row 0: broadcast, cache-resident) and are zeroed with a select after the load:
  // a lane-conditional load would compile to a branch + vmcnt(0) per K-step that drains the
  // whole weight prefetch (cdna_hip_programming.md §5 "Three .s-level traps" (c)).
  const act_t* xr[MT];
  if constexpr (XL) {
    act_t* xs = reinterpret_cast<act_t*>(lds + (WAVES + 1) * RT * MT * 256);
    if (xfast) {
      xput<WAVES * 64>(xp, a, S.K, S.K, xs, lds, [](int k) { return k; });
    } else if (a.xf) {
      // fused RMSNorm of the residual rows (the decode-time `rmsnorm` launch folded into the GEMV
      // that consumes it: every workgroup normalises the few rows itself, reading them from L2)
      const int K = S.K;
      typedef act_t act4 __attribute__((ext_vector_type(4)));
      if (a.ssq_in) ssq_inv<WAVES * 64>(a.ssq_in, a.ldss, a.nss_in, mcount, K, a.eps, lds + 64);
      for (int m = 0; m < mcount; ++m) {
        const float* xrow = a.xf + (size_t)m * a.ldxf;
        float inv;
        if (a.ssq_in) {
          inv = lds[64 + m];
        } else {
          float ss = 0.f;
          for (int i = threadIdx.x * 4; i < K; i += WAVES * 256) {
            const float4 v = *reinterpret_cast<const float4*>(xrow + i);
            ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
          if (lane == 0) lds[wave] = ss;
          __syncthreads();
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) tot += lds[w];
          __syncthreads();
          inv = rsqrtf(tot / (float)K + a.eps);
        }
        for (int i = threadIdx.x * 4; i < K; i += WAVES * 256) {
          const float4 v = *reinterpret_cast<const float4*>(xrow + i);
          const float4 w = *reinterpret_cast<const float4*>(a.nw + i);
          *reinterpret_cast<act4*>(xs + (size_t)m * K + i) =
              act4{(act_t)(v.x * inv * w.x), (act_t)(v.y * inv * w.y), (act_t)(v.z * inv * w.z), (act_t)(v.w * inv * w.w)};
        }
      }
    } else {
      const int kc = S.K >> 3;                       // 16-B chunks per row
      for (int i = threadIdx.x; i < mcount * kc; i += WAVES * 64) {
        const int row = i / kc, c = i - row * kc;
        *reinterpret_cast<u32x4*>(xs + (size_t)row * S.K + c * 8) = ld16(a.x + (size_t)row * a.ldx + c * 8);
      }
    }
    __syncthreads();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r;
      xr[mt] = xs + (size_t)(m < mcount ? m : 0) * S.K;
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r;
      int src = m < mcount ? m : -1;
      if (S.xmap) src = (m < mcount) ? S.xmap[m] : -1;
      xr[mt] = a.x + (size_t)(src >= 0 ? src : 0) * a.ldx;
    }
  }
  auto step = [&](Raw (&w)[RT], int sb) {
    // 1) activation fragments of this super-block (issued before this step's weight reload)
    f16x8 xa[8][MT];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xa[t][mt] = *reinterpret_cast<const f16x8*>(xr[mt] + sb * 256 + xoff<T>(t, g));
    // the scheduler must not sink these loads below the weight reload (the in-order vmcnt
    // wait for a late x load would then also wait for the reload)
    __builtin_amdgcn_sched_barrier(0);
    // 2) dequant (waits only for this buffer's loads, issued two steps ago)
    f16x8 wf[RT][8];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) dequant<T>(w[rt], g, wf[rt]);
    __builtin_amdgcn_sched_barrier(0);
    // 3) reload the buffer DEPTH super-blocks ahead
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) w[rt] = load_raw<T, true>(W, rowc[rt], min(sb + DEPTH, sbl), g);
    __builtin_amdgcn_sched_barrier(0);
    // 4) MFMA
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f16x8 x8 = xa[t][mt];   // rows >= mcount only reach output rows that are never stored
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          acc[rt][mt] = mfma16(x8, wf[rt][t], acc[rt][mt]);
      }
    }
  };
  int sb = sb0;
  if constexpr (DEPTH == 4) {
    for (; sb + 3 < sb1; sb += 4) {
      step(wA, sb);
      step(wB, sb + 1);
      step(wC, sb + 2);
      step(wD, sb + 3);
    }
    if (sb < sb1) step(wA, sb);
    if (sb + 1 < sb1) step(wB, sb + 1);
    if (sb + 2 < sb1) step(wC, sb + 2);
  } else {
    for (; sb + 1 < sb1; sb += 2) {
      step(wA, sb);
      step(wB, sb + 1);
    }
    if (sb < sb1) step(wA, sb);
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
  if (a.epi == EPI_ROPE) {
    // a head's pair (2i, 2i+1) = tile rows (rr, rr+1): tiles are 16-row aligned and D is even
    for (int e = threadIdx.x; e < RT * 8 * ncols; e += WAVES * 64) {
      const int bb = e % ncols, rr = 2 * (e / ncols);
      const int row = row0 + rr;
      if (bb >= mcount || row >= S.rows) continue;
      const int col = S.ycol + row;              // column of the fused Q|K|V output
      float x0 = tile[rr * ncols + bb], x1 = tile[(rr + 1) * ncols + bb];
      if (a.bias) {
        x0 += a.bias[col];
        x1 += a.bias[col + 1];
      }
      const int h = col / a.D, dd = col - h * a.D;
      const long s = a.slot[bb];
      __bf16* d = nullptr;
      if (h < a.Hq + a.Hkv) {
        const float2 c = reinterpret_cast<const float2*>(a.cs + (size_t)a.pos[bb] * a.D)[dd >> 1];
        const float y0 = x0 * c.x - x1 * c.y, y1 = x0 * c.y + x1 * c.x;
        x0 = y0;
        x1 = y1;
        if (h < a.Hq) d = a.q_out + (size_t)bb * a.ldq + col;
        else if (s >= 0) d = a.kc + ((size_t)s * a.Hkv + (h - a.Hq)) * a.D + dd;
      } else if (s >= 0) {
        d = a.vc + ((size_t)s * a.Hkv + (h - a.Hq - a.Hkv)) * a.D + dd;
      }
      if (d) {
        typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<bf2*>(d) = bf2{(__bf16)x0, (__bf16)x1};
      }
    }
    return;
  }
  if (a.epi == EPI_SWIGLU) {
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
      reinterpret_cast<act_t*>(a.y)[(size_t)yrow * a.ldy + n] = (act_t)(silu(gv) * uv);
    }
    return;
  }
  float sq = 0.f;        // ssq_out: this thread's share of sum(x^2); its token bb = threadIdx.x % ncols
  for (int e = threadIdx.x; e < RT * 16 * ncols; e += WAVES * 64) {
    const int bb = e % ncols, rr = e / ncols;
    const int row = row0 + rr;
    if (bb >= mcount || row >= S.rows) continue;
    const float v = tile[rr * ncols + bb];
    const int yrow = S.ymap ? S.ymap[bb] : bb;
    const size_t off = (size_t)yrow * a.ldy + S.ycol + row;
    if (a.epi == EPI_F32) {
      reinterpret_cast<float*>(a.y)[off] = v;
    } else if (a.epi == EPI_ADD_F32) {
      float* p = reinterpret_cast<float*>(a.y) + off;
      const float nv = *p + v;
      *p = nv;
      sq += nv * nv;
    } else if (a.epi == EPI_ACT) {
      reinterpret_cast<act_t*>(a.y)[off] = (act_t)v;
    }
  }
  if (a.ssq_out) {
    // per-token share of sum(x^2) over this workgroup's rows -> slot blockIdx.x (the host checks
    // (WAVES * 64) % ncols == 0, so a thread's elements all belong to one token)
    __syncthreads();                       // the tile reads above are done: reuse the reduce area
    lds[threadIdx.x] = sq;
    __syncthreads();
    if (threadIdx.x < min(mcount, ncols)) {
      float t = 0.f;
      for (int j = threadIdx.x; j < WAVES * 64; j += ncols) t += lds[j];
      a.ssq_out[(size_t)threadIdx.x * a.ldss + blockIdx.x] = t;
    }
  }
  if (a.onw) {
    // residual + RMSNorm fusion: the next layer's input norm runs in the last workgroup
    int* flag = reinterpret_cast<int*>(lds);
    if (!last_arriver(a.cnt, gridDim.x, flag)) return;
    rows_rmsnorm<WAVES * 64>(reinterpret_cast<const float*>(a.y), a.ldy, mcount, a.pad, a.onw, a.eps, a.hout, a.ldh,
                             lds + 16);
    if (a.wr) route_rows<WAVES * 64>(a, mcount, a.pad, lds + 16);
    return;
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

// KSET 0: Q4_K/Q6_K (the Q4_K_M mix); KSET 1: Q5_K/Q6_K/Q8_0; KSET 2: plain F16/BF16/F32. Splitting the format
// switch keeps the register budget of the quantised kernels small (a switch case's
// VGPR demand is paid by every case).
template <int WAVES, int RT, int MT, int KSET, bool XL = false>
__global__ __launch_bounds__(WAVES * 64) void qgemv_kernel(SegList segs, GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  int tile = blockIdx.x;
  Seg S = segs.s[0];
  if (a.sel) {
    const int slot = blockIdx.x / a.sel_tiles;
    const int e = a.sel[slot] - a.sel_base;
    if (e < 0 || e >= segs.nseg) return;
    for (int s2 = 0; s2 < slot; ++s2)
      if (a.sel[s2] - a.sel_base == e) return;     // expert already served by an earlier slot
#pragma unroll
    for (int i = 1; i < 8; ++i)
      if (i == e) S = segs.s[i];                 // static indices: no scratch copy of the arg array
    tile = S.tile_begin + blockIdx.x % a.sel_tiles;
  } else {
#pragma unroll
    for (int i = 1; i < 8; ++i)
      if (i < segs.nseg && tile >= segs.s[i].tile_begin) S = segs.s[i];
  }
  if (S.mcount && *S.mcount <= 0) return;     // MoE expert with no routed tokens
  const int row0 = (tile - S.tile_begin) * RT * 16;
  if constexpr (KSET == 0) {
    switch (S.type) {
      case QT_Q4_K: gemv_tile<QT_Q4_K, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_Q6_K: gemv_tile<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      default: break;
    }
  } else if constexpr (KSET == 1) {
    switch (S.type) {
      case QT_Q5_K: gemv_tile<QT_Q5_K, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_Q6_K: gemv_tile<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_Q8_0: gemv_tile<QT_Q8_0, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      default: break;
    }
  } else if constexpr (KSET == 3) {
    switch (S.type) {
      case QT_Q51: gemv_tile<QT_Q51, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_Q6_K: gemv_tile<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_Q8_0: gemv_tile<QT_Q8_0, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      default: break;
    }
  } else {
    switch (S.type) {
      case QT_F16: gemv_tile<QT_F16, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_BF16: gemv_tile<QT_BF16, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      case QT_F32: gemv_tile<QT_F32, WAVES, RT, MT, XL>(S, row0, a, lds); break;
      default: break;
    }
  }
}

// ===========================================================================
// Path B (batch >= ~16): waves split ROWS, not K. The activation tile of the current
// 256-wide super-block (M x 256 f16, XOR-swizzled 16-B chunks) is staged once per
// workgroup in LDS (double-buffered) and read by every wave with ds_read_b128, so x is
// fetched from L2 once per WAVES*RT*16 weight rows instead of once per 16. Optional
// split-K over workgroups (KS > 1) writes fp32 partial slabs; splitk_reduce applies
// the epilogue in a fixed order (deterministic, no float atomics).
// ===========================================================================
constexpr size_t XL_LDS_BYTES = 48 * 1024;    // path-B XL: largest staged x slice
#ifndef NLS_XL_DEPTH
#define NLS_XL_DEPTH 2
#endif
constexpr int XL_DEPTH = NLS_XL_DEPTH;         // path-B XL: weight super-blocks in flight per wave
#ifndef NLS_XL_DEPTH2
#define NLS_XL_DEPTH2 2
#endif
constexpr int XL_DEPTH2 = NLS_XL_DEPTH2;       // ... with two 16-row tiles per wave (RT = 2: batch-1 gate|up)

DEVI int lds_off(int row, int k) {            // element offset in a [rows][256] f16 tile
  const int ch = (k >> 3) ^ (row & 15);
  return row * 256 + ch * 8 + (k & 7);
}

// XL (few rows, MT = 1): the workgroup's whole x slice [M][K/ks] is staged in LDS once, so the main
// loop issues only weight loads -- no per-step global x load whose in-order vmcnt wait would drain the
// DEPTH-deep weight prefetch, and no per-step barrier (batch-1 gate|up / down / lm_head streaming).
// NA: activation tiles actually multiplied (<= MT, the LDS allocation): MoE blocks carry a device-side
// row count, so a 128-row block with ~64 routed rows runs 4 tiles, not 8. xm / ym: MoE row maps
// (block-local row -> x row / y row; nullptr: plain rows).
template <int T, int WAVES, int RT, int MT, bool XL = false, int NA = MT>
DEVI void mm_tile(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, act_t* lds,
                  const int* xm = nullptr, const int* ym = nullptr) {
  static_assert(NA >= 1 && NA <= MT, "active tiles exceed the staged tile");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const WDesc W{S.w, S.rows, S.K};
  const int nb = S.K >> 8;
  const int sb0 = (nb * kslice) / ks, sb1 = (nb * (kslice + 1)) / ks;
  const int M = a.M;
  const int base = row0 + wave * RT * 16;
  int rowc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) rowc[rt] = min(base + rt * 16 + r, S.rows - 1);

  constexpr int NT = WAVES * 64;
  f32x4 acc[RT][NA];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < NA; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (XL) {
    static_assert(MT == 1, "XL stages one activation tile");
    typedef typename RawOf<T>::type Raw;
    // no per-step x traffic here, so the weight stream can run XL_DEPTH super-blocks ahead
    constexpr int DEPTH = RT == 1 ? (sizeof(Raw) <= 48 ? XL_DEPTH : (sizeof(Raw) <= 80 ? 4 : 2))
                                  : (sizeof(Raw) <= 48 ? XL_DEPTH2 : 2);
    Raw wb[DEPTH][RT];
    const int sbl = max(sb1 - 1, sb0);
    XPre xp;              // batch 1: the x slice's loads go out first (xpre), the weight prologue after them
    const bool xfast = xpre<NT>(xp, a, M, S.K, sb0 * 256, (sb1 - sb0) * 256);
    if (sb0 < sb1) {      // weight prologue: the x staging below overlaps its latency
#pragma unroll
      for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) wb[d][rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + d, sbl), g);
    }
    // x slice -> LDS [sb - sb0][M][256] (XOR-swizzled 16-B chunks)
    const int kc = (sb1 - sb0) * 32;
    if (xfast) {
      xput<NT>(xp, a, S.K, (sb1 - sb0) * 256, lds, reinterpret_cast<float*>(lds + (size_t)M * kc * 8),
               [M](int k) { return (k >> 8) * M * 256 + lds_off(0, k & 255); });
    } else if (a.xf) {
      // fused input RMSNorm from the producer's partial sums of squares (the slice may be a
      // split-K part of the row; the norm needs the whole row: launch_b requires ssq_in here)
      float* inv = reinterpret_cast<float*>(lds + (size_t)M * kc * 8);
      ssq_inv<NT>(a.ssq_in, a.ldss, a.nss_in, M, S.K, a.eps, inv);
      typedef act_t act8 __attribute__((ext_vector_type(8)));
      for (int i = threadIdx.x; i < M * kc; i += NT) {
        const int row = i / kc, c = i - row * kc;
        const size_t k0 = (size_t)sb0 * 256 + c * 8;
        const float* xp = a.xf + (size_t)row * a.ldxf + k0;
        const float4 v0 = *reinterpret_cast<const float4*>(xp), v1 = *reinterpret_cast<const float4*>(xp + 4);
        const float4 w0 = *reinterpret_cast<const float4*>(a.nw + k0), w1 = *reinterpret_cast<const float4*>(a.nw + k0 + 4);
        const float s = inv[row];
        *reinterpret_cast<act8*>(lds + (size_t)(c >> 5) * M * 256 + lds_off(row, (c & 31) * 8)) =
            act8{(act_t)(v0.x * s * w0.x), (act_t)(v0.y * s * w0.y), (act_t)(v0.z * s * w0.z), (act_t)(v0.w * s * w0.w),
                 (act_t)(v1.x * s * w1.x), (act_t)(v1.y * s * w1.y), (act_t)(v1.z * s * w1.z), (act_t)(v1.w * s * w1.w)};
      }
    } else {
      for (int i = threadIdx.x; i < M * kc; i += NT) {
        const int row = i / kc, c = i - row * kc;
        *reinterpret_cast<u32x4*>(lds + (size_t)(c >> 5) * M * 256 + lds_off(row, (c & 31) * 8)) =
            ld16(a.x + (size_t)row * a.ldx + (size_t)sb0 * 256 + c * 8);
      }
    }
    __syncthreads();
    const int xrow = min(r, M - 1);      // rows >= M feed outputs that are never stored
    auto step = [&](Raw (&w)[RT], int sb) {
      const act_t* xb = lds + (size_t)(sb - sb0) * M * 256;
      f16x8 xa[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) xa[t] = *reinterpret_cast<const f16x8*>(xb + lds_off(xrow, xoff<T>(t, g)));
      __builtin_amdgcn_sched_barrier(0);
      f16x8 wf[RT][8];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) dequant<T>(w[rt], g, wf[rt]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) w[rt] = load_raw<T, true>(W, rowc[rt], min(sb + DEPTH, sbl), g);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][0] = mfma16(xa[t], wf[rt][t], acc[rt][0]);
    };
    // buffer d always holds super-blocks = d (mod DEPTH): fixed roles, fully unrolled (no copies of
    // registers with loads in flight, no runtime-indexed register arrays)
    int sb = sb0;
    for (; sb + DEPTH - 1 < sb1; sb += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) step(wb[d], sb + d);
    }
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
      if (sb + d < sb1) step(wb[d], sb + d);
  } else {
  constexpr int NCH = (NA * 16 * 32) / NT;               // 16-B chunks staged per thread (active rows)
  static_assert((NA * 16 * 32) % NT == 0, "staging must divide evenly");
  // large tiles stage x in two halves (half the staging registers)
  constexpr bool SPLITX = NA >= 4 && NCH % 2 == 0;
  constexpr int NCHR = SPLITX ? NCH / 2 : NCH;
  u32x4 xst[NCHR];
  // source row of each staged chunk (fixed for the whole K loop): rows >= M only feed output rows that
  // are never stored -- clamp, never branch; MoE blocks gather through xm
  // (two 16-bit row indices per register: the 8-tile instance sits at the 256-VGPR limit)
  uint32_t xsr[(NCH + 1) / 2];
#pragma unroll
  for (int c = 0; c < (NCH + 1) / 2; ++c) xsr[c] = 0u;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int row = min((int)((threadIdx.x + c * NT) >> 5), M - 1);
    xsr[c >> 1] |= (uint32_t)(xm ? xm[row] : row) << (16 * (c & 1));
  }
  auto load_xh = [&](int sb, int h) {
#pragma unroll
    for (int c = 0; c < NCHR; ++c) {
      const int idx = threadIdx.x + (c + h * NCHR) * NT;
      const int ch = idx & 31, cc = c + h * NCHR;
      const uint32_t row = (xsr[cc >> 1] >> (16 * (cc & 1))) & 0xFFFFu;
      xst[c] = ld16(a.x + (size_t)row * a.ldx + sb * 256 + ch * 8);
    }
  };
  auto store_xh = [&](int buf, int h) {
#pragma unroll
    for (int c = 0; c < NCHR; ++c) {
      const int idx = threadIdx.x + (c + h * NCHR) * NT;
      const int row = idx >> 5, ch = idx & 31;
      *reinterpret_cast<u32x4*>(lds + buf * (MT * 16 * 256) + lds_off(row, ch * 8)) = xst[c];
    }
  };
  auto stage_full = [&](int sb, int buf) {      // prologue: both halves
    load_xh(sb, 0);
    store_xh(buf, 0);
    if constexpr (SPLITX) {
      load_xh(sb, 1);
      store_xh(buf, 1);
    }
  };

  typedef typename RawOf<T>::type Raw;
  // weight-stream depth: few-row launches (MT <= 2) are latency-bound on the weight stream (batch-1
  // gate|up: one 128-row workgroup per CU), so keep 4 super-blocks in flight per wave there
  constexpr int DEPTH = (MT <= 2 && RT == 1 && sizeof(Raw) <= 80) ? 4 : 2;
  Raw wA[RT], wB[RT], wC[RT], wD[RT];
  const int sbl = max(sb1 - 1, sb0);
  if (sb0 < sb1) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) wA[rt] = load_raw<T, true>(W, rowc[rt], sb0, g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) wB[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 1, sbl), g);
    if constexpr (DEPTH == 4) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) wC[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 2, sbl), g);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) wD[rt] = load_raw<T, true>(W, rowc[rt], min(sb0 + 3, sbl), g);
    }
    stage_full(sb0, 0);
  }
  __syncthreads();
  // fixed buffer roles, unrolled by two (see path A); x for sb+1 is staged through the other
  // LDS buffer while sb is computed
  auto step = [&](Raw (&w)[RT], int sb) {
    const int buf = (sb - sb0) & 1;
    const int nxt = min(sb + 1, sbl);  // unconditional (clamped): see path A
    load_xh(nxt, 0);
    __builtin_amdgcn_sched_barrier(0);
    const act_t* xb = lds + buf * (MT * 16 * 256);
    if constexpr (MT >= 4) {
      // large tiles: per-K-step fragments (scales once per super-block), weight buffer reloaded
      // after its last use; x half 0 written after K-steps 0-3, half 1 loaded then, written last
      typename ScOf<T>::type sc[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) prep_sc<T>(w[rt], g, sc[rt]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (SPLITX && t == 4) {
          store_xh(buf ^ 1, 0);
          load_xh(nxt, 1);
        }
        f16x8 wt[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) wt[rt] = frag_t<T>(w[rt], sc[rt], t);
        const int ko = xoff<T>(t, g);
#pragma unroll
        for (int mt = 0; mt < NA; ++mt) {
          const f16x8 xa = *reinterpret_cast<const f16x8*>(xb + lds_off(mt * 16 + r, ko));
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
            acc[rt][mt] = mfma16(xa, wt[rt], acc[rt][mt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) w[rt] = load_raw<T, true>(W, rowc[rt], min(sb + DEPTH, sbl), g);
      store_xh(buf ^ 1, SPLITX ? 1 : 0);
    } else {
      f16x8 wf[RT][8];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) dequant<T>(w[rt], g, wf[rt]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) w[rt] = load_raw<T, true>(W, rowc[rt], min(sb + DEPTH, sbl), g);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int ko = xoff<T>(t, g);
#pragma unroll
        for (int mt = 0; mt < NA; ++mt) {
          const f16x8 xa = *reinterpret_cast<const f16x8*>(xb + lds_off(mt * 16 + r, ko));
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
            acc[rt][mt] = mfma16(xa, wf[rt][t], acc[rt][mt]);
        }
      }
      store_xh(buf ^ 1, 0);
    }
    __syncthreads();
  };
  int sb = sb0;
  if constexpr (DEPTH == 4) {
    for (; sb + 3 < sb1; sb += 4) {
      step(wA, sb);
      step(wB, sb + 1);
      step(wC, sb + 2);
      step(wD, sb + 3);
    }
    if (sb < sb1) step(wA, sb);
    if (sb + 1 < sb1) step(wB, sb + 1);
    if (sb + 2 < sb1) step(wC, sb + 2);
  } else {
    for (; sb + 1 < sb1; sb += 2) {
      step(wA, sb);
      step(wB, sb + 1);
    }
    if (sb < sb1) step(wA, sb);
  }
  }   // !XL

  // ---- epilogue straight from the accumulators ---------------------------------
  // lane holds rows (base + rt*16 + r), batch rows mt*16 + 4g + i
  if (ks > 1) {
    const int ntot = a.pad;      // total output columns (all segments, raw rows)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = base + rt * 16 + r;
      if (row >= S.rows) continue;
#pragma unroll
      for (int mt = 0; mt < NA; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = mt * 16 + 4 * g + i;
          if (b >= M) continue;
          if (ym)        // mapped split-K: slab row = the token's y row, columns shared by every expert
            ws[((size_t)kslice * a.mtot + ym[b]) * ntot + S.ycol + row] = acc[rt][mt][i];
          else
            ws[((size_t)kslice * a.mtot + a.m0 + b) * ntot + S.tile_begin_col + row] = acc[rt][mt][i];
        }
    }
    return;
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = base + rt * 16 + r;
#pragma unroll
    for (int mt = 0; mt < NA; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = mt * 16 + 4 * g + i;
        const float v = acc[rt][mt][i] * a.alpha;
        if (a.epi == EPI_SWIGLU) {
          const float u = __shfl_xor(v, 8, 64);
          if (r < 8 && b < M && row < S.rows) {
            const int n = S.ycol + ((base + rt * 16) >> 1) + r;
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
        if (a.argmax) {
          unsigned long long k = (row < S.rows) ? argmax_key(v, S.ycol + row) : 0ull;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long ok = __shfl_xor(k, o, 64);
            k = ok > k ? ok : k;
          }
          if (r == 0 && b < M) atomicMax(a.argmax + b, k);
        }
      }
    }
  }
}

// Active-tile dispatch: only the 8-wave, 2-row-tile, 8-tile instance (the MoE grouped launch) picks NA
// per block -- {2, 4, 6, 8}, rounded up to even to bound the instantiations; the rest run NA = MT.
template <int T, int WAVES, int RT, int MT, bool XL>
DEVI void mm_tile_na(const Seg& S, int row0, int kslice, int ks, const GemvArgs& a, float* ws, act_t* lds,
                     const int* xm, const int* ym) {
  if constexpr (MT == 8 && WAVES == 8 && RT == 2 && !XL) {
    const int na = ((a.M + 15) / 16 + 1) & ~1;
    if (na <= 2) mm_tile<T, WAVES, RT, MT, XL, 2>(S, row0, kslice, ks, a, ws, lds, xm, ym);
    else if (na <= 4) mm_tile<T, WAVES, RT, MT, XL, 4>(S, row0, kslice, ks, a, ws, lds, xm, ym);
    else if (na <= 6) mm_tile<T, WAVES, RT, MT, XL, 6>(S, row0, kslice, ks, a, ws, lds, xm, ym);
    else mm_tile<T, WAVES, RT, MT, XL, 8>(S, row0, kslice, ks, a, ws, lds, xm, ym);
  } else {
    mm_tile<T, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, lds, xm, ym);
  }
}

template <int WAVES, int RT, int MT, int KSET, bool XL = false>
__global__ __launch_bounds__(WAVES * 64) void qmm_kernel(SegList segs, GemvArgs a, int ks, float* ws, int ntiles,
                                                         int nmb) {
  extern __shared__ __attribute__((aligned(16))) act_t xlds[];
  int tile, kslice = 0, mb = 0;
  if (nmb > 1) {
    // Large M (prefill / big decode batches): blocks of MT*16 activation rows. The workgroups
    // sharing one weight tile are placed on ONE XCD (dispatch assigns workgroup i to XCD i % 8),
    // so each weight tile is fetched from HBM once per XCD L2 instead of once per m-block.
    // With split-K (ks > 1) the K slices of a tile are also kept on its XCD.
    const int i = blockIdx.x, xcd = i & 7, j = i >> 3;
    kslice = j % ks;
    mb = (j / ks) % nmb;
    tile = (j / ks / nmb) * 8 + xcd;
    if (tile >= ntiles) return;
  } else {
    tile = blockIdx.x / ks;
    kslice = blockIdx.x % ks;
  }
  Seg S = segs.s[0];
#pragma unroll
  for (int i = 1; i < 8; ++i)
    if (i < segs.nseg && tile >= segs.s[i].tile_begin) S = segs.s[i];
  // MoE grouped launch: the expert's routed-row count lives on the device; m-blocks past it exit
  // before reading any weights (the grid is sized for every token on one expert)
  const int m0 = mb * MT * 16;
  const int mrows = S.mcount ? min(*S.mcount, a.M) : a.M;
  if (m0 >= mrows) return;
  const int* xm = S.xmap ? S.xmap + m0 : nullptr;
  const int* ym = S.ymap ? S.ymap + m0 : nullptr;
  a.m0 = m0;
  if (!xm) a.x += (size_t)m0 * a.ldx;
  const size_t esz = (a.epi == EPI_F32 || a.epi == EPI_ADD_F32 || a.epi == EPI_ARGMAX) ? 4 : 2;
  if (!ym) a.y = (char*)a.y + (size_t)m0 * a.ldy * esz;
  if (a.argmax) a.argmax += m0;
  a.M = min(MT * 16, mrows - m0);
  const int row0 = (tile - S.tile_begin) * WAVES * RT * 16;
  if constexpr (KSET == 0) {
    switch (S.type) {
      case QT_Q4_K: mm_tile_na<QT_Q4_K, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_Q6_K: mm_tile_na<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      default: break;
    }
  } else if constexpr (KSET == 1) {
    switch (S.type) {
      case QT_Q5_K: mm_tile_na<QT_Q5_K, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_Q6_K: mm_tile_na<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_Q8_0: mm_tile_na<QT_Q8_0, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      default: break;
    }
  } else if constexpr (KSET == 3) {
    switch (S.type) {
      case QT_Q51: mm_tile_na<QT_Q51, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_Q6_K: mm_tile_na<QT_Q6_K, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_Q8_0: mm_tile_na<QT_Q8_0, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      default: break;
    }
  } else {
    switch (S.type) {
      case QT_F16: mm_tile<QT_F16, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_BF16: mm_tile<QT_BF16, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      case QT_F32: mm_tile<QT_F32, WAVES, RT, MT, XL>(S, row0, kslice, ks, a, ws, xlds, xm, ym); break;
      default: break;
    }
  }
}

// Split-K reduction + epilogue. ws: [ks][M][ntot] fp32 (ntot = raw output rows over all segments)
struct RedSeg { int col0, rows, ycol, pad; };
struct RedList { RedSeg s[8]; int nseg, pad[3]; };

static __global__ void splitk_reduce_kernel(const float* __restrict__ ws, int ks, int M, int ntot, RedList rl,
                                     GemvArgs a) {
  const int b = blockIdx.y;
  const bool swiglu = a.epi == EPI_SWIGLU;
  const int nout = swiglu ? ntot / 2 : ntot;
  unsigned long long best = 0ull;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nout; j += gridDim.x * blockDim.x) {
    int col = swiglu ? (j >> 3) * 16 + (j & 7) : j;
    RedSeg S = rl.s[0];
    for (int i = 1; i < rl.nseg; ++i)
      if (col >= rl.s[i].col0) S = rl.s[i];
    float v = 0.f, u = 0.f;
    for (int k = 0; k < ks; ++k) {
      v += ws[((size_t)k * M + b) * ntot + col];
      if (swiglu) u += ws[((size_t)k * M + b) * ntot + col + 8];
    }
    v *= a.alpha;
    u *= a.alpha;
    const int row = col - S.col0;
    if (swiglu) {
      const int n = S.ycol + (row >> 4) * 8 + (row & 7);
      reinterpret_cast<act_t*>(a.y)[(size_t)b * a.ldy + n] = (act_t)(silu(v) * u);
      continue;
    }
    const size_t off = (size_t)b * a.ldy + S.ycol + row;
    if (a.epi == EPI_F32) reinterpret_cast<float*>(a.y)[off] = v;
    else if (a.epi == EPI_ADD_F32) reinterpret_cast<float*>(a.y)[off] += v;
    else if (a.epi == EPI_ACT) reinterpret_cast<act_t*>(a.y)[off] = (act_t)v;
    if (a.argmax) {
      const unsigned long long k = argmax_key(v, S.ycol + row);
      best = k > best ? k : best;
    }
  }
  if (a.argmax) {
    // one atomic per workgroup and row (a per-element atomicMax on the one key of a row serialises
    // ~128K updates for an lm_head: 27 us of a 2.2 ms batch-1 step)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long ok = __shfl_xor(best, o, 64);
      best = ok > best ? ok : best;
    }
    __shared__ unsigned long long red[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = red[w] > best ? red[w] : best;
      if (best) atomicMax(a.argmax + b, best);
    }
  }
}


// ---- launch helpers, one kernel type-set (KSET) per translation unit -------------------------
template <int WAVES, int RT, int MT, int KSET>
int launch_t(const SegList& sl, int ntiles, const GemvArgs& a, hipStream_t st) {
  const size_t lds = (size_t)(WAVES + 1) * RT * MT * 256 * sizeof(float);
  if constexpr (MT == 1) {      // stage the activation rows in LDS when they fit (batch-1 decode)
    bool mapped = false;
    for (int i = 0; i < sl.nseg; ++i) mapped |= sl.s[i].xmap != nullptr || sl.s[i].mcount != nullptr;
    const size_t xbytes = (size_t)a.M * sl.s[0].K * sizeof(act_t);
    if (!mapped && lds + xbytes <= 64 * 1024) {
      hipLaunchKernelGGL((qgemv_kernel<WAVES, RT, MT, KSET, true>), dim3(ntiles), dim3(WAVES * 64), lds + xbytes,
                         st, sl, a);
      return (int)hipGetLastError();
    }
  }
  if (a.xf) return -1;          // fused input norm needs the staged (MT = 1, unmapped, fitting) path
  hipLaunchKernelGGL((qgemv_kernel<WAVES, RT, MT, KSET>), dim3(ntiles), dim3(WAVES * 64), lds, st, sl, a);
  return (int)hipGetLastError();
}

template <int WAVES, int RT, int KSET>
int launch_mt(int mt, const SegList& sl, int nt, const GemvArgs& a, hipStream_t st) {
  switch (mt) {
    case 1: return launch_t<WAVES, RT, 1, KSET>(sl, nt, a, st);
    case 2: return launch_t<WAVES, RT, 2, KSET>(sl, nt, a, st);
    case 3: return launch_t<WAVES, RT, 3, KSET>(sl, nt, a, st);
    case 4: return launch_t<WAVES, RT, 4, KSET>(sl, nt, a, st);
  }
  return -1;
}

template <int WAVES, int RT, int MT, int KSET>
int launch_b(const SegList& sl, int ntiles, int ks, float* ws, const GemvArgs& a, hipStream_t st, int nmb) {
  const size_t lds = (size_t)2 * MT * 16 * 256 * sizeof(act_t);
  const int grid = nmb > 1 ? ((ntiles + 7) / 8) * 8 * nmb * ks : ntiles * ks;
  if constexpr (MT == 1) {      // few rows: stage the whole x slice once (XL) when it fits
    bool mapped = false;
    int kmax = 0;
    for (int i = 0; i < sl.nseg; ++i) {
      mapped |= sl.s[i].xmap != nullptr || sl.s[i].mcount != nullptr;
      kmax = max(kmax, sl.s[i].K);
    }
    const size_t xbytes = (size_t)a.M * (((kmax >> 8) + ks - 1) / ks) * 256 * sizeof(act_t);
    if (nmb == 1 && !mapped && xbytes <= XL_LDS_BYTES) {
      const size_t need = a.xf ? xbytes + 64 * sizeof(float) : xbytes;     // + inv-rms scratch
      hipLaunchKernelGGL((qmm_kernel<WAVES, RT, 1, KSET, true>), dim3(grid), dim3(WAVES * 64), max(need, lds), st,
                         sl, a, ks, ws, ntiles, nmb);
      return (int)hipGetLastError();
    }
  }
  if (a.xf) return -1;          // fused input norm: the staged (XL) path only
  if constexpr (WAVES == 7) {   // (the 7-wave instance exists for the staged batch-1 path only)
    return -1;
  } else {
    hipLaunchKernelGGL((qmm_kernel<WAVES, RT, MT, KSET>), dim3(grid), dim3(WAVES * 64), lds, st, sl, a, ks, ws,
                       ntiles, nmb);
    return (int)hipGetLastError();
  }
}

template <int WAVES, int RT, int KSET>
int launch_b_mt(int mt, const SegList& sl, int nt, int ks, float* ws, const GemvArgs& a, hipStream_t st, int nmb) {
  switch (mt) {
    case 1: return launch_b<WAVES, RT, 1, KSET>(sl, nt, ks, ws, a, st, nmb);
    case 2: return launch_b<WAVES, RT, 2, KSET>(sl, nt, ks, ws, a, st, nmb);
    case 3: return launch_b<WAVES, RT, 3, KSET>(sl, nt, ks, ws, a, st, nmb);
    case 4: return launch_b<WAVES, RT, 4, KSET>(sl, nt, ks, ws, a, st, nmb);
    case 8: return launch_b<WAVES, RT, 8, KSET>(sl, nt, ks, ws, a, st, nmb);
  }
  return -1;
}

// Entry of one type-set: path A (mode 0) or path B (mode 1) for every (waves, rt, mt).
template <int KSET>
int launch_kset(int mode, int waves, int rt, int mt, const SegList& sl, int tiles, int ks, float* ws,
                const GemvArgs& a, hipStream_t st, int nmb) {
  if (mode == 1) {
    // 7 waves x one 16-row tile (112 rows per workgroup): 28672 gate|up rows = 256 workgroups, one per CU
    // (4 waves x 2 tiles leave 32 CUs idle at 224); batch-1 staged (XL) launches only
    if (waves == 7) return rt == 1 && mt == 1 ? launch_b<7, 1, 1, KSET>(sl, tiles, ks, ws, a, st, nmb) : -1;
    if (waves == 8) return rt == 1 ? launch_b_mt<8, 1, KSET>(mt, sl, tiles, ks, ws, a, st, nmb)
                                   : launch_b_mt<8, 2, KSET>(mt, sl, tiles, ks, ws, a, st, nmb);
    return rt == 1 ? launch_b_mt<4, 1, KSET>(mt, sl, tiles, ks, ws, a, st, nmb)
                   : launch_b_mt<4, 2, KSET>(mt, sl, tiles, ks, ws, a, st, nmb);
  }
  if (waves == 8) return rt == 1 ? launch_mt<8, 1, KSET>(mt, sl, tiles, a, st) : launch_mt<8, 2, KSET>(mt, sl, tiles, a, st);
  return rt == 1 ? launch_mt<4, 1, KSET>(mt, sl, tiles, a, st) : launch_mt<4, 2, KSET>(mt, sl, tiles, a, st);
}

int launch_k0(int, int, int, int, const SegList&, int, int, float*, const GemvArgs&, hipStream_t, int);
int launch_k1(int, int, int, int, const SegList&, int, int, float*, const GemvArgs&, hipStream_t, int);
int launch_k2(int, int, int, int, const SegList&, int, int, float*, const GemvArgs&, hipStream_t, int);
int launch_k3(int, int, int, int, const SegList&, int, int, float*, const GemvArgs&, hipStream_t, int);

}  // namespace nls_gemv
