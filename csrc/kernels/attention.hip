// Paged grouped-query attention for decode (and prefill expressed as per-token
// causal decode), gfx950. SURVEY.md §2F attn_decode_paged.
//
// KV cache (one layer): k/v [num_slots][Hkv][D] bf16, slot = block_table[seq][pos / BS] * BS + pos % BS.
// Grid: (tokens, Hkv, n_split). A workgroup handles the G = Hq/Hkv query heads that
// share one KV head over one context chunk (split-K / flash-decoding), so a KV row
// is read from HBM once per (token, kv head, chunk) and used by all G heads.
// Lane map: D/8 lanes per key (16 B each = 8 dims), 64/(D/8) keys per wave in flight;
// every lane group keeps its own online-softmax state (m, l, o) which the workgroup
// merges through LDS at the end. With n_split > 1 unnormalised partials go to a
// workspace and are merged (log-sum-exp in base 2) either by the LAST active split of each
// (token, kv head) to finish -- an agent-scope ticket in `cnt`, no second launch -- or, without
// counters, by attn_combine.
#include "common.h"

// NLS_ATTN_PREFETCH2=1 streams K/V two tiles ahead; A/B on MI355X (B=1/16, P=4096) measured it
// 0.3-0.8 % slower than one tile ahead (profiles/attn_prefetch_split_ab.txt), so it is off.
#ifndef NLS_ATTN_PREFETCH2
#define NLS_ATTN_PREFETCH2 0
#endif

namespace {

constexpr float LOG2E = 1.4426950408889634f;

// Keys per flash-decoding split. chunk > 0: fixed; chunk < 0: balanced over n_split with at least
// -chunk keys; chunk == 0: balanced with at least 64 keys below 1K of context, 128 at 1K-2K and 256 above
// (batch-1 A/B, profiles/attn_split_policy_b1.txt: 64-key splits win on short contexts, where the split's
// dependent K/V fetch chain dominates; 128-256-key splits at 1K-4K, where the merge of many partials does).
// With up to 64 splits at batch 1 (models/llama.py _SPLIT_CAP), 8K-32K contexts get 32-64 splits of
// 256-512 keys: 512 workgroups keep enough K/V in flight to stream the cache at HBM rate.
__device__ __forceinline__ int split_chunk(int chunk, int ctx, int n_split, int bs, int short_min = 64) {
  if (chunk > 0) return chunk;
  const int mn = chunk ? -chunk : (ctx >= 2048 ? 256 : (ctx >= 1024 ? 128 : short_min));
  return max(mn, ((ctx + n_split - 1) / n_split + bs - 1) / bs * bs);
}

template <int D, int G, typename KV, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void attn_decode_kernel(
    const __bf16* __restrict__ q, long ldq, const KV* __restrict__ kc, const KV* __restrict__ vc,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ tok_seq,
    const int* __restrict__ ctx_len, int Hkv, int bs, float scale, int chunk, int n_split,
    act_t* __restrict__ out, long ldo, float* __restrict__ part_o, float* __restrict__ part_ml,
    int* __restrict__ cnt) {
  constexpr int LPT = D / 8;          // lanes per key
  constexpr int TPW = 64 / LPT;       // keys per wave per step
  constexpr int NSTREAM = WAVES * TPW;  // independent softmax streams per workgroup (keys per step)
  constexpr int NT = 64 * WAVES;
  const int t = blockIdx.x, kh = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int dl = lane % LPT, ts = lane / LPT;
  const int stream = wave * TPW + ts;
  const int Hq = Hkv * G;

  const int ctx = ctx_len[t];
  chunk = split_chunk(chunk, ctx, n_split, bs);
  const int start = split * chunk;
  if (n_split > 1 && start >= ctx && ctx > 0) return;       // inactive split: combine skips it
  const int end = min(ctx, start + chunk);
  const int* bt = block_tables + (size_t)tok_seq[t] * bt_stride;

  // q for the G heads of this kv head, this lane's 8 dims, pre-scaled for exp2
  float qf[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const u32x4 raw = ld16(q + (size_t)t * ldq + (size_t)(kh * G + h) * D + 8 * dl);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      qf[h][2 * i] = bf2f(raw[i] & 0xFFFF) * scale * LOG2E;
      qf[h][2 * i + 1] = bf2f(raw[i] >> 16) * scale * LOG2E;
    }
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[h][i] = 0.f;
  }

  // Block-table entries are prefetched 64 at a time (one per lane) and broadcast with
  // shuffles; the K/V rows of step i+1 are in flight while step i is computed.
  const int b0 = start / bs;
  const int nblk = (end + bs - 1) / bs;
  int btw = -1, btreg = 0;
  // base is wave-uniform, pos = base + stream (per lane)
  auto slot_of = [&](int pos, int base) -> long {
    const int win = (base / bs - b0) >> 6;
    if (win != btw) {
      btw = win;
      const int e = b0 + win * 64 + lane;
      btreg = e < nblk ? bt[e] : 0;
    }
    const int bi = pos / bs - b0;
    int blk = __shfl(btreg, bi & 63, 64);
    if ((bi >> 6) != win) blk = bt[b0 + bi];      // key straddles the next 64-block window
    return (long)blk * bs + (pos % bs);
  };
  auto kv_off = [&](int pos, int base) -> size_t { return ((size_t)slot_of(pos, base) * Hkv + kh) * D + 8 * dl; };

  // K/V rows PF steps ahead in flight (long contexts at small batch are latency-bound on this chain)
  typedef KVRaw<KV> R;
  typename R::raw kr{}, vr{}, k1{}, v1{};
  if (start < end) {
    const int p0 = min(start + stream, end - 1);
    const size_t off = kv_off(p0, start);
    kr = R::ld(kc + off);
    vr = R::ld(vc + off);
    if (NLS_ATTN_PREFETCH2 && start + NSTREAM < end) {
      const int p1 = min(start + NSTREAM + stream, end - 1);
      const size_t o1 = kv_off(p1, start + NSTREAM);
      k1 = R::ld(kc + o1);
      v1 = R::ld(vc + o1);
    }
  }
  for (int base = start; base < end; base += NSTREAM) {
    const int pos = base + stream;
    const bool valid = pos < end;
    constexpr int PF = NLS_ATTN_PREFETCH2 ? 2 : 1;
    typename R::raw kn = PF == 2 ? k1 : kr, vn = PF == 2 ? v1 : vr;
    if (base + PF * NSTREAM < end) {
      const int pn = min(pos + PF * NSTREAM, end - 1);
      const size_t off = kv_off(pn, base + PF * NSTREAM);
      kn = R::ld(kc + off);
      vn = R::ld(vc + off);
    }
    float kf[8], vf[8];
    const u32x4 kb = R::bf16(kr), vb = R::bf16(vr);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kf[2 * i] = bf2f(kb[i] & 0xFFFF);
      kf[2 * i + 1] = bf2f(kb[i] >> 16);
      vf[2 * i] = bf2f(vb[i] & 0xFFFF);
      vf[2 * i + 1] = bf2f(vb[i] >> 16);
    }
    float s[G];
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += qf[h][i] * kf[i];
#pragma unroll
      for (int o2 = LPT / 2; o2 > 0; o2 >>= 1) acc += __shfl_xor(acc, o2, 64);
      s[h] = valid ? acc : -INFINITY;
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float mn = fmaxf(m[h], s[h]);
      if (mn == -INFINITY) continue;
      const float c = exp2f(m[h] - mn);
      const float p = exp2f(s[h] - mn);
      m[h] = mn;
      l[h] = l[h] * c + p;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] = o[h][i] * c + p * vf[i];
    }
    if constexpr (PF == 2) {
      kr = k1;
      vr = v1;
      k1 = kn;
      v1 = vn;
    } else {
      kr = kn;
      vr = vn;
    }
  }

  // ---- merge the streams. 8 waves: first the TPW streams of each wave with shuffles (log-sum-exp,
  // base 2), then the WAVES per-wave results through LDS (keeps the LDS area at 16 KiB); 4 waves: all
  // NSTREAM streams through LDS directly (measured faster at batch 512, where the merge is a larger
  // share of a short workgroup: profiles/attn_waves_ab.txt)
  constexpr bool SHFL = WAVES == 8;
  constexpr int NM = SHFL ? WAVES : NSTREAM;     // partials merged through LDS
  const int slotm = SHFL ? wave : stream;
#pragma unroll
  for (int off = LPT; SHFL && off < 64; off <<= 1) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float mo = __shfl_xor(m[h], off, 64), lo = __shfl_xor(l[h], off, 64);
      const float mn = fmaxf(m[h], mo);
      const float a = m[h] == -INFINITY ? 0.f : exp2f(m[h] - mn);
      const float b = mo == -INFINITY ? 0.f : exp2f(mo - mn);
      l[h] = l[h] * a + lo * b;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] = o[h][i] * a + __shfl_xor(o[h][i], off, 64) * b;
      m[h] = mn;
    }
  }
  __shared__ float sml[NM][G][2];
  __shared__ float so[NM][G][D];
  if (!SHFL || ts == 0) {
    if (dl == 0) {
#pragma unroll
      for (int h = 0; h < G; ++h) {
        sml[slotm][h][0] = m[h];
        sml[slotm][h][1] = l[h];
      }
    }
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i) so[slotm][h][8 * dl + i] = o[h][i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * D; e += NT) {
    const int h = e / D, d = e - h * D;
    float M = -INFINITY;
#pragma unroll
    for (int s2 = 0; s2 < NM; ++s2) M = fmaxf(M, sml[s2][h][0]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int s2 = 0; s2 < NM; ++s2) {
        const float ms = sml[s2][h][0];
        if (ms == -INFINITY) continue;
        const float f = exp2f(ms - M);
        L += sml[s2][h][1] * f;
        O += so[s2][h][d] * f;
      }
    }
    const int qh = kh * G + h;
    if (n_split == 1) {
      out[(size_t)t * ldo + (size_t)qh * D + d] = (act_t)(L > 0.f ? O / L : 0.f);
    } else {
      const size_t pi = ((size_t)t * Hq + qh) * n_split + split;
      part_o[pi * D + d] = O;
      if (d == 0) {
        part_ml[2 * pi] = M;
        part_ml[2 * pi + 1] = L;
      }
    }
  }
  if (n_split == 1 || !cnt) return;
  // Fused combine. Splits past the context returned before reaching here (ctx == 0 rows: all run),
  // so the active count is known; the last one to arrive merges them (Guideline 16 ticket).
  const int na = ctx > 0 ? min(n_split, (ctx + chunk - 1) / chunk) : n_split;
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* c = cnt + (size_t)t * Hkv + kh;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == na - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  for (int e = threadIdx.x; e < G * D; e += NT) {
    const int h = e / D, d = e - h * D;
    const int qh = kh * G + h;
    const size_t pb = ((size_t)t * Hq + qh) * n_split;
    float M = -INFINITY;
#pragma unroll 8
    for (int s2 = 0; s2 < na; ++s2) M = fmaxf(M, part_ml[2 * (pb + s2)]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll 8
      for (int s2 = 0; s2 < na; ++s2) {
        const float ms = part_ml[2 * (pb + s2)];
        if (ms == -INFINITY) continue;
        const float f = exp2f(ms - M);
        L += part_ml[2 * (pb + s2) + 1] * f;
        O += part_o[(pb + s2) * D + d] * f;
      }
    }
    out[(size_t)t * ldo + (size_t)qh * D + d] = (act_t)(L > 0.f ? O / L : 0.f);
  }
}

template <int D>
__global__ void attn_combine_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                    const int* __restrict__ ctx_len, int Hq, int n_split, int chunk, int bs,
                                    act_t* __restrict__ out, long ldo, int short_min = 64) {
  const int t = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  const int ctx = ctx_len[t];
  chunk = split_chunk(chunk, ctx, n_split, bs, short_min);
  const int na = min(n_split, (ctx + chunk - 1) / chunk);   // active splits (others never wrote)
  const size_t pb = ((size_t)t * Hq + h) * n_split;
  float M = -INFINITY;
  for (int s = 0; s < na; ++s) M = fmaxf(M, part_ml[2 * (pb + s)]);
  float L = 0.f, O = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < na; ++s) {
      const float ms = part_ml[2 * (pb + s)];
      if (ms == -INFINITY) continue;
      const float f = exp2f(ms - M);
      L += part_ml[2 * (pb + s) + 1] * f;
      O += part_o[(pb + s) * D + d] * f;
    }
  }
  out[(size_t)t * ldo + (size_t)h * D + d] = (act_t)(L > 0.f ? O / L : 0.f);
}

// ---------------------------------------------------------------------------------------------------
// Decode attention on MFMA (large grids: batch x kv heads >= 1K workgroups). The VALU kernel above
// spends ~170 vector instructions per 4 keys of a wave (dot products, cross-lane sums, the online
// softmax and 32 FMAs of P.V per lane): at batch 512 it runs at ~3.5 TB/s of K/V, bound by issue, not
// HBM (tools/attn_layout_probe.py: time linear in the context at every length). Here the G query heads
// of a kv head are the 16 COLUMNS of the MFMA tiles (G <= 16, the rest zero), so per 32 keys a wave
// issues 16 v_mfma_f32_16x16x32_bf16 and softmaxes 8 values per lane:
//   S^T = K Q^T   A = K rows straight from HBM into registers (lane (g, r): key r, dims 8g..8g+7 of
//                 each 32-dim k-step), B = Q^T (lane column r = head r, loaded once)
//   O^T += V^T P^T  A = V^T through LDS: the 32-key V tile is stored row-major with a 16-byte chunk XOR
//                 swizzle and read back transposed by ds_read_b64_tr_b16 (cdna_hip_programming.md T10);
//                 B = P^T straight from the S^T accumulators (lane (g, r) holds keys 4g..4g+3 of each
//                 16-key n-tile for head r: the MFMA's k order is free, so V^T's transposed reads take
//                 rows {4g..4g+3} and {16+4g..16+4g+3} to match)
// The O^T accumulators keep head r in lane column r -- exactly where the softmax state of head r lives,
// so the rescale needs no cross-lane traffic. One wave per workgroup; the next 32 keys' K/V loads are
// in flight while the current ones are computed. Splits and the fused combine as the VALU kernel.
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Merge of the na (<= 64) flash-decoding partials of (token t, kv head kh), run by the last split to
// finish, with every thread busy and no per-split round trip in series: one wave per head reduces the
// splits' (m, l) across its lanes into per-split weights f_s = 2^(m_s - M) / L (LDS), then each thread
// sums f_s * O_s for 4 dims of a head over a share of the splits (16-byte loads, all independent) and
// the shares are added through LDS. smem: >= 16 * 64 + 64 * WAVES * 4 floats.
template <int WAVES, int D>
DEVI void merge_splits(const float* __restrict__ part_o, const float* __restrict__ part_ml, int t, int kh, int G,
                       int Hq, int n_split, int na, act_t* __restrict__ out, long ldo, float* smem) {
  constexpr int NT = 64 * WAVES;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* f = smem;                                   // [16 heads][64 splits]
  f32x4* red = reinterpret_cast<f32x4*>(smem + 16 * 64);   // [NT] partial sums
  for (int h = wave; h < G; h += WAVES) {
    const size_t pb = ((size_t)t * Hq + kh * G + h) * n_split;
    const float ms = lane < na ? part_ml[2 * (pb + lane)] : -INFINITY;
    const float ls = lane < na ? part_ml[2 * (pb + lane) + 1] : 0.f;
    float M = ms;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    const float w = ms == -INFINITY ? 0.f : exp2f(ms - M);
    float L = w * ls;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) L += __shfl_xor(L, o, 64);
    f[h * 64 + lane] = L > 0.f ? w / L : 0.f;
  }
  __syncthreads();
  const int items = G * (D / 4);                     // (head, 4 dims)
  const int parts = items >= NT ? 1 : NT / items;    // split shares per item
  for (int i0 = 0; i0 < items; i0 += NT) {
    const int it = i0 + threadIdx.x % min(items, NT), pt = threadIdx.x / min(items, NT);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (it < items && pt < parts) {
      const int h = it / (D / 4), d4 = it % (D / 4);
      const size_t pb = ((size_t)t * Hq + kh * G + h) * n_split;
      const float* fw = f + h * 64;
#pragma unroll 4
      for (int s2 = pt; s2 < na; s2 += parts)
        acc += fw[s2] * *reinterpret_cast<const f32x4*>(part_o + (pb + s2) * D + 4 * d4);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (pt == 0 && it < items) {
      for (int p2 = 1; p2 < parts; ++p2) acc += red[threadIdx.x + p2 * min(items, NT)];
      const int h = it / (D / 4), d4 = it % (D / 4);
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<h4*>(out + (size_t)t * ldo + (size_t)(kh * G + h) * D + 4 * d4) =
          h4{(_Float16)acc[0], (_Float16)acc[1], (_Float16)acc[2], (_Float16)acc[3]};
    }
    __syncthreads();
  }
}


// D: head dimension, 128 (Llama / Mistral / Qwen2) or 64 (Granite-3.0): V rows of 2D bytes (D / 8 16-byte chunks, XOR
// swizzled within the row), 32 / 64 lanes per V row on the loads
template <typename KV, int WAVES, int D>
__global__ __launch_bounds__(64 * WAVES) void attn_decode_mfma_kernel(
    const __bf16* __restrict__ q, long ldq, const KV* __restrict__ kc, const KV* __restrict__ vc,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ tok_seq,
    const int* __restrict__ ctx_len, int Hkv, int G, int bs, float scale, int chunk, int n_split,
    act_t* __restrict__ out, long ldo, float* __restrict__ part_o, float* __restrict__ part_ml,
    int* __restrict__ cnt) {
  static_assert(D == 128 || D == 64, "head dimension");
  constexpr int NKK = D / 32, NDT = D / 16, KG = 32;
  constexpr int NCH = D / 8, LPR = NCH, RPI = 64 / LPR, NVL = KG / RPI;   // V: chunks per row, lanes per row,
                                                                          // rows per load, loads per 32 keys
  typedef KVRaw<KV> R;
  // per wave: one 32-key V tile (8 KiB; a wave's LDS ops run in order, so the next group's V is written
  // after this group's transposed reads without a second buffer); the space is reused for the cross-wave
  // merge and the split merge at the end
  constexpr int VB = WAVES * KG * D * 2, MB = WAVES > 1 ? (2 * WAVES * 16 + WAVES * 16 * D) * 4 : 0,
                CB = (16 * 64 + 64 * WAVES * 4) * 4;
  constexpr int SMEM = VB > MB ? (VB > CB ? VB : CB) : (MB > CB ? MB : CB);
  __shared__ __attribute__((aligned(16))) uint8_t Vsm[SMEM];
  const int t = blockIdx.x, kh = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const int wave = WAVES == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* Vs = Vsm + wave * KG * D * 2;
  const int Hq = Hkv * G;
  const int ctx = ctx_len[t];
  // short contexts: at least one 32-key group per wave of the workgroup per split (>= 64 keys)
  chunk = split_chunk(chunk, ctx, n_split, bs, KG * WAVES > 64 ? KG * WAVES : 64);
  const int start = split * chunk;
  if (n_split > 1 && start >= ctx && ctx > 0) return;       // inactive split: combine skips it
  const int end = min(ctx, start + chunk);
  // active splits: with ONE (short context) the split writes the output itself -- no partials, no ticket
  const int na = ctx > 0 ? min(n_split, (ctx + chunk - 1) / chunk) : n_split;
  const bool direct = n_split == 1 || (na == 1 && cnt);
  const int* bt = block_tables + (size_t)tok_seq[t] * bt_stride;
  const float sl2 = scale * LOG2E;

  bf16x8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    qf[kk] = bf16x8{};
    if (r < G) qf[kk] = *reinterpret_cast<const bf16x8*>(q + (size_t)t * ldq + (size_t)(kh * G + r) * D + kk * 32 + 8 * g);
  }
  f32x4 o[NDT];
#pragma unroll
  for (int c = 0; c < NDT; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  // Block-table entries come from a register window (lane i holds entry b0 + 64 * win + i, refreshed once
  // per 64 blocks), broadcast per 32-key group as wave-uniform values: the K/V loads of a group no
  // longer wait on a dependent block-table fetch (the chain that bound long contexts at small batch).
  // A group [base, base + 32) touches blocks base / bs .. (base + 31) / bs: at most NGB of them.
  constexpr int NGB = 4;                       // bs >= 16 (host-checked): <= 3 blocks per group
  const int b0 = start / bs;
  int btw = -1, btreg = 0;
  int gblk[NGB] = {0, 0, 0, 0};
  auto group_blocks = [&](int base) __attribute__((always_inline)) {
    const int bi0 = base / bs - b0;
    const int nbg = (min(base + KG, end) - 1) / bs - base / bs + 1;     // blocks this group touches
    const int win = bi0 >> 6;
    if (win != btw) {
      btw = win;
      const int e = b0 + win * 64 + lane;
      btreg = e * bs < end ? bt[e] : 0;
    }
#pragma unroll
    for (int i = 0; i < NGB; ++i) {
      const int bi = bi0 + i;
      // (a block past the register window: one wave-uniform direct read)
      if (i < nbg) gblk[i] = (bi >> 6) == win ? __builtin_amdgcn_readlane(btreg, bi & 63) : bt[b0 + bi];
    }
  };
  auto kv_row = [&](int p, int base) -> size_t {       // element offset of key p's row for this kv head
    const int pc = min(p, end - 1);
    const int lb = pc / bs - base / bs;                // 0 .. NGB - 1
    const int blk = lb == 0 ? gblk[0] : (lb == 1 ? gblk[1] : (lb == 2 ? gblk[2] : gblk[3]));
    return ((size_t)((long)blk * bs + pc % bs) * Hkv + kh) * D;
  };
  // swizzled byte offset of 16-byte chunk ch of V row `row` (2D-byte rows): D = 128 conflict-free for the
  // transposed reads and the row writes (cdna_hip_programming.md T10, layout (b)); D = 64: chunk ^ (row & 7)
  auto voff = [](int row, int ch) {
    if constexpr (D == 128) return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
    else return row * (2 * D) + 16 * (ch ^ (row & (NCH - 1)));
  };
  // K of 32 keys: [n-tile][k-step]; V of 32 keys: NVL rows per lane (row = RPI i + lane / LPR, chunk lane % LPR)
  typename R::raw kr[2][NKK], vr[NVL];
  auto load = [&](int base, typename R::raw (&K)[2][NKK], typename R::raw (&V)[NVL]) __attribute__((always_inline)) {
    group_blocks(base);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const size_t o0 = kv_row(base + 16 * nt + r, base);
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) K[nt][kk] = R::ld(kc + o0 + kk * 32 + 8 * g);
    }
#pragma unroll
    for (int i = 0; i < NVL; ++i) V[i] = R::ld(vc + kv_row(base + RPI * i + lane / LPR, base) + 8 * (lane % LPR));
  };
  auto store_v = [&](int buf, typename R::raw (&V)[NVL]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NVL; ++i)
      *reinterpret_cast<u32x4*>(Vs + voff(RPI * i + lane / LPR, lane % LPR)) = R::bf16(V[i]);
  };
  // wave w takes the 32-key groups w, w + WAVES, ... of the workgroup's range
  const int ngrp_all = end > start ? (end - start + KG - 1) / KG : 0;
  const int ngrp = ngrp_all > wave ? (ngrp_all - wave + WAVES - 1) / WAVES : 0;
  if (ngrp > 0) {
    load(start + wave * KG, kr, vr);
    store_v(0, vr);
  }
  for (int j = 0; j < ngrp; ++j) {
    const int base = start + (j * WAVES + wave) * KG;
    typename R::raw kn[2][NKK], vn[NVL];
    const bool more = j + 1 < ngrp;
    if (more) load(base + WAVES * KG, kn, vn);
    // ---- S^T = K Q^T: s[nt][i] = S[head r][key base + 16 nt + 4 g + i]
    f32x4 s[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
        s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, R::bf16(kr[nt][kk])), qf[kk],
                                                        s[nt], 0, 0, 0);
    }
    // ---- online softmax of head r (base 2), keys past `end` masked
    float mx = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = base + 16 * nt + 4 * g + i < end ? s[nt][i] * sl2 : -INFINITY;
        s[nt][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = m == -INFINITY ? 0.f : exp2f(m - mn);
    float ps = 0.f;
    bf16x8 pb;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = s[nt][i] == -INFINITY ? 0.f : exp2f(s[nt][i] - mn);
        ps += pv;
        pb[4 * nt + i] = (__bf16)pv;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = mn;
    // ---- O^T = O^T * alpha + V^T P^T over the 32 keys; V^T fragment of dim tile c: transposed reads of
    // rows {4g+q} and {16+4g+q}, columns 16c + 4p .. +3 (lane 4q + p of the group supplies the address)
    const uint8_t* vb = Vs;
    const int qq = r >> 2, pp = r & 3;
#pragma unroll
    for (int c = 0; c < NDT; ++c) {
      const int ch = 2 * c + (pp >> 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(vb + voff(4 * g + qq, ch) + 8 * (pp & 1)));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(vb + voff(16 + 4 * g + qq, ch) + 8 * (pp & 1)));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 a8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a8), pb, o[c] * alpha, 0, 0, 0);
    }
    if (more) {
      store_v((j + 1) & 1, vn);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) kr[nt][kk] = kn[nt][kk];
    }
  }

  // ---- output. WAVES > 1: merge the waves' partial (m, l, O) of each head through LDS (the V tiles'
  // space), every thread finishing (head, dim) elements; WAVES == 1: lane (g, r) holds dims 16c + 4g + i of
  // head r in registers
  if constexpr (WAVES > 1) {
    float* mb = reinterpret_cast<float*>(Vsm);                      // [WAVES][16] m, [WAVES][16] l
    float* ob = mb + 2 * WAVES * 16;                                  // [WAVES][16 heads][D]
    __syncthreads();                                                  // every wave is done with its V tiles
    if (g == 0) {
      mb[wave * 16 + r] = m;
      mb[(WAVES + wave) * 16 + r] = l;
    }
#pragma unroll
    for (int c = 0; c < NDT; ++c)
      *reinterpret_cast<f32x4*>(ob + ((size_t)wave * 16 + r) * D + 16 * c + 4 * g) = o[c];
    __syncthreads();
    for (int e = threadIdx.x; e < G * D; e += 64 * WAVES) {
      const int h = e / D, d = e - h * D;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) M = fmaxf(M, mb[w * 16 + h]);
      float L = 0.f, O = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) {
        const float mw = mb[w * 16 + h];
        const float f = mw == -INFINITY ? 0.f : exp2f(mw - M);
        L += mb[(WAVES + w) * 16 + h] * f;
        O += ob[((size_t)w * 16 + h) * D + d] * f;
      }
      const int qh2 = kh * G + h;
      if (direct) {
        out[(size_t)t * ldo + (size_t)qh2 * D + d] = (act_t)(L > 0.f ? O / L : 0.f);
      } else {
        const size_t pi = ((size_t)t * Hq + qh2) * n_split + split;
        part_o[pi * D + d] = O;
        if (d == 0) {
          part_ml[2 * pi] = M;
          part_ml[2 * pi + 1] = L;
        }
      }
    }
    if (direct) return;
  } else {
    const int qh = kh * G + r;
    if (direct) {
      if (r < G) {
        const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
        for (int c = 0; c < NDT; ++c) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<h4*>(out + (size_t)t * ldo + (size_t)qh * D + 16 * c + 4 * g) =
              h4{(_Float16)(o[c][0] * inv), (_Float16)(o[c][1] * inv), (_Float16)(o[c][2] * inv),
                 (_Float16)(o[c][3] * inv)};
        }
      }
      return;
    }
    if (r < G) {
      const size_t pi = ((size_t)t * Hq + qh) * n_split + split;
#pragma unroll
      for (int c = 0; c < NDT; ++c) *reinterpret_cast<f32x4*>(part_o + pi * D + 16 * c + 4 * g) = o[c];
      if (g == 0) {
        part_ml[2 * pi] = m;
        part_ml[2 * pi + 1] = l;
      }
    }
  }
  if (!cnt) return;
  // fused combine: the last active split of (token, kv head) to arrive merges them (as the VALU kernel)
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cp = cnt + (size_t)t * Hkv + kh;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == na - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(cp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  merge_splits<WAVES, D>(part_o, part_ml, t, kh, G, Hq, n_split, na, out, ldo,
                      reinterpret_cast<float*>(Vsm));
}

template <int D, int G>
void launch_attn(dim3 grid, hipStream_t st, const __bf16* q, long ldq, const void* kc, const void* vc,
                 const int* bt, int bts, const int* ts, const int* cl, int Hkv, int bs, float scale, int chunk,
                 int ns, act_t* out, long ldo, float* po, float* pml, int* cnt, bool kv8, int waves) {
#define NLS_ATTN_L(KVT, W)                                                                                      \
  hipLaunchKernelGGL((attn_decode_kernel<D, G, KVT, W>), grid, dim3(64 * W), 0, st, q, ldq, (const KVT*)kc,      \
                     (const KVT*)vc, bt, bts, ts, cl, Hkv, bs, scale, chunk, ns, out, ldo, po, pml, cnt)
  if (kv8) {
    if (waves == 8) NLS_ATTN_L(uint8_t, 8); else NLS_ATTN_L(uint8_t, 4);
  } else {
    if (waves == 8) NLS_ATTN_L(__bf16, 8); else NLS_ATTN_L(__bf16, 4);
  }
#undef NLS_ATTN_L
}

}  // namespace

namespace {

// workspace: part_o [T*Hq*n_split*D] f32, part_ml [T*Hq*n_split*2] f32 (only if n_split > 1);
// cnt: int32 [T*Hkv], zero (re-armed by every launch): the splits merge in-kernel; null: attn_combine
static int attn_decode_impl(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                            int bt_stride, const int* tok_seq, const int* ctx_len, int T, int Hq, int Hkv, int D,
                            int block_size, float scale, int chunk, int n_split, void* out, long ldo, float* part_o,
                            float* part_ml, int* cnt, void* stream, bool kv8) {
  if (Hq % Hkv || n_split < 1 || (chunk > 0 && chunk % block_size) || 64 % (64 / (D / 8)) ||
      (4 * 64 / (D / 8)) > 64 * block_size)
    return -1;
  const int G = Hq / Hkv;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(T, Hkv, n_split);
  // D = 128 / 64: the MFMA kernel -- one wave per workgroup once the grid fills the chip (>= 1K workgroups),
  // else four waves splitting the workgroup's keys (more K/V in flight per (token, kv head, split): long
  // contexts at small batch). NLS_ATTN_MFMA=0 keeps the VALU kernel.
  static const int mf = [] { const char* e = getenv("NLS_ATTN_MFMA"); return e ? atoi(e) : -1; }();
  if ((D == 128 || D == 64) && G <= 16 && mf != 0 && block_size >= 16 && n_split <= 64) {
    // NLS_ATTN_MFMA_BIG: workgroups from which the one-wave form is taken (default 1024; A/B knob)
    static const long big_at = [] { const char* e = getenv("NLS_ATTN_MFMA_BIG"); return e ? atol(e) : 1024L; }();
    const bool big = (long)T * Hkv * n_split >= big_at;
    // grids of <= 256 workgroups: 8 waves each (one workgroup per CU: 192 VGPRs), so a 256-key context is one
    // pass; up to 1K workgroups: 4 waves (two per CU). NLS_ATTN_MFMA_WAVES=4|8 forces one. The split policy
    // (models/llama.py attn_splits) aims at 256 workgroups at small batch.
    static const int mwf = [] { const char* e = getenv("NLS_ATTN_MFMA_WAVES"); return e ? atoi(e) : 0; }();
    const int mw = mwf == 4 || mwf == 8 ? mwf : ((long)T * Hkv * n_split <= 256 ? 8 : 4);
#define NLS_ATTN_M(KVT, W, DD)                                                                                 \
  hipLaunchKernelGGL((attn_decode_mfma_kernel<KVT, W, DD>), grid, dim3(64 * W), 0, st, (const __bf16*)q, ldq,   \
                     (const KVT*)kc, (const KVT*)vc, block_tables, bt_stride, tok_seq, ctx_len, Hkv, G, block_size, \
                     scale, chunk, n_split, (act_t*)out, ldo, part_o, part_ml, cnt)
#define NLS_ATTN_MD(DD)                                                                                         \
    if (kv8) {                                                                                                  \
      if (big) NLS_ATTN_M(uint8_t, 1, DD); else if (mw == 4) NLS_ATTN_M(uint8_t, 4, DD); else NLS_ATTN_M(uint8_t, 8, DD); \
    } else {                                                                                                    \
      if (big) NLS_ATTN_M(__bf16, 1, DD); else if (mw == 4) NLS_ATTN_M(__bf16, 4, DD); else NLS_ATTN_M(__bf16, 8, DD);   \
    }
    if (D == 128) { NLS_ATTN_MD(128) } else { NLS_ATTN_MD(64) }
#undef NLS_ATTN_MD
#undef NLS_ATTN_M
    if (n_split > 1 && !cnt) {    // (the short-context split size of the launched variant)
      if (D == 128)
        hipLaunchKernelGGL(attn_combine_kernel<128>, dim3(T, Hq), dim3(128), 0, st, part_o, part_ml, ctx_len, Hq,
                           n_split, chunk, block_size, (act_t*)out, ldo, big ? 64 : 32 * mw);
      else
        hipLaunchKernelGGL(attn_combine_kernel<64>, dim3(T, Hq), dim3(64), 0, st, part_o, part_ml, ctx_len, Hq,
                           n_split, chunk, block_size, (act_t*)out, ldo, big ? 64 : 32 * mw);
    }
    return (int)hipGetLastError();
  }
  // waves per workgroup: 8 (twice the keys in flight per step) while the grid is small -- batch 1 / 16 at
  // 4K context 2.93 -> 2.68 / 5.19 -> 4.76 ms/step, batch 1 at 128 2.24 -> 2.17 -- and 4 once the grid
  // fills the chip (batch 512: 12.97 vs 13.74), profiles/attn_waves_ab.txt. NLS_ATTN_WAVES=4|8 forces.
  static const int forced = [] { const char* e = getenv("NLS_ATTN_WAVES"); return e ? atoi(e) : 0; }();
  const int waves = forced == 4 || forced == 8 ? forced : ((long)T * Hkv * n_split < 1024 ? 8 : 4);
  const __bf16* qq = (const __bf16*)q;
  act_t* o = (act_t*)out;
#define NLS_ATTN_CASE(DD, GG)                                                                                 \
  if (D == DD && G == GG) {                                                                                  \
    launch_attn<DD, GG>(grid, st, qq, ldq, kc, vc, block_tables, bt_stride, tok_seq, ctx_len, Hkv, block_size, \
                        scale, chunk, n_split, o, ldo, part_o, part_ml, cnt, kv8, waves);                         \
  } else
  // G = Hq/Hkv of the supported families: 1 (MHA), 2/4/8 (Llama/Mixtral), 3/5/6/7 (Qwen2 sizes, e.g. 28/4)
  NLS_ATTN_CASE(128, 1) NLS_ATTN_CASE(128, 2) NLS_ATTN_CASE(128, 3) NLS_ATTN_CASE(128, 4) NLS_ATTN_CASE(128, 5)
  NLS_ATTN_CASE(128, 6) NLS_ATTN_CASE(128, 7) NLS_ATTN_CASE(128, 8)
  NLS_ATTN_CASE(64, 1) NLS_ATTN_CASE(64, 2) NLS_ATTN_CASE(64, 3) NLS_ATTN_CASE(64, 4) NLS_ATTN_CASE(64, 5)
  NLS_ATTN_CASE(64, 6) NLS_ATTN_CASE(64, 7) NLS_ATTN_CASE(64, 8) { return -1; }
#undef NLS_ATTN_CASE
  if (n_split > 1 && !cnt) {
    if (D == 128)
      hipLaunchKernelGGL(attn_combine_kernel<128>, dim3(T, Hq), dim3(128), 0, st, part_o, part_ml, ctx_len, Hq,
                         n_split, chunk, block_size, o, ldo);
    else
      hipLaunchKernelGGL(attn_combine_kernel<64>, dim3(T, Hq), dim3(64), 0, st, part_o, part_ml, ctx_len, Hq,
                         n_split, chunk, block_size, o, ldo);
  }
  return (int)hipGetLastError();
}

}  // namespace (host)

extern "C" {

int nls_attn_decode(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                    int bt_stride, const int* tok_seq, const int* ctx_len, int T, int Hq, int Hkv, int D,
                    int block_size, float scale, int chunk, int n_split, void* out, long ldo, float* part_o,
                    float* part_ml, int* cnt, void* stream) {
  return attn_decode_impl(q, ldq, kc, vc, block_tables, bt_stride, tok_seq, ctx_len, T, Hq, Hkv, D, block_size, scale,
                          chunk, n_split, out, ldo, part_o, part_ml, cnt, stream, false);
}

// the same over an fp8 (OCP e4m3) K/V cache
int nls_attn_decode8(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                     int bt_stride, const int* tok_seq, const int* ctx_len, int T, int Hq, int Hkv, int D,
                     int block_size, float scale, int chunk, int n_split, void* out, long ldo, float* part_o,
                     float* part_ml, int* cnt, void* stream) {
  return attn_decode_impl(q, ldq, kc, vc, block_tables, bt_stride, tok_seq, ctx_len, T, Hq, Hkv, D, block_size, scale,
                          chunk, n_split, out, ldo, part_o, part_ml, cnt, stream, true);
}

}  // extern "C"
