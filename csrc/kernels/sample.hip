// Batched token sampling on the GPU: repetition / presence / frequency penalties,
// temperature, top-k, min-p, top-p and the final draw -- one workgroup per row, one launch
// for every sampled request of a step (SURVEY.md §2F sample_topk_topp).
//
// No sort over the vocabulary: top-k and top-p become VALUE thresholds found by two histogram
// passes over block-wide counts / masses (k-th largest logit; the logit above which the kept
// probability mass reaches top_p), and the draw is an inverse-CDF walk in INDEX order over
// the kept tokens (same distribution as sampling in sorted order). The uniform variate comes
// from the host (per-request seeded generator), so seeded requests stay reproducible.
#include "common.h"

namespace {

struct SampleParams {
  float temperature, top_p, min_p, repeat_penalty, presence_penalty, frequency_penalty, u;
  int top_k, n_hist, pad;
};

constexpr int NT = 1024;

DEVI float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

DEVI float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

// Keep-threshold by two histogram passes (instead of ~32 bisection scans of the vocabulary): bins
// over [a, b] (bin 0 = highest logits) accumulate the weight w of each kept logit (count: 1; mass:
// exp((l - mx) * it)); the bin where the running weight from the top reaches `target` is refined by a
// second histogram over that bin alone. Returns t: keeping l >= t reaches `target` (sub-bin ties are
// kept, resolution (b - a) / NB^2).
constexpr int NB = 1024;
DEVI float hist_threshold(const float* __restrict__ l, int V, float a, float b, float keep_lo, bool count, float mx,
                          float it, float target, float* hbin, float* red) {
  float above = 0.f;                    // weight strictly above the current search range
  for (int pass = 0; pass < 2; ++pass) {
    if (!(b > a)) break;
    for (int i = threadIdx.x; i < NB; i += NT) hbin[i] = 0.f;
    __syncthreads();
    const float scale = (float)NB / (b - a);
    for (int i = threadIdx.x; i < V; i += NT) {
      const float v = l[i];
      if (v >= a && v <= b && v >= keep_lo && v > -INFINITY) {     // NaN / -inf never binned
        const int bin = min(NB - 1, (int)((b - v) * scale));
        atomicAdd(&hbin[bin], count ? 1.f : __expf((v - mx) * it));
      }
    }
    __syncthreads();
    // running weight from the top: one wave scans the bins, 16 per lane
    __shared__ int s_bin;
    __shared__ float s_before;
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      float mine = 0.f;
#pragma unroll
      for (int j = 0; j < NB / 64; ++j) mine += hbin[lane * (NB / 64) + j];
      float incl = mine;                              // inclusive prefix over lanes
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
      }
      const float excl = incl - mine;
      const bool cross = above + incl >= target && above + excl < target;
      const unsigned long long m = __ballot(cross);
      const int owner = m ? __ffsll((long long)m) - 1 : 63;
      if (lane == owner) {
        float acc = above + excl;
        int bin = lane * (NB / 64) + NB / 64 - 1;
        for (int j = 0; j < NB / 64; ++j) {
          const float w = hbin[lane * (NB / 64) + j];
          if (acc + w >= target) { bin = lane * (NB / 64) + j; break; }
          acc += w;
        }
        s_bin = bin;
        s_before = acc;
      }
    }
    __syncthreads();
    const int bin = s_bin;
    above = s_before;
    const float nb = b - (float)bin / scale, na = b - (float)(bin + 1) / scale;
    b = nb;
    a = na;
    __syncthreads();
  }
  return a;
}

// Max and sum exp((l - max) * it) of a row in ONE pass (online rescaling), non-finite entries skipped.
DEVI void block_max_z(const float* __restrict__ l, int V, float it, float& mx, float& z, float* red) {
  float m = -INFINITY, s = 0.f;
#pragma unroll 8
  for (int i = threadIdx.x; i < V; i += NT) {
    const float v = l[i];
    if (!(v > -INFINITY)) continue;                  // -inf and NaN
    if (v > m) {
      s = s * __expf((m - v) * it) + 1.f;
      m = v;
    } else {
      s += __expf((v - m) * it);
    }
  }
  mx = block_max(m, red);
  z = block_sum(m > -INFINITY ? s * __expf((m - mx) * it) : 0.f, red);
}

// The draw: inverse CDF in index order over the kept logits (l >= lo), u in [0, 1). Weights are summed
// per 64-token tile (a wave per tile, coalesced), the tile sums are scanned block-wide, and one wave scans
// the tile that holds the target -- no serial walk over chunks or tokens. Returns the token in every thread.
constexpr int MAXT = 4096;                            // 64-token tiles: V <= 262144
DEVI int draw_index_order(const float* __restrict__ l, int V, float lo, float mx, float it, float u, float* tile,
                          float* red, int* s_tok) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = (V + 63) >> 6;
#pragma unroll 4
  for (int t = w; t < nt; t += NT / 64) {
    const int i = (t << 6) + lane;
    float x = 0.f;
    if (i < V) {
      const float v = l[i];
      if (v >= lo && v > -INFINITY) x = __expf((v - mx) * it);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) tile[t] = x;
  }
  __shared__ int s_tile;
  __shared__ float s_before;
  if (threadIdx.x == 0) s_tile = -1;
  __syncthreads();
  // exclusive scan of per-thread tile runs [per * tid, per * tid + per)
  const int per = (nt + NT - 1) / NT;
  const int t0 = threadIdx.x * per;
  float loc = 0.f;
  for (int j = 0; j < per; ++j)
    if (t0 + j < nt) loc += tile[t0 + j];
  float incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) red[w] = incl;
  __syncthreads();
  float off = 0.f, Z = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const float r = red[i];
    off += i < w ? r : 0.f;
    Z += r;
  }
  const float target = u * Z;
  const float excl = off + incl - loc;
  if (loc > 0.f && excl <= target && target < excl + loc) {
    float acc = excl;
    for (int j = 0; j < per && t0 + j < nt; ++j) {
      const float x = tile[t0 + j];
      if (x > 0.f && acc + x > target) {
        s_tile = t0 + j;
        s_before = acc;
        break;
      }
      acc += x;
    }
  }
  __syncthreads();
  int t = s_tile;
  float before = s_before;
  bool last = false;
  if (t < 0) {                                        // rounding at the very end: the last kept token
    int mine = -1;
    for (int j = per - 1; j >= 0; --j)
      if (t0 + j < nt && tile[t0 + j] > 0.f) { mine = t0 + j; break; }
    t = (int)block_max((float)mine, red);             // exact for tile ids < 2^24
    last = true;
  }
  if (w == 0) {
    int tok = -1;
    if (t >= 0) {
      const int i = (t << 6) + lane;
      float x = 0.f;
      if (i < V) {
        const float v = l[i];
        if (v >= lo && v > -INFINITY) x = __expf((v - mx) * it);
      }
      const unsigned long long kept = __ballot(x > 0.f);
      if (!last) {
        float c = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float y = __shfl_up(c, o, 64);
          if (lane >= o) c += y;
        }
        const unsigned long long hit = __ballot(x > 0.f && before + c > target);
        if (hit) tok = (t << 6) + __ffsll((long long)hit) - 1;
      }
      if (tok < 0 && kept) tok = (t << 6) + 63 - __clzll((long long)kept);
    }
    if (lane == 0) *s_tok = tok < 0 ? 0 : tok;       // nothing kept: a non-finite row -> a valid id anyway
  }
  __syncthreads();
  return *s_tok;
}

// ---- top-k fast path (0 < top_k <= KFAST, the usual chat payload: top_k 40): after the top-k threshold
// (two histogram passes) every kept logit is compacted into LDS in ONE more pass, and min-p, top-p and the
// draw run on those <= CCAP entries -- 4 passes over the vocabulary instead of 8. The k-th largest value is
// taken exactly from the sorted candidates (the binned threshold keeps its sub-bin ties), so the kept set,
// the top-p cut and the index-order draw are those of the CPU twin (engine/sampling.py sample_rows).
constexpr int KFAST = 256;
constexpr int CCAP = 512;

// block bitonic sort of CCAP (key, idx) pairs in LDS: by value, descending (ties: lower index first), or by
// index, ascending. Padding entries carry (-inf, INT_MAX) and end up last either way.
DEVI void bitonic_pairs(float* key, int* idx, bool byval) {
  for (int k = 2; k <= CCAP; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < CCAP; i += NT) {
        const int l = i ^ j;
        if (l > i) {
          const float ka = key[i], kb = key[l];
          const int ia = idx[i], ib = idx[l];
          const bool a_first = byval ? (ka > kb || (ka == kb && ia < ib)) : ia < ib;
          if (((i & k) == 0) != a_first) {
            key[i] = kb;
            key[l] = ka;
            idx[i] = ib;
            idx[l] = ia;
          }
        }
      }
    }
  __syncthreads();
}

// inclusive block scan of one value per thread (NT threads)
DEVI float block_incl_scan(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  __syncthreads();
  if (lane == 63) red[w] = incl;
  __syncthreads();
  float off = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) off += i < w ? red[i] : 0.f;
  return off + incl;
}

// Returns the token (every thread), or -1 (every thread) when the compacted set overflows CCAP (a row with
// massive ties at the threshold): the caller then takes the general path.
DEVI int sample_topk_fast(const float* __restrict__ l, int V, const SampleParams& p, float u, float mx, float mn,
                          float it, float* red, float* sk, int* sidx, float* hbin) {
  __shared__ int s_n, s_pick, s_last;
  __shared__ float s_tot, s_thr, s_z;
  const float t = hist_threshold(l, V, mn, mx, -INFINITY, true, mx, it, (float)p.top_k, hbin, red);
  if (threadIdx.x == 0) {
    s_n = 0;
    s_pick = 0x7FFFFFFF;
    s_last = -1;
    s_thr = 0.f;              // (no crossing found through rounding: keep the whole top-k set)
  }
  __syncthreads();
  for (int i = threadIdx.x; i < V; i += NT) {
    const float v = l[i];
    if (v >= t && v > -INFINITY) {
      const int at = atomicAdd(&s_n, 1);
      if (at < CCAP) {
        sk[at] = v;
        sidx[at] = i;
      }
    }
  }
  __syncthreads();
  const int n = s_n;
  if (n > CCAP || n < 1) return -1;
  for (int i = n + threadIdx.x; i < CCAP; i += NT) {
    sk[i] = -INFINITY;
    sidx[i] = 0x7FFFFFFF;
  }
  bitonic_pairs(sk, sidx, true);
  // exact k-th largest (ties kept), then min-p
  float lo = sk[min(p.top_k, n) - 1];
  if (p.min_p > 0.f) lo = fmaxf(lo, mx + p.temperature * __logf(p.min_p));
  const int j = threadIdx.x;
  const bool in = j < n && sk[j] >= lo;
  float w = in ? __expf((sk[j] - mx) * it) : 0.f;
  if (p.top_p < 1.f) {
    // smallest top set (by value) whose mass reaches top_p of the kept mass; ties of its last weight kept
    const float cum = block_incl_scan(w, red);
    if (j == NT - 1) s_tot = cum;
    __syncthreads();
    const float target = p.top_p * s_tot;
    if (in && cum >= target && cum - w < target) s_thr = w;
    __syncthreads();
    if (w < s_thr) w = 0.f;
  }
  // the draw: inverse CDF in INDEX order over the kept entries
  __syncthreads();
  if (j < CCAP) sk[j] = w;
  // by index (weights ride along as keys)
  for (int k = 2; k <= CCAP; k <<= 1)
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < CCAP; i += NT) {
        const int o = i ^ jj;
        if (o > i && (((i & k) == 0) != (sidx[i] < sidx[o]))) {
          const float kt = sk[i];
          sk[i] = sk[o];
          sk[o] = kt;
          const int it2 = sidx[i];
          sidx[i] = sidx[o];
          sidx[o] = it2;
        }
      }
    }
  __syncthreads();
  const float wj = j < CCAP ? sk[j] : 0.f;
  const float cdf = block_incl_scan(wj, red);
  if (j == NT - 1) s_z = cdf;
  __syncthreads();
  const float target = u * s_z;
  if (wj > 0.f && cdf > target) atomicMin(&s_pick, j);
  if (wj > 0.f) atomicMax(&s_last, j);
  __syncthreads();
  const int at = s_pick != 0x7FFFFFFF ? s_pick : s_last;
  return at >= 0 ? sidx[at] : 0;
}

// One row: penalties over the history window h[0, n_hist) (any order), then greedy / temperature /
// top-k / min-p / top-p and the draw with uniform u. The token is returned in EVERY thread.
DEVI int sample_one(float* __restrict__ l, int V, const SampleParams& p, float u, const int* __restrict__ h,
                    int n_hist, float* red, float* s_chunk, int* s_tok, float* hbin) {
  // 1) penalties on the distinct ids of the history window (llama.cpp-style semantics)
  if (n_hist > 0 && (p.repeat_penalty != 1.f || p.presence_penalty != 0.f || p.frequency_penalty != 0.f)) {
    const int j = threadIdx.x;
    if (j < n_hist) {
      const int id = h[j];
      bool first = true;
      int cnt = 0;
      for (int i = 0; i < n_hist; ++i) {
        if (h[i] == id) {
          ++cnt;
          if (i < j) first = false;
        }
      }
      if (first && id >= 0 && id < V) {
        float v = l[id];
        if (p.repeat_penalty != 1.f) v = v > 0.f ? v / p.repeat_penalty : v * p.repeat_penalty;
        v -= p.presence_penalty + p.frequency_penalty * (float)cnt;
        l[id] = v;
      }
    }
    __syncthreads();
  }
  // 2) greedy: plain arg-max (lowest index on ties)
  const bool trunc = (p.top_k > 0 && p.top_k < V) || p.min_p > 0.f;
  const float it = p.temperature > 0.f ? 1.f / p.temperature : 0.f;
  if (p.temperature > 0.f && p.top_k > 0 && p.top_k <= KFAST && p.top_k < V && s_chunk != nullptr) {
    float m = -INFINITY, mnv = INFINITY;
    for (int i = threadIdx.x; i < V; i += NT) {
      const float v = l[i];
      if (v > -INFINITY) {
        m = fmaxf(m, v);
        mnv = fminf(mnv, v);
      }
    }
    const float fmx = block_max(m, red), fmn = -block_max(-mnv, red);
    if (fmx > -INFINITY) {
      const int tok = sample_topk_fast(l, V, p, u, fmx, fmn, it, red, s_chunk,
                                       reinterpret_cast<int*>(s_chunk + CCAP), hbin);
      if (tok >= 0) return tok;
    }
  }
  float mx = -INFINITY, Z = 0.f;
  if (p.temperature > 0.f && !trunc) {
    block_max_z(l, V, it, mx, Z, red);               // max and the untruncated mass in one pass
  } else {
    for (int i = threadIdx.x; i < V; i += NT) mx = fmaxf(mx, l[i]);
    mx = block_max(mx, red);
  }
  if (p.temperature <= 0.f) {
    int best = 0x7FFFFFFF;
    for (int i = threadIdx.x; i < V; i += NT)
      if (l[i] == mx) best = min(best, i);
    float b = (float)best;   // exact for V < 2^24
    b = -block_max(-b, red);
    // no logit equals the max only when the row is all NaN: never hand an out-of-range id to the
    // next step's embedding gather (chained decode feeds next_ids straight back on the device)
    return b < (float)V ? (int)b : 0;
  }
  // 3) keep-threshold on the logit scale: top-k (k-th largest) and min-p (p >= min_p * p_max)
  float lo = -INFINITY;
  if (p.top_k > 0 && p.top_k < V) {
    // lower search bound over FINITE logits only: a masked (-inf) entry would make the bin scale 0
    // and its bin index NaN, and the threshold -inf would keep the whole vocabulary
    float mn = INFINITY;
    for (int i = threadIdx.x; i < V; i += NT) {
      const float v = l[i];
      if (v > -INFINITY) mn = fminf(mn, v);
    }
    mn = -block_max(-mn, red);
    lo = hist_threshold(l, V, mn, mx, -INFINITY, true, mx, it, (float)p.top_k, hbin, red);
  }
  if (p.min_p > 0.f) lo = fmaxf(lo, mx + p.temperature * __logf(p.min_p));
  // 4) top-p: logit threshold above which the kept mass reaches top_p of the kept total
  if (p.top_p < 1.f) {
    if (trunc) {
      Z = 0.f;
      for (int i = threadIdx.x; i < V; i += NT)
        if (l[i] >= lo) Z += __expf((l[i] - mx) * it);
      Z = block_sum(Z, red);
    }
    // tokens more than 30 temperatures below the max carry < e^-30 of the mass each: search above them
    const float a = fmaxf(lo, mx - 30.f * p.temperature);
    lo = fmaxf(lo, hist_threshold(l, V, a, mx, lo, false, mx, it, p.top_p * Z, hbin, red));
  }
  // 5) inverse CDF in index order over the kept tokens
  return draw_index_order(l, V, lo, mx, it, u, s_chunk, red, s_tok);
}

__global__ __launch_bounds__(NT) void sample_kernel(float* __restrict__ logits, long ld, int V,
                                                    const SampleParams* __restrict__ params,
                                                    const int* __restrict__ hist, int hist_stride,
                                                    int* __restrict__ out) {
  __shared__ float red[NT / 64];
  __shared__ float s_chunk[MAXT];
  __shared__ int s_tok;
  __shared__ float hbin[NB];
  const int row = blockIdx.x;
  const SampleParams p = params[row];
  const int tok = sample_one(logits + (size_t)row * ld, V, p, p.u, hist + (size_t)row * hist_stride, p.n_hist, red,
                             s_chunk, &s_tok, hbin);
  if (threadIdx.x == 0) out[row] = tok;
}

// counter-based uniform in [0, 1): splitmix64 of (seed, position) -- reproducible per seeded request
DEVI float uniform01(unsigned long long seed, int pos) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (unsigned long long)(pos + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.f / 16777216.f);
}

// In-graph sampling of a decode step: rows whose params ask for sampling replace the fused arg-max
// token in next_ids with a draw; the uniform comes from (seed, position), the penalty window is a
// per-row ring of the last HIST tokens indexed by absolute position (the host fills it when the row
// is assigned, every sampled step appends its token), so sampled rows stay on the chained
// asynchronous decode path (no host round trip, no logits copy).
__global__ __launch_bounds__(NT) void sample_decode_kernel(float* __restrict__ logits, long ld, int V,
                                                           const SampleParams* __restrict__ params,
                                                           const unsigned long long* __restrict__ seeds,
                                                           const int* __restrict__ pos, const int* __restrict__ ctx_len,
                                                           int* __restrict__ hist, int hist_stride,
                                                           int* __restrict__ next_ids) {
  __shared__ float red[NT / 64];
  __shared__ float s_chunk[MAXT];
  __shared__ int s_tok;
  __shared__ float hbin[NB];
  const int row = blockIdx.x;
  const SampleParams p = params[row];
  const bool penal = p.repeat_penalty != 1.f || p.presence_penalty != 0.f || p.frequency_penalty != 0.f;
  if (ctx_len[row] <= 0 || (p.temperature <= 0.f && !penal)) return;     // padding / greedy row
  const int ps = pos[row];
  int* h = hist + (size_t)row * hist_stride;
  const int n_hist = min(hist_stride, ps + 1);
  const int tok = sample_one(logits + (size_t)row * ld, V, p, uniform01(seeds[row], ps), h, n_hist, red, s_chunk,
                             &s_tok, hbin);
  if (threadIdx.x == 0) {
    next_ids[row] = tok;
    h[(ps + 1) % hist_stride] = tok;
  }
}

// Tensor-parallel variant: the row is the gathered candidate list of every rank (values `cand` [n, M] in
// vocabulary order, global ids `ids`, (-inf, -1) padding) instead of the full vocabulary. The history ring
// (token ids) is mapped to candidate positions first -- a history token outside the candidates cannot
// reach the kept set (the engine only takes this path when penalties can only LOWER logits and top-k fits
// the candidates: Engine._cand_ok) -- then the same sampler draws a position, whose id is the token.
constexpr int MAXC = 1024;
__global__ __launch_bounds__(NT) void sample_decode_cand_kernel(float* __restrict__ cand, long ld, int M,
                                                                const int* __restrict__ ids, long ldi,
                                                                const SampleParams* __restrict__ params,
                                                                const unsigned long long* __restrict__ seeds,
                                                                const int* __restrict__ pos,
                                                                const int* __restrict__ ctx_len,
                                                                int* __restrict__ hist, int hist_stride,
                                                                int* __restrict__ next_ids) {
  __shared__ float red[NT / 64];
  __shared__ float s_chunk[MAXT];
  __shared__ int s_tok;
  __shared__ float hbin[NB];
  __shared__ int s_ids[MAXC];
  __shared__ int s_hpos[NT];
  const int row = blockIdx.x;
  const SampleParams p = params[row];
  const bool penal = p.repeat_penalty != 1.f || p.presence_penalty != 0.f || p.frequency_penalty != 0.f;
  if (ctx_len[row] <= 0 || (p.temperature <= 0.f && !penal)) return;     // padding / greedy row
  const int* idr = ids + (size_t)row * ldi;
  for (int i = threadIdx.x; i < M; i += NT) s_ids[i] = idr[i];
  const int ps = pos[row];
  int* h = hist + (size_t)row * hist_stride;
  const int n_hist = min(hist_stride, ps + 1);
  __syncthreads();
  if (threadIdx.x < n_hist) {
    const int id = h[threadIdx.x];
    int at = -1;
    if (id >= 0)
      for (int i = 0; i < M; ++i)
        if (s_ids[i] == id) {
          at = i;
          break;
        }
    s_hpos[threadIdx.x] = at;
  }
  __syncthreads();
  const int j = sample_one(cand + (size_t)row * ld, M, p, uniform01(seeds[row], ps), s_hpos, n_hist, red, s_chunk,
                           &s_tok, hbin);
  if (threadIdx.x == 0) {
    const int tok = (j >= 0 && j < M && s_ids[j] >= 0) ? s_ids[j] : 0;
    next_ids[row] = tok;
    h[(ps + 1) % hist_stride] = tok;
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Tensor-parallel sampling: per row, the C largest logits of this rank's vocab shard in VOCABULARY order, written as
// (f32 value bits, global token id) straight into the [2][n][C] int32 source buffer of the candidate all-gather
// (parallel/comm.py gather_candidates) -- the round-5 graph ran PyTorch's radix top-k + sort + gather + fill + stack
// here (profiles/tp_graph_nodes_r05.txt). One 256-thread workgroup per row:
//   * radix select of the k-th largest order-preserving key (k = min(C, valid)): four 8-bit histogram passes over
//     the row (L2-resident after the first), each bin found by a wave-0 suffix scan; T = that key, need_eq = how many
//     keys equal to T belong to the top k (the lowest indices first: deterministic, ties never exceed k);
//   * compaction in index order: each thread owns a contiguous chunk, counts its keys > T and == T, a block
//     exclusive scan gives every thread its output offset, and it writes its selected entries in order.
// Shards with fewer than C tokens pad with (-inf, -1), as the host reference does.
constexpr int TCT = 256;

DEVI uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// exclusive prefix sums over the workgroup of two per-thread counts (TCT threads); returns via refs
DEVI void block_excl2(int a, int b, int& ea, int& eb, int* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int ia = a, ib = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int ta = __shfl_up(ia, o, 64), tb = __shfl_up(ib, o, 64);
    if (lane >= o) {
      ia += ta;
      ib += tb;
    }
  }
  if (lane == 63) {
    red[w] = ia;
    red[4 + w] = ib;
  }
  __syncthreads();
  int oa = 0, ob = 0;
#pragma unroll
  for (int i = 0; i < TCT / 64; ++i)
    if (i < w) {
      oa += red[i];
      ob += red[4 + i];
    }
  ea = oa + ia - a;
  eb = ob + ib - b;
}

__global__ __launch_bounds__(TCT) void topc_kernel(const float* __restrict__ logits, long ld, int valid, int C,
                                                   int vocab_lo, int* __restrict__ out, long plane) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_bin, s_above;
  __shared__ int red[8];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* x = logits + (size_t)row * ld;
  int* ov = out + (size_t)row * C;
  int* oi = out + plane + (size_t)row * C;
  const int k = min(C, max(valid, 0));
  for (int j = k + tid; j < C; j += TCT) {          // padding of a short shard
    ov[j] = (int)0xFF800000u;
    oi[j] = -1;
  }
  if (k <= 0) return;
  uint32_t prefix = 0u, mask = 0u;
  int need = k;                                       // keys still to take at the current prefix
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0u;
    __syncthreads();
    for (int i = tid; i < valid; i += TCT) {
      const uint32_t key = okey(x[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 64) {                                   // wave 0: lane l holds bins 4l..4l+3; suffix sums over lanes
      const uint32_t h0 = hist[4 * tid], h1 = hist[4 * tid + 1], h2 = hist[4 * tid + 2], h3 = hist[4 * tid + 3];
      const uint32_t ls = h0 + h1 + h2 + h3;
      uint32_t sfx = ls;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_down(sfx, o, 64);
        if (tid + o < 64) sfx += t;
      }
      uint32_t above = sfx - ls;                      // keys in bins above this lane's four
      const uint32_t hh[4] = {h0, h1, h2, h3};
#pragma unroll
      for (int e = 3; e >= 0; --e) {
        const uint32_t c = above + hh[e];
        if (above < (uint32_t)need && c >= (uint32_t)need) {
          s_bin = 4u * tid + e;
          s_above = above;
        }
        above = c;
      }
    }
    __syncthreads();
    prefix |= s_bin << shift;
    mask |= 255u << shift;
    need -= (int)s_above;
    __syncthreads();                                  // s_bin / hist reused by the next pass
  }
  // keys > prefix: k - need of them, all taken; keys == prefix: the first `need` in index order
  const int chunk = (valid + TCT - 1) / TCT;
  const int c0 = min(valid, tid * chunk), c1 = min(valid, c0 + chunk);
  int ngt = 0, neq = 0;
  for (int i = c0; i < c1; ++i) {
    const uint32_t key = okey(x[i]);
    ngt += key > prefix;
    neq += key == prefix;
  }
  int gt, eq;
  block_excl2(ngt, neq, gt, eq, red);
  for (int i = c0; i < c1; ++i) {
    const float v = x[i];
    const uint32_t key = okey(v);
    int pos = -1;
    if (key > prefix) {
      pos = gt + min(eq, need);
      ++gt;
    } else if (key == prefix) {
      if (eq < need) pos = gt + eq;
      ++eq;
    }
    if (pos >= 0) {
      ov[pos] = __float_as_int(v);
      oi[pos] = vocab_lo + i;
    }
  }
}

}  // namespace

// per row r < n: the C largest of logits[r][0, valid) in vocabulary order -> out[0][r][:] (f32 bits), out[1][r][:]
// (vocab_lo + index); plane = n * C (the offset of the id plane)
extern "C" int nls_topc(const float* logits, long ld, int n, int valid, int C, int vocab_lo, int* out, void* stream) {
  if (n < 1 || C < 1 || C > (1 << 16)) return -1;
  hipLaunchKernelGGL(topc_kernel, dim3(n), dim3(TCT), 0, (hipStream_t)stream, logits, ld, valid, C, vocab_lo, out,
                     (long)n * C);
  return (int)hipGetLastError();
}

extern "C" int nls_sample_decode_cand(void* cand, long ld, int n, int M, const int* ids, long ldi, const void* params,
                                      const void* seeds, const int* pos, const int* ctx_len, int* hist, int hist_stride,
                                      int* next_ids, void* stream) {
  if (n < 1 || M < 1 || M > MAXC || hist_stride < 1 || hist_stride > NT) return -1;
  hipLaunchKernelGGL(sample_decode_cand_kernel, dim3(n), dim3(NT), 0, (hipStream_t)stream, (float*)cand, ld, M, ids,
                     ldi, (const SampleParams*)params, (const unsigned long long*)seeds, pos, ctx_len, hist,
                     hist_stride, next_ids);
  return (int)hipGetLastError();
}

extern "C" int nls_sample(void* logits, long ld, int n, int V, const void* params, const int* hist, int hist_stride,
                          int* out, void* stream) {
  if (n < 1 || V < 1 || V > 64 * MAXT) return -1;
  hipLaunchKernelGGL(sample_kernel, dim3(n), dim3(NT), 0, (hipStream_t)stream, (float*)logits, ld, V,
                     (const SampleParams*)params, hist, hist_stride, out);
  return (int)hipGetLastError();
}

extern "C" int nls_sample_params_size() { return (int)sizeof(SampleParams); }

extern "C" int nls_sample_decode(void* logits, long ld, int n, int V, const void* params, const void* seeds,
                                 const int* pos, const int* ctx_len, int* hist, int hist_stride, int* next_ids,
                                 void* stream) {
  if (n < 1 || V < 1 || V > 64 * MAXT || hist_stride < 1 || hist_stride > NT) return -1;
  hipLaunchKernelGGL(sample_decode_kernel, dim3(n), dim3(NT), 0, (hipStream_t)stream, (float*)logits, ld, V,
                     (const SampleParams*)params, (const unsigned long long*)seeds, pos, ctx_len, hist, hist_stride,
                     next_ids);
  return (int)hipGetLastError();
}
