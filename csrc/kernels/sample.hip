// Batched token sampling on the GPU: repetition / presence / frequency penalties,
// temperature, top-k, min-p, top-p and the final draw -- one workgroup per row, one launch
// for every sampled request of a step (SURVEY.md §2F sample_topk_topp).
//
// No sort over the vocabulary: top-k and top-p become VALUE thresholds found by bisection
// over block-wide counts / sums (k-th largest logit; the logit above which the kept
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

__global__ __launch_bounds__(NT) void sample_kernel(float* __restrict__ logits, long ld, int V,
                                                    const SampleParams* __restrict__ params,
                                                    const int* __restrict__ hist, int hist_stride,
                                                    int* __restrict__ out) {
  __shared__ float red[NT / 64];
  __shared__ float s_chunk[NT];
  const int row = blockIdx.x;
  const SampleParams p = params[row];
  float* l = logits + (size_t)row * ld;

  // 1) penalties on the distinct ids of the history window (llama.cpp-style semantics)
  if (p.n_hist > 0 && (p.repeat_penalty != 1.f || p.presence_penalty != 0.f || p.frequency_penalty != 0.f)) {
    const int* h = hist + (size_t)row * hist_stride;
    const int j = threadIdx.x;
    if (j < p.n_hist) {
      const int id = h[j];
      bool first = true;
      int cnt = 0;
      for (int i = 0; i < p.n_hist; ++i) {
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
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < V; i += NT) mx = fmaxf(mx, l[i]);
  mx = block_max(mx, red);
  if (p.temperature <= 0.f) {
    int best = 0x7FFFFFFF;
    for (int i = threadIdx.x; i < V; i += NT)
      if (l[i] == mx) best = min(best, i);
    float b = (float)best;   // exact for V < 2^24
    b = -block_max(-b, red);
    if (threadIdx.x == 0) out[row] = (int)b;
    return;
  }
  const float it = 1.f / p.temperature;
  // 3) keep-threshold on the logit scale: top-k (k-th largest) and min-p (p >= min_p * p_max)
  float lo = -INFINITY;
  if (p.top_k > 0 && p.top_k < V) {
    float a = mx - 1.f, b = mx;         // find the largest t with count(l >= t) >= k
    // widen the lower bracket until it holds k values
    for (int it2 = 0; it2 < 40; ++it2) {
      float c = 0.f;
      for (int i = threadIdx.x; i < V; i += NT) c += l[i] >= a ? 1.f : 0.f;
      c = block_sum(c, red);
      if (c >= (float)p.top_k) break;
      a = mx - 2.f * (mx - a);
    }
    for (int it2 = 0; it2 < 32; ++it2) {
      const float t = 0.5f * (a + b);
      float c = 0.f;
      for (int i = threadIdx.x; i < V; i += NT) c += l[i] >= t ? 1.f : 0.f;
      c = block_sum(c, red);
      if (c >= (float)p.top_k) a = t; else b = t;
    }
    lo = a;
  }
  if (p.min_p > 0.f) lo = fmaxf(lo, mx + p.temperature * __logf(p.min_p));
  // 4) top-p: logit threshold above which the kept mass reaches top_p of the kept total
  float Z = 0.f;
  for (int i = threadIdx.x; i < V; i += NT)
    if (l[i] >= lo) Z += __expf((l[i] - mx) * it);
  Z = block_sum(Z, red);
  if (p.top_p < 1.f) {
    float a = lo == -INFINITY ? mx - 80.f * p.temperature : lo, b = mx;
    for (int it2 = 0; it2 < 32; ++it2) {
      const float t = 0.5f * (a + b);
      float s = 0.f;
      for (int i = threadIdx.x; i < V; i += NT)
        if (l[i] >= t && l[i] >= lo) s += __expf((l[i] - mx) * it);
      s = block_sum(s, red);
      if (s >= p.top_p * Z) a = t; else b = t;
    }
    lo = fmaxf(lo, a);
    Z = 0.f;
    for (int i = threadIdx.x; i < V; i += NT)
      if (l[i] >= lo) Z += __expf((l[i] - mx) * it);
    Z = block_sum(Z, red);
  }
  // 5) inverse CDF in index order: contiguous chunk per thread, scan of chunk sums
  const int per = (V + NT - 1) / NT;
  const int i0 = threadIdx.x * per, i1 = min(V, i0 + per);
  float cs = 0.f;
  for (int i = i0; i < i1; ++i)
    if (l[i] >= lo) cs += __expf((l[i] - mx) * it);
  s_chunk[threadIdx.x] = cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float target = p.u * Z;
    float acc = 0.f;
    int owner = -1;
    for (int t = 0; t < NT; ++t) {
      if (acc + s_chunk[t] > target && s_chunk[t] > 0.f) { owner = t; break; }
      acc += s_chunk[t];
    }
    int tok = -1, last = -1;
    if (owner >= 0) {
      const int a0 = owner * per, a1 = min(V, a0 + per);
      for (int i = a0; i < a1; ++i) {
        if (l[i] < lo) continue;
        last = i;
        acc += __expf((l[i] - mx) * it);
        if (acc > target) { tok = i; break; }
      }
      if (tok < 0) tok = last;
    }
    if (tok < 0) {            // rounding at the very end: the last kept token
      for (int i = V - 1; i >= 0; --i)
        if (l[i] >= lo) { tok = i; break; }
    }
    out[row] = tok;
  }
}

}  // namespace

extern "C" int nls_sample(void* logits, long ld, int n, int V, const void* params, const int* hist, int hist_stride,
                          int* out, void* stream) {
  if (n < 1 || V < 1) return -1;
  hipLaunchKernelGGL(sample_kernel, dim3(n), dim3(NT), 0, (hipStream_t)stream, (float*)logits, ld, V,
                     (const SampleParams*)params, hist, hist_stride, out);
  return (int)hipGetLastError();
}

extern "C" int nls_sample_params_size() { return (int)sizeof(SampleParams); }
