// Elementwise / normalisation / positional / gather kernels (gfx950), SURVEY.md §2F:
// embed_gather_q, rmsnorm, rope (+ paged KV append), dequant_* (prefill + tests),
// logits argmax. All f16/bf16/f32 traffic is 16-B vectorised where rows allow it
// (cdna_hip_programming.md Guideline 13).
#include "common.h"
#include "moe_route.h"

namespace {

DEVI float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int BS>
DEVI float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) t += sh[i];
  __syncthreads();
  return t;
}

// ---------------------------------------------------------------------------
// RMSNorm: out_f16[m] = x[m] * rsqrt(mean(x^2) + eps) * w      (x f32, fp32 accumulate)
// Single pass: each of the 512 threads keeps its <= 4 float4 of the row in registers
// (D <= 8192), so the row is read once and the kernel is one reduction deep.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void rmsnorm_kernel(const float* __restrict__ x, long ldx,
                                                      const float* __restrict__ w,
                                                      act_t* __restrict__ out, long ldo, int D,
                                                      float eps) {
  __shared__ float sh[8];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float4 v[4], wv[4];
  float ss = 0.f;
  // the norm weights are loaded with the row, not after the reduction: one HBM round trip per
  // launch instead of two (a decode-time norm is latency-bound, B=1 profile: 65 per token)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
    v[j] = i < D ? *reinterpret_cast<const float4*>(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    wv[j] = i < D ? *reinterpret_cast<const float4*>(w + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  ss = block_sum<512>(ss, sh);
  const float inv = rsqrtf(ss / (float)D + eps);
  act_t* o = out + (size_t)blockIdx.x * ldo;
  typedef act_t act4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
    if (i < D) {
      const float4 ww = wv[j];
      act4 r = {(act_t)(v[j].x * inv * ww.x), (act_t)(v[j].y * inv * ww.y), (act_t)(v[j].z * inv * ww.z),
                (act_t)(v[j].w * inv * ww.w)};
      *reinterpret_cast<act4*>(o + i) = r;
    }
  }
}

// Fused split-K reduce + residual add + RMSNorm (row-parallel projections): the GEMM left
// ks fp32 partial slabs ws[k][M][D]; x[m] += alpha * sum_k ws[k][m] (fixed order: deterministic),
// then out[m] = f16(rmsnorm(x[m]) * w). One launch instead of reduce + norm, and x is read once.
#ifndef NLS_SLAB_RUNTIME
#define NLS_SLAB_RUNTIME 0   // 1: always the runtime-ks kernels (A/B build tag)
#endif
// KS > 0: the split count as a constant -- every slab load of the row is issued before the first add (ks is a
// runtime loop bound otherwise, and each slab's loads wait for the previous add chain); KS = 0: any ks.
template <int KS>
__global__ __launch_bounds__(512) void splitk_add_rmsnorm_kernel(const float* __restrict__ ws, int ks, int M,
                                                                 float alpha, float* __restrict__ x, long ldx,
                                                                 const float* __restrict__ w,
                                                                 act_t* __restrict__ out, long ldo, int D,
                                                                 float eps) {
  __shared__ float sh[8];
  const int m = blockIdx.x;
  float* xr = x + (size_t)m * ldx;
  float4 v[4], wv[4];
  float ss = 0.f;
  const int nk = KS > 0 ? KS : ks;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
    wv[j] = i < D ? *reinterpret_cast<const float4*>(w + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
    if (i < D) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (KS > 0) {
        float4 p[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) p[k] = *reinterpret_cast<const float4*>(ws + ((size_t)k * M + m) * D + i);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          acc.x += p[k].x; acc.y += p[k].y; acc.z += p[k].z; acc.w += p[k].w;
        }
      } else {
        for (int k = 0; k < nk; ++k) {
          const float4 p = *reinterpret_cast<const float4*>(ws + ((size_t)k * M + m) * D + i);
          acc.x += p.x; acc.y += p.y; acc.z += p.z; acc.w += p.w;
        }
      }
      float4 r = *reinterpret_cast<const float4*>(xr + i);
      r.x += alpha * acc.x; r.y += alpha * acc.y; r.z += alpha * acc.z; r.w += alpha * acc.w;
      *reinterpret_cast<float4*>(xr + i) = r;
      v[j] = r;
    } else {
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  }
  ss = block_sum<512>(ss, sh);
  const float inv = rsqrtf(ss / (float)D + eps);
  act_t* o = out + (size_t)m * ldo;
  typedef act_t act4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
    if (i < D) {
      const float4 ww = wv[j];
      act4 r = {(act_t)(v[j].x * inv * ww.x), (act_t)(v[j].y * inv * ww.y), (act_t)(v[j].z * inv * ww.z),
                (act_t)(v[j].w * inv * ww.w)};
      *reinterpret_cast<act4*>(o + i) = r;
    }
  }
}

// f32 -> f32 variant (final norm feeding an fp32 reference / lm-head in f32)
__global__ __launch_bounds__(256) void rmsnorm_f32_kernel(const float* __restrict__ x, long ldx,
                                                          const float* __restrict__ w,
                                                          float* __restrict__ out, long ldo, int D,
                                                          float eps) {
  __shared__ float sh[8];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float ss = 0.f;
  for (int i = threadIdx.x; i < D; i += 256) ss += xr[i] * xr[i];
  ss = block_sum<256>(ss, sh);
  const float inv = rsqrtf(ss / (float)D + eps);
  for (int i = threadIdx.x; i < D; i += 256) out[(size_t)blockIdx.x * ldo + i] = xr[i] * inv * w[i];
}

// ---------------------------------------------------------------------------
// RoPE on q,k (+ write k,v to the paged cache slot) for each token.
// qkv row: [Hq*D | Hkv*D | Hkv*D] f32. cs: [max_pos][D/2][2] (cos, sin) f32.
// neox=0: adjacent pairs (2i, 2i+1) -- GGUF llama "NORM" rope; neox=1: (i, i+D/2).
// ---------------------------------------------------------------------------
// `ks` > 1: the QKV projection left split-K partial slabs (qkv = ks slabs of [T][ldqkv], stride
// `slab` floats) and this kernel sums them in fixed order while rotating (fused reduce + RoPE).
template <typename KV, int KS = 0>     // KS > 0: the slab count as a constant (all slab loads issued first)
__global__ __launch_bounds__(256) void rope_kv_kernel(const float* __restrict__ qkv, long ldqkv, int ks, long slab,
                                                      const float* __restrict__ bias,
                                                      const int* __restrict__ pos,
                                                      const int* __restrict__ slot,
                                                      const float* __restrict__ cs,
                                                      __bf16* __restrict__ q_out, long ldq,
                                                      KV* __restrict__ kc, KV* __restrict__ vc,
                                                      int Hq, int Hkv, int D, int neox) {
  // Vectorised: every thread owns 4 consecutive columns (16-B slab loads, 8-B bf16 stores).
  const int t = blockIdx.x;
  const float* row = qkv + (size_t)t * ldqkv;
  auto ld4 = [&](int col) {
    float4 v;
    if constexpr (KS > 0) {
      float4 u[KS];
#pragma unroll
      for (int k = 0; k < KS; ++k) u[k] = *reinterpret_cast<const float4*>(row + (size_t)k * slab + col);
      v = u[0];
#pragma unroll
      for (int k = 1; k < KS; ++k) {
        v.x += u[k].x; v.y += u[k].y; v.z += u[k].z; v.w += u[k].w;
      }
    } else {
      v = *reinterpret_cast<const float4*>(row + col);
      for (int k = 1; k < ks; ++k) {
        const float4 u = *reinterpret_cast<const float4*>(row + (size_t)k * slab + col);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
      }
    }
    if (bias) {     // QKV projection bias (Qwen2), added before the rotation
      const float4 u = *reinterpret_cast<const float4*>(bias + col);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    return v;
  };
  typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
  auto st4 = [](__bf16* d, float a, float b, float c, float e) {
    *reinterpret_cast<bf4*>(d) = bf4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)e};
  };
  const int p = pos[t];
  const long s = slot[t];  // int32 slot index, widened
  const int half = D >> 1;
  const float* c = cs + (size_t)p * D;   // [D/2][2] (cos, sin)
  // head h < Hq: q (bf16); else the K cache row of kv head h - Hq (KV type)
  auto st = [&](int h, int col, float a, float b, float c2, float e) {
    if (h < Hq) st4(q_out + (size_t)t * ldq + h * D + col, a, b, c2, e);
    else kv_st4(kc + ((size_t)s * Hkv + (h - Hq)) * D + col, a, b, c2, e);
  };
  const int nh = s >= 0 ? Hq + Hkv : Hq;         // padded rows (slot -1) write no K/V
  if (!neox) {
    // adjacent pairs: columns col..col+3 = pairs col/2, col/2+1
    for (int idx = threadIdx.x; idx < nh * (D / 4); idx += blockDim.x) {
      const int h = idx / (D / 4), col = 4 * (idx - h * (D / 4));
      const float4 x = ld4(h * D + col);
      const float4 cw = *reinterpret_cast<const float4*>(c + col);   // (cos, sin) of pairs col/2, col/2+1
      st(h, col, x.x * cw.x - x.y * cw.y, x.x * cw.y + x.y * cw.x, x.z * cw.z - x.w * cw.w,
         x.z * cw.w + x.w * cw.z);
    }
  } else {
    // NEOX halves: columns i..i+3 pair with i+half..i+half+3
    for (int idx = threadIdx.x; idx < nh * (half / 4); idx += blockDim.x) {
      const int h = idx / (half / 4), i = 4 * (idx - h * (half / 4));
      const float4 a = ld4(h * D + i), b = ld4(h * D + half + i);
      const float4 c0 = *reinterpret_cast<const float4*>(c + 2 * i), c1 = *reinterpret_cast<const float4*>(c + 2 * i + 4);
      const float cc[4] = {c0.x, c0.z, c1.x, c1.z}, sn[4] = {c0.y, c0.w, c1.y, c1.w};
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
      float y0[4], y1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        y0[u] = av[u] * cc[u] - bv[u] * sn[u];
        y1[u] = av[u] * sn[u] + bv[u] * cc[u];
      }
      st(h, i, y0[0], y0[1], y0[2], y0[3]);
      st(h, half + i, y1[0], y1[1], y1[2], y1[3]);
    }
  }
  if (s >= 0) {
    const int v0 = (Hq + Hkv) * D;
    KV* vd = vc + (size_t)s * Hkv * D;
    for (int i = 4 * threadIdx.x; i < Hkv * D; i += 4 * blockDim.x) {
      const float4 v = ld4(v0 + i);
      kv_st4(vd + i, v.x, v.y, v.z, v.w);
    }
  }
}

// ---------------------------------------------------------------------------
// Embedding gather + dequant: out[t, :] = scale * W[ids[t], :]
// ---------------------------------------------------------------------------
// Embedding gather: one workgroup per token. The format switch is resolved once per launch (template)
// and the element loop unrolled, so the loads of many elements are in flight together (a per-element
// format switch kept successive elements' loads in series: 11.7 us for one 4096-wide row at batch 1).
// Chained decode (`next_ids` set): the token is next_ids[t] where use_prev[t] != 0, else ids[t], and the
// choice is written back to ids[t] (the separate torch.where launch folded in).
// Grid (tokens, K / 256): one element per thread, so a row costs one round of loads, not K / 256 of them.
template <int TYPE>
DEVI void embed_row(const WDesc& W, int id, float* __restrict__ o, float scale) {
  const int k = blockIdx.y * 256 + threadIdx.x;
  if (k < W.K) o[k] = scale * dequant_elem(W, TYPE, id, k);
}

__global__ __launch_bounds__(256) void embed_kernel(int* __restrict__ ids, WDesc W, int type,
                                                    float* __restrict__ out, long ldo, float scale,
                                                    const int* __restrict__ next_ids, const int* __restrict__ use_prev) {
  const int t = blockIdx.x;
  int id = ids[t];
  if (next_ids) {
    if (use_prev[t]) id = next_ids[t];
    __syncthreads();                         // every thread has read ids[t] before it is rewritten
    // slice 0 records the choice; another slice may read ids[t] before or after that store and picks the
    // same id either way (where use_prev[t] is set, next_ids[t] wins over whatever ids[t] holds)
    if (threadIdx.x == 0 && blockIdx.y == 0) ids[t] = id;
  }
  // clamped: a bad id (device-chained decode feeds sampled ids back without a host check) must not
  // become a wild address
  id = min(max(id, 0), W.rows - 1);
  float* o = out + (size_t)t * ldo;
  switch (type) {
    case QT_F32: embed_row<QT_F32>(W, id, o, scale); break;
    case QT_F16: embed_row<QT_F16>(W, id, o, scale); break;
    case QT_BF16: embed_row<QT_BF16>(W, id, o, scale); break;
    case QT_Q8_0: embed_row<QT_Q8_0>(W, id, o, scale); break;
    case QT_Q4_K: embed_row<QT_Q4_K>(W, id, o, scale); break;
    case QT_Q5_K: embed_row<QT_Q5_K>(W, id, o, scale); break;
    case QT_Q6_K: embed_row<QT_Q6_K>(W, id, o, scale); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------
// Whole-tensor dequant to f16 (tests / debugging). One wave = 16 rows
// x one 256 super-block, using the same register dequant as the GEMV.
// ---------------------------------------------------------------------------
template <int T>
__global__ __launch_bounds__(256) void dequant_kernel(WDesc W, act_t* __restrict__ out, long ldo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int row = blockIdx.x * 16 + r;
  const int sb = blockIdx.y * 4 + wave;
  if (sb >= (W.K >> 8)) return;
  const int rowc = min(row, W.rows - 1);
  auto raw = load_raw<T, false>(W, rowc, sb, g);
  f16x8 wf[8];
  dequant<T>(raw, g, wf);
  if (row >= W.rows) return;
#pragma unroll
  for (int t = 0; t < 8; ++t)
    *reinterpret_cast<f16x8*>(out + (size_t)row * ldo + sb * 256 + xoff<T>(t, g)) = wf[t];
}

// ---------------------------------------------------------------------------
// Greedy argmax over logits rows (standalone; the lm-head GEMV can also fuse it)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ logits, long ld, int V,
                                                      int* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const float* row = logits + (size_t)blockIdx.x * ld;
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  for (int i = threadIdx.x; i < V; i += 1024) {
    const float v = row[i];
    if (v > bv) { bv = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    bv = sv[0]; bi = si[0];
    for (int i = 1; i < 16; ++i)
      if (sv[i] > bv || (sv[i] == bv && si[i] < bi)) { bv = sv[i]; bi = si[i]; }
    out[blockIdx.x] = bi;
  }
}

// unpack the fused-argmax u64 keys into token ids
// keys -> token ids; with `rearm` the keys are zeroed after the read (the next step's fused arg-max then
// needs no reset launch)
__global__ void argmax_unpack_kernel(unsigned long long* __restrict__ keys, int n, int* __restrict__ out,
                                     int rearm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    out[i] = (int)(0xFFFFFFFFu - (uint32_t)(keys[i] & 0xFFFFFFFFull));
    if (rearm) keys[i] = 0ull;
  }
}

// residual += sum_k w[t,k] * y[t*topk + k]   (MoE combine, deterministic order)
// SET: resid = alpha * sum instead of +=  (a tensor-parallel rank's partial combine from zero: no fill launch in the
// decode graph before it)
template <bool SET>
__global__ __launch_bounds__(256) void moe_combine_kernel(const float* __restrict__ y, const float* __restrict__ w,
                                                          int topk, float* __restrict__ resid, long ldr,
                                                          int D, float alpha) {
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < D; i += 256) {
    float s = 0.f;
    for (int k = 0; k < topk; ++k) s += w[t * topk + k] * y[((size_t)t * topk + k) * D + i];
    if (SET) resid[(size_t)t * ldr + i] = alpha * s;
    else resid[(size_t)t * ldr + i] += alpha * s;
  }
}

// combine + the next layer's input RMSNorm in one launch (single rank, few tokens): resid[t] +=
// alpha * sum_j w[t,j] * y[t*k+j]; h[t] = f16(rmsnorm(resid[t]) * nw). One workgroup per token: every
// load of a thread's 4-float groups is issued before any arithmetic (a loop that loads, adds and
// stores per element serialises ~16 dependent round trips per thread: 13 us at batch 1).
template <int KMAX>
__global__ __launch_bounds__(256) void moe_combine_norm_kernel(const float* __restrict__ y, const float* __restrict__ w,
                                                               int topk, float* __restrict__ resid, long ldr, int D,
                                                               float alpha, const float* __restrict__ nw, float eps,
                                                               act_t* __restrict__ h, long ldh) {
  __shared__ float sh[8];
  constexpr int NV = 4;                        // float4 groups per thread per pass (D <= 4096 in one pass)
  const int t = blockIdx.x;
  float* xr = resid + (size_t)t * ldr;
  float wk[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) wk[j] = j < topk ? w[t * topk + j] * alpha : 0.f;
  float ss = 0.f;
  for (int base = threadIdx.x * 4; base < D; base += 256 * 4 * NV) {
    float4 xv[NV], yv[KMAX][NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = base + u * 1024;
      xv[u] = i < D ? *reinterpret_cast<const float4*>(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < KMAX; ++j)
        yv[j][u] = (j < topk && i < D) ? *reinterpret_cast<const float4*>(y + ((size_t)t * topk + j) * D + i)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = base + u * 1024;
      float4 v = xv[u];
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        v.x += wk[j] * yv[j][u].x;
        v.y += wk[j] * yv[j][u].y;
        v.z += wk[j] * yv[j][u].z;
        v.w += wk[j] * yv[j][u].w;
      }
      xv[u] = v;
      if (i < D) *reinterpret_cast<float4*>(xr + i) = v;
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  }
  ss = block_sum<256>(ss, sh);
  const float inv = rsqrtf(ss / (float)D + eps);
  typedef act_t act4 __attribute__((ext_vector_type(4)));
  for (int i = threadIdx.x * 4; i < D; i += 1024) {
    const float4 v = *reinterpret_cast<const float4*>(xr + i);
    const float4 g = *reinterpret_cast<const float4*>(nw + i);
    *reinterpret_cast<act4*>(h + (size_t)t * ldh + i) =
        act4{(act_t)(v.x * inv * g.x), (act_t)(v.y * inv * g.y), (act_t)(v.z * inv * g.z), (act_t)(v.w * inv * g.w)};
  }
}

// MoE router: softmax over E logits -> top-k (renormalised) -> per-expert row lists.
__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, int T, int E, int k,
                                                        int renorm, float* __restrict__ topw,
                                                        int* __restrict__ counts, int* __restrict__ xrows,
                                                        int* __restrict__ yrows, int cap, int* __restrict__ sel) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gridDim.x == 1) {      // one workgroup (<= 4 tokens): zero the counts here (no host memset launch)
    for (int e = threadIdx.x; e < E; e += 256) counts[e] = 0;
    __syncthreads();
  }
  if (t >= T || E > 64 || k > 8 || k > E) return;    // host checks these too
  route_one(logits + (size_t)t * E, t, lane, E, k, renorm, topw, counts, xrows, yrows, cap, sel);
}

// MoE decode at <= 4 tokens: the post-attention RMSNorm (h = f16(x * rsqrt(mean(x^2) + eps) * nw), as
// rmsnorm_kernel), the router logits h . Wr[e] (Wr: the router's f16 copy, [E][D] row-major -- the
// router GEMV also multiplies f16 weights) and the top-k route (route_one) in ONE launch, where batch-1
// Mixtral ran three latency-bound ones (rmsnorm 4.5 + router GEMV 7.2 + route 4.5 us per layer,
// profiles/moe_selected_experts.txt).
template <int E>
__global__ __launch_bounds__(512) void moe_norm_route_kernel(
    const float* __restrict__ x, long ldx, const float* __restrict__ nw, float eps, int D,
    const act_t* __restrict__ wr, act_t* __restrict__ h, long ldh, float* __restrict__ logits, int T, int k,
    int renorm, float* __restrict__ topw, int* __restrict__ counts, int* __restrict__ xrows, int* __restrict__ yrows,
    int cap, int* __restrict__ sel) {
  __shared__ float sh[8];
  __shared__ float red[8][E];
  __shared__ float lg[4][E];
  for (int e = threadIdx.x; e < E; e += 512) counts[e] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  typedef act_t act4 __attribute__((ext_vector_type(4)));
  // the router rows do not depend on x: issue their loads first, once for all tokens, so the HBM latency overlaps
  // the x / norm-weight loads and the norm's block reduction instead of following them
  act4 w4r[4][E];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (threadIdx.x + j * 512) * 4;
#pragma unroll
    for (int e = 0; e < E; ++e)
      w4r[j][e] = i < D ? *reinterpret_cast<const act4*>(wr + (size_t)e * D + i) : act4{0, 0, 0, 0};
  }
  for (int t = 0; t < T; ++t) {
    const float* xr = x + (size_t)t * ldx;
    float4 v[4], wv[4];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = (threadIdx.x + j * 512) * 4;
      v[j] = i < D ? *reinterpret_cast<const float4*>(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      wv[j] = i < D ? *reinterpret_cast<const float4*>(nw + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
    }
    ss = block_sum<512>(ss, sh);
    const float inv = rsqrtf(ss / (float)D + eps);
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = (threadIdx.x + j * 512) * 4;
      if (i < D) {
        const float4 ww = wv[j];
        const act4 r = {(act_t)(v[j].x * inv * ww.x), (act_t)(v[j].y * inv * ww.y), (act_t)(v[j].z * inv * ww.z),
                        (act_t)(v[j].w * inv * ww.w)};
        *reinterpret_cast<act4*>(h + (size_t)t * ldh + i) = r;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const act4 w4 = w4r[j][e];
          acc[e] += (float)r.x * (float)w4.x + (float)r.y * (float)w4.y + (float)r.z * (float)w4.z +
                    (float)r.w * (float)w4.w;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float a = wave_sum(acc[e]);
      if (lane == 0) red[wave][e] = a;
    }
    __syncthreads();
    if (threadIdx.x < E) {
      float s2 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) s2 += red[w][threadIdx.x];
      lg[t][threadIdx.x] = s2;
      logits[(size_t)t * E + threadIdx.x] = s2;
    }
    __syncthreads();
  }
  if (wave < T) route_one(lg[wave], wave, lane, E, k, renorm, topw, counts, xrows, yrows, cap, sel);
}

// MoE router logits for many tokens (prefill chunks, decode batches > 4): logits[t][e] = h[t] . Wr[e] with Wr
// the router's f16 copy [E][D]. The router is E (2-8) rows: the GEMV/GEMM tiles (128 weight rows per
// workgroup, 128-row activation blocks) ran it on M / 128 workgroups with 15/16 of each MFMA idle -- ~50 us per
// layer at 256 tokens (profiles/rocprof_mixtral_b256_quant_experts.txt). Here a workgroup takes TPB tokens:
// each thread keeps its 8-value slices of the E router rows in registers per 16-byte chunk of D and dots them
// with every token's slice (f32 accumulation), then one wave sum + an LDS sum over the 8 waves per (token,
// expert).
// `zero` (optional, nz ints): the following route launch's expert counts, zeroed here by workgroup 0 (stream
// order puts the previous layer's expert GEMMs, their last readers, before this launch) -- no memset launch.
template <int E, int TPB>
__global__ __launch_bounds__(512) void router_logits_kernel(const act_t* __restrict__ h, long ldh,
                                                            const act_t* __restrict__ wr, int D,
                                                            float* __restrict__ logits, int T, int* __restrict__ zero,
                                                            int nz) {
  __shared__ float red[TPB][8][E];
  if (zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < nz; i += 512) zero[i] = 0;
  typedef act_t act8 __attribute__((ext_vector_type(8)));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t0 = blockIdx.x * TPB;
  float acc[TPB][E];
#pragma unroll
  for (int t = 0; t < TPB; ++t)
#pragma unroll
    for (int e = 0; e < E; ++e) acc[t][e] = 0.f;
  for (int c = threadIdx.x * 8; c < D; c += 512 * 8) {
    act8 w[E];
#pragma unroll
    for (int e = 0; e < E; ++e) w[e] = *reinterpret_cast<const act8*>(wr + (size_t)e * D + c);
#pragma unroll
    for (int t = 0; t < TPB; ++t) {
      if (t0 + t >= T) break;
      const act8 x = *reinterpret_cast<const act8*>(h + (size_t)(t0 + t) * ldh + c);
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[t][e] += (float)x[i] * (float)w[e][i];
    }
  }
#pragma unroll
  for (int t = 0; t < TPB; ++t)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float a = wave_sum(acc[t][e]);
      if (lane == 0) red[t][wave][e] = a;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < TPB * E; i += 512) {
    const int t = i / E, e = i % E;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[t][w][e];
    if (t0 + t < T) logits[(size_t)(t0 + t) * E + e] = v;
  }
}

// SwiGLU pass after a library GEMM on the gate/up weights (ops "mode 7"): the GEMM's f16 output h keeps
// the weights' [g0..g7, u0..u7] interleave per 16 columns, so out[m, 8j + i] = silu(alpha * h[m, 16j + i]) *
// alpha * h[m, 16j + 8 + i]. One thread per 8 outputs: two 16-B loads, one 16-B store (HBM-bound).
__global__ __launch_bounds__(256) void swiglu16_kernel(const act_t* __restrict__ h, long ldh, int ng, float alpha,
                                                       act_t* __restrict__ out, long ldo) {
  const int m = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= ng) return;
  const act_t* src = h + (size_t)m * ldh + 16 * j;
  const f16x8 g = *reinterpret_cast<const f16x8*>(src);
  const f16x8 u = *reinterpret_cast<const f16x8*>(src + 8);
  f16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float gv = alpha * (float)g[i];
    o[i] = (act_t)(gv / (1.f + __expf(-gv)) * (alpha * (float)u[i]));
  }
  *reinterpret_cast<f16x8*>(out + (size_t)m * ldo + 8 * j) = o;
}

// Touch `bytes` of device memory (16-B loads, grid-stride over the whole grid) so that a later kernel finds them
// in the memory-side Infinity Cache (MALL, 256 MB) / L2 instead of HBM -- the batch-1 decode experiment: stream
// the NEXT projection's weights while a latency-bound kernel (attention, a GEMV's tail) leaves HBM idle. The
// loaded words feed a sum that is stored only if it equals a value it never takes (keeps the loads alive).
__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ p, long n16, uint32_t never,
                                                       uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const long stride = (long)gridDim.x * 256 * 4;
  for (long i = (long)blockIdx.x * 256 * 4 + threadIdx.x; i < n16; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < n16 ? p[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == never && sink) sink[threadIdx.x] = acc;
}

}  // namespace

// ===========================================================================
// Paged attention (decode and prefill-as-decode): see attention.hip
// ===========================================================================

extern "C" {

int nls_prefetch(const void* p, long bytes, int blocks, void* stream) {
  if (bytes <= 0) return 0;
  hipLaunchKernelGGL(prefetch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, bytes / 16,
                     0x9E3779B9u, (uint32_t*)nullptr);
  return (int)hipGetLastError();
}

int nls_rmsnorm(const float* x, long ldx, const float* w, void* out, long ldo, int M, int D, float eps,
                int out_f32, void* stream) {
  if (D % 4 || D > 8192) return -1;
  if (out_f32)
    hipLaunchKernelGGL(rmsnorm_f32_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, x, ldx, w,
                       (float*)out, ldo, D, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel, dim3(M), dim3(512), 0, (hipStream_t)stream, x, ldx, w,
                       (act_t*)out, ldo, D, eps);
  return (int)hipGetLastError();
}

int nls_splitk_add_rmsnorm(const float* ws, int ks, int M, float alpha, float* x, long ldx, const float* w,
                           void* out, long ldo, int D, float eps, void* stream) {
  if (D % 4 || D > 8192 || ks < 1) return -1;
  const int kc = NLS_SLAB_RUNTIME ? 0 : ks;
  auto k = kc == 2 ? splitk_add_rmsnorm_kernel<2> : kc == 3 ? splitk_add_rmsnorm_kernel<3>
         : kc == 4 ? splitk_add_rmsnorm_kernel<4> : kc == 1 ? splitk_add_rmsnorm_kernel<1> : splitk_add_rmsnorm_kernel<0>;
  hipLaunchKernelGGL(k, dim3(M), dim3(512), 0, (hipStream_t)stream, ws, ks, M, alpha, x, ldx, w, (act_t*)out, ldo, D,
                     eps);
  return (int)hipGetLastError();
}

int nls_rope_kv(const float* qkv, long ldqkv, int ks, long slab, const float* bias, const int* pos, const int* slot,
                const float* cs, void* q_out, long ldq, void* kc, void* vc, int T, int Hq, int Hkv, int D, int neox,
                void* stream) {
  if (ks < 1 || D % 8) return -1;
  const int nk = NLS_SLAB_RUNTIME ? 0 : ks;
  auto k = nk == 1 ? rope_kv_kernel<__bf16, 1> : nk == 2 ? rope_kv_kernel<__bf16, 2> : nk == 3 ? rope_kv_kernel<__bf16, 3>
         : nk == 4 ? rope_kv_kernel<__bf16, 4> : rope_kv_kernel<__bf16, 0>;
  hipLaunchKernelGGL(k, dim3(T), dim3(256), 0, (hipStream_t)stream, qkv, ldqkv, ks, slab, bias, pos,
                     slot, cs, (__bf16*)q_out, ldq, (__bf16*)kc, (__bf16*)vc, Hq, Hkv, D, neox);
  return (int)hipGetLastError();
}

// the same with an fp8 (OCP e4m3) K/V cache
int nls_rope_kv8(const float* qkv, long ldqkv, int ks, long slab, const float* bias, const int* pos, const int* slot,
                 const float* cs, void* q_out, long ldq, void* kc, void* vc, int T, int Hq, int Hkv, int D, int neox,
                 void* stream) {
  if (ks < 1 || D % 8) return -1;
  hipLaunchKernelGGL(rope_kv_kernel<uint8_t>, dim3(T), dim3(256), 0, (hipStream_t)stream, qkv, ldqkv, ks, slab, bias,
                     pos, slot, cs, (__bf16*)q_out, ldq, (uint8_t*)kc, (uint8_t*)vc, Hq, Hkv, D, neox);
  return (int)hipGetLastError();
}

int nls_embed(const int* ids, int T, const void* w, int type, int rows, int K, float* out, long ldo,
              float scale, void* stream) {
  WDesc W{(const uint8_t*)w, rows, K};
  hipLaunchKernelGGL(embed_kernel, dim3(T, (K + 255) / 256), dim3(256), 0, (hipStream_t)stream, const_cast<int*>(ids),
                     W, type, out, ldo, scale, nullptr, nullptr);
  return (int)hipGetLastError();
}

// chained decode: ids[t] = use_prev[t] ? next_ids[t] : ids[t], then the gather
int nls_embed_prev(int* ids, const int* next_ids, const int* use_prev, int T, const void* w, int type, int rows,
                   int K, float* out, long ldo, float scale, void* stream) {
  WDesc W{(const uint8_t*)w, rows, K};
  hipLaunchKernelGGL(embed_kernel, dim3(T, (K + 255) / 256), dim3(256), 0, (hipStream_t)stream, ids, W, type, out,
                     ldo, scale, next_ids, use_prev);
  return (int)hipGetLastError();
}

int nls_dequant(const void* w, int type, int rows, int K, void* out, long ldo, void* stream) {
  if (K % 256) return -1;
  WDesc W{(const uint8_t*)w, rows, K};
  dim3 grid((rows + 15) / 16, ((K >> 8) + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  act_t* o = (act_t*)out;
  switch (type) {
    case QT_Q4_K: hipLaunchKernelGGL(dequant_kernel<QT_Q4_K>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_Q5_K: hipLaunchKernelGGL(dequant_kernel<QT_Q5_K>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_Q6_K: hipLaunchKernelGGL(dequant_kernel<QT_Q6_K>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_Q8_0: hipLaunchKernelGGL(dequant_kernel<QT_Q8_0>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_Q51: hipLaunchKernelGGL(dequant_kernel<QT_Q51>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_F16: hipLaunchKernelGGL(dequant_kernel<QT_F16>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_BF16: hipLaunchKernelGGL(dequant_kernel<QT_BF16>, grid, dim3(256), 0, st, W, o, ldo); break;
    case QT_F32: hipLaunchKernelGGL(dequant_kernel<QT_F32>, grid, dim3(256), 0, st, W, o, ldo); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// h: f16 [M, ncol] (interleaved gate/up GEMM output, row stride ldh); out: f16 [M, ncol / 2] (stride ldo)
int nls_swiglu16(const void* h, long ldh, int M, int ncol, float alpha, void* out, long ldo, void* stream) {
  if (M < 1 || ncol % 16 || ldh % 8 || ldo % 8 || ((uintptr_t)h & 15) || ((uintptr_t)out & 15)) return -1;
  const int ng = ncol / 16;
  hipLaunchKernelGGL(swiglu16_kernel, dim3((ng + 255) / 256, M), dim3(256), 0, (hipStream_t)stream,
                     (const act_t*)h, ldh, ng, alpha, (act_t*)out, ldo);
  return (int)hipGetLastError();
}

int nls_argmax(const float* logits, long ld, int M, int V, int* out, void* stream) {
  hipLaunchKernelGGL(argmax_kernel, dim3(M), dim3(1024), 0, (hipStream_t)stream, logits, ld, V, out);
  return (int)hipGetLastError();
}

int nls_argmax_unpack(const void* keys, int n, int* out, void* stream) {
  hipLaunchKernelGGL(argmax_unpack_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     (unsigned long long*)keys, n, out, 0);
  return (int)hipGetLastError();
}

int nls_argmax_unpack_rearm(void* keys, int n, int* out, void* stream) {
  hipLaunchKernelGGL(argmax_unpack_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     (unsigned long long*)keys, n, out, 1);
  return (int)hipGetLastError();
}

// counts: zeroed inside the kernel when T <= 4 (one workgroup), else by the caller; sel (optional):
// [T*k] expert id of each (token, slot)
int nls_moe_route(const float* logits, int T, int E, int k, int renorm, float* topw, int* counts, int* xrows,
                  int* yrows, int cap, int* sel, void* stream) {
  if (E > 64 || k > 8) return -1;
  hipLaunchKernelGGL(moe_route_kernel, dim3((T + 3) / 4), dim3(256), 0, (hipStream_t)stream, logits, T, E, k,
                     renorm, topw, counts, xrows, yrows, cap, sel);
  return (int)hipGetLastError();
}

// x f32 [T][ldx] residual rows, nw f32 [D], wr f16 [E][D], h f16 [T][ldh] (out), logits f32 [T][E] (out)
// router logits of T tokens (see router_logits_kernel): h f16 [T][ldh], wr f16 [E][D], logits f32 [T][E]
int nls_router_logits(const void* h, long ldh, const void* wr, int D, int E, float* logits, int T, int* zero, int nz,
                      void* stream) {
  if (T < 1 || D % 8 || ldh % 8) return -1;
  // one token per 8-wave workgroup: a 4096-wide row is one 16-byte chunk per thread, and the grid has T
  // workgroups (4 tokens per 4-wave workgroup measured 11.2 us per launch at 256 tokens: 64 workgroups)
  constexpr int TPB = 1;
  const dim3 grid((T + TPB - 1) / TPB);
  hipStream_t st = (hipStream_t)stream;
#define NLS_RL(EE)                                                                                             \
  if (E == EE) {                                                                                               \
    hipLaunchKernelGGL((router_logits_kernel<EE, TPB>), grid, dim3(512), 0, st, (const act_t*)h, ldh,            \
                       (const act_t*)wr, D, logits, T, zero, nz);                                              \
    return (int)hipGetLastError();                                                                             \
  }
  NLS_RL(2) NLS_RL(4) NLS_RL(8)
#undef NLS_RL
  return -1;
}

int nls_moe_norm_route(const float* x, long ldx, const float* nw, float eps, int D, const void* wr, void* h, long ldh,
                       float* logits, int T, int E, int k, int renorm, float* topw, int* counts, int* xrows, int* yrows,
                       int cap, int* sel, void* stream) {
  if (T < 1 || T > 4 || D % 4 || D > 8192 || k < 1 || k > E || ldx % 4 || ldh % 4) return -1;
  hipStream_t st = (hipStream_t)stream;
#define NLS_MNR(EE)                                                                                              \
  if (E == EE) {                                                                                               \
    hipLaunchKernelGGL(moe_norm_route_kernel<EE>, dim3(1), dim3(512), 0, st, x, ldx, nw, eps, D, (const act_t*)wr, \
                       (act_t*)h, ldh, logits, T, k, renorm, topw, counts, xrows, yrows, cap, sel);             \
    return (int)hipGetLastError();                                                                             \
  }
  NLS_MNR(2) NLS_MNR(4) NLS_MNR(8)
#undef NLS_MNR
  return -1;
}

int nls_moe_combine(const float* y, const float* w, int T, int topk, float* resid, long ldr, int D, float alpha,
                    int set, void* stream) {
  if (set)
    hipLaunchKernelGGL(moe_combine_kernel<true>, dim3(T), dim3(256), 0, (hipStream_t)stream, y, w, topk, resid, ldr, D,
                       alpha);
  else
    hipLaunchKernelGGL(moe_combine_kernel<false>, dim3(T), dim3(256), 0, (hipStream_t)stream, y, w, topk, resid, ldr,
                       D, alpha);
  return (int)hipGetLastError();
}

int nls_moe_combine_norm(const float* y, const float* w, int T, int topk, float* resid, long ldr, int D, float alpha,
                         const float* nw, float eps, void* h, long ldh, void* stream) {
  if (D % 4 || topk > 8 || topk < 1) return -1;
  if (topk <= 2)
    hipLaunchKernelGGL(moe_combine_norm_kernel<2>, dim3(T), dim3(256), 0, (hipStream_t)stream, y, w, topk, resid, ldr,
                       D, alpha, nw, eps, (act_t*)h, ldh);
  else
    hipLaunchKernelGGL(moe_combine_norm_kernel<8>, dim3(T), dim3(256), 0, (hipStream_t)stream, y, w, topk, resid, ldr,
                       D, alpha, nw, eps, (act_t*)h, ldh);
  return (int)hipGetLastError();
}

}  // extern "C"
