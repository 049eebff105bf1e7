// MoE top-k route of one token (shared by the route kernels in ops.hip and the o-projection GEMV that
// folds the FFN norm + router + route into its last workgroup, qgemv_impl.h).
#pragma once
#include "common.h"

// logits [T][E] f32; outputs: topw [T][k], counts [E] (must be zeroed), rows [E][T*k]
// (segment-local x row = token t, y row = t*k + j).
// One wave per token, lane e holds expert e (E <= 64): softmax and the k arg-max rounds are wave
// reductions, so nothing is indexed at run time (no scratch). NaN / inf logits: a NaN never wins a
// comparison, ties and NaNs resolve to the lowest unused expert, so k distinct valid experts are
// always chosen.
// One wave routes token t from its E logits `lt` (global or LDS).
DEVI void route_one(const float* __restrict__ lt, int t, int lane, int E, int k, int renorm, float* __restrict__ topw,
                    int* __restrict__ counts, int* __restrict__ xrows, int* __restrict__ yrows, int cap,
                    int* __restrict__ sel) {
  const bool live = lane < E;
  const float l = live ? lt[lane] : -INFINITY;
  float mx = l;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  const float p = live ? __expf(l - mx) : 0.f;
  float sum = p;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  bool used = !live;
  float wsum = 0.f, myw = 0.f;
  int myj = -1;
  for (int j = 0; j < k; ++j) {
    // arg-max over unused experts: key = (value ordered, lowest index wins ties); NaN -> lowest key
    const float v = used ? -INFINITY : p;
    uint32_t u = __float_as_uint(v);
    u = (v != v) ? 0u : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
    unsigned long long key = used ? 0ull : (((unsigned long long)u << 32) | (uint32_t)(63 - lane) | (1ull << 31));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long ok = __shfl_xor(key, o, 64);
      key = ok > key ? ok : key;
    }
    const int be = 63 - (int)(key & 63);
    const float bv = __shfl(p, be, 64);
    const float w = bv / sum;
    wsum += w;
    if (lane == be) {
      used = true;
      myw = w;
      myj = j;
    }
  }
  if (myj >= 0) {
    if (sel) sel[t * k + myj] = lane;           // routed expert of (token, slot): device-selected launches
    topw[t * k + myj] = renorm ? myw / wsum : myw;
    const int pos = atomicAdd(counts + lane, 1);
    xrows[lane * cap + pos] = t;
    yrows[lane * cap + pos] = t * k + myj;
  }
}

