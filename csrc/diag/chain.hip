// Batch-1 stage-handoff probe (tools/diag/fencefree_chain.py): a chain of L dependent M=1 GEMVs
// x_{l+1} = f16(S_l * (W_l x_l)), W_l 4096 x 4096 4-bit (nibble - 8, one f32 scale per row; 8 MiB per link, about
// a Q4_K projection's bytes), run
//   serial      -- one launch per link, x read with plain loads after the kernel boundary (the decode graph today);
//   ff_link     -- one launch per link, the links alternating over two graph branches with no graph edge between
//                  them: every link issues its weight loads, then polls its input x_l (no fence anywhere);
//   persistent  -- one launch for the whole chain, 256 co-resident workgroups, per link: (prefetch), wait, compute,
//                  publish -- again without a fence.
// Fence-free handoff: every x word is self-tagged -- (tag << 16) | f16 bits -- and written / polled with relaxed
// agent-scope atomics (global, sc1: past this CU's L1 and never a stale line of the reader's XCD), so a reader
// that sees the tag has the value in the same word: no release / acquire, no counters, no L2 writeback or
// invalidate (what made the r05 device-dependency 3.7x slower, profiles/b1_overlap_r05.txt). The tag is the
// replay's epoch, bumped on the device by chain_init at the start of each replay, so a replayed graph never
// matches a previous replay's words. Every poll is bounded (max_spins); a timed-out workgroup counts it in err[0],
// stops waiting for the rest of the launch and keeps publishing, so the grid always drains.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int D = 4096, NT = 256, RW = 16, NWG = D / RW, NJ = 8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ uint32_t pack(float v, uint32_t tag) {
  return (tag << 16) | (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v);
}
__device__ __forceinline__ float unpack(uint32_t w) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu));
}

// weights of (link, workgroup): chunk (j, t) of 16 B at ((link * NWG + wg) * NJ + j) * NT + t; thread t owns row
// 16 wg + (t >> 4) and K range 256 (t & 15) + 32 j + [0, 32): dword d, nibble n -> k = 256 c + 32 j + 8 d + n
struct W8 { u32x4 v[NJ]; };
__device__ __forceinline__ void load_w(W8& w, const u32x4* W, int link, int wg, int t) {
  const u32x4* p = W + ((size_t)link * NWG + wg) * NJ * NT + t;
#pragma unroll
  for (int j = 0; j < NJ; ++j) w.v[j] = __builtin_nontemporal_load(p + j * NT);
}

// LDS copy of x in f32, 4 floats of padding every 256 values: the 16 K-chunk lanes of a row hit distinct banks
__device__ __forceinline__ int xi(int k) { return k + 4 * (k >> 8); }
constexpr int XS = D + 4 * (D / 256);

__device__ __forceinline__ float dot_row(const W8& w, const float* xs, int c) {
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t q = w.v[j][d];
      const int k = 256 * c + 32 * j + 8 * d;
      const float4 a = *reinterpret_cast<const float4*>(xs + xi(k));
      const float4 b = *reinterpret_cast<const float4*>(xs + xi(k) + 4);
      acc += (float)((int)(q & 15u) - 8) * a.x + (float)((int)((q >> 4) & 15u) - 8) * a.y +
             (float)((int)((q >> 8) & 15u) - 8) * a.z + (float)((int)((q >> 12) & 15u) - 8) * a.w +
             (float)((int)((q >> 16) & 15u) - 8) * b.x + (float)((int)((q >> 20) & 15u) - 8) * b.y +
             (float)((int)((q >> 24) & 15u) - 8) * b.z + (float)((int)(q >> 28) - 8) * b.w;
    }
  // the 16 K-chunk lanes of the row are adjacent lanes of one wave
  acc += __shfl_xor(acc, 8, 16);
  acc += __shfl_xor(acc, 4, 16);
  acc += __shfl_xor(acc, 2, 16);
  acc += __shfl_xor(acc, 1, 16);
  return acc;
}

// thread t stages words [16 t, 16 t + 16) of x_l: all 8 pairs loaded, then checked, until every tag matches
template <bool FF>
__device__ __forceinline__ bool stage_x(const uint32_t* Xl, uint32_t tag, float* xs, int t, long max_spins,
                                        int* err) {
  const unsigned long long* p = reinterpret_cast<const unsigned long long*>(Xl + 16 * t);
  for (long spin = 0;; ++spin) {
    unsigned long long v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = FF ? __hip_atomic_load((const gu64*)(p + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : p[i];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) ok &= ((uint32_t)v[i] >> 16) == tag && (uint32_t)(v[i] >> 48) == tag;
    if (ok || !FF) {
      if (!ok) atomicAdd(err + 1, 1);     // serial: the kernel boundary must have made every word current
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xs[xi(16 * t + 2 * i)] = unpack((uint32_t)v[i]);
        xs[xi(16 * t + 2 * i + 1)] = unpack((uint32_t)(v[i] >> 32));
      }
      return true;
    }
    if (spin >= max_spins) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void publish(uint32_t* Xn, int row, float y, uint32_t tag, bool ff) {
  const uint32_t w = pack(y, tag);
  if (ff) __hip_atomic_store((gu32*)(Xn + row), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else Xn[row] = w;
}

// one workgroup: bump the epoch (1..65535) and write x_0 with it
__global__ __launch_bounds__(256) void chain_init_kernel(uint32_t* epoch, uint32_t* X, const uint16_t* x0) {
  __shared__ uint32_t tag;
  if (threadIdx.x == 0) {
    tag = *epoch % 65535u + 1u;
    *epoch = tag;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += NT)
    __hip_atomic_store((gu32*)(X + i), (tag << 16) | x0[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one link; FF: poll the tagged input (after issuing the weight loads) and publish with agent-scope stores
template <bool FF>
__global__ __launch_bounds__(256) void chain_link_kernel(const u32x4* W, const float* scale, uint32_t* X, int link,
                                                        const uint32_t* epoch, long max_spins, int* err) {
  __shared__ float xs[XS];
  const int t = threadIdx.x, wg = blockIdx.x, r = t >> 4, c = t & 15;
  const uint32_t tag = *epoch;
  W8 w;
  load_w(w, W, link, wg, t);
  if (!stage_x<FF>(X + (size_t)link * D, tag, xs, t, max_spins, err)) atomicAdd(err, 1);
  __syncthreads();
  const float acc = dot_row(w, xs, c);
  if (c == 0) publish(X + (size_t)(link + 1) * D, RW * wg + r, acc * scale[(size_t)link * D + RW * wg + r], tag, FF);
}

// the whole chain in one launch (NWG co-resident workgroups). PF 0: weights loaded after the wait; 1: this link's
// weights issued before the wait; 2: the next link's weights issued before this link's wait (one link ahead)
template <int PF>
__global__ __launch_bounds__(256) void chain_persistent_kernel(const u32x4* W, const float* scale, uint32_t* X, int L,
                                                              const uint32_t* epoch, long max_spins, int* err) {
  __shared__ float xs[XS];
  __shared__ int s_dead;
  const int t = threadIdx.x, wg = blockIdx.x, r = t >> 4, c = t & 15;
  const uint32_t tag = *epoch;
  if (t == 0) s_dead = 0;
  W8 cur, nxt;
  if (PF == 2) load_w(cur, W, 0, wg, t);
  for (int l = 0; l < L; ++l) {
    if (PF == 1) load_w(cur, W, l, wg, t);
    if (PF == 2 && l + 1 < L) load_w(nxt, W, l + 1, wg, t);
    __syncthreads();    // the previous link's LDS reads are done; s_dead is current
    if (!s_dead && !stage_x<true>(X + (size_t)l * D, tag, xs, t, max_spins, err)) {
      atomicAdd(err, 1);
      s_dead = 1;       // stop waiting for the rest of this launch (keep publishing: the peers never stall on us)
    }
    __syncthreads();
    if (PF == 0) load_w(cur, W, l, wg, t);
    const float acc = dot_row(cur, xs, c);
    if (c == 0) publish(X + (size_t)(l + 1) * D, RW * wg + r, acc * scale[(size_t)l * D + RW * wg + r], tag, true);
    if (PF == 2) cur = nxt;
  }
}
}  // namespace

extern "C" {
int chain_dims(int* d) {
  d[0] = D; d[1] = NWG; d[2] = NJ; d[3] = NT;
  return 0;
}
int chain_init(void* epoch, void* X, const void* x0, void* stream) {
  chain_init_kernel<<<1, NT, 0, (hipStream_t)stream>>>((uint32_t*)epoch, (uint32_t*)X, (const uint16_t*)x0);
  return (int)hipGetLastError();
}
int chain_link(const void* W, const float* scale, void* X, int link, const void* epoch, int ff, long max_spins,
               int* err, void* stream) {
  if (ff)
    chain_link_kernel<true><<<NWG, NT, 0, (hipStream_t)stream>>>((const u32x4*)W, scale, (uint32_t*)X, link,
                                                                 (const uint32_t*)epoch, max_spins, err);
  else
    chain_link_kernel<false><<<NWG, NT, 0, (hipStream_t)stream>>>((const u32x4*)W, scale, (uint32_t*)X, link,
                                                                  (const uint32_t*)epoch, max_spins, err);
  return (int)hipGetLastError();
}
int chain_persistent(const void* W, const float* scale, void* X, int L, const void* epoch, int pf, long max_spins,
                     int* err, void* stream) {
  // every workgroup must be resident at once: one per CU at most is needed, check the device has NWG slots
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  hipError_t e;
  if (pf == 0) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_persistent_kernel<0>, NT, 0);
  else if (pf == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_persistent_kernel<1>, NT, 0);
  else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_persistent_kernel<2>, NT, 0);
  if (e != hipSuccess || (long)cus * per_cu < NWG) return -2;
  const u32x4* w = (const u32x4*)W;
  uint32_t* x = (uint32_t*)X;
  const uint32_t* ep = (const uint32_t*)epoch;
  hipStream_t s = (hipStream_t)stream;
  if (pf == 0) chain_persistent_kernel<0><<<NWG, NT, 0, s>>>(w, scale, x, L, ep, max_spins, err);
  else if (pf == 1) chain_persistent_kernel<1><<<NWG, NT, 0, s>>>(w, scale, x, L, ep, max_spins, err);
  else chain_persistent_kernel<2><<<NWG, NT, 0, s>>>(w, scale, x, L, ep, max_spins, err);
  return (int)hipGetLastError();
}
}
