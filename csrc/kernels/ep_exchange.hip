// Expert-parallel decode exchange (SURVEY.md §2G "EP all-to-all", BASELINE config 5), capturable in the decode
// hipGraph: every rank holds every token's hidden state (tensor-parallel attention), computes ITS experts' outputs
// for the (token, slot) rows routed to them, and this kernel pushes exactly those rows to every peer over the
// IPC-mapped receive buffers, then fills the rows the peers own from its own receive buffer -- so each rank ends
// with the full [T * k, d] expert output and runs the ordinary single-GPU weighted combine (slot order, fp32),
// bit-identical to TP = 1 and on every rank, with no all-reduce of [T, d] partials that are mostly zeros (EP8, top-2
// of 8: each rank owns ~1/4 of the rows; 7 x 16 KiB pushes per owned row instead of a 7 x 16 KiB all-reduce push
// per TOKEN). The routing is replicated (every rank ran the same router on the same hidden states), so a receiver
// knows which peer owns each row without any count exchange.
//
// Protocol: per-row flags carrying the full 32-bit call generation (no wrap-around aliasing), written by the owner
// after its row data has completed; the receiver polls the flag, then reads the row. Rows and flags are
// double-buffered by generation parity. Memory ordering across devices (xGMI) -- the rehearsals cannot exercise it,
// every "peer" is the same HBM:
//   * owner: row data by system-scope stores (write-through, nothing parked in this XCD's L2) -> every storing wave
//     `s_waitcnt vmcnt(0)` -> workgroup barrier -> ONE system-scope release fence (buffer_wbl2 sc0 sc1: anything the
//     stores left in L2 is written back before any flag) -> `s_waitcnt vmcnt(0)` in inline asm (the compiler may
//     drop its own after the write-back, MI355X_MICROARCH.md "Compiler hazard") -> barrier -> flag stores;
//   * receiver: ONE relaxed system-scope poll of the flag -> system-scope acquire fence (invalidates this CU's
//     caches: no row line read before the flag can be served stale) -> `s_waitcnt vmcnt(0)` -> barrier -> the row
//     by system-scope loads.
// The release / acquire pair is the Guideline-16 form extended to system scope; the system-scope stores and loads
// alone (round 5) relied on write-through ordering that is not architecturally promised across devices.
// Debug (NLS_EPX_CHECK=1, on in the EP rehearsal tests): the owner also publishes a checksum of each pushed row (a
// wrapping sum of its 32-bit words) before the flag; the receiver recomputes it over the words it read and raises
// the error word with code 2 on a mismatch -- a mixed or torn row on real xGMI fails the step instead of decoding. Generations are per workgroup of a FIXED grid (EPX_WGS): workgroup g owns rows g, g + G, ...
// in every call on every rank, so its counter advances in lock-step everywhere (hipGraph replays included). A
// workgroup pushes all of its rows before it polls for any, and the grid is small, so no poll can wait on work
// queued behind it (profiles/tp_oneshot_eager_r05.txt); ranks sharing one GPU shrink it (nls_epx_set_wgs). Polls
// are bounded: a timeout raises the error word of every rank (the engine reads it with each step's tokens) and the
// kernel exits.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nls_epx {

#define EPX_MAX_RANKS 8
#define EPX_THREADS 256
#define EPX_WGS 64

struct Peers {
  float* buf[EPX_MAX_RANKS];
};

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void st8(float* p, float2 v) {
  __hip_atomic_store((gu64*)p, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float2 ld8(const float* p) {
  const unsigned long long u = __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
}

// receive-buffer layout (floats / words): rows [2][cap][D] | flags [2][cap] | error word (+ 63 spare) | checksums [2][cap]
__host__ __device__ __forceinline__ size_t rows_words(int cap, int D) { return (size_t)2 * cap * D; }
__host__ __device__ __forceinline__ size_t err_word(int cap, int D) { return rows_words(cap, D) + (size_t)2 * cap; }
__host__ __device__ __forceinline__ size_t sum_words(int cap, int D) { return err_word(cap, D) + 64; }

// wrapping sum of a row's 32-bit words over the workgroup (order-independent: every thread's partial, then LDS)
__device__ __forceinline__ unsigned row_sum(unsigned part, unsigned* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = part;
  __syncthreads();
  unsigned t = 0u;
#pragma unroll
  for (int i = 0; i < EPX_THREADS / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(EPX_THREADS) void epx_kernel(float* __restrict__ y, long ldy, int n, int D,
                                                          const int* __restrict__ sel, int per, int rank, int world,
                                                          Peers P, int cap, unsigned* __restrict__ wg_gen,
                                                          int* __restrict__ err, long max_spins, int check) {
  __shared__ unsigned s_gen;
  __shared__ int s_ok;
  __shared__ unsigned s_red[EPX_THREADS / 64];
  const int g = blockIdx.x, G = gridDim.x;
  if (threadIdx.x == 0) s_gen = __hip_atomic_load((const gu32*)(wg_gen + g), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const unsigned gen = s_gen;
  const int par = (int)(gen & 1u);
  // 1) push the rows this rank's experts produced to every peer (+ the debug checksum of each)
  for (int j = g; j < n; j += G) {
    if (sel[j] / per != rank) continue;
    const float* src = y + (size_t)j * ldy;
    unsigned part = 0u;
    const int p0 = rank == 0 ? 1 : 0;                 // the checksum covers the words sent (to any one peer)
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      float* dst = P.buf[p] + ((size_t)par * cap + j) * D;
      for (int c = 2 * threadIdx.x; c < D; c += 2 * EPX_THREADS) {
        const float2 v = *reinterpret_cast<const float2*>(src + c);
        st8(dst + c, v);
        if (p == p0) part += __float_as_uint(v.x) + __float_as_uint(v.y);
      }
    }
    if (check) {
      const unsigned sum = row_sum(part, s_red);
      if (threadIdx.x == 0)
        for (int p = 0; p < world; ++p)
          if (p != rank)
            __hip_atomic_store((gu32*)(P.buf[p] + sum_words(cap, D)) + (size_t)par * cap + j, sum, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {     // one system-scope release for all of the workgroup's row stores, before any flag
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // ... then their flags (the data of every pushed row has completed and is released)
  for (int j = g + (int)threadIdx.x * G; j < n; j += G * EPX_THREADS) {
    if (sel[j] / per != rank) continue;
    for (int p = 0; p < world; ++p)
      if (p != rank)
        __hip_atomic_store((gu32*)(P.buf[p] + rows_words(cap, D)) + (size_t)par * cap + j, gen, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2) the rows the peers own: wait for each flag, then copy the row into y
  const float* mine = P.buf[rank];
  const unsigned* flags = reinterpret_cast<const unsigned*>(mine + rows_words(cap, D));
  bool failed = false, bad = false;
  for (int j = g; j < n; j += G) {
    if (sel[j] / per == rank) continue;
    if (threadIdx.x == 0) {
      long spins = 0;
      bool ok = false;
      if (!failed) {
        while (!(ok = __hip_atomic_load((const gu32*)(flags + (size_t)par * cap + j), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM) == gen) &&
               ++spins < max_spins)
          __builtin_amdgcn_s_sleep(2);
        if (ok) {                 // acquire: nothing of the row may be served from before the flag
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      s_ok = ok;
    }
    __syncthreads();
    if (s_ok) {
      const float* src = mine + ((size_t)par * cap + j) * D;
      float* dst = y + (size_t)j * ldy;
      unsigned part = 0u;
      for (int c = 2 * threadIdx.x; c < D; c += 2 * EPX_THREADS) {
        const float2 v = ld8(src + c);
        *reinterpret_cast<float2*>(dst + c) = v;
        part += __float_as_uint(v.x) + __float_as_uint(v.y);
      }
      if (check) {
        const unsigned got = row_sum(part, s_red);
        const unsigned want = __hip_atomic_load((const gu32*)(mine + sum_words(cap, D)) + (size_t)par * cap + j,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (got != want) bad = true;
      }
    } else {
      failed = true;
    }
    __syncthreads();     // s_ok is reused by the next row
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store((gu32*)(wg_gen + g), gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (failed || bad) {      // 1: a poll timed out; 2: a received row failed its checksum (NLS_EPX_CHECK)
      const unsigned code = failed ? 1u : 2u;
      atomicMax(err, (int)code);
      for (int p = 0; p < world; ++p)
        __hip_atomic_store((gu32*)(P.buf[p] + err_word(cap, D)), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace nls_epx

// workgroups of the exchange grid: EPX_WGS, fewer when several ranks share one GPU (nls_epx_set_wgs, the same value on
// every rank before the first call: a workgroup's generation counter follows its row set g, g + G, ...)
static int g_epx_wgs = EPX_WGS;

extern "C" {

int nls_epx_set_wgs(int n) {
  if (n < 1 || n > EPX_WGS) return -1;
  g_epx_wgs = n;
  return 0;
}

// bytes of one rank's receive buffer for up to `cap` rows of D floats (rows, flags, error word, checksums)
long nls_epx_bytes(int cap, int D) { return (long)(nls_epx::sum_words(cap, D) + 2L * cap) * 4L; }

int nls_epx_wgs() { return EPX_WGS; }     // generation counters to allocate (the largest grid)

// zero the flags and the error word of a freshly allocated (or reset) receive buffer
int nls_epx_init(void* buf, int cap, int D, void* stream) {
  return (int)hipMemsetAsync((float*)buf + nls_epx::rows_words(cap, D), 0, (size_t)(2 * cap + 64) * 4,
                             (hipStream_t)stream);
}

// y [n, ldy] f32: rows j with sel[j] / per == rank are this rank's (pushed), the others are filled from the peers
int nls_epx_run(void* y, long ldy, int n, int D, const int* sel, int per, int rank, int world, void* const* peers,
                int cap, unsigned* wg_gen, int* err, long max_spins, int check, void* stream) {
  if (world < 2 || world > EPX_MAX_RANKS || rank < 0 || rank >= world || n < 0 || n > cap || D % 2 || ldy % 2 ||
      per < 1)
    return -1;
  if (n == 0) return 0;
  nls_epx::Peers P;
  for (int i = 0; i < EPX_MAX_RANKS; ++i) P.buf[i] = i < world ? (float*)peers[i] : nullptr;
  hipLaunchKernelGGL(nls_epx::epx_kernel, dim3(g_epx_wgs), dim3(EPX_THREADS), 0, (hipStream_t)stream, (float*)y, ldy, n,
                     D, sel, per, rank, world, P, cap, wg_gen, err, max_spins, check);
  return (int)hipGetLastError();
}

int nls_epx_err_clear(void* buf, int cap, int D, void* stream) {
  return (int)hipMemsetAsync((float*)buf + nls_epx::err_word(cap, D), 0, 4, (hipStream_t)stream);
}

int nls_epx_err_fetch(void* buf, int cap, int D, void* host, void* stream) {
  return (int)hipMemcpyAsync(host, (float*)buf + nls_epx::err_word(cap, D), 4, hipMemcpyDeviceToHost,
                             (hipStream_t)stream);
}

}  // extern "C"
