// One-shot small-message all-reduce over peer-mapped (IPC) device memory -- the decode-size
// (8-64 KiB .. 1 MiB) row-parallel reduction of tensor-parallel layers.
//
// xGMI is point-to-point (7 links per GPU), so instead of a ring (2*(N-1) latency hops) every
// rank pushes its whole message to every peer at once (N-1 links in parallel), then sums the N
// slices locally in RANK ORDER, so every rank gets a bit-identical result (the replicated residual
// stream never drifts between shards).
//
// Synchronisation is carried by the data itself: each fp32 value travels as one 8-byte granule
// {epoch:32 | bits:32} written with ONE system-scope atomic store; the consumer polls its granules
// with system-scope atomic loads until every tag equals the current epoch. No flags, no fences,
// no ordering between payload and signal to get wrong. Receive buffers are uncached device memory
// (hipDeviceMallocUncached), so polls always observe HBM.
//
// Double-buffered by epoch parity: a rank can be at most one call ahead of any peer (it cannot
// finish call c+1 without every peer's call-c+1 data, which a peer writes only after finishing c).
// The grid is FIXED (AR_BLOCKS x AR_THREADS, grid-stride), so element -> block is the same on every
// call and per-block epoch counters (local memory, advanced by the block itself) stay in lock-step
// across ranks and across hipGraph replays (no per-launch argument is frozen into a graph).
// Spins are bounded: on timeout the block records an error code and exits (never hangs the GPU).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AR_MAX_RANKS 8
#define AR_BLOCKS 32
#define AR_THREADS 512

struct ArPeers {
  unsigned long long* buf[AR_MAX_RANKS];
};

__device__ __forceinline__ void st_sys(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sys(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(AR_THREADS) void oneshot_ar_kernel(float* __restrict__ data, long n, ArPeers P,
                                                                 int world, int rank, long cap,
                                                                 unsigned* __restrict__ epochs,
                                                                 int* __restrict__ err, long max_spins) {
  __shared__ unsigned s_ep;
  __shared__ int s_fail;
  if (threadIdx.x == 0) {
    s_ep = epochs[blockIdx.x] + 1u;
    if (s_ep == 0u) s_ep = 1u;  // epoch 0 is the zero-initialised (never written) tag
    s_fail = 0;
  }
  __syncthreads();
  const unsigned ep = s_ep;
  const int par = (int)(ep & 1u);
  const long stride = (long)AR_BLOCKS * AR_THREADS;
  // 1) push: my value -> slot [par][rank] of every peer (one 8-byte atomic granule per value)
  for (long i = (long)blockIdx.x * AR_THREADS + threadIdx.x; i < n; i += stride) {
    const unsigned long long g = ((unsigned long long)ep << 32) | __float_as_uint(data[i]);
    for (int p = 0; p < world; ++p)
      if (p != rank) st_sys(P.buf[p] + ((long)(par * world + rank)) * cap + i, g);
  }
  // 2) gather + reduce in rank order (bit-identical on every rank)
  unsigned long long* mine = P.buf[rank];
  bool failed = false;  // after one timeout, stop waiting (the error code is already recorded)
  for (long i = (long)blockIdx.x * AR_THREADS + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int p = 0; p < world; ++p) {
      float v;
      if (p == rank) {
        v = data[i];
      } else {
        unsigned long long* src = mine + ((long)(par * world + p)) * cap + i;
        unsigned long long x = ld_sys(src);
        long spins = 0;
        while (!failed && (unsigned)(x >> 32) != ep) {
          if (++spins > max_spins) {
            failed = true;
            s_fail = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          x = ld_sys(src);
        }
        v = __uint_as_float((unsigned)(x & 0xFFFFFFFFull));
      }
      acc += v;
    }
    data[i] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    epochs[blockIdx.x] = ep;
    if (s_fail) atomicExch(err, 1);
  }
}

// Fused row-parallel epilogue for tensor-parallel decode: x[b] += sum_r part_r[b] (rank order, one-shot
// over the same IPC buffers), then h[b] = f16(rmsnorm(x[b]) * w) -- the all-reduce, the residual add and
// the NEXT layer's input RMSNorm in one launch (vs all-reduce + norm launches; the residual row is read
// and written once). One block per activation row; each block keeps its own epoch (all TP ranks replay
// the same launches with the same row count, so block b's epoch advances in lock-step on every rank).
// Receive slots: [parity][rank][row < rowcap][D] granules inside the same peer buffers.
#define ARN_MAXV 16     // D <= ARN_MAXV * AR_THREADS elements per row kept in registers
__global__ __launch_bounds__(AR_THREADS) void oneshot_ar_addnorm_kernel(
    const float* __restrict__ part, long ldp, float* __restrict__ x, long ldx, const float* __restrict__ nw,
    _Float16* __restrict__ h, long ldh, int D, float eps, ArPeers P, int world, int rank, long rowcap,
    unsigned* __restrict__ epochs, int* __restrict__ err, long max_spins, long sp, long sx, long sh, long se) {
  __shared__ unsigned s_ep;
  __shared__ int s_fail;
  __shared__ float s_red[AR_THREADS / 64];
  const int b = blockIdx.x;
  if (gridDim.y > 1) {
    // single-GPU simulation: ALL ranks in one grid (blockIdx.y = rank, per-rank operand strides), so
    // the ranks' blocks are co-scheduled by construction (separate streams may share a hardware queue)
    rank = blockIdx.y;
    part += rank * sp;
    x += rank * sx;
    h += rank * sh;
    epochs += rank * se;
  }
  if (threadIdx.x == 0) {
    s_ep = epochs[b] + 1u;
    if (s_ep == 0u) s_ep = 1u;
    s_fail = 0;
  }
  __syncthreads();
  const unsigned ep = s_ep;
  const int par = (int)(ep & 1u);
  const float* pr = part + (size_t)b * ldp;
  // 1) push this rank's partial row to every peer
  for (int i = threadIdx.x; i < D; i += AR_THREADS) {
    const unsigned long long g = ((unsigned long long)ep << 32) | __float_as_uint(pr[i]);
    for (int p = 0; p < world; ++p)
      if (p != rank) st_sys(P.buf[p] + (((long)(par * world + rank)) * rowcap + b) * D + i, g);
  }
  // 2) rank-ordered sum + residual add (bit-identical on every rank), sum of squares in registers
  unsigned long long* mine = P.buf[rank];
  float xr[ARN_MAXV];
  float ss = 0.f;
  bool failed = false;
#pragma unroll
  for (int j = 0; j < ARN_MAXV; ++j) {
    const int i = threadIdx.x + j * AR_THREADS;
    xr[j] = 0.f;
    if (i >= D) continue;
    float acc = 0.f;
    for (int p = 0; p < world; ++p) {
      float v;
      if (p == rank) {
        v = pr[i];
      } else {
        unsigned long long* src = mine + (((long)(par * world + p)) * rowcap + b) * D + i;
        unsigned long long g = ld_sys(src);
        long spins = 0;
        while (!failed && (unsigned)(g >> 32) != ep) {
          if (++spins > max_spins) {
            failed = true;
            s_fail = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          g = ld_sys(src);
        }
        v = __uint_as_float((unsigned)(g & 0xFFFFFFFFull));
      }
      acc += v;
    }
    const float xi = x[(size_t)b * ldx + i] + acc;
    x[(size_t)b * ldx + i] = xi;
    xr[j] = xi;
    ss += xi * xi;
  }
  // 3) RMSNorm of the updated row
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < AR_THREADS / 64; ++w) tot += s_red[w];
  const float inv = rsqrtf(tot / (float)D + eps);
#pragma unroll
  for (int j = 0; j < ARN_MAXV; ++j) {
    const int i = threadIdx.x + j * AR_THREADS;
    if (i < D) h[(size_t)b * ldh + i] = (_Float16)(xr[j] * inv * nw[i]);
  }
  if (threadIdx.x == 0) {
    epochs[b] = ep;
    if (s_fail) atomicExch(err, 1);
  }
}

extern "C" {

// bytes of one rank's receive buffer for messages of up to `cap` floats
long nls_ar_buffer_bytes(long cap, int world) { return 2L * world * cap * 8L; }

int nls_ar_alloc(long cap, int world, void** buf, void* ipc_handle /* hipIpcMemHandle_t, 64 B */) {
  if (world < 1 || world > AR_MAX_RANKS) return -1;
  size_t bytes = (size_t)nls_ar_buffer_bytes(cap, world);
  hipError_t e = hipExtMallocWithFlags(buf, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*buf, 0, bytes);
  if (e != hipSuccess) return (int)e;
  if (ipc_handle) {
    e = hipIpcGetMemHandle((hipIpcMemHandle_t*)ipc_handle, *buf);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

int nls_ar_open(const void* ipc_handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, ipc_handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int nls_ar_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int nls_ar_free(void* ptr) { return (int)hipFree(ptr); }

int nls_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

int nls_ar_blocks() { return AR_BLOCKS; }

int nls_ar_addnorm_sim(const float*, long, float*, long, const float*, void*, long, int, int, float, void* const*, int,
                       int, long, unsigned*, int*, long, void*, int, long, long, long, long);

// rows x D fused all-reduce + residual + RMSNorm; rows * D <= cap / 1 (the same buffers), `epochs` holds
// one counter per row block (>= rowcap entries)
int nls_ar_addnorm(const float* part, long ldp, float* x, long ldx, const float* nw, void* h, long ldh, int rows,
                   int D, float eps, void* const* peers, int world, int rank, long cap, unsigned* epochs, int* err,
                   long max_spins, void* stream) {
  return nls_ar_addnorm_sim(part, ldp, x, ldx, nw, h, ldh, rows, D, eps, peers, world, rank, cap, epochs, err,
                            max_spins, stream, 0, 0, 0, 0, 0);
}

// sim_ranks > 1: every rank in one launch (rank r's operands at base + r * stride) -- SimulatedGroup
int nls_ar_addnorm_sim(const float* part, long ldp, float* x, long ldx, const float* nw, void* h, long ldh, int rows,
                       int D, float eps, void* const* peers, int world, int rank, long cap, unsigned* epochs, int* err,
                       long max_spins, void* stream, int sim_ranks, long sp, long sx, long sh, long se) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || rows < 1 || D < 1 ||
      D > ARN_MAXV * AR_THREADS)
    return -1;
  const long rowcap = cap / D;
  if (rows > rowcap) return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (unsigned long long*)peers[i] : nullptr;
  if (sim_ranks > 1 && sim_ranks != world) return -1;
  hipLaunchKernelGGL(oneshot_ar_addnorm_kernel, dim3(rows, sim_ranks > 1 ? sim_ranks : 1), dim3(AR_THREADS), 0,
                     (hipStream_t)stream, part, ldp, x, ldx, nw, (_Float16*)h, ldh, D, eps, P, world, rank, rowcap,
                     epochs, err, max_spins, sp, sx, sh, se);
  return (int)hipGetLastError();
}

int nls_ar_run(float* data, long n, void* const* peers, int world, int rank, long cap, unsigned* epochs,
               int* err, long max_spins, void* stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n > cap) return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (unsigned long long*)peers[i] : nullptr;
  hipLaunchKernelGGL(oneshot_ar_kernel, dim3(AR_BLOCKS), dim3(AR_THREADS), 0, (hipStream_t)stream, data, n, P,
                     world, rank, cap, epochs, err, max_spins);
  return (int)hipGetLastError();
}

}  // extern "C"
