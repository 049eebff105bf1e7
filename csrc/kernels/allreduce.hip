// One-shot small-message all-reduce over peer-mapped (IPC) device memory -- the decode-size
// (8-64 KiB .. 1 MiB) row-parallel reduction of tensor-parallel layers.
//
// xGMI is point-to-point (7 links per GPU), so instead of a ring (2*(N-1) latency hops) every
// rank pushes its whole message to every peer at once (N-1 links in parallel), then sums the N
// slices locally in RANK ORDER, so every rank gets a bit-identical result (the replicated residual
// stream never drifts between shards).
//
// Synchronisation is carried by the data itself, 4 bytes per value: each fp32 travels with its two
// low mantissa bits replaced by a 2-bit epoch tag (value rounded to 30 bits: relative error <= 2^-22)
// and the consumer polls until every dword of a 16-byte load carries the current tag. A naturally
// aligned dword is written and read atomically, so a 16-byte store that reaches the peer in pieces
// is still checked dword by dword: no flags, no fences, no payload/signal ordering to get wrong.
// Receive buffers are uncached device memory (hipDeviceMallocUncached): polls always observe HBM.
//
// Why a 2-bit tag suffices: slots are double-buffered by epoch parity and a rank can be at most one
// call ahead of any peer (it cannot finish call c+1 without every peer's call-c+1 data, which a peer
// writes only after finishing c). Epochs are kept per SLOT BLOCK (per row slice in the fused add+norm)
// and a call writes every granule of every block it advances, so at epoch e a slot holds the peer's
// epoch e - 2 granule or its epoch e granule -- a skipped block keeps its epoch too. The plain all-reduce and
// the gather never write their own receive slots (see SlotBlocks below), nor does the fused add+norm by default.
// (Rounds 3-5 re-tagged each consumed granule with the other parity's tag, AR_OPT_RETAG, because the simulated-rank
// test failed without it. The cause, found in round 6, was elsewhere: the row's normaliser read the other slices'
// x with PLAIN loads after a one-thread agent-scope acquire, and such a load can still return a pre-add copy of the
// slice -- "x exact (memory is right), h wrong (normalised from a stale read)". The normaliser now reads x with
// agent-scope loads (wt_load4, sc1): with the re-tag off the test passes with them and fails with plain reads, the
// r05 failure reproduced on demand (profiles/ar_retag_cause_r06.txt). NLS_AR_RETAG=1 restores the re-tag.)
// Eager (non-captured) calls timed out in rounds 3-4 on two ranks sharing ONE GPU: the fused add+norm launched one
// workgroup per (row, slice), its polling waves filled the GPU and the PEER rank's preceding kernels could not be
// scheduled until the poll expired (device-clock timestamps of both ranks, profiles/tp_oneshot_eager_r05.txt). The
// add+norm now runs on a bounded grid (every workgroup pushes all of its items before polling), and eager calls
// take these kernels again (parallel/comm.py).
// Every rank uses the ROUNDED value of its own partial too, so the sums stay bit-identical.
//
// Element -> workgroup maps are fixed (the plain all-reduce runs a FIXED grid, grid-stride; the
// fused add+norm maps row b, 256-column slice c to a workgroup on XCD b % 8 for a given D), so the per-
// workgroup epoch counters (device memory, advanced by the workgroup itself) stay in lock-step
// across ranks and across hipGraph replays (no per-launch argument is frozen into a graph).
// Spins are bounded: on timeout a workgroup raises the error word of EVERY rank (an extra 256-byte
// area after the receive slots, written over xGMI) and its own, then exits -- never hangs the GPU;
// the engine reads its error word after each decode step and fails the step's requests.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define AR_MAX_RANKS 8
#define AR_BLOCKS 32
#define AR_THREADS 512
#define ARN_THREADS 64          // fused add+norm: one wave per 256-column slice
#define ARN_VPB (ARN_THREADS * 4)
#define AR_ERR_BYTES 256

struct ArPeers {
  uint32_t* buf[AR_MAX_RANKS];
};

__device__ __forceinline__ uint32_t ar_pack(float v, uint32_t tag) {
  return ((__float_as_uint(v) + 2u) & ~3u) | tag;     // round to 30 bits, tag in the low 2
}
__device__ __forceinline__ float ar_val(uint32_t g) { return __uint_as_float(g & ~3u); }
__device__ __forceinline__ bool ar_tagged(uint4 g, uint32_t tag) {
  return ((g.x & 3u) == tag) & ((g.y & 3u) == tag) & ((g.z & 3u) == tag) & ((g.w & 3u) == tag);
}
__device__ __forceinline__ uint4 ar_pack4(float4 v, uint32_t tag) {
  return make_uint4(ar_pack(v.x, tag), ar_pack(v.y, tag), ar_pack(v.z, tag), ar_pack(v.w, tag));
}
__device__ __forceinline__ float4 ar_val4(uint4 g) {
  return make_float4(ar_val(g.x), ar_val(g.y), ar_val(g.z), ar_val(g.w));
}

// Every word another workgroup or another rank reads goes through GLOBAL (address space 1) atomic accesses
// with an explicit scope -- never flat, never plain (cdna_hip_programming.md Guideline 16 recipe; round 3
// used flat `volatile` accesses, and a granule pushed through the peer's IPC mapping could stay invisible to
// the owner's poll: 2-process rehearsal, round 4). A 16-byte granule is two 8-byte halves; every dword
// carries the tag, so a torn granule just fails the tag check until both halves have landed.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void ar_store(uint32_t* p, uint4 g) {
  gu64* q = (gu64*)p;
  __hip_atomic_store(q, ((unsigned long long)g.y << 32) | g.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 1, ((unsigned long long)g.w << 32) | g.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint4 ar_load(const uint32_t* p) {
  const gu64* q = (const gu64*)p;
  const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}
// the same granule read by a read-modify-write (OR 0): performed where the memory's atomics are
// performed, never answered from a cache line of this CU's or this XCD's hierarchy
__device__ __forceinline__ uint4 ar_load_rmw(const uint32_t* p) {
  gu64* q = (gu64*)p;
  const unsigned long long a = __hip_atomic_fetch_or(q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long b = __hip_atomic_fetch_or(q + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}
__device__ __forceinline__ uint32_t xcc_id() {
  // HW_REG_XCC_ID (hwreg 20), bits [3:0]: the XCD this wave runs on (diagnostics only)
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
}
// a float4 other workgroups of this launch read (the residual slice of the fused add+norm): write-through
__device__ __forceinline__ void wt_store4(float* p, float4 v) {
  gu64* q = (gu64*)p;
  __hip_atomic_store(q, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ... and its reader: agent-scope loads (sc1: no L1, no stale line of this XCD from before the write)
__device__ __forceinline__ float4 wt_load4(const float* p) {
  const gu64* q = (const gu64*)p;
  const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)), __uint_as_float((uint32_t)b),
                     __uint_as_float((uint32_t)(b >> 32)));
}

// this rank's error word and the peers' (after the 2 x world x cap receive slots)
__device__ __forceinline__ uint32_t* ar_err_word(uint32_t* buf, int world, long cap) {
  return buf + 2L * world * cap;
}
__device__ void ar_raise(const ArPeers& P, int world, long cap, int* err) {
  atomicExch(err, 1);
  for (int p = 0; p < world; ++p)
    __hip_atomic_store((gu32*)ar_err_word(P.buf[p], world, cap), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// per-workgroup epoch counters: read / advanced with `sc0 sc1` (volatile) accesses, never through a possibly
// stale line of another XCD's L2 -- a counter's workgroup need not run on the same XCD from one launch to the
// next (the fused add+norm's grid depends on the row count, and hipGraph replays alternate with eager calls)
__device__ __forceinline__ unsigned ep_load(const unsigned* p) {
  return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ep_store(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// read-modify-write forms (AR_OPT_EP_RMW): the counter word is never answered from a cache line
__device__ __forceinline__ unsigned ep_load_rmw(unsigned* p) {
  return __hip_atomic_fetch_add((gu32*)p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ep_store_rmw(unsigned* p, unsigned v) {
  __hip_atomic_exchange((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// diagnostics of the first timed-out poll of a buffer set: words 1..7 of this rank's error area (a, b, epoch,
// peer, the first dword seen -- its tag is the low 2 bits --, a marker, the kernel: 1 sum, 2 add+norm,
// 3 gather, 4 arg-max), read back by OneShotAllReduce.debug_state
__device__ void ar_diag(uint32_t* mine, int world, long cap, int kid, long a, long b, unsigned ep, int peer,
                        uint32_t seen) {
  uint32_t* dw = ar_err_word(mine, world, cap);
  if (atomicCAS(dw + 6, 0u, 0xA11u) == 0u) {
    dw[1] = (uint32_t)a;
    dw[2] = (uint32_t)b;
    dw[3] = ep;
    dw[4] = (uint32_t)peer;
    dw[5] = seen;
    dw[7] = (uint32_t)kid;
  }
}

// more of the first add+norm timeout (words 8..18, written by the lane that recorded words 1..7): the four
// dwords its last poll saw, its lane's column, its XCD, the epoch counter as read again at the timeout, and the
// granule as an atomic read-modify-write sees it (memory's view, no cache line in between)
__device__ void ar_diag2(uint32_t* mine, int world, long cap, uint4 seen, uint32_t col, unsigned ep_now, uint4 rmw) {
  uint32_t* dw = ar_err_word(mine, world, cap);
  if (atomicCAS(dw + 19, 0u, 0xB22u) == 0u) {
    dw[8] = seen.x;
    dw[9] = seen.y;
    dw[10] = seen.z;
    dw[11] = seen.w;
    dw[12] = col;
    dw[13] = xcc_id();
    dw[14] = ep_now;
    dw[15] = rmw.x;
    dw[16] = rmw.y;
    dw[17] = rmw.z;
    dw[18] = rmw.w;
  }
}

// launch-option bits carried above the spin budget (host: ar_opts(), env NLS_AR_POLL_INV / NLS_AR_RETAG)
constexpr long AR_OPT_POLL_INV = 1L << 62;    // system-scope acquire (L2 invalidate) before every re-poll
constexpr long AR_OPT_RETAG = 1L << 61;       // fused add+norm: re-tag consumed granules (rounds 3-5; off by default)
constexpr long AR_OPT_EP_RMW = 1L << 60;      // epoch counters read / written by atomic read-modify-writes
constexpr long AR_OPT_POLL_RMW = 1L << 59;    // peer granules polled by atomic read-modify-writes (OR 0)
constexpr long AR_OPT_PROBE = 1L << 58;       // fused add+norm: read every push back (RMW) and log a mismatch
constexpr long AR_OPT_XCHECK = 1L << 57;      // fused add+norm: the row's normaliser re-sums x^2 from the x it reads
                                              // and logs a disagreement with the slices' shares (words 32..39)
constexpr long AR_OPT_XPLAIN = 1L << 56;      // fused add+norm: the normaliser reads x with plain loads (round-5 form)
constexpr long AR_SPIN_MASK = (1L << 48) - 1;

__device__ __forceinline__ unsigned ep_get(unsigned* p, long opts) {
  return (opts & AR_OPT_EP_RMW) ? ep_load_rmw(p) : ep_load(p);
}
__device__ __forceinline__ void ep_put(unsigned* p, unsigned v, long opts) {
  if (opts & AR_OPT_EP_RMW)
    ep_store_rmw(p, v);
  else
    ep_store(p, v);
}

// poll one 16-byte granule of peer data until every dword carries `tag` (bounded)
__device__ __forceinline__ uint4 ar_poll(const uint32_t* src, uint32_t tag, long max_spins, bool& failed) {
  const bool rmw = max_spins & AR_OPT_POLL_RMW;
  uint4 g = rmw ? ar_load_rmw(src) : ar_load(src);
  long spins = 0;
  const long budget = max_spins & AR_SPIN_MASK;
  while (!failed && !ar_tagged(g, tag)) {
    if (++spins > budget) {
      failed = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
    if (max_spins & AR_OPT_POLL_INV) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    g = rmw ? ar_load_rmw(src) : ar_load(src);
  }
  return g;
}

// ---------------------------------------------------------------------------------------------
// Epochs per SLOT BLOCK, full coverage, no consumed-tag rewrite. The receive slots of a grid-stride
// collective are cut into fixed blocks of BLK granules; a call advances the epoch of every block that
// overlaps its message and writes ALL granules of those blocks (the tail past the message carries a
// dummy payload with the current tag), so at epoch e a slot of a block holds the peer's epoch e - 2
// granule (tag (e - 2) & 3) or its epoch e granule, whatever the message sizes of the calls in between.
// Round 3 re-tagged each consumed granule instead (the consumer's own store into its receive slot), and
// on one GPU shared by two ranks an eager call after decode-graph replays could read that rewrite back
// instead of the peer's newer granule (2-process rehearsal, round 4). Block b belongs to workgroup
// b % gridDim.x in every call (fixed grids), which keeps its epoch counter's reads and writes ordered.
template <int BLK>
struct SlotBlocks {
  long nb;                     // blocks of this call
  int first, step, mine;       // this workgroup's blocks: first, first + step, ... (mine of them)
  __device__ SlotBlocks(long granules) {
    nb = (granules + BLK - 1) / BLK;
    first = blockIdx.x;
    step = gridDim.x;
    mine = nb > first ? (int)((nb - 1 - first) / step + 1) : 0;
  }
};
constexpr int AR_MAX_WG_BLOCKS = 64;   // slot blocks per workgroup at the largest message (host-checked)

// this workgroup's block epochs -> LDS (advanced by one: the epoch of THIS call)
__device__ __forceinline__ void blocks_begin(unsigned* epochs, int first, int step, int mine, unsigned* s_ep,
                                             long opts) {
  for (int j = threadIdx.x; j < mine; j += blockDim.x) s_ep[j] = ep_get(epochs + first + (long)j * step, opts) + 1u;
  __syncthreads();
}
__device__ __forceinline__ void blocks_end(unsigned* epochs, int first, int step, int mine, const unsigned* s_ep,
                                           long opts) {
  __syncthreads();
  for (int j = threadIdx.x; j < mine; j += blockDim.x) ep_put(epochs + first + (long)j * step, s_ep[j], opts);
}

// plain all-reduce (MoE expert outputs, generic decode-size sums): fixed grid, slot blocks of
// AR_THREADS granules (16 B, n % 4 == 0), data reduced in place
__global__ __launch_bounds__(AR_THREADS) void oneshot_ar_kernel(float* __restrict__ data, long n, ArPeers P,
                                                                 int world, int rank, long cap,
                                                                 unsigned* __restrict__ epochs,
                                                                 int* __restrict__ err, long max_spins) {
  __shared__ unsigned s_ep[AR_MAX_WG_BLOCKS];
  __shared__ int s_fail;
  const long n4 = n >> 2;
  const SlotBlocks<AR_THREADS> B(n4);
  if (threadIdx.x == 0) s_fail = 0;
  blocks_begin(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  // 1) push: my (rounded, tagged) values -> slot [par][rank] of every peer, 16 B per lane
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const long i = ((long)B.first + (long)j * B.step) * AR_THREADS + threadIdx.x;
    const float4 d = i < n4 ? reinterpret_cast<const float4*>(data)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const uint4 g = ar_pack4(d, ep & 3u);
    for (int p = 0; p < world; ++p)
      if (p != rank) ar_store(P.buf[p] + ((long)((ep & 1u) * world + rank)) * cap + 4 * i, g);
  }
  // 2) gather + reduce in rank order (bit-identical on every rank)
  uint32_t* mine = P.buf[rank];
  bool failed = false;   // after one timeout, stop waiting (the error word is raised below)
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const uint32_t tag = ep & 3u;
    const long i = ((long)B.first + (long)j * B.step) * AR_THREADS + threadIdx.x;
    const float4 d = i < n4 ? reinterpret_cast<const float4*>(data)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 own = ar_val4(ar_pack4(d, tag));
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < world; ++p) {
      float4 v = own;
      if (p != rank) {
        const bool was = failed;
        const uint4 gv = ar_poll(mine + ((long)((ep & 1u) * world + p)) * cap + 4 * i, tag, max_spins, failed);
        if (failed && !was) ar_diag(mine, world, cap, 1, i, n4, ep, p, gv.x);
        v = ar_val4(gv);
      }
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (i < n4) reinterpret_cast<float4*>(data)[i] = acc;
  }
  if (failed) s_fail = 1;
  blocks_end(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  if (threadIdx.x == 0 && s_fail) ar_raise(P, world, cap, err);
}

// ---------------------------------------------------------------------------------------------
// Fused row-parallel epilogue for tensor-parallel decode: x[b] += sum_r part_r[b] (rank order, one-shot
// over the same IPC buffers), then h[b] = f16(rmsnorm(x[b]) * w) -- the all-reduce, the residual add and
// the NEXT layer's input RMSNorm in one launch. Workgroup (b, c) moves row b's 256-column slice c
// (a 70B row of 8192 columns is spread over 32 workgroups, so at batch 1 the 7 x 32 KiB of pushes and
// polls run on 32 CUs), adds it into the residual and leaves its share of sum(x^2); the slice that
// arrives last at the row's ticket (agent-scope release / acquire, cdna_hip_programming.md Guideline
// 16) sums the shares and normalises the whole row. Receive slots: [parity][rank][cap], row b at b * D.
// NLS_AR_PROBE timing history of the fused add+norm (this process's launches only): per workgroup slot eidx, the
// last AR_PROBE_DEPTH (32) epochs as {epoch, xcc, t_start, t_pushed, t_polled} on the device-wide 100 MHz clock (wall_clock64), which
// two ranks sharing one GPU read identically -- a timed-out poll is placed against the peer's push of that epoch
#define AR_PROBE_SLOTS 4096
#define AR_PROBE_DEPTH 32
struct ArProbeRec {
  unsigned ep, xcc;
  unsigned long long t0, t1, t2;
};
__device__ ArProbeRec g_ar_probe[AR_PROBE_SLOTS * AR_PROBE_DEPTH];

// Items (row-rank rr, slice c) of one launch: rows rr = xcd + 8 m sit on XCD xcd (their tickets, shares and
// residual slices stay inside one L2: a row spread over XCDs normalised with stale shares, round 4); the k
// workgroups of an XCD take items m * nblk + c = j, j + k, ...
struct AnItem {
  int rr, c;
};
__device__ __forceinline__ AnItem an_item(int xcd, int k, int j, int t, int nblk) {
  const int idx = j + t * k;
  return AnItem{xcd + 8 * (idx / nblk), idx % nblk};
}

// Bounded grid (round 5): a launch has at most nls_ar_norm_wgs() workgroups (default 128, NLS_AR_NORM_WGS), each
// pushing ALL of its items before it polls for any. One workgroup per item (rows x D/256 of them) put 1,664
// polling waves on the GPU for a 52-row eager prefill chunk at D=8192; on one MI355X shared by two ranks the
// PEER rank's preceding GEMM could then not be scheduled, its push came only after the owner's bounded poll had
// expired (device-clock timestamps of both ranks, profiles/tp_oneshot_eager_r05.txt) -- the eager timeout of
// rounds 3-4. Half the CUs at most now wait in this kernel.
#define ARN_MAX_ITEMS 64
__global__ __launch_bounds__(ARN_THREADS) void oneshot_ar_addnorm_kernel(
    const float* __restrict__ part0, long ldp, float* __restrict__ x0, long ldx, const float* __restrict__ nw,
    _Float16* __restrict__ h0, long ldh, int D, float eps, ArPeers P, int world, int rank0, long cap,
    unsigned* __restrict__ epochs0, int* __restrict__ tickets0, float* __restrict__ ssq0, int* __restrict__ err,
    long max_spins, int sim, long sp, long sx, long sh, long se, long st, long sq, int nblk, int nrr) {
  __shared__ unsigned s_ep[ARN_MAX_ITEMS];
  __shared__ int s_last;
  const int L = blockIdx.x, xcd = L & 7, j = L >> 3, k = gridDim.x >> 3;
  const int mx = nrr > xcd ? (nrr - xcd + 7) / 8 : 0;           // rows of this XCD
  const int nit = mx * nblk > j ? (mx * nblk - 1 - j) / k + 1 : 0;  // items of this workgroup (<= ARN_MAX_ITEMS)
  if (nit == 0) return;
  const bool probe_on = (max_spins & AR_OPT_PROBE) && sim == 1;
  const unsigned long long t0 = probe_on ? (unsigned long long)wall_clock64() : 0ull;
  // the epochs of this call, one per item (a slice's counter is only ever touched by its own item)
  for (int t = threadIdx.x; t < nit; t += ARN_THREADS) {
    const AnItem it = an_item(xcd, k, j, t, nblk);
    const int r = sim > 1 ? it.rr % sim : 0, b = sim > 1 ? it.rr / sim : it.rr;
    s_ep[t] = ep_get(epochs0 + r * se + b * nblk + it.c, max_spins) + 1u;
  }
  __syncthreads();
  // 1) push: every item's partial slice to every peer
  for (int t = 0; t < nit; ++t) {
    const AnItem it = an_item(xcd, k, j, t, nblk);
    const int rank = sim > 1 ? it.rr % sim : rank0, b = sim > 1 ? it.rr / sim : it.rr;
    const float* part = part0 + (sim > 1 ? rank * sp : 0);
    const unsigned ep = s_ep[t];
    const int par = (int)(ep & 1u), col = it.c * ARN_VPB + 4 * threadIdx.x;
    if (col >= D) continue;
    const uint4 g = ar_pack4(*reinterpret_cast<const float4*>(part + (size_t)b * ldp + col), ep & 3u);
    for (int p = 0; p < world; ++p)
      if (p != rank) ar_store(P.buf[p] + ((long)(par * world + rank)) * cap + (long)b * D + col, g);
    if (max_spins & AR_OPT_PROBE) {
      // diagnostics: the pushed granule as memory holds it right after the store has completed; a mismatch is
      // logged in THIS rank's error area (words 24..31: marker, row, slice, epoch, peer, written, read back, col)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int p = 0; p < world; ++p) {
        if (p == rank) continue;
        const uint4 rb = ar_load_rmw(P.buf[p] + ((long)(par * world + rank)) * cap + (long)b * D + col);
        if (rb.x != g.x || rb.y != g.y || rb.z != g.z || rb.w != g.w) {
          uint32_t* dw = ar_err_word(P.buf[rank], world, cap);
          if (atomicCAS(dw + 24, 0u, 0xC33u) == 0u) {
            dw[25] = (uint32_t)b;
            dw[26] = (uint32_t)it.c;
            dw[27] = ep;
            dw[28] = (uint32_t)p;
            dw[29] = g.x;
            dw[30] = rb.x;
            dw[31] = (uint32_t)col;
          }
        }
      }
    }
  }
  const unsigned long long t1 = probe_on ? (unsigned long long)wall_clock64() : 0ull;
  // 2) per item: rank-ordered sum + residual add (bit-identical on every rank). Every call that advances an item's
  //    epoch has the peer write ALL of the slice's granules, so the protocol needs no re-tag of consumed granules
  //    (AR_OPT_RETAG, NLS_AR_RETAG=1, kept as an option; see the header for why rounds 3-5 had it on).
  bool failed = false;   // after one timeout, stop waiting (the error words are raised below)
  for (int t = 0; t < nit; ++t) {
    const AnItem it = an_item(xcd, k, j, t, nblk);
    const int rank = sim > 1 ? it.rr % sim : rank0, b = sim > 1 ? it.rr / sim : it.rr;
    const int ro = sim > 1 ? rank : 0;
    float* x = x0 + ro * sx;
    _Float16* h = h0 + ro * sh;
    unsigned* epochs = epochs0 + ro * se;
    int* tickets = tickets0 + ro * st;
    float* ssq = ssq0 + ro * sq;
    const float* part = part0 + ro * sp;
    const int c = it.c, eidx = b * nblk + c;
    const unsigned ep = s_ep[t];
    const uint32_t tag = ep & 3u;
    const int par = (int)(ep & 1u), col = c * ARN_VPB + 4 * threadIdx.x;
    float ss = 0.f;
    if (col < D) {
      uint32_t* mine = P.buf[rank];
      const float4 own = ar_val4(ar_pack4(*reinterpret_cast<const float4*>(part + (size_t)b * ldp + col), tag));
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int p = 0; p < world; ++p) {
        float4 v = own;
        if (p != rank) {
          uint32_t* src = mine + ((long)(par * world + p)) * cap + (long)b * D + col;
          const bool was = failed;
          const uint4 gv = ar_poll(src, tag, max_spins, failed);
          if (failed && !was) {
            ar_diag(mine, world, cap, 2, b, c, ep, p, gv.x);
            ar_diag2(mine, world, cap, gv, (uint32_t)col, ep_get(epochs + eidx, max_spins), ar_load_rmw(src));
          }
          v = ar_val4(gv);
          if (max_spins & AR_OPT_RETAG) {
            const uint32_t ct = (ep + 1u) & 3u;
            ar_store(src, make_uint4(ct, ct, ct, ct));
          }
        }
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      float4* xp = reinterpret_cast<float4*>(x + (size_t)b * ldx + col);
      float4 xv = *xp;
      xv.x += acc.x;
      xv.y += acc.y;
      xv.z += acc.z;
      xv.w += acc.w;
      wt_store4(reinterpret_cast<float*>(xp), xv);
      ss = xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    const unsigned long long fm = __ballot(failed);
    if (probe_on && threadIdx.x == 0 && eidx < AR_PROBE_SLOTS) {
      ArProbeRec& r = g_ar_probe[eidx * AR_PROBE_DEPTH + (ep & (AR_PROBE_DEPTH - 1))];
      r.ep = ep;
      r.xcc = xcc_id() | (fm ? 0x100u : 0u);
      r.t0 = t0;
      r.t1 = t1;
      r.t2 = (unsigned long long)wall_clock64();
    }
    // 3) publish the slice (x stores + share), then the row ticket: the last slice normalises the row
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      __hip_atomic_store((gu32*)(ssq + eidx), __float_as_uint(ss), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ep_put(epochs + eidx, ep, max_spins);
      if (fm) ar_raise(P, world, cap, err);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_last = __hip_atomic_fetch_add((__attribute__((address_space(1))) int*)(tickets + b), 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
    }
    __syncthreads();
    if (s_last) {
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((gu32*)(tickets + b), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      float tot = 0.f;
      for (int i = threadIdx.x; i < nblk; i += ARN_THREADS)
        tot += __uint_as_float(__hip_atomic_load((const gu32*)(ssq + (size_t)b * nblk + i), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
      const float inv = rsqrtf(tot / (float)D + eps);
      const float* xr = x + (size_t)b * ldx;
      _Float16* hr = h + (size_t)b * ldh;
      // the other slices' x were written by other workgroups (write-through, agent scope): read them the same way
      // (agent-scope loads bypass this CU's L1 and any stale line of an earlier kernel's read), not by plain loads
      const bool plain = max_spins & AR_OPT_XPLAIN;
      if (max_spins & AR_OPT_XCHECK) {
        float s2 = 0.f;
        for (int i = 4 * threadIdx.x; i < D; i += 4 * ARN_THREADS) {
          const float4 xv = plain ? *reinterpret_cast<const float4*>(xr + i) : wt_load4(xr + i);
          s2 += xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
        if (threadIdx.x == 0 && fabsf(s2 - tot) > 1e-4f * fabsf(tot) + 1e-6f) {
          uint32_t* dw = ar_err_word(P.buf[rank], world, cap);
          if (atomicCAS(dw + 32, 0u, 0xD44u) == 0u) {
            dw[33] = (uint32_t)b;
            dw[34] = __float_as_uint(tot);
            dw[35] = __float_as_uint(s2);
            dw[36] = ep;
            dw[37] = (uint32_t)rank;
            dw[38] = xcc_id();
          }
        }
      }
#pragma unroll 4
      for (int i = 4 * threadIdx.x; i < D; i += 4 * ARN_THREADS) {
        const float4 xv = plain ? *reinterpret_cast<const float4*>(xr + i) : wt_load4(xr + i);
        const float4 wv = *reinterpret_cast<const float4*>(nw + i);
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 o;
        o[0] = (_Float16)(xv.x * inv * wv.x);
        o[1] = (_Float16)(xv.y * inv * wv.y);
        o[2] = (_Float16)(xv.z * inv * wv.z);
        o[3] = (_Float16)(xv.w * inv * wv.w);
        *reinterpret_cast<h4*>(hr + i) = o;
      }
    }
    __syncthreads();     // s_last is reused by the next item
  }
}

// ---------------------------------------------------------------------------------------------
// Lossless one-shot all-gather of 32-bit words, and the fused vocab-parallel arg-max built on it --
// the two exchanges of a tensor-parallel decode step besides the sums, so a captured TP decode graph
// holds no RCCL call. Every word travels as two tagged dwords carrying 16 payload bits each (token
// ids, packed arg-max keys and fp32 candidate logits arrive bit-exact, unlike the 30-bit sums above);
// a 16-byte granule holds two words. Same slot / parity / consumed-tag protocol and bounded polls as
// the all-reduce, on a buffer set of its own with its own fixed grid (AG_BLOCKS x AG_THREADS, grid-
// stride over granules) and per-workgroup epochs, shared by the gather and the arg-max.
#define AG_BLOCKS 16
#define AG_THREADS 256

__device__ __forceinline__ uint4 ag_pack2(uint32_t a, uint32_t b, uint32_t tag) {
  return make_uint4(((a & 0xFFFFu) << 2) | tag, ((a >> 16) << 2) | tag, ((b & 0xFFFFu) << 2) | tag,
                    ((b >> 16) << 2) | tag);
}
__device__ __forceinline__ uint2 ag_unpack2(uint4 g) {
  return make_uint2((g.x >> 2) | ((g.y >> 2) << 16), (g.z >> 2) | ((g.w >> 2) << 16));
}

// src: this rank's n2 granules (2 * n2 words, laid out as `narr` arrays of rows x C words); dst receives
// every rank's words with the rank inside the row: dst[a][row][p * C + c] (arrays of rows x world*C) --
// per-rank top-C candidate lists come out as one vocabulary-ordered row per sequence. Slot blocks of
// AG_THREADS granules (see SlotBlocks).
__global__ __launch_bounds__(AG_THREADS) void oneshot_gather_kernel(const uint32_t* __restrict__ src, long n2,
                                                                     uint32_t* __restrict__ dst, int C, long per_arr,
                                                                     ArPeers P, int world, int rank, long cap,
                                                                     unsigned* __restrict__ epochs,
                                                                     int* __restrict__ err, long max_spins) {
  __shared__ unsigned s_ep[AR_MAX_WG_BLOCKS];
  __shared__ int s_fail;
  const SlotBlocks<AG_THREADS> B(n2);
  if (threadIdx.x == 0) s_fail = 0;
  blocks_begin(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  auto out_at = [&](long w, int p) -> uint32_t* {
    const long a = w / per_arr, rem = w - a * per_arr, r = rem / C, c = rem - r * C;
    return dst + a * per_arr * world + r * (long)world * C + (long)p * C + c;
  };
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const long i = ((long)B.first + (long)j * B.step) * AG_THREADS + threadIdx.x;
    const uint2 v = i < n2 ? reinterpret_cast<const uint2*>(src)[i] : make_uint2(0u, 0u);
    const uint4 g = ag_pack2(v.x, v.y, ep & 3u);
    for (int p = 0; p < world; ++p)
      if (p != rank) ar_store(P.buf[p] + ((long)((ep & 1u) * world + rank)) * cap + 4 * i, g);
    if (i < n2) {
      uint32_t* o = out_at(2 * i, rank);
      o[0] = v.x;
      o[1] = v.y;
    }
  }
  uint32_t* mine = P.buf[rank];
  bool failed = false;
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const long i = ((long)B.first + (long)j * B.step) * AG_THREADS + threadIdx.x;
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      const bool was = failed;
      const uint4 gv = ar_poll(mine + ((long)((ep & 1u) * world + p)) * cap + 4 * i, ep & 3u, max_spins, failed);
      if (failed && !was) ar_diag(mine, world, cap, 3, i, n2, ep, p, gv.x);
      const uint2 v = ag_unpack2(gv);
      if (i < n2) {
        uint32_t* o = out_at(2 * i, p);       // C even: both words of a granule share the row
        o[0] = v.x;
        o[1] = v.y;
      }
    }
  }
  if (failed) s_fail = 1;
  blocks_end(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  if (threadIdx.x == 0 && s_fail) ar_raise(P, world, cap, err);
}

// Vocab-parallel greedy pick: each rank's fused arg-max key of row i (ordered value bits << 32 | ~local id)
// is rebased to the global id (~local - vocab_lo == ~(local + vocab_lo)), exchanged (one granule per row),
// and the unsigned max over ranks gives the same token on every rank; the key is re-armed (0) for the next
// lm-head launch. Replaces xor / sub / RCCL MAX all-reduce / xor / unpack. Slot blocks as the gather.
__global__ __launch_bounds__(AG_THREADS) void oneshot_argmax_kernel(unsigned long long* __restrict__ keys, int n,
                                                                     unsigned vocab_lo, int* __restrict__ next_ids,
                                                                     ArPeers P, int world, int rank, long cap,
                                                                     unsigned* __restrict__ epochs,
                                                                     int* __restrict__ err, long max_spins) {
  __shared__ unsigned s_ep[AR_MAX_WG_BLOCKS];
  __shared__ int s_fail;
  const SlotBlocks<AG_THREADS> B(n);
  if (threadIdx.x == 0) s_fail = 0;
  blocks_begin(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const long i = ((long)B.first + (long)j * B.step) * AG_THREADS + threadIdx.x;
    const unsigned long long k = i < n ? keys[i] : 0ull;
    const uint4 g = ag_pack2((uint32_t)k - vocab_lo, (uint32_t)(k >> 32), ep & 3u);
    for (int p = 0; p < world; ++p)
      if (p != rank) ar_store(P.buf[p] + ((long)((ep & 1u) * world + rank)) * cap + 4L * i, g);
  }
  uint32_t* mine = P.buf[rank];
  bool failed = false;
  for (int j = 0; j < B.mine; ++j) {
    const unsigned ep = s_ep[j];
    const long i = ((long)B.first + (long)j * B.step) * AG_THREADS + threadIdx.x;
    const unsigned long long k = i < n ? keys[i] : 0ull;
    unsigned long long best = (k & 0xFFFFFFFF00000000ull) | (unsigned long long)((uint32_t)k - vocab_lo);
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      const bool was = failed;
      const uint4 gv = ar_poll(mine + ((long)((ep & 1u) * world + p)) * cap + 4L * i, ep & 3u, max_spins, failed);
      if (failed && !was) ar_diag(mine, world, cap, 4, i, n, ep, p, gv.x);
      const uint2 v = ag_unpack2(gv);
      const unsigned long long c = ((unsigned long long)v.y << 32) | v.x;
      best = c > best ? c : best;
    }
    if (i < n) {
      next_ids[i] = (int)~(uint32_t)best;
      keys[i] = 0ull;
    }
  }
  if (failed) s_fail = 1;
  blocks_end(epochs, B.first, B.step, B.mine, s_ep, max_spins);
  if (threadIdx.x == 0 && s_fail) ar_raise(P, world, cap, err);
}

__global__ void ar_err_clear_kernel(uint32_t* w) { *w = 0u; }

// every receive slot back to its initial tag (parity 0: 1, parity 1: 0) and the error word cleared -- the
// state after nls_ar_alloc; used (with zeroed epochs, on every rank, between barriers) after a timeout
__global__ void ar_reinit_kernel(uint32_t* buf, long half) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * half + AR_ERR_BYTES / 4; i += stride)
    buf[i] = i < half ? 0x01010101u : 0u;
}

// workgroups of one fused add+norm launch at most (multiple of 8, >= 8): NLS_AR_NORM_WGS, else the value the host
// set for this process (nls_ar_set_norm_wgs: fewer when several ranks share one GPU), default 128
static int g_norm_wgs = 128;
static int nls_ar_norm_wgs() {
  static const int env = [] {
    const char* e = getenv("NLS_AR_NORM_WGS");
    return e ? atoi(e) : 0;
  }();
  int v = env > 0 ? env : g_norm_wgs;
  v = v < 8 ? 8 : (v > 4096 ? 4096 : v);
  return v & ~7;
}

static long ar_opts(long max_spins) {
  static const long opts = [] {
    long o = 0;
    const char* a = getenv("NLS_AR_POLL_INV");
    const char* b = getenv("NLS_AR_RETAG");
    const char* c = getenv("NLS_AR_EP_RMW");
    const char* d = getenv("NLS_AR_POLL_RMW");
    if (a && atoi(a)) o |= AR_OPT_POLL_INV;
    if (b && atoi(b)) o |= AR_OPT_RETAG;       // default off since round 6 (header comment)
    const char* e = getenv("NLS_AR_PROBE");
    const char* f = getenv("NLS_AR_XCHECK");
    const char* g = getenv("NLS_AR_XPLAIN");
    if (c && atoi(c)) o |= AR_OPT_EP_RMW;
    if (d && atoi(d)) o |= AR_OPT_POLL_RMW;
    if (e && atoi(e)) o |= AR_OPT_PROBE;
    if (f && atoi(f)) o |= AR_OPT_XCHECK;
    if (g && atoi(g)) o |= AR_OPT_XPLAIN;
    return o;
  }();
  return (max_spins & AR_SPIN_MASK) | opts;
}

extern "C" {

// Polling footprint when R ranks share ONE GPU (the one-GPU rehearsal): a polling wave parked on a CU keeps a
// whole-CU kernel (a GEMM taking every VGPR / the LDS of a CU) of a co-resident rank from being placed there, so
// (R - 1) ranks' add+norm grids must leave most CUs whole -- at world 4 three 128-workgroup grids covered every CU
// and a peer's GEMM started only after the polls had expired (device-clock probes, profiles/tp_oneshot_world4_r05.txt).
// Separate GPUs (R = 1): 128. Every rank must set the same value before its first launch (the grid is part of the
// per-slice epoch bookkeeping of captured graphs only through the item -> workgroup map, which all ranks share).
int nls_ar_set_norm_wgs(int n) {
  if (n < 8 || n > 4096) return -1;
  g_norm_wgs = n & ~7;
  return 0;
}
int nls_ar_get_norm_wgs() { return nls_ar_norm_wgs(); }

// bytes of one rank's receive buffer for messages of up to `cap` floats (+ its error word area)
long nls_ar_buffer_bytes(long cap, int world) { return 2L * world * cap * 4L + AR_ERR_BYTES; }

int nls_ar_alloc(long cap, int world, void** buf, void* ipc_handle /* hipIpcMemHandle_t, 64 B */) {
  if (world < 1 || world > AR_MAX_RANKS || cap % 4) return -1;
  size_t bytes = (size_t)nls_ar_buffer_bytes(cap, world);
  // receive buffers: uncached device memory by default; NLS_AR_ALLOC=fine (fine-grained, coherent across
  // agents) or coarse (plain hipMalloc) for A/Bs of the IPC visibility on one shared GPU
  static const int kind = [] {
    const char* e = getenv("NLS_AR_ALLOC");
    return !e ? 0 : (e[0] == 'f' ? 1 : (e[0] == 'c' ? 2 : 0));
  }();
  hipError_t e = kind == 2 ? hipMalloc(buf, bytes)
                           : hipExtMallocWithFlags(buf, bytes, kind == 1 ? hipDeviceMallocFinegrained
                                                                         : hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  // parity-0 slots start with tag 1, parity-1 slots (and the error word) with tag 0: no epoch of a
  // slot's parity ever carries its initial tag
  e = hipMemset(*buf, 0, bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*buf, 0x01, (size_t)world * cap * 4);
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

// epoch counters of the plain all-reduce / the gather + arg-max: one per slot block of a `cap`-float buffer
long nls_ar_epoch_slots(long cap) { return (cap / 4 + AR_THREADS - 1) / AR_THREADS; }
long nls_ag_epoch_slots(long cap) { return (cap / 4 + AG_THREADS - 1) / AG_THREADS; }

// workgroups per row of the fused add+norm (its epoch / share / ticket layout: [rows][nls_ar_row_blocks])
int nls_ar_row_blocks(int D) { return (D + ARN_VPB - 1) / ARN_VPB; }

// this rank's error word (raised by any rank whose poll timed out): async copy to `host` (pinned), clear
int nls_ar_err_fetch(void* buf, long cap, int world, void* host, void* stream) {
  return (int)hipMemcpyAsync(host, (char*)buf + 2L * world * cap * 4L, 4, hipMemcpyDeviceToHost, (hipStream_t)stream);
}
// the first words of this rank's error area (word 0: the error word; 1..6: diagnostics of the first timeout)
int nls_ar_err_words(void* buf, long cap, int world, void* host, int n, void* stream) {
  return (int)hipMemcpyAsync(host, (char*)buf + 2L * world * cap * 4L, 4L * n, hipMemcpyDeviceToHost,
                             (hipStream_t)stream);
}
// n words at word offset `off` of a receive buffer (diagnostics: a timed-out slot as memory holds it)
int nls_ar_peek(void* buf, long off, int n, void* host, void* stream) {
  return (int)hipMemcpyAsync(host, (char*)buf + 4L * off, 4L * n, hipMemcpyDeviceToHost, (hipStream_t)stream);
}
// NLS_AR_PROBE: the timing history of add+norm workgroup slot `eidx` (AR_PROBE_DEPTH records of 32 bytes)
int nls_ar_probe_depth() { return AR_PROBE_DEPTH; }
int nls_ar_probe_hist(int eidx, void* host) {
  if (eidx < 0 || eidx >= AR_PROBE_SLOTS) return -1;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ar_probe), sizeof(ArProbeRec) * AR_PROBE_DEPTH,
                                  sizeof(ArProbeRec) * AR_PROBE_DEPTH * (size_t)eidx, hipMemcpyDeviceToHost);
}
int nls_ar_err_clear(void* buf, long cap, int world, void* stream) {
  hipLaunchKernelGGL(ar_err_clear_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     (uint32_t*)((char*)buf + 2L * world * cap * 4L));
  return (int)hipGetLastError();
}

int nls_ar_addnorm_sim(const float*, long, float*, long, const float*, void*, long, int, int, float, void* const*, int,
                       int, long, unsigned*, int*, float*, int*, long, void*, int, long, long, long, long, long, long);

// rows x D fused all-reduce + residual + RMSNorm; rows * D <= cap (the same buffers). `epochs`, `ssq`:
// rowcap * nls_ar_row_blocks(D) entries; `tickets`: rowcap zero-initialised ints (left zeroed)
int nls_ar_addnorm(const float* part, long ldp, float* x, long ldx, const float* nw, void* h, long ldh, int rows,
                   int D, float eps, void* const* peers, int world, int rank, long cap, unsigned* epochs, int* tickets,
                   float* ssq, int* err, long max_spins, void* stream) {
  return nls_ar_addnorm_sim(part, ldp, x, ldx, nw, h, ldh, rows, D, eps, peers, world, rank, cap, epochs, tickets,
                            ssq, err, max_spins, stream, 0, 0, 0, 0, 0, 0, 0);
}

// sim_ranks > 1: every rank in one launch (rank r's operands at base + r * stride) -- SimulatedGroup
int nls_ar_addnorm_sim(const float* part, long ldp, float* x, long ldx, const float* nw, void* h, long ldh, int rows,
                       int D, float eps, void* const* peers, int world, int rank, long cap, unsigned* epochs,
                       int* tickets, float* ssq, int* err, long max_spins, void* stream, int sim_ranks, long sp,
                       long sx, long sh, long se, long st, long sq) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || rows < 1 || D < 4 || D % 4 || ldp % 4 ||
      ldx % 4 || ldh % 4)
    return -1;
  const long rowcap = cap / D;
  if (rows > rowcap) return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (uint32_t*)peers[i] : nullptr;
  if (sim_ranks > 1 && sim_ranks != world) return -1;
  const int sim = sim_ranks > 1 ? sim_ranks : 1;
  const int nblk = nls_ar_row_blocks(D), nrr = rows * sim;
  // bounded grid: per XCD, k workgroups over its ceil(nrr / 8) rows x nblk slices (one item each when they fit)
  const int per_xcd = nblk * ((nrr + 7) / 8);
  int k = per_xcd < nls_ar_norm_wgs() / 8 ? per_xcd : nls_ar_norm_wgs() / 8;
  if ((per_xcd + k - 1) / k > ARN_MAX_ITEMS) k = (per_xcd + ARN_MAX_ITEMS - 1) / ARN_MAX_ITEMS;
  hipLaunchKernelGGL(oneshot_ar_addnorm_kernel, dim3(8 * k), dim3(ARN_THREADS), 0,
                     (hipStream_t)stream, part, ldp, x, ldx, nw, (_Float16*)h, ldh, D, eps, P, world, rank, cap, epochs,
                     tickets, ssq, err, ar_opts(max_spins), sim, sp, sx, sh, se, st, sq, nblk, nrr);
  return (int)hipGetLastError();
}

int nls_ag_blocks() { return AG_BLOCKS; }

// all-gather of 2 * n2 words (narr arrays of per_arr = rows * C words; C even) -> dst (see the kernel)
int nls_ag_run(const void* src, long n2, void* dst, int C, long per_arr, void* const* peers, int world, int rank,
               long cap, unsigned* epochs, int* err, long max_spins, void* stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n2 < 0 || C < 2 || C % 2 ||
      per_arr < C || per_arr % C || (2 * n2) % per_arr || cap % (4 * AG_THREADS) ||
      4 * ((n2 + AG_THREADS - 1) / AG_THREADS) * AG_THREADS > cap ||
      (n2 + AG_THREADS - 1) / AG_THREADS > (long)AG_BLOCKS * AR_MAX_WG_BLOCKS)
    return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (uint32_t*)peers[i] : nullptr;
  hipLaunchKernelGGL(oneshot_gather_kernel, dim3(AG_BLOCKS), dim3(AG_THREADS), 0, (hipStream_t)stream,
                     (const uint32_t*)src, n2, (uint32_t*)dst, C, per_arr, P, world, rank, cap, epochs, err,
                     ar_opts(max_spins));
  return (int)hipGetLastError();
}

// keys (u64 [n], fused arg-max of this rank's vocab shard starting at vocab_lo) -> next_ids on every rank
int nls_ag_argmax(void* keys, int n, int vocab_lo, void* next_ids, void* const* peers, int world, int rank, long cap,
                  unsigned* epochs, int* err, long max_spins, void* stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n < 1 || vocab_lo < 0 ||
      cap % (4 * AG_THREADS) || 4L * ((n + AG_THREADS - 1) / AG_THREADS) * AG_THREADS > cap ||
      (n + AG_THREADS - 1) / AG_THREADS > (long)AG_BLOCKS * AR_MAX_WG_BLOCKS)
    return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (uint32_t*)peers[i] : nullptr;
  hipLaunchKernelGGL(oneshot_argmax_kernel, dim3(AG_BLOCKS), dim3(AG_THREADS), 0, (hipStream_t)stream,
                     (unsigned long long*)keys, n, (unsigned)vocab_lo, (int*)next_ids, P, world, rank, cap, epochs, err,
                     ar_opts(max_spins));
  return (int)hipGetLastError();
}

// this rank's receive buffer back to the freshly allocated state (callers: every rank, no kernel in flight)
int nls_ar_reinit(void* buf, long cap, int world, void* stream) {
  if (world < 1 || world > AR_MAX_RANKS || cap % 4) return -1;
  hipLaunchKernelGGL(ar_reinit_kernel, dim3(256), dim3(256), 0, (hipStream_t)stream, (uint32_t*)buf,
                     (long)world * cap);
  return (int)hipGetLastError();
}

int nls_ar_run(float* data, long n, void* const* peers, int world, int rank, long cap, unsigned* epochs,
               int* err, long max_spins, void* stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n > cap || n % 4 || cap % (4 * AR_THREADS) ||
      (n / 4 + AR_THREADS - 1) / AR_THREADS > (long)AR_BLOCKS * AR_MAX_WG_BLOCKS)
    return -1;
  ArPeers P;
  for (int i = 0; i < AR_MAX_RANKS; ++i) P.buf[i] = i < world ? (uint32_t*)peers[i] : nullptr;
  hipLaunchKernelGGL(oneshot_ar_kernel, dim3(AR_BLOCKS), dim3(AR_THREADS), 0, (hipStream_t)stream, data, n, P,
                     world, rank, cap, epochs, err, ar_opts(max_spins));
  return (int)hipGetLastError();
}

}  // extern "C"
