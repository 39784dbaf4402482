// Peer-to-peer all-reduce over xGMI for small and medium messages (SURVEY.md
// N6): the latency path that vLLM's custom all-reduce provides on ROCm when
// TP > 1 (the reference turns it off on its CPU pod,
// /root/reference/pods/vllm-cpu-pod.yaml:19). RCCL stays the bandwidth path.
//
// Every rank owns one IPC-shareable staging buffer (data) and one uncached
// signal block; both are mapped into every peer (hipIpcOpenMemHandle), so a
// kernel on rank r loads peer data and stores peer flags directly over the
// point-to-point xGMI links -- with 8 MI355X each peer is one link, so the N-1
// remote reads of a one-shot reduce run on N-1 links at once.
//
// Algorithms (one kernel launch each, no host round trip):
//   one-shot: copy-in -> barrier -> out = sum_p peer_p            (reads (N-1) x bytes)
//   two-shot: copy-in -> barrier -> reduce own 1/N segment in place
//             -> barrier -> gather the N reduced segments          (reads 2(N-1)/N x bytes)
// followed by an end barrier so the next call's copy-in cannot overwrite data
// a slower peer is still reading.
//
// Synchronisation is per workgroup: block b of every rank handles the same
// element set, so a flag exchange between the block-b's of all ranks orders
// exactly the data they share. A flag store is a system-scope release (L2
// write-back of the copied data before the flag), a flag poll a system-scope
// acquire (L2/L1 invalidate before the peer data is read). Flags carry an epoch
// (the host's, or -- epoch argument 0 -- a per-block counter kept in the rank's
// own signal block, so a captured hipGraph replays correctly: every replay
// reads and bumps the counter on the device) that changes on every call, so
// flags never need resetting. Every poll
// is bounded by a wall-clock timeout (s_memrealtime, 100 MHz): a missing peer
// sets a bit in *err and the kernel drains instead of hanging the GPU.
#include <cstring>

#include "kgs_common.h"

namespace kgs {
namespace ar {

constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 128;
constexpr int THREADS = 512;
constexpr int PHASES = 4;

struct Signal {
  unsigned flag[PHASES][MAX_BLOCKS][MAX_RANKS];
  unsigned epoch[MAX_BLOCKS];  // device-side call counter of this rank's block b
};

struct Ptrs {
  uint4* data[MAX_RANKS];
  Signal* sig[MAX_RANKS];
};

// Input/output of the rank(s) this launch serves: slot 0 for a normal launch;
// slot r for rank r when one launch plays every rank (single-GPU test mode).
struct IO {
  const uint4* in[MAX_RANKS];
  uint4* out[MAX_RANKS];
};

// rank_arg >= 0: this launch is rank rank_arg, blocks 0..nb-1.
// rank_arg <  0: one launch of nranks*nb blocks plays every rank; block
//                rank*nb + b is block b of that rank (all co-resident, so the
//                flag protocol runs exactly as across GPUs).
struct Who {
  int rank, b, slot;
};
__device__ __forceinline__ Who who(int rank_arg, int nb) {
  if (rank_arg >= 0) return {rank_arg, (int)blockIdx.x, 0};
  const int r = blockIdx.x / nb;
  return {r, (int)blockIdx.x - r * nb, r};
}

// host epoch, or (host_epoch == 0) this block's device counter + 1, skipping 0
__device__ __forceinline__ unsigned call_epoch(const Ptrs& P, const Who& me, unsigned host_epoch) {
  if (host_epoch) return host_epoch;
  const unsigned e = P.sig[me.rank]->epoch[me.b] + 1;
  return e ? e : 1;
}

// after the end barrier: the next launch (stream-ordered) sees the new counter
__device__ __forceinline__ void commit_epoch(const Ptrs& P, const Who& me, unsigned host_epoch, unsigned e) {
  if (!host_epoch && threadIdx.x == 0) P.sig[me.rank]->epoch[me.b] = e;
}

__device__ __forceinline__ unsigned long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// All NR ranks' block b meet; thread p < NR talks to peer p.
//
// The ordering across GPUs is spelled out in the ISA, not left to the atomic's
// expansion (tests/test_kernel_resources.py pins it): a release-store
// expansion emitted `buffer_wbl2 sc0 sc1` directly followed by the flag store
// whenever an earlier s_waitcnt vmcnt(0) had already retired everything else
// (the waitcnt pass dropped the wait after the write-back), so the flag could
// overtake the L2 write-back of the data a peer reads over xGMI. Now:
//   every wave   s_waitcnt vmcnt(0)           its own data stores reached L2
//   s_barrier                                 all waves' stores are in L2
//   flag thread  buffer_wbl2 sc0 sc1          write L2 back (system scope)
//                s_waitcnt vmcnt(0)           ... and wait until it is done
//                global_store flag sc0 sc1
//   poll         global_load sc0 sc1; s_waitcnt vmcnt(0); buffer_inv sc0 sc1
//                s_waitcnt vmcnt(0)           invalidate done before the barrier
//   s_barrier                                 then any wave may read peer data
template <int NR>
__device__ __forceinline__ void block_barrier(const Ptrs& P, int rank, int b, int phase, unsigned epoch,
                                              unsigned long timeout, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < NR) {
    const int p = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: buffer_wbl2 sc0 sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&P.sig[p]->flag[phase][b][rank], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* mine = &P.sig[rank]->flag[phase][b][p];
    const unsigned long t0 = now_ticks();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (now_ticks() - t0 > timeout) {
        atomicOr(err, 1 << phase);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// 16-byte vectors: 8 bf16 or 4 f32 lanes, accumulated in f32.
template <bool BF16>
struct Acc {
  float v[8];
  __device__ __forceinline__ void set(const uint4& x) {
    if constexpr (BF16) {
      const unsigned w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = bf2f((unsigned short)(w[i] & 0xffff));
        v[2 * i + 1] = bf2f((unsigned short)(w[i] >> 16));
      }
    } else {
      v[0] = __uint_as_float(x.x);
      v[1] = __uint_as_float(x.y);
      v[2] = __uint_as_float(x.z);
      v[3] = __uint_as_float(x.w);
    }
  }
  __device__ __forceinline__ void add(const uint4& x) {
    Acc<BF16> t;
    t.set(x);
#pragma unroll
    for (int i = 0; i < (BF16 ? 8 : 4); ++i) v[i] += t.v[i];
  }
  __device__ __forceinline__ uint4 get() const {
    if constexpr (BF16) {
      return make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                        pack_bf16x2(v[6], v[7]));
    } else {
      return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    }
  }
};

// Peers are summed in rank order 0..NR-1 on every rank, so all ranks produce
// bitwise-identical results.
template <bool BF16, int NR>
__device__ __forceinline__ uint4 reduce_at(const Ptrs& P, long i) {
  uint4 x[NR];
#pragma unroll
  for (int p = 0; p < NR; ++p) x[p] = P.data[p][i];  // NR independent loads in flight
  Acc<BF16> a;
  a.set(x[0]);
#pragma unroll
  for (int p = 1; p < NR; ++p) a.add(x[p]);
  return a.get();
}

// First index >= lo of this thread's grid-stride sequence i0, i0+stride, ...
__device__ __forceinline__ long first_at_or_after(long i0, long stride, long lo) {
  return i0 >= lo ? i0 : i0 + ((lo - i0 + stride - 1) / stride) * stride;
}

template <bool BF16, int NR>
__global__ __launch_bounds__(THREADS) void allreduce_oneshot(Ptrs P, IO io, int rank_arg, int nb, long nvec,
                                                             unsigned epoch, unsigned long timeout, int* err) {
  const Who me = who(rank_arg, nb);
  const unsigned host_epoch = epoch;
  epoch = call_epoch(P, me, host_epoch);
  const long stride = (long)nb * THREADS;
  const long i0 = (long)me.b * THREADS + threadIdx.x;
  const uint4* __restrict__ in = io.in[me.slot];
  uint4* __restrict__ out = io.out[me.slot];
  uint4* mine = P.data[me.rank];
  for (long i = i0; i < nvec; i += stride) mine[i] = in[i];
  block_barrier<NR>(P, me.rank, me.b, 0, epoch, timeout, err);
  for (long i = i0; i < nvec; i += stride) out[i] = reduce_at<BF16, NR>(P, i);
  block_barrier<NR>(P, me.rank, me.b, 3, epoch, timeout, err);
  commit_epoch(P, me, host_epoch, epoch);
}

template <bool BF16, int NR>
__global__ __launch_bounds__(THREADS) void allreduce_twoshot(Ptrs P, IO io, int rank_arg, int nb, long nvec,
                                                             unsigned epoch, unsigned long timeout, int* err) {
  const Who me = who(rank_arg, nb);
  const unsigned host_epoch = epoch;
  epoch = call_epoch(P, me, host_epoch);
  const long stride = (long)nb * THREADS;
  const long i0 = (long)me.b * THREADS + threadIdx.x;
  const uint4* __restrict__ in = io.in[me.slot];
  uint4* __restrict__ out = io.out[me.slot];
  uint4* mine = P.data[me.rank];
  for (long i = i0; i < nvec; i += stride) mine[i] = in[i];
  block_barrier<NR>(P, me.rank, me.b, 0, epoch, timeout, err);
  // reduce-scatter: own segment, written in place (peers only read their own
  // segments of this buffer in this phase)
  const long lo = me.rank * nvec / NR, hi = (me.rank + 1) * nvec / NR;
  for (long i = first_at_or_after(i0, stride, lo); i < hi; i += stride) mine[i] = reduce_at<BF16, NR>(P, i);
  block_barrier<NR>(P, me.rank, me.b, 1, epoch, timeout, err);
  // all-gather: segment s from rank s
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    const long slo = s * nvec / NR, shi = (s + 1) * nvec / NR;
    const uint4* src = P.data[s];
    for (long i = first_at_or_after(i0, stride, slo); i < shi; i += stride) out[i] = src[i];
  }
  block_barrier<NR>(P, me.rank, me.b, 3, epoch, timeout, err);
  commit_epoch(P, me, host_epoch, epoch);
}

template <bool BF16, int NR>
hipError_t launch(int algo, const Ptrs& P, const IO& io, int rank_arg, int nb, long nvec, unsigned epoch,
                  unsigned long timeout, int* err, hipStream_t s) {
  const dim3 grid(rank_arg >= 0 ? nb : nb * NR);
  if (algo == 0)
    hipLaunchKernelGGL((allreduce_oneshot<BF16, NR>), grid, dim3(THREADS), 0, s, P, io, rank_arg, nb, nvec, epoch,
                       timeout, err);
  else
    hipLaunchKernelGGL((allreduce_twoshot<BF16, NR>), grid, dim3(THREADS), 0, s, P, io, rank_arg, nb, nvec, epoch,
                       timeout, err);
  return hipGetLastError();
}

template <bool BF16>
hipError_t dispatch(int nranks, int algo, const Ptrs& P, const IO& io, int rank_arg, int nb, long nvec,
                    unsigned epoch, unsigned long timeout, int* err, hipStream_t s) {
#define KGS_AR_CASE(n) \
  case n: return launch<BF16, n>(algo, P, io, rank_arg, nb, nvec, epoch, timeout, err, s);
  switch (nranks) {
    KGS_AR_CASE(1)
    KGS_AR_CASE(2)
    KGS_AR_CASE(3)
    KGS_AR_CASE(4)
    KGS_AR_CASE(5)
    KGS_AR_CASE(6)
    KGS_AR_CASE(7)
    default: return launch<BF16, 8>(algo, P, io, rank_arg, nb, nvec, epoch, timeout, err, s);
  }
#undef KGS_AR_CASE
}

}  // namespace ar
}  // namespace kgs

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

KGS_EXPORT int kgs_ar_signal_bytes() { return (int)sizeof(kgs::ar::Signal); }
KGS_EXPORT int kgs_ar_max_blocks() { return kgs::ar::MAX_BLOCKS; }
KGS_EXPORT int kgs_ar_max_ranks() { return kgs::ar::MAX_RANKS; }

// Device allocation outside torch's caching allocator, so that the IPC handle
// names exactly this buffer. uncached=1 for signal blocks (polled by peers).
KGS_EXPORT int kgs_ar_alloc(size_t bytes, int uncached, void** out) {
  *out = nullptr;
  hipError_t e = uncached ? hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached) : hipMalloc(out, bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, bytes);
}

KGS_EXPORT int kgs_ar_free(void* p) { return (int)hipFree(p); }

KGS_EXPORT int kgs_ar_ipc_handle(void* p, void* handle_out /* 64 B */) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

KGS_EXPORT int kgs_ar_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

KGS_EXPORT int kgs_ar_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

KGS_EXPORT int kgs_ar_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// data / sigs: nranks device pointers valid in this process (own + opened
// peers). nbytes must be a multiple of 16; cap_bytes is the size of every
// staging buffer. dtype 0 = f32, 1 = bf16. algo 0 = one-shot, 1 = two-shot.
// rank >= 0: in/out point to this rank's tensors. rank == -1 (single-GPU test
// mode): ONE launch plays all nranks ranks, in/out are arrays of nranks device
// pointers (host memory), every staging buffer is local.
KGS_EXPORT int kgs_ar_run(void* const* data, void* const* sigs, int nranks, int rank, const void* in, void* out,
                          long nbytes, long cap_bytes, int dtype, int algo, unsigned epoch, int blocks,
                          double timeout_s, int* err, hipStream_t stream) {
  using namespace kgs::ar;
  if (nranks < 1 || nranks > MAX_RANKS || rank < -1 || rank >= nranks) return KGS_ERR_ARG;
  if (dtype != 0 && dtype != 1) return KGS_ERR_ARG;
  if (algo != 0 && algo != 1) return KGS_ERR_ARG;
  if (nbytes <= 0 || nbytes % 16 || nbytes > cap_bytes) return KGS_ERR_SHAPE;
  if (blocks < 1 || blocks > MAX_BLOCKS) return KGS_ERR_ARG;
  if (!(timeout_s > 0.0) || timeout_s > 600.0) return KGS_ERR_ARG;
  Ptrs P = {};
  for (int p = 0; p < nranks; ++p) {
    if (!data[p] || !sigs[p] || (uintptr_t)data[p] % 16) return KGS_ERR_ALIGN;
    P.data[p] = (uint4*)data[p];
    P.sig[p] = (Signal*)sigs[p];
  }
  IO io = {};
  const int nio = rank >= 0 ? 1 : nranks;
  for (int r = 0; r < nio; ++r) {
    const void* i = rank >= 0 ? in : ((const void* const*)in)[r];
    void* o = rank >= 0 ? out : ((void* const*)out)[r];
    if (!i || !o || ((uintptr_t)i | (uintptr_t)o) % 16) return KGS_ERR_ALIGN;
    io.in[r] = (const uint4*)i;
    io.out[r] = (uint4*)o;
  }
  const long nvec = nbytes / 16;
  const unsigned long ticks = (unsigned long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  hipError_t e = dtype == 1 ? dispatch<true>(nranks, algo, P, io, rank, blocks, nvec, epoch, ticks, err, stream)
                            : dispatch<false>(nranks, algo, P, io, rank, blocks, nvec, epoch, ticks, err, stream);
  return (int)e;
}
