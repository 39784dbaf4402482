// Tile-ticket slots for the persistent GEMMs (gemm_w4p.h, gemm_w4f8.h), host side.
//
// A persistent launch hands out tiles through 8 per-XCD counters (tickets)
// plus one exit counter, in one 64-byte slot; its last workgroup resets all
// nine to zero before the kernel ends. Two launches that run at the same time
// must never share a slot: their tickets would interleave and each would skip
// the tiles the other took (wrong output, no error). Ownership rules:
//
//  * eager launch (stream not capturing): the slot of its (device, stream).
//    Launches on one stream are ordered, so the slot is used by one kernel at a
//    time and the exit reset leaves it zero for the next. hipStreamPerThread is
//    a different stream on every thread, so it is keyed by thread as well.
//    Every new stream gets a NEW slot; the pool grows in chunks (it never wraps
//    onto a live slot).
//  * launch captured into a hipGraph: a slot of its own, taken from a reserve
//    allocated before the capture and never given to anything else. A graph
//    exec replayed on any stream, while eager GEMMs run on the capture stream or
//    while another graph from the same stream replays, therefore uses its own
//    counters. The capture also records a zeroing kernel node for the slot
//    (tq_zero_slot, not a memset node: see below) in front of the GEMM's node,
//    so every replay starts from zero whatever an earlier
//    replay left (one exec replayed concurrently with itself -- HIP does not
//    document that it serialises those -- can then only compute a tile twice,
//    with identical inputs and output, never skip one). That holds for
//    epilogues that only WRITE C. A read-modify-write epilogue (EPI_ADDC:
//    C += A.B^T) computed twice adds twice, so kgs_gemm_bf16_nt_addc never
//    takes a slot while its stream is capturing (it runs the one-shot grid).
//  * no slot (reserve empty during a capture, allocation failure): nullptr and
//    the caller runs the one-shot grid, which needs no counters.
//
// Pool memory is allocated and zeroed outside any capture and outside the pool
// lock, and never freed: 64 B per stream or captured launch. A new chunk is
// zeroed on the pool's own non-blocking stream and only THAT stream is
// synchronised (one 16 KiB memset is all it ever holds): the caller's stream
// -- possibly queued behind a long kernel -- is never waited on, and no other
// thread's tile_queue() call waits behind the growth.
// Owners are found through a hash map keyed by (stream, thread).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace kgs {

constexpr int TQ_INTS = 16;     // 8 tickets + exit counter, padded to 64 B
constexpr int TQ_ERR = 15;      // padding word a kernel sets when it read an impossible ticket (sticky)
constexpr int TQ_CHUNK = 256;   // slots per pool allocation (16 KiB)
constexpr int TQ_RESERVE = 64;  // free slots kept for captures
constexpr int TQ_DEVICES = 64;

struct TileQueueStats {
  long slots;          // allocated
  long stream_slots;   // owned by a (stream[, thread])
  long capture_slots;  // owned by a captured launch
  long fallbacks;      // calls that returned nullptr
  long grow_failures;  // pool growths that failed (each starts a backoff)
};

// Zero one 64-byte slot on `stream` with a KERNEL (tile_queue_zero.h; one
// definition per library). In a hipGraph capture it becomes a kernel node like
// every other node. In round 5 a captured hipMemsetAsync -- a memset node --
// in the serving engine's decode graph did not zero the slot: after the
// graph's first replay it held 64 bytes of host-pointer-like words
// (0x00005639_00004020, 0x000073fd_988f2020, ...), i.e. garbage tickets; with a
// word whose high bit was set the persistent GEMM turned it into a negative
// tile index and the run died with hipErrorIllegalAddress
// (profiles/r5/fault/README.md). A pure-HIP reproducer (memset node -> copy ->
// dirty, 1600 replays, serial and concurrent) zeroes correctly on ROCm 7.2 and
// on torch's HIP 7.0 (profiles/r6/memset/README.md): memset nodes do not fail
// on their own; what in that capture made this one fail is not isolated.
// tests/test_serve_gpu.py now asserts the serving graphs hold no memset node.
hipError_t tq_zero_slot(int* slot, hipStream_t stream);

namespace tq_detail {

struct OwnerKey {
  hipStream_t stream;
  std::thread::id thread;  // only for hipStreamPerThread
  bool operator==(const OwnerKey& o) const { return stream == o.stream && thread == o.thread; }
};

struct OwnerHash {
  size_t operator()(const OwnerKey& k) const {
    return std::hash<const void*>()((const void*)k.stream) ^
           (std::hash<std::thread::id>()(k.thread) * 0x9e3779b97f4a7c15ull);
  }
};

struct DevicePool {
  std::vector<int*> chunks;  // every allocation, for tile_queue_check
  std::vector<int*> free_slots;
  std::unordered_map<OwnerKey, int*, OwnerHash> owners;
  hipStream_t zero_stream = nullptr;  // private, non-blocking; touched only by the growing thread
  bool growing = false;               // one growth at a time per device
  int grow_backoff = 0;               // eager calls to skip growing for after a failed growth
  bool warned = false;                // capture fallback reported once
  long slots = 0, capture_slots = 0, fallbacks = 0, grow_failures = 0;
};

inline std::mutex& mu() {
  static std::mutex m;
  return m;
}
inline DevicePool* pools() {
  static DevicePool p[TQ_DEVICES];
  return p;
}

// One chunk of zeroed slots for device `dev`, made WITHOUT the pool lock by
// the one thread that set P.growing: hipMalloc, a memset on the pool's private
// stream, a sync of that stream. nullptr on failure.
inline int* new_chunk(DevicePool& P, int dev) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return nullptr;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
  int* p = nullptr;
  // The zeroing stream is HIGH priority. HIP multiplexes streams onto a few
  // hardware queues per priority (GPU_MAX_HW_QUEUES, 4 here); a normal-priority
  // private stream can share its hardware queue with a caller's stream, and
  // then the chunk's memset -- and this thread's sync on it -- waits behind
  // whatever that stream is running (measured: a 50 ms CU hold on the caller's
  // stream made its first persistent GEMM call take 50 ms of host time). High
  // priority streams come from their own queue pool.
  bool ok = P.zero_stream != nullptr;
  if (!ok) {
    int least = 0, greatest = 0;
    ok = (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
          hipStreamCreateWithPriority(&P.zero_stream, hipStreamNonBlocking, greatest) == hipSuccess) ||
         hipStreamCreateWithFlags(&P.zero_stream, hipStreamNonBlocking) == hipSuccess;
  }
  ok = ok && hipMalloc(&p, sizeof(int) * TQ_INTS * TQ_CHUNK) == hipSuccess;
  ok = ok && hipMemsetAsync(p, 0, sizeof(int) * TQ_INTS * TQ_CHUNK, P.zero_stream) == hipSuccess &&
       hipStreamSynchronize(P.zero_stream) == hipSuccess;
  if (cur != dev) (void)hipSetDevice(cur);
  if (!ok && p) {
    (void)hipFree(p);
    p = nullptr;
  }
  return p;
}

// Grow device `dev`'s pool by one chunk; called with `lock` held, releases it
// around the allocation. Returns false if another thread is already growing
// the pool or the allocation failed.
// After a failure (memory nearly full, no stream) the next TQ_GROW_BACKOFF
// eager calls do not retry: hipMalloc and stream creation stay off the hot path.
constexpr int TQ_GROW_BACKOFF = 256;
inline bool grow(DevicePool& P, int dev, std::unique_lock<std::mutex>& lock) {
  if (P.growing) return false;
  if (P.grow_backoff > 0) {
    --P.grow_backoff;
    return false;
  }
  P.growing = true;
  lock.unlock();
  int* p = new_chunk(P, dev);
  lock.lock();
  P.growing = false;
  if (!p) {
    P.grow_backoff = TQ_GROW_BACKOFF;
    ++P.grow_failures;
    return false;
  }
  for (int i = TQ_CHUNK - 1; i >= 0; --i) P.free_slots.push_back(p + i * TQ_INTS);
  P.chunks.push_back(p);
  P.slots += TQ_CHUNK;
  return true;
}

}  // namespace tq_detail

inline int* tile_queue(hipStream_t stream) {
  using namespace tq_detail;
  int dev = 0;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess || dev < 0 || dev >= TQ_DEVICES) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::unique_lock<std::mutex> lock(mu());
  DevicePool& P = pools()[dev];
  if (capturing) {
    // no allocation or sync inside a capture: a reserved slot, or the one-shot grid
    int* s = P.free_slots.empty() ? nullptr : P.free_slots.back();
    if (s == nullptr || tq_zero_slot(s, stream) != hipSuccess) {
      ++P.fallbacks;
      if (!P.warned) {
        P.warned = true;
        std::fprintf(stderr, "[kgs] tile_queue: no reserved ticket slot for a captured persistent GEMM on device "
                             "%d; the capture runs the one-shot grid (an eager launch refills the reserve)\n", dev);
      }
      return nullptr;
    }
    P.free_slots.pop_back();  // owned by this graph node for the life of the process
    ++P.capture_slots;
    return s;
  }
  const bool per_thread = stream == hipStreamPerThread;
  const OwnerKey key{stream, per_thread ? std::this_thread::get_id() : std::thread::id()};
  auto it = P.owners.find(key);
  int* s = it == P.owners.end() ? nullptr : it->second;
  // keep the capture reserve filled: captures cannot allocate, eager calls can
  // (a known stream's calls refill it too)
  if ((int)P.free_slots.size() <= TQ_RESERVE) grow(P, dev, lock);
  if (s != nullptr) return s;
  if (P.free_slots.empty()) {
    ++P.fallbacks;
    return nullptr;
  }
  s = P.free_slots.back();
  P.free_slots.pop_back();
  P.owners.emplace(key, s);
  return s;
}

// The pool invariant, checked from the host: with no persistent GEMM running on
// device `dev`, every int of every slot is zero -- tickets and exit counter
// (each launch's last workgroup resets them) and the padding (nothing writes
// it). A nonzero word means a launch did not finish its reset or something
// wrote into the pool; the next eager launch on that slot would take wrong
// tickets. Copies the pool to the host (synchronous): the caller makes sure no
// GEMM is in flight. out[0..3] = {dirty slots, dirty words, first dirty value,
// its word index in the pool}; out[4] = the first dirty slot's device address,
// out[5..20] its 16 words (what overwrote it names the writer); out[21] = slots
// whose error word (TQ_ERR) is set: a persistent GEMM read a ticket no launch
// could have issued and stopped taking tiles, so its output is incomplete.
// Returns 0 or a hipError_t.
constexpr int TQ_CHECK_OUT = 5 + TQ_INTS + 1;
inline int tile_queue_check(int dev, long* out) {
  using namespace tq_detail;
  for (int i = 0; i < TQ_CHECK_OUT; ++i) out[i] = 0;
  out[3] = -1;
  if (dev < 0 || dev >= TQ_DEVICES) return 0;
  std::lock_guard<std::mutex> lock(mu());
  const DevicePool& P = pools()[dev];
  std::vector<int> h(TQ_INTS * TQ_CHUNK);
  long base = 0;
  for (int* c : P.chunks) {
    const hipError_t e = hipMemcpy(h.data(), c, sizeof(int) * h.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return (int)e;
    for (int sl = 0; sl < TQ_CHUNK; ++sl) {
      bool dirty = false;
      for (int i = 0; i < TQ_INTS; ++i) {
        const int v = h[sl * TQ_INTS + i];
        if (v == 0) continue;
        dirty = true;
        if (out[1]++ == 0) {
          out[2] = v;
          out[3] = base + sl * TQ_INTS + i;
          out[4] = (long)(uintptr_t)(c + sl * TQ_INTS);
          for (int j = 0; j < TQ_INTS; ++j) out[5 + j] = h[sl * TQ_INTS + j];
        }
      }
      out[0] += dirty;
      out[5 + TQ_INTS] += h[sl * TQ_INTS + TQ_ERR] != 0;
    }
    base += TQ_INTS * TQ_CHUNK;
  }
  return 0;
}

inline TileQueueStats tile_queue_stats(int dev) {
  using namespace tq_detail;
  TileQueueStats st{0, 0, 0, 0, 0};
  if (dev < 0 || dev >= TQ_DEVICES) return st;
  std::lock_guard<std::mutex> lock(mu());
  const DevicePool& P = pools()[dev];
  st.slots = P.slots;
  st.stream_slots = (long)P.owners.size();
  st.capture_slots = P.capture_slots;
  st.fallbacks = P.fallbacks;
  st.grow_failures = P.grow_failures;
  return st;
}

}  // namespace kgs
