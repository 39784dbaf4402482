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
//    counters. The capture also records a 64-byte memset of the slot in front
//    of the kernel node, so every replay starts from zero whatever an earlier
//    replay left (one exec replayed concurrently with itself -- HIP does not
//    document that it serialises those -- can then only compute a tile twice,
//    with identical inputs and output, never skip one).
//  * no slot (reserve empty during a capture, allocation failure): nullptr and
//    the caller runs the one-shot grid, which needs no counters.
//
// Pool memory is allocated and zeroed outside any capture (hipMalloc +
// stream-ordered memset + sync of the calling stream) and never freed: 64 B
// per stream or captured launch.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <thread>
#include <vector>

namespace kgs {

constexpr int TQ_INTS = 16;     // 8 tickets + exit counter, padded to 64 B
constexpr int TQ_CHUNK = 256;   // slots per pool allocation (16 KiB)
constexpr int TQ_RESERVE = 64;  // free slots kept for captures
constexpr int TQ_DEVICES = 64;

struct TileQueueStats {
  long slots;          // allocated
  long stream_slots;   // owned by a (stream[, thread])
  long capture_slots;  // owned by a captured launch
  long fallbacks;      // calls that returned nullptr
};

namespace tq_detail {

struct Owner {
  hipStream_t stream;
  std::thread::id thread;  // only for hipStreamPerThread
  int* slot;
};

struct DevicePool {
  std::vector<int*> free_slots;
  std::vector<Owner> owners;
  long slots = 0, capture_slots = 0, fallbacks = 0;
};

inline std::mutex& mu() {
  static std::mutex m;
  return m;
}
inline DevicePool* pools() {
  static DevicePool p[TQ_DEVICES];
  return p;
}

// one more chunk of zeroed slots for device `dev` (caller holds mu, not capturing)
inline bool grow(DevicePool& P, int dev, hipStream_t stream) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return false;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return false;
  int* p = nullptr;
  bool ok = hipMalloc(&p, sizeof(int) * TQ_INTS * TQ_CHUNK) == hipSuccess;
  ok = ok && hipMemsetAsync(p, 0, sizeof(int) * TQ_INTS * TQ_CHUNK, stream) == hipSuccess &&
       hipStreamSynchronize(stream) == hipSuccess;
  if (cur != dev) (void)hipSetDevice(cur);
  if (!ok) {
    if (p) (void)hipFree(p);
    return false;
  }
  for (int i = TQ_CHUNK - 1; i >= 0; --i) P.free_slots.push_back(p + i * TQ_INTS);
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
  std::lock_guard<std::mutex> lock(mu());
  DevicePool& P = pools()[dev];
  if (capturing) {
    // no allocation or sync inside a capture: a reserved slot, or the one-shot grid
    if (P.free_slots.empty()) {
      ++P.fallbacks;
      return nullptr;
    }
    int* s = P.free_slots.back();
    if (hipMemsetAsync(s, 0, sizeof(int) * TQ_INTS, stream) != hipSuccess) {
      ++P.fallbacks;
      return nullptr;
    }
    P.free_slots.pop_back();  // owned by this graph node for the life of the process
    ++P.capture_slots;
    return s;
  }
  const bool per_thread = stream == hipStreamPerThread;
  const std::thread::id me = per_thread ? std::this_thread::get_id() : std::thread::id();
  for (const Owner& o : P.owners)
    if (o.stream == stream && o.thread == me) return o.slot;
  if ((int)P.free_slots.size() <= TQ_RESERVE && !grow(P, dev, stream) && P.free_slots.empty()) {
    ++P.fallbacks;
    return nullptr;
  }
  int* s = P.free_slots.back();
  P.free_slots.pop_back();
  P.owners.push_back(Owner{stream, me, s});
  return s;
}

inline TileQueueStats tile_queue_stats(int dev) {
  using namespace tq_detail;
  TileQueueStats st{0, 0, 0, 0};
  if (dev < 0 || dev >= TQ_DEVICES) return st;
  std::lock_guard<std::mutex> lock(mu());
  const DevicePool& P = pools()[dev];
  st.slots = P.slots;
  st.stream_slots = (long)P.owners.size();
  st.capture_slots = P.capture_slots;
  st.fallbacks = P.fallbacks;
  return st;
}

}  // namespace kgs
