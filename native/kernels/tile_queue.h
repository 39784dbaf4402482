// Tile-ticket slots for the persistent GEMMs (gemm_w4p.h), host side.
//
// A persistent launch hands out tiles through 8 per-XCD counters (tickets)
// plus one exit counter; its last workgroup resets all nine to zero before the
// kernel ends, so the next launch on the same stream starts from zero without a
// memset. Launches on DIFFERENT streams may run concurrently, so each
// (device, stream) pair gets its own 64-byte slot. The pool is allocated and
// zeroed once per device, on first use (a first use inside hipGraph capture
// returns nullptr and the caller runs the one-shot grid); a process that uses
// more than SLOTS streams per device wraps
// around, which is only safe if the wrapped streams never overlap.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>

namespace kgs {

constexpr int TQ_INTS = 16;   // 8 tickets + exit counter, padded to 64 B
constexpr int TQ_SLOTS = 64;  // streams per device
constexpr int TQ_DEVICES = 64;

inline int* tile_queue(hipStream_t stream) {
  static std::mutex mu;
  static int* pool[TQ_DEVICES] = {};
  static hipStream_t owner[TQ_DEVICES][TQ_SLOTS] = {};
  static int used[TQ_DEVICES] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= TQ_DEVICES) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!pool[dev]) {
    // no allocation or device-wide sync while the stream is being captured
    // into a hipGraph: the caller falls back to the one-shot grid
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, sizeof(int) * TQ_INTS * TQ_SLOTS) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, sizeof(int) * TQ_INTS * TQ_SLOTS) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    pool[dev] = p;
  }
  const int n = used[dev] < TQ_SLOTS ? used[dev] : TQ_SLOTS;
  for (int i = 0; i < n; ++i)
    if (owner[dev][i] == stream) return pool[dev] + i * TQ_INTS;
  const int slot = used[dev]++ % TQ_SLOTS;
  owner[dev][slot] = stream;
  return pool[dev] + slot * TQ_INTS;
}

}  // namespace kgs
