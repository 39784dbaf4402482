// Host-only stand-in for the few HIP runtime calls native/kernels/tile_queue.h
// makes, so its slot-ownership logic can be compiled with g++ and tested on a
// CPU (tests/test_tile_queue_host.py). Memory is plain host memory; a
// "capture" is a flag per stream; memsets are recorded.
#pragma once
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

typedef int hipError_t;
typedef struct ihipStream_t* hipStream_t;
typedef int hipDevice_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
typedef enum { hipStreamCaptureStatusNone = 0, hipStreamCaptureStatusActive = 1 } hipStreamCaptureStatus;
#define hipStreamPerThread ((hipStream_t)2)
enum { hipStreamDefault = 0, hipStreamNonBlocking = 1 };

namespace fakehip {
inline int& cur_dev() { static int d = 0; return d; }
inline std::map<hipStream_t, int>& stream_dev() { static std::map<hipStream_t, int> m; return m; }
inline std::map<hipStream_t, bool>& capturing() { static std::map<hipStream_t, bool> m; return m; }
inline int& mallocs() { static int n = 0; return n; }
inline int& malloc_budget() { static int n = 1 << 30; return n; }
struct Memset { void* p; size_t n; hipStream_t s; bool captured; };
inline std::vector<Memset>& memsets() { static std::vector<Memset> v; return v; }
inline std::vector<hipStream_t>& syncs() { static std::vector<hipStream_t> v; return v; }
inline std::vector<hipStream_t>& created() { static std::vector<hipStream_t> v; return v; }
}  // namespace fakehip

inline hipError_t hipGetDevice(int* d) { *d = fakehip::cur_dev(); return hipSuccess; }
inline hipError_t hipSetDevice(int d) { fakehip::cur_dev() = d; return hipSuccess; }
inline hipError_t hipStreamGetDevice(hipStream_t s, hipDevice_t* d) {
  auto it = fakehip::stream_dev().find(s);
  *d = it == fakehip::stream_dev().end() ? fakehip::cur_dev() : it->second;
  return hipSuccess;
}
inline hipError_t hipStreamIsCapturing(hipStream_t s, hipStreamCaptureStatus* st) {
  *st = fakehip::capturing()[s] ? hipStreamCaptureStatusActive : hipStreamCaptureStatusNone;
  return hipSuccess;
}
inline hipError_t hipMalloc(void* p, size_t n) {
  if (fakehip::malloc_budget()-- <= 0) return hipErrorOutOfMemory;
  ++fakehip::mallocs();
  *(void**)p = std::malloc(n);
  return hipSuccess;
}
template <class T>
inline hipError_t hipMalloc(T** p, size_t n) { return hipMalloc((void*)p, n); }
inline hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t s) {
  fakehip::memsets().push_back({p, n, s, fakehip::capturing()[s]});
  if (!fakehip::capturing()[s]) std::memset(p, v, n);
  return hipSuccess;
}
enum hipMemcpyKind { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2 };
inline hipError_t hipMemcpy(void* dst, const void* src, size_t n, hipMemcpyKind) {
  std::memcpy(dst, src, n);
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t s) {
  fakehip::syncs().push_back(s);
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags) {
  static long next = 0x7000000;
  *s = (hipStream_t)(next += 16);
  fakehip::stream_dev()[*s] = fakehip::cur_dev();
  fakehip::created().push_back(*s);
  return flags == hipStreamNonBlocking ? hipSuccess : 1;
}
namespace fakehip {
inline std::vector<int>& priorities() {
  static std::vector<int> v;
  return v;
}
}  // namespace fakehip
inline hipError_t hipDeviceGetStreamPriorityRange(int* least, int* greatest) {
  *least = 0;
  *greatest = -1;
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned flags, int priority) {
  fakehip::priorities().push_back(priority);
  return hipStreamCreateWithFlags(s, flags);
}
