// kgs-rccl-bench: single-process, multi-GPU RCCL all-reduce sweep.
//
// One process drives every GPU the pod was allocated (ncclCommInitAll, one HIP
// stream per GPU, grouped launches), so no cross-process IPC / shared memory is
// needed -- the simplest way to exercise xGMI from a pod holding amd.com/gpu: 8
// (BASELINE.json config 4). Reports, per message size, the time
// of one all-reduce, algorithm bandwidth (bytes/t) and bus bandwidth
// (algbw * 2(n-1)/n), and checks the sum.
//
//   kgs-rccl-bench [--ngpus N] [--min-bytes B] [--max-bytes B] [--factor F]
//                  [--iters I] [--warmup W] [--dtype f32|bf16] [--json]
//
// The C++ twin of kgs.parallel.allreduce.allreduce_sweep (torch.distributed,
// one process per GPU). The reference has no collectives at all.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                                     \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)
#define NCCLCHECK(x)                                                                    \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      std::exit(3);                                                                     \
    }                                                                                   \
  } while (0)

__global__ void fill_f32(float* p, size_t n, float v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) p[i] = v;
}

// counts elements != v (after the sum); bf16 buffers are checked as raw bits
__global__ void check_f32(const float* p, size_t n, float v, unsigned long long* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long b = 0;
  for (; i < n; i += stride) b += (p[i] != v);
  if (b) atomicAdd(bad, b);
}

__global__ void fill_bf16(unsigned short* p, size_t n, float v) {
  unsigned u = __float_as_uint(v);
  unsigned short h = (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) p[i] = h;
}

struct Args {
  int ngpus = 0;
  size_t min_bytes = 8, max_bytes = 1ull << 30;
  int factor = 2, iters = 20, warmup = 5;
  bool bf16 = false, json = false;
};

static Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", k.c_str());
        std::exit(1);
      }
      return argv[++i];
    };
    if (k == "--ngpus") a.ngpus = std::atoi(next());
    else if (k == "--min-bytes") a.min_bytes = std::strtoull(next(), nullptr, 10);
    else if (k == "--max-bytes") a.max_bytes = std::strtoull(next(), nullptr, 10);
    else if (k == "--factor") a.factor = std::atoi(next());
    else if (k == "--iters") a.iters = std::atoi(next());
    else if (k == "--warmup") a.warmup = std::atoi(next());
    else if (k == "--dtype") a.bf16 = std::string(next()) == "bf16";
    else if (k == "--json") a.json = true;
    else {
      std::fprintf(stderr,
                   "usage: %s [--ngpus N] [--min-bytes B] [--max-bytes B] [--factor F] [--iters I] "
                   "[--warmup W] [--dtype f32|bf16] [--json]\n",
                   argv[0]);
      std::exit(1);
    }
  }
  if (a.factor < 2) a.factor = 2;
  return a;
}

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  int n = a.ngpus > 0 ? std::min(a.ngpus, ndev) : ndev;
  if (n < 1) {
    std::fprintf(stderr, "no GPUs visible\n");
    return 1;
  }
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  NCCLCHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  const size_t esize = a.bf16 ? 2 : 4;
  const ncclDataType_t dt = a.bf16 ? ncclBfloat16 : ncclFloat32;
  std::vector<void*> buf(n);
  std::vector<hipStream_t> st(n);
  std::vector<hipEvent_t> e0(n), e1(n);
  std::vector<unsigned long long*> bad(n);
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipMalloc(&buf[i], a.max_bytes));
    HIPCHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    HIPCHECK(hipEventCreate(&e0[i]));
    HIPCHECK(hipEventCreate(&e1[i]));
    HIPCHECK(hipMalloc(&bad[i], sizeof(unsigned long long)));
  }
  if (!a.json)
    std::printf("# kgs-rccl-bench: %d GPU(s), dtype %s, %d iters\n# %12s %10s %10s %10s %6s\n", n,
                a.bf16 ? "bf16" : "f32", a.iters, "bytes", "time_us", "algbw_GBs", "busbw_GBs", "check");
  const double busf = n > 1 ? 2.0 * (n - 1) / n : 0.0;
  double peak = 0;
  for (size_t bytes = std::max(a.min_bytes, esize); bytes <= a.max_bytes; bytes *= a.factor) {
    const size_t cnt = bytes / esize;
    // correctness: rank i contributes (i+1); expect n(n+1)/2 everywhere
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(i));
      if (a.bf16)
        hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, st[i], (unsigned short*)buf[i], cnt, (float)(i + 1));
      else
        hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, st[i], (float*)buf[i], cnt, (float)(i + 1));
    }
    NCCLCHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i) NCCLCHECK(ncclAllReduce(buf[i], buf[i], cnt, dt, ncclSum, comms[i], st[i]));
    NCCLCHECK(ncclGroupEnd());
    unsigned long long nbad = 0;
    if (!a.bf16) {
      for (int i = 0; i < n; ++i) {
        HIPCHECK(hipSetDevice(i));
        HIPCHECK(hipMemsetAsync(bad[i], 0, sizeof(unsigned long long), st[i]));
        hipLaunchKernelGGL(check_f32, dim3(1024), dim3(256), 0, st[i], (const float*)buf[i], cnt,
                           (float)(n * (n + 1) / 2), bad[i]);
        unsigned long long h = 0;
        HIPCHECK(hipMemcpyAsync(&h, bad[i], sizeof h, hipMemcpyDeviceToHost, st[i]));
        HIPCHECK(hipStreamSynchronize(st[i]));
        nbad += h;
      }
    }
    for (int w = 0; w < a.warmup; ++w) {
      NCCLCHECK(ncclGroupStart());
      for (int i = 0; i < n; ++i) NCCLCHECK(ncclAllReduce(buf[i], buf[i], cnt, dt, ncclSum, comms[i], st[i]));
      NCCLCHECK(ncclGroupEnd());
    }
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipStreamSynchronize(st[i]));
      HIPCHECK(hipEventRecord(e0[i], st[i]));
    }
    for (int it = 0; it < a.iters; ++it) {
      NCCLCHECK(ncclGroupStart());
      for (int i = 0; i < n; ++i) NCCLCHECK(ncclAllReduce(buf[i], buf[i], cnt, dt, ncclSum, comms[i], st[i]));
      NCCLCHECK(ncclGroupEnd());
    }
    float worst_ms = 0;
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipEventRecord(e1[i], st[i]));
      HIPCHECK(hipEventSynchronize(e1[i]));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      worst_ms = std::max(worst_ms, ms);
    }
    const double t = worst_ms / 1e3 / a.iters;
    const double algbw = bytes / t / 1e9, busbw = algbw * busf;
    peak = std::max(peak, busbw);
    if (a.json)
      std::printf("{\"bytes\": %zu, \"n_gpus\": %d, \"dtype\": \"%s\", \"time_us\": %.2f, \"algbw_gbs\": %.2f, "
                  "\"busbw_gbs\": %.2f, \"wrong\": %llu}\n",
                  bytes, n, a.bf16 ? "bf16" : "f32", t * 1e6, algbw, busbw, nbad);
    else
      std::printf("  %12zu %10.2f %10.2f %10.2f %6s\n", bytes, t * 1e6, algbw, busbw, nbad ? "FAIL" : "ok");
    std::fflush(stdout);
    if (nbad) return 4;
  }
  if (!a.json) std::printf("# peak busbw %.1f GB/s over %d GPU(s)\n", peak, n);
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(i));
    hipFree(buf[i]);
    hipFree(bad[i]);
    ncclCommDestroy(comms[i]);
  }
  return 0;
}
