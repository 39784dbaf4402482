// Pure-HIP reproducer for the round-5 serving fault's suspected cause (VERDICT r5
// item 3; profiles/r5/fault/README.md): does a hipMemsetAsync captured into a
// hipGraph (a memset node) zero its 64 bytes on every replay?
//
// No torch, no kgs library. Each of G graphs captures, on its own stream,
//
//     memset node:  hipMemsetAsync(slot_g, 0, 64)
//     kernel node:  copy_out(slot_g -> seen_g)          (what a GEMM would read)
//     kernel node:  dirty(slot_g, pattern)              (leave the slot non-zero,
//                                                        as a launch that did not
//                                                        reset would)
//     P extra kernel nodes with pointer arguments (busy(), a stand-in for the
//     serving graph's other nodes)
//
// and the graphs are replayed R times each, interleaved, in two modes:
//   serial      replay g, synchronise, check seen_g == 0
//   concurrent  all G graphs launched back to back on their G streams, then one
//               synchronise, then check every seen_g
// Every replay's copy must be 64 zero bytes: the memset node ran after the
// previous replay's dirty() and before this replay's copy_out(). A word that
// is not zero is printed with its replay, graph and mode. The output ends with
// one JSON line: the ROCm / HIP runtime and driver versions and the counts.
//
// Also checked the same way, as the control: the zeroing done by a kernel node
// (zero64(), what tile_queue.h records since round 5) in G more graphs.
//
// Bounded: every kernel is one workgroup of 64 lanes writing in range; R and G
// are capped; each synchronise is a plain hipStreamSynchronize.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

constexpr int WORDS = 16;  // 64 bytes, the ticket slot

__global__ void copy_out(const int* slot, int* seen) {
  if (threadIdx.x < WORDS) seen[threadIdx.x] = slot[threadIdx.x];
}
__global__ void dirty(int* slot, int pattern) {
  if (threadIdx.x < WORDS) slot[threadIdx.x] = pattern ^ (int)threadIdx.x;
}
__global__ void zero64(int* slot) {
  if (threadIdx.x < WORDS) slot[threadIdx.x] = 0;
}
__global__ void busy(float* buf, const float* src, int n, long tag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = src[i] * 0.5f + (float)(tag & 7);
}

static std::string rocm_version() {
  std::ifstream f("/opt/rocm/.info/version");
  std::string v;
  if (f) std::getline(f, v);
  return v.empty() ? "unknown" : v;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? std::atoi(argv[1]) : 4;
  const int R = argc > 2 ? std::atoi(argv[2]) : 200;
  const int P = argc > 3 ? std::atoi(argv[3]) : 8;
  if (G < 1 || G > 16 || R < 1 || R > 5000 || P < 0 || P > 64) {
    std::fprintf(stderr, "usage: graph_memset_repro [G<=16] [R<=5000] [P<=64]\n");
    return 2;
  }
  int rt = 0, drv = 0;
  CK(hipRuntimeGetVersion(&rt));
  CK(hipDriverGetVersion(&drv));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));

  const int n = 1 << 16;
  float *buf = nullptr, *src = nullptr;
  CK(hipMalloc(&buf, n * sizeof(float)));
  CK(hipMalloc(&src, n * sizeof(float)));
  CK(hipMemset(src, 0, n * sizeof(float)));

  struct Case {
    const char* kind;  // "memset_node" | "kernel_node"
    int* slot;
    int* seen;
    hipStream_t s;
    hipGraphExec_t exec;
  };
  std::vector<Case> cases;
  for (int kind = 0; kind < 2; ++kind) {
    for (int g = 0; g < G; ++g) {
      Case c{kind == 0 ? "memset_node" : "kernel_node", nullptr, nullptr, nullptr, nullptr};
      CK(hipMalloc(&c.slot, WORDS * sizeof(int)));
      CK(hipMalloc(&c.seen, WORDS * sizeof(int)));
      CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
      // start dirty: the first replay must zero it too
      hipLaunchKernelGGL(dirty, dim3(1), dim3(64), 0, c.s, c.slot, 0x5a5a0000 + g);
      CK(hipStreamSynchronize(c.s));
      hipGraph_t graph;
      CK(hipStreamBeginCapture(c.s, hipStreamCaptureModeThreadLocal));
      if (kind == 0) CK(hipMemsetAsync(c.slot, 0, WORDS * sizeof(int), c.s));
      else hipLaunchKernelGGL(zero64, dim3(1), dim3(64), 0, c.s, c.slot);
      hipLaunchKernelGGL(copy_out, dim3(1), dim3(64), 0, c.s, c.slot, c.seen);
      hipLaunchKernelGGL(dirty, dim3(1), dim3(64), 0, c.s, c.slot, 0x7fd00000 + g);
      for (int p = 0; p < P; ++p)
        hipLaunchKernelGGL(busy, dim3(n / 256), dim3(256), 0, c.s, buf, src, n, (long)p + 100L * g);
      CK(hipStreamEndCapture(c.s, &graph));
      // the memset graphs must really contain a memset node (what the run tests)
      size_t nn = 0;
      CK(hipGraphGetNodes(graph, nullptr, &nn));
      std::vector<hipGraphNode_t> nodes(nn);
      CK(hipGraphGetNodes(graph, nodes.data(), &nn));
      int memsets = 0;
      for (auto nd : nodes) {
        hipGraphNodeType t;
        CK(hipGraphNodeGetType(nd, &t));
        memsets += t == hipGraphNodeTypeMemset;
      }
      if (memsets != (kind == 0 ? 1 : 0)) {
        std::fprintf(stderr, "graph %d (%s): %d memset nodes\n", g, c.kind, memsets);
        return 2;
      }
      CK(hipGraphInstantiate(&c.exec, graph, nullptr, nullptr, 0));
      CK(hipGraphDestroy(graph));
      cases.push_back(c);
    }
  }

  long checked[2] = {0, 0}, bad[2] = {0, 0};
  int printed = 0;
  std::vector<int> h(WORDS);
  auto check = [&](Case& c, int kind, int r, const char* mode) {
    CK(hipMemcpy(h.data(), c.seen, WORDS * sizeof(int), hipMemcpyDeviceToHost));
    ++checked[kind];
    bool ok = true;
    for (int w = 0; w < WORDS; ++w) ok = ok && h[w] == 0;
    if (!ok) {
      ++bad[kind];
      if (printed++ < 20) {
        std::printf("NONZERO %s mode=%s replay=%d slot=%p words:", c.kind, mode, r, (void*)c.slot);
        for (int w = 0; w < WORDS; ++w) std::printf(" %08x", (unsigned)h[w]);
        std::printf("\n");
      }
    }
  };
  for (int r = 0; r < R; ++r) {
    // serial
    for (size_t i = 0; i < cases.size(); ++i) {
      Case& c = cases[i];
      CK(hipMemsetAsync(c.seen, 0xff, WORDS * sizeof(int), c.s));  // seen = -1: a skipped copy shows
      CK(hipGraphLaunch(c.exec, c.s));
      CK(hipStreamSynchronize(c.s));
      check(c, i < (size_t)G ? 0 : 1, r, "serial");
    }
    // concurrent: every graph in flight at once on its own stream
    for (auto& c : cases) CK(hipMemsetAsync(c.seen, 0xff, WORDS * sizeof(int), c.s));
    for (auto& c : cases) CK(hipGraphLaunch(c.exec, c.s));
    for (auto& c : cases) CK(hipStreamSynchronize(c.s));
    for (size_t i = 0; i < cases.size(); ++i) check(cases[i], i < (size_t)G ? 0 : 1, r, "concurrent");
    if ((r + 1) % 50 == 0) {
      std::printf("replays %d: memset_node bad %ld / %ld, kernel_node bad %ld / %ld\n", r + 1, bad[0], checked[0],
                  bad[1], checked[1]);
      std::fflush(stdout);
    }
  }
  for (auto& c : cases) {
    CK(hipGraphExecDestroy(c.exec));
    CK(hipStreamDestroy(c.s));
    CK(hipFree(c.slot));
    CK(hipFree(c.seen));
  }
  CK(hipFree(buf));
  CK(hipFree(src));
  std::printf("{\"probe\": \"graph_memset_repro\", \"rocm\": \"%s\", \"hip_runtime_version\": %d, "
              "\"hip_driver_version\": %d, \"gcn_arch\": \"%s\", \"graphs_per_kind\": %d, \"replays\": %d, "
              "\"extra_nodes\": %d, \"memset_node_checks\": %ld, \"memset_node_nonzero\": %ld, "
              "\"kernel_node_checks\": %ld, \"kernel_node_nonzero\": %ld}\n",
              rocm_version().c_str(), rt, drv, prop.gcnArchName, G, R, P, checked[0], bad[0], checked[1], bad[1]);
  return bad[0] || bad[1] ? 1 : 0;
}
