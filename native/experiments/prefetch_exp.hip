// Infinity Cache (MALL) prefetch probe (round 5, experiments library only).
//
// kgs_exp_mall_touch: read `bytes` of a buffer with plain 16-B loads from
// `nwg` workgroups, so its lines are in the 256 MiB die-level cache before a
// kernel that streams them (a decode projection's weights, while the previous
// projection still runs). The loaded words feed one predicated store that in
// practice never fires, so the loads cannot be dropped. Meant to run on a side
// stream with few workgroups: they share CUs with the running GEMM, whose
// workgroups leave most wave slots free.
#include "kgs_common.h"

namespace kgs {
namespace exp {

constexpr int TOUCH_UNROLL = 8;

__global__ __launch_bounds__(256) void mall_touch(const uint4* __restrict__ p, long n16, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  const long step = (long)gridDim.x * 256 * TOUCH_UNROLL;
  for (long i = (long)blockIdx.x * 256 * TOUCH_UNROLL + threadIdx.x; i < n16; i += step) {
    uint4 v[TOUCH_UNROLL];
#pragma unroll
    for (int u = 0; u < TOUCH_UNROLL; ++u) {
      const long j = i + (long)u * 256;
      v[u] = j < n16 ? p[j] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < TOUCH_UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

}  // namespace exp
}  // namespace kgs

KGS_EXPORT int kgs_exp_mall_touch(const void* p, long bytes, int nwg, unsigned* sink, hipStream_t s) {
  if (p == nullptr || sink == nullptr || bytes < 16 || nwg <= 0 || (uintptr_t)p % 16) return KGS_ERR_ARG;
  hipLaunchKernelGGL(kgs::exp::mall_touch, dim3(nwg), dim3(256), 0, s, (const uint4*)p, bytes / 16, sink);
  return (int)hipGetLastError();
}
