// The one definition of kgs::tq_zero_slot (tile_queue.h) for a library:
// include it from exactly one translation unit of each library that uses the
// ticket pool (gemm_bf16.hip for libkgs_kernels, gemm_w4h.hip for the
// experiments library).
#pragma once

#include "tile_queue.h"

namespace kgs {

__global__ __launch_bounds__(64) void tq_zero_kernel(int* __restrict__ slot) {
  if (threadIdx.x < TQ_INTS) slot[threadIdx.x] = 0;
}

hipError_t tq_zero_slot(int* slot, hipStream_t stream) {
  hipLaunchKernelGGL(tq_zero_kernel, dim3(1), dim3(64), 0, stream, slot);
  return hipGetLastError();
}

}  // namespace kgs
