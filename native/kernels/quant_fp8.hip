// Dynamic per-tensor fp8 (OCP e4m3fn) quantisation for gfx950, device-resident:
//
//   amax  = max |x|                         (amax_kernel, one f32 atomic per block)
//   scale = max(amax, tiny) / 448            (every quantize block derives it)
//   q     = e4m3(clamp(x / scale, +-448))    (v_cvt_pk_fp8_f32, RNE)
//
// The scale stays in device memory (out2[1]) and the fp8 GEMM reads it in its
// epilogue (kgs_gemm_fp8_nt_dev), so a W8A8 Linear forward -- quantise the
// activation, GEMM against pre-quantised weights -- never synchronises with
// the host and can be captured in a hipGraph.
//
// gfx950's fp8 conversion and MFMA use the OCP e4m3 format (torch.float8_e4m3fn),
// not MI300's fnuz variant (MI355X_MICROARCH.md, matrix cores).
#include "kgs_common.h"

namespace kgs {
namespace q8 {

constexpr int THREADS = 256;
constexpr float E4M3_MAX = 448.f;

template <bool BF16>
__device__ __forceinline__ void load8(const void* x, long i, float v[8]) {
  if constexpr (BF16) {
    const bf16x8 h = ((const bf16x8*)x)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bf2f((unsigned short)h[e]);
  } else {
    const f32x4 a = ((const f32x4*)x)[2 * i], b = ((const f32x4*)x)[2 * i + 1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      v[4 + e] = b[e];
    }
  }
}

// out2[0] = max |x| as f32 bits (non-negative floats order like unsigned ints)
template <bool BF16>
__global__ __launch_bounds__(THREADS) void amax_kernel(const void* __restrict__ x, long n8, unsigned* out2) {
  float m = 0.f;
  const long stride = (long)gridDim.x * THREADS;
  for (long i = (long)blockIdx.x * THREADS + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load8<BF16>(x, i, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_down(m, off, 64));
  __shared__ float red[THREADS / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int w = 1; w < THREADS / 64; ++w) t = fmaxf(t, red[w]);
    atomicMax(out2, __float_as_uint(t));
  }
}

template <bool BF16>
__global__ __launch_bounds__(THREADS) void quantize_kernel(const void* __restrict__ x, long n8,
                                                           float* __restrict__ out2, uint2* __restrict__ y) {
  const float amax = __uint_as_float(((const unsigned*)out2)[0]);
  const float scale = fmaxf(amax, 1e-12f) / E4M3_MAX;
  const float inv = 1.f / scale;
  const long stride = (long)gridDim.x * THREADS;
  for (long i = (long)blockIdx.x * THREADS + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load8<BF16>(x, i, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e] * inv, -E4M3_MAX), E4M3_MAX);
    unsigned lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
    unsigned hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
    y[i] = make_uint2(lo, hi);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out2[1] = scale;
}

// the amax accumulator's reset, as a kernel: inside a hipGraph capture a
// hipMemsetAsync becomes a memset node, and in round 5 a memset node in the
// captured serving graph left garbage instead of zeros (tile_queue.h
// tq_zero_slot). A pure-HIP reproducer does not fail on its own, on ROCm 7.2 or
// on torch's HIP 7.0 (profiles/r6/memset/README.md), so the trigger is in the
// capture context, not isolated; captured paths use kernel nodes either way.
__global__ __launch_bounds__(64) void zero_amax(unsigned* __restrict__ out2) {
  if (threadIdx.x == 0) out2[0] = 0u;
}

}  // namespace q8
}  // namespace kgs

// x: n elements (f32 dtype 0 / bf16 dtype 1), 16-B aligned, n % 8 == 0.
// y: n bytes of e4m3. out2: 2 floats of device memory -> [amax bits, scale].
KGS_EXPORT int kgs_quantize_fp8(const void* x, long n, int dtype, void* y, void* out2, hipStream_t s) {
  if (n <= 0 || n % 8) return KGS_ERR_SHAPE;
  if (dtype != 0 && dtype != 1) return KGS_ERR_ARG;
  if (((uintptr_t)x | (uintptr_t)y) % 16 || (uintptr_t)out2 % 8) return KGS_ERR_ALIGN;
  const long n8 = n / 8;
  long blocks = (n8 + kgs::q8::THREADS - 1) / kgs::q8::THREADS;
  const int grid = (int)(blocks < 2048 ? blocks : 2048);
  hipLaunchKernelGGL(kgs::q8::zero_amax, dim3(1), dim3(64), 0, s, (unsigned*)out2);
  if (dtype == 1) {
    hipLaunchKernelGGL(kgs::q8::amax_kernel<true>, dim3(grid), dim3(kgs::q8::THREADS), 0, s, x, n8, (unsigned*)out2);
    hipLaunchKernelGGL(kgs::q8::quantize_kernel<true>, dim3(grid), dim3(kgs::q8::THREADS), 0, s, x, n8,
                       (float*)out2, (uint2*)y);
  } else {
    hipLaunchKernelGGL(kgs::q8::amax_kernel<false>, dim3(grid), dim3(kgs::q8::THREADS), 0, s, x, n8,
                       (unsigned*)out2);
    hipLaunchKernelGGL(kgs::q8::quantize_kernel<false>, dim3(grid), dim3(kgs::q8::THREADS), 0, s, x, n8,
                       (float*)out2, (uint2*)y);
  }
  return (int)hipGetLastError();
}
