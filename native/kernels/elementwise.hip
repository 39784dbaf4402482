// Memory-bound helper kernels for gfx950: vector add (the config-2 "HIP
// vector-add" smoke of BASELINE.json), bf16 transpose (layout change feeding the
// NT GEMM in backward passes) and a fused checksum used by the workload to
// verify results without copying tensors to the host.
//
// All loads/stores are 16 bytes per lane (cdna_hip_programming.md Guideline 13)
// and grids are capped at 256 CUs x 8 blocks with a grid-stride loop
// (Guideline 11).
#include "kgs_common.h"

namespace kgs {

constexpr int EW_THREADS = 256;
constexpr int EW_MAX_BLOCKS = 256 * 8;

__global__ __launch_bounds__(EW_THREADS) void vadd_f32(const float4* __restrict__ a, const float4* __restrict__ b,
                                                       float4* __restrict__ c, long n4) {
  const long stride = (long)gridDim.x * EW_THREADS;
  for (long i = (long)blockIdx.x * EW_THREADS + threadIdx.x; i < n4; i += stride) {
    float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

__global__ void vadd_f32_tail(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ c,
                              long start, long n) {
  long i = start + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

__global__ __launch_bounds__(EW_THREADS) void vadd_bf16(const bf16x8* __restrict__ a, const bf16x8* __restrict__ b,
                                                        bf16x8* __restrict__ c, long n8) {
  const long stride = (long)gridDim.x * EW_THREADS;
  for (long i = (long)blockIdx.x * EW_THREADS + threadIdx.x; i < n8; i += stride) {
    bf16x8 x = a[i], y = b[i], z;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      z[e] = (short)f2bf(bf2f((unsigned short)x[e]) + bf2f((unsigned short)y[e]));
    c[i] = z;
  }
}

__global__ void vadd_bf16_tail(const unsigned short* __restrict__ a, const unsigned short* __restrict__ b,
                               unsigned short* __restrict__ c, long start, long n) {
  long i = start + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

// out[c][r] = in[r][c]; 64x64 tile through LDS (+1 pad column: conflict-free
// column reads with 2-byte elements packed in 4-byte banks is not needed here,
// the pad just breaks the power-of-two stride).
__global__ __launch_bounds__(256) void transpose_bf16(const unsigned short* __restrict__ in,
                                                      unsigned short* __restrict__ out, int rows, int cols,
                                                      int ld_in, int ld_out) {
  __shared__ unsigned short tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int r = r0 + ty + 4 * k, cc = c0 + tx;
    tile[ty + 4 * k][tx] = (r < rows && cc < cols) ? in[(long)r * ld_in + cc] : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int oc = c0 + ty + 4 * k, orr = r0 + tx;  // output row = input col
    if (oc < cols && orr < rows) out[(long)oc * ld_out + orr] = tile[tx][ty + 4 * k];
  }
}

// Sum of |x| and sum of x over a bf16 tensor, accumulated in f32 per block and
// combined with one f32 atomic per block per quantity (Guideline 12).
__global__ __launch_bounds__(EW_THREADS) void checksum_bf16(const bf16x8* __restrict__ x, long n8,
                                                            float* __restrict__ out2) {
  float s = 0.f, sa = 0.f;
  const long stride = (long)gridDim.x * EW_THREADS;
  for (long i = (long)blockIdx.x * EW_THREADS + threadIdx.x; i < n8; i += stride) {
    bf16x8 v = x[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = bf2f((unsigned short)v[e]);
      s += f;
      sa += fabsf(f);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_down(s, off, 64);
    sa += __shfl_down(sa, off, 64);
  }
  __shared__ float red[2][EW_THREADS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { red[0][w] = s; red[1][w] = sa; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f, ta = 0.f;
#pragma unroll
    for (int i = 0; i < EW_THREADS / 64; ++i) { t += red[0][i]; ta += red[1][i]; }
    atomicAdd(out2, t);
    atomicAdd(out2 + 1, ta);
  }
}

static int blocks_for(long n) {
  long b = (n + EW_THREADS - 1) / EW_THREADS;
  if (b < 1) b = 1;
  return (int)(b < EW_MAX_BLOCKS ? b : EW_MAX_BLOCKS);
}

}  // namespace kgs

KGS_EXPORT int kgs_vector_add_f32(const void* a, const void* b, void* c, long n, hipStream_t s) {
  if (n < 0) return KGS_ERR_SHAPE;
  if (n == 0) return 0;
  const bool aligned = ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)c % 16 == 0);
  long n4 = aligned ? n / 4 : 0;
  if (n4) hipLaunchKernelGGL(kgs::vadd_f32, dim3(kgs::blocks_for(n4)), dim3(kgs::EW_THREADS), 0, s,
                             (const float4*)a, (const float4*)b, (float4*)c, n4);
  long rest = n - n4 * 4;
  if (rest)
    hipLaunchKernelGGL(kgs::vadd_f32_tail, dim3((rest + 255) / 256), dim3(256), 0, s, (const float*)a,
                       (const float*)b, (float*)c, n4 * 4, n);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_vector_add_bf16(const void* a, const void* b, void* c, long n, hipStream_t s) {
  if (n < 0) return KGS_ERR_SHAPE;
  if (n == 0) return 0;
  const bool aligned = ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)c % 16 == 0);
  long n8 = aligned ? n / 8 : 0;
  if (n8) hipLaunchKernelGGL(kgs::vadd_bf16, dim3(kgs::blocks_for(n8)), dim3(kgs::EW_THREADS), 0, s,
                             (const bf16x8*)a, (const bf16x8*)b, (bf16x8*)c, n8);
  long rest = n - n8 * 8;
  if (rest)
    hipLaunchKernelGGL(kgs::vadd_bf16_tail, dim3((rest + 255) / 256), dim3(256), 0, s,
                       (const unsigned short*)a, (const unsigned short*)b, (unsigned short*)c, n8 * 8, n);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_transpose_bf16(const void* in, void* out, int rows, int cols, int ld_in, int ld_out,
                                  hipStream_t s) {
  if (rows <= 0 || cols <= 0 || ld_in < cols || ld_out < rows) return KGS_ERR_SHAPE;
  dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  hipLaunchKernelGGL(kgs::transpose_bf16, grid, dim3(256), 0, s, (const unsigned short*)in, (unsigned short*)out,
                     rows, cols, ld_in, ld_out);
  return (int)hipGetLastError();
}

// out2 must hold 2 floats, zeroed by the caller (sum, sum|x|). n % 8 == 0, 16-B aligned.
KGS_EXPORT int kgs_checksum_bf16(const void* x, long n, void* out2, hipStream_t s) {
  if (n < 0 || n % 8 || (uintptr_t)x % 16) return KGS_ERR_ALIGN;
  if (n == 0) return 0;
  hipLaunchKernelGGL(kgs::checksum_bf16, dim3(kgs::blocks_for(n / 8)), dim3(kgs::EW_THREADS), 0, s,
                     (const bf16x8*)x, n / 8, (float*)out2);
  return (int)hipGetLastError();
}
