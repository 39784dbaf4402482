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

// U vectors per thread per trip, all loads issued before the first add, so a
// wave keeps 2*U 16-B loads in flight (HBM streaming wants bytes in flight,
// not more waves). NT: non-temporal loads/stores (streamed once, keep them out
// of the way of L2/MALL residents).
template <int U, bool NT>
__global__ __launch_bounds__(EW_THREADS) void vadd_f32(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                       f32x4* __restrict__ c, long n4) {
  const long stride = (long)gridDim.x * EW_THREADS;
  long i = (long)blockIdx.x * EW_THREADS + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
      y[u] = NT ? __builtin_nontemporal_load(b + i + u * stride) : b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(x[u] + y[u], c + i + u * stride); else c[i + u * stride] = x[u] + y[u];
    }
  }
  for (; i < n4; i += stride) c[i] = a[i] + b[i];
}

__global__ void vadd_f32_tail(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ c,
                              long start, long n) {
  long i = start + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

__device__ __forceinline__ bf16x8 add_bf16x8(const bf16x8& x, const bf16x8& y) {
  bf16x8 z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (short)f2bf(bf2f((unsigned short)x[e]) + bf2f((unsigned short)y[e]));
  return z;
}

template <int U, bool NT>
__global__ __launch_bounds__(EW_THREADS) void vadd_bf16(const bf16x8* __restrict__ a, const bf16x8* __restrict__ b,
                                                        bf16x8* __restrict__ c, long n8) {
  const long stride = (long)gridDim.x * EW_THREADS;
  long i = (long)blockIdx.x * EW_THREADS + threadIdx.x;
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    bf16x8 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
      y[u] = NT ? __builtin_nontemporal_load(b + i + u * stride) : b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bf16x8 z = add_bf16x8(x[u], y[u]);
      if (NT) __builtin_nontemporal_store(z, c + i + u * stride); else c[i + u * stride] = z;
    }
  }
  for (; i < n8; i += stride) c[i] = add_bf16x8(a[i], b[i]);
}

__global__ void vadd_bf16_tail(const unsigned short* __restrict__ a, const unsigned short* __restrict__ b,
                               unsigned short* __restrict__ c, long start, long n) {
  long i = start + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

// out[c][r] = in[r][c] with 16-B global accesses on both sides: a 64x64 tile
// is loaded as 8-element row chunks into LDS (row pitch 72 elements = 144 B
// keeps 16-B alignment and staggers banks), then each thread gathers 8
// consecutive INPUT rows of one column from LDS and writes them as one 16-B
// output chunk; 8 lanes cover one 128-B output row segment. Needs cols, rows, ld_in, ld_out % 8 == 0 and 16-B aligned
// pointers; transpose_bf16 below handles everything else.
constexpr int TP = 72;
__global__ __launch_bounds__(256) void transpose_bf16_v8(const bf16x8* __restrict__ in, bf16x8* __restrict__ out,
                                                         int rows, int cols, int ld_in8, int ld_out8) {
  __shared__ __attribute__((aligned(16))) unsigned short tile[64 * TP];
  // diagonal block order: blocks that run together write output rows spread
  // over the column tiles instead of 64-row strides of one power-of-two pitch
  // (HBM channel camping on square power-of-two shapes)
  const int bx = (blockIdx.x + blockIdx.y) % gridDim.x;
  const int r0 = blockIdx.y * 64, c0 = bx * 64;
  const int t = threadIdx.x;
  // load: 64 rows x 8 chunks = 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = t + k * 256, r = idx >> 3, ch = idx & 7;
    const int gr = r0 + r, gc = c0 + ch * 8;
    bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (gr < rows && gc < cols) v = in[(long)gr * ld_in8 + (gc >> 3)];
    *(bf16x8*)&tile[r * TP + ch * 8] = v;
  }
  __syncthreads();
  // store: a wave writes 8 output rows x 128 contiguous bytes per instruction
  // (lane>>3 = output row, lane&7 = 16-B chunk = 8 input rows)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int col = (t >> 3) + k * 32, rb = (t & 7) * 8;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)tile[(rb + j) * TP + col];
    const int oc = c0 + col, orr = r0 + rb;
    if (oc < cols && orr < rows) out[(long)oc * ld_out8 + (orr >> 3)] = v;
  }
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

// RCCL-shaped stand-in for a collective's kernel on ONE GPU (bench/overlap.py):
// a fixed, small number of workgroups ("channels") each streams its slice of
// dst += src, `passes` times. A ring all-reduce kernel has this footprint --
// tens of long-lived workgroups, memory-bound -- so it measures whether such a
// kernel gets CUs next to a GEMM that fills every CU, without needing peers.
__global__ __launch_bounds__(EW_THREADS) void comm_standin_f32(f32x4* __restrict__ dst, const f32x4* __restrict__ src,
                                                              long nvec, int passes) {
  const long per = (nvec + gridDim.x - 1) / gridDim.x;
  const long lo = per * blockIdx.x;
  const long hi = lo + per < nvec ? lo + per : nvec;
  for (int p = 0; p < passes; ++p)
    for (long i = lo + threadIdx.x; i < hi; i += EW_THREADS) dst[i] += src[i];
}

// Collective stand-in by TIME (bench/overlap_rccl.py): each workgroup holds its
// CU for `ticks` of the constant wall clock from the moment it starts, the way
// an RCCL channel's workgroup sits on a CU for the length of the collective.
// With dynamic LDS > 32 KiB (launch argument) no 128 KiB GEMM workgroup fits
// beside it, and the GEMM waves need a whole SIMD's registers anyway.
__global__ __launch_bounds__(256) void cu_hold(long ticks) {
  const long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

static int blocks_for(long n) {
  long b = (n + EW_THREADS - 1) / EW_THREADS;
  if (b < 1) b = 1;
  return (int)(b < EW_MAX_BLOCKS ? b : EW_MAX_BLOCKS);
}

}  // namespace kgs

namespace {

// Streaming configurations (variant): unroll, non-temporal, block cap.
struct EwCfg {
  int unroll;
  bool nt;
  long max_blocks;
};
constexpr EwCfg EW_CFGS[] = {
    {1, false, 1L << 30},            // 0: default = one-shot grid (measured best, profiles/elementwise.json)
    {1, false, kgs::EW_MAX_BLOCKS},  // 1: one vector per trip
    {2, false, kgs::EW_MAX_BLOCKS},  // 2
    {4, false, kgs::EW_MAX_BLOCKS},  // 3
    {4, true, kgs::EW_MAX_BLOCKS},   // 4: non-temporal
    {1, false, 1L << 30},            // 5: one-shot grid, no loop
    {4, false, 1024},                // 6: fewer blocks
};
constexpr int EW_NCFG = sizeof(EW_CFGS) / sizeof(EW_CFGS[0]);

int ew_blocks(long nvec, const EwCfg& c) {
  long b = (nvec + (long)kgs::EW_THREADS * c.unroll - 1) / ((long)kgs::EW_THREADS * c.unroll);
  if (b < 1) b = 1;
  return (int)(b < c.max_blocks ? b : c.max_blocks);
}

}  // namespace

#define KGS_EW_LAUNCH(KERNEL, VT, a, b, c, nvec, cfg, s)                                                     \
  do {                                                                                                        \
    const dim3 g(ew_blocks(nvec, cfg)), blk(kgs::EW_THREADS);                                                 \
    if (cfg.unroll == 4 && cfg.nt)                                                                            \
      hipLaunchKernelGGL((KERNEL<4, true>), g, blk, 0, s, (const VT*)a, (const VT*)b, (VT*)c, nvec);          \
    else if (cfg.unroll == 4)                                                                                 \
      hipLaunchKernelGGL((KERNEL<4, false>), g, blk, 0, s, (const VT*)a, (const VT*)b, (VT*)c, nvec);         \
    else if (cfg.unroll == 2)                                                                                 \
      hipLaunchKernelGGL((KERNEL<2, false>), g, blk, 0, s, (const VT*)a, (const VT*)b, (VT*)c, nvec);         \
    else                                                                                                      \
      hipLaunchKernelGGL((KERNEL<1, false>), g, blk, 0, s, (const VT*)a, (const VT*)b, (VT*)c, nvec);         \
  } while (0)

KGS_EXPORT int kgs_vector_add_f32_v(const void* a, const void* b, void* c, long n, int variant, hipStream_t s) {
  if (n < 0) return KGS_ERR_SHAPE;
  if (variant < 0 || variant >= EW_NCFG) return KGS_ERR_ARG;
  if (n == 0) return 0;
  const bool aligned = ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)c % 16 == 0);
  long n4 = aligned ? n / 4 : 0;
  if (n4) KGS_EW_LAUNCH(kgs::vadd_f32, f32x4, a, b, c, n4, EW_CFGS[variant], s);
  long rest = n - n4 * 4;
  if (rest)
    hipLaunchKernelGGL(kgs::vadd_f32_tail, dim3((rest + 255) / 256), dim3(256), 0, s, (const float*)a,
                       (const float*)b, (float*)c, n4 * 4, n);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_vector_add_bf16_v(const void* a, const void* b, void* c, long n, int variant, hipStream_t s) {
  if (n < 0) return KGS_ERR_SHAPE;
  if (variant < 0 || variant >= EW_NCFG) return KGS_ERR_ARG;
  if (n == 0) return 0;
  const bool aligned = ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)c % 16 == 0);
  long n8 = aligned ? n / 8 : 0;
  if (n8) KGS_EW_LAUNCH(kgs::vadd_bf16, bf16x8, a, b, c, n8, EW_CFGS[variant], s);
  long rest = n - n8 * 8;
  if (rest)
    hipLaunchKernelGGL(kgs::vadd_bf16_tail, dim3((rest + 255) / 256), dim3(256), 0, s,
                       (const unsigned short*)a, (const unsigned short*)b, (unsigned short*)c, n8 * 8, n);
  return (int)hipGetLastError();
}

// dst += src (f32, n % 4 == 0, 16-B aligned) on `nblocks` workgroups, `passes` times.
// lds_bytes: dynamic LDS reserved per workgroup (unused by the kernel) -- with
// more than 32 KiB a workgroup cannot share a CU with a 128 KiB GEMM workgroup,
// like a collective kernel that needs its own CU.
KGS_EXPORT int kgs_comm_standin_f32(void* dst, const void* src, long n, int nblocks, int passes, int lds_bytes,
                                    hipStream_t s) {
  if (n <= 0 || n % 4 || nblocks <= 0 || passes <= 0) return KGS_ERR_SHAPE;
  if (lds_bytes < 0 || lds_bytes > 160 * 1024) return KGS_ERR_ARG;
  if ((uintptr_t)dst % 16 || (uintptr_t)src % 16) return KGS_ERR_ALIGN;
  hipLaunchKernelGGL(kgs::comm_standin_f32, dim3(nblocks), dim3(kgs::EW_THREADS), lds_bytes, s, (f32x4*)dst,
                     (const f32x4*)src, n / 4, passes);
  return (int)hipGetLastError();
}

// nblocks workgroups of 256 threads, each holding a CU for `usec` microseconds
// (kgs::cu_hold). lds_bytes of dynamic LDS per workgroup (<= 160 KiB).
KGS_EXPORT int kgs_cu_hold(int nblocks, double usec, int lds_bytes, hipStream_t s) {
  if (nblocks <= 0 || usec < 0 || usec > 1e7) return KGS_ERR_SHAPE;
  if (lds_bytes < 0 || lds_bytes > 160 * 1024) return KGS_ERR_ARG;
  static int khz[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return KGS_ERR_ARG;
  if (!khz[dev] && (hipDeviceGetAttribute(&khz[dev], hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
                    khz[dev] <= 0))
    khz[dev] = 100000;  // gfx9 constant clock: 100 MHz
  const long ticks = (long)(usec * 1e-3 * khz[dev]);
  hipLaunchKernelGGL(kgs::cu_hold, dim3(nblocks), dim3(256), lds_bytes, s, ticks);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_vector_add_f32(const void* a, const void* b, void* c, long n, hipStream_t s) {
  return kgs_vector_add_f32_v(a, b, c, n, 0, s);
}

KGS_EXPORT int kgs_vector_add_bf16(const void* a, const void* b, void* c, long n, hipStream_t s) {
  return kgs_vector_add_bf16_v(a, b, c, n, 0, s);
}

// variant 0 = auto (16-B path when rows, cols, both ld % 8 == 0 and pointers
// are 16-B aligned), 1 = element-wise tile, 2 = force the 16-B path.
KGS_EXPORT int kgs_transpose_bf16_v(const void* in, void* out, int rows, int cols, int ld_in, int ld_out, int variant,
                                    hipStream_t s) {
  if (rows <= 0 || cols <= 0 || ld_in < cols || ld_out < rows) return KGS_ERR_SHAPE;
  const bool v8ok = rows % 8 == 0 && cols % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 &&
                    ((uintptr_t)in | (uintptr_t)out) % 16 == 0;
  if (variant == 2 && !v8ok) return KGS_ERR_ALIGN;
  if (variant < 0 || variant > 2) return KGS_ERR_ARG;
  dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (variant != 1 && v8ok)
    hipLaunchKernelGGL(kgs::transpose_bf16_v8, grid, dim3(256), 0, s, (const bf16x8*)in, (bf16x8*)out, rows, cols,
                       ld_in / 8, ld_out / 8);
  else
    hipLaunchKernelGGL(kgs::transpose_bf16, grid, dim3(256), 0, s, (const unsigned short*)in, (unsigned short*)out,
                       rows, cols, ld_in, ld_out);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_transpose_bf16(const void* in, void* out, int rows, int cols, int ld_in, int ld_out,
                                  hipStream_t s) {
  return kgs_transpose_bf16_v(in, out, rows, cols, ld_in, ld_out, 0, s);
}

// out2 must hold 2 floats, zeroed by the caller (sum, sum|x|). n % 8 == 0, 16-B aligned.
KGS_EXPORT int kgs_checksum_bf16(const void* x, long n, void* out2, hipStream_t s) {
  if (n < 0 || n % 8 || (uintptr_t)x % 16) return KGS_ERR_ALIGN;
  if (n == 0) return 0;
  hipLaunchKernelGGL(kgs::checksum_bf16, dim3(kgs::blocks_for(n / 8)), dim3(kgs::EW_THREADS), 0, s,
                     (const bf16x8*)x, n / 8, (float*)out2);
  return (int)hipGetLastError();
}
