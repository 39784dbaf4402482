// Fused decoder-block glue for gfx950: the HBM-bound ops between the GEMMs of a
// Llama-style block, each one pass over its tensors with 16-B accesses.
//
//   * add_rmsnorm : x' = x + d (bf16 residual stream, written back),
//                   y = rmsnorm(x') * w          -- one wave per row
//   * rope_qkv    : rotate-half (neox) RoPE on the q and k heads of the fused
//                   QKV projection output, in place, from an fp32 cos/sin table
//   * silu_mul    : SwiGLU's silu(g) * u from the fused gate|up output
//   * *_fp8 forms of add_rmsnorm / silu_mul and quant_rows: e4m3 output with a
//     per-row (per-token) dynamic scale, so the W8A8 GEMM that consumes the
//     activation needs no separate amax + quantise passes
//
// All math is fp32 with one bf16 rounding per output. The PyTorch version of
// the same block (kgs/models/llama.py, backend "torch") runs ~10 kernels per op
// here with fp32 intermediates in HBM; profiles/llama_prefill_kernels_v0.md has
// the numbers that motivated these kernels.
#include "kgs_common.h"

namespace kgs {
namespace tfm {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

constexpr float E4M3_MAX = 448.f;

// 8 floats (already divided by the scale) -> 8 e4m3 bytes (OCP e4m3fn, RNE)
__device__ __forceinline__ uint2 to_e4m3x8(const float* v) {
  float c[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) c[e] = fminf(fmaxf(v[e], -E4M3_MAX), E4M3_MAX);
  unsigned lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  unsigned hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return make_uint2(lo, hi);
}

// One wave per row; lane owns 16-B chunks lane + 64*j (j < NC) -- a wave reads
// 1 KB contiguous per j. cols == 512 * NC.
// Q8: y is written as e4m3 bytes with a per-row scale ys[row] = amax/448
// (per-token dynamic quantisation for the fp8 GEMM that consumes y).
template <int NC, bool Q8 = false>
__global__ __launch_bounds__(256) void add_rmsnorm(unsigned short* __restrict__ x, const unsigned short* __restrict__ d,
                                                   unsigned short* __restrict__ xo,
                                                   const unsigned short* __restrict__ w,
                                                   unsigned short* __restrict__ y, int rows, long ldx, long ldy,
                                                   float eps, float* __restrict__ ys = nullptr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16x8* xr = (const bf16x8*)(x + row * ldx);
  float v[NC][8];
  bf16x8 xv[NC], dv[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) xv[j] = xr[lane + 64 * j];
  if (d != nullptr) {
    const bf16x8* dr = (const bf16x8*)(d + row * ldx);
#pragma unroll
    for (int j = 0; j < NC; ++j) dv[j] = dr[lane + 64 * j];
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (d != nullptr) {
      bf16x8 s;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        s[e] = (short)f2bf(bf2f((unsigned short)xv[j][e]) + bf2f((unsigned short)dv[j][e]));
      xv[j] = s;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[j][e] = bf2f((unsigned short)xv[j][e]);
      ss += v[j][e] * v[j][e];
    }
  }
  if (d != nullptr) {
    bf16x8* xw = (bf16x8*)(xo + row * ldx);
#pragma unroll
    for (int j = 0; j < NC; ++j) xw[lane + 64 * j] = xv[j];
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)(NC * 512) + eps);
  const bf16x8* wr = (const bf16x8*)w;
  if constexpr (Q8) {
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const bf16x8 wv = wr[lane + 64 * j];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[j][e] = v[j][e] * r * bf2f((unsigned short)wv[e]);
        am = fmaxf(am, fabsf(v[j][e]));
      }
    }
    am = wave_max(am);
    const float sc = fmaxf(am, 1e-12f) / E4M3_MAX, inv = 1.f / sc;
    uint2* yq = (uint2*)((unsigned char*)y + row * ldy);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] *= inv;
      yq[lane + 64 * j] = to_e4m3x8(v[j]);
    }
    if (lane == 0) ys[row] = sc;
  } else {
    bf16x8* yr = (bf16x8*)(y + row * ldy);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const bf16x8 wv = wr[lane + 64 * j];
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(v[j][e] * r * bf2f((unsigned short)wv[e]));
      yr[lane + 64 * j] = o;
    }
  }
}

// bf16 rows -> e4m3 rows + per-row scales; one wave per row, cols == 512 * NC
template <int NC>
__global__ __launch_bounds__(256) void quant_rows(const unsigned short* __restrict__ x, unsigned char* __restrict__ y,
                                                  float* __restrict__ ys, int rows, long ldx, long ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16x8* xr = (const bf16x8*)(x + row * ldx);
  float v[NC][8];
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const bf16x8 h = xr[lane + 64 * j];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[j][e] = bf2f((unsigned short)h[e]);
      am = fmaxf(am, fabsf(v[j][e]));
    }
  }
  am = wave_max(am);
  const float sc = fmaxf(am, 1e-12f) / E4M3_MAX, inv = 1.f / sc;
  uint2* yq = (uint2*)(y + row * ldy);
#pragma unroll
  for (int j = 0; j < NC; ++j) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[j][e] *= inv;
    yq[lane + 64 * j] = to_e4m3x8(v[j]);
  }
  if (lane == 0) ys[row] = sc;
}

// SwiGLU with per-row e4m3 output: one 256-thread block per row, CPT 8-wide
// chunks per thread held in registers across the block's amax reduction.
template <int CPT>
__global__ __launch_bounds__(256) void silu_mul_q8(const unsigned short* __restrict__ gu, unsigned char* __restrict__ out,
                                                   float* __restrict__ ys, int inter, long ld_in, long ld_out) {
  __shared__ float red[4];
  const long r = blockIdx.x;
  const int tid = threadIdx.x, nch = inter / 8;
  const bf16x8* gp = (const bf16x8*)(gu + r * ld_in);
  const bf16x8* up = (const bf16x8*)(gu + r * ld_in + inter);
  float v[CPT][8];
  float am = 0.f;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = tid + 256 * k;
    if (c < nch) {
      const bf16x8 g = __builtin_nontemporal_load(gp + c);
      const bf16x8 u = __builtin_nontemporal_load(up + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gf = bf2f((unsigned short)g[e]);
        // round through bf16 like the bf16 path, so both paths quantise the same values
        v[k][e] = bf2f(f2bf(gf / (1.0f + __expf(-gf)) * bf2f((unsigned short)u[e])));
        am = fmaxf(am, fabsf(v[k][e]));
      }
    }
  }
  am = wave_max(am);
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = fmaxf(am, 1e-12f) / E4M3_MAX, inv = 1.f / sc;
  uint2* oq = (uint2*)(out + r * ld_out);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = tid + 256 * k;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[k][e] *= inv;
      oq[c] = to_e4m3x8(v[k]);
    }
  }
  if (tid == 0) ys[r] = sc;
}

// Thread = one 8-wide chunk of the first half of one (token, head); it also
// owns the matching chunk of the second half (rotate-half pairs i, i + hd/2).
__global__ __launch_bounds__(256) void rope_qkv(unsigned short* __restrict__ qkv, const float* __restrict__ cosv,
                                                const float* __restrict__ sinv, const int* __restrict__ pos,
                                                long tokens, int heads, int hd, long ld, int seq) {
  const int cph = hd / 16;  // chunks per head (first half)
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= tokens * heads * cph) return;
  const long t = idx / (heads * cph);
  const int rem = (int)(idx - t * heads * cph);
  const int h = rem / cph, c = rem - h * cph;
  const int p = pos != nullptr ? pos[t] : (int)(t % seq);
  unsigned short* base = qkv + t * ld + (long)h * hd + 8 * c;
  bf16x8* p1 = (bf16x8*)base;
  bf16x8* p2 = (bf16x8*)(base + hd / 2);
  const bf16x8 a = *p1, b = *p2;
  const f32x4* cp = (const f32x4*)(cosv + (long)p * (hd / 2) + 8 * c);
  const f32x4* sp = (const f32x4*)(sinv + (long)p * (hd / 2) + 8 * c);
  const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
  bf16x8 o1, o2;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float cs = e < 4 ? c0[e] : c1[e - 4];
    const float sn = e < 4 ? s0[e] : s1[e - 4];
    const float x1 = bf2f((unsigned short)a[e]), x2 = bf2f((unsigned short)b[e]);
    o1[e] = (short)f2bf(rope_lo(x1, x2, cs, sn));
    o2[e] = (short)f2bf(rope_hi(x1, x2, cs, sn));
  }
  *p1 = o1;
  *p2 = o2;
}

__global__ __launch_bounds__(256) void silu_mul(const unsigned short* __restrict__ gu, unsigned short* __restrict__ out,
                                                long rows, int inter, long ld_in, long ld_out) {
  const int cpr = inter / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * cpr) return;
  const long r = idx / cpr;
  const int c = (int)(idx - r * cpr);
  const bf16x8 g = __builtin_nontemporal_load((const bf16x8*)(gu + r * ld_in) + c);
  const bf16x8 u = __builtin_nontemporal_load((const bf16x8*)(gu + r * ld_in + inter) + c);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gf = bf2f((unsigned short)g[e]);
    o[e] = (short)f2bf(gf / (1.0f + __expf(-gf)) * bf2f((unsigned short)u[e]));
  }
  ((bf16x8*)(out + r * ld_out))[c] = o;
}

// Split-K reduce fused with the residual add and the RMSNorm that follow a
// decode projection (o, down): d = bf16(sum_s P[s][row]) with the slice order
// and rounding of kgs::splitk_reduce, x' = bf16(x + d) written back, y =
// rmsnorm(x') * w. One 256-thread workgroup per row (a decode batch of 256
// rows fills the 256 CUs; add_rmsnorm's wave-per-row grid would use 64 of
// them); thread t owns the 8-column chunks t + 256 j, cols == 2048 * NJ. The
// partial tiles never round-trip through a bf16 delta in HBM and the separate
// add_rmsnorm launch disappears.
// NSL > 0: the slice count at compile time, so every partial load of a thread
// is issued before the first add (a run-time slice loop waits out one cache
// latency per slice); 0 = run-time count.
template <int NJ, int NSL>
__global__ __launch_bounds__(256) void splitk_add_rmsnorm(const float* __restrict__ P, int nslice, long MN,
                                                          unsigned short* __restrict__ x,
                                                          const unsigned short* __restrict__ w,
                                                          unsigned short* __restrict__ y, int cols, long ldx,
                                                          long ldy, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x, t = threadIdx.x;
  bf16x8* xr = (bf16x8*)(x + row * ldx);
  // the residual chunks and the norm weight are loaded next to the partials:
  // the weight would otherwise cost a second memory round trip after the
  // row-sum barrier
  const bf16x8* wr = (const bf16x8*)w;
  bf16x8 xin[NJ], wv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    xin[j] = xr[t + 256 * j];
    wv[j] = wr[t + 256 * j];
  }
  float v[NJ][8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const long e = (long)row * cols + 8 * (t + 256 * j);
    f32x4 a, b;
    if constexpr (NSL > 0) {
      f32x4 pa[NSL], pb[NSL];
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) {
        pa[sl] = *(const f32x4*)(P + sl * MN + e);
        pb[sl] = *(const f32x4*)(P + sl * MN + e + 4);
      }
      a = pa[0];
      b = pb[0];
#pragma unroll
      for (int sl = 1; sl < NSL; ++sl) {
        a += pa[sl];
        b += pb[sl];
      }
    } else {
      a = *(const f32x4*)(P + e);
      b = *(const f32x4*)(P + e + 4);
      for (int sl = 1; sl < nslice; ++sl) {
        a += *(const f32x4*)(P + sl * MN + e);
        b += *(const f32x4*)(P + sl * MN + e + 4);
      }
    }
    const bf16x8 xv = xin[j];
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = bf2f(f2bf(k < 4 ? a[k] : b[k - 4]));
      o[k] = (short)f2bf(bf2f((unsigned short)xv[k]) + d);
      v[j][k] = bf2f((unsigned short)o[k]);
      ss += v[j][k] * v[j][k];
    }
    xr[t + 256 * j] = o;
  }
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  ss = (red[0] + red[1]) + (red[2] + red[3]);
  const float r = rsqrtf(ss / (float)cols + eps);
  bf16x8* yr = (bf16x8*)(y + row * ldy);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (short)f2bf(v[j][k] * r * bf2f((unsigned short)wv[j][k]));
    yr[t + 256 * j] = o;
  }
}

// Greedy decoding: argmax over each row of [rows, cols] bf16 logits, int64 out,
// torch.argmax's answer (the first index of the maximum; NaN counts as the
// maximum). One 1024-thread workgroup per row: a 128k-vocab row is 16 wide
// loads per thread (torch's generic reduce ran 40 us for ONE such row).
__device__ __forceinline__ bool am_better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(1024) void argmax_rows(const unsigned short* __restrict__ x, long long* __restrict__ out,
                                                    int cols, long ld) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x, t = threadIdx.x;
  const bf16x8* xr = (const bf16x8*)(x + row * ld);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  // eight 16-B loads per thread in flight (clamped indices, no branches around
  // the loads): a load-compare chain would wait out one memory latency per load
  const int nch = cols / 8;
  for (int c0 = t; c0 < nch; c0 += 1024 * 8) {
    bf16x8 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_nontemporal_load(xr + min(c0 + 1024 * j, nch - 1));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + 1024 * j;
      if (c >= nch) break;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f((unsigned short)v[j][e]);
        if (am_better(f, 8 * c + e, bv, bi)) {
          bv = f;
          bi = 8 * c + e;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (am_better(ov, oi, bv, bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if ((t & 63) == 0) {
    sv[t >> 6] = bv;
    si[t >> 6] = bi;
  }
  __syncthreads();
  if (t < 64) {
    bv = t < 16 ? sv[t] : -INFINITY;
    bi = t < 16 ? si[t] : 0x7fffffff;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (am_better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (t == 0) out[row] = bi == 0x7fffffff ? 0 : bi;
  }
}

}  // namespace tfm
}  // namespace kgs

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// x: [rows, ld] bf16 logits (cols % 8 == 0, ld % 8 == 0, 16-B aligned); out: int64 [rows]
KGS_EXPORT int kgs_argmax_rows_bf16(const void* x, long long* out, int rows, int cols, long ld, hipStream_t s) {
  if (rows < 0 || cols <= 0 || ld < cols) return KGS_ERR_SHAPE;
  if (cols % 8 || ld % 8 || !al16(x)) return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(kgs::tfm::argmax_rows, dim3(rows), dim3(1024), 0, s, (const unsigned short*)x, out, cols, ld);
  return (int)hipGetLastError();
}

// P: nslice fp32 partial products [nslice][rows][cols] (gemm_nt_w4x without its
// reduce); x: [rows, ldx] residual stream, updated in place; w: [cols]; y: out.
// cols a multiple of 2048 up to 8192.
KGS_EXPORT int kgs_splitk_add_rmsnorm_bf16(const float* P, int nslice, void* x, const void* w, void* y, int rows,
                                          int cols, long ldx, long ldy, float eps, hipStream_t s) {
  if (rows < 0 || cols <= 0 || nslice <= 0) return KGS_ERR_SHAPE;
  if (cols % 2048 || cols > 8192 || ldx < cols || ldy < cols) return KGS_ERR_SHAPE;
  if (!al16(P) || !al16(x) || !al16(w) || !al16(y) || ldx % 8 || ldy % 8) return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  using namespace kgs::tfm;
  const long MN = (long)rows * cols;
  auto X = (unsigned short*)x;
  auto W = (const unsigned short*)w;
  auto Y = (unsigned short*)y;
  const int nj = cols / 2048;
  if (nj < 1 || nj > 4) return KGS_ERR_SHAPE;
#define KGS_SARN(NJ, NSL)                                                                                           \
  hipLaunchKernelGGL((splitk_add_rmsnorm<NJ, NSL>), dim3(rows), dim3(256), 0, s, P, nslice, MN, X, W, Y, cols, ldx, \
                     ldy, eps)
#define KGS_SARN_NJ(NJ)                                           \
  switch (nslice) {                                               \
    case 2: KGS_SARN(NJ, 2); break;                               \
    case 4: KGS_SARN(NJ, 4); break;                               \
    case 8: KGS_SARN(NJ, 8); break;                               \
    default: KGS_SARN(NJ, 0); break;                              \
  }
  switch (nj) {
    case 1: KGS_SARN_NJ(1); break;
    case 2: KGS_SARN_NJ(2); break;
    case 3: KGS_SARN_NJ(3); break;
    default: KGS_SARN_NJ(4); break;
  }
#undef KGS_SARN_NJ
#undef KGS_SARN
  return (int)hipGetLastError();
}

// x: [rows, cols] residual stream; d: optional delta (same ld) -- when given,
// xo = x + d is written (xo may alias x) and normalised; w: [cols]; y: out.
// cols must be a multiple of 512 up to 8192; ld multiples of 8.
KGS_EXPORT int kgs_add_rmsnorm_bf16(void* x, const void* d, void* xo, const void* w, void* y, int rows, int cols,
                                   long ldx, long ldy, float eps, hipStream_t s) {
  if (rows < 0 || cols <= 0) return KGS_ERR_SHAPE;
  if (cols % 512 || cols > 8192 || ldx < cols || ldy < cols) return KGS_ERR_SHAPE;
  if (!al16(x) || !al16(w) || !al16(y) || (d && (!al16(d) || !al16(xo))) || ldx % 8 || ldy % 8) return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  if (d != nullptr && xo == nullptr) xo = x;
  using namespace kgs::tfm;
  const dim3 g((rows + 3) / 4), b(256);
  auto X = (unsigned short*)x;
  auto D = (const unsigned short*)d;
  auto XO = (unsigned short*)xo;
  auto W = (const unsigned short*)w;
  auto Y = (unsigned short*)y;
  switch (cols / 512) {
#define KGS_NC(n) \
  case n: hipLaunchKernelGGL(add_rmsnorm<n>, g, b, 0, s, X, D, XO, W, Y, rows, ldx, ldy, eps); break;
    KGS_NC(1) KGS_NC(2) KGS_NC(3) KGS_NC(4) KGS_NC(5) KGS_NC(6) KGS_NC(7) KGS_NC(8)
    KGS_NC(9) KGS_NC(10) KGS_NC(11) KGS_NC(12) KGS_NC(13) KGS_NC(14) KGS_NC(15) KGS_NC(16)
#undef KGS_NC
    default: return KGS_ERR_SHAPE;
  }
  return (int)hipGetLastError();
}

// qkv: [tokens, ld] with the `heads` rotated heads (q heads then k heads)
// first; cos/sin: fp32 [max_pos, hd/2]; pos: optional int32 [tokens], else
// position = token % seq (batch-major prefill).
KGS_EXPORT int kgs_rope_qkv_bf16(void* qkv, const float* cosv, const float* sinv, const int* pos, long tokens,
                                int heads, int hd, long ld, int seq, hipStream_t s) {
  if (tokens < 0 || heads <= 0 || hd <= 0 || seq <= 0) return KGS_ERR_SHAPE;
  if (hd % 16 || ld < (long)heads * hd) return KGS_ERR_SHAPE;
  if (!al16(qkv) || !al16(cosv) || !al16(sinv) || ld % 8) return KGS_ERR_ALIGN;
  const long n = tokens * heads * (hd / 16);
  if (n == 0) return 0;
  hipLaunchKernelGGL(kgs::tfm::rope_qkv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (unsigned short*)qkv, cosv, sinv, pos, tokens, heads, hd, ld, seq);
  return (int)hipGetLastError();
}

// gu: [rows, ld_in] holding gate (cols [0, inter)) and up (cols [inter, 2*inter));
// out: [rows, ld_out] = silu(gate) * up.
KGS_EXPORT int kgs_silu_mul_bf16(const void* gu, void* out, long rows, int inter, long ld_in, long ld_out,
                                hipStream_t s) {
  if (rows < 0 || inter <= 0 || inter % 8 || ld_in < 2L * inter || ld_out < inter) return KGS_ERR_SHAPE;
  if (!al16(gu) || !al16(out) || ld_in % 8 || ld_out % 8) return KGS_ERR_ALIGN;
  const long n = rows * (inter / 8);
  if (n == 0) return 0;
  hipLaunchKernelGGL(kgs::tfm::silu_mul, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (const unsigned short*)gu, (unsigned short*)out, rows, inter, ld_in, ld_out);
  return (int)hipGetLastError();
}

// fp8 (e4m3) output with per-row scales ys[rows]: y is [rows, ldy] bytes.
KGS_EXPORT int kgs_add_rmsnorm_fp8(void* x, const void* d, void* xo, const void* w, void* y, float* ys, int rows,
                                  int cols, long ldx, long ldy, float eps, hipStream_t s) {
  if (rows < 0 || cols <= 0) return KGS_ERR_SHAPE;
  if (cols % 512 || cols > 8192 || ldx < cols || ldy < cols) return KGS_ERR_SHAPE;
  if (!al16(x) || !al16(w) || !al16(y) || ((uintptr_t)ys & 3) || (d && (!al16(d) || !al16(xo))) || ldx % 8 ||
      ldy % 16)
    return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  if (d != nullptr && xo == nullptr) xo = x;
  using namespace kgs::tfm;
  const dim3 g((rows + 3) / 4), b(256);
  auto X = (unsigned short*)x;
  auto D = (const unsigned short*)d;
  auto XO = (unsigned short*)xo;
  auto W = (const unsigned short*)w;
  auto Y = (unsigned short*)y;
  switch (cols / 512) {
#define KGS_NC(n) \
  case n: hipLaunchKernelGGL((add_rmsnorm<n, true>), g, b, 0, s, X, D, XO, W, Y, rows, ldx, ldy, eps, ys); break;
    KGS_NC(1) KGS_NC(2) KGS_NC(4) KGS_NC(6) KGS_NC(8) KGS_NC(10) KGS_NC(12) KGS_NC(16)
#undef KGS_NC
    default: return KGS_ERR_SHAPE;
  }
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_quant_rows_fp8(const void* x, void* y, float* ys, int rows, int cols, long ldx, long ldy,
                                 hipStream_t s) {
  if (rows < 0 || cols <= 0 || cols % 512 || cols > 8192 || ldx < cols || ldy < cols) return KGS_ERR_SHAPE;
  if (!al16(x) || !al16(y) || ((uintptr_t)ys & 3) || ldx % 8 || ldy % 16) return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  using namespace kgs::tfm;
  const dim3 g((rows + 3) / 4), b(256);
  auto X = (const unsigned short*)x;
  auto Y = (unsigned char*)y;
  switch (cols / 512) {
#define KGS_NC(n) \
  case n: hipLaunchKernelGGL(quant_rows<n>, g, b, 0, s, X, Y, ys, rows, ldx, ldy); break;
    KGS_NC(1) KGS_NC(2) KGS_NC(4) KGS_NC(6) KGS_NC(8) KGS_NC(10) KGS_NC(12) KGS_NC(16)
#undef KGS_NC
    default: return KGS_ERR_SHAPE;
  }
  return (int)hipGetLastError();
}

// silu(gate) * up -> e4m3 [rows, ld_out] bytes + per-row scales; inter <= 32768.
KGS_EXPORT int kgs_silu_mul_fp8(const void* gu, void* out, float* ys, long rows, int inter, long ld_in, long ld_out,
                               hipStream_t s) {
  if (rows < 0 || inter <= 0 || inter % 8 || inter > 32768 || ld_in < 2L * inter || ld_out < inter)
    return KGS_ERR_SHAPE;
  if (!al16(gu) || !al16(out) || ((uintptr_t)ys & 3) || ld_in % 8 || ld_out % 16) return KGS_ERR_ALIGN;
  if (rows == 0) return 0;
  if (rows > 0x7fffffff) return KGS_ERR_SHAPE;
  using namespace kgs::tfm;
  const int cpt = (inter / 8 + 255) / 256;
  auto G = (const unsigned short*)gu;
  auto O = (unsigned char*)out;
  const dim3 g((unsigned)rows), b(256);
  switch (cpt) {
#define KGS_CPT(n) \
  case n: hipLaunchKernelGGL(silu_mul_q8<n>, g, b, 0, s, G, O, ys, inter, ld_in, ld_out); break;
    KGS_CPT(1) KGS_CPT(2) KGS_CPT(3) KGS_CPT(4) KGS_CPT(5) KGS_CPT(6) KGS_CPT(7) KGS_CPT(8)
    KGS_CPT(9) KGS_CPT(10) KGS_CPT(11) KGS_CPT(12) KGS_CPT(13) KGS_CPT(14) KGS_CPT(15) KGS_CPT(16)
#undef KGS_CPT
    default: return KGS_ERR_SHAPE;
  }
  return (int)hipGetLastError();
}
