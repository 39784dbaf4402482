// Fused decoder-block glue for gfx950: the HBM-bound ops between the GEMMs of a
// Llama-style block, each one pass over its tensors with 16-B accesses.
//
//   * add_rmsnorm : x' = x + d (bf16 residual stream, written back),
//                   y = rmsnorm(x') * w          -- one wave per row
//   * rope_qkv    : rotate-half (neox) RoPE on the q and k heads of the fused
//                   QKV projection output, in place, from an fp32 cos/sin table
//   * silu_mul    : SwiGLU's silu(g) * u from the fused gate|up output
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

// One wave per row; lane owns 16-B chunks lane + 64*j (j < NC) -- a wave reads
// 1 KB contiguous per j. cols == 512 * NC.
template <int NC>
__global__ __launch_bounds__(256) void add_rmsnorm(unsigned short* __restrict__ x, const unsigned short* __restrict__ d,
                                                   unsigned short* __restrict__ xo,
                                                   const unsigned short* __restrict__ w,
                                                   unsigned short* __restrict__ y, int rows, long ldx, long ldy,
                                                   float eps) {
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
    o1[e] = (short)f2bf(x1 * cs - x2 * sn);
    o2[e] = (short)f2bf(x2 * cs + x1 * sn);
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

}  // namespace tfm
}  // namespace kgs

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

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
