// Shared device helpers for the kgs gfx950 kernels.
//
// Everything here is written for CDNA4 (gfx950, wave64, MFMA, LDS-DMA). There is
// no CUDA path and no multi-arch dispatch: kernels are compiled with
// `--offload-arch=gfx950` only (see kgs/utils/build.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define KGS_LDS __attribute__((address_space(3)))
#define KGS_GLB __attribute__((address_space(1)))

#define KGS_EXPORT extern "C" __attribute__((visibility("default")))

// Error codes returned by the C ABI (0 = success, >0 = hipError_t, <0 = ours).
enum {
  KGS_OK = 0,
  KGS_ERR_SHAPE = -1,      // non-positive or overflowing dimension
  KGS_ERR_ALIGN = -2,      // pointer / leading-dimension alignment
  KGS_ERR_ARG = -3,        // unknown enum value
};

namespace kgs {

// Round-to-nearest-even f32 -> bf16 bits. hipcc lowers the __bf16 cast to
// v_cvt_pk_bf16_f32 on gfx950, which also keeps NaNs NaN
// (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ unsigned short f2bf(float x) {
  __bf16 h = (__bf16)x;
  return __builtin_bit_cast(unsigned short, h);
}

__device__ __forceinline__ float bf2f(unsigned short h) {
  return __builtin_bit_cast(float, ((unsigned)h) << 16);
}

// RoPE rotation of the pair (x1, x2) = (d, d + 64): (x1 cos - x2 sin,
// x2 cos + x1 sin), each as ONE fma on the other element's rounded product.
// Every kernel that rotates uses these (rope_cache and its split-K / grouped
// forms, the fused skinny-GEMM and attention prologues, the prompt RoPE): they
// are compared bit for bit, and hipcc's fp-contract would otherwise choose per
// call site which product to fuse.
__device__ __forceinline__ float rope_lo(float x1, float x2, float cs, float sn) {
  return __builtin_fmaf(x1, cs, -(x2 * sn));
}
__device__ __forceinline__ float rope_hi(float x1, float x2, float cs, float sn) {
  return __builtin_fmaf(x2, cs, x1 * sn);
}

// Two f32 -> a packed bf16 pair in one v_cvt_pk_bf16_f32. Two f2bf calls
// compile to two conversions (each with a dummy second source) plus a v_perm:
// three VALU ops where one does, on every epilogue and P-fragment pack.
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}

// 8 bf16 (one 16-B store's worth): bf16(x + d) per element, as add_rmsnorm rounds
// the residual add (EPI_ADDC: x the stored residual, d the rounded product).
__device__ __forceinline__ uint4 add_bf16x8(uint4 x, uint4 d) {
  const unsigned xs[4] = {x.x, x.y, x.z, x.w}, ds[4] = {d.x, d.y, d.z, d.w};
  unsigned o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = bf2f((unsigned short)(xs[k] & 0xffff)) + bf2f((unsigned short)(ds[k] & 0xffff));
    const float hi = bf2f((unsigned short)(xs[k] >> 16)) + bf2f((unsigned short)(ds[k] >> 16));
    o[k] = pack_bf16x2(lo, hi);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// s[base .. base + 7] -> a bf16x8 MFMA fragment, four v_cvt_pk_bf16_f32
template <class V>
__device__ __forceinline__ bf16x8 pack_bf16x8(const V& s, int base) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t u = {pack_bf16x2(s[base], s[base + 1]), pack_bf16x2(s[base + 2], s[base + 3]),
                     pack_bf16x2(s[base + 4], s[base + 5]), pack_bf16x2(s[base + 6], s[base + 7])};
  return __builtin_bit_cast(bf16x8, u);
}

// Cross-lane exchanges on gfx950's half-swaps (one VALU op each, no LDS round
// trip like the ds_bpermute behind __shfl_xor). With both operands = x,
// permlane32_swap returns {x of lanes 0-31 in both halves, x of lanes 32-63 in
// both halves}; permlane16_swap does the same for each pair of 16-lane rows.
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), true, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), true, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), true, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor16_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), true, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// the value of lane l ^ 32
__device__ __forceinline__ float lane_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), true, false);
  return __uint_as_float((__lane_id() & 32) ? r[0] : r[1]);
}

// 16-byte LDS-DMA: each lane's 16 global bytes land at lds_base + lane*16
// (lds_base must be wave-uniform). The swizzle, if any, is applied to the
// per-lane *source* address (cdna_hip_programming.md rule 21).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((KGS_GLB void*)gsrc, (KGS_LDS void*)lds_base, 16, 0, 0);
}

// Bijective XCD-aware remap of a 1-D grid: blocks that the dispatcher deals to
// the same XCD (bid % 8 equal) get a contiguous range of logical ids, so
// neighbouring output tiles share that XCD's L2 (guide T1).
__host__ __device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Epilogue activations (fused into the GEMM store).
// EPI_ADDC: C = bf16(C + bf16(acc)), the residual add of a projection read and
// written in the store (round 5, the prompt pass's o / down: add_rmsnorm's add
// with the same two roundings, leaving it a plain rmsnorm). No bias.
enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RELU = 3, EPI_BIAS_SILU = 4, EPI_ADDC = 5 };

template <int EPI>
constexpr bool epi_bias() { return EPI != EPI_NONE && EPI != EPI_ADDC; }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  // tanh via exp: stable for |u| large.
  float e = __expf(-2.0f * fabsf(u));
  float t = (1.0f - e) / (1.0f + e);
  t = u < 0.f ? -t : t;
  return 0.5f * x * (1.0f + t);
}

template <int EPI>
__device__ __forceinline__ float epilogue(float v, float b) {
  if constexpr (EPI == EPI_NONE || EPI == EPI_ADDC) return v;
  v += b;
  if constexpr (EPI == EPI_BIAS_GELU) return gelu_tanh(v);
  if constexpr (EPI == EPI_BIAS_RELU) return v > 0.f ? v : 0.f;
  if constexpr (EPI == EPI_BIAS_SILU) return v / (1.0f + __expf(-v));
  return v;
}

}  // namespace kgs
