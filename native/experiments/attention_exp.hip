// Measured alternatives of the flash-attention forward (native/kernels/attention.hip):
// the one-wave-per-SIMD, named-register kernel of attention_w4.h. Built into the
// opt-in libkgs_experiments.so; numbers in profiles/r4/attention/.
#include "attention_w4.h"

// Same operand contract as kgs_attn_fwd_bf16_ex, with S % 256 == 0; `stamps`
// (optional) selects the timing build.
KGS_EXPORT int kgs_exp_attn4_fwd_bf16(const void* q, const void* k, const void* v, void* o, int B, int S, int Sk,
                                      int H, int HKV, int hd, long ldq, long ldk, long ldv, long ldo, float scale,
                                      int causal, void* stamps, int variant, hipStream_t s) {
  using namespace kgs::attn4;
  if (B <= 0 || S <= 0 || H <= 0 || HKV <= 0 || H % HKV) return KGS_ERR_SHAPE;
  if (hd != HD || S % QB || Sk < S || (Sk - S) % KB) return KGS_ERR_SHAPE;
  if (ldq < (long)H * HD || ldk < (long)HKV * HD || ldv < (long)HKV * HD || ldo < (long)H * HD) return KGS_ERR_SHAPE;
  const uintptr_t al = (uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o;
  if ((al & 15) || (ldq | ldk | ldv | ldo) & 7) return KGS_ERR_ALIGN;
  const long nwg = (long)B * H * (S / QB);
  if (nwg > 0x7fffffff) return KGS_ERR_SHAPE;
  Args a{(const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o,
         ldq, ldk, ldv, ldo, B, S, H, HKV, scale * 1.4426950408889634f, causal ? 1 : 0, Sk, Sk - S,
         (long long*)stamps};
  // variant 0 only (a register-staged K/V variant measured slower and was
  // removed, profiles/r4/attention); stamps: the timing build,
  // long long[64 workgroups][4 waves][64 tiles][8]
  if (variant != 0) return KGS_ERR_ARG;
  if (stamps)
    hipLaunchKernelGGL(fwd<true>, dim3((unsigned)nwg), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(fwd<false>, dim3((unsigned)nwg), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
