// Launcher of the persistent four-wave bf16 GEMM (gemm_w4p.h) for the aligned
// fast path of kgs_gemm_bf16_nt (gemm_bf16.hip, variant 3 with K >= 384 and
// more 256x256 tiles than CUs). A separate translation unit so that it and
// gemm_bf16.hip compile in parallel.
//
// Measured routing (interleaved medians, TFLOP/s):
//  * persistent vs the one-shot grid of the same K-step: 8192^3 1654 vs 1628,
//    16384^2x8192 1628 vs 1602, 8192x28672x4096 1600 vs 1559
//    (profiles/r3/gemm_persistent_production.json);
//  * tall problems (M > N) take the mirrored order (GROUP_N, B's DMAs first),
//    as the one-shot kernel does (profiles/r3/gemm_long_k.md);
//  * long K (> 8192) takes tile groups of 8 instead of 4: 4096x8192x14336 1616
//    vs 1590, 8192x4096x14336 (mirror) 1612 vs 1597; at K = 8192 the two are
//    even (profiles/r3/gemm_persistent_maps_long_k.json).
#include "gemm_w4f8.h"
#include "gemm_w4p.h"

namespace kgs {

template <int EPI>
hipError_t launch_w4p(const unsigned short* A, const unsigned short* B, unsigned short* C, const unsigned short* bias,
                      int M, int N, int K, int lda, int ldb, int ldc, int cus, int* tq, hipStream_t s) {
  const int tiles = (M / 256) * (N / 256);
  const dim3 pg(tiles < cus ? tiles : cus);
  const bool tall = M > N, longk = K > 8192;
  if (tall && longk)
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 140000008>), pg, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                       tq);
  else if (tall)
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 140000000>), pg, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                       tq);
  else if (longk)
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 8>), pg, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc, tq);
  else if (EPI == EPI_NONE && tiles > 2 * cus && tiles <= 8 * cus && K / 64 >= 8)
    // 3-8 tiles per CU, plain C: stored non-temporally, and half of each tile's C deferred
    // (gemm_w4p.h DD 4, SPS 4: 16 of a lane's 32 units held in VGPRs and stored 4 at a time at
    // the end of the next tile's K-steps 0-3). Every tile change drains 32 MiB of C stores at
    // once (4 MiB per XCD, the whole L2) and the step waits for it (3.4 % of the 8192^3 bench
    // step, profiles/r5/gemm/store_drain); nt stores shorten the drain: 8192^3 +0.5 / +0.5 /
    // +1.0 % on three boxes (profiles/r4/gemm/ntstore_sweep_boxD.json, profiles/r4/validate_b,
    // profiles/r5/gemm/store_drain); the deferral a further 0.41 / 0.40 / 0.46 % on three boxes
    // (profiles/r6/gemm/deferred). At 16 tiles per CU (16384^2x8192) nt measured -1.2 % and
    // the deferral nothing, and K < 512 has too few K-steps for the peeled ones.
    // (DD / SPS spelled per EPI so the other epilogues reuse their one instance of the default)
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 0, 1, EPI == EPI_NONE, false, 0, EPI == EPI_NONE ? 4 : 0,
                                         EPI == EPI_NONE ? 4 : 2>),
                       pg, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc, tq);
  else if (EPI == EPI_NONE && tiles > 2 * cus && tiles <= 8 * cus)
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 0, 1, EPI == EPI_NONE>), pg, dim3(256), 0, s, A, B, C, bias, M, N, K,
                       lda, ldb, ldc, tq);
  else
    hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI, 0>), pg, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc, tq);
  return hipGetLastError();
}

// SwiGLU (B = fused [gate; up] weight, N = 2I rows; C = [M, I]): the prefill
// gate|up, with the one-shot SwiGLU kernel's K-step and tile order (X 1000000),
// so the result is bitwise the one-shot kernel's
hipError_t launch_w4p_swiglu(const unsigned short* A, const unsigned short* B, unsigned short* C, int M, int N,
                             int K, int lda, int ldb, int ldc, int cus, int* tq, hipStream_t s) {
  const int tiles = (M / 256) * (N / 256);
  const dim3 pg(tiles < cus ? tiles : cus);
  hipLaunchKernelGGL((w4p::gemm_nt_w4p<EPI_NONE, 1000000>), pg, dim3(256), 0, s, A, B, C, nullptr, M, N, K, lda, ldb,
                     ldc, tq);
  return hipGetLastError();
}

#define KGS_LAUNCH_W4P(EPI)                                                                                         \
  template hipError_t launch_w4p<EPI>(const unsigned short*, const unsigned short*, unsigned short*,              \
                                      const unsigned short*, int, int, int, int, int, int, int, int*, hipStream_t);
KGS_LAUNCH_W4P(EPI_NONE)
KGS_LAUNCH_W4P(EPI_BIAS)
KGS_LAUNCH_W4P(EPI_BIAS_GELU)
KGS_LAUNCH_W4P(EPI_BIAS_RELU)
KGS_LAUNCH_W4P(EPI_BIAS_SILU)
KGS_LAUNCH_W4P(EPI_ADDC)
#undef KGS_LAUNCH_W4P

// fp8 (e4m3): lengths and leading dimensions of A / B in 16-bit words
template <int EPI>
hipError_t launch_fp8_w4p(const unsigned short* A, const unsigned short* B, unsigned short* C,
                          const unsigned short* bias, int M, int N, int Kw, int ldaw, int ldbw, int ldc, float alpha,
                          const float* alpha_ptr, int cus, int* tq, hipStream_t s) {
  // the bf16 kernel's maps, by bytes: tall problems the mirrored order, rows
  // longer than 16 KiB (Kw > 8192 words) tile groups of 8
  const int tiles = (M / 256) * (N / 256);
  const dim3 pg(tiles < cus ? tiles : cus);
  const bool tall = M > N, longk = Kw > 8192;
  if (tall && longk)
    hipLaunchKernelGGL((w4f8::gemm_fp8_w4p<EPI, 140000008>), pg, dim3(256), 0, s, A, B, C, bias, M, N, Kw, ldaw,
                       ldbw, ldc, alpha, alpha_ptr, tq);
  else if (tall)
    hipLaunchKernelGGL((w4f8::gemm_fp8_w4p<EPI, 140000000>), pg, dim3(256), 0, s, A, B, C, bias, M, N, Kw, ldaw,
                       ldbw, ldc, alpha, alpha_ptr, tq);
  else if (longk)
    hipLaunchKernelGGL((w4f8::gemm_fp8_w4p<EPI, 8>), pg, dim3(256), 0, s, A, B, C, bias, M, N, Kw, ldaw, ldbw, ldc,
                       alpha, alpha_ptr, tq);
  else
    hipLaunchKernelGGL((w4f8::gemm_fp8_w4p<EPI, 0>), pg, dim3(256), 0, s, A, B, C, bias, M, N, Kw, ldaw, ldbw, ldc,
                       alpha, alpha_ptr, tq);
  return hipGetLastError();
}

#define KGS_LAUNCH_FP8(EPI)                                                                                      \
  template hipError_t launch_fp8_w4p<EPI>(const unsigned short*, const unsigned short*, unsigned short*,        \
                                          const unsigned short*, int, int, int, int, int, int, float,           \
                                          const float*, int, int*, hipStream_t);
KGS_LAUNCH_FP8(EPI_NONE)
KGS_LAUNCH_FP8(EPI_BIAS)
KGS_LAUNCH_FP8(EPI_BIAS_GELU)
KGS_LAUNCH_FP8(EPI_BIAS_RELU)
KGS_LAUNCH_FP8(EPI_BIAS_SILU)
#undef KGS_LAUNCH_FP8

}  // namespace kgs
