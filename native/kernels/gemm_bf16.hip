// bf16 GEMM for gfx950 (MI355X / CDNA4), hand-written on MFMA + LDS-DMA.
//
//   C[M,N] (bf16) = epilogue( A[M,K] · B[N,K]^T )      f32 accumulation
//
// Both operands are K-contiguous ("NT", the torch.nn.Linear weight layout), so
// every MFMA fragment is one 16-byte LDS read.
//
// Kernels (variant numbers are the C ABI's `variant` argument):
//
//  * gemm_nt_w4 -- the hot path since round 2 (aligned shapes, variant 3; see
//      gemm_w4.h): the same 256x256x64 tile and LDS image with four waves of
//      128x128, two barriers per 128-MFMA K-step. Interleaved against the
//      8-wave kernel below: +2-3 % at 4096^3..16384^2x8192.
//
//  * gemm_nt_256 -- the 8-wave ping-pong (aligned shapes), variant 1; still the
//      engine of the bounded / fp8 / K-major / split-K paths below.
//      256x256x64 block tile, 512 threads = 8 waves as 2(M) x 4(N), each wave
//      owns 128x64 of C as 2x2 quadrants of 64x32 (4x2 MFMA 16x16x32 tiles).
//      A and B K-tiles are split into 128-row halves (A0 A1 B0 B1, 16 KiB each)
//      staged by `global_load_lds_dwordx4` into a 2-deep ring (128 KiB LDS, one
//      workgroup per CU). The wave->row map is interleaved so that a quadrant
//      phase touches exactly one A half and one B half; with that, a half-tile
//      can be restaged independently of the other halves of its K-tile.
//
//      K-loop: 8 phases per iteration (2 K-tiles x 4 quadrants). Phase p:
//         ds_read the quadrant's fragments (8 / 4 / 8 / 4 x ds_read_b128)
//         issue one half-tile (2 x glds per wave), 7 half-tiles ahead
//         s_waitcnt vmcnt(10)           <- 5 half-tiles stay in flight
//         s_barrier ; lgkmcnt(0) ; 16 x MFMA ; s_barrier
//      Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave's
//      MFMA block overlaps its partner's LDS-read/DMA-issue block. The pipeline
//      itself (and the RAW/WAR accounting of its schedules, next to phase<>())
//      is in gemm_pipeline.h.
//      LDS image: 128-byte rows, 16-byte chunk c stored at c ^ ((row >> 1) & 7),
//      which makes every ds_read_b128 16-lane group hit 16 distinct bank slots
//      (conflict-free, SQ_LDS_BANK_CONFLICT = 0); the swizzle is applied to the
//      glds SOURCE address. Grid: one block per 256x256 tile, XCD-bijective
//      remap, then GROUP_M=4 grouped order so the 32 co-resident tiles of an
//      XCD form a 4x8 patch sharing A/B panels (L2 hit 81 % = 1 - 12/64).
//      Template S selects schedule knobs; the measured alternatives and timing
//      probes live in native/experiments/gemm_experiments.hip, built into a
//      separate opt-in libkgs_experiments.so (profiles/gemm_tuning.md).
//
//  * fp8 (kgs_gemm_fp8_nt) and the K-major layouts (kgs_gemm_bf16) are the same
//      pipeline with the scaled fp8 MFMA / ds_read_b64_tr_b16 fragments.
//
//  * gemm_nt_256<.., S|512> (variant 16, "bounded") -- the same pipeline for any
//      M, N and K % 8 == 0: operands are read by `buffer_load_dwordx4 ... lds`
//      through buffer resources that end at the last valid row, so rows past M/N
//      and K-chunks past K land as zeros; the store tail is predicated. `auto`
//      uses it whenever the aligned path does not apply.
//
//  * gemm_nt_generic (variant 2) -- any shape/stride (bounds-checked, register
//      staged, 128x128x32 tile). Used for odd K / strides and as the tests' twin.
//
// C ABI: kgs_gemm_bf16_nt / kgs_gemm_bf16 / kgs_gemm_fp8_nt (bottom of file), loaded from Python via ctypes
// (kgs/ops/_lib.py) and from the C++ benches.
//
// Reference parity: the reference (kind-gpu-sim) has no kernels at all -- its
// test pod only echoes (pods/rocm-gpu-test-pod.yaml:9, Readme.md:16-20). This is
// the in-pod hot path required by BASELINE.json configs 3-4.
#include "gemm_pipeline.h"
#include "gemm_w4.h"
#include "gemm_w4p.h"
#include "tile_queue.h"
#include "tile_queue_zero.h"

namespace kgs {

namespace gen {

// Generic bounds-checked NT GEMM: 128x128x32 tile, 256 threads (2x2 waves of
// 64x64), register-staged loads with zero fill, padded LDS rows.
constexpr int BM = 128, BN = 128, BK = 32;
constexpr int ROWB = BK * 2 + 16;  // 80-byte padded row

__device__ __forceinline__ bf16x8 load8(const unsigned short* __restrict__ P, int ld, int row, int nrows,
                                        int k, int K, bool vec_ok) {
  bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row >= nrows) return v;
  const unsigned short* p = P + (long)row * ld + k;
  if (vec_ok && k + 8 <= K) return *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (k + e < K) v[e] = (short)p[e];
  return v;
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_nt_generic(const unsigned short* __restrict__ A,
                                                       const unsigned short* __restrict__ B,
                                                       unsigned short* __restrict__ C,
                                                       const unsigned short* __restrict__ bias,
                                                       int M, int N, int K, int lda, int ldb, int ldc,
                                                       int vec_ok) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BM * ROWB];
  char* sA = smem;
  char* sB = smem + BM * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int tm = blockIdx.y, tn = blockIdx.x;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // each thread stages 2 chunks of A and 2 of B: row = tid/4 (+64), chunk = tid%4
  const int lr = tid >> 2, lc = tid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  for (int k0 = 0; k0 < K; k0 += BK) {
    bf16x8 a0 = load8(A, lda, m0 + lr, M, k0 + lc * 8, K, vec_ok);
    bf16x8 a1 = load8(A, lda, m0 + lr + 64, M, k0 + lc * 8, K, vec_ok);
    bf16x8 b0 = load8(B, ldb, n0 + lr, N, k0 + lc * 8, K, vec_ok);
    bf16x8 b1 = load8(B, ldb, n0 + lr + 64, N, k0 + lc * 8, K, vec_ok);
    __syncthreads();
    *(bf16x8*)(sA + lr * ROWB + lc * 16) = a0;
    *(bf16x8*)(sA + (lr + 64) * ROWB + lc * 16) = a1;
    *(bf16x8*)(sB + lr * ROWB + lc * 16) = b0;
    *(bf16x8*)(sB + (lr + 64) * ROWB + lc * 16) = b1;
    __syncthreads();
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(sA + (wr * 64 + i * 16 + fr) * ROWB + fq * 16);
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = *(const bf16x8*)(sB + (wc * 64 + n * 16 + fr) * ROWB + fq * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n], af[i], acc[i][n], 0, 0, 0);
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + wr * 64 + i * 16 + fr;
    if (row >= M) continue;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = n0 + wc * 64 + n * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (col + e < N) {
          float b = (EPI != EPI_NONE) ? bf2f(bias[col + e]) : 0.f;
          C[(long)row * ldc + col + e] = f2bf(epilogue<EPI>(acc[i][n][e], b));
        }
      }
    }
  }
}

}  // namespace gen

// Compute units of the current device (the persistent grid size), cached per device.
static int cu_count() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!n[dev]) {
    int v = 0;
    n[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n[dev];
}

// gemm_persistent.hip
hipError_t launch_w4p_swiglu(const unsigned short* A, const unsigned short* B, unsigned short* C, int M, int N,
                             int K, int lda, int ldb, int ldc, int cus, int* tq, hipStream_t s);
template <int EPI>
hipError_t launch_w4p(const unsigned short* A, const unsigned short* B, unsigned short* C, const unsigned short* bias,
                      int M, int N, int K, int lda, int ldb, int ldc, int cus, int* tq, hipStream_t s);

template <int EPI>
static hipError_t launch(int variant, const unsigned short* A, const unsigned short* B, unsigned short* C,
                         const unsigned short* bias, int M, int N, int K, int lda, int ldb, int ldc,
                         hipStream_t s) {
  // Production S = 7: balanced schedule, no s_setprio, GROUP_M 4 (measured best
  // at 4096^3..16384^2x8192 in interleaved A/B, profiles/gemm_tuning.md).
  const dim3 grid256((M / g256::BM) * (N / g256::BN));
  // persistent only with more tiles than CUs: with one tile per workgroup it
  // saves nothing and its ticket fetch costs (4096^3: 1483 vs 1543 one-shot)
  const bool pers = variant == 3 && K >= 384 && (M / 256) * (N / 256) > cu_count();
  int* tq = pers ? tile_queue(s) : nullptr;
  if (tq) {
    // the persistent four-wave kernel (gemm_persistent.hip, round 3)
    const hipError_t e = launch_w4p<EPI>(A, B, C, bias, M, N, K, lda, ldb, ldc, cu_count(), tq, s);
    if (e != hipSuccess) return e;
  } else if (variant == 3 || variant == 4) {
    using Kn = w4::Knobs<256, 256>;
    if (M > N) {
      // tall problems run the mirror image of the default schedule: GROUP_N tile
      // order (MAP 4) and B's DMAs first. The kernel is then what the default one
      // is for the transposed problem, which is the faster orientation: at
      // 8192x4096x14336 the default order made all eight XCDs of a wave read the
      // same B columns (1456-1531 TFLOP/s); the mirror runs 1587, as fast as
      // 4096x8192x14336 (profiles/r3/gemm_long_k.md)
      hipLaunchKernelGGL((w4::gemm_nt_w4<EPI, 256, 0, Kn::B1, Kn::R, Kn::P, Kn::ORD, 140000000>), grid256, dim3(256),
                         0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
    } else {
      hipLaunchKernelGGL((w4::gemm_nt_w4<EPI>), grid256, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
    }
  } else if (variant == 1) {
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb,
                       ldc, 1.0f, nullptr);
  } else if (variant == 16) {
    // the same pipeline on any M, N and K % 8 == 0: buffer-resource loads zero
    // the rows / K-chunks past the edges, stores are predicated
    const dim3 gridb(((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN));
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 512>), gridb, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb,
                       ldc, 1.0f, nullptr);
  } else {
    const int vec_ok = ((lda % 8) == 0 && (ldb % 8) == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0);
    dim3 grid((N + gen::BN - 1) / gen::BN, (M + gen::BM - 1) / gen::BM);
    hipLaunchKernelGGL(gen::gemm_nt_generic<EPI>, grid, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                       vec_ok);
  }
  return hipGetLastError();
}

}  // namespace kgs

static_assert(kgs::w4p::TQ_ERR_WORD == kgs::TQ_ERR, "the kernels' error word is the pool's");

// Ticket-slot pool of the persistent GEMMs on device `dev` (tile_queue.h):
// out = {slots allocated, stream-owned, capture-owned, nullptr fallbacks, failed growths}.
KGS_EXPORT int kgs_tile_queue_stats(int dev, long* out) {
  const kgs::TileQueueStats st = kgs::tile_queue_stats(dev);
  out[0] = st.slots;
  out[1] = st.stream_slots;
  out[2] = st.capture_slots;
  out[3] = st.fallbacks;
  out[4] = st.grow_failures;
  return 0;
}

// Test hook: the ticket slot stream `s` owns (taken now if it has none), so a
// GPU test can corrupt it and check that the persistent kernels report the
// impossible tickets instead of faulting or skipping tiles silently.
KGS_EXPORT int kgs_tile_queue_slot(hipStream_t s, void** out) {
  *out = kgs::tile_queue(s);
  return *out ? 0 : KGS_ERR_ARG;
}

// The quiescent-pool invariant (tile_queue.h tile_queue_check): out = {dirty
// slots, dirty words, first dirty value, its word index, the first dirty slot's
// address, its 16 words, slots with the impossible-ticket error word set}. No
// GEMM may be in flight.
KGS_EXPORT int kgs_tile_queue_check(int dev, long* out) { return kgs::tile_queue_check(dev, out); }

// Can the 256x256 pipelined kernel take this problem?
KGS_EXPORT int kgs_gemm_bf16_nt_fast_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda,
                                        int ldb, int ldc) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (M % 256 || N % 256 || K % 128) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8) return 0;  // 16-B operand DMA and 16-B C stores
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return 0;
  // 32-bit per-lane offsets: (255 rows) * ld must fit
  if ((long)lda * 256 >= (1L << 31) || (long)ldb * 256 >= (1L << 31)) return 0;
  return 1;
}

// Can the four-wave kernel (variant 3) take this problem? The fast-path shape
// rules plus 32-bit buffer-resource byte offsets over a 256-row panel.
KGS_EXPORT int kgs_gemm_bf16_nt_w4_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda,
                                      int ldb, int ldc) {
  if (!kgs_gemm_bf16_nt_fast_ok(A, B, C, M, N, K, lda, ldb, ldc)) return 0;
  return (long)lda * 512 < (1L << 31) && (long)ldb * 512 < (1L << 31);
}

// Can the bounded 256x256 kernel (variant 16) take this problem? Any M, N;
// K, the leading dimensions and the pointers in 16-B units.
KGS_EXPORT int kgs_gemm_bf16_nt_bounded_ok(const void* A, const void* B, const void* C, int M, int N, int K,
                                           int lda, int ldb, int ldc) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % 8 || lda % 8 || ldb % 8 || ldc % 8) return 0;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return 0;
  // buffer offsets are 32-bit: 256 rows * ld * 2 B must stay below the OOB offset
  if ((long)lda * 512 >= kgs::g256::OOB_OFFSET || (long)ldb * 512 >= kgs::g256::OOB_OFFSET) return 0;
  return 1;
}

KGS_EXPORT int kgs_gemm_bf16_nt_w4x_ex(const void* A, const void* B, void* C, float* ws, int M, int N, int K,
                                       int lda, int ldb, int ldc, int bn, int nslice, int bm, int flags,
                                       hipStream_t stream);

// variant: 0 = auto, 1 = force the 256x256 8-wave ping-pong, 2 = force generic,
//          3 = force the four-wave kernel (256x256 tiles; persistent when
//          K >= 384 and there are more tiles than CUs), 4 = the four-wave
//          kernel's one-shot grid (one workgroup
//          per tile), 16 = force the bounded 256x256 pipeline. Anything else
//          is rejected.
// Auto on a grid of at most 128 256x256 tiles (half the CUs or fewer) runs the
// four-wave kernel on smaller tiles: 256x128 / 128x256 up to 128 tiles, 128x128
// up to 64 -- 1.13-1.23x hipBLASLt there, where 256x256 tiles leave CUs idle
// (profiles/r3/gemm_small_grid.json).
// C[M, N] = bf16(C + bf16(A . B^T)): a projection with the residual add in its
// epilogue (EPI_ADDC; the prompt pass's o / down, whose add_rmsnorm becomes a
// plain rmsnorm -- same roundings, so bitwise the unfused pair). The aligned
// four-wave path only (kgs_gemm_bf16_nt_w4_ok); persistent with more tiles
// than CUs on an eager stream, else (and in any hipGraph capture) the one-shot
// grid (tall problems in the mirrored order).
KGS_EXPORT int kgs_gemm_bf16_nt_addc(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                     int ldc, hipStream_t stream) {
  using namespace kgs;
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (!kgs_gemm_bf16_nt_w4_ok(A, B, C, M, N, K, lda, ldb, ldc)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  const long tiles = (long)(M / 256) * (N / 256);
  // A captured launch never takes a ticket slot: tile_queue.h lets one exec
  // replayed concurrently with itself compute a tile twice, and this epilogue
  // (C += A.B^T) would then add twice. Captures run the one-shot grid.
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return KGS_ERR_ARG;
  int* tq = (K >= 384 && tiles > cu_count() && cs == hipStreamCaptureStatusNone) ? tile_queue(stream) : nullptr;
  if (tq) {
    const hipError_t e = launch_w4p<EPI_ADDC>(a, b, c, nullptr, M, N, K, lda, ldb, ldc, cu_count(), tq, stream);
    return e == hipSuccess ? 0 : (int)e;
  }
  using Kn = w4::Knobs<256, 256>;
  const dim3 grid((unsigned)tiles);
  if (M > N)
    hipLaunchKernelGGL((w4::gemm_nt_w4<EPI_ADDC, 256, 0, Kn::B1, Kn::R, Kn::P, Kn::ORD, 140000000>), grid, dim3(256), 0,
                       stream, a, b, c, nullptr, M, N, K, lda, ldb, ldc);
  else
    hipLaunchKernelGGL((w4::gemm_nt_w4<EPI_ADDC>), grid, dim3(256), 0, stream, a, b, c, nullptr, M, N, K, lda, ldb,
                       ldc);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_gemm_bf16_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                                int ldb, int ldc, int epi, int variant, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (epi != kgs::EPI_NONE && bias == nullptr) return KGS_ERR_ARG;
  // the fast epilogue reads the bias 4 elements (8 B) at a time
  const int bias_ok = epi == kgs::EPI_NONE || (uintptr_t)bias % 8 == 0;
  const int fast = kgs_gemm_bf16_nt_fast_ok(A, B, C, M, N, K, lda, ldb, ldc) && bias_ok;
  const int w4 = kgs_gemm_bf16_nt_w4_ok(A, B, C, M, N, K, lda, ldb, ldc) && bias_ok;
  const int bounded = kgs_gemm_bf16_nt_bounded_ok(A, B, C, M, N, K, lda, ldb, ldc) && bias_ok;
  int v;
  if (variant == 0) v = w4 ? 3 : fast ? 1 : bounded ? 16 : 2;
  else if (variant == 3 || variant == 4) { if (!w4) return KGS_ERR_ALIGN; v = variant; }
  else if (variant == 16) { if (!bounded) return KGS_ERR_ALIGN; v = 16; }
  else if (variant == 1) { if (!fast) return KGS_ERR_ALIGN; v = 1; }
  else if (variant == 2) v = 2;
  else return KGS_ERR_ARG;
  if (variant == 0 && v == 3 && epi == kgs::EPI_NONE) {
    const long tiles = (long)(M / 256) * (N / 256);
    if (tiles <= 64) return kgs_gemm_bf16_nt_w4x_ex(A, B, C, nullptr, M, N, K, lda, ldb, ldc, 128, 1, 128, 0, stream);
    if (tiles <= 128) {
      const bool wide = M < N;
      return kgs_gemm_bf16_nt_w4x_ex(A, B, C, nullptr, M, N, K, lda, ldb, ldc, wide ? 256 : 128, 1, wide ? 128 : 256,
                                     0, stream);
    }
  }
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  hipError_t e;
  switch (epi) {
    case kgs::EPI_NONE: e = kgs::launch<kgs::EPI_NONE>(v, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS: e = kgs::launch<kgs::EPI_BIAS>(v, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS_GELU: e = kgs::launch<kgs::EPI_BIAS_GELU>(v, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS_RELU: e = kgs::launch<kgs::EPI_BIAS_RELU>(v, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS_SILU: e = kgs::launch<kgs::EPI_BIAS_SILU>(v, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    default: return KGS_ERR_ARG;
  }
  return (int)e;
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3fn) GEMM: C = epilogue(alpha * A . B^T), A [M,K] and B [N,K]
// fp8 K-contiguous, C bf16. The same 256x256 pipeline with the scaled
// 16x16x128 f8f6f4 MFMA: the kernel sees each fp8 row as K/2 16-bit words, so
// the LDS-DMA, swizzle and schedule are byte-for-byte those of the bf16 path.
// variant 0 = auto, 1 = aligned (M, N % 256, K % 256), 16 = bounded (any M, N;
// K % 16). Lengths and leading dimensions are in fp8 elements (= bytes).
// ---------------------------------------------------------------------------
namespace kgs {
// gemm_persistent.hip: the four-wave persistent fp8 kernel (gemm_w4f8.h)
template <int EPI>
hipError_t launch_fp8_w4p(const unsigned short* A, const unsigned short* B, unsigned short* C,
                          const unsigned short* bias, int M, int N, int Kw, int ldaw, int ldbw, int ldc, float alpha,
                          const float* alpha_ptr, int cus, int* tq, hipStream_t s);
}  // namespace kgs

namespace {

// v 3: the four-wave persistent kernel (aligned, Kw >= 384 words, more tiles
// than CUs); falls back to the 8-wave aligned kernel without a ticket slot
template <int EPI>
hipError_t launch_fp8(int v, const unsigned short* A, const unsigned short* B, unsigned short* C,
                      const unsigned short* bias, int M, int N, int Kw, int ldaw, int ldbw, int ldc, float alpha,
                      const float* alpha_ptr, hipStream_t s) {
  using namespace kgs;
  const dim3 grid_al((M / g256::BM) * (N / g256::BN));
  if (v == 3) {
    if (int* tq = tile_queue(s))
      return launch_fp8_w4p<EPI>(A, B, C, bias, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, cu_count(), tq, s);
    v = 1;
  }
  if (v == 1) {
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 1024>), grid_al, dim3(512), 0, s, A, B, C, bias, M, N, Kw, ldaw,
                       ldbw, ldc, alpha, alpha_ptr);
  } else {
    const dim3 grid(((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN));
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 512 + 1024>), grid, dim3(512), 0, s, A, B, C, bias, M, N, Kw,
                       ldaw, ldbw, ldc, alpha, alpha_ptr);
  }
  return hipGetLastError();
}

}  // namespace

KGS_EXPORT int kgs_gemm_fp8_nt_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda, int ldb,
                                  int ldc, int bounded) {
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return 0;
  if (K % 16 || lda % 16 || ldb % 16 || ldc % 8) return 0;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return 0;
  if ((long)(lda / 2) * 512 >= kgs::g256::OOB_OFFSET || (long)(ldb / 2) * 512 >= kgs::g256::OOB_OFFSET) return 0;
  if (!bounded && (M % 256 || N % 256 || K % 256)) return 0;
  return 1;
}

// alpha_ptr: optional device float multiplied into alpha in the epilogue (the
// dynamic activation scale written by kgs_quantize_fp8), so no host sync.
KGS_EXPORT int kgs_gemm_fp8_nt_dev(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                                   int lda, int ldb, int ldc, float alpha, const float* alpha_ptr, int epi,
                                   int variant, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (epi != kgs::EPI_NONE && (bias == nullptr || (uintptr_t)bias % 8)) return KGS_ERR_ARG;
  const int fast = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 0);
  const int bounded = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 1);
  // the four-wave persistent kernel: K >= 768 fp8 (384 words), 32-bit offsets
  // over a 256-row panel, more tiles than CUs (round 3, gemm_w4f8.h)
  const int w4p = fast && K >= 768 && (long)(lda / 2) * 512 < (1L << 31) && (long)(ldb / 2) * 512 < (1L << 31);
  int v;
  if (variant == 0) v = w4p && (M / 256) * (N / 256) > kgs::cu_count() ? 3 : fast ? 1 : 16;
  else if (variant == 1 || variant == 16) v = variant;
  else if (variant == 3) { if (!w4p) return KGS_ERR_ALIGN; v = 3; }
  else return KGS_ERR_ARG;
  if (!(v == 16 ? bounded : fast)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  const int Kw = K / 2, ldaw = lda / 2, ldbw = ldb / 2;  // fp8 rows as 16-bit words
  hipError_t e;
  switch (epi) {
    case kgs::EPI_NONE:
      e = launch_fp8<kgs::EPI_NONE>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, stream);
      break;
    case kgs::EPI_BIAS:
      e = launch_fp8<kgs::EPI_BIAS>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, stream);
      break;
    case kgs::EPI_BIAS_GELU:
      e = launch_fp8<kgs::EPI_BIAS_GELU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, stream);
      break;
    case kgs::EPI_BIAS_RELU:
      e = launch_fp8<kgs::EPI_BIAS_RELU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, stream);
      break;
    case kgs::EPI_BIAS_SILU:
      e = launch_fp8<kgs::EPI_BIAS_SILU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, alpha_ptr, stream);
      break;
    default: return KGS_ERR_ARG;
  }
  return (int)e;
}

// Per-row activation scales (W8A8 with per-token dynamic activation scales):
// C = epilogue(alpha * row_scale[m] * A . B^T). EPI_NONE / EPI_BIAS only.
KGS_EXPORT int kgs_gemm_fp8_nt_rows(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                                    int lda, int ldb, int ldc, float alpha, const float* row_scale, int epi,
                                    int variant, hipStream_t stream) {
  using namespace kgs;
  if (M <= 0 || N <= 0 || K <= 0) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (row_scale == nullptr || (uintptr_t)row_scale % 4) return KGS_ERR_ARG;
  if (epi != EPI_NONE && epi != EPI_BIAS) return KGS_ERR_ARG;
  if (epi != EPI_NONE && (bias == nullptr || (uintptr_t)bias % 8)) return KGS_ERR_ARG;
  const int fast = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 0);
  const int bounded = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 1);
  int v;
  if (variant == 0) v = fast ? 1 : 16;
  else if (variant == 1 || variant == 16) v = variant;
  else return KGS_ERR_ARG;
  if (!(v == 16 ? bounded : fast)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  const int Kw = K / 2, ldaw = lda / 2, ldbw = ldb / 2;
  constexpr int RS = 524288 + 1024 + 7;
  if (v == 1) {
    const dim3 grid((M / g256::BM) * (N / g256::BN));
    if (epi == EPI_NONE)
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, RS>), grid, dim3(512), 0, stream, a, b, c, bb, M, N, Kw, ldaw,
                         ldbw, ldc, alpha, row_scale);
    else
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI_BIAS, RS>), grid, dim3(512), 0, stream, a, b, c, bb, M, N, Kw, ldaw,
                         ldbw, ldc, alpha, row_scale);
  } else {
    const dim3 grid(((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN));
    if (epi == EPI_NONE)
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, RS + 512>), grid, dim3(512), 0, stream, a, b, c, bb, M, N, Kw,
                         ldaw, ldbw, ldc, alpha, row_scale);
    else
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI_BIAS, RS + 512>), grid, dim3(512), 0, stream, a, b, c, bb, M, N, Kw,
                         ldaw, ldbw, ldc, alpha, row_scale);
  }
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_gemm_fp8_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                               int ldb, int ldc, float alpha, int epi, int variant, hipStream_t stream) {
  return kgs_gemm_fp8_nt_dev(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, nullptr, epi, variant, stream);
}

// ---------------------------------------------------------------------------
// General layouts: C[M,N] = epilogue(op(A) . op(B)) with
//   ta = 0: A stored [M][K] (K contiguous)     ta = 1: A stored [K][M]
//   tb = 0: B stored [N][K] (the NT layout)    tb = 1: B stored [K][N]
// The transposed operands go through the same pipeline: their half-tiles are
// staged as [64 k][128 cols] and read with ds_read_b64_tr_b16, so no
// materialised transpose is needed (Linear backward: dX = dY.W is tb=1,
// dW = dY^T.X is ta=1, tb=1). Aligned shapes only (M, N % 256, K % 128).
// ---------------------------------------------------------------------------
namespace {

template <int EPI, int T>
hipError_t launch_t(const unsigned short* A, const unsigned short* B, unsigned short* C, const unsigned short* bias,
                    int M, int N, int K, int lda, int ldb, int ldc, hipStream_t s) {
  using namespace kgs;
  const dim3 grid((M / g256::BM) * (N / g256::BN));
  hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + T>), grid, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                     1.0f, nullptr);
  return hipGetLastError();
}

template <int EPI>
hipError_t launch_layout(int ta, int tb, const unsigned short* A, const unsigned short* B, unsigned short* C,
                         const unsigned short* bias, int M, int N, int K, int lda, int ldb, int ldc, hipStream_t s) {
  if constexpr (EPI == kgs::EPI_NONE) {
    if (ta == 2) return launch_t<EPI, 2048 + 8192>(A, B, C, bias, M, N, K, lda, ldb, ldc, s);   // probe
    if (ta == 3) return launch_t<EPI, 2048 + 16384>(A, B, C, bias, M, N, K, lda, ldb, ldc, s);  // probe
  }
  if (ta && tb) return launch_t<EPI, 2048 + 4096>(A, B, C, bias, M, N, K, lda, ldb, ldc, s);
  if (ta) return launch_t<EPI, 2048>(A, B, C, bias, M, N, K, lda, ldb, ldc, s);
  return launch_t<EPI, 4096>(A, B, C, bias, M, N, K, lda, ldb, ldc, s);
}

}  // namespace

// ---------------------------------------------------------------------------
// split-K for short-M GEMMs (decode batches of 128-256 rows): the 256x256
// pipeline over nslice K-slices (gemm_nt_256 S bit 20) writes fp32 partial
// tiles, splitk_reduce sums them into bf16 C. With N / 256 tiles alone such a
// GEMM fills a fraction of the 256 CUs (the Llama-3-8B down projection has 16
// tiles); the slices fill the rest.
// ---------------------------------------------------------------------------
namespace kgs {
// NSL > 0: slice count at compile time -- a thread issues all its partial loads
// before the first add instead of waiting out one cache latency per slice.
template <int NSL>
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ P, unsigned short* __restrict__ C,
                                                     int M, int N, int ldc, int nslice) {
  const long e = ((long)blockIdx.x * 256 + threadIdx.x) * 8;  // 8 consecutive columns of one row
  const long MN = (long)M * N;
  if (e >= MN) return;
  const int row = (int)(e / N), col = (int)(e - (long)row * N);
  f32x4 a, b;
  if constexpr (NSL > 0) {
    f32x4 pa[NSL], pb[NSL];
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      pa[s] = *(const f32x4*)(P + s * MN + e);
      pb[s] = *(const f32x4*)(P + s * MN + e + 4);
    }
    a = pa[0];
    b = pb[0];
#pragma unroll
    for (int s = 1; s < NSL; ++s) {
      a += pa[s];
      b += pb[s];
    }
  } else {
    a = *(const f32x4*)(P + e);
    b = *(const f32x4*)(P + e + 4);
    for (int s = 1; s < nslice; ++s) {
      a += *(const f32x4*)(P + s * MN + e);
      b += *(const f32x4*)(P + s * MN + e + 4);
    }
  }
  uint4 o;
  o.x = pack_bf16x2(a[0], a[1]);
  o.y = pack_bf16x2(a[2], a[3]);
  o.z = pack_bf16x2(b[0], b[1]);
  o.w = pack_bf16x2(b[2], b[3]);
  *(uint4*)(C + (long)row * ldc + col) = o;
}

// SwiGLU consumer of a split-K gate|up GEMM (round 3): P holds nslice fp32
// partials [M][2I] of a fused gate|up product (gate columns [0, I), up [I, 2I));
// out[m][j] = silu(g) * u with g, u the slice sums rounded to bf16 first -- the
// roundings of gemm_nt + silu_mul. One thread: 8 consecutive outputs.
template <int NSL>
__global__ __launch_bounds__(256) void splitk_reduce_swiglu(const float* __restrict__ P,
                                                            unsigned short* __restrict__ out, int M, int I, int ldo,
                                                            int nslice) {
  const long e = ((long)blockIdx.x * 256 + threadIdx.x) * 8;  // index into [M][I]
  const long MI = (long)M * I, MN = 2 * MI;
  if (e >= MI) return;
  const int row = (int)(e / I), col = (int)(e - (long)row * I);
  const float* pg = P + (long)row * 2 * I + col;
  const float* pu = pg + I;
  f32x4 g0, g1, u0, u1;
  if constexpr (NSL > 0) {
    f32x4 a[NSL][4];
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      a[s][0] = *(const f32x4*)(pg + s * MN);
      a[s][1] = *(const f32x4*)(pg + s * MN + 4);
      a[s][2] = *(const f32x4*)(pu + s * MN);
      a[s][3] = *(const f32x4*)(pu + s * MN + 4);
    }
    g0 = a[0][0], g1 = a[0][1], u0 = a[0][2], u1 = a[0][3];
#pragma unroll
    for (int s = 1; s < NSL; ++s) {
      g0 += a[s][0];
      g1 += a[s][1];
      u0 += a[s][2];
      u1 += a[s][3];
    }
  } else {
    g0 = *(const f32x4*)pg, g1 = *(const f32x4*)(pg + 4), u0 = *(const f32x4*)pu, u1 = *(const f32x4*)(pu + 4);
    for (int s = 1; s < nslice; ++s) {
      g0 += *(const f32x4*)(pg + s * MN);
      g1 += *(const f32x4*)(pg + s * MN + 4);
      u0 += *(const f32x4*)(pu + s * MN);
      u1 += *(const f32x4*)(pu + s * MN + 4);
    }
  }
  float r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float g = bf2f(f2bf(k < 4 ? g0[k] : g1[k - 4]));
    const float u = bf2f(f2bf(k < 4 ? u0[k] : u1[k - 4]));
    r[k] = g / (1.0f + __expf(-g)) * u;
  }
  uint4 o;
  o.x = pack_bf16x2(r[0], r[1]);
  o.y = pack_bf16x2(r[2], r[3]);
  o.z = pack_bf16x2(r[4], r[5]);
  o.w = pack_bf16x2(r[6], r[7]);
  *(uint4*)(out + (long)row * ldo + col) = o;
}

inline void launch_splitk_reduce(const float* P, unsigned short* C, int M, int N, int ldc, int nslice,
                                 hipStream_t s) {
  const dim3 g((unsigned)(((long)M * N / 8 + 255) / 256)), b(256);
  switch (nslice) {
    case 2: hipLaunchKernelGGL(splitk_reduce<2>, g, b, 0, s, P, C, M, N, ldc, nslice); break;
    case 4: hipLaunchKernelGGL(splitk_reduce<4>, g, b, 0, s, P, C, M, N, ldc, nslice); break;
    case 8: hipLaunchKernelGGL(splitk_reduce<8>, g, b, 0, s, P, C, M, N, ldc, nslice); break;
    default: hipLaunchKernelGGL(splitk_reduce<0>, g, b, 0, s, P, C, M, N, ldc, nslice); break;
  }
}
}  // namespace kgs

// Four-wave kernel for short-M (decode-batch) GEMMs: tile width bn (256 or 128),
// tile height bm (256 or 128: 65-128-row batches waste no MFMAs on padding rows),
// any M (rows past M read as zeros, stores predicated), and nslice K-slices
// (nslice > 1: fp32 partial tiles into ws, then splitk_reduce; with C == nullptr
// the reduce is left to a fused consumer such as kgs_splitk_add_rmsnorm_bf16 or
// kgs_rope_cache_bf16, which read ws directly). Requirements:
// N % bn == 0, (K / nslice) % 128 == 0, lda/ldb/ldc % 8, 16-B aligned pointers.
namespace {
template <int BN, int TM, int X>
void launch_w4x_x(dim3 grid, hipStream_t s, const unsigned short* a, const unsigned short* b, unsigned short* out,
                  int M, int N, int ks, int lda, int ldb, int ld, int mode) {
  using namespace kgs;
  using Kn = w4::Knobs<w4::tile_m<TM>(), BN>;
#define KGS_W4X(MD)                                                                                               \
  hipLaunchKernelGGL((w4::gemm_nt_w4<EPI_NONE, BN, TM | MD, Kn::B1, Kn::R, Kn::P, Kn::ORD, X>), grid, dim3(256), 0, s, \
                     a, b, out, nullptr, M, N, ks, lda, ldb, ld)
  switch (mode) {
    case 0: KGS_W4X(0); break;
    case 1: KGS_W4X(1); break;
    case 2: KGS_W4X(2); break;
    default: KGS_W4X(3); break;
  }
#undef KGS_W4X
}

// LDS stages of the w4x entries: flags bits 4-5 = stages - 2 (gemm_w4.h
// stages<MODE>), only where NS stages fit in 160 KiB
constexpr bool stages_fit(int bm, int bn, int ns) { return ns * (bm + bn) * 128 <= 160 * 1024; }

// flags bit 0 (packed): B stored tile-panel major ([N / bn][K / 64][bn][64],
// gemm_w4.h PACKB); bits 4-5: extra LDS stages
template <int BN, int TM>
int launch_w4x(dim3 grid, hipStream_t s, const unsigned short* a, const unsigned short* b, unsigned short* out,
               int M, int N, int ks, int lda, int ldb, int ld, int mode, int flags) {
  constexpr int BM = kgs::w4::tile_m<TM>();
  const bool packed = flags & 1;
  if (flags & 2) {  // weights (B) non-temporal: two LDS stages only
    if (flags & 0x30) return KGS_ERR_ARG;
    if (packed) launch_w4x_x<BN, TM, 1000005200>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
    else launch_w4x_x<BN, TM, 5200>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
    return 0;
  }
  switch (flags & 0x30) {
    case 0x00:
      if (packed) launch_w4x_x<BN, TM, 1000000000>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
      else launch_w4x_x<BN, TM, 0>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
      return 0;
    case 0x10:
      if constexpr (stages_fit(BM, BN, 3)) {
        if (packed) launch_w4x_x<BN, TM | 0x10, 1000000000>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
        else launch_w4x_x<BN, TM | 0x10, 0>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
        return 0;
      }
      break;
    case 0x20:
      if constexpr (stages_fit(BM, BN, 4)) {
        if (packed) launch_w4x_x<BN, TM | 0x20, 1000000000>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
        else launch_w4x_x<BN, TM | 0x20, 0>(grid, s, a, b, out, M, N, ks, lda, ldb, ld, mode);
        return 0;
      }
      break;
  }
  return KGS_ERR_ARG;
}

template <int BN, int TM, int X>
void launch_w4sw_x(dim3 grid, hipStream_t s, const unsigned short* a, const unsigned short* b, unsigned short* c,
                   int M, int N, int K, int lda, int ldb, int ldc, bool aligned_m) {
  using namespace kgs;
  constexpr int BM = w4::tile_m<TM>();
  using Kn = w4::Knobs<BM, BN>;
  if (aligned_m)
    hipLaunchKernelGGL((w4::gemm_nt_w4<EPI_NONE, BN, TM, Kn::B1, Kn::R, Kn::P, Kn::ORD, X>), grid, dim3(256), 0, s, a,
                       b, c, nullptr, M, N, K, lda, ldb, ldc);
  else
    hipLaunchKernelGGL((w4::gemm_nt_w4<EPI_NONE, BN, TM | 1, Kn::B1, Kn::R, Kn::P, Kn::ORD, X>), grid, dim3(256), 0, s,
                       a, b, c, nullptr, M, N, K, lda, ldb, ldc);
}

template <int BN, int TM>
int launch_w4sw(dim3 grid, hipStream_t s, const unsigned short* a, const unsigned short* b, unsigned short* c, int M,
                int N, int K, int lda, int ldb, int ldc, bool aligned_m, int flags) {
  constexpr int BM = kgs::w4::tile_m<TM>();
  const bool packed = flags & 1;
  if (flags & 2) {  // weights (B) non-temporal: two LDS stages only
    if (flags & 0x30) return KGS_ERR_ARG;
    if (packed) launch_w4sw_x<BN, TM, 1001005200>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
    else launch_w4sw_x<BN, TM, 1005200>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
    return 0;
  }
  switch (flags & 0x30) {
    case 0x00:
      if (packed) launch_w4sw_x<BN, TM, 1001000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
      else launch_w4sw_x<BN, TM, 1000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
      return 0;
    case 0x10:
      if constexpr (stages_fit(BM, BN, 3)) {
        if (packed) launch_w4sw_x<BN, TM | 0x10, 1001000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
        else launch_w4sw_x<BN, TM | 0x10, 1000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
        return 0;
      }
      break;
    case 0x20:
      if constexpr (stages_fit(BM, BN, 4)) {
        if (packed) launch_w4sw_x<BN, TM | 0x20, 1001000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
        else launch_w4sw_x<BN, TM | 0x20, 1000000>(grid, s, a, b, c, M, N, K, lda, ldb, ldc, aligned_m);
        return 0;
      }
      break;
  }
  return KGS_ERR_ARG;
}
}  // namespace

KGS_EXPORT int kgs_gemm_bf16_nt_w4x_ex(const void* A, const void* B, void* C, float* ws, int M, int N, int K,
                                       int lda, int ldb, int ldc, int bn, int nslice, int bm, int flags,
                                       hipStream_t stream);

KGS_EXPORT int kgs_gemm_bf16_nt_w4x(const void* A, const void* B, void* C, float* ws, int M, int N, int K, int lda,
                                    int ldb, int ldc, int bn, int nslice, int bm, hipStream_t stream) {
  return kgs_gemm_bf16_nt_w4x_ex(A, B, C, ws, M, N, K, lda, ldb, ldc, bn, nslice, bm, 0, stream);
}

// flags bit 0: B is the tile-panel-major copy of a [N, K] weight
// ([N / bn][K / 64][bn][64], kgs.ops.gemm.pack_w4x_weight) and ldb must be K;
// bit 1: B's loads non-temporal (two stages only); bits 4-5: LDS stages - 2
// (0..2, where they fit in 160 KiB)
KGS_EXPORT int kgs_gemm_bf16_nt_w4x_ex(const void* A, const void* B, void* C, float* ws, int M, int N, int K,
                                       int lda, int ldb, int ldc, int bn, int nslice, int bm, int flags,
                                       hipStream_t stream) {
  using namespace kgs;
  if (flags & ~0x33 || (flags & 0x30) == 0x30) return KGS_ERR_ARG;
  if ((flags & 1) && ldb != K) return KGS_ERR_SHAPE;
  if (M <= 0 || N <= 0 || K <= 0 || nslice <= 0 || K % nslice) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if ((bn != 128 && bn != 256) || (bm != 128 && bm != 256)) return KGS_ERR_ARG;
  const int ks = K / nslice;
  if (N % bn || ks % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  if ((long)lda * 512 >= (1L << 31) || (long)ldb * 512 >= (1L << 31)) return KGS_ERR_SHAPE;
  if (nslice > 1 && (ws == nullptr || (uintptr_t)ws % 16)) return KGS_ERR_ARG;
  if (nslice == 1 && C == nullptr) return KGS_ERR_ARG;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  const int ntm = (M + bm - 1) / bm;
  const dim3 grid(ntm * (N / bn) * nslice);
  unsigned short* out = nslice > 1 ? (unsigned short*)ws : c;
  const int ld = nslice > 1 ? N : ldc;
  const int mode = (M % bm == 0 ? 0 : 1) | (nslice > 1 ? 2 : 0);
  int rc;
  if (bm == 256) {
    if (bn == 256) rc = launch_w4x<256, 0>(grid, stream, a, b, out, M, N, ks, lda, ldb, ld, mode, flags);
    else rc = launch_w4x<128, 0>(grid, stream, a, b, out, M, N, ks, lda, ldb, ld, mode, flags);
  } else {
    if (bn == 256) rc = launch_w4x<256, 8>(grid, stream, a, b, out, M, N, ks, lda, ldb, ld, mode, flags);
    else rc = launch_w4x<128, 8>(grid, stream, a, b, out, M, N, ks, lda, ldb, ld, mode, flags);
  }
  if (rc) return rc;
  if (nslice > 1 && c != nullptr) launch_splitk_reduce(ws, c, M, N, ldc, nslice, stream);
  return (int)hipGetLastError();
}

// SwiGLU decode GEMM on the four-wave kernel: B is a fused gate|up weight
// [N = 2I, K] (gate rows first); C[M, I] = silu(A . gate^T) * (A . up^T) with
// both products rounded to bf16 first (the roundings of gemm + silu_mul). Any
// M; tiles bm x bn (256 / 128 each); N % bn == 0, K % 128 == 0, lda/ldb/ldc % 8,
// 16-B aligned pointers.
KGS_EXPORT int kgs_gemm_bf16_nt_w4x_swiglu_ex(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                                              int ldb, int ldc, int bn, int bm, int flags, hipStream_t stream);

KGS_EXPORT int kgs_gemm_bf16_nt_w4x_swiglu(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                                           int ldb, int ldc, int bn, int bm, hipStream_t stream) {
  return kgs_gemm_bf16_nt_w4x_swiglu_ex(A, B, C, M, N, K, lda, ldb, ldc, bn, bm, 0, stream);
}

// flags bit 0: B is the SwiGLU-packed copy of the fused gate|up weight
// (kgs.ops.gemm.pack_w4x_weight(..., swiglu=True)), ldb must be K; bits 4-5:
// LDS stages - 2 (as kgs_gemm_bf16_nt_w4x_ex)
KGS_EXPORT int kgs_gemm_bf16_nt_w4x_swiglu_ex(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                                              int ldb, int ldc, int bn, int bm, int flags, hipStream_t stream) {
  using namespace kgs;
  if (flags & ~0x33 || (flags & 0x30) == 0x30) return KGS_ERR_ARG;
  if ((flags & 1) && ldb != K) return KGS_ERR_SHAPE;
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N / 2) return KGS_ERR_SHAPE;
  if ((bn != 128 && bn != 256) || (bm != 128 && bm != 256)) return KGS_ERR_ARG;
  if (N % bn || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  if ((long)lda * 512 >= (1L << 31) || (long)ldb * 512 >= (1L << 31)) return KGS_ERR_SHAPE;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  const dim3 grid(((M + bm - 1) / bm) * (N / bn));
  const bool aligned_m = M % bm == 0;
  // prompt-pass shapes (256 x 256 tiles, aligned M, more tiles than CUs): the
  // persistent kernel with the same K-step (bitwise the one-shot result)
  if (bm == 256 && bn == 256 && aligned_m && flags == 0 && K >= 384 && (long)(M / 256) * (N / 256) > cu_count()) {
    if (int* tq = tile_queue(stream)) {
      const hipError_t e = launch_w4p_swiglu(a, b, c, M, N, K, lda, ldb, ldc, cu_count(), tq, stream);
      return e == hipSuccess ? 0 : (int)e;
    }
  }
  int rc;
  if (bm == 256) {
    if (bn == 256) rc = launch_w4sw<256, 0>(grid, stream, a, b, c, M, N, K, lda, ldb, ldc, aligned_m, flags);
    else rc = launch_w4sw<128, 0>(grid, stream, a, b, c, M, N, K, lda, ldb, ldc, aligned_m, flags);
  } else {
    if (bn == 256) rc = launch_w4sw<256, 8>(grid, stream, a, b, c, M, N, K, lda, ldb, ldc, aligned_m, flags);
    else rc = launch_w4sw<128, 8>(grid, stream, a, b, c, M, N, K, lda, ldb, ldc, aligned_m, flags);
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

// C[M, N] (bf16) = A[M, K] . B[N, K]^T over nslice K-slices; ws holds nslice *
// M * N floats. K / nslice must be a multiple of 128 (aligned M % 256 == 0,
// N % 256 == 0) or of 8 (any M, N % 8 == 0: the bounded pipeline).
KGS_EXPORT int kgs_gemm_bf16_nt_splitk(const void* A, const void* B, void* C, float* ws, int M, int N, int K, int lda,
                                       int ldb, int ldc, int nslice, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || nslice <= 0 || K % nslice) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N || N % 8 || ldc % 8) return KGS_ERR_SHAPE;
  if (ws == nullptr) return KGS_ERR_ARG;
  const int ks = K / nslice;
  if ((uintptr_t)ws % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  const bool fast = kgs_gemm_bf16_nt_fast_ok(A, B, C, M, N, ks, lda, ldb, ldc) && ks % 128 == 0;
  const bool bounded = kgs_gemm_bf16_nt_bounded_ok(A, B, C, M, N, ks, lda, ldb, ldc);
  if (!fast && !bounded) return KGS_ERR_ALIGN;
  using namespace kgs;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  const int ntm = (M + g256::BM - 1) / g256::BM, ntn = (N + g256::BN - 1) / g256::BN;
  const dim3 grid(ntm * ntn * nslice);
  if (fast)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 7 + 1048576>), grid, dim3(512), 0, stream, a, b,
                       (unsigned short*)ws, nullptr, M, N, ks, lda, ldb, N, 1.0f, nullptr);
  else
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 7 + 512 + 1048576>), grid, dim3(512), 0, stream, a, b,
                       (unsigned short*)ws, nullptr, M, N, ks, lda, ldb, N, 1.0f, nullptr);
  launch_splitk_reduce(ws, (unsigned short*)C, M, N, ldc, nslice, stream);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_gemm_bf16_layout_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda,
                                       int ldb, int ldc, int ta, int tb) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (M % 256 || N % 256 || K % 128) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8) return 0;
  if (lda < (ta ? M : K) || ldb < (tb ? N : K) || ldc < N) return 0;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return 0;
  // per-tile 32-bit lane offsets: 256 rows (NT) or 64 k-rows (transposed) times ld
  if ((long)lda * 256 >= (1L << 31) || (long)ldb * 256 >= (1L << 31)) return 0;
  return 1;
}

KGS_EXPORT int kgs_gemm_bf16(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                             int ldb, int ldc, int ta, int tb, int epi, hipStream_t stream) {
  if (!ta && !tb) return kgs_gemm_bf16_nt(A, B, C, bias, M, N, K, lda, ldb, ldc, epi, 0, stream);
  if (epi != kgs::EPI_NONE && (bias == nullptr || (uintptr_t)bias % 8)) return KGS_ERR_ARG;
  if (!kgs_gemm_bf16_layout_ok(A, B, C, M, N, K, lda, ldb, ldc, ta, tb)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  hipError_t e;
  switch (epi) {
    case kgs::EPI_NONE: e = launch_layout<kgs::EPI_NONE>(ta, tb, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS: e = launch_layout<kgs::EPI_BIAS>(ta, tb, a, b, c, bb, M, N, K, lda, ldb, ldc, stream); break;
    case kgs::EPI_BIAS_GELU:
      e = launch_layout<kgs::EPI_BIAS_GELU>(ta, tb, a, b, c, bb, M, N, K, lda, ldb, ldc, stream);
      break;
    case kgs::EPI_BIAS_RELU:
      e = launch_layout<kgs::EPI_BIAS_RELU>(ta, tb, a, b, c, bb, M, N, K, lda, ldb, ldc, stream);
      break;
    case kgs::EPI_BIAS_SILU:
      e = launch_layout<kgs::EPI_BIAS_SILU>(ta, tb, a, b, c, bb, M, N, K, lda, ldb, ldc, stream);
      break;
    default: return KGS_ERR_ARG;
  }
  return (int)e;
}

// out[M][I] = silu(sum_s P[s][:, :I]) * sum_s P[s][:, I:] (bf16-rounded sums): the
// consumer of kgs_gemm_bf16_nt_w4x(C = nullptr, ...) on a fused gate|up weight.
KGS_EXPORT int kgs_splitk_reduce_swiglu_bf16(const float* P, void* out, int nslice, int M, int I, int ldo,
                                            hipStream_t s) {
  using namespace kgs;
  if (nslice <= 0 || M <= 0 || I <= 0 || I % 8 || ldo < I || ldo % 8) return KGS_ERR_SHAPE;
  if ((uintptr_t)P % 16 || (uintptr_t)out % 16) return KGS_ERR_ALIGN;
  const dim3 g((unsigned)(((long)M * I / 8 + 255) / 256)), b(256);
  auto o = (unsigned short*)out;
  switch (nslice) {
    case 2: hipLaunchKernelGGL(splitk_reduce_swiglu<2>, g, b, 0, s, P, o, M, I, ldo, nslice); break;
    case 4: hipLaunchKernelGGL(splitk_reduce_swiglu<4>, g, b, 0, s, P, o, M, I, ldo, nslice); break;
    default: hipLaunchKernelGGL(splitk_reduce_swiglu<0>, g, b, 0, s, P, o, M, I, ldo, nslice); break;
  }
  return (int)hipGetLastError();
}
