// Measured alternatives of the four-wave GEMM (native/kernels/gemm_w4.h): the
// K-step schedule knobs B1 / R / P / ORD / X of gemm_nt_w4. Built into the
// opt-in libkgs_experiments.so; names and ids in kgs/ops/experiments.py (W4H),
// numbers in profiles/gemm_tuning.md ("Four-wave kernel").
#include "gemm_w4.h"
#include "gemm_w4f8.h"
#include "gemm_w4p.h"
#include "tile_queue.h"
#include "tile_queue_zero.h"

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// variant = table id below; template <B1, R, P, ORD, X>, X = 10000 W + 100 AUX + GROUP_M
// (W = DMA window in MFMAs, AUX = DMA cache bits, 0 = default). Aligned shapes
// only: M, N % 256, K % 128, lda/ldb/ldc % 8, 16-B aligned operands.
KGS_EXPORT int kgs_exp_gemm_w4h(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                                int variant, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  if ((long)lda * 256 * 2 >= (1L << 31) || (long)ldb * 256 * 2 >= (1L << 31)) return KGS_ERR_SHAPE;
  const dim3 grid((M / 256) * (N / 256));
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
#define KGS_W4H(ID, B1, R, P, ORD, X)                                                                         \
  case ID:                                                                                                    \
    hipLaunchKernelGGL((kgs::w4::gemm_nt_w4<kgs::EPI_NONE, 256, 0, B1, R, P, ORD, X>), grid, dim3(256), 0, s, a, b, c, \
                       nullptr, M, N, K, lda, ldb, ldc);                                                      \
    break;
  // ids: kgs/ops/experiments.py W4H (name = w4h_ORD_B1_R_P_X)
  // ids 101..: the persistent kernel (gemm_w4p.h) with knob bag X (tile map,
  // DMA order; see gemm_w4.h tile_of / dma_any); K >= 384, one workgroup per CU
  if (variant > 100) {
    if (K < 384) return KGS_ERR_SHAPE;
    const int ntiles = (M / 256) * (N / 256);
    const dim3 pg(ntiles < cu_count() ? ntiles : cu_count());
    int* tq = kgs::tile_queue(s);
    if (!tq) return KGS_ERR_ARG;
#define KGS_W4P(ID, X, DYN)                                                                                    \
  case ID:                                                                                                          \
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, X, DYN>), pg, dim3(256), 0, s, a, b, c, nullptr, M, N, K, \
                       lda, ldb, ldc, tq);                                                                              \
    break;
    // ids: kgs/ops/experiments.py W4P
    switch (variant) {
      KGS_W4P(101, 0, true)
      KGS_W4P(102, 140000000, true)
      KGS_W4P(103, 8, true)
      KGS_W4P(104, 10000000, true)
      KGS_W4P(105, 140000008, true)
      KGS_W4P(106, 40000000, true)
      KGS_W4P(107, 100000000, true)
      KGS_W4P(108, 200000000, true)
      KGS_W4P(109, 140000002, true)
      // C stored non-temporally: default / mirror G8 maps
      case 131:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, true>), pg, dim3(256), 0, s, a, b, c, nullptr, M,
                           N, K, lda, ldb, ldc, tq);
        break;
      case 132:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000008, 1, true>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 133:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 8, 1, true>), pg, dim3(256), 0, s, a, b, c, nullptr, M,
                           N, K, lda, ldb, ldc, tq);
        break;
      case 134:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000000, 1, true>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      // round 4: LDS layout 1 (linear rows, conflict-free placement; gemm_w4p.h Lay<1>)
      case 135:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 1>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 136:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000008, 1, false, false, 1>), pg, dim3(256), 0, s,
                           a, b, c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 137:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 8, 1, false, false, 1>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 138:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000000, 1, false, false, 1>), pg, dim3(256), 0, s,
                           a, b, c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      // round 4: MFMA order inside a k-sub (gemm_w4p.h ord_of): i-major / n-major, default and mirror G8 maps
      case 139:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 10>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 140:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 30>), pg, dim3(256), 0, s, a, b, c,
                           nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 141:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000008, 1, false, false, 10>), pg, dim3(256), 0, s,
                           a, b, c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 142:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 140000008, 1, false, false, 30>), pg, dim3(256), 0, s,
                           a, b, c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      // round 5: C store measurement builds (gemm_w4p.h (L / 100) % 10): no store / drain after the stores
      case 143:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 100>), pg, dim3(256), 0, s, a, b,
                           c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 144:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 200>), pg, dim3(256), 0, s, a, b,
                           c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      case 145:
        hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 300>), pg, dim3(256), 0, s, a, b,
                           c, nullptr, M, N, K, lda, ldb, ldc, tq);
        break;
      // round 6: deferred C stores (gemm_w4p.h DD, SPS): SPS units per lane stored at the end of each of the
      // next tile's first DD K-steps; ids and names in kgs/ops/experiments.py (w4pq_*)
#define KGS_W4PQ(ID, X, NT, DD, SPS)                                                                          \
  case ID:                                                                                                    \
    if (K / 64 < ((DD + 2) & ~1) + 2) return KGS_ERR_SHAPE;                                                   \
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, X, 1, NT, false, 0, DD, SPS>), pg, dim3(256), 0, s, a, \
                       b, c, nullptr, M, N, K, lda, ldb, ldc, tq);                                             \
    break;
      KGS_W4PQ(146, 0, true, 8, 2)
      KGS_W4PQ(147, 0, true, 4, 4)
      KGS_W4PQ(148, 0, true, 8, 1)
      KGS_W4PQ(149, 0, true, 10, 2)
      KGS_W4PQ(150, 0, true, 16, 1)
      KGS_W4PQ(151, 0, false, 8, 2)
      KGS_W4PQ(152, 140000008, false, 8, 2)
      KGS_W4PQ(153, 0, true, 12, 1)
      KGS_W4PQ(154, 140000008, true, 8, 2)
      KGS_W4PQ(155, 8, true, 8, 2)
      // fewer storing K-steps, more stores each (4 x 4 led the first sweep)
      KGS_W4PQ(156, 0, true, 1, 16)
      KGS_W4PQ(157, 0, true, 2, 8)
      KGS_W4PQ(158, 0, true, 3, 6)
      KGS_W4PQ(159, 0, true, 2, 10)
      KGS_W4PQ(160, 0, true, 4, 5)
      KGS_W4PQ(161, 140000008, false, 4, 4)
      KGS_W4PQ(162, 140000008, true, 4, 4)
      KGS_W4PQ(163, 0, false, 4, 4)
      KGS_W4PQ(164, 8, false, 4, 4)
      KGS_W4PQ(165, 140000008, false, 2, 8)
      KGS_W4PQ(166, 0, false, 2, 8)
#undef KGS_W4PQ
      // round 6: one barrier per K-step (gemm_w4p.h (L / 1000) % 10 == 1), DMA window W = (L / 10^4) % 100
#define KGS_W4PB(ID, X, NT, L, DD, SPS)                                                                       \
  case ID:                                                                                                    \
    if (K / 64 < ((DD + 2) & ~1) + 2) return KGS_ERR_SHAPE;                                                   \
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, X, 1, NT, false, L, DD, SPS>), pg, dim3(256), 0, s, a, \
                       b, c, nullptr, M, N, K, lda, ldb, ldc, tq);                                             \
    break;
      KGS_W4PB(167, 0, true, 1000, 0, 2)
      KGS_W4PB(168, 0, true, 481000, 0, 2)
      KGS_W4PB(169, 0, true, 321000, 0, 2)
      KGS_W4PB(170, 0, true, 1000, 4, 4)
      KGS_W4PB(171, 140000008, false, 1000, 0, 2)
      KGS_W4PB(172, 8, false, 1000, 0, 2)
      KGS_W4PB(173, 0, false, 1000, 0, 2)
      KGS_W4PB(174, 0, true, 641000, 0, 2)
      // round 6: K-step schedule (gemm_w4p.h (L / 10^7) % 10: barrier 1 after MFMA B1, R MFMAs after
      // barrier 2) on the production 3-8-tiles-per-CU route (nt C, deferred 4 x 4) and on the tall G8 map
      KGS_W4PB(175, 0, true, 10000000, 4, 4)
      KGS_W4PB(176, 0, true, 20000000, 4, 4)
      KGS_W4PB(177, 0, true, 30000000, 4, 4)
      KGS_W4PB(178, 0, true, 40000000, 4, 4)
      KGS_W4PB(179, 140000008, false, 20000000, 0, 2)
      KGS_W4PB(180, 140000008, false, 30000000, 0, 2)
      KGS_W4PB(181, 0, true, 50000000, 4, 4)
      KGS_W4PB(182, 0, true, 60000000, 4, 4)
      KGS_W4PB(183, 0, true, 70000000, 4, 4)
      KGS_W4PB(184, 140000008, false, 50000000, 0, 2)
#undef KGS_W4PB
      // the static walk (v, v + G, ...: no ticket atomics), default / mirror / G8 / mirror G8
      KGS_W4P(121, 0, false)
      KGS_W4P(122, 140000000, false)
      KGS_W4P(123, 8, false)
      KGS_W4P(124, 140000008, false)
      default: return KGS_ERR_ARG;
    }
#undef KGS_W4P
    return (int)hipGetLastError();
  }
  switch (variant) {
    KGS_W4H(1, 24, 20, 1, 1, 0)
    KGS_W4H(2, 24, 20, 1, 1, 160000)
    KGS_W4H(3, 24, 20, 1, 1, 320000)
    KGS_W4H(4, 24, 20, 1, 1, 480000)
    KGS_W4H(5, 20, 20, 1, 1, 160000)
    KGS_W4H(6, 20, 24, 1, 1, 320000)
    KGS_W4H(7, 24, 20, 1, 1, 2)
    KGS_W4H(8, 24, 20, 1, 1, 8)
    KGS_W4H(9, 24, 20, 1, 1, 16)
    KGS_W4H(10, 24, 20, 1, 1, 32)
    KGS_W4H(11, 24, 20, 1, 1, 10000000)
    KGS_W4H(12, 24, 20, 1, 1, 20000000)
    KGS_W4H(13, 24, 20, 1, 1, 30000000)
    KGS_W4H(14, 24, 20, 1, 1, 40000000)
    KGS_W4H(15, 24, 20, 1, 1, 40000008)
    KGS_W4H(16, 24, 20, 1, 1, 40000002)
    KGS_W4H(17, 24, 20, 1, 1, 140000000)
    KGS_W4H(18, 24, 20, 1, 1, 240000000)
    KGS_W4H(19, 24, 20, 1, 1, 100000000)
    KGS_W4H(20, 24, 20, 1, 1, 200000000)
    default: return KGS_ERR_ARG;
  }
#undef KGS_W4H
  return (int)hipGetLastError();
}

// The production persistent kernel (default tile map, X = 0) with a chosen
// first-ticket mode and grid: mode 1 = static first ticket (production),
// 2 = every ticket from the queue; grid = workgroups (<= tiles; 0 = one per
// CU). For the collective-interaction sweep (bench/overlap_rccl.py).
KGS_EXPORT int kgs_exp_gemm_w4p_grid(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                     int ldc, int mode, int grid, hipStream_t s) {
  if (M <= 0 || N <= 0 || K < 384 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  if ((long)lda * 256 * 2 >= (1L << 31) || (long)ldb * 256 * 2 >= (1L << 31)) return KGS_ERR_SHAPE;
  const int ntiles = (M / 256) * (N / 256);
  if (grid <= 0) grid = cu_count();
  if (grid > ntiles) grid = ntiles;
  int* tq = kgs::tile_queue(s);
  if (!tq) return KGS_ERR_ARG;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  if (mode == 1)
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1>), dim3(grid), dim3(256), 0, s, a, b, c, nullptr, M,
                       N, K, lda, ldb, ldc, tq);
  else if (mode == 2)
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 2>), dim3(grid), dim3(256), 0, s, a, b, c, nullptr, M,
                       N, K, lda, ldb, ldc, tq);
  else
    return KGS_ERR_ARG;
  return (int)hipGetLastError();
}

// The persistent kernel's timing build (gemm_w4p.h TS) with tile map `map`
// (table below; 0 and 1 are production's for square / tall long-K problems). `stamps`: long long[grid][16], grid = min(tiles, CUs) (returned in *grid_out).
// Wait stamps of the persistent kernel (gemm_w4p.h WSB, round 6): s_memtime cycles every wave spent in
// its lgkm wait, barrier 1, vm wait and barrier 2, per K-step category. stamps: long long[grid][4][16].
// variant 0: production at 3-8 tiles per CU (nt C, deferred 4 x 4); 1: nt C, nothing deferred;
// 2: the tall long-K map (mirrored G8, temporal C); 3: map 0, temporal C (16 tiles per CU).
KGS_EXPORT int kgs_exp_gemm_w4p_waits(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                      int ldc, int variant, void* stamps, int* grid_out, hipStream_t s) {
  if (M <= 0 || N <= 0 || K < 768 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16 || !stamps) return KGS_ERR_ALIGN;
  if ((long)lda * 256 * 2 >= (1L << 31) || (long)ldb * 256 * 2 >= (1L << 31)) return KGS_ERR_SHAPE;
  const int ntiles = (M / 256) * (N / 256);
  const int grid = ntiles < cu_count() ? ntiles : cu_count();
  if (grid_out) *grid_out = grid;
  int* tq = kgs::tile_queue(s);
  if (!tq) return KGS_ERR_ARG;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto ts = (const unsigned short*)stamps;
  using namespace kgs::w4p;
  switch (variant) {
    case 0:
      hipLaunchKernelGGL((gemm_nt_w4p<kgs::EPI_NONE, 0, 1, true, false, 1000000, 4, 4>), dim3(grid), dim3(256), 0, s,
                         a, b, c, ts, M, N, K, lda, ldb, ldc, tq);
      break;
    case 1:
      hipLaunchKernelGGL((gemm_nt_w4p<kgs::EPI_NONE, 0, 1, true, false, 1000000>), dim3(grid), dim3(256), 0, s, a, b,
                         c, ts, M, N, K, lda, ldb, ldc, tq);
      break;
    case 2:
      hipLaunchKernelGGL((gemm_nt_w4p<kgs::EPI_NONE, 140000008, 1, false, false, 1000000>), dim3(grid), dim3(256), 0,
                         s, a, b, c, ts, M, N, K, lda, ldb, ldc, tq);
      break;
    case 3:
      hipLaunchKernelGGL((gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 1000000>), dim3(grid), dim3(256), 0, s, a,
                         b, c, ts, M, N, K, lda, ldb, ldc, tq);
      break;
    default:
      return KGS_ERR_ARG;
  }
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_exp_gemm_w4p_stamps(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                       int ldc, int map, void* stamps, int* grid_out, hipStream_t s) {
  if (M <= 0 || N <= 0 || K < 384 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16 || !stamps) return KGS_ERR_ALIGN;
  if ((long)lda * 256 * 2 >= (1L << 31) || (long)ldb * 256 * 2 >= (1L << 31)) return KGS_ERR_SHAPE;
  const int ntiles = (M / 256) * (N / 256);
  const int grid = ntiles < cu_count() ? ntiles : cu_count();
  if (grid_out) *grid_out = grid;
  int* tq = kgs::tile_queue(s);
  if (!tq) return KGS_ERR_ARG;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto ts = (const unsigned short*)stamps;
#define KGS_W4PT(ID, X)                                                                                          \
  case ID:                                                                                                        \
    hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, X, 1, false, true>), dim3(grid), dim3(256), 0, s, a, b, \
                       c, ts, M, N, K, lda, ldb, ldc, tq);                                                        \
    break;
  // map: 0 default, 1 mirrored G8 (production tall long-K), 2 G8, 3 mirrored, 4..6 XCD-blocked MAP 1..3
  switch (map) {
    KGS_W4PT(0, 0)
    KGS_W4PT(1, 140000008)
    KGS_W4PT(2, 8)
    KGS_W4PT(3, 140000000)
    KGS_W4PT(4, 10000000)
    KGS_W4PT(5, 20000000)
    KGS_W4PT(6, 30000000)
    default: return KGS_ERR_ARG;
  }
#undef KGS_W4PT
  return (int)hipGetLastError();
}

// fp8 four-wave persistent kernel (gemm_w4f8.h) with schedule knobs B1 / R / P
// and tile-map X; ids 40.. (kgs/ops/experiments.py W4F8). Aligned shapes,
// K (fp8) >= 768 and % 256; lengths in fp8 elements.
template <int B1_, int R_, int P_>
struct FK {
  static constexpr int B1 = B1_, R = R_, P = P_;
};

KGS_EXPORT int kgs_exp_gemm_fp8_w4f8(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                     int ldc, float alpha, int variant, hipStream_t s) {
  if (M <= 0 || N <= 0 || K < 768 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 256 || lda % 16 || ldb % 16 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  if ((long)(lda / 2) * 512 >= (1L << 31) || (long)(ldb / 2) * 512 >= (1L << 31)) return KGS_ERR_SHAPE;
  int* tq = kgs::tile_queue(s);
  if (!tq) return KGS_ERR_ARG;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  const int Kw = K / 2, ldaw = lda / 2, ldbw = ldb / 2;
  const int ntiles = (M / 256) * (N / 256);
  const dim3 pg(ntiles < cu_count() ? ntiles : cu_count());
#define KGS_W4F8(ID, X, B1, R, P)                                                                                   \
  case ID:                                                                                                          \
    hipLaunchKernelGGL((kgs::w4f8::gemm_fp8_w4p<kgs::EPI_NONE, X, FK<B1, R, P>>), pg, dim3(256), 0, s, a, b, c,     \
                       nullptr, M, N, Kw, ldaw, ldbw, ldc, alpha, nullptr, tq);                                     \
    break;
  switch (variant) {
    KGS_W4F8(40, 0, 12, 24, 1)
    KGS_W4F8(41, 0, 12, 12, 2)
    KGS_W4F8(42, 0, 10, 12, 2)
    KGS_W4F8(43, 0, 16, 24, 1)
    KGS_W4F8(44, 0, 10, 24, 1)
    KGS_W4F8(45, 0, 12, 20, 2)
    KGS_W4F8(46, 8, 12, 24, 1)
    KGS_W4F8(47, 140000000, 12, 24, 1)
    KGS_W4F8(48, 0, 14, 12, 2)
    KGS_W4F8(49, 0, 12, 8, 3)
    KGS_W4F8(50, 0, 10, 8, 3)
    KGS_W4F8(51, 0, 12, 6, 4)
    default: return KGS_ERR_ARG;
  }
#undef KGS_W4F8
  return (int)hipGetLastError();
}
