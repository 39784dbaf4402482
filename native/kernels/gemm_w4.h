// gemm_w4: the production 256x256x64 bf16 NT GEMM for gfx950 (MI355X) with
// FOUR waves (one per SIMD), each wave a 128x128 block of C (64 16x16 MFMA
// accumulators = 256 AGPRs), two 64 KiB LDS stages filled by
// buffer_load ... lds, and TWO barriers per 128-MFMA K-step.
//
// Why four waves: the 8-wave ping-pong of gemm_pipeline.h hands the matrix pipe
// over between the two waves of a SIMD every 16 MFMAs, and each hand-over costs
// about 90 cycles per 256-cycle MFMA block (profiles/gemm_tuning.md probe 9).
// Here a wave keeps the matrix pipe for a whole K-step and hides its own LDS
// reads and DMA issues in the gaps between its MFMAs, so the synchronisation is
// paid every 2048 MFMA cycles instead of every 256. LDS read traffic also drops
// by a third (a wave reads 128 rows of A and 128 of B per K-step; the 8-wave
// kernel reads 128 + 64 per wave with twice as many waves).
//
// K-step t (stage s = t & 1), fragments double-buffered by k-sub (32 k each):
//   part 1  MFMAs on k-sub 0 (f0) while the 16 ds_reads of k-sub 1 (f1) are
//           issued from stage s
//   barrier 1 (after MFMA B1): every wave's reads of stage s retired -> free
//   part 2a MFMAs on f1 with the 16 LDS-DMA issues of K-tile t+2 into stage s
//           spread over them (spreading wins: packed issue costs 7-13 %)
//   barrier 2 (R MFMAs before the end): vmcnt(16) -> K-tile t+1 has landed
//   part 2b last R MFMAs on f1 with the ds_reads of k-sub 0 of K-tile t+1
// The MFMA order inside a k-sub (ORD 1) is a growing square over (i, n) with
// reads alternating b0 a0 b1 a1 ..., so the first MFMA of a k-sub waits for 2
// reads, not 9. Knobs B1/R/P/ORD/X and their measurements:
// profiles/gemm_tuning.md (section "Four-wave kernel"); the measured
// alternatives are instantiated in native/experiments/gemm_w4h.hip.
//
// The LDS image is the 8-wave kernel's (128-B rows, 16-B chunk c of row r at
// c ^ ((r >> 1) & 7)): conflict-free ds_read_b128 fragments.
//
// Register allocation: the accumulators are NAMED AGPRs (acc_regs.h: fragment
// (i, n) in a[4q : 4q+3], q = NB i + n), reserved by KGS_ACC_RESERVE and
// touched only by asm. With the builtin MFMA hipcc renames accumulators between
// the two unrolled K-steps and repairs the loop with ~700 v_accvgpr moves per
// iteration; tied "+a" C++ operands (rounds 2-3) kept them in place inside the
// loop but let the allocator shuffle them at the loop exit, before the s_nop
// hazard padding (v_accvgpr_read of a[248:251] four instructions after the MFMA
// that wrote it; the SiLU-epilogue instantiation returned stale fragments).
// Named registers leave the allocator nothing to move, and the epilogue's asm
// reads stay after the padding (volatile asm keeps program order).
#pragma once

#include <type_traits>

#include "acc_regs.h"
#include "kgs_common.h"


// Generalisations (round 2, for the serving decode GEMMs):
//   BN   256 (production square tile) or 128 (256x128: twice the tiles for the
//        short-M / narrow-N decode projections); a wave owns 128 x BN/2.
//   MODE bit 0  bounded M: A rows past M read as zeros (buffer resource ends at
//               the last valid row), stores predicated -- any M, e.g. a decode
//               batch of 200.
//   MODE bit 1  split-K: gridDim.x = tiles x slices; slice s computes K columns
//               [s K, (s + 1) K) and stores an fp32 partial tile to
//               ((float*)C)[s][M][N] for kgs::splitk_reduce.
//   MODE bit 3  128-row tiles (BM 128): each wave owns 64 x BN/2 (4 A fragments
//               per k-sub). For decode batches of 65-128 rows a 256-row tile
//               spends half its MFMAs on rows past M; this one does not.
//   X digit 10^6  SwiGLU: B is a fused gate|up weight of N = 2I rows (gate rows
//               [0, I), up rows [I, 2I)). A tile stages gate and up rows in
//               alternating 32-row DMA groups (gate block tn BN/2 .., up block
//               I + tn BN/2 ..), so every wave holds the gate and up columns of
//               the same outputs, and the epilogue stores silu(g) * u: a
//               [M, I] activation with no [M, 2I] round trip and no silu_mul
//               launch. Same roundings as gate|up GEMM + silu_mul.

namespace kgs {
namespace w4 {

constexpr int BK = 64;
constexpr int GM = 4;  // tile-group height (production choice)

template <int BM, int BN>
struct Shape {
  static_assert(BN == 256 || BN == 128, "BN must be 256 or 128");
  static_assert(BM == 256 || BM == 128, "BM must be 256 or 128");
  static constexpr int MA = BM / 32;         // A fragments per wave per k-sub (8 or 4)
  static constexpr int NB = BN / 32;         // B fragments per wave per k-sub (8 or 4)
  static constexpr int OPA = BM * BK * 2;    // A operand of one stage: 32 or 16 KiB
  static constexpr int OPB = BN * BK * 2;    // B operand of one stage: 32 or 16 KiB
  static constexpr int STAGE = OPA + OPB;
  static constexpr int LDS_BYTES = 2 * STAGE;
  static constexpr int HM = MA * NB;         // MFMAs per k-sub
  static constexpr int KM = 2 * HM;          // MFMAs per K-step
  static constexpr int NR = MA + NB;         // fragment reads per k-sub
};

// DMA instructions per wave per stage: A BM rows / (8 rows x 4 waves), B BN / 32
template <int BM, int BN>
constexpr int dma_per_stage() { return BM / 32 + BN / 32; }

struct Ctx {
  char* smem;
  __amdgpu_buffer_rsrc_t ra, rb;
  __amdgpu_buffer_rsrc_t rb2;  // SwiGLU: the up block (rb holds the gate block)
  int voa, vob;     // per-lane DMA byte offsets (row, swizzled chunk)
  int sa32, sb32;   // bytes between DMA row groups (32 rows)
  int w, wr, wc;
  int ro0, ro1;     // per-lane fragment byte offsets, k-sub 0 / 1
  int nt;
};

template <int MA, int NB>
struct Frag {
  bf16x8 a[MA];
  bf16x8 b[NB];
};

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// DMA instruction j of operand OP (0 = A: j < BM/32, 1 = B: j < BN/32) for the
// K-tile starting at k0 into stage st: rows j*32 + w*8 + lane/8, 1 KiB = 8 rows
// of 128 B. AUX: cache-policy bits of the load (0 = default; 16 = sc1). SW:
// SwiGLU staging of B (groups alternate gate / up, see the MODE notes above).
template <int BM, int BN, int OP, int AUX = 0, bool SW = false, bool PK = false>
__device__ __forceinline__ void dma(const Ctx& c, int st, int j, int k0) {
  using S = Shape<BM, BN>;
  char* dst = c.smem + st * S::STAGE + OP * S::OPA + (j * 4 + c.w) * 1024;
  if constexpr (OP == 1 && PK) {
    // packed B ([N/BN][K/BK][BN][BK], see PACKB): K-tile k0 / BK of this
    // panel is one contiguous BN x 128 B block
    const int so = j * c.sb32 + k0 * BN * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rb, (KGS_LDS void*)dst, 16, c.vob, so, 0, AUX);
  } else if constexpr (OP == 1 && SW) {
    const int so = (j >> 1) * c.sb32 + k0 * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds((j & 1) ? c.rb2 : c.rb, (KGS_LDS void*)dst, 16, c.vob, so, 0, AUX);
  } else {
    const int so = j * (OP ? c.sb32 : c.sa32) + k0 * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(OP ? c.rb : c.ra, (KGS_LDS void*)dst, 16, OP ? c.vob : c.voa, so, 0,
                                             AUX);
  }
}

// X: the knob bag of the kernel template (GROUP_M = X % 100, AUX = X / 100 % 100,
// DMA window = X / 10^4 % 100, SW = X / 10^6 % 10, MAP = X / 10^7 % 10,
// DMA operand order = X / 10^8 % 10, packed B = X / 10^9 == 1). AUX < 50: the
// cache-policy bits of both operands' loads; AUX >= 50: AUX - 50 on B's loads
// only (52: B non-temporal -- decode weights that one CU streams once -- while
// A, re-read by every workgroup, keeps the default policy).
template <int BM, int BN, int X>
__device__ __forceinline__ void dma_any(const Ctx& c, int st, int j, int k0) {
  constexpr int AUXX = (X / 100) % 100;
  constexpr int AUX = AUXX >= 50 ? AUXX - 50 : AUXX;   // B
  constexpr int AUXA = AUXX >= 50 ? 0 : AUXX;          // A
  constexpr bool SW = (X / 1000000) % 10 != 0;
  constexpr int ORDB = (X / 100000000) % 10;  // 1: the B operand's DMAs first, 2: A and B interleaved
  constexpr bool PK = (X / 1000000000) == 1;  // B packed by K-tile (PACKB)
  constexpr int JA = BM / 32, JB = BN / 32;
  if constexpr (ORDB == 1) {
    if (j < JB) dma<BM, BN, 1, AUX, SW, PK>(c, st, j, k0); else dma<BM, BN, 0, AUXA>(c, st, j - JB, k0);
  } else if constexpr (ORDB == 2 && JA == JB) {
    if (j & 1) dma<BM, BN, 1, AUX, SW, PK>(c, st, j >> 1, k0); else dma<BM, BN, 0, AUXA>(c, st, j >> 1, k0);
  } else {
    if (j < JA) dma<BM, BN, 0, AUXA>(c, st, j, k0); else dma<BM, BN, 1, AUX, SW, PK>(c, st, j - JA, k0);
  }
}

__device__ __forceinline__ bf16x8 frag(const char* p) { return *(const bf16x8*)p; }

template <int BM, int BN, int SUB>
__device__ __forceinline__ const char* abase(const Ctx& c, int st) {
  return c.smem + st * Shape<BM, BN>::STAGE + c.wr * (BM / 2) * 128 + (SUB ? c.ro1 : c.ro0);
}
template <int BM, int BN, int SUB>
__device__ __forceinline__ const char* bbase(const Ctx& c, int st) {
  return c.smem + st * Shape<BM, BN>::STAGE + Shape<BM, BN>::OPA + c.wc * (BN / 2) * 128 + (SUB ? c.ro1 : c.ro0);
}

// One MFMA on the named accumulator (I, N). Operands swapped (B first) so a lane
// holds C[m = lane&15][n = 4*(lane>>4)+e]. asm MFMAs are invisible to the
// hazard recognizer: the only hazard left (AGPR results read by VALU) is padded
// before the epilogue.
template <int MA, int NB, int I, int N>
__device__ __forceinline__ void mma(const Frag<MA, NB>& f) {
  accr::mfma<I * NB + N>(f.b[N], f.a[I]);
}

// Compile-time loop: f(std::integral_constant<int, i>) for i in [B, E).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Row I of the wave's accumulator grid (NB fragments) into VGPRs.
template <int NB, int I, int N = 0>
__device__ __forceinline__ void read_row(f32x4 (&v)[NB]) {
  if constexpr (N < NB) {
    v[N] = accr::read<I * NB + N>();
    read_row<NB, I, N + 1>(v);
  }
}

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// MFMA order inside a k-sub. ORD 0: i-major (a[i] over all n), reads b0..b(NB-1)
// then a0..a(MA-1). ORD 2: n-major (b[n] over all i), reads a0..a(MA-1) then
// b0..b(NB-1). ORD 1: "growing square": reads alternate b0 a0 b1 a1 ...
// (then the remaining fragments of the larger side), and each MFMA (i, n) runs
// right after the read that completes its pair, so the first MFMA of a k-sub
// waits for 2 reads.
struct MOrder {
  unsigned char i[64], n[64];
};

// read r of a k-sub: which fragment (0 = b, 1 = a) and its index
constexpr int rd_isa(int ord, int ma, int nb, int r) {
  return ord == 0 ? (r >= nb)
       : ord == 2 ? (r < ma)
                  : (r < 2 * (ma < nb ? ma : nb) ? (r & 1) : (ma > nb ? 1 : 0));
}
constexpr int rd_idx(int ord, int ma, int nb, int r) {
  return ord == 0 ? (r < nb ? r : r - nb)
       : ord == 2 ? (r < ma ? r : r - ma)
                  : (r < 2 * (ma < nb ? ma : nb) ? (r >> 1) : r - (ma < nb ? ma : nb));
}

constexpr MOrder make_order(int ord, int ma, int nb) {
  MOrder o{};
  int k = 0;
  if (ord == 0) {
    for (int i = 0; i < ma; ++i)
      for (int n = 0; n < nb; ++n) { o.i[k] = i; o.n[k] = n; ++k; }
    return o;
  }
  if (ord == 2) {  // n-major: B fragment n (the MFMA's first operand) held for ma MFMAs
    for (int n = 0; n < nb; ++n)
      for (int i = 0; i < ma; ++i) { o.i[k] = i; o.n[k] = n; ++k; }
    return o;
  }
  bool ha[8] = {}, hb[8] = {};
  for (int r = 0; r < ma + nb; ++r) {
    const int x = rd_idx(ord, ma, nb, r);
    if (rd_isa(ord, ma, nb, r)) {
      ha[x] = true;
      for (int n = 0; n < nb; ++n)
        if (hb[n]) { o.i[k] = x; o.n[k] = n; ++k; }
    } else {
      hb[x] = true;
      for (int i = 0; i < ma; ++i)
        if (ha[i]) { o.i[k] = i; o.n[k] = x; ++k; }
    }
  }
  return o;
}

template <int ORD, int MA, int NB>
struct Order {
  static constexpr MOrder o = make_order(ORD, MA, NB);
};

struct StepPtrs {
  const char *pa1, *pb1, *pa0, *pb0;
  int k0;
};

// s_waitcnt vmcnt(N) for the per-stage DMA counts of the tile shapes
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if constexpr (N == 36) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
  else if constexpr (N == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if constexpr (N >= 0 && N < 64) {
    // other counts (gemm_w4p.h deferred C stores: ND + stores per K-step): the
    // gfx9 encoding vmcnt[3:0] | vmcnt[5:4] << 14, expcnt 7, lgkmcnt 15
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
    __builtin_amdgcn_sched_barrier(0);
  } else {
    static_assert(N == 8, "unsupported vmcnt");
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
}

// MFMA k of the K-step and what follows it, all decided at compile time:
//   k < NR              ds_read f1 (k-sub 1 of this K-tile) read k
//   k == B1 - 1         lgkmcnt(0) + barrier 1 (stage ST free)
//   k in [B1, KM - R)   the ND LDS-DMA issues of K-tile t+2, evenly spread
//   k == KM - R - 1     vmcnt((NS - 1) ND) + barrier 2 (K-tile t+1 visible)
//   k >= KM - R         P ds_reads of f0 (K-tile t+1, k-sub 0) after each MFMA
template <int BM, int BN, int ST, int B1, int R, int P, int ORD, int X, int NS, int K>
__device__ __forceinline__ void kbody(const Ctx& c, const StepPtrs& sp, Frag<BM / 32, BN / 32>& f0,
                                      Frag<BM / 32, BN / 32>& f1) {
  using S = Shape<BM, BN>;
  constexpr int MA = S::MA, NB = S::NB, KM = S::KM, HM = S::HM, NR = S::NR, ND = dma_per_stage<BM, BN>();
  if constexpr (K < KM) {
    constexpr int mi = Order<ORD, MA, NB>::o.i[K % HM], mn = Order<ORD, MA, NB>::o.n[K % HM];
    if constexpr (K < HM) mma<MA, NB, mi, mn>(f0); else mma<MA, NB, mi, mn>(f1);
    if constexpr (K < NR) {
      constexpr int x = rd_idx(ORD, MA, NB, K);
      if constexpr (rd_isa(ORD, MA, NB, K)) f1.a[x] = frag(sp.pa1 + x * 2048); else f1.b[x] = frag(sp.pb1 + x * 2048);
    }
    if constexpr (K >= B1 && K < KM - R) {
      // MFMAs that carry the DMA issues: the whole window, or the first W (X / 10000 % 100) of it
      constexpr int NW = ((X / 10000) % 100) ? (X / 10000) % 100 : KM - R - B1;
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        if (B1 + (j * NW) / ND == K) dma_any<BM, BN, X>(c, ST, j, sp.k0);
      }
    }
    if constexpr (K >= KM - R) {
      constexpr int q = K - (KM - R);
#pragma unroll
      for (int e = q * P; e < (q + 1) * P && e < NR; ++e) {
        const int x = rd_idx(ORD, MA, NB, e);
        if (rd_isa(ORD, MA, NB, e)) f0.a[x] = frag(sp.pa0 + x * 2048); else f0.b[x] = frag(sp.pb0 + x * 2048);
      }
    }
    fence();
    if constexpr (K == B1 - 1) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage ST retired
      bar();
    }
    if constexpr (K == KM - R - 1) {
      // own DMA of K-tile t+1 landed (the (NS - 1) ND issued after it belong to t+2 .. t+NS)
      wait_vm<(NS - 1) * ND>();
      bar();
    }
    kbody<BM, BN, ST, B1, R, P, ORD, X, NS, K + 1>(c, sp, f0, f1);
  }
}

// One K-step: a single pinned sequence of KM MFMAs (the first half on f0 = k-sub 0,
// the second on f1 = k-sub 1) with the reads, DMA issues and the two barriers
// placed between them (kbody).
template <int BM, int BN, int ST, int B1, int R, int P, int ORD, int X, int NS = 2>
__device__ __forceinline__ void kstep(const Ctx& c, Frag<BM / 32, BN / 32>& f0, Frag<BM / 32, BN / 32>& f1,
                                      int t) {
  using S = Shape<BM, BN>;
  static_assert(B1 >= S::NR && B1 + dma_per_stage<BM, BN>() <= S::KM - R && S::NR <= R * P, "bad K-step schedule");
  StepPtrs sp;
  sp.pa1 = abase<BM, BN, 1>(c, ST);
  sp.pb1 = bbase<BM, BN, 1>(c, ST);
  sp.pa0 = abase<BM, BN, 0>(c, (ST + 1) % NS);
  sp.pb0 = bbase<BM, BN, 0>(c, (ST + 1) % NS);
  int tl = t + NS;
  tl = tl < c.nt ? tl : c.nt - 1;  // past the end: harmless re-load into the free stage
  sp.k0 = tl * BK;
  kbody<BM, BN, ST, B1, R, P, ORD, X, NS, 0>(c, sp, f0, f1);
}

// Production knobs per tile shape: barrier 1 after MFMA B1, R MFMAs after
// barrier 2, P reads per MFMA there, growing-square order, GROUP_M 4.
template <int BM, int BN>
struct Knobs;
template <>
struct Knobs<256, 256> {
  static constexpr int B1 = 24, R = 20, P = 1, ORD = 1, X = 0;
};
template <>
struct Knobs<256, 128> {
  static constexpr int B1 = 18, R = 16, P = 1, ORD = 1, X = 0;
};
template <>
struct Knobs<128, 256> {
  static constexpr int B1 = 18, R = 16, P = 1, ORD = 1, X = 0;
};
template <>
struct Knobs<128, 128> {
  static constexpr int B1 = 10, R = 10, P = 1, ORD = 1, X = 0;
};

template <int MODE>
constexpr int tile_m() { return (MODE & 8) ? 128 : 256; }

// MODE bits 4-5: LDS stages - 2 (round 3, decode GEMMs). With NS stages the
// DMAs of K-tile t + NS are issued during K-step t, so NS - 1 K-tiles are in
// flight while one is consumed: for the short-M, weight-streaming shapes the
// K-step is bound by load latency, not by the MFMAs.
template <int MODE>
constexpr int stages() { return 2 + ((MODE >> 4) & 3); }

// XCD-blocked tile map (X digit 10^7 = MAP, round 3). The default map
// (xcd_remap + GROUP_M) gives XCD x a contiguous run of tile ids; with groups
// along M that makes all eight XCDs of a wave work on the SAME B columns at the
// same time (8192 x 4096: wave 1 = every A row x tn 0..7), so every B line is
// requested by all eight XCDs at once and the wave's footprint (all of A + half
// of B) is 294 MB at K = 14336, more than the 256 MB MALL. MAP 1..3 give each
// wave (256 tiles, one per CU) a compact super-block and split it into eight
// XCD blocks, so a line is shared by at most four XCDs:
//   MAP 1: XCD block 8 (M) x 4 (N) tiles, XCD blocks 2 x 4   -> super-block 16 x 16
//   MAP 2: XCD block 4 x 8,              XCD blocks 4 x 2   -> 16 x 16
//   MAP 3: XCD block 8 x 4,              XCD blocks 4 x 2   -> 32 x 8
//   MAP 4: not blocked -- the default GROUP_M map with M and N exchanged
// Waves walk super-blocks N-fastest, so consecutive waves share A rows. The
// hardware dispatches workgroup b to XCD b % 8 and the first 256 workgroups
// form wave 1, so XCD x's loc-th workgroup (loc = b / 8) takes tile loc % 32 of
// its block loc / 32 of super-block loc / 32. Shapes whose tile grid is not a
// whole number of super-blocks keep the default map (returns false).
template <int MAP>
__host__ __device__ __forceinline__ bool blocked_tile(int bid, int ntm, int ntn, int& tm, int& tn) {
  static_assert(MAP >= 1 && MAP <= 3, "blocked maps are 1..3");
  constexpr int XBM = MAP == 2 ? 4 : 8, XBN = MAP == 2 ? 8 : 4;  // XCD block, tiles
  constexpr int AM = MAP == 1 ? 2 : 4, AN = 8 / AM;               // XCD blocks per super-block
  constexpr int SBM = XBM * AM, SBN = XBN * AN, PER = XBM * XBN;
  if (ntm % SBM || ntn % SBN) return false;
  const int xcd = bid & 7, loc = bid >> 3;
  const int sb = loc / PER, p = loc % PER;
  const int nsbn = ntn / SBN;
  const int sbm = sb / nsbn, sbn = sb - sbm * nsbn;
  const int xm = xcd % AM, xn = xcd / AM;
  tm = sbm * SBM + xm * XBM + p % XBM;
  tn = sbn * SBN + xn * XBN + p / XBM;
  return true;
}

// Workgroup -> (split-K slice, tile row, tile column): the default map
// (xcd_remap + GROUP_M), a blocked map (MAP 1..3) or GROUP_N (MAP 4). A
// bijection from [0, grid) onto slices x tiles for every MAP
// (tests/test_gemm_tile_map.py checks it on the host).
template <int X, bool SPLITK>
__host__ __device__ __forceinline__ void tile_of(int bid, int grid, int ntm, int ntn, int& slice, int& tm, int& tn) {
  const int nwg = ntm * ntn;
  // split-K: remap over the whole grid, so the blocks of one XCD share a slice
  const int nslice = SPLITK ? grid / nwg : 1;
  const int wga = SPLITK ? xcd_remap(bid, nwg * nslice) : xcd_remap(bid, nwg);
  slice = SPLITK ? wga / nwg : 0;
  const int wg = SPLITK ? wga - slice * nwg : wga;
  constexpr int G = (X % 100) ? X % 100 : GM;
  constexpr int MAP = (X / 10000000) % 10;
  bool mapped = false;
  if constexpr (!SPLITK && MAP >= 1 && MAP <= 3) mapped = blocked_tile<MAP>(bid, ntm, ntn, tm, tn);
  if constexpr (!SPLITK && MAP == 4) {
    // the default map mirrored: groups of G tile-COLUMNS walked down M. For
    // M > N this is what the default map is for the transposed problem, e.g.
    // 8192 x 4096 x 14336 then gets 4096 x 8192 x 14336's order.
    const int per_group = G * ntm;
    const int group = wg / per_group;
    const int first_n = group * G;
    const int gsz = ntn - first_n < G ? ntn - first_n : G;
    tn = first_n + (wg % per_group) % gsz;
    tm = (wg % per_group) / gsz;
    mapped = true;
  }
  if (!mapped) {
    const int per_group = G * ntn;
    const int group = wg / per_group;
    const int first_m = group * G;
    const int gsz = ntm - first_m < G ? ntm - first_m : G;
    tm = first_m + (wg % per_group) % gsz;
    tn = (wg % per_group) / gsz;
  }
}

template <int EPI, int BN = 256, int MODE = 0, int B1 = Knobs<tile_m<MODE>(), BN>::B1,
          int R = Knobs<tile_m<MODE>(), BN>::R, int P = Knobs<tile_m<MODE>(), BN>::P,
          int ORD = Knobs<tile_m<MODE>(), BN>::ORD, int X = Knobs<tile_m<MODE>(), BN>::X>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int BM = tile_m<MODE>();
  using S = Shape<BM, BN>;
  constexpr int MA = S::MA, NB = S::NB, ND = dma_per_stage<BM, BN>();
  constexpr bool SW = (X / 1000000) % 10 != 0;
  static_assert(!SW || (EPI == EPI_NONE && (MODE & 2) == 0), "SwiGLU: no bias epilogue, no split-K");
  constexpr bool BNDM = (MODE & 1) != 0, SPLITK = (MODE & 2) != 0;
  // X digit 10^9 = 1, PACKB (round 3, decode weights): B is stored tile-panel
  // major, [N / BN][K / BK][BN][BK], so each K-step's B block is ONE contiguous
  // BN x 128 B run in HBM instead of BN rows 128 B each, K * 2 bytes apart. For
  // SwiGLU the panel already holds the gate / up 32-row groups interleaved.
  constexpr bool PACKB = (X / 1000000000) == 1;
  constexpr int NS = stages<MODE>();
  static_assert(NS * S::STAGE <= 160 * 1024, "LDS stages exceed 160 KiB");
  __shared__ __attribute__((aligned(1024))) char smem[NS * S::STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = BNDM ? (M + BM - 1) / BM : M / BM, ntn = N / BN;
  int slice, tm, tn;
  tile_of<X, SPLITK>((int)blockIdx.x, (int)gridDim.x, ntm, ntn, slice, tm, tn);
  const int rows_a = BNDM ? min(M - tm * BM, BM) : BM;

  Ctx c;
  c.smem = smem;
  c.w = w;
  c.wr = w >> 1;
  c.wc = w & 1;
  c.nt = K / BK;
  const long koff = SPLITK ? (long)slice * K : 0;  // split-K: K is the slice length
  c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * BM * lda + koff), 0, rows_a * lda * 2, 0x00020000);
  if constexpr (PACKB) {
    // B packed by K-tile: tile column tn's panel is (ldb / BK) blocks of BN x BK
    // (ldb = the full K), slice s starts at block s K / BK; rows 128 B apart
    c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * BN * ldb + koff * BN), 0, K * BN * 2,
                                             0x00020000);
  } else if constexpr (SW) {
    c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * (BN / 2) * ldb + koff), 0, (BN / 2) * ldb * 2,
                                             0x00020000);
    c.rb2 = __builtin_amdgcn_make_buffer_rsrc((void*)(B + ((long)N / 2 + (long)tn * (BN / 2)) * ldb + koff), 0,
                                              (BN / 2) * ldb * 2, 0x00020000);
  } else {
    c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * BN * ldb + koff), 0, BN * ldb * 2, 0x00020000);
  }
  c.sa32 = 32 * lda * 2;
  c.sb32 = 32 * (PACKB ? BK : ldb) * 2;
  {
    const int row = w * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    c.voa = (row * lda + ch * 8) * 2;
    c.vob = (row * (PACKB ? BK : ldb) + ch * 8) * 2;
    const int fr = lane & 15, fq = lane >> 4, f = fr >> 1;
    c.ro0 = fr * 128 + ((fq ^ f) * 16);
    c.ro1 = fr * 128 + (((4 + fq) ^ f) * 16);
  }

  KGS_ACC_RESERVE();
  static_for<0, MA * NB>([](auto q) { accr::zero<decltype(q)::value>(); });

  // prologue: K-tiles 0 .. NS-1 into stages 0 .. NS-1, k-sub 0 of K-tile 0 into f0
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int kt = (st < c.nt ? st : c.nt - 1) * BK;
#pragma unroll
    for (int j = 0; j < ND; ++j) dma_any<BM, BN, X>(c, st, j, kt);
  }
  wait_vm<(NS - 1) * ND>();
  bar();
  Frag<MA, NB> f0, f1;
  {
    const char* pa = abase<BM, BN, 0>(c, 0);
    const char* pb = bbase<BM, BN, 0>(c, 0);
#pragma unroll
    for (int e = 0; e < S::NR; ++e) {  // same order as the loop's reads
      const int x = rd_idx(ORD, MA, NB, e);
      if (rd_isa(ORD, MA, NB, e)) f0.a[x] = frag(pa + x * 2048); else f0.b[x] = frag(pb + x * 2048);
    }
  }
  // nothing outstanding on lgkm at loop entry: otherwise the waitcnt pass merges
  // the preheader's scalar loads into the loop header and waits lgkmcnt(0) there
  __builtin_amdgcn_s_waitcnt(0xc07f);

  if constexpr (NS == 2) {
    for (int t = 0; t < c.nt; t += 2) {
      kstep<BM, BN, 0, B1, R, P, ORD, X>(c, f0, f1, t);
      kstep<BM, BN, 1, B1, R, P, ORD, X>(c, f0, f1, t + 1);
    }
  } else {
    // K-tile t lives in stage t % NS; the tail steps of a partial round are
    // skipped uniformly by the whole workgroup
    for (int t = 0; t < c.nt; t += NS) {
      kstep<BM, BN, 0, B1, R, P, ORD, X, NS>(c, f0, f1, t);
      if (t + 1 < c.nt) kstep<BM, BN, 1, B1, R, P, ORD, X, NS>(c, f0, f1, t + 1);
      if (t + 2 < c.nt) kstep<BM, BN, 2 % NS, B1, R, P, ORD, X, NS>(c, f0, f1, t + 2);
      if constexpr (NS == 4)
        if (t + 3 < c.nt) kstep<BM, BN, 3, B1, R, P, ORD, X, NS>(c, f0, f1, t + 3);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail re-loads before LDS is released
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA -> v_accvgpr_read hazard

  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (SPLITK) {
    // fp32 partial tile, row-major [M][N]: one 16-B store per lane per fragment
    float* part = (float*)C + (long)slice * M * N;
    static_for<0, MA>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int row = tm * BM + c.wr * (BM / 2) + i * 16 + fr;
      f32x4 v[NB];
      read_row<NB, i>(v);
      if (BNDM && row >= M) return;
#pragma unroll
      for (int n = 0; n < NB; ++n)
        *(f32x4*)(part + (long)row * N + tn * BN + c.wc * (BN / 2) + n * 16 + fq * 4) = v[n];
    });
    return;
  }
  if constexpr (SW) {
    // out fragment q (16 columns) = silu(gate fragment ng) * up fragment ng + 2,
    // ng = 4 (q / 2) + q % 2; pairs (q, q + 1) share one 16-B store per lane
    static_for<0, MA>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int row = tm * BM + c.wr * (BM / 2) + i * 16 + fr;
      unsigned short* crow = C + (long)row * ldc;
      const bool row_ok = !BNDM || row < M;
      f32x4 v[NB];
      read_row<NB, i>(v);
#pragma unroll
      for (int q = 0; q < NB / 2; q += 2) {
        uint2 o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ng = 4 * ((q + h) / 2) + (q + h) % 2;
          const f32x4 g = v[ng], u = v[ng + 2];
          float r[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gf = bf2f(f2bf(g[e]));
            r[e] = gf / (1.0f + __expf(-gf)) * bf2f(f2bf(u[e]));
          }
          o[h].x = pack_bf16x2(r[0], r[1]);
          o[h].y = pack_bf16x2(r[2], r[3]);
        }
        auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
        auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
        const uint4 qv = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        const int col0 = tn * (BN / 2) + c.wc * (BN / 4) + q * 16;
        if (row_ok) *(uint4*)(crow + col0 + (fq & 1) * 16 + (fq >> 1) * 8) = qv;
      }
    });
    return;
  }
  // epilogue: bias + activation, then pair n-tiles (n, n+1) with
  // v_permlane16_swap -> one 16-B store per lane (guide T21)
  float bv[NB][4];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[n][e] = 0.f;
    if constexpr (epi_bias<EPI>()) {
      const bf16x4 bb = *(const bf16x4*)(bias + tn * BN + c.wc * (BN / 2) + n * 16 + fq * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[n][e] = bf2f((unsigned short)bb[e]);
    }
  }
  static_for<0, MA>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int row = tm * BM + c.wr * (BM / 2) + i * 16 + fr;
    unsigned short* crow = C + (long)row * ldc;
    const bool row_ok = !BNDM || row < M;
    // EPI_ADDC: the row group's residual chunks are loaded together, before
    // the first store (one memory latency per group, not one per store)
    uint4 old[NB / 2];
    if constexpr (EPI == EPI_ADDC) {
#pragma unroll
      for (int p = 0; p < NB / 2; ++p)
        old[p] = row_ok ? *(const uint4*)(crow + tn * BN + c.wc * (BN / 2) + p * 32 + (fq & 1) * 16 + (fq >> 1) * 8)
                        : make_uint4(0, 0, 0, 0);
    }
    f32x4 vr[NB];
    read_row<NB, i>(vr);
#pragma unroll
    for (int n = 0; n < NB; n += 2) {
      uint2 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 v = vr[n + h];
        o[h].x = pack_bf16x2(epilogue<EPI>(v[0], bv[n + h][0]), epilogue<EPI>(v[1], bv[n + h][1]));
        o[h].y = pack_bf16x2(epilogue<EPI>(v[2], bv[n + h][2]), epilogue<EPI>(v[3], bv[n + h][3]));
      }
      auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
      auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
      const uint4 qv = make_uint4(sx[0], sy[0], sx[1], sy[1]);
      const int col0 = tn * BN + c.wc * (BN / 2) + n * 16;
      uint4* dst = (uint4*)(crow + col0 + (fq & 1) * 16 + (fq >> 1) * 8);
      if constexpr (EPI == EPI_ADDC) {
        if (row_ok) *dst = add_bf16x8(old[n / 2], qv);
      } else {
        if (row_ok) *dst = qv;
      }
    }
  });
}

}  // namespace w4
}  // namespace kgs
