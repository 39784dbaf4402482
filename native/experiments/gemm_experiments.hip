// Measured alternatives to the production GEMM (native/kernels/gemm_bf16.hip),
// kept so every result in profiles/gemm_tuning.md can be re-run. Built into
// its own opt-in library, kgs/_native/libkgs_experiments.so (never loaded by
// production code; Python: kgs.ops.experiments). Variant ids:
//
//  * 15 narrow_store -- production schedule with the 2 x 8-B store tail.
//  * 20 persistent -- the production pipeline as a persistent tile walk.
//  * 21/22 vgpr_stage(2) -- VGPR staging instead of LDS-DMA.
//  * fp8 17-19 -- GROUP_M 8 / 16 / 2 of the fp8 pipeline.
//  * gemm_nt_256pl (14) -- lockstep 8 waves with in-wave software pipelining.
//  * gemm_nt_256p32 (10) -- 32-MFMA phases (half the barriers), 160 KiB ring.
//  * gemm_nt_256w4 (3) -- 4 waves x 128x128 with AGPR-pinned asm MFMAs.
//  * S-knob instantiations of the production pipeline (4-9, 11-13): setprio,
//    GROUP_M, first schedule, lockstep, and the L2 / 2xMFMA timing probes.
//
// All of them are correct (bitwise equal to production where they compute the
// product) except the timing probes 9 and 11, which are wrong by construction.
#include "gemm_pipeline.h"

namespace kgs {

// ---------------------------------------------------------------------------
// gemm_nt_256pl: lockstep 8 waves, in-wave software pipelining, ONE barrier per
// 16-MFMA phase. Both waves of a SIMD run their MFMA blocks concurrently (32
// MFMAs per SIMD per barrier), and each phase's ds_reads fetch the NEXT
// quadrant's fragments, so LDS latency hides under the MFMAs instead of behind
// a partner wave. Two A fragment sets (A0/A1 halves) and two B sets:
//   phase q0 (A0,B0) reads B1(t)   q1 (A0,B1) reads A1(t)
//   phase q2 (A1,B0) reads -       q3 (A1,B1) reads A0(t+1), B0(t+1)
// Stream B0,A0,B1,A1, half-tile h issued at phase h-8, vmcnt(10):
//   RAW: every half-tile is read >= 6 phases after its issue (5 in flight);
//   WAR: a slot is refilled >= 1 phase after its last read, and reads of phase
//        r are retired (lgkmcnt(0)) before the barrier that ends phase r.
// ---------------------------------------------------------------------------
namespace gpl {

using g256::BM;
using g256::BN;
using g256::BK;
using g256::HALF_BYTES;
using g256::BUF_BYTES;
using g256::LDS_BYTES;
using g256::P_A0;
using g256::P_A1;
using g256::P_B0;
using g256::P_B1;
constexpr int GM = 4;

struct Regs {
  bf16x8 a[2][4][2];      // [A half][m-tile][k-sub]
  bf16x8 b[2][2][2];      // [B half][n-tile][k-sub]
  f32x4 acc[2][4][2][2];  // [m-half][m-tile][n-half][n-tile]
};

template <int AH>
__device__ __forceinline__ void read_a(const g256::Ctx& c, Regs& R, const char* half) {
  const char* p = half + c.wr * 64 * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    R.a[AH][i][0] = *(const bf16x8*)(p + i * 16 * 128 + c.ro0);
    R.a[AH][i][1] = *(const bf16x8*)(p + i * 16 * 128 + c.ro1);
  }
}

template <int BH>
__device__ __forceinline__ void read_b(const g256::Ctx& c, Regs& R, const char* half) {
  const char* p = half + c.wc * 32 * 128;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    R.b[BH][n][0] = *(const bf16x8*)(p + n * 16 * 128 + c.ro0);
    R.b[BH][n][1] = *(const bf16x8*)(p + n * 16 * 128 + c.ro1);
  }
}

template <int MH, int NH>
__device__ __forceinline__ void mma(Regs& R) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        R.acc[MH][i][NH][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(R.b[NH][n][s], R.a[MH][i][s],
                                                                        R.acc[MH][i][NH][n], 0, 0, 0);
}

template <int QP>
__device__ __forceinline__ void phase(const g256::Ctx& c, Regs& R, int it) {
  constexpr int q = QP & 3;
  constexpr int cbuf = QP >> 2;
  const char* buf = c.smem + cbuf * BUF_BYTES;
  const char* nbuf = c.smem + (cbuf ^ 1) * BUF_BYTES;
  if constexpr (q == 0) read_b<1>(c, R, buf + P_B1 * HALF_BYTES);
  if constexpr (q == 1) read_a<1>(c, R, buf + P_A1 * HALF_BYTES);
  if constexpr (q == 3) {
    read_a<0>(c, R, nbuf + P_A0 * HALF_BYTES);
    read_b<0>(c, R, nbuf + P_B0 * HALF_BYTES);
  }
  // half-tile h = 8*it + QP + 8; stream B0,A0,B1,A1
  constexpr int hoff = QP + 8;
  constexpr int toff = hoff >> 2;
  constexpr int jp = hoff & 3;
  constexpr int part = jp == 0 ? P_B0 : jp == 1 ? P_A0 : jp == 2 ? P_B1 : P_A1;
  int t = 2 * it + toff;
  t = t < c.nt ? t : c.nt - 1;
  g256::issue<part>(c, toff & 1, t * BK);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (q == 0) mma<0, 0>(R);
  if constexpr (q == 1) mma<0, 1>(R);
  if constexpr (q == 2) mma<1, 0>(R);
  if constexpr (q == 3) mma<1, 1>(R);
  __builtin_amdgcn_sched_barrier(0);
  // vmcnt(10) lgkmcnt(0) as one builtin so hipcc's waitcnt pass sees it
  __builtin_amdgcn_s_waitcnt(0x0070 | (10 & 15) | ((10 >> 4) << 14));
  g256::bar();
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm_nt_256pl(const unsigned short* __restrict__ A,
                                                     const unsigned short* __restrict__ B,
                                                     unsigned short* __restrict__ C,
                                                     const unsigned short* __restrict__ bias,
                                                     int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = GM * ntn;
  const int group = wg / per_group;
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  g256::Ctx c;
  c.smem = smem;
  c.Ag = A + (long)tm * BM * lda;
  c.Bg = B + (long)tn * BN * ldb;
  c.a_half = 128L * lda;
  c.b_half = 128L * ldb;
  c.w = w;
  c.wr = w >> 2;
  c.wc = w & 3;
  c.nt = K / BK;
  {
    const int r0 = w * 16 + (lane >> 3), r1 = r0 + 8;
    const int c0 = (lane & 7) ^ ((r0 >> 1) & 7);
    const int c1 = (lane & 7) ^ ((r1 >> 1) & 7);
    c.offA0 = r0 * lda + c0 * 8;
    c.offA1 = r1 * lda + c1 * 8;
    c.offB0 = r0 * ldb + c0 * 8;
    c.offB1 = r1 * ldb + c1 * 8;
    const int fr = lane & 15, fq = lane >> 4, f = fr >> 1;
    c.ro0 = fr * 128 + ((fq ^ f) * 16);
    c.ro1 = fr * 128 + (((4 + fq) ^ f) * 16);
  }
  Regs R;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int n = 0; n < 2; ++n) R.acc[a][i][b][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: half-tiles 0..7 = K-tiles 0 and 1 (B0 A0 B1 A1 each)
  const int k1 = (c.nt > 1 ? 1 : 0) * BK;
  g256::issue<P_B0>(c, 0, 0);
  g256::issue<P_A0>(c, 0, 0);
  g256::issue<P_B1>(c, 0, 0);
  g256::issue<P_A1>(c, 0, 0);
  g256::issue<P_B0>(c, 1, k1);
  g256::issue<P_A0>(c, 1, k1);
  g256::issue<P_B1>(c, 1, k1);
  g256::issue<P_A1>(c, 1, k1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // B0, A0 of K-tile 0
  g256::bar();
  read_a<0>(c, R, smem + P_A0 * HALF_BYTES);
  read_b<0>(c, R, smem + P_B0 * HALF_BYTES);
  __builtin_amdgcn_s_waitcnt(0x0070 | (10 & 15) | ((10 >> 4) << 14));  // B1 of K-tile 0; frags in
  g256::bar();

  const int iters = c.nt >> 1;
  for (int it = 0; it < iters; ++it) {
    phase<0>(c, R, it);
    phase<1>(c, R, it);
    phase<2>(c, R, it);
    phase<3>(c, R, it);
    phase<4>(c, R, it);
    phase<5>(c, R, it);
    phase<6>(c, R, it);
    phase<7>(c, R, it);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = tm * BM + mh * 128 + c.wr * 64 + i * 16 + fr;
      unsigned short* crow = C + (long)row * ldc;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int col = tn * BN + nh * 128 + c.wc * 32 + n * 16 + fq * 4;
          f32x4 v = R.acc[mh][i][nh][n];
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI != EPI_NONE) {
            bf16x4 bb = *(const bf16x4*)(bias + col);
#pragma unroll
            for (int e = 0; e < 4; ++e) bv[e] = bf2f((unsigned short)bb[e]);
          }
          uint2 o;
          o.x = pack_bf16x2(epilogue<EPI>(v[0], bv[0]), epilogue<EPI>(v[1], bv[1]));
          o.y = pack_bf16x2(epilogue<EPI>(v[2], bv[2]), epilogue<EPI>(v[3], bv[3]));
          *(uint2*)(crow + col) = o;
        }
    }
}

}  // namespace gpl

// ---------------------------------------------------------------------------
// gemm_nt_256p32: the ping-pong with 32-MFMA blocks (half the barriers of g256).
//
// Same block tile, wave layout, fragments and LDS image as g256, but a phase is
// a whole m-half x both n-halves (32 MFMAs per wave) and a K-tile takes two
// phases: X(t) = m-half 0 (reads A0, B0, B1), Y(t) = m-half 1 (reads A1).
// Barrier overhead per MFMA halves; the price is LDS: a 32-MFMA phase consumes
// 32 KiB, so the half-tile ring grows to 10 slots (160 KiB, the whole LDS) and
// only the trailing wave group (waves 4-7) issues the LDS-DMA -- a slot may
// then be refilled one phase after its last read instead of two.
// Half-tile h = 4t + pos (pos: A0, B0, B1, A1) lives in slot h % 10; phase P
// (X(t) = 2t, Y(t) = 2t+1) issues h = 2P+8 and 2P+9 (4 glds each per trailing
// wave) and waits vmcnt(16) (two phases of DMA in flight).
//   RAW: every half-tile is read >= 3 phases after its issue (vmcnt(16) in
//        phase p retires everything issued up to p-2);
//   WAR: h+10 is issued >= 1 phase after h's last read, by the trailing group,
//        whose issue point (after its barrier 2p) follows every read of phase
//        p-1 on both groups.
// ---------------------------------------------------------------------------
namespace g32 {

using g256::BM;
using g256::BN;
using g256::BK;
using g256::HALF_BYTES;
constexpr int SLOTS = 10;
constexpr int LDS_BYTES = SLOTS * HALF_BYTES;  // 160 KiB
constexpr int GM = 4;

struct Ctx {
  char* smem;
  const unsigned short* Ag;
  const unsigned short* Bg;
  long a_half, b_half;
  int offA[4], offB[4];  // trailing-wave glds source offsets (elements), 4 x 8 rows
  int ro0, ro1;
  int wr, wc, w, nt;
};

__device__ __forceinline__ const char* slot_ptr(const Ctx& c, int h) {
  return c.smem + (h % SLOTS) * HALF_BYTES;
}

// pos 0 A0, 1 B0, 2 B1, 3 A1 ; issued by waves 4-7 only (4 x glds of 8 rows each)
template <int POS>
__device__ __forceinline__ void issue_half(const Ctx& c, int h) {
  int t = h >> 2;
  t = t < c.nt ? t : c.nt - 1;  // past the end: reload the last tile into a dead slot
  const unsigned short* src;
  const int* off;
  if constexpr (POS == 0 || POS == 3) {
    src = c.Ag + (POS == 3 ? c.a_half : 0) + t * BK;
    off = c.offA;
  } else {
    src = c.Bg + (POS == 2 ? c.b_half : 0) + t * BK;
    off = c.offB;
  }
  char* dst = c.smem + (h % SLOTS) * HALF_BYTES + (c.w - 4) * 4096;
#pragma unroll
  for (int j = 0; j < 4; ++j) glds16(src + off[j], dst + j * 1024);
}

template <int Y>
__device__ __forceinline__ void phase(const Ctx& c, g256::Regs& R, int t) {
  const int h0 = 4 * t;
  if constexpr (Y == 0) {
    g256::read_a(c, R, slot_ptr(c, h0 + 0));
    g256::read_b<0>(c, R, slot_ptr(c, h0 + 1));
    g256::read_b<1>(c, R, slot_ptr(c, h0 + 2));
  } else {
    g256::read_a(c, R, slot_ptr(c, h0 + 3));
  }
  if (c.wr == 1) {
    if constexpr (Y == 0) {
      issue_half<0>(c, h0 + 8);
      issue_half<1>(c, h0 + 9);
    } else {
      issue_half<2>(c, h0 + 10);
      issue_half<3>(c, h0 + 11);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  g256::bar();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  g256::mma_quadrant<Y, 0>(R);
  g256::mma_quadrant<Y, 1>(R);
  g256::bar();
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm_nt_256p32(const unsigned short* __restrict__ A,
                                                      const unsigned short* __restrict__ B,
                                                      unsigned short* __restrict__ C,
                                                      const unsigned short* __restrict__ bias,
                                                      int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = GM * ntn;
  const int group = wg / per_group;
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  Ctx c;
  c.smem = smem;
  c.Ag = A + (long)tm * BM * lda;
  c.Bg = B + (long)tn * BN * ldb;
  c.a_half = 128L * lda;
  c.b_half = 128L * ldb;
  c.w = w;
  c.wr = w >> 2;
  c.wc = w & 3;
  c.nt = K / BK;
  {
    // trailing wave b = w-4 fills half-tile rows b*32 + j*8 + lane/8 (j = 0..3)
    const int b = (w & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = b * 32 + j * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      c.offA[j] = r * lda + ch * 8;
      c.offB[j] = r * ldb + ch * 8;
    }
    const int fr = lane & 15, fq = lane >> 4, f = fr >> 1;
    c.ro0 = fr * 128 + ((fq ^ f) * 16);
    c.ro1 = fr * 128 + (((4 + fq) ^ f) * 16);
  }
  g256::Regs R;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int n = 0; n < 2; ++n) R.acc[a][i][b][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (c.wr == 1) {
    // prologue: half-tiles 0..7 (K-tiles 0 and 1)
    issue_half<0>(c, 0);
    issue_half<1>(c, 1);
    issue_half<2>(c, 2);
    issue_half<3>(c, 3);
    issue_half<0>(c, 4);
    issue_half<1>(c, 5);
    issue_half<2>(c, 6);
    issue_half<3>(c, 7);
    asm volatile("s_waitcnt vmcnt(20)" ::: "memory");  // A0 B0 B1 of K-tile 0 landed
  }
  g256::bar();
  if (c.wr == 1) g256::bar();  // stagger: waves 4-7 trail by one barrier

  for (int t = 0; t < c.nt; ++t) {
    phase<0>(c, R, t);
    phase<1>(c, R, t);
  }
  if (c.wr == 0) g256::bar();  // balance the stagger barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = tm * BM + mh * 128 + c.wr * 64 + i * 16 + fr;
      unsigned short* crow = C + (long)row * ldc;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int col = tn * BN + nh * 128 + c.wc * 32 + n * 16 + fq * 4;
          f32x4 v = R.acc[mh][i][nh][n];
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI != EPI_NONE) {
            bf16x4 bb = *(const bf16x4*)(bias + col);
#pragma unroll
            for (int e = 0; e < 4; ++e) bv[e] = bf2f((unsigned short)bb[e]);
          }
          uint2 o;
          o.x = pack_bf16x2(epilogue<EPI>(v[0], bv[0]), epilogue<EPI>(v[1], bv[1]));
          o.y = pack_bf16x2(epilogue<EPI>(v[2], bv[2]), epilogue<EPI>(v[3], bv[3]));
          *(uint2*)(crow + col) = o;
        }
    }
}

}  // namespace g32

// ---------------------------------------------------------------------------
// gemm_nt_256w4: 256x256 tile, 4 waves (one per SIMD), each wave 128x128 of C
// (64 accumulators = 256 AGPRs), BK=32 stages in a 4-deep LDS-DMA ring.
//
// One barrier per 64-MFMA K-step. In step t a wave issues the glds for K-tile
// t+4 (into the stage K-tile t vacated: its fragments are already in
// registers), ds_reads K-tile t+1's fragments into the second register set and
// runs the 64 MFMAs of K-tile t, interleaved by sched_group_barrier so the LDS
// and DMA issue hides in the MFMA gaps. LDS traffic per K-tile is 2/3 of the
// 8-wave kernel's (each wave reads 128 rows of A and of B instead of 128 + 64).
// LDS image: 64-byte rows, 16-byte chunk c of row r at c ^ ((4 - (r>>2)) & 3):
// every ds_read_b128 16-lane group hits 16 distinct bank slots.
// ---------------------------------------------------------------------------
namespace g4 {

constexpr int BM = 256, BN = 256, BK = 32, STAGES = 4;
constexpr int ROWB = BK * 2;                  // 64-byte rows
constexpr int OPB = 256 * ROWB;               // one operand of one stage: 16 KiB
constexpr int STAGE_BYTES = 2 * OPB;          // A + B
constexpr int LDS_BYTES = STAGES * STAGE_BYTES;  // 128 KiB
constexpr int GROUP_M = 8;

__device__ __forceinline__ int swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

struct Frags {
  bf16x8 a[8];      // A fragments; a[i] is refilled with the next K-tile's row block i
  bf16x8 b[2][8];   // B fragments, double-buffered across K-tiles (static set index)
  f32x4 acc[8][8];  // 256 accumulator registers, pinned to AGPRs by the asm constraint
};

struct Ctx {
  char* smem;
  const unsigned short* Ag;
  const unsigned short* Bg;
  int ga[4], gb[4];  // per-lane glds source offsets (elements) for the 4 row blocks
  int ro;            // per-lane ds_read byte offset inside a 16-row block
  int wr, wc, w, nt;
};

__device__ __forceinline__ const char* a_base(const Ctx& c, int stage) {
  return c.smem + stage * STAGE_BYTES + c.wr * 128 * ROWB + c.ro;
}
__device__ __forceinline__ const char* b_base(const Ctx& c, int stage) {
  return c.smem + stage * STAGE_BYTES + OPB + c.wc * 128 * ROWB + c.ro;
}

// One MFMA whose accumulator lives in AGPRs. Issued as asm so the register
// allocator keeps each of the 64 accumulators in place across the K-loop (the
// builtin form makes hipcc rotate accumulators through v_accvgpr_{read,write}).
// Operands come from ds_read (not VALU), so no wait states are needed in front;
// the only hazard -- an MFMA result read by VALU -- is padded after the loop.
__device__ __forceinline__ void mfma16(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

__device__ __forceinline__ void issue_tile(const Ctx& c, int t, int stage) {
  t = t < c.nt ? t : c.nt - 1;
  const int k0 = t * BK;
  char* dA = c.smem + stage * STAGE_BYTES + c.w * 1024;
#pragma unroll
  for (int j = 0; j < 4; ++j) glds16(c.Ag + k0 + c.ga[j], dA + j * 4096);
#pragma unroll
  for (int j = 0; j < 4; ++j) glds16(c.Bg + k0 + c.gb[j], dA + OPB + j * 4096);
}

__device__ __forceinline__ void sync_step() {
  // s_waitcnt vmcnt(16) lgkmcnt(0): own glds of K-tile t+2 landed, own ds_reads
  // of K-tile t+1 done. The builtin (not asm) lets hipcc's waitcnt pass see it,
  // so it does not add a conservative lgkmcnt(0) in front of the next step's
  // first MFMA (which would also wait for that step's freshly issued reads).
  __builtin_amdgcn_s_waitcnt(0x4070);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// K-step t: 8 groups, one per A row block i: {glds of K-tile t+4 (A blocks
// 0-3, then B blocks 0-3) into the stage K-tile t vacated; ds_read next B[i];
// 8 MFMAs of row i; ds_read next A[i] into the registers row i just released}.
template <int SET>
__device__ __forceinline__ void step(const Ctx& c, Frags& f, int t) {
  const int nxt = (t + 1) & 3;
  const char* sa = a_base(c, nxt);
  const char* sb = b_base(c, nxt);
  int tl = t + 4;
  tl = tl < c.nt ? tl : c.nt - 1;  // past the end: re-load the last tile into a dead stage
  const int k0 = tl * BK;
  char* dA = c.smem + (t & 3) * STAGE_BYTES + c.w * 1024;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < 4)
      glds16(c.Ag + k0 + c.ga[i], dA + i * 4096);
    else
      glds16(c.Bg + k0 + c.gb[i - 4], dA + OPB + (i - 4) * 4096);
    f.b[SET ^ 1][i] = *(const bf16x8*)(sb + i * 16 * ROWB);
#pragma unroll
    for (int n = 0; n < 8; ++n) mfma16(f.acc[i][n], f.b[SET][n], f.a[i]);
    f.a[i] = *(const bf16x8*)(sa + i * 16 * ROWB);
    __builtin_amdgcn_sched_barrier(0);
  }
  sync_step();
}

template <int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_256w4(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = GROUP_M * ntn;
  const int group = wg / per_group;
  const int first_m = group * GROUP_M;
  const int gsz = min(ntm - first_m, GROUP_M);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  Ctx c;
  c.smem = smem;
  c.Ag = A + (long)tm * BM * lda;
  c.Bg = B + (long)tn * BN * ldb;
  c.w = w;
  c.wr = w >> 1;
  c.wc = w & 1;
  c.nt = K / BK;
  {
    // glds j of wave w fills stage rows j*64 + w*16 + lane/4, physical chunk lane&3
    const int rl = lane >> 2;
    const int ch = (lane & 3) ^ swz(rl);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = j * 64 + w * 16 + rl;
      c.ga[j] = row * lda + ch * 8;
      c.gb[j] = row * ldb + ch * 8;
    }
    const int fr = lane & 15, fq = lane >> 4;
    c.ro = fr * ROWB + ((fq ^ swz(fr)) * 16);
  }
  Frags f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 8; ++n) f.acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_tile(c, 0, 0);
  issue_tile(c, 1, 1);
  issue_tile(c, 2, 2);
  issue_tile(c, 3, 3);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // K-tile 0 landed
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  {
    const char* sa = a_base(c, 0);
    const char* sb = b_base(c, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f.a[i] = *(const bf16x8*)(sa + i * 16 * ROWB);
      f.b[0][i] = *(const bf16x8*)(sb + i * 16 * ROWB);
    }
  }
  sync_step();  // K-tile 1 visible, K-tile 0 fragments in registers

  for (int t = 0; t < c.nt; t += 2) {
    step<0>(c, f, t);
    step<1>(c, f, t + 1);
  }
  // MFMA results -> VALU reads in the epilogue: pad the hazard (asm MFMAs are
  // invisible to hipcc's hazard recognizer), drain the tail prefetches.
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(f.acc[i][n]));  // reads stay after the padding

  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = tm * BM + c.wr * 128 + i * 16 + fr;
    unsigned short* crow = C + (long)row * ldc;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int col = tn * BN + c.wc * 128 + n * 16 + fq * 4;
      f32x4 v = f.acc[i][n];
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI != EPI_NONE) {
        bf16x4 bb = *(const bf16x4*)(bias + col);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = bf2f((unsigned short)bb[e]);
      }
      uint2 o;
      o.x = pack_bf16x2(epilogue<EPI>(v[0], bv[0]), epilogue<EPI>(v[1], bv[1]));
      o.y = pack_bf16x2(epilogue<EPI>(v[2], bv[2]), epilogue<EPI>(v[3], bv[3]));
      *(uint2*)(crow + col) = o;
    }
  }
}

}  // namespace g4

// Measured alternatives (variants 3-14): kept so every number in
// profiles/gemm_tuning.md can be reproduced. Production never routes here.
template <int EPI>
static hipError_t launch_experiment(int variant, const unsigned short* A, const unsigned short* B,
                                    unsigned short* C, const unsigned short* bias, int M, int N, int K, int lda,
                                    int ldb, int ldc, hipStream_t s) {
  const dim3 grid256((M / g256::BM) * (N / g256::BN));
  if (variant >= 4 && variant <= 8) {
    // tuning experiments (no-epilogue only)
    if constexpr (EPI == EPI_NONE) {
      if (variant == 4)  // with s_setprio around the MFMA blocks
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 5>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 5)  // GROUP_M 8
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 3>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 6)  // first schedule (12/4/8/0 reads, look-ahead 5), setprio, GROUP_M 8
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 0>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 7)  // GROUP_M 2
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 15>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 8)  // GROUP_M 16
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 11>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (variant == 9 || variant == 11 || variant == 12 || variant == 13) {
    if constexpr (EPI == EPI_NONE) {
      if (variant == 9)  // timing probe: every MFMA block doubled (wrong C)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 16>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 11)  // timing probe: all blocks load the same (L2-resident) tiles (wrong C)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 32>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f, nullptr);
      if (variant == 12)  // lockstep: no ping-pong stagger
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 64>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K,
                           lda, ldb, ldc, 1.0f, nullptr);
      if (variant == 13)  // lockstep, one barrier per phase
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 64 + 128>), grid256, dim3(512), 0, s, A, B, C, bias, M, N,
                           K, lda, ldb, ldc, 1.0f, nullptr);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (variant == 21) {
    // VGPR staging (global_load + ds_write) instead of LDS-DMA, 4 phases in flight
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 131072>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                       ldb, ldc, 1.0f, nullptr);
  } else if (variant == 22) {
    // VGPR staging, 2 phases in flight
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 131072 + 262144>), grid256, dim3(512), 0, s, A, B, C, bias, M, N,
                       K, lda, ldb, ldc, 1.0f, nullptr);
  } else if (variant == 14) {
    hipLaunchKernelGGL(gpl::gemm_nt_256pl<EPI>, grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else if (variant == 10) {
    hipLaunchKernelGGL(g32::gemm_nt_256p32<EPI>, grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else if (variant == 3) {
    dim3 grid((M / g4::BM) * (N / g4::BN));
    hipLaunchKernelGGL(g4::gemm_nt_256w4<EPI>, grid, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else if (variant == 15) {
    // production schedule with the narrow (2 x 8-B per lane) store tail
    if constexpr (EPI != EPI_NONE) return hipErrorInvalidValue;
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 256>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                       ldb, ldc, 1.0f, nullptr);
  } else if (variant == 20) {
    // persistent: one block per CU walking the tiles (measured slightly slower)
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    const int nwg = (M / g256::BM) * (N / g256::BN);
    const dim3 gridp(nwg < cus ? nwg : cus);
    hipLaunchKernelGGL((g256::gemm_nt_256_persist<EPI, 7 + 32768>), gridp, dim3(512), 0, s, A, B, C, bias, M, N, K,
                       lda, ldb, ldc, 1.0f, nullptr);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kgs

// The same eligibility as the production fast path (M, N % 256, K % 128,
// 16-B aligned operands and rows).
static bool exp_fast_ok(const void* A, const void* B, const void* C, int M, int N, int K, int lda, int ldb,
                        int ldc) {
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return false;
  if (M % 256 || N % 256 || K % 128 || lda % 8 || ldb % 8 || ldc % 8) return false;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return false;
  return (long)lda * 256 < (1L << 31) && (long)ldb * 256 < (1L << 31);
}

// bf16 NT experiments: variants 3-15, 20-22. Returns 0 or a KGS_ERR_* / hipError_t.
KGS_EXPORT int kgs_exp_gemm_bf16_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                                    int lda, int ldb, int ldc, int epi, int variant, hipStream_t s) {
  if (!((variant >= 3 && variant <= 15) || (variant >= 20 && variant <= 22))) return KGS_ERR_ARG;
  if (epi != kgs::EPI_NONE && (bias == nullptr || (uintptr_t)bias % 8)) return KGS_ERR_ARG;
  if (!exp_fast_ok(A, B, C, M, N, K, lda, ldb, ldc)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  hipError_t e;
  switch (epi) {
    case kgs::EPI_NONE: e = kgs::launch_experiment<kgs::EPI_NONE>(variant, a, b, c, bb, M, N, K, lda, ldb, ldc, s); break;
    case kgs::EPI_BIAS: e = kgs::launch_experiment<kgs::EPI_BIAS>(variant, a, b, c, bb, M, N, K, lda, ldb, ldc, s); break;
    case kgs::EPI_BIAS_GELU:
      e = kgs::launch_experiment<kgs::EPI_BIAS_GELU>(variant, a, b, c, bb, M, N, K, lda, ldb, ldc, s);
      break;
    case kgs::EPI_BIAS_RELU:
      e = kgs::launch_experiment<kgs::EPI_BIAS_RELU>(variant, a, b, c, bb, M, N, K, lda, ldb, ldc, s);
      break;
    case kgs::EPI_BIAS_SILU:
      e = kgs::launch_experiment<kgs::EPI_BIAS_SILU>(variant, a, b, c, bb, M, N, K, lda, ldb, ldc, s);
      break;
    default: return KGS_ERR_ARG;
  }
  return (int)e;
}

// fp8 e4m3 tile-group height experiments (aligned shapes, no epilogue):
// 17 = GROUP_M 8, 18 = GROUP_M 16, 19 = GROUP_M 2; round 3: 20 / 21 / 22 = GROUP_N
// 4 / 8 / 2 (S bit 21). Lengths in fp8 elements.
KGS_EXPORT int kgs_exp_gemm_fp8_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                   int ldc, float alpha, int variant, hipStream_t s) {
  using namespace kgs;
  if (variant < 17 || variant > 22) return KGS_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (M % 256 || N % 256 || K % 256 || lda % 16 || ldb % 16 || ldc % 8) return KGS_ERR_ALIGN;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  const int Kw = K / 2, ldaw = lda / 2, ldbw = ldb / 2;
  const dim3 grid((M / g256::BM) * (N / g256::BN));
  if (variant == 17)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 3 + 1024>), grid, dim3(512), 0, s, a, b, c, nullptr, M, N, Kw,
                       ldaw, ldbw, ldc, alpha, nullptr);
  if (variant == 18)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 11 + 1024>), grid, dim3(512), 0, s, a, b, c, nullptr, M, N, Kw,
                       ldaw, ldbw, ldc, alpha, nullptr);
  if (variant == 19)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 15 + 1024>), grid, dim3(512), 0, s, a, b, c, nullptr, M, N, Kw,
                       ldaw, ldbw, ldc, alpha, nullptr);
  if (variant == 20)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 7 + 1024 + 2097152>), grid, dim3(512), 0, s, a, b, c, nullptr, M,
                       N, Kw, ldaw, ldbw, ldc, alpha, nullptr);
  if (variant == 21)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 3 + 1024 + 2097152>), grid, dim3(512), 0, s, a, b, c, nullptr, M,
                       N, Kw, ldaw, ldbw, ldc, alpha, nullptr);
  if (variant == 22)
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI_NONE, 15 + 1024 + 2097152>), grid, dim3(512), 0, s, a, b, c, nullptr, M,
                       N, Kw, ldaw, ldbw, ldc, alpha, nullptr);
  return (int)hipGetLastError();
}

// Diagnostic build: the production schedule with s_memtime stamps (S bit 16).
// stamps: 4 * STAMP_N u64 (blocks 0..3); layout in gemm_pipeline.h (stamp()).
KGS_EXPORT int kgs_gemm_bf16_nt_stamps(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                       int ldc, void* stamps, hipStream_t s) {
  if (M % 256 || N % 256 || K % 128 || (K / 128) < kgs::g256::STAMP_IT0 + kgs::g256::STAMP_ITS) return KGS_ERR_SHAPE;
  const dim3 grid((M / 256) * (N / 256));
  hipLaunchKernelGGL((kgs::g256::gemm_nt_256<kgs::EPI_NONE, 7 + 65536>), grid, dim3(512), 0, s,
                     (const unsigned short*)A, (const unsigned short*)B, (unsigned short*)C, nullptr, M, N, K, lda,
                     ldb, ldc, 1.0f, (const float*)stamps);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_gemm_stamp_n() { return kgs::g256::STAMP_N; }
