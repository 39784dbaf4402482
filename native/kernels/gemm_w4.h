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
// Register allocation: the accumulators MUST stay tied. With the builtin MFMA
// hipcc renames accumulators between the two unrolled K-steps and repairs the
// loop with ~700 v_accvgpr moves per iteration; the asm form with a "+a"
// operand keeps each accumulator in place (0 moves, checked in the ISA).
#pragma once

#include "kgs_common.h"

namespace kgs {
namespace w4 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int OPB = 256 * BK * 2;    // one operand of one stage: 32 KiB
constexpr int STAGE = 2 * OPB;       // A + B: 64 KiB
constexpr int LDS_BYTES = 2 * STAGE;  // 128 KiB
constexpr int GM = 4;                // tile-group height (production choice)

struct Ctx {
  char* smem;
  __amdgpu_buffer_rsrc_t ra, rb;
  int voa, vob;     // per-lane DMA byte offsets (row, swizzled chunk)
  int sa32, sb32;   // bytes between DMA row groups (32 rows)
  int w, wr, wc;
  int ro0, ro1;     // per-lane fragment byte offsets, k-sub 0 / 1
  int nt;
};

struct Frag {
  bf16x8 a[8];
  bf16x8 b[8];
};

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// DMA instruction j (0..7) of operand OP for K-tile starting at k0 into stage st:
// rows j*32 + w*8 + lane/8 of the tile, 1 KiB = 8 rows of 128 B.
// AUX: cache-policy bits of the load (0 = default; 16 = sc1)
template <int OP, int AUX = 0>
__device__ __forceinline__ void dma(const Ctx& c, int st, int j, int k0) {
  char* dst = c.smem + st * STAGE + OP * OPB + (j * 4 + c.w) * 1024;
  const int so = j * (OP ? c.sb32 : c.sa32) + k0 * 2;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(OP ? c.rb : c.ra, (KGS_LDS void*)dst, 16, OP ? c.vob : c.voa, so, 0, AUX);
}

__device__ __forceinline__ bf16x8 frag(const char* p) { return *(const bf16x8*)p; }

template <int SUB>
__device__ __forceinline__ const char* abase(const Ctx& c, int st) {
  return c.smem + st * STAGE + c.wr * 128 * 128 + (SUB ? c.ro1 : c.ro0);
}
template <int SUB>
__device__ __forceinline__ const char* bbase(const Ctx& c, int st) {
  return c.smem + st * STAGE + OPB + c.wc * 128 * 128 + (SUB ? c.ro1 : c.ro0);
}

// One MFMA on an accumulator pinned to AGPRs: the tied "+a" operand keeps each
// of the 64 accumulators in one place across the K-loop (the builtin form lets
// the register allocator rename accumulators and then repair the loop with
// hundreds of v_accvgpr moves per K-step). Operands swapped (B first) so a lane
// holds C[m = lane&15][n = 4*(lane>>4)+e]. asm MFMAs are invisible to the
// hazard recognizer: the only hazard left (AGPR results read by VALU) is padded
// before the epilogue.
__device__ __forceinline__ void mma(f32x4 (&acc)[8][8], const Frag& f, int i, int n) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][n]) : "v"(f.b[n]), "v"(f.a[i]));
}

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// One K-step as a single pinned sequence of 128 MFMAs (k < 64 on f0 = k-sub 0,
// k >= 64 on f1 = k-sub 1) with its other instructions placed after MFMA k:
//   k in [0, 16)          ds_read f1 fragment k (B frags first: MFMA k-sub order is i-major)
//   k == B1 - 1           lgkmcnt(0) + barrier 1 (stage ST free)
//   k in [B1, 128 - R)    the 16 LDS-DMA issues of K-tile t+2, evenly spread
//   k == 128 - R - 1      vmcnt(16) + barrier 2 (K-tile t+1 visible)
//   k in [128 - R, ...)   P ds_reads of f0 (K-tile t+1, k-sub 0) after each MFMA
// MFMA order inside a k-sub. ORD 0: i-major (a[i] over all n), reads b0..b7 then
// a0..a7. ORD 1: "growing square": reads alternate b0 a0 b1 a1 ..., and MFMA
// (i, n) runs as soon as both of its fragments have been read, so the first
// MFMA of a k-sub needs 2 reads instead of 9.
struct MOrder {
  unsigned char i[64], n[64];
};
constexpr MOrder make_order(int ord) {
  MOrder o{};
  int k = 0;
  if (ord == 0) {
    for (int i = 0; i < 8; ++i)
      for (int n = 0; n < 8; ++n) { o.i[k] = i; o.n[k] = n; ++k; }
  } else {
    for (int m = 0; m < 8; ++m) {
      for (int j = 0; j < m; ++j) { o.i[k] = j; o.n[k] = m; ++k; }  // after b[m]
      for (int j = 0; j <= m; ++j) { o.i[k] = m; o.n[k] = j; ++k; }  // after a[m]
    }
  }
  return o;
}
constexpr MOrder ORDERS[2] = {make_order(0), make_order(1)};

// read r of a k-sub: which fragment (0 = b, 1 = a) and its index
constexpr int rd_isa(int ord, int r) { return ord == 0 ? (r >= 8) : (r & 1); }
constexpr int rd_idx(int ord, int r) { return ord == 0 ? (r & 7) : (r >> 1); }

struct StepPtrs {
  const char *pa1, *pb1, *pa0, *pb0;
  int k0;
};

// MFMA k of the K-step and what follows it, all decided at compile time.
template <int ST, int B1, int R, int P, int ORD, int X, int K>
__device__ __forceinline__ void kbody(const Ctx& c, const StepPtrs& sp, Frag& f0, Frag& f1, f32x4 (&acc)[8][8]) {
  if constexpr (K < 128) {
    constexpr int mi = ORDERS[ORD].i[K & 63], mn = ORDERS[ORD].n[K & 63];
    if constexpr (K < 64) mma(acc, f0, mi, mn); else mma(acc, f1, mi, mn);
    if constexpr (K < 16) {
      constexpr int x = rd_idx(ORD, K);
      if constexpr (rd_isa(ORD, K)) f1.a[x] = frag(sp.pa1 + x * 2048); else f1.b[x] = frag(sp.pb1 + x * 2048);
    }
    if constexpr (K >= B1 && K < 128 - R) {
      // MFMAs that carry the DMA issues: the whole window, or the first W (X / 10000) of it
      constexpr int ND = (X / 10000) ? X / 10000 : 128 - R - B1;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (B1 + (j * ND) / 16 == K) {
          if (j < 8) dma<0, (X / 100) % 100>(c, ST, j, sp.k0); else dma<1, (X / 100) % 100>(c, ST, j - 8, sp.k0);
        }
      }
    }
    if constexpr (K >= 128 - R) {
      constexpr int q = K - (128 - R);
#pragma unroll
      for (int e = q * P; e < (q + 1) * P && e < 16; ++e) {
        const int x = rd_idx(ORD, e);
        if (rd_isa(ORD, e)) f0.a[x] = frag(sp.pa0 + x * 2048); else f0.b[x] = frag(sp.pb0 + x * 2048);
      }
    }
    fence();
    if constexpr (K == B1 - 1) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage ST retired
      bar();
    }
    if constexpr (K == 128 - R - 1) {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // own DMA of K-tile t+1 landed
      bar();
    }
    kbody<ST, B1, R, P, ORD, X, K + 1>(c, sp, f0, f1, acc);
  }
}

// One K-step as a single pinned sequence of 128 MFMAs (k < 64 on f0 = k-sub 0,
// k >= 64 on f1 = k-sub 1) with its other instructions placed after MFMA k:
//   k in [0, 16)          ds_read f1 fragment k (B frags first: MFMA k-sub order is i-major)
//   k == B1 - 1           lgkmcnt(0) + barrier 1 (stage ST free)
//   k in [B1, 128 - R)    the 16 LDS-DMA issues of K-tile t+2, evenly spread
//   k == 128 - R - 1      vmcnt(16) + barrier 2 (K-tile t+1 visible)
//   k in [128 - R, ...)   P ds_reads of f0 (K-tile t+1, k-sub 0) after each MFMA
template <int ST, int B1, int R, int P, int ORD, int X>
__device__ __forceinline__ void kstep(const Ctx& c, Frag& f0, Frag& f1, f32x4 (&acc)[8][8], int t) {
  static_assert(B1 >= 16 && B1 + 16 <= 128 - R && 16 <= R * P, "bad K-step schedule");
  StepPtrs sp;
  sp.pa1 = abase<1>(c, ST);
  sp.pb1 = bbase<1>(c, ST);
  sp.pa0 = abase<0>(c, ST ^ 1);
  sp.pb0 = bbase<0>(c, ST ^ 1);
  int tl = t + 2;
  tl = tl < c.nt ? tl : c.nt - 1;  // past the end: harmless re-load into the free stage
  sp.k0 = tl * BK;
  kbody<ST, B1, R, P, ORD, X, 0>(c, sp, f0, f1, acc);
}

// Production knobs: barrier 1 after MFMA 24, 20 MFMAs after barrier 2, one
// read per MFMA there, growing-square order, GROUP_M 4, default cache policy.
constexpr int PB1 = 24, PR = 20, PP = 1, PORD = 1, PX = 0;

template <int EPI, int B1 = PB1, int R = PR, int P = PP, int ORD = PORD, int X = PX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int G = (X % 100) ? X % 100 : GM;
  const int per_group = G * ntn;
  const int group = wg / per_group;
  const int first_m = group * G;
  const int gsz = min(ntm - first_m, G);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  Ctx c;
  c.smem = smem;
  c.w = w;
  c.wr = w >> 1;
  c.wc = w & 1;
  c.nt = K / BK;
  c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * BM * lda), 0, BM * lda * 2, 0x00020000);
  c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * BN * ldb), 0, BN * ldb * 2, 0x00020000);
  c.sa32 = 32 * lda * 2;
  c.sb32 = 32 * ldb * 2;
  {
    const int row = w * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    c.voa = (row * lda + ch * 8) * 2;
    c.vob = (row * ldb + ch * 8) * 2;
    const int fr = lane & 15, fq = lane >> 4, f = fr >> 1;
    c.ro0 = fr * 128 + ((fq ^ f) * 16);
    c.ro1 = fr * 128 + (((4 + fq) ^ f) * 16);
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tiles 0 and 1 into stages 0 and 1, k-sub 0 of K-tile 0 into f0
#pragma unroll
  for (int j = 0; j < 8; ++j) dma<0, (X / 100) % 100>(c, 0, j, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma<1, (X / 100) % 100>(c, 0, j, 0);
  const int k1 = (c.nt > 1 ? 1 : 0) * BK;
#pragma unroll
  for (int j = 0; j < 8; ++j) dma<0, (X / 100) % 100>(c, 1, j, k1);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma<1, (X / 100) % 100>(c, 1, j, k1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  bar();
  Frag f0, f1;
  {
    const char* pa = abase<0>(c, 0);
    const char* pb = bbase<0>(c, 0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {  // same order as the loop's reads
      const int x = rd_idx(ORD, e);
      if (rd_isa(ORD, e)) f0.a[x] = frag(pa + x * 2048); else f0.b[x] = frag(pb + x * 2048);
    }
  }
  // nothing outstanding on lgkm at loop entry: otherwise the waitcnt pass merges
  // the preheader's scalar loads into the loop header and waits lgkmcnt(0) there
  __builtin_amdgcn_s_waitcnt(0xc07f);

  for (int t = 0; t < c.nt; t += 2) {
    kstep<0, B1, R, P, ORD, X>(c, f0, f1, acc, t);
    kstep<1, B1, R, P, ORD, X>(c, f0, f1, acc, t + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail re-loads before LDS is released
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA -> v_accvgpr_read hazard

  // epilogue: bias + activation, then pair n-tiles (n, n+1) with
  // v_permlane16_swap -> one 16-B store per lane (guide T21)
  const int fr = lane & 15, fq = lane >> 4;
  float bv[8][4];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[n][e] = 0.f;
    if constexpr (EPI != EPI_NONE) {
      const bf16x4 bb = *(const bf16x4*)(bias + tn * BN + c.wc * 128 + n * 16 + fq * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[n][e] = bf2f((unsigned short)bb[e]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = tm * BM + c.wr * 128 + i * 16 + fr;
    unsigned short* crow = C + (long)row * ldc;
#pragma unroll
    for (int n = 0; n < 8; n += 2) {
      uint2 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 v = acc[i][n + h];
        o[h].x = pack_bf16x2(epilogue<EPI>(v[0], bv[n + h][0]), epilogue<EPI>(v[1], bv[n + h][1]));
        o[h].y = pack_bf16x2(epilogue<EPI>(v[2], bv[n + h][2]), epilogue<EPI>(v[3], bv[n + h][3]));
      }
      auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
      auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
      const uint4 qv = make_uint4(sx[0], sy[0], sx[1], sy[1]);
      const int col0 = tn * BN + c.wc * 128 + n * 16;
      *(uint4*)(crow + col0 + (fq & 1) * 16 + (fq >> 1) * 8) = qv;
    }
  }
}

}  // namespace w4
}  // namespace kgs
