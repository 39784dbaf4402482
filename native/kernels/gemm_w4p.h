// gemm_w4p: the four-wave 256x256x64 bf16 NT GEMM of gemm_w4.h made PERSISTENT.
//
// One workgroup per CU takes tiles from a per-XCD ticket queue (below) in the
// production tile order (tile_of, so every tile lands on the XCD it had in the
// one-shot grid, and the tiles in flight at any moment are the same set). The
// LDS-DMA stream does not stop at a tile boundary: the last two K-steps of a
// tile load K-tiles 0 and 1 of the NEXT tile into the stages they free, and the
// last R MFMAs read the next tile's first fragments, exactly as they read K-tile
// t + 1 inside a tile. Between two tiles a wave only runs its epilogue (256
// v_accvgpr_read, bf16 packing, 32 16-byte stores) while the next tile's first
// two K-tiles are already on their way. The one-shot grid instead drains,
// exits, dispatches a new workgroup, recomputes addresses and waits for two
// K-tiles from memory before its first MFMA, at every tile.
//
// Why a separate kernel: with the accumulators as C++ values ("+a" operands),
// an outer tile loop makes the register allocator move them (round 2: 124-132
// v_accvgpr_mov inside the MFMA loop and wrong results, profiles/gemm_tuning.md
// "Persistent four-wave kernel"). Here the accumulator tile is NAMED: q = 8 i + n
// lives in a[4q : 4q+3] (acc_regs.h), reserved by KGS_ACC_RESERVE and touched
// only by asm, so the allocator has nothing to rename. The first k-sub of a
// tile's first K-step writes with C = 0 (mfma0), which is the reset.
//
// Tiles are handed out dynamically, not as v, v + G, v + 2G: a workgroup that
// starts late (its CU held by another kernel, e.g. an RCCL all-reduce launched
// on a side stream just before the GEMM) must not keep its share of tiles
// waiting, or the whole GEMM waits for it. Workgroup b serves XCD label
// x = b & 7 (the dispatcher deals workgroups to XCDs round robin), whose tiles
// are the one-shot ids v = x + 8 t, t = 0, 1, .... Its first ticket is its rank
// among the workgroups of label x; every later one is that count plus
// atomicAdd(q[x]) (struct Tick: issued after barrier 2 of the tile's first
// K-step, stored to LDS after barrier 2 of the second, read by every wave
// before the last two K-steps, which load the next tile). The last
// workgroup to leave (exit counter q[8]) zeroes q[0..8] for the next launch on
// the stream (tile_queue.h: every stream, and every launch captured into a
// hipGraph, owns its slot; no two concurrent launches share one).
//
// K-step schedule, LDS image, DMA placement, barriers and MFMA order are
// gemm_w4.h's (Knobs<256, 256>: B1 24, R 20, P 1, growing-square order), so the
// result is bitwise the one-shot kernel's (tests/test_kernels_gpu.py).
#pragma once

#include "acc_regs.h"
#include "gemm_w4.h"

namespace kgs {
namespace w4p {

using w4::BK;
using w4::Ctx;
using w4::Frag;
using w4::StepPtrs;

constexpr int BM = 256, BN = 256;
using S = w4::Shape<BM, BN>;
using Kn = w4::Knobs<BM, BN>;
constexpr int MA = S::MA, NB = S::NB;

// LDS image layouts (template parameter L of the kernel).
//   L 0: gemm_w4.h's. A DMA instruction brings 8 consecutive 128-B rows; the
//        16-B chunk c of row r lands at c ^ ((r >> 1) & 7), which is done by
//        permuting the SOURCE address of the lanes of a row.
//   L 1 (round 4 experiment): every row is read by 8 consecutive lanes in
//        address order (no permutation inside a row). The rows are placed so
//        the fragment reads stay conflict-free. A 32-row group is 4 DMA
//        instructions k = 0..3, 1056 B apart (so instruction k starts at bank
//        unit 2k), and the group is padded to 4352 B (17 x 256). Instruction
//        k holds 4 rows of each 16-row fragment f in slots 4f + p:
//          k0: 0 1 4 5   k1: 2 3 6 7   k2: 12 13 8 9   k3: 14 15 10 11
//        In ds_read_b128 lane group {0-3, 12-15, 20-27}, rows {0-3, 12-15}
//        read chunk q at 16-B units 2k + 8 (p & 1) + q (the 8 even units + q),
//        and rows 4-11 read chunk q + 1 at the 8 odd units + q. The other
//        three lane groups have the same structure, shifted.
template <int L>
struct Lay;
template <>
struct Lay<0> {
  static constexpr int GROUP = 4096;  // bytes per 32-row group
  static constexpr int OPA = S::OPA, STAGE = S::STAGE;
  __device__ static constexpr int frag_off(int x) { return x * 2048; }
  __device__ static int dma_dst(int j, int w) { return (j * 4 + w) * 1024; }
  // row of the 32-row group and 16-B chunk that lane `lane` of wave `w` DMAs
  __device__ static void dma_lane(int lane, int w, int& row, int& ch) {
    row = w * 8 + (lane >> 3);
    ch = (lane & 7) ^ ((row >> 1) & 7);
  }
  __device__ static int read_lane(int fr, int chunk) { return fr * 128 + ((chunk ^ (fr >> 1)) * 16); }
};
template <>
struct Lay<1> {
  static constexpr int GROUP = 4352, KSTRIDE = 1056;
  static constexpr int OPA = (BM / 32) * GROUP, STAGE = OPA + (BN / 32) * GROUP;
  __device__ static constexpr int frag_off(int x) { return (x >> 1) * GROUP + (x & 1) * 512; }
  __device__ static int dma_dst(int j, int w) { return j * GROUP + w * KSTRIDE; }
  __device__ static void dma_lane(int lane, int w, int& row, int& ch) {
    // slot s = lane / 8 = 4 f + p; table row (k = w, p)
    const int p = (lane >> 3) & 3, f = lane >> 5;
    const int s1 = (w & 1) * 2 + (w >> 1) * 12;  // first S1 row of instruction k: 0 2 12 14
    const int s2 = 4 + (w & 1) * 2 + (w >> 1) * 4;  // first S2 row: 4 6 8 10
    row = 16 * f + ((p < 2) ? s1 + p : s2 + p - 2);
    ch = lane & 7;
  }
  __device__ static int read_lane(int fr, int chunk) {
    const int k = ((fr >> 1) & 1) + 2 * (fr >> 3);
    const int p = (fr & 1) + 2 * (((fr >> 2) ^ (fr >> 3)) & 1);
    return k * KSTRIDE + p * 128 + chunk * 16;
  }
};

// L / 10 (experiments): the MFMA order inside a k-sub, L / 10 - 1 (gemm_w4.h
// make_order: 0 i-major, 1 growing square, 2 n-major); 0 = Knobs (growing square).
constexpr int ord_of(int L) { return (L / 10) % 10 ? (L / 10) % 10 - 1 : Kn::ORD; }
// (L / 10^7) % 10 (experiments): the K-step schedule, barrier 1 after MFMA B1 and R MFMAs after
// barrier 2 (the DMA window is [B1, KM - R)); 0 = Knobs (B1 24, R 20). 1: 20 / 20, 2: 24 / 16,
// 3: 20 / 16, 4: 18 / 16 (a wider DMA window; the f1 reads end at MFMA NR = 16); 5: 20 / 24,
// 6: 18 / 24, 7: 24 / 24 (a longer read tail for the next K-step's first fragments).
constexpr int b1_of(int L) {
  constexpr int b1[8] = {Kn::B1, 20, 24, 20, 18, 20, 18, 24};
  return b1[(L / 10000000) % 10 & 7];
}
constexpr int r_of(int L) {
  constexpr int r[8] = {Kn::R, 20, 16, 16, 16, 24, 24, 24};
  return r[(L / 10000000) % 10 & 7];
}

template <int L>
__device__ __forceinline__ const char* pabase(const Ctx& c, int st, int sub) {
  return c.smem + st * Lay<L % 10>::STAGE + c.wr * 4 * Lay<L % 10>::GROUP + (sub ? c.ro1 : c.ro0);
}
template <int L>
__device__ __forceinline__ const char* pbbase(const Ctx& c, int st, int sub) {
  return c.smem + st * Lay<L % 10>::STAGE + Lay<L % 10>::OPA + c.wc * 4 * Lay<L % 10>::GROUP + (sub ? c.ro1 : c.ro0);
}

// DMA instruction j (A: j < 8, then B) of the K-tile at k0 into stage st, in
// layout L, with gemm_w4.h's operand order (X / 10^8) and cache bits (X / 100).
template <int L, int X>
__device__ __forceinline__ void pdma(const Ctx& c, int st, int j, int k0) {
  if constexpr (L % 10 == 0) {
    w4::dma_any<BM, BN, X>(c, st, j, k0);
  } else {
    constexpr int AUXX = (X / 100) % 100;
    constexpr int AUXB = AUXX >= 50 ? AUXX - 50 : AUXX, AUXA = AUXX >= 50 ? 0 : AUXX;
    constexpr int ORDB = (X / 100000000) % 10;
    static_assert(ORDB != 2, "layout 1: A-then-B or B-then-A DMA order only");
    constexpr int JA = BM / 32;
    const bool isb = ORDB == 1 ? j < JA : j >= JA;
    const int jj = ORDB == 1 ? (isb ? j : j - JA) : (isb ? j - JA : j);
    char* dst = c.smem + st * Lay<L % 10>::STAGE + (isb ? Lay<L % 10>::OPA : 0) + Lay<L % 10>::dma_dst(jj, c.w);
    const int so = jj * (isb ? c.sb32 : c.sa32) + k0 * 2;
    if (isb)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rb, (KGS_LDS void*)dst, 16, c.vob, so, 0, AUXB);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(c.ra, (KGS_LDS void*)dst, 16, c.voa, so, 0, AUXA);
  }
}

template <bool ZERO, int I, int N>
__device__ __forceinline__ void pmma(const Frag<MA, NB>& f) {
  if constexpr (ZERO) accr::mfma0<I * NB + N>(f.b[N], f.a[I]);
  else accr::mfma<I * NB + N>(f.b[N], f.a[I]);
}

// The next tile's ticket (DYN): wave 0 lane 0 issues the atomic right after
// barrier 2 of a tile's K-step 0 -- after that K-step's DMAs, so the vmcnt wait
// that barrier needs does not include it -- and stores the ticket to LDS right
// after barrier 2 of K-step 1, whose vmcnt wait did include it (no stall if it
// took less than a K-step). All waves read the slot before the tile's last two
// K-steps, at least one barrier later (K >= 384).
struct Tick {
  int* qx;    // this label's counter (through a non-uniform address, see the kernel)
  int* slot;  // LDS
  int tk;
};
// The wait-stamp build's ticket ((L / 10^6) % 10 == 1, experiments): plus the s_memtime cycles this
// wave spent in [category][lgkm wait, barrier 1, vm wait, barrier 2]; category 0 = a tile's K-steps
// 0-1, 1 = the steady loop, 2 = the last two (the next tile's DMAs).
struct TickW : Tick {
  unsigned long long ws[12];
};
template <bool W>
__device__ __forceinline__ auto make_tick(int* qx, int* slot) {
  if constexpr (W) return TickW{{qx, slot, 0}, {}};
  else return Tick{qx, slot, 0};
}

// gemm_w4.h's kbody with named accumulators: MFMA K of the K-step plus what
// follows it. The DMA issues use `cd` (this tile's or the next tile's buffer
// resources) and K-tile sp.k0 / BK; everything LDS-side uses `c`. TK: 1 =
// issue the ticket atomic after barrier 2, 2 = publish the ticket there.
template <int ST, int X, bool ZERO, int TK, int K, int L = 0, int WX = 0, int CAT = 1, class TQ = Tick>
__device__ __forceinline__ void pbody(const Ctx& c, const Ctx& cd, const StepPtrs& sp, Frag<MA, NB>& f0,
                                      Frag<MA, NB>& f1, TQ& tq) {
  constexpr int B1 = b1_of(L), R = r_of(L), P = Kn::P, ORD = ord_of(L);
  constexpr int KM = S::KM, HM = S::HM, NR = S::NR, ND = w4::dma_per_stage<BM, BN>();
  static_assert(B1 >= NR && B1 + ND <= KM - R && NR <= R * P, "bad K-step schedule");
  if constexpr (K < KM) {
    constexpr int mi = w4::Order<ORD, MA, NB>::o.i[K % HM], mn = w4::Order<ORD, MA, NB>::o.n[K % HM];
    if constexpr (K < HM) pmma<ZERO, mi, mn>(f0); else pmma<false, mi, mn>(f1);
    if constexpr (K < NR) {
      constexpr int x = w4::rd_idx(ORD, MA, NB, K);
      if constexpr (w4::rd_isa(ORD, MA, NB, K)) f1.a[x] = w4::frag(sp.pa1 + Lay<L % 10>::frag_off(x));
      else f1.b[x] = w4::frag(sp.pb1 + Lay<L % 10>::frag_off(x));
    }
    if constexpr (K >= B1 && K < KM - R) {
      // DMA window: the MFMAs [B1, KM - R), or the first W of them ((L / 10^4) % 100, experiments)
      constexpr int NW = (L / 10000) % 100 ? (L / 10000) % 100 : KM - R - B1;
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        if (B1 + (j * NW) / ND == K) pdma<L, X>(cd, ST, j, sp.k0);
      }
    }
    if constexpr (K >= KM - R) {
      constexpr int q = K - (KM - R);
#pragma unroll
      for (int e = q * P; e < (q + 1) * P && e < NR; ++e) {
        const int x = w4::rd_idx(ORD, MA, NB, e);
        if (w4::rd_isa(ORD, MA, NB, e)) f0.a[x] = w4::frag(sp.pa0 + Lay<L % 10>::frag_off(x));
        else f0.b[x] = w4::frag(sp.pb0 + Lay<L % 10>::frag_off(x));
      }
    }
    w4::fence();
    // OB ((L / 1000) % 10 == 1, experiments): ONE barrier per K-step. At MFMA B1 - 1 the wave waits for
    // its own DMAs of K-tile t + 1 (issued by the previous K-step; nothing younger but WX stores) and
    // for its reads of stage ST, then a barrier: stage ST is free for this step's DMAs AND K-tile t + 1
    // is visible for the f0 reads of the last R MFMAs, so the barrier at KM - R - 1 goes.
    constexpr bool OB = (L / 1000) % 10 == 1;
    // WSB ((L / 10^6) % 10 == 1, experiments): s_memtime around each wait and barrier (Tick::ws). A
    // stamp's result is used right after the barrier it follows, before any LDS read is issued, so
    // the lgkmcnt wait it needs costs only its own latency.
    constexpr bool WSB = (L / 1000000) % 10 == 1;
    if constexpr (K == B1 - 1) {
      unsigned long long t0 = 0, t1 = 0;
      if constexpr (WSB) t0 = __builtin_amdgcn_s_memtime();
      if constexpr (OB) w4::wait_vm<WX>();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage ST retired
      if constexpr (WSB) t1 = __builtin_amdgcn_s_memtime();
      w4::bar();
      if constexpr (WSB) {
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        tq.ws[CAT * 4 + 0] += t1 - t0;
        tq.ws[CAT * 4 + 1] += t2 - t1;
      }
      if constexpr (OB && TK == 1) {
        if (threadIdx.x == 0) tq.tk = atomicAdd(tq.qx, 1);
      } else if constexpr (OB && TK == 2) {
        if (threadIdx.x == 0) *tq.slot = tq.tk;
      }
    }
    if constexpr (K == KM - R - 1 && !OB) {
      unsigned long long t3 = 0, t4 = 0;
      if constexpr (WSB) t3 = __builtin_amdgcn_s_memtime();
      w4::wait_vm<ND + WX>();  // own DMA of the next K-tile landed (WX: younger stores, see the kernel)
      if constexpr (WSB) t4 = __builtin_amdgcn_s_memtime();
      w4::bar();
      if constexpr (WSB) {
        const unsigned long long t5 = __builtin_amdgcn_s_memtime();
        tq.ws[CAT * 4 + 2] += t4 - t3;
        tq.ws[CAT * 4 + 3] += t5 - t4;
      }
      if constexpr (TK == 1) {
        if (threadIdx.x == 0) tq.tk = atomicAdd(tq.qx, 1);
      } else if constexpr (TK == 2) {
        if (threadIdx.x == 0) *tq.slot = tq.tk;
      }
    }
    pbody<ST, X, ZERO, TK, K + 1, L, WX, CAT, TQ>(c, cd, sp, f0, f1, tq);
  }
}

// One K-step on stage ST; its DMAs bring K-tile kd (of cd's tile) into ST.
template <int ST, int X, bool ZERO, int TK = 0, int L = 0, int WX = 0, int CAT = 1, class TQ = Tick>
__device__ __forceinline__ void pstep(const Ctx& c, const Ctx& cd, Frag<MA, NB>& f0, Frag<MA, NB>& f1, int kd,
                                      TQ& tq) {
  StepPtrs sp;
  sp.pa1 = pabase<L>(c, ST, 1);
  sp.pb1 = pbbase<L>(c, ST, 1);
  sp.pa0 = pabase<L>(c, ST ^ 1, 0);
  sp.pb0 = pbbase<L>(c, ST ^ 1, 0);
  sp.k0 = kd * BK;
  pbody<ST, X, ZERO, TK, 0, L, WX, CAT, TQ>(c, cd, sp, f0, f1, tq);
}

// Epilogue of one tile, pairs of accumulators (q, q + 1) = (i, n), (i, n + 1):
// bias + activation, pack to bf16, pair n-tiles with v_permlane16_swap -> one
// 16-B store per lane (the one-shot kernel's epilogue, reading named AGPRs).
template <int EPI, int Q, bool NTST = false, int CST = 0>
__device__ __forceinline__ void pepi(const Ctx& c, unsigned short* __restrict__ C, int ldc, int tm, int tn,
                                     const float (&bv)[NB][4]) {
  if constexpr (Q < MA * NB) {
    constexpr int i = Q / NB, n = Q % NB;
    const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
    const f32x4 v0 = accr::read<Q>(), v1 = accr::read<Q + 1>();
    uint2 o[2];
    o[0].x = pack_bf16x2(epilogue<EPI>(v0[0], bv[n][0]), epilogue<EPI>(v0[1], bv[n][1]));
    o[0].y = pack_bf16x2(epilogue<EPI>(v0[2], bv[n][2]), epilogue<EPI>(v0[3], bv[n][3]));
    o[1].x = pack_bf16x2(epilogue<EPI>(v1[0], bv[n + 1][0]), epilogue<EPI>(v1[1], bv[n + 1][1]));
    o[1].y = pack_bf16x2(epilogue<EPI>(v1[2], bv[n + 1][2]), epilogue<EPI>(v1[3], bv[n + 1][3]));
    auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
    auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
    const uint4 qv = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    const int row = tm * BM + c.wr * (BM / 2) + i * 16 + fr;
    const int col0 = tn * BN + c.wc * (BN / 2) + n * 16;
    uint4* dst = (uint4*)(C + (long)row * ldc + col0 + (fq & 1) * 16 + (fq >> 1) * 8);
    if constexpr (NTST) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = {qv.x, qv.y, qv.z, qv.w};
      __builtin_nontemporal_store(v, (u32x4*)dst);
    } else if constexpr (CST == 1) {
      if (ldc < 0) *dst = qv;  // measurement build: C is never written (ldc > 0), the packing stays
    } else {
      *dst = qv;
    }
    pepi<EPI, Q + 2, NTST, CST>(c, C, ldc, tm, tn, bv);
  }
}

// Deferred C stores (kernel template DD > 0, round 6). At a tile change every
// workgroup stores its 128 KiB of C at once: 32 MiB chip-wide, about 5.7 us of
// HBM write time, and the next tile's first K-step waits for all of it (vmcnt
// counts loads and stores in issue order, so a wait for a DMA issued after the
// stores is a wait for the stores: 3.4 % of the 8192^3 bench step,
// profiles/r5/gemm/store_drain/README.md). With DD > 0 the epilogue stores only
// the first UI = 32 - DD * SPS 16-byte units per lane; the last DD * SPS are
// packed into VGPRs (d[]) and stored SPS at a time at the end of the next
// tile's K-steps 0 .. DD - 1, where they drain behind MFMA work. The K-step
// after a storing one waits vmcnt(ND + SPS): the stores issued after the DMA it
// waits for are younger, so they may still be in flight. On the first tile the
// "deferred stores" go to a zero-size buffer (dropped by the range check, still
// counted), so every K-step's wait count is a constant. The last tile's
// deferred units are stored after the loop.
template <int EPI, int Q>
__device__ __forceinline__ uint4 punit(const float (&bv)[NB][4]) {
  constexpr int n = Q % NB;
  const f32x4 v0 = accr::read<Q>(), v1 = accr::read<Q + 1>();
  uint2 o[2];
  o[0].x = pack_bf16x2(epilogue<EPI>(v0[0], bv[n][0]), epilogue<EPI>(v0[1], bv[n][1]));
  o[0].y = pack_bf16x2(epilogue<EPI>(v0[2], bv[n][2]), epilogue<EPI>(v0[3], bv[n][3]));
  o[1].x = pack_bf16x2(epilogue<EPI>(v1[0], bv[n + 1][0]), epilogue<EPI>(v1[1], bv[n + 1][1]));
  o[1].y = pack_bf16x2(epilogue<EPI>(v1[2], bv[n + 1][2]), epilogue<EPI>(v1[3], bv[n + 1][3]));
  auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
  auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
  return make_uint4(sx[0], sy[0], sx[1], sy[1]);
}

typedef unsigned int w4p_u32x4 __attribute__((ext_vector_type(4)));

// Epilogue with the last DEF units deferred into d[] (units Q / 2 >= UI).
template <int EPI, int Q, int UI, int DEF, bool NTST>
__device__ __forceinline__ void pepi_d(const Ctx& c, unsigned short* __restrict__ C, int ldc, int tm, int tn,
                                       const float (&bv)[NB][4], uint4 (&d)[DEF]) {
  if constexpr (Q < MA * NB) {
    constexpr int i = Q / NB, n = Q % NB;
    const uint4 qv = punit<EPI, Q>(bv);
    if constexpr (Q / 2 < UI) {
      const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
      const int row = tm * BM + c.wr * (BM / 2) + i * 16 + fr;
      const int col0 = tn * BN + c.wc * (BN / 2) + n * 16;
      uint4* dst = (uint4*)(C + (long)row * ldc + col0 + (fq & 1) * 16 + (fq >> 1) * 8);
      if constexpr (NTST) {
        const w4p_u32x4 v = {qv.x, qv.y, qv.z, qv.w};
        __builtin_nontemporal_store(v, (w4p_u32x4*)dst);
      } else {
        *dst = qv;
      }
    } else {
      d[Q / 2 - UI] = qv;
    }
    pepi_d<EPI, Q + 2, UI, DEF, NTST>(c, C, ldc, tm, tn, bv, d);
  }
}

// Deferred units [U0, U0 + CNT) of the tile whose C block `rc` covers (rows at
// stride ldc from the tile's corner); voff: this lane's byte offset in the block.
template <int UI, int U0, int CNT, int DEF, bool NTST>
__device__ __forceinline__ void dstore(const uint4 (&d)[DEF], __amdgpu_buffer_rsrc_t rc, int voff, int ldc) {
  w4::static_for<0, CNT>([&](auto e) {
    constexpr int u = U0 + decltype(e)::value, Q = 2 * (UI + u), i = Q / NB, n = Q % NB;
    const w4p_u32x4 v = {d[u].x, d[u].y, d[u].z, d[u].w};
    // column offset in the instruction's immediate, row group in soffset
    __builtin_amdgcn_raw_buffer_store_b128(v, rc, voff + n * 32, i * 32 * ldc, NTST ? 2 : 0);
  });
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_c(unsigned short* C, int tm, int tn, int ldc) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(C + (long)tm * BM * ldc + tn * BN), 0, BM * ldc * 2, 0x00020000);
}

// Residual-add epilogue (EPI_ADDC): row group I's four 16-B residual chunks
// per lane (`old`) were loaded before its stores, and group I + 1's are issued
// before group I's stores, so a tile's epilogue waits out about one memory
// latency instead of one per store (32 per wave): +15 % on the prompt pass's o
// projection when each store read its chunk itself.
template <int I>
__device__ __forceinline__ void pepi_addc(const Ctx& c, unsigned short* __restrict__ C, int ldc, int tm, int tn,
                                          const uint4 (&old)[NB / 2]) {
  if constexpr (I < MA) {
    const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
    unsigned short* rowp = C + (long)(tm * BM + c.wr * (BM / 2) + I * 16 + fr) * ldc + tn * BN + c.wc * (BN / 2) +
                           (fq & 1) * 16 + (fq >> 1) * 8;
    uint4 nxt[NB / 2];
    if constexpr (I + 1 < MA) {
#pragma unroll
      for (int p = 0; p < NB / 2; ++p) nxt[p] = *(const uint4*)(rowp + 16L * ldc + p * 32);
    }
    w4::static_for<0, NB / 2>([&](auto pc) {
      constexpr int p = decltype(pc)::value, q = I * NB + 2 * p;
      const f32x4 v0 = accr::read<q>(), v1 = accr::read<q + 1>();
      const unsigned x0 = pack_bf16x2(v0[0], v0[1]), y0 = pack_bf16x2(v0[2], v0[3]);
      const unsigned x1 = pack_bf16x2(v1[0], v1[1]), y1 = pack_bf16x2(v1[2], v1[3]);
      auto sx = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
      auto sy = __builtin_amdgcn_permlane16_swap(y0, y1, false, false);
      *(uint4*)(rowp + p * 32) = add_bf16x8(old[p], make_uint4(sx[0], sy[0], sx[1], sy[1]));
    });
    pepi_addc<I + 1>(c, C, ldc, tm, tn, nxt);
  }
}

// SwiGLU epilogue (X's SW digit, gemm_w4.h's one-shot SW epilogue on named
// accumulators): B's 256 rows of a tile are 128 gate and 128 up rows staged in
// alternating 32-row DMA groups, so a wave's fragment columns ng = 0, 1, 4, 5
// are gate and ng + 2 the matching up columns; output fragment pair (QQ, QQ + 1)
// = silu(gate) * up of fragments ng(QQ), ng(QQ + 1), both products rounded to
// bf16 first (the roundings of GEMM + silu_mul). C is [M, N / 2].
template <int Q>
__device__ __forceinline__ uint2 swiglu4() {
  constexpr int i = Q / NB, qh = Q % NB, ng = 4 * (qh / 2) + qh % 2;
  const f32x4 g = accr::read<i * NB + ng>(), u = accr::read<i * NB + ng + 2>();
  float r[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float gf = bf2f(f2bf(g[e]));
    r[e] = gf / (1.0f + __expf(-gf)) * bf2f(f2bf(u[e]));
  }
  return make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]));
}

template <int I, int QQ>
__device__ __forceinline__ void pepi_sw(const Ctx& c, unsigned short* __restrict__ C, int ldc, int tm, int tn) {
  if constexpr (I < MA) {
    if constexpr (QQ < NB / 2) {
      const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
      const uint2 o0 = swiglu4<I * NB + QQ>(), o1 = swiglu4<I * NB + QQ + 1>();
      auto sx = __builtin_amdgcn_permlane16_swap(o0.x, o1.x, false, false);
      auto sy = __builtin_amdgcn_permlane16_swap(o0.y, o1.y, false, false);
      const uint4 qv = make_uint4(sx[0], sy[0], sx[1], sy[1]);
      const int row = tm * BM + c.wr * (BM / 2) + I * 16 + fr;
      const int col0 = tn * (BN / 2) + c.wc * (BN / 4) + QQ * 16;
      *(uint4*)(C + (long)row * ldc + col0 + (fq & 1) * 16 + (fq >> 1) * 8) = qv;
      pepi_sw<I, QQ + 2>(c, C, ldc, tm, tn);
    } else {
      pepi_sw<I + 1, 0>(c, C, ldc, tm, tn);
    }
  }
}

// A ticket no launch could have issued. One launch hands label x at most ntx
// queue tickets (raw values 0 .. ntx - 1); with 64 launches sharing a slot as
// the bound, a raw value >= 64 ntx -- or a negative one -- means the slot was
// corrupted. The workgroup then stops taking tiles (the callers' range checks:
// no address is ever formed from it) and this marks the slot's error word,
// which tile_queue_check reports, so the tiles it skipped never pass silently
// (ADVICE r5). The word is not reset by the exit reset (words 0..8): sticky.
constexpr int TQ_ERR_WORD = 15;  // tile_queue.h TQ_ERR
__device__ __forceinline__ void mark_bad_ticket(int* q, int raw, int ntx) {
  if ((unsigned)raw >= 64u * (unsigned)ntx && threadIdx.x == 0)
    atomicExch(q + TQ_ERR_WORD, (int)(0x80000000u | ((unsigned)raw & 0x7fffffffu)));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_a(const unsigned short* A, int tm, int lda) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * BM * lda), 0, BM * lda * 2, 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_b(const unsigned short* B, int tn, int ldb) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * BN * ldb), 0, BN * ldb * 2, 0x00020000);
}
// B of tile column tn; SwiGLU: its 128 gate rows (rb) and the matching 128 up
// rows N / 2 further (rb2), as gemm_w4.h's SW staging reads them
template <bool SW>
__device__ __forceinline__ void set_b(Ctx& c, const unsigned short* B, int tn, int ldb, int N) {
  if constexpr (SW) {
    c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * (BN / 2) * ldb), 0, (BN / 2) * ldb * 2,
                                             0x00020000);
    c.rb2 = __builtin_amdgcn_make_buffer_rsrc((void*)(B + ((long)N / 2 + (long)tn * (BN / 2)) * ldb), 0,
                                              (BN / 2) * ldb * 2, 0x00020000);
  } else {
    c.rb = rsrc_b(B, tn, ldb);
  }
}

// Aligned shapes only (M, N % 256, K % 128 with K >= 384; 16-B operands); the
// grid is at most the tile count. X: gemm_w4.h's knob bag (tile map, DMA order).
// q: this launch's zeroed ticket slot (tile_queue.h), zero again on return.
// DYN: 1 = per-XCD ticket queue, first ticket static (the workgroup's rank in
// its label: no atomic before the first DMA); 2 = every ticket from the queue,
// the first one too (a workgroup that starts late -- its CU held by a
// collective launched just before -- takes only the tiles still left);
// 0 = the static walk v, v + G, v + 2G (q unused), for measurements.
// NTST: C stored non-temporally (production at 3-8 tiles per CU, gemm_persistent.hip; the output is not re-read
// by this launch, so it need not displace A / B lines in L2 / MALL).
// TS: timing build (experiments only, EPI_NONE): `bias` is a long long[grid][16]
// buffer; workgroup b writes [0] its start (s_memrealtime, 100 MHz), [1] HW_ID |
// XCC_ID << 32, [2 + j] the end of its j-th tile's epilogue (j < 11), [13] its
// exit (after the queue's exit counter / reset), [14] the end of its last tile,
// [15] tiles.
// L: LDS image layout (L % 10, Lay above) and MFMA order ((L / 10) % 10, ord_of); 0 = production.
// (L / 100) % 10, the C store (experiments only, EPI_NONE): 1 = no store (output not written),
// 2 = s_waitcnt vmcnt(0) right after each tile's stores (measurement builds: how much of a tile
// change waits on its stores -- gfx950 counts stores and loads in one vmcnt, so the next tile's
// first DMA wait also covers them); 3 = that first wait counts the tile's stores as younger ops
// (vmcnt(ND + stores)), so it waits for the next tile's K-tile 1 only.
// DD, SPS: deferred C stores (see pepi_d): SPS 16-B units per lane stored at the end of each of the next
// tile's first DD K-steps (0 = off, the epilogue stores everything). Needs K / 64 >= PEEL + 2 (below).
template <int EPI, int X = 0, int DYN = 1, bool NTST = false, bool TS = false, int L = 0, int DD = 0, int SPS = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4p(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int* __restrict__ q) {
  constexpr int ND = w4::dma_per_stage<BM, BN>();
  // the two stages plus one int at the end: the next tile's ticket, from wave 0.
  // One LDS object, not a second __shared__ variable: with two, hipcc's LDS-DMA
  // alias tracking put an s_waitcnt vmcnt(0) before every K-step's first
  // fragment read (all DMAs in flight drained).
  static_assert(2 * Lay<L % 10>::STAGE + 16 <= 160 * 1024, "LDS image exceeds 160 KiB");
  __shared__ __attribute__((aligned(1024))) char smem[2 * Lay<L % 10>::STAGE + 16];
  int& tslot = *(int*)(smem + 2 * Lay<L % 10>::STAGE);
  KGS_ACC_RESERVE();
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, ntiles = ntm * ntn;
  static_assert(!TS || EPI == EPI_NONE, "timing build: bias carries the stamp buffer");
  // X digit 10^6: SwiGLU (B = fused [gate; up], N = 2I rows, C = [M, I]); tiles
  // are 256 B rows = 128 gate + 128 up, ntn = N / 256
  constexpr bool SW = (X / 1000000) % 10 != 0;
  static_assert(!SW || (EPI == EPI_NONE && L == 0 && !NTST), "SwiGLU: no bias, production layout");
  static_assert(EPI != EPI_ADDC || !NTST, "the residual add reads C");
  constexpr int CST = (L / 100) % 10;
  static_assert(CST == 0 || (EPI == EPI_NONE && !SW && !NTST && !TS), "store measurement builds: plain C only");
  // CST 3: VMEM ops one epilogue issues per wave after the next tile's K-tile-1 DMAs (pepi: one
  // 16-B store per accumulator pair). vmcnt completes in issue order, loads and stores alike (hipcc
  // itself counts younger stores this way: vmcnt(3) for the first load of store, load, load, load, store); a count
  // at most the true number keeps every K-tile-1 DMA outside the allowed ops.
  constexpr int WXS = CST == 3 ? MA * NB / 2 : 0;
  constexpr int DEF = DD * SPS, UI = MA * NB / 2 - DEF;  // deferred / immediate units per lane
  // K-steps of a tile peeled out of the runtime loop: the storing ones, the one after them (its wait
  // counts their stores), rounded up to a stage pair
  constexpr int PEEL = DD ? ((DD + 2) & ~1) : 2;
  static_assert(DD == 0 || (EPI != EPI_ADDC && !SW && CST == 0 && L % 10 == 0), "deferred stores: plain tiles");
  static_assert(DEF >= 0 && UI >= 0 && (DD == 0 || SPS > 0), "deferred stores: at most a tile's units");
  static_assert((L / 1000) % 10 == 0 || (CST == 0 && !TS), "one-barrier K-step: no store measurement builds");
  constexpr bool WSK = (L / 1000000) % 10 == 1;  // wait-stamp build (pbody WSB)
  static_assert(!WSK || (EPI == EPI_NONE && !TS && !SW), "wait stamps: bias carries the stamp buffer");
  const unsigned long long wst0 = WSK ? __builtin_amdgcn_s_memtime() : 0ull;
  int wtiles = 0;
  long long* const ts = TS ? (long long*)bias + (long)blockIdx.x * 16 : nullptr;
  int ntile_done = 0;
  if constexpr (TS) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID, all 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));  // XCC_ID[3:0]
    if (threadIdx.x == 0) {
      ts[0] = t0;
      ts[1] = (long long)hw | ((long long)xcc << 32);
    }
  }

  Ctx c;
  c.smem = smem;
  c.w = w;
  c.wr = w >> 1;
  c.wc = w & 1;
  c.nt = K / BK;
  c.sa32 = 32 * lda * 2;
  c.sb32 = 32 * ldb * 2;
  {
    int row, ch;
    Lay<L % 10>::dma_lane(lane, w, row, ch);
    c.voa = (row * lda + ch * 8) * 2;
    c.vob = (row * ldb + ch * 8) * 2;
    const int fr = lane & 15, fq = lane >> 4;
    c.ro0 = Lay<L % 10>::read_lane(fr, fq);
    c.ro1 = Lay<L % 10>::read_lane(fr, 4 + fq);
  }
  const int x = blockIdx.x & 7;             // XCD label
  const int ntx = (ntiles - x + 7) >> 3;     // its tiles: v = x + 8 t, t < ntx
  // DYN: t is a ticket of label x (tile v = x + 8 t, t < ntx). The first one is
  // static, the workgroup's rank in its label (no atomic + barrier before the
  // first DMA: that cost 1.2 % at 3 tiles per CU); the queue numbers the rest
  // from nwx on. Against an RCCL-shaped collective holding 16-64 CUs for
  // 0.1-0.7 ms the static first ticket was faster than DYN 2 in all 18 cells
  // with the collective issued before the GEMMs (the bench step's order) and
  // within 2.3 % either way when issued after the first GEMM
  // (profiles/r4/overlap_rccl_README.md). Static walk: t = v.
  const int nwx = ((int)gridDim.x - x + 7) >> 3;  // workgroups of label x
  const int lim = DYN ? ntx : ntiles;
  const int base = DYN == 1 ? nwx : 0;  // queue tickets are numbered from here
  int t;
  if constexpr (DYN == 2) {
    if (threadIdx.x == 0) tslot = atomicAdd(q + x, 1);
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(tslot);
  } else {
    t = DYN ? (int)blockIdx.x >> 3 : (int)blockIdx.x;
  }
  // unsigned: a ticket outside [0, lim) -- a corrupted slot -- ends the
  // workgroup instead of becoming a tile index (no address from it, ever)
  if constexpr (DYN == 2) mark_bad_ticket(q, t, ntx);
  if ((unsigned)t >= (unsigned)lim) {  // (DYN 2: queue empty when this workgroup started; DYN 0/1: never with grid <= tiles)
    if (DYN && threadIdx.x == 0 && atomicAdd(q + 8, 1) == (int)gridDim.x - 1)
      for (int i = 0; i <= 8; ++i) atomicExch(q + i, 0);
    return;
  }
  int sl, tm, tn;
  w4::tile_of<X, false>(DYN ? x + 8 * t : t, ntiles, ntm, ntn, sl, tm, tn);
  c.ra = rsrc_a(A, tm, lda);
  set_b<SW>(c, B, tn, ldb, N);

  // prologue: K-tiles 0, 1 of the first tile into stages 0, 1; k-sub 0 of K-tile 0 into f0
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int j = 0; j < ND; ++j) pdma<L, X>(c, st, j, st * BK);
  // CST 3: K-tile 1 too, so the first tile's K-step 0 (no epilogue before it) may wait vmcnt(ND + WXS)
  if constexpr (WXS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else w4::wait_vm<ND>();
  w4::bar();
  Frag<MA, NB> f0, f1;
  {
    const char* pa = pabase<L>(c, 0, 0);
    const char* pb = pbbase<L>(c, 0, 0);
#pragma unroll
    for (int e = 0; e < S::NR; ++e) {
      const int x = w4::rd_idx(ord_of(L), MA, NB, e);
      if (w4::rd_isa(ord_of(L), MA, NB, e)) f0.a[x] = w4::frag(pa + Lay<L % 10>::frag_off(x));
      else f0.b[x] = w4::frag(pb + Lay<L % 10>::frag_off(x));
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);

  const int nt = c.nt;
  // The in-loop ticket fetch goes through an address hipcc cannot prove
  // uniform: for a uniform one its atomic optimizer broadcasts the result with
  // v_readfirstlane right after the atomic, i.e. an s_waitcnt vmcnt(0) (every
  // DMA in flight) at the top of each tile. This way the first use, after
  // K-step 0, waits only for the atomic.
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  auto tq = make_tick<WSK>(q + x + vzero, &tslot);
  // deferred stores: the previous tile's C block (first tile: zero-size, stores dropped)
  uint4 dq[DEF > 0 ? DEF : 1];
  __amdgpu_buffer_rsrc_t rprev = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, 0, 0x00020000);
  int voffc = 0;
  if constexpr (DEF > 0) {
#pragma unroll
    for (int u = 0; u < DEF; ++u) dq[u] = make_uint4(0, 0, 0, 0);
    const int fr = lane & 15, fq = lane >> 4;
    voffc = ((c.wr * (BM / 2) + fr) * ldc + c.wc * (BN / 2) + (fq & 1) * 16 + (fq >> 1) * 8) * 2;
  }
  for (;;) {
    if constexpr (DD > 0) {
      w4::static_for<0, PEEL>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        constexpr int TKJ = DYN ? (J == 0 ? 1 : J == 1 ? 2 : 0) : 0;
        constexpr int WXJ = (J >= 1 && J <= DD) ? SPS : 0;
        pstep<J & 1, X, J == 0, TKJ, L, WXJ, J < 2 ? 0 : 1>(c, c, f0, f1, J + 2, tq);
        if constexpr (J < DD) dstore<UI, J * SPS, SPS, DEF, NTST>(dq, rprev, voffc, ldc);
      });
    } else {
      pstep<0, X, true, DYN ? 1 : 0, L, WXS, 0>(c, c, f0, f1, 2, tq);   // ticket atomic after its barrier 2
      pstep<1, X, false, DYN ? 2 : 0, L, 0, 0>(c, c, f0, f1, 3, tq);  // ticket to LDS after its barrier 2
    }
    for (int t = PEEL; t < nt - 2; t += 2) {
      pstep<0, X, false, 0, L>(c, c, f0, f1, t + 2, tq);
      pstep<1, X, false, 0, L>(c, c, f0, f1, t + 3, tq);
    }
    const int raw = DYN ? __builtin_amdgcn_readfirstlane(tslot) : 0;
    if constexpr (DYN != 0) mark_bad_ticket(q, raw, ntx);
    const int tnx = DYN ? base + raw : t + (int)gridDim.x;
    const bool more = (unsigned)tnx < (unsigned)lim;  // see the first ticket's check
    int tmn = tm, tnn = tn;
    if (more) w4::tile_of<X, false>(DYN ? x + 8 * tnx : tnx, ntiles, ntm, ntn, sl, tmn, tnn);
    Ctx cn = c;
    cn.ra = rsrc_a(A, tmn, lda);
    set_b<SW>(cn, B, tnn, ldb, N);
    // the last two K-steps bring the next tile's K-tiles 0 and 1 (no next tile:
    // harmless re-loads of this tile's last K-tile into the freed stages)
    pstep<0, X, false, 0, L, 0, 2>(c, cn, f0, f1, more ? 0 : nt - 1, tq);
    pstep<1, X, false, 0, L, 0, 2>(c, cn, f0, f1, more ? 1 : nt - 1, tq);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // MFMA -> v_accvgpr_read
    if constexpr (SW) pepi_sw<0, 0>(c, C, ldc, tm, tn);
    float bv[NB][4];
    if constexpr (!SW) {
      const int fq = lane >> 4;
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
    }
    if constexpr (EPI == EPI_ADDC) {
      const int fr = lane & 15, fq = lane >> 4;
      const unsigned short* r0 =
          C + (long)(tm * BM + c.wr * (BM / 2) + fr) * ldc + tn * BN + c.wc * (BN / 2) + (fq & 1) * 16 + (fq >> 1) * 8;
      uint4 old0[NB / 2];
#pragma unroll
      for (int p = 0; p < NB / 2; ++p) old0[p] = *(const uint4*)(r0 + p * 32);
      pepi_addc<0>(c, C, ldc, tm, tn, old0);
    } else if constexpr (DEF > 0) {
      pepi_d<EPI, 0, UI, DEF, NTST>(c, C, ldc, tm, tn, bv, dq);
      rprev = rsrc_c(C, tm, tn, ldc);
    } else if constexpr (!SW) {
      pepi<EPI, 0, NTST, CST>(c, C, ldc, tm, tn, bv);
      if constexpr (CST == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (TS) {
      const long long te = (long long)__builtin_amdgcn_s_memrealtime();
      if (threadIdx.x == 0 && ntile_done < 11) ts[2 + ntile_done] = te;
      ++ntile_done;
      if (threadIdx.x == 0) {
        ts[14] = te;
        ts[15] = ntile_done;
      }
    }
    if constexpr (WSK) ++wtiles;
    if (!more) break;
    t = tnx;
    tm = tmn;
    tn = tnn;
    c.ra = cn.ra;
    c.rb = cn.rb;
    c.rb2 = cn.rb2;
  }
  if constexpr (DEF > 0) dstore<UI, 0, DEF, DEF, NTST>(dq, rprev, voffc, ldc);  // the last tile's deferred units
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail re-loads before LDS is released
  if constexpr (DYN != 0) {
    if (threadIdx.x == 0 && atomicAdd(q + 8, 1) == (int)gridDim.x - 1)  // last one out resets the queue
      for (int i = 0; i <= 8; ++i) atomicExch(q + i, 0);
  }
  if constexpr (TS) {
    __syncthreads();
    const long long tx = (long long)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) ts[13] = tx;
  }
  if constexpr (WSK) {
    // per wave: long long[grid][4][16] = ws[0..11], start, end (s_memtime), tiles
    const unsigned long long wst1 = __builtin_amdgcn_s_memtime();
    long long* const wb = (long long*)bias + ((long)blockIdx.x * 4 + w) * 16;
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 12; ++j) wb[j] = (long long)tq.ws[j];
      wb[12] = (long long)wst0;
      wb[13] = (long long)wst1;
      wb[14] = wtiles;
    }
  }
}

}  // namespace w4p
}  // namespace kgs
