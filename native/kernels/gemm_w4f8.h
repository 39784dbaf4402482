// gemm_w4f8: fp8 (OCP e4m3) NT GEMM on the persistent four-wave structure of
// gemm_w4p.h. C (bf16) = act(alpha * A . B^T + bias), A [M, K], B [N, K] fp8.
//
// Bytes: a K-tile is 256 rows x 128 fp8 (= 64 16-bit words, the bf16 kernel's
// 128-byte rows), so the LDS-DMA, the XOR swizzle, the stages and the tile
// walk are gemm_w4.h / gemm_w4p.h byte for byte (the host passes K and the
// leading dimensions in 16-bit words). What differs is the MFMA:
// v_mfma_f32_16x16x128_f8f6f4 takes a whole 128-byte K-tile row per operand
// (32 bytes per lane: the two 16-byte fragments the bf16 kernel reads as its
// two k-subs, concatenated), twice the bf16 FLOPs for the same bytes moved.
// A K-step is 64 MFMAs per wave (8 x 8 accumulators) of twice the bf16 MFMA's
// cycles -- the bf16 K-step's matrix time -- over the same 64 KiB of LDS-DMA.
//
// Registers: every MFMA of a K-step needs BOTH halves of its A and B rows, so
// the bf16 kernel's "k-sub 0 while k-sub 1 is read" split does not exist. The
// K-step is split by A rows instead:
//   H1  MFMAs (i = 0..3, n = 0..7), growing-square order; during the first 8
//       the A rows 4..7 of this K-tile are read (8 ds_read_b128)
//   H2  MFMAs (i = 4..7, n = 0..7), i-major
//   barrier 1 after MFMA B1 - 1 (this K-tile's reads retired: the stage is free),
//   the 16 DMAs of K-tile t + 2 spread up to barrier 2 (vmcnt: K-tile t + 1
//   landed, KM - R - 1), then the 24 reads of K-tile t + 1 that H1 needs first
//   (B rows 0..7 into the other B set, A rows 0..3, whose last use was H1)
//   P per MFMA over the last R (FKnobs: B1 12, R 12, P 2).
// A: 8 x 32 B (64 VGPRs), B: two sets of 8 x 32 B (128 VGPRs): ~220 VGPRs
// next to the 256 named accumulator AGPRs (acc_regs.h).
#pragma once

#include "acc_regs.h"
#include "gemm_w4.h"
#include "gemm_w4p.h"

namespace kgs {
namespace w4f8 {

using w4::BK;
using w4::Ctx;
using w4p::Tick;

constexpr int BM = 256, BN = 256, MA = 8, NB = 8;
using S = w4::Shape<BM, BN>;
constexpr int KM = 64;   // MFMAs per K-step
constexpr int ND = w4::dma_per_stage<BM, BN>();
// Schedule knobs: barrier 1 after MFMA B1 - 1, R MFMAs after barrier 2, P reads
// of K-tile t + 1 after each of them (24 reads). Production 12 / 12 / 2: the
// DMA window grows from 28 to 40 MFMAs; 8192^3 3426 vs 3378 (12 / 24 / 1),
// 8192x6144x4096 3129 vs 3068 TFLOP/s (profiles/r3/gemm_fp8_w4f8_knobs.json).
struct FKnobs {
  static constexpr int B1 = 12, R = 12, P = 2;
};

struct FragF8 {
  bf16x8 a[MA][2];     // this K-tile's A rows (two 16-byte halves)
  bf16x8 b[2][NB][2];  // B rows, two sets: K-step t uses set t & 1
};

__device__ __forceinline__ accr::i32x8 cat(const bf16x8& lo, const bf16x8& hi) {
  typedef short s16 __attribute__((ext_vector_type(16)));
  const s16 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  return __builtin_bit_cast(accr::i32x8, v);
}

template <bool ZERO, int P, int I, int N>
__device__ __forceinline__ void fmma(const FragF8& f) {
  if constexpr (ZERO) accr::mfma0_f8<I * NB + N>(cat(f.b[P][N][0], f.b[P][N][1]), cat(f.a[I][0], f.a[I][1]));
  else accr::mfma_f8<I * NB + N>(cat(f.b[P][N][0], f.b[P][N][1]), cat(f.a[I][0], f.a[I][1]));
}

// read e (0..23) of a K-tile's H1 operands: fragment r = e / 2 of the
// growing-square read order over (A rows 0..3, B rows 0..7), half e % 2
// (half 0 / 1 = the bf16 kernel's k-sub 0 / 1 chunk of the row, abase / bbase
// <.., 0 / 1>: the swizzle makes the hi chunk +-64 B away depending on the row)
template <int SET, int E>
__device__ __forceinline__ void h1_read(FragF8& f, const char* const (&pa)[2], const char* const (&pb)[2]) {
  constexpr int r = E / 2, h = E % 2;
  constexpr int x = w4::rd_idx(1, 4, NB, r);
  if constexpr (w4::rd_isa(1, 4, NB, r)) f.a[x][h] = w4::frag(pa[h] + x * 2048);
  else f.b[SET][x][h] = w4::frag(pb[h] + x * 2048);
}

// One MFMA slot K of the K-step on stage ST (= B set) and what follows it.
template <int ST, int X, bool ZERO, int TK, int B1, int R, int P, int K>
__device__ __forceinline__ void fbody(const Ctx& c, const Ctx& cd, int k0, FragF8& f, Tick& tq) {
  static_assert(B1 >= 8 + 1 && KM - R >= 32 + 8 && R * P >= 24, "A rows 0..3 are re-read only after H1");
  if constexpr (K < KM) {
    if constexpr (K < 32) {
      constexpr int i = w4::Order<1, 4, NB>::o.i[K], n = w4::Order<1, 4, NB>::o.n[K];
      fmma<ZERO, ST, i, n>(f);
    } else {
      fmma<ZERO, ST, 4 + (K - 32) / NB, (K - 32) % NB>(f);
    }
    if constexpr (K < 8) {  // A rows 4..7 of this K-tile
      constexpr int i = 4 + K / 2, h = K % 2;
      f.a[i][h] = w4::frag(w4::abase<BM, BN, h>(c, ST) + i * 2048);
    }
    if constexpr (K >= B1 && K < KM - R) {
      constexpr int NW = KM - R - B1;
#pragma unroll
      for (int j = 0; j < ND; ++j)
        if (B1 + (j * NW) / ND == K) w4::dma_any<BM, BN, X>(cd, ST, j, k0);
    }
    if constexpr (K >= KM - R && (K - (KM - R)) * P < 24) {  // H1 operands of K-tile t + 1 (stage / B set ST ^ 1)
      const char* const pa[2] = {w4::abase<BM, BN, 0>(c, ST ^ 1), w4::abase<BM, BN, 1>(c, ST ^ 1)};
      const char* const pb[2] = {w4::bbase<BM, BN, 0>(c, ST ^ 1), w4::bbase<BM, BN, 1>(c, ST ^ 1)};
      constexpr int e0 = (K - (KM - R)) * P;
      w4::static_for<e0, (e0 + P < 24 ? e0 + P : 24)>([&](auto e) { h1_read<ST ^ 1, decltype(e)::value>(f, pa, pb); });
    }
    w4::fence();
    if constexpr (K == B1 - 1) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage ST retired
      w4::bar();
    }
    if constexpr (K == KM - R - 1) {
      w4::wait_vm<ND>();
      w4::bar();
      if constexpr (TK == 1) {
        if (threadIdx.x == 0) tq.tk = atomicAdd(tq.qx, 1);
      } else if constexpr (TK == 2) {
        if (threadIdx.x == 0) *tq.slot = tq.tk;
      }
    }
    fbody<ST, X, ZERO, TK, B1, R, P, K + 1>(c, cd, k0, f, tq);
  }
}

template <int ST, int X, bool ZERO, int TK, class KN>
__device__ __forceinline__ void fstep(const Ctx& c, const Ctx& cd, FragF8& f, int kd, Tick& tq) {
  fbody<ST, X, ZERO, TK, KN::B1, KN::R, KN::P, 0>(c, cd, kd * BK, f, tq);
}

// epilogue: alpha * acc (+ bias, activation), bf16, paired n-tiles, 16-B stores
template <int EPI, int Q>
__device__ __forceinline__ void fepi(const Ctx& c, unsigned short* __restrict__ C, int ldc, int tm, int tn,
                                     float alpha, const float (&bv)[NB][4]) {
  if constexpr (Q < MA * NB) {
    constexpr int i = Q / NB, n = Q % NB;
    const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
    const f32x4 v0 = accr::read<Q>() * alpha, v1 = accr::read<Q + 1>() * alpha;
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
    *(uint4*)(C + (long)row * ldc + col0 + (fq & 1) * 16 + (fq >> 1) * 8) = qv;
    fepi<EPI, Q + 2>(c, C, ldc, tm, tn, alpha, bv);
  }
}

// Aligned shapes: M, N % 256, K (fp8 elements) % 256 with K >= 768 (Kw >= 384
// words: the ticket read needs a barrier between K-step 1 and the last pair).
// Kw / ldaw / ldbw are in 16-bit words (fp8 elements / 2); ldc in bf16
// elements. alpha *= *alpha_ptr when alpha_ptr is given (dynamic activation
// scale). q: this launch's ticket slot (tile_queue.h). Grid <= tiles.
template <int EPI, int X = 0, class KN = FKnobs>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_fp8_w4p(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, int M, int N, int Kw, int ldaw, int ldbw, int ldc, float alpha,
    const float* __restrict__ alpha_ptr, int* __restrict__ q) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * S::STAGE + 16];
  int& tslot = *(int*)(smem + 2 * S::STAGE);
  KGS_ACC_RESERVE();
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, ntiles = ntm * ntn;
  if (alpha_ptr) alpha *= *alpha_ptr;

  Ctx c;
  c.smem = smem;
  c.w = w;
  c.wr = w >> 1;
  c.wc = w & 1;
  c.nt = Kw / BK;
  c.sa32 = 32 * ldaw * 2;
  c.sb32 = 32 * ldbw * 2;
  {
    const int row = w * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    c.voa = (row * ldaw + ch * 8) * 2;
    c.vob = (row * ldbw + ch * 8) * 2;
    const int fr = lane & 15, fq = lane >> 4, fs = fr >> 1;
    c.ro0 = fr * 128 + ((fq ^ fs) * 16);
    c.ro1 = fr * 128 + (((4 + fq) ^ fs) * 16);
  }
  const int x = blockIdx.x & 7;
  const int ntx = (ntiles - x + 7) >> 3;
  const int nwx = ((int)gridDim.x - x + 7) >> 3;
  int t = (int)blockIdx.x >> 3;
  if (t >= ntx) {  // (never with the host's grid <= tiles)
    if (threadIdx.x == 0 && atomicAdd(q + 8, 1) == (int)gridDim.x - 1)
      for (int i = 0; i <= 8; ++i) atomicExch(q + i, 0);
    return;
  }
  int sl, tm, tn;
  w4::tile_of<X, false>(x + 8 * t, ntiles, ntm, ntn, sl, tm, tn);
  c.ra = w4p::rsrc_a(A, tm, ldaw);
  c.rb = w4p::rsrc_b(B, tn, ldbw);

#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int j = 0; j < ND; ++j) w4::dma_any<BM, BN, X>(c, st, j, st * BK);
  w4::wait_vm<ND>();
  w4::bar();
  FragF8 f;
  {
    const char* const pa[2] = {w4::abase<BM, BN, 0>(c, 0), w4::abase<BM, BN, 1>(c, 0)};
    const char* const pb[2] = {w4::bbase<BM, BN, 0>(c, 0), w4::bbase<BM, BN, 1>(c, 0)};
    w4::static_for<0, 24>([&](auto e) { h1_read<0, decltype(e)::value>(f, pa, pb); });
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);

  const int nt = c.nt;
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  Tick tq{q + x + vzero, &tslot, 0};
  for (;;) {
    fstep<0, X, true, 1, KN>(c, c, f, 2, tq);
    fstep<1, X, false, 2, KN>(c, c, f, 3, tq);
    for (int k = 2; k < nt - 2; k += 2) {
      fstep<0, X, false, 0, KN>(c, c, f, k + 2, tq);
      fstep<1, X, false, 0, KN>(c, c, f, k + 3, tq);
    }
    const int raw = __builtin_amdgcn_readfirstlane(tslot);
    w4p::mark_bad_ticket(q, raw, ntx);  // a corrupted slot is reported (gemm_w4p.h)
    const int tnx = nwx + raw;
    const bool more = (unsigned)tnx < (unsigned)ntx;  // a ticket outside [0, ntx) never becomes a tile index
    int tmn = tm, tnn = tn;
    if (more) w4::tile_of<X, false>(x + 8 * tnx, ntiles, ntm, ntn, sl, tmn, tnn);
    Ctx cn = c;
    cn.ra = w4p::rsrc_a(A, tmn, ldaw);
    cn.rb = w4p::rsrc_b(B, tnn, ldbw);
    fstep<0, X, false, 0, KN>(c, cn, f, more ? 0 : nt - 1, tq);
    fstep<1, X, false, 0, KN>(c, cn, f, more ? 1 : nt - 1, tq);
    // MFMA -> v_accvgpr_read: the 16x16x128 fp8 MFMA has more passes than the bf16 one
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    float bv[NB][4];
    {
      const int fq = lane >> 4;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[n][e] = 0.f;
        if constexpr (EPI != EPI_NONE) {
          const bf16x4 bb = *(const bf16x4*)(bias + tn * BN + c.wc * (BN / 2) + n * 16 + fq * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[n][e] = bf2f((unsigned short)bb[e]);
        }
      }
    }
    fepi<EPI, 0>(c, C, ldc, tm, tn, alpha, bv);
    if (!more) break;
    t = tnx;
    tm = tmn;
    tn = tnn;
    c.ra = cn.ra;
    c.rb = cn.rb;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && atomicAdd(q + 8, 1) == (int)gridDim.x - 1)
    for (int i = 0; i <= 8; ++i) atomicExch(q + i, 0);
}

}  // namespace w4f8
}  // namespace kgs
