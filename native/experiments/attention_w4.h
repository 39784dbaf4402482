// Flash-attention forward, round 4: ONE wave per SIMD, 64 query rows per wave
// (q-blocks qb = 0, 1 of 32 rows), 256 rows per workgroup, registers owned by
// name. The math, fragment layouts and LDS image are attention.hip's (swapped
// QK^T on v_mfma_f32_32x32x16_bf16, the S^T block reused as the P.V operand, V
// by ds_read_b64_tr_b16, K/V tiles of 64 keys by LDS-DMA into a double buffer,
// deferred-max rescale); what changes is where the registers live and what
// runs beside each MFMA:
//
//   O (128), Q (64) and the tile's K fragments (64) sit in named AGPRs
//   (attn_regs.h), so the arch VGPRs hold only S, V, P and the softmax: hipcc
//   cannot move the accumulators, and every K / V fragment read feeds BOTH
//   q-blocks (half the LDS read traffic per FLOP of attention.hip).
//
//   Per tile, four sections of 16 MFMAs, each MFMA followed by a fixed slice
//   of other work (pinned with sched_barrier, the GEMM's kbody technique; at
//   most two v_exp_f32 per MFMA gap):
//     A  QK^T(qb 0)  | one V fragment read (2 x ds_read_b64_tr_b16) per MFMA
//     B  QK^T(qb 1)  | softmax(qb 0): row max, exchange, the t = 0 keys, the
//                      first 6 t = 1 keys
//        lgkm / vm waits, barrier
//     C  P.V(qb 0), t = 0 keys first | softmax(qb 0) other t = 1 keys; softmax(qb 1):
//                      row max, exchange, t = 0 keys
//     D  P.V(qb 1)   | softmax(qb 1) t = 1 keys; then the K fragments of tile
//                      j + 1 into the K AGPRs and the LDS-DMA of tile j + 2
//   P.V runs over the t = 0 keys first, so the exponentials of the t = 1 keys
//   overlap the MFMAs that do not need them.
//
//   Causal: the wave's q-blocks are row blocks w and 7 - w of the workgroup's
//   256 rows, so the four waves (one per SIMD) run nearly the same number of
//   tiles; a diagonal tile past all of q-block 0's rows runs sections A-C
//   without q-block 0 (a second copy of the code, no per-slot branches).
//
// With one wave per SIMD nothing hides a stall, and three cost most of the
// time found by the timing build (profiles/r4/attention):
//   - a branch per MFMA slot (~40 cycles each): the wave index is made
//     wave-uniform (readfirstlane) and section D exists in two copies, with and
//     without the DMA of tile j + 2, instead of guarding each slot;
//   - the vmcnt(0) hipcc puts before a builtin ds_read_tr when an LDS-DMA is in
//     flight (its alias check cannot separate the two buffers): V reads are asm;
//   - three VALU ops per bf16 pair (kgs_common.h pack_bf16x2 now uses one).
//
// Hazards hipcc does not see (asm MFMAs, asm LDS reads): S is read by VALU only
// after a tied s_nop pad that follows the next section's first MFMA; O is read
// (rescale, epilogue) at least one section after the last P.V into it, and
// after a pad at the end; K AGPRs are rewritten in D, a barrier after the last
// QK^T; V fragment registers are read only after the barrier's lgkmcnt(0) (the
// ISA is checked for any earlier use of them, see docs/architecture.md).
#pragma once

#include <type_traits>

#include "attn_regs.h"
#include "kgs_common.h"

namespace kgs {
namespace attn4 {

using atr::f32x16;
typedef short bf16x4s __attribute__((ext_vector_type(4)));

constexpr int HD = 128;
constexpr int WR = 64;      // query rows per wave
constexpr int QB = 4 * WR;  // rows per workgroup
constexpr int KB = 64;      // keys per tile
constexpr int TILE_BYTES = KB * HD * 2;
constexpr float NEG = -1.0e30f;
constexpr float RESCALE = 8.0f;  // deferred-max threshold (log2 units): P <= 256

struct Args {
  const unsigned short* q;
  const unsigned short* k;
  const unsigned short* v;
  unsigned short* o;
  long ldq, ldk, ldv, ldo;
  int B, S, H, HKV;
  float sl2;
  int causal;
  int Sk;
  int qoff;
  long long* ts;  // timing build (TS): per (workgroup < 64, wave) s_memtime stamps, else unused
};

__device__ __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int off(int r, int c) { return 256 * r + 16 * (c ^ swz(r)); }

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// MFMA (asm) -> VALU read of its VGPR result: wait states the hazard
// recognizer cannot insert for an asm MFMA. Tied to s so that nothing reading
// s is scheduled above it.
__device__ __forceinline__ void pad_s(f32x16& s) { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(s)); }

// An asm MFMA reads its VGPR operands after issue, and hipcc, which cannot
// see that, would recycle a fragment's registers for VALU temporaries right
// after the MFMA that last names it (first cut: every P.V whose operands died
// in its own slot computed garbage). keep() extends the operands' live range
// into a later slot.
__device__ __forceinline__ void keep(const bf16x8& x) { asm volatile("" ::"v"(x)); }

__device__ __forceinline__ bf16x8 pack8(const f32x16& s, int base) { return pack_bf16x8(s, base); }

// Online softmax of one q-block's tile (two 32x32 S^T blocks, lane = one query
// row), in pieces the MFMA slots place: the row max over 8 scores (maxpart),
// the xor-32 exchange + deferred rescale of l and the AGPR-resident O (xchg),
// p = exp2(s sl2 - m sl2) with the row sum (exps), and the bf16 packing of one
// P.V operand (pack).
template <int QBI>
struct Softmax {
  f32x16 (&s)[2];
  float& m;
  float& l;
  bf16x8 (&pf)[2][2];
  float sl2;
  float mx, msl;

  template <int I>
  __device__ __forceinline__ void maxpart() {
    constexpr int t = I / 2, r0 = (I % 2) * 8;
    if constexpr (I == 0) mx = m;
#pragma unroll
    for (int r = r0; r < r0 + 8; ++r) mx = fmaxf(mx, s[t][r]);
  }
  __device__ __forceinline__ void xchg() {
    mx = xor32_max(mx);
    const bool grow = (mx - m) * sl2 > RESCALE;
    if (__any(grow)) {
      const float mn = grow ? mx : m;
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * sl2);
      m = mn;
      l *= alpha;
      atr::oscale<QBI, 0>(alpha);
      atr::oscale<QBI, 1>(alpha);
      atr::oscale<QBI, 2>(alpha);
      atr::oscale<QBI, 3>(alpha);
    }
    msl = m * sl2;
  }
  template <int T, int R0, int N>
  __device__ __forceinline__ void exps() {
#pragma unroll
    for (int r = R0; r < R0 + N; ++r) {
      const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[T][r], sl2, -msl));
      s[T][r] = p;
      l += p;
    }
  }
  template <int T, int SP>
  __device__ __forceinline__ void pack() {
    pf[T][SP] = pack8(s[T], 8 * SP);
  }
};

// causal mask of a diagonal tile: scores of keys past the lane's row -> NEG
__device__ __forceinline__ void mask_diag(f32x16 (&s)[2], int kv0, int hh, int rowlim) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kv = kv0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (kv > rowlim) s[t][r] = NEG;
    }
}

// TS: timing build. Workgroups 0..63 stamp s_memtime (shader cycles) at the
// start of every tile and after each of its sections, per wave: ts[((blk * 4 +
// w) * 64 + min(j, 63)) * 8 + e], e = 0 tile start, 1 after A, 2 after B, 3
// after the barrier, 4 after C, 5 after D.
template <bool TS = false>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void fwd(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE_BYTES];  // [buf][K, V]
  KGS_ATTN_RESERVE();

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hh = lane >> 5;
  const int nqb = a.S / QB;
  const bool stamp = TS && blockIdx.x < 64;
  auto ts = [&](int j, int e) {
    if constexpr (TS) {
      const long long t = (long long)__builtin_amdgcn_s_memtime();
      if (stamp && lane == 0) a.ts[(((long)blockIdx.x * 4 + w) * 64 + (j < 63 ? j : 63)) * 8 + e] = t;
    }
  };
  const int nwg = gridDim.x;
  int lid = blockIdx.x;
  if ((nwg & 31) == 0) {  // 8 consecutive slots of one XCD: 4 heads of one KV group
    const int t = lid >> 3, x = lid & 7;
    lid = ((t >> 2) << 5) | (x << 2) | (t & 3);
  }
  const int per = a.B * a.H;
  const int qi = lid / per, rem = lid - qi * per;
  const int qbk = a.causal ? nqb - 1 - qi : qi;  // heaviest first
  const int b = rem / a.H, h = rem - b * a.H;
  const int kvh = h / (a.H / a.HKV);

  // the wave's two 32-row q-blocks are blocks w and 7 - w of the workgroup's
  // 256 rows, so the four waves reach about the same causal depth
  const int q0 = qbk * QB;
  const int rb0 = q0 + 32 * w, rb1 = q0 + 32 * (7 - w);
  const long tok0 = (long)b * a.S;
  const long ktok0 = (long)b * a.Sk;
  const int qoff = a.qoff;

  static_for<0, 2>([&](auto qbc) {
    constexpr int qb = decltype(qbc)::value;
    static_for<0, 4>([&](auto dc) { atr::ozero<qb, decltype(dc)::value>(); });
    const bf16x8* qp = (const bf16x8*)(a.q + (tok0 + (qb ? rb1 : rb0) + l32) * a.ldq + (long)h * HD + 8 * hh);
    static_for<0, 8>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      atr::qwrite<qb, ks>(qp[2 * ks]);
    });
  });

  const unsigned short* kbase = a.k + ktok0 * a.ldk + (long)kvh * HD;
  const unsigned short* vbase = a.v + ktok0 * a.ldv + (long)kvh * HD;
  // LDS-DMA piece p (0..7) of this wave's share of tile jn: 1 KiB = 4 rows of
  // the K (p even) or V (p odd) tile, into buffer sb
  auto dma_piece = [&](int jn, int sb, int p) {
    const int ch = 4 * w + (p >> 1);
    const int r = 4 * ch + (lane >> 4), c = (lane & 15) ^ swz(r);
    const long row = (long)jn * KB + r;
    if (p & 1) glds16(vbase + row * a.ldv + 8 * c, smem[sb][1] + 1024 * ch);
    else glds16(kbase + row * a.ldk + 8 * c, smem[sb][0] + 1024 * ch);
  };
  auto dma_tiles = [&](int jn, int sb) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_piece(jn, sb, p);
  };
  // LDS byte address of this lane's K fragment (t, ks) in buffer sb
  const unsigned kbase_lds = (unsigned)(uintptr_t)(KGS_LDS char*)smem[0][0];
  auto kaddr = [&](int sb, int t, int ks) -> unsigned {
    return kbase_lds + (unsigned)(sb * 2 * TILE_BYTES + off(32 * t + l32, 2 * ks + hh));
  };
  const int g = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  bf16x8 vf[4][2][2];
  // V fragment reads as asm: with the builtin, hipcc's LDS-DMA alias check
  // cannot tell buffer j from the buffer the DMA of tile j + 1 fills and puts
  // a vmcnt(0) at the top of section A (a full wait for the DMA issued one
  // section earlier). The fragments are used after the barrier's lgkmcnt(0)
  // only, and nothing between reads their registers (checked in the ISA).
  auto read_v = [&](const char* Vs, int d, int t, int sp) {
    const int c0 = 4 * d + 2 * (g & 1) + (tp >> 1);
    const int kvb = 32 * t + 16 * sp + 4 * hh + tq;
    const unsigned vl = (unsigned)(uintptr_t)(const KGS_LDS char*)Vs + 8 * (tp & 1);
    bf16x4s x, y;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x) : "v"(vl + (unsigned)off(kvb, c0)));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(y) : "v"(vl + (unsigned)off(kvb + 8, c0)));
    vf[d][t][sp] = __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  const int ntile = a.causal ? (qoff + q0 + QB) / KB : a.Sk / KB;
  const int wlast = qoff + rb1 + 31;  // this wave's last row (causal limit)

  dma_tiles(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): Q and tile 0
  __syncthreads();
  if (ntile > 1) dma_tiles(1, 1);
  static_for<0, 16>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    atr::kread<k / 8, k % 8>(kaddr(0, k / 8, k % 8));
  });

  float m0 = NEG, l0 = 0.f, m1 = NEG, l1 = 0.f;
  const float sl2 = a.sl2;

  for (int j = 0; j < ntile; ++j) {
    const int buf = j & 1;
    const int kv0 = j * KB;
    const bool act = !a.causal || kv0 <= wlast;
    const bool act0 = !a.causal || kv0 <= qoff + rb0 + 31;  // q-block 0 has rows in tile j
    f32x16 s0[2], s1[2];
    bf16x8 pf0[2][2], pf1[2][2];
    Softmax<0> sm0{s0, m0, l0, pf0, sl2, 0.f, 0.f};
    Softmax<1> sm1{s1, m1, l1, pf1, sl2, 0.f, 0.f};
    ts(j, 0);
    if (act) {
      const char* Vs = smem[buf][1];
      // K(j) in its AGPRs, in two steps: the t = 0 fragments (the first 8 of
      // the 16 reads) now, the rest before the first t = 1 MFMA (slot 8, after
      // 16 V reads: lgkmcnt(15), the counter's ceiling, over-waits by one)
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      fence();
      // (sections A-C in two copies: a causal diagonal tile past all of
      //  q-block 0's rows runs q-block 1 only)
      auto sec_ab = [&](auto q0c) {
        constexpr bool Q0 = decltype(q0c)::value;
        // A: QK^T(qb 0), one V fragment per MFMA
        static_for<0, 16>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if constexpr (k == 8) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
          if constexpr (Q0) atr::qk<0, k / 8, k % 8, k % 8 == 0>(s0[k / 8]);
          read_v(Vs, k / 4, (k / 2) % 2, k % 2);
          fence();
        });
        ts(j, 1);
        // B: QK^T(qb 1) | max, exchange and the t = 0 half of softmax(qb 0)
        static_for<0, 16>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          atr::qk<1, k / 8, k % 8, k % 8 == 0>(s1[k / 8]);
          if constexpr (Q0) {
            if constexpr (k == 0) {
              pad_s(s0[1]);  // (s0[0]'s last MFMA is 8 MFMAs back)
              if (a.causal && kv0 + KB - 1 > qoff + rb0) mask_diag(s0, kv0, hh, qoff + rb0 + l32);
            }
            if constexpr (k < 4) sm0.template maxpart<k>();
            if constexpr (k == 4) sm0.xchg();
            if constexpr (k >= 5 && k < 13) sm0.template exps<0, 2 * (k - 5), 2>();
            if constexpr (k == 13) sm0.template pack<0, 0>();
            if constexpr (k == 14) sm0.template pack<0, 1>();
            // the first 6 t = 1 scores here: section C carries the q-block 1
            // max and exchange as well and ran ~600 cycles longer than B
            if constexpr (k >= 13) sm0.template exps<1, 2 * (k - 13), 2>();
          }
          fence();
        });
      };
      if (act0) sec_ab(std::true_type{});
      else sec_ab(std::false_type{});
      ts(j, 2);
    }
    // tile j's V is in registers and tile j + 1 has landed: after the barrier
    // buffer j is free for tile j + 2 (its DMA is issued in section D)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __syncthreads();
    ts(j, 3);
    const bool dnext = j + 2 < ntile;
    if (act) {
      // C: P.V(qb 0), t = 0 keys first | the t = 1 half of softmax(qb 0), then
      //    max, exchange and the t = 0 half of softmax(qb 1)
      auto sec_c = [&](auto q0c) {
        constexpr bool Q0 = decltype(q0c)::value;
        static_for<0, 16>([&](auto kc) {
          constexpr int k = decltype(kc)::value, t = k / 8, sp = (k % 8) / 4, d = k % 4;
          if constexpr (Q0) {
            atr::pv<0, d>(vf[d][t][sp], pf0[t][sp]);
            if constexpr (k >= 2) {  // operands of the P.V two slots back
              constexpr int kk = k - 2;
              keep(vf[kk % 4][kk / 8][(kk % 8) / 4]);
              keep(pf0[kk / 8][(kk % 8) / 4]);
            }
          }
          if constexpr (k == 0) {
            pad_s(s1[1]);
            if (a.causal && kv0 + KB - 1 > qoff + rb1) mask_diag(s1, kv0, hh, qoff + rb1 + l32);
          }
          if constexpr (Q0 && k < 5) sm0.template exps<1, 6 + 2 * k, 2>();
          if constexpr (k < 4) sm1.template maxpart<k>();
          if constexpr (Q0 && k == 1) sm0.template pack<1, 0>();
          if constexpr (k == 5) sm1.xchg();
          if constexpr (Q0 && k == 5) sm0.template pack<1, 1>();
          if constexpr (k >= 8) sm1.template exps<0, 2 * (k - 8), 2>();
          if constexpr (k == 12) sm1.template pack<0, 0>();
          if constexpr (k == 15) sm1.template pack<0, 1>();
          fence();
        });
      };
      if (act0) sec_c(std::true_type{});
      else sec_c(std::false_type{});
      ts(j, 4);
      // D: P.V(qb 1) | the t = 1 half of softmax(qb 1), then the K fragments
      //    of tile j + 1 into their AGPRs and the LDS-DMA of tile j + 2
      // (two copies, with and without the tile j + 2 pieces, so no slot
      // branches)
      auto sec_d = [&](auto dnc) {
      static_for<0, 16>([&](auto kc) {
        constexpr int k = decltype(kc)::value, t = k / 8, sp = (k % 8) / 4, d = k % 4;
        atr::pv<1, d>(vf[d][t][sp], pf1[t][sp]);
        if constexpr (k >= 2) {
          constexpr int kk = k - 2;
          keep(vf[kk % 4][kk / 8][(kk % 8) / 4]);
          keep(pf1[kk / 8][(kk % 8) / 4]);
        } else {  // section C's last two
          constexpr int kk = 14 + k;
          keep(vf[kk % 4][kk / 8][(kk % 8) / 4]);
          keep(pf0[kk / 8][(kk % 8) / 4]);
        }
        if constexpr (k < 8) sm1.template exps<1, 2 * k, 2>();
        if constexpr (k == 4) sm1.template pack<1, 0>();
        if constexpr (k == 7) sm1.template pack<1, 1>();
        if constexpr (k >= 8) {
          // K(j + 1) fragments (in LDS since the barrier) into the K AGPRs,
          // unconditionally -- LDS in bounds -- and used only by a wave that
          // has rows in tile j + 1 (in section C they cost ~150 cycles there
          // against ~40 here, profiles/r4/attention)
          constexpr int f0 = 2 * (k - 8);
          atr::kread<f0 / 8, f0 % 8>(kaddr(buf ^ 1, f0 / 8, f0 % 8));
          atr::kread<(f0 + 1) / 8, (f0 + 1) % 8>(kaddr(buf ^ 1, (f0 + 1) / 8, (f0 + 1) % 8));
          if constexpr (decltype(dnc)::value) dma_piece(j + 2, buf, k - 8);
        }
        fence();
      });
      };
      if (dnext) sec_d(std::true_type{});
      else sec_d(std::false_type{});
      // the last two P.V read their operands after issue: hold them a while
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::"v"(vf[2][1][1]), "v"(vf[3][1][1]), "v"(pf1[1][1]));
      ts(j, 5);
    } else if (dnext) {
      // a causal wave past its last row still fills its share of the tiles
#pragma unroll
      for (int p = 0; p < 8; ++p) dma_piece(j + 2, buf, p);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last P.V -> v_accvgpr_read

  static_for<0, 2>([&](auto qbc) {
    constexpr int qb = decltype(qbc)::value;
    const float inv = 1.0f / xor32_sum(qb ? l1 : l0);
    unsigned short* op = a.o + (tok0 + (qb ? rb1 : rb0) + l32) * a.ldo + (long)h * HD;
    static_for<0, 4>([&](auto dc) {
      constexpr int d = decltype(dc)::value;
      const f32x16 o = atr::oread<qb, d>();
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int dcol = 32 * d + 8 * r4 + 4 * hh;
        uint2 pk;
        pk.x = pack_bf16x2(o[4 * r4 + 0] * inv, o[4 * r4 + 1] * inv);
        pk.y = pack_bf16x2(o[4 * r4 + 2] * inv, o[4 * r4 + 3] * inv);
        *(uint2*)(op + dcol) = pk;
      }
    });
  });
}

}  // namespace attn4
}  // namespace kgs
