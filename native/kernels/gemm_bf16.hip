// bf16 GEMM for gfx950 (MI355X / CDNA4), hand-written on MFMA + LDS-DMA.
//
//   C[M,N] (bf16) = epilogue( A[M,K] · B[N,K]^T )      f32 accumulation
//
// Both operands are K-contiguous ("NT", the torch.nn.Linear weight layout), so
// every MFMA fragment is one 16-byte LDS read.
//
// Kernels (variant numbers are the C ABI's `variant` argument):
//
//  * gemm_nt_256 -- the hot path (M%256 == N%256 == 0, K%128 == 0), variant 1.
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
//      MFMA block overlaps its partner's LDS-read/DMA-issue block. The RAW/WAR
//      accounting of both schedules is next to phase<>() below.
//      LDS image: 128-byte rows, 16-byte chunk c stored at c ^ ((row >> 1) & 7),
//      which makes every ds_read_b128 16-lane group hit 16 distinct bank slots
//      (conflict-free, SQ_LDS_BANK_CONFLICT = 0); the swizzle is applied to the
//      glds SOURCE address. Grid: one block per 256x256 tile, XCD-bijective
//      remap, then GROUP_M=4 grouped order so the 32 co-resident tiles of an
//      XCD form a 4x8 patch sharing A/B panels (L2 hit 81 % = 1 - 12/64).
//      Template S selects schedule knobs; variants 4-9 and 11 are the measured
//      alternatives and timing probes (profiles/gemm_tuning.md).
//
//  * gemm_nt_256p32 (variant 10) -- 32-MFMA phases (half the barriers) with a
//      160 KiB 10-slot ring; correct but 10 % slower (kept as a measured
//      negative result: its trailing waves issue 8 glds per phase).
//
//  * gemm_nt_256w4 (variant 3) -- 4 waves x 128x128 with AGPR-pinned asm MFMAs;
//      correct, ~15 % slower (LDS-DMA issue inside the MFMA stream).
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
// C ABI: kgs_gemm_bf16_nt(...) (bottom of file), loaded from Python via ctypes
// (kgs/ops/_lib.py) and from the C++ benches.
//
// Reference parity: the reference (kind-gpu-sim) has no kernels at all -- its
// test pod only echoes (pods/rocm-gpu-test-pod.yaml:9, Readme.md:16-20). This is
// the in-pod hot path required by BASELINE.json configs 3-4.
#include "kgs_common.h"

namespace kgs {
namespace g256 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF_BYTES = 128 * BK * 2;   // 16 KiB: 128 rows x 128 B
constexpr int BUF_BYTES = 4 * HALF_BYTES;  // A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * BUF_BYTES;   // 2-deep ring = 128 KiB
constexpr int P_A0 = 0, P_A1 = 1, P_B0 = 2, P_B1 = 3;
constexpr int LOOKAHEAD = 5;               // half-tiles issued ahead of use
constexpr int GROUP_M = 8;

struct Regs {
  bf16x8 a[4][2];        // A fragments of the current m-half: [m-tile][k-sub]
  bf16x8 b[2][2][2];     // B fragments of both n-halves: [n-half][n-tile][k-sub]
  f32x4 acc[2][4][2][2]; // [m-half][m-tile][n-half][n-tile]
};

struct Ctx {
  char* smem;
  const unsigned short* Ag;  // A + tile_m*256*lda
  const unsigned short* Bg;  // B + tile_n*256*ldb
  long a_half;               // 128*lda (elements)
  long b_half;
  int offA0, offA1, offB0, offB1;  // per-lane glds source offsets (elements)
  int ro0, ro1;                    // per-lane ds_read byte offsets for k-sub 0/1
  int wr, wc, w;                   // wave coordinates (wave-uniform)
  int nt;                          // number of K-tiles
  // bounded mode (S bit 9): operands read through buffer resources whose
  // num_records ends at the last valid row, so rows >= M (N) load zeros; lanes
  // whose 16-B chunk starts at k >= K get an out-of-range offset (zeros too).
  __amdgpu_buffer_rsrc_t ra, rb;
  int K, kc0, kc1;                 // K and the lane's logical chunk column (elements)
  int a_half_i, b_half_i;          // 128*lda, 128*ldb as int
  // transposed operands (S bits 11/12: A stored [K][M] / B stored [K][N]):
  // half-tiles are [64 k][128 cols] with 256-B rows, read with
  // ds_read_b64_tr_b16; see read_a_tr / read_b_tr
  long a_kstride, b_kstride;       // elements between consecutive k (lda / ldb)
  int tr_base;                     // per-lane byte offset of the tr-read block
  int tr_x;                        // per-lane chunk XOR (2 * gsw)
  // persistent mode (S bit 15): operand panels of the tile this block does next
  const unsigned short* Ag2;
  const unsigned short* Bg2;
  int has_next;
};

constexpr int OOB_OFFSET = 0x7FFFFFF0;  // > every num_records the bounded path builds

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int PART, bool BND = false, bool TR = false>
__device__ __forceinline__ void issue(const Ctx& c, int buf, int k0, bool nxt = false) {
  char* dst = c.smem + buf * BUF_BYTES + PART * HALF_BYTES + c.w * 2048;
  if constexpr (TR) {
    // operand stored [K][cols]: the half-tile is 64 k-rows x 128 columns; the
    // per-lane offsets already hold row*ld + swizzled column
    constexpr bool isA = PART == P_A0 || PART == P_A1;
    const unsigned short* src = (isA ? c.Ag : c.Bg) + ((PART == P_A1 || PART == P_B1) ? 128 : 0) +
                                (long)k0 * (isA ? c.a_kstride : c.b_kstride);
    glds16(src + (isA ? c.offA0 : c.offB0), dst);
    glds16(src + (isA ? c.offA1 : c.offB1), dst + 1024);
    return;
  }
  if constexpr (BND) {
    constexpr bool isA = PART == P_A0 || PART == P_A1;
    const int half = PART == P_A1 ? c.a_half_i : PART == P_B1 ? c.b_half_i : 0;
    const int o0 = (isA ? c.offA0 : c.offB0) + half + k0;
    const int o1 = (isA ? c.offA1 : c.offB1) + half + k0;
    const int v0 = k0 + c.kc0 < c.K ? o0 * 2 : OOB_OFFSET;
    const int v1 = k0 + c.kc1 < c.K ? o1 * 2 : OOB_OFFSET;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? c.ra : c.rb, (KGS_LDS void*)dst, 16, v0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? c.ra : c.rb, (KGS_LDS void*)(dst + 1024), 16, v1, 0, 0, 0);
    return;
  }
  const unsigned short* src;
  int o0, o1;
  if constexpr (PART == P_A0 || PART == P_A1) {
    src = (nxt ? c.Ag2 : c.Ag) + (PART == P_A1 ? c.a_half : 0) + k0;
    o0 = c.offA0; o1 = c.offA1;
  } else {
    src = (nxt ? c.Bg2 : c.Bg) + (PART == P_B1 ? c.b_half : 0) + k0;
    o0 = c.offB0; o1 = c.offB1;
  }
  glds16(src + o0, dst);
  glds16(src + o1, dst + 1024);
}

// Read the 4 m-tiles x 2 k-subs of A for this wave from half-tile `part`.
template <class CtxT>
__device__ __forceinline__ void read_a(const CtxT& c, Regs& R, const char* half) {
  const char* p = half + c.wr * 64 * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    R.a[i][0] = *(const bf16x8*)(p + i * 16 * 128 + c.ro0);
    R.a[i][1] = *(const bf16x8*)(p + i * 16 * 128 + c.ro1);
  }
}

template <int NH, class CtxT>
__device__ __forceinline__ void read_b(const CtxT& c, Regs& R, const char* half) {
  const char* p = half + c.wc * 32 * 128;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    R.b[NH][n][0] = *(const bf16x8*)(p + n * 16 * 128 + c.ro0);
    R.b[NH][n][1] = *(const bf16x8*)(p + n * 16 * 128 + c.ro1);
  }
}

// Transposed operands. Half-tile image: [64 k][128 cols] bf16, 256-B rows,
// 16-B chunk c of row r stored at c ^ (2 * gsw(r)), gsw(r) = (r & 3) | ((r >> 3) & 1) << 2.
// An MFMA fragment (8 consecutive k of one column per lane) is two
// ds_read_b64_tr_b16: in each 16-lane group, lane 4q+p addresses row k0+q,
// columns 4p..4p+3 and receives its own column over the 4 rows. Per 32-lane
// half the 8 rows {0-3, 8-11} (+4 for the second read) hit 8 distinct gsw
// values, so the 16 chunks read land on 16 distinct bank groups: no conflicts.
typedef short bf16x4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 tr_frag(const char* p) {
  const bf16x4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((KGS_LDS bf16x4s*)p);
  const bf16x4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((KGS_LDS bf16x4s*)(p + 4 * 256));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// column chunk base `ch` (even) -> byte offset of this lane's tr-read address
__device__ __forceinline__ int tr_col(const Ctx& c, int ch) { return ((ch ^ c.tr_x) << 4) + c.tr_base; }

__device__ __forceinline__ void read_a_tr(const Ctx& c, Regs& R, const char* half) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const char* p = half + tr_col(c, c.wr * 8 + 2 * i);
    R.a[i][0] = tr_frag(p);
    R.a[i][1] = tr_frag(p + 32 * 256);
  }
}

template <int NH>
__device__ __forceinline__ void read_b_tr(const Ctx& c, Regs& R, const char* half) {
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const char* p = half + tr_col(c, c.wc * 4 + 2 * n);
    R.b[NH][n][0] = tr_frag(p);
    R.b[NH][n][1] = tr_frag(p + 32 * 256);
  }
}

// S bit 13 / 14 (timing probes, wrong results): keep the transposed DMA but read
// with ds_read_b128 (13), or keep the tr reads but DMA in the NT pattern (14)
template <int S>
__device__ __forceinline__ void rd_a(const Ctx& c, Regs& R, const char* half) {
  if constexpr ((S & 2048) && !(S & 8192)) read_a_tr(c, R, half); else read_a(c, R, half);
}

template <int NH, int S>
__device__ __forceinline__ void rd_b(const Ctx& c, Regs& R, const char* half) {
  if constexpr (S & 4096) read_b_tr<NH>(c, R, half); else read_b<NH>(c, R, half);
}

template <int PART, int S>
__device__ __forceinline__ void issue_s(const Ctx& c, int buf, int k0, bool nxt = false) {
  constexpr bool isA = PART == P_A0 || PART == P_A1;
  constexpr bool tr = (S & 16384) ? false : isA ? (S & 2048) != 0 : (S & 4096) != 0;
  issue<PART, (S & 512) != 0, tr>(c, buf, k0, nxt);
}

typedef int i32x8 __attribute__((ext_vector_type(8)));

// Two 16-B fragments (k-sub 0 and 1 of the same 128-byte LDS row slice) as one
// 32-B operand of the fp8 MFMA.
__device__ __forceinline__ i32x8 cat32(const bf16x8& lo, const bf16x8& hi) {
  typedef short s16 __attribute__((ext_vector_type(16)));
  s16 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  return __builtin_bit_cast(i32x8, v);
}

template <int MH, int NH, bool FP8 = false>
__device__ __forceinline__ void mma_quadrant(Regs& R) {
  if constexpr (FP8) {
    // fp8 (OCP e4m3) mode: the LDS rows hold 128 fp8 K-values; one scaled
    // 16x16x128 MFMA (unit E8M0 scales = 2^0) consumes what the bf16 path does
    // in two 16x16x32 ones -- twice the FLOPs for the same bytes moved. Lane
    // group g holds K-bytes [16g,16g+16) and [64+16g,64+16g+16) of its row, for
    // A and B alike, so the K pairing is consistent (the sum is order-free).
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        R.acc[MH][i][NH][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            cat32(R.b[NH][n][0], R.b[NH][n][1]), cat32(R.a[i][0], R.a[i][1]), R.acc[MH][i][NH][n], 0, 0, 0, 127,
            0, 127);
    return;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        // operands swapped (B first) so each lane ends up holding 4
        // consecutive output COLUMNS of one row: C[m = lane&15][n = 4*(lane>>4)+e]
        R.acc[MH][i][NH][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            R.b[NH][n][s], R.a[i][s], R.acc[MH][i][NH][n], 0, 0, 0);
}

// Two schedules (template S):
//  S=0  quadrants (0,0)(0,1)(1,1)(1,0); stream A0,B0,B1,A1; look-ahead 5;
//       ds_reads per phase 12/4/8/0; vmcnt(6).
//  S=1  quadrants (0,0)(0,1)(1,0)(1,1); stream B0,A0,B1,A1; look-ahead 7;
//       B0 of the NEXT K-tile is read in phase 3 (its last use is now phase 2),
//       so reads per phase are 8/4/8/4 and no partner MFMA block waits on a
//       12-read burst; 5 half-tiles stay in flight (vmcnt(10)).
//       Hazards (half-tile (t,pos) issued at phase 4t+pos-7, every read at
//       distance 6 from its issue, every slot re-issued 2 phases after its last
//       read): RAW needs distance >= 6 for vmcnt(10); WAR needs >= 2 with the
//       one-barrier stagger -- both hold for all four slots.
template <int QP, int S>
__device__ __forceinline__ void phase(const Ctx& c, Regs& R, int it) {
  constexpr int q = QP & 3;
  constexpr int cbuf = QP >> 2;
  const char* buf = c.smem + cbuf * BUF_BYTES;
  if constexpr ((S & 1) == 0) {
    if constexpr (q == 0) {
      rd_a<S>(c, R, buf + P_A0 * HALF_BYTES);
      rd_b<0, S>(c, R, buf + P_B0 * HALF_BYTES);
    } else if constexpr (q == 1) {
      rd_b<1, S>(c, R, buf + P_B1 * HALF_BYTES);
    } else if constexpr (q == 2) {
      rd_a<S>(c, R, buf + P_A1 * HALF_BYTES);
    }
  } else {
    if constexpr (q == 0) rd_a<S>(c, R, buf + P_A0 * HALF_BYTES);
    if constexpr (q == 1) rd_b<1, S>(c, R, buf + P_B1 * HALF_BYTES);
    if constexpr (q == 2) rd_a<S>(c, R, buf + P_A1 * HALF_BYTES);
    if constexpr (q == 3) rd_b<0, S>(c, R, c.smem + (cbuf ^ 1) * BUF_BYTES + P_B0 * HALF_BYTES);
  }
  // prefetch half-tile h = 8*it + QP + look-ahead
  constexpr int LA = (S & 1) == 0 ? LOOKAHEAD : 7;
  constexpr int hoff = QP + LA;
  constexpr int toff = hoff >> 2;
  constexpr int jp = hoff & 3;
  constexpr int part = (S & 1) == 0 ? (jp == 0 ? P_A0 : jp == 1 ? P_B0 : jp == 2 ? P_B1 : P_A1)
                                    : (jp == 0 ? P_B0 : jp == 1 ? P_A0 : jp == 2 ? P_B1 : P_A1);
  int t = 2 * it + toff;
  if constexpr (S & 32768) {
    // persistent: past the end the stream continues into the next tile's first
    // K-tiles (same slots, same parity: nt is even), so the pipeline never drains
    if (t >= c.nt && c.has_next) {
      issue_s<part, S>(c, toff & 1, (t - c.nt) * BK, true);
    } else {
      t = t < c.nt ? t : c.nt - 1;
      issue_s<part, S>(c, toff & 1, t * BK);
    }
  } else {
    t = t < c.nt ? t : c.nt - 1;  // past the end: harmless re-load of the last tile
    issue_s<part, S>(c, toff & 1, t * BK);
  }
  if constexpr ((S & 1) == 0)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  bar();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (!(S & 2)) __builtin_amdgcn_s_setprio(1);
  if constexpr (S & 16) {  // timing experiment only: twice the MFMAs per phase (wrong results)
    if constexpr (q == 0) mma_quadrant<0, 0, (S & 1024) != 0>(R);
    if constexpr (q == 1) mma_quadrant<0, 1, (S & 1024) != 0>(R);
    if constexpr (q == 2) mma_quadrant<1, 0, (S & 1024) != 0>(R);
    if constexpr (q == 3) mma_quadrant<1, 1, (S & 1024) != 0>(R);
  }
  if constexpr (q == 0) mma_quadrant<0, 0, (S & 1024) != 0>(R);
  if constexpr (q == 1) mma_quadrant<0, 1, (S & 1024) != 0>(R);
  if constexpr (q == 2) {
    if constexpr ((S & 1) == 0) mma_quadrant<1, 1, (S & 1024) != 0>(R); else mma_quadrant<1, 0, (S & 1024) != 0>(R);
  }
  if constexpr (q == 3) {
    if constexpr ((S & 1) == 0) mma_quadrant<1, 0, (S & 1024) != 0>(R); else mma_quadrant<1, 1, (S & 1024) != 0>(R);
  }
  if constexpr (!(S & 2)) __builtin_amdgcn_s_setprio(0);
  // S bit 7 (with bit 6, lockstep): one barrier per phase. Still race-free: the
  // slot a phase's DMA overwrites was last read >= 2 phases earlier, i.e. before
  // the previous phase's barrier on every wave.
  if constexpr (!(S & 128)) bar();
}

// Epilogue: lane holds C[row][col..col+3] for every (mh, i, nh, n); bias and
// activation fused, bf16 out through the widened (16-B) store tail.
template <int EPI, int S>
__device__ __forceinline__ void store_tile(const Ctx& c, const Regs& R, unsigned short* __restrict__ C,
                                           const unsigned short* __restrict__ bias, int M, int N, int ldc,
                                           float alpha, int tm, int tn, int lane) {
  constexpr bool BND = (S & 512) != 0;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = tm * BM + mh * 128 + c.wr * 64 + i * 16 + fr;
      unsigned short* crow = C + (long)row * ldc;
      // bounded mode: rows past M are dropped (the permlane swaps below stay
      // wave-uniform, only the stores are predicated)
      const bool row_ok = !BND || row < M;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        uint2 o[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int col = tn * BN + nh * 128 + c.wc * 32 + n * 16 + fq * 4;
          f32x4 v = R.acc[mh][i][nh][n];
          if constexpr (S & 1024) v *= alpha;  // fp8: per-tensor dequant scale sa*sb
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI != EPI_NONE) {
            if (!BND || col + 4 <= N) {
              bf16x4 bb = *(const bf16x4*)(bias + col);
#pragma unroll
              for (int e = 0; e < 4; ++e) bv[e] = bf2f((unsigned short)bb[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) bv[e] = col + e < N ? bf2f(bias[col + e]) : 0.f;
            }
          }
          o[n].x = pack_bf16x2(epilogue<EPI>(v[0], bv[0]), epilogue<EPI>(v[1], bv[1]));
          o[n].y = pack_bf16x2(epilogue<EPI>(v[2], bv[2]), epilogue<EPI>(v[3], bv[3]));
        }
        const int col0 = tn * BN + nh * 128 + c.wc * 32;
        if constexpr (S & 256) {
          // narrow store tail (A/B reference): two 8-B stores per lane
          *(uint2*)(crow + col0 + fq * 4) = o[0];
          *(uint2*)(crow + col0 + 16 + fq * 4) = o[1];
        } else {
          // widened store tail (guide T21, 16-lane form): v_permlane16_swap
          // exchanges rows 1<->0 and 3<->2 of the lane grid, so even-fq lanes
          // end up with 8 consecutive n=0 columns and odd-fq lanes with the
          // matching n=1 columns -> one 16-B store per lane instead of two 8-B.
          auto sx = __builtin_amdgcn_permlane16_swap(o[0].x, o[1].x, false, false);
          auto sy = __builtin_amdgcn_permlane16_swap(o[0].y, o[1].y, false, false);
          // even fq: (own n0, partner n0) = (sx[0], sx[1]) ... odd fq likewise for n1
          const uint4 q = make_uint4(sx[0], sy[0], sx[1], sy[1]);
          const int cw = col0 + (fq & 1) * 16 + (fq >> 1) * 8;
          if (!BND || (row_ok && cw + 8 <= N)) {
            *(uint4*)(crow + cw) = q;
          } else if (row_ok) {
            const unsigned wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (cw + e < N) crow[cw + e] = (unsigned short)(wd[e >> 1] >> ((e & 1) * 16));
          }
        }
      }
    }
}

template <int EPI, int S>
__global__ __launch_bounds__(512) void gemm_nt_256(const unsigned short* __restrict__ A,
                                                   const unsigned short* __restrict__ B,
                                                   unsigned short* __restrict__ C,
                                                   const unsigned short* __restrict__ bias,
                                                   int M, int N, int K, int lda, int ldb, int ldc,
                                                   float alpha) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  constexpr bool BND = (S & 512) != 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = BND ? (M + BM - 1) / BM : M / BM, ntn = BND ? (N + BN - 1) / BN : N / BN, nwg = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  // S bits 2-3 select the tile-group height (experiment knob): 8, 4, 16, 2
  constexpr int GM = ((S >> 2) & 3) == 0 ? GROUP_M : ((S >> 2) & 3) == 1 ? 4 : ((S >> 2) & 3) == 2 ? 16 : 2;
  const int per_group = GM * ntn;
  const int group = wg / per_group;
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  const int tm = first_m + (wg % per_group) % gsz;
  const int tn = (wg % per_group) / gsz;

  Ctx c;
  c.smem = smem;
  // S bit 5: timing probe -- every block loads tile (0,0) (L2-resident operands)
  c.Ag = ((S & 2048) && !(S & 16384)) ? A + (long)tm * BM : A + (long)((S & 32) ? 0 : tm) * BM * lda;
  c.Bg = (S & 4096) ? B + (long)tn * BN : B + (long)((S & 32) ? 0 : tn) * BN * ldb;
  c.a_kstride = lda;
  c.b_kstride = ldb;
  c.a_half = 128L * lda;
  c.b_half = 128L * ldb;
  c.w = w;
  c.wr = w >> 2;
  c.wc = w & 3;
  c.nt = K / BK;
  if constexpr (BND) {
    c.nt = (((K + BK - 1) / BK) + 1) & ~1;  // whole K-loop iterations; tail tiles load zeros
    c.K = K;
    c.a_half_i = 128 * lda;
    c.b_half_i = 128 * ldb;
    const int rows_a = min(M - tm * BM, BM), rows_b = min(N - tn * BN, BN);
    c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)c.Ag, 0, rows_a * lda * 2, 0x00020000);
    c.rb = __builtin_amdgcn_make_buffer_rsrc((void*)c.Bg, 0, rows_b * ldb * 2, 0x00020000);
  }
  {
    // glds j (0/1) of wave w fills half-tile rows w*16 + j*8 + lane/8; lane's
    // physical 16-B chunk is lane&7 and holds logical chunk (lane&7)^f(row).
    const int r0 = w * 16 + (lane >> 3), r1 = r0 + 8;
    const int c0 = (lane & 7) ^ ((r0 >> 1) & 7);
    const int c1 = (lane & 7) ^ ((r1 >> 1) & 7);
    c.offA0 = r0 * lda + c0 * 8;
    c.offA1 = r1 * lda + c1 * 8;
    c.offB0 = r0 * ldb + c0 * 8;
    c.offB1 = r1 * ldb + c1 * 8;
    c.kc0 = c0 * 8;
    c.kc1 = c1 * 8;
    if constexpr ((S & 2048) || (S & 4096)) {
      // [64 k][128 col] half-tiles: glds j of wave w fills rows 4*(2w+j) + lane/16;
      // lane's physical chunk lane&15 holds logical chunk (lane&15) ^ (2 gsw(row))
      const int tr0 = 4 * (2 * w) + (lane >> 4), tr1 = tr0 + 4;
      const int g0 = (tr0 & 3) | (((tr0 >> 3) & 1) << 2), g1 = (tr1 & 3) | (((tr1 >> 3) & 1) << 2);
      const int lc0 = (lane & 15) ^ (2 * g0), lc1 = (lane & 15) ^ (2 * g1);
      if constexpr ((S & 2048) && !(S & 16384)) {
        c.offA0 = tr0 * lda + lc0 * 8;
        c.offA1 = tr1 * lda + lc1 * 8;
      }
      if constexpr (S & 4096) {
        c.offB0 = tr0 * ldb + lc0 * 8;
        c.offB1 = tr1 * ldb + lc1 * 8;
      }
      // tr reads: 16-lane group g (= lane>>4) takes rows 8g + q (q = (lane&15)>>2)
      // and columns 4p..4p+3 (p = lane&3) of the fragment's 16-column block
      const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
      c.tr_x = 2 * (q | ((g & 1) << 2));
      c.tr_base = (8 * g + q) * 256 + (pp >> 1) * 16 + (pp & 1) * 8;
    }
    // fragment read: row lane&15, logical chunk 4*s + lane/16
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

  const int k1 = (c.nt > 1 ? 1 : 0) * BK;
  if constexpr ((S & 1) == 0) {
    // prologue: half-tiles 0..4 = A0 B0 B1 A1 of tile 0, A0 of tile 1
    issue_s<P_A0, S>(c, 0, 0);
    issue_s<P_B0, S>(c, 0, 0);
    issue_s<P_B1, S>(c, 0, 0);
    issue_s<P_A1, S>(c, 0, 0);
    issue_s<P_A0, S>(c, 1, k1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A0,B0 of tile 0 landed
    bar();
  } else {
    // prologue: half-tiles 0..6 = B0 A0 B1 A1 of tile 0, B0 A0 B1 of tile 1
    issue_s<P_B0, S>(c, 0, 0);
    issue_s<P_A0, S>(c, 0, 0);
    issue_s<P_B1, S>(c, 0, 0);
    issue_s<P_A1, S>(c, 0, 0);
    issue_s<P_B0, S>(c, 1, k1);
    issue_s<P_A0, S>(c, 1, k1);
    issue_s<P_B1, S>(c, 1, k1);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // B0,A0 of tile 0 landed
    bar();
    rd_b<0, S>(c, R, smem + P_B0 * HALF_BYTES);  // phase 0 reads A0 itself
  }
  // stagger: waves 4-7 trail by one barrier (S bit 6: lockstep experiment, no stagger)
  if (!(S & 64) && c.wr == 1) bar();

  const int iters = c.nt >> 1;
  for (int it = 0; it < iters; ++it) {
    phase<0, S>(c, R, it);
    phase<1, S>(c, R, it);
    phase<2, S>(c, R, it);
    phase<3, S>(c, R, it);
    phase<4, S>(c, R, it);
    phase<5, S>(c, R, it);
    phase<6, S>(c, R, it);
    phase<7, S>(c, R, it);
  }
  if (!(S & 64) && c.wr == 0) bar();  // balance the stagger barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain tail prefetches

  store_tile<EPI, S>(c, R, C, bias, M, N, ldc, alpha, tm, tn, lane);
}

// Persistent variant (S bit 15, balanced schedule, aligned shapes): one block
// per CU walks tiles vb = blockIdx.x, +gridDim.x, ... in the same XCD-remapped,
// grouped order the one-shot grid would run them. The look-ahead DMA of a
// tile's last phases already fetches the next tile's first 7 half-tiles and
// B0(0) fragments, so the next tile's loads are in flight while this tile's
// epilogue stores drain; the wave groups keep their one-barrier stagger across
// tiles. RAW/WAR accounting is unchanged: the half-tile stream is simply
// continuous across tile boundaries.
__device__ __forceinline__ void tile_coords(int vb, int nwg, int ntm, int ntn, int& tm, int& tn) {
  const int wg = xcd_remap(vb, nwg);
  constexpr int GM = 4;
  const int per_group = GM * ntn;
  const int group = wg / per_group;
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  tm = first_m + (wg % per_group) % gsz;
  tn = (wg % per_group) / gsz;
}

template <int EPI, int S>
__global__ __launch_bounds__(512) void gemm_nt_256_persist(const unsigned short* __restrict__ A,
                                                           const unsigned short* __restrict__ B,
                                                           unsigned short* __restrict__ C,
                                                           const unsigned short* __restrict__ bias,
                                                           int M, int N, int K, int lda, int ldb, int ldc,
                                                           float alpha) {
  static_assert((S & 1) && (S & 32768) && !(S & 512) && !(S & (2048 | 4096)), "persistent: aligned NT only");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  int vb = blockIdx.x;
  int tm, tn;
  tile_coords(vb, nwg, ntm, ntn, tm, tn);

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
  int vb2 = vb + gridDim.x;
  c.has_next = vb2 < nwg;
  int tm2 = 0, tn2 = 0;
  if (c.has_next) tile_coords(vb2, nwg, ntm, ntn, tm2, tn2);
  c.Ag2 = A + (long)tm2 * BM * lda;
  c.Bg2 = B + (long)tn2 * BN * ldb;

  Regs R;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int n = 0; n < 2; ++n) R.acc[a][i][b][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int k1 = (c.nt > 1 ? 1 : 0) * BK;
  issue<P_B0>(c, 0, 0);
  issue<P_A0>(c, 0, 0);
  issue<P_B1>(c, 0, 0);
  issue<P_A1>(c, 0, 0);
  issue<P_B0>(c, 1, k1);
  issue<P_A0>(c, 1, k1);
  issue<P_B1>(c, 1, k1);
  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  bar();
  read_b<0>(c, R, smem + P_B0 * HALF_BYTES);
  if (c.wr == 1) bar();

  const int iters = c.nt >> 1;
  for (;;) {
    for (int it = 0; it < iters; ++it) {
      phase<0, S>(c, R, it);
      phase<1, S>(c, R, it);
      phase<2, S>(c, R, it);
      phase<3, S>(c, R, it);
      phase<4, S>(c, R, it);
      phase<5, S>(c, R, it);
      phase<6, S>(c, R, it);
      phase<7, S>(c, R, it);
    }
    store_tile<EPI, S>(c, R, C, bias, M, N, ldc, alpha, tm, tn, lane);
    if (!c.has_next) break;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int n = 0; n < 2; ++n) R.acc[a][i][b][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    tm = tm2;
    tn = tn2;
    c.Ag = c.Ag2;
    c.Bg = c.Bg2;
    vb2 += gridDim.x;
    c.has_next = vb2 < nwg;
    if (c.has_next) {
      tile_coords(vb2, nwg, ntm, ntn, tm2, tn2);
      c.Ag2 = A + (long)tm2 * BM * lda;
      c.Bg2 = B + (long)tn2 * BN * ldb;
    }
  }
  if (c.wr == 0) bar();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace g256

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

template <int EPI>
static hipError_t launch(int variant, const unsigned short* A, const unsigned short* B, unsigned short* C,
                         const unsigned short* bias, int M, int N, int K, int lda, int ldb, int ldc,
                         hipStream_t s) {
  // S: bit0 schedule (1 = balanced 8/4/8/4 reads, look-ahead 7), bit1 no
  // s_setprio, bits2-3 GROUP_M (0:8 1:4 2:16 3:2). Production = 7 (measured
  // best at 4096^3..16384^2x8192 in interleaved A/B, profiles/gemm_tuning.md).
  const dim3 grid256((M / g256::BM) * (N / g256::BN));
  if (variant == 1) {
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb,
                       ldc, 1.0f);
  } else if (variant == 20) {
    // persistent: one block per CU walking the tiles (aligned shapes)
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    const int nwg = (M / g256::BM) * (N / g256::BN);
    const dim3 gridp(nwg < cus ? nwg : cus);
    hipLaunchKernelGGL((g256::gemm_nt_256_persist<EPI, 7 + 32768>), gridp, dim3(512), 0, s, A, B, C, bias, M, N, K,
                       lda, ldb, ldc, 1.0f);
  } else if (variant == 16) {
    // the same pipeline on any M, N and K % 8 == 0: buffer-resource loads zero
    // the rows / K-chunks past the edges, stores are predicated
    const dim3 gridb(((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN));
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 512>), gridb, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb,
                       ldc, 1.0f);
  } else if (variant >= 4 && variant <= 8) {
    // tuning experiments (no-epilogue only)
    if constexpr (EPI == EPI_NONE) {
      if (variant == 4)  // with s_setprio around the MFMA blocks
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 5>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f);
      if (variant == 5)  // GROUP_M 8
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 3>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f);
      if (variant == 6)  // first schedule (12/4/8/0 reads, look-ahead 5), setprio, GROUP_M 8
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 0>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f);
      if (variant == 7)  // GROUP_M 2
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 15>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f);
      if (variant == 8)  // GROUP_M 16
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 11>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                           ldb, ldc, 1.0f);
    } else {
      return hipErrorInvalidValue;
    }
  } else if (variant == 11) {
    // timing probe: production schedule, all blocks load the same (L2-resident) tiles (wrong C)
    if constexpr (EPI == EPI_NONE)
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 32>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                         ldb, ldc, 1.0f);
  } else if (variant == 15) {
    // production schedule with the narrow (2 x 8-B per lane) store tail, for A/B
    if constexpr (EPI == EPI_NONE)
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 256>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                         ldb, ldc, 1.0f);
  } else if (variant == 14) {
    hipLaunchKernelGGL(gpl::gemm_nt_256pl<EPI>, grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else if (variant == 12 || variant == 13) {
    // lockstep experiments: no ping-pong stagger (12), and with one barrier per phase (13)
    if constexpr (EPI == EPI_NONE) {
      if (variant == 12)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 64>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K,
                           lda, ldb, ldc, 1.0f);
      else
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 64 + 128>), grid256, dim3(512), 0, s, A, B, C, bias, M, N,
                           K, lda, ldb, ldc, 1.0f);
    }
  } else if (variant == 10) {
    hipLaunchKernelGGL(g32::gemm_nt_256p32<EPI>, grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else if (variant == 9) {
    // timing probe: production schedule with every MFMA block doubled (wrong C)
    if constexpr (EPI == EPI_NONE) {
      hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 16>), grid256, dim3(512), 0, s, A, B, C, bias, M, N, K, lda,
                         ldb, ldc, 1.0f);
    } else {
      return hipErrorInvalidValue;
    }
  } else if (variant == 3) {
    dim3 grid((M / g4::BM) * (N / g4::BN));
    hipLaunchKernelGGL(g4::gemm_nt_256w4<EPI>, grid, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc);
  } else {
    const int vec_ok = ((lda % 8) == 0 && (ldb % 8) == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0);
    dim3 grid((N + gen::BN - 1) / gen::BN, (M + gen::BM - 1) / gen::BM);
    hipLaunchKernelGGL(gen::gemm_nt_generic<EPI>, grid, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                       vec_ok);
  }
  return hipGetLastError();
}

}  // namespace kgs

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

// variant: 0 = auto, 1 = force 256x256 8-wave ping-pong, 2 = force generic,
//          3 = force 256x256 4-wave (both pipelined variants need the same eligibility).
KGS_EXPORT int kgs_gemm_bf16_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                                int ldb, int ldc, int epi, int variant, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (epi != kgs::EPI_NONE && bias == nullptr) return KGS_ERR_ARG;
  // the fast epilogue reads the bias 4 elements (8 B) at a time
  const int bias_ok = epi == kgs::EPI_NONE || (uintptr_t)bias % 8 == 0;
  const int fast = kgs_gemm_bf16_nt_fast_ok(A, B, C, M, N, K, lda, ldb, ldc) && bias_ok;
  const int bounded = kgs_gemm_bf16_nt_bounded_ok(A, B, C, M, N, K, lda, ldb, ldc) && bias_ok;
  int v;
  if (variant == 0) v = fast ? 1 : bounded ? 16 : 2;
  else if (variant == 16) { if (!bounded) return KGS_ERR_ALIGN; v = 16; }
  else if (variant == 1) { if (!fast) return KGS_ERR_ALIGN; v = 1; }
  else if (variant == 2) v = 2;
  else if ((variant >= 3 && variant <= 15) || variant == 20) { if (!fast) return KGS_ERR_ALIGN; v = variant; }
  else return KGS_ERR_ARG;
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
namespace {

template <int EPI>
hipError_t launch_fp8(int v, const unsigned short* A, const unsigned short* B, unsigned short* C,
                      const unsigned short* bias, int M, int N, int Kw, int ldaw, int ldbw, int ldc, float alpha,
                      hipStream_t s) {
  using namespace kgs;
  const dim3 grid_al((M / g256::BM) * (N / g256::BN));
  if (v == 1) {
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 1024>), grid_al, dim3(512), 0, s, A, B, C, bias, M, N, Kw, ldaw,
                       ldbw, ldc, alpha);
  } else if (v >= 17 && v <= 19) {
    // tile-group height experiments for fp8 (aligned shapes): GROUP_M 8 / 16 / 2
    if constexpr (EPI == EPI_NONE) {
      if (v == 17)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 3 + 1024>), grid_al, dim3(512), 0, s, A, B, C, bias, M, N, Kw,
                           ldaw, ldbw, ldc, alpha);
      if (v == 18)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 11 + 1024>), grid_al, dim3(512), 0, s, A, B, C, bias, M, N, Kw,
                           ldaw, ldbw, ldc, alpha);
      if (v == 19)
        hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 15 + 1024>), grid_al, dim3(512), 0, s, A, B, C, bias, M, N, Kw,
                           ldaw, ldbw, ldc, alpha);
    }
  } else {
    const dim3 grid(((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN));
    hipLaunchKernelGGL((g256::gemm_nt_256<EPI, 7 + 512 + 1024>), grid, dim3(512), 0, s, A, B, C, bias, M, N, Kw,
                       ldaw, ldbw, ldc, alpha);
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

KGS_EXPORT int kgs_gemm_fp8_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                               int ldb, int ldc, float alpha, int epi, int variant, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return KGS_ERR_SHAPE;
  if (lda < K || ldb < K || ldc < N) return KGS_ERR_SHAPE;
  if (epi != kgs::EPI_NONE && (bias == nullptr || (uintptr_t)bias % 8)) return KGS_ERR_ARG;
  const int fast = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 0);
  const int bounded = kgs_gemm_fp8_nt_ok(A, B, C, M, N, K, lda, ldb, ldc, 1);
  int v;
  if (variant == 0) v = fast ? 1 : 16;
  else if (variant == 1 || variant == 16 || (variant >= 17 && variant <= 19)) v = variant;
  else return KGS_ERR_ARG;
  if (!(v == 16 ? bounded : fast)) return KGS_ERR_ALIGN;
  auto a = (const unsigned short*)A;
  auto b = (const unsigned short*)B;
  auto c = (unsigned short*)C;
  auto bb = (const unsigned short*)bias;
  const int Kw = K / 2, ldaw = lda / 2, ldbw = ldb / 2;  // fp8 rows as 16-bit words
  hipError_t e;
  switch (epi) {
    case kgs::EPI_NONE: e = launch_fp8<kgs::EPI_NONE>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, stream); break;
    case kgs::EPI_BIAS: e = launch_fp8<kgs::EPI_BIAS>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, stream); break;
    case kgs::EPI_BIAS_GELU:
      e = launch_fp8<kgs::EPI_BIAS_GELU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, stream);
      break;
    case kgs::EPI_BIAS_RELU:
      e = launch_fp8<kgs::EPI_BIAS_RELU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, stream);
      break;
    case kgs::EPI_BIAS_SILU:
      e = launch_fp8<kgs::EPI_BIAS_SILU>(v, a, b, c, bb, M, N, Kw, ldaw, ldbw, ldc, alpha, stream);
      break;
    default: return KGS_ERR_ARG;
  }
  return (int)e;
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
                     1.0f);
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
