// Decode-path kernels for gfx950: the memory-bound half of LLM serving (one new
// token per sequence per step), written around layouts chosen for the MFMA
// operand maps so that every hot load is a contiguous 1 KB wave access.
//
//   * skinny GEMM   y[M, N] = x[M, K] . W[N, K]^T for a decode batch M <= 256.
//                   W is PREPACKED once (kgs/ops/decode.py pack_weight) into
//                   16-row x 32-k MFMA A-fragments: [N/16][K/32][64 lanes][8],
//                   so a wave streams its rows as back-to-back 1 KB loads
//                   straight into registers (no LDS round trip for the weight
//                   bytes). x (small, L2-resident) is staged through LDS in
//                   fragment order, read from global in whole rows, and shared
//                   by the 4 waves of a workgroup. Split-K across workgroups
//                   when N alone cannot fill 256 CUs: the last workgroup of a
//                   strip (agent-scope release/acquire ticket) reduces the fp32
//                   slabs and writes bf16 -- one launch, graph-capturable.
//   * rope_cache    rotate-half RoPE on the q and k heads of a fused QKV row and
//                   scatter k, v into the paged KV cache (one launch for both).
//   * paged decode attention: one wave per (sequence, KV head, context split);
//                   the GQA group's query heads are the 16 columns of
//                   S^T = K . Q^T (v_mfma_f32_16x16x32_bf16) and O^T = V^T . P^T
//                   takes the S^T accumulator as its B operand with no lane
//                   movement. The cache page layout is the MFMA fragment order
//                   itself (kv_k_index / kv_v_index) -- 16 contiguous 1 KB loads
//                   per 32-token page -- and context splits are merged
//                   (log-sum-exp) by the split that finishes last, in-launch.
#include "kgs_common.h"

#include <type_traits>

namespace kgs {
namespace dec {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int HD = 128;                // head_dim
constexpr int PAGE = 32;               // tokens per KV-cache page
constexpr int PAGE_ELEMS = PAGE * HD;  // per (page, kv head, K|V): 4096 bf16 = 8 KB

// --- KV cache page layout (per page, per kv head: K region then V region) ---
// K (token tau, dim d): S^T = K.Q^T A-fragments, 16-token halves t, k-steps ks
__host__ __device__ __forceinline__ int kv_k_index(int tau, int d) {
  const int t = tau >> 4, r = tau & 15, ks = d >> 5, g = (d >> 3) & 3, j = d & 7;
  return (((t * 4 + ks) * 64) + g * 16 + r) * 8 + j;
}
// V (token tau, dim d): O^T = V^T.P^T A-fragments, 16-dim tiles dt; the k
// (token) order within a fragment is the order S^T's accumulator hands P over:
// lane group g holds tokens {4g..4g+3} of half 0 then {16+4g..16+4g+3}.
__host__ __device__ __forceinline__ int kv_v_index(int tau, int d) {
  const int dt = d >> 4, m = d & 15, g = (tau >> 2) & 3, j = (tau & 3) + 4 * (tau >> 4);
  return ((dt * 64) + g * 16 + m) * 8 + j;
}

// over the four 16-lane rows (lanes of one column), on the permlane swaps
__device__ __forceinline__ float wmax16(float v) { return xor32_max(xor16_max(v)); }
__device__ __forceinline__ float wsum16(float v) { return xor32_sum(xor16_sum(v)); }

// In-launch hand-offs (split-K slabs, attention split partials): producers store
// WRITE-THROUGH (sc1 buffer stores) and drain, so they need no release fence (a
// release is a buffer_wbl2 of the whole XCD L2 per wave: decode attention ran
// 8x slower with one per split); the single consumer (last arriver) takes ONE
// agent-scope acquire before reading -- without it a reader on another XCD sees
// stale lines of a reused workspace (measured: wrong merges whenever splits
// landed on different XCDs). cdna_hip_programming.md Guideline 16, recipe R1.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}
__device__ __forceinline__ f32x4v ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ void st1_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, float a) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, a), r, off, 0, 16);
}
__device__ __forceinline__ float ld1_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}

// ---------------------------------------------------------------------------
// skinny GEMM
// ---------------------------------------------------------------------------
// Workgroup = 4 waves = a strip of 64*R rows of W (wave w: 16-row tiles
// (strip*4 + w)*R .. +R-1) x all Mp = 16*MT columns, over one K range.
// x chunk per stage: KC k-steps of 32 x Mp rows, double buffered in LDS. The
// next chunk's x loads are issued a whole chunk (16 k-steps, ~2 us of weight
// streaming) before they are needed -- shorter distances stall on L2 latency
// (measured: KC 4 at Mp 64 ran 1.4x slower); W fragments stream through a
// register ring PF k-steps deep. Mp > 64 keeps KC 2 (VGPR-bound; the serving
// engine routes those batches to hipBLASLt, profiles/decode_kernels.md).
template <int MT, int KC_>
struct SkinnyCfg {
  static constexpr int KC = KC_;                    // k-steps per x chunk
  static constexpr int CHUNK_SLOTS = KC * MT * 64;  // 16-B slots per chunk
  static constexpr int LOADS = CHUNK_SLOTS / 256;   // per thread per chunk
};

// Fused epilogues (runtime flags in SkinnyEpi::mode, uniform per launch):
//   EPI_SWIGLU  W is the fused gate|up weight packed so that 16-row tile t holds
//               gate rows 8t..8t+7 then up rows 8t..8t+7 (kgs/ops/decode.py
//               pack_swiglu); lane l (gate) pairs with lane l ^ 32 (up) and
//               writes silu(g) * u, so y is [M, N/2].
//   EPI_RMS     RMSNorm folded into the GEMM: x is the raw residual stream,
//               the norm weight is folded into W, and each output row m is
//               scaled by rsqrt(ss_in[m] * inv_k + eps) -- ss_in being the
//               row's sum of squares, accumulated by the producer of x.
//   EPI_RESID   residual update y[m, n] += acc (y = the residual stream, in
//               place) and ss_out[m] += sum over n of the new y^2 (fp32
//               atomics), the statistic the next EPI_RMS consumer needs.
//   ss_zero     zeroed by workgroup 0 at kernel start (the sum-of-squares
//               buffer of the previous layer boundary, already consumed).
//   EPI_ROPE    W is the fused qkv weight packed so that in every q / k head
//               16-row tile t holds dims 8t..8t+7 then 64+8t..64+8t+7
//               (kgs/ops/decode.py rope_rows): lane l pairs with lane l ^ 32,
//               rotates (rotate-half RoPE at pos[m], fp32 cos/sin tables), stores
//               the row in the original order, and writes k / v into the bf16
//               paged cache slot slot[m] -- the rope_cache launch, folded in.
// Together they remove both add_rmsnorm launches, the SwiGLU launch and the
// RoPE / KV-write launch from a decode layer (kgs/serve/model.py fused path).
enum { EPI_SWIGLU = 1, EPI_RMS = 2, EPI_RESID = 4, EPI_ROPE = 8 };
struct SkinnyEpi {
  int mode;
  const float* ss_in;
  float* ss_out;
  float* ss_zero;
  float inv_k, eps;
  const float* wscale;  // W8: per packed row dequant scale
  // EPI_ROPE
  const float* cosv;
  const float* sinv;
  const int* pos;
  const int* slot;
  unsigned short* cache;  // this layer's bf16 pages [pages][HKV][2][4096]
  int H, HKV;
};

// W8 (weight-only fp8, "W8A16"): W is OCP e4m3 in the same fragment order, 8 B
// per lane per fragment (512 B wave loads: half the HBM bytes), dequantised to
// bf16 in registers (v_cvt_pk_f32_fp8, times the lane's row scale, RNE to
// bf16); x, the MFMA and every epilogue stay bf16/fp32.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <bool W8>
using WFrag = typename std::conditional<W8, u32x2, bf16x8>::type;

// 8 floats -> 8 OCP e4m3 bytes (saturating at +-448, RNE)
__device__ __forceinline__ uint2 tfm_e4m3x8(const float* v) {
  float c[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) c[e] = fminf(fmaxf(v[e], -448.f), 448.f);
  unsigned lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  unsigned hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return make_uint2(lo, hi);
}

__device__ __forceinline__ bf16x8 dequant8(u32x2 v, float s) {
  bf16x8 o;
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], false);  // bytes 0, 1
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], true);   // bytes 2, 3
    o[4 * w + 0] = (short)f2bf(lo[0] * s);
    o[4 * w + 1] = (short)f2bf(lo[1] * s);
    o[4 * w + 2] = (short)f2bf(hi[0] * s);
    o[4 * w + 3] = (short)f2bf(hi[1] * s);
  }
  return o;
}

// EROPE: the EPI_ROPE instantiation (qkv of the fused decode layer only, so
// the other projections keep the lean epilogue's registers); its RoPE tables,
// positions and cache slots are loaded at kernel start, under the main loop.
// KIN (batch <= 16, MT 1): the four waves share one strip of 16 R rows and
// split its K range four ways instead of each taking its own rows, so a
// 4096-row projection fills 256 CUs with no cross-workgroup split-K (the slab
// stores, the ticket and the last arriver's reduce are ~3-4 us of a 12-14 us
// batch-1 launch); the waves' partial tiles are summed through LDS. x comes
// straight from global/L2 through the W ring (no LDS staging): chunk = KC
// k-steps per wave, k_per_chunk = 4 * 32 * KC.
template <int R, int MT, int KC_, bool W8 = false, bool EROPE = false, bool KIN = false>
__global__ __launch_bounds__(256, (MT * KC_ > 32 || R * MT >= 16) ? 1 : 2) void skinny(const void* __restrict__ wpv, const unsigned short* __restrict__ x,
                                                 unsigned short* __restrict__ y, float* __restrict__ ws,
                                                 int* __restrict__ cnt, int M, int N, int K, long ldx, long ldy,
                                                 int ksplit, int chunks_per_split, SkinnyEpi ep) {
  using C = SkinnyCfg<MT, KC_>;
  constexpr int KC = C::KC;
  // W ring depth in k-steps (divides KC); fp8 fragments are half the bytes, so
  // twice the depth keeps the same bytes in flight (a 16-deep bf16 ring at
  // batch 1 measured the same per launch: the fixed launch / split-K costs, not
  // the bytes in flight, set a batch-1 launch's time)
  constexpr int PF = KC < (W8 ? 16 : 8) ? KC : (W8 ? 16 : 8);
  // the only __shared__ object (a second one can make hipcc drain vmcnt before
  // every ds_read, cdna_hip_programming.md s5 trap 4a); the split-K "last
  // arriver" flag reuses its first word after the main loop
  static_assert(!KIN || (MT == 1 && PF == KC), "KIN: batch <= 16, one ring round per chunk");
  __shared__ __attribute__((aligned(16))) bf16x8 xs[2][KIN ? 2 * R * 64 : C::CHUNK_SLOTS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nstrip = N / ((KIN ? 16 : 64) * R);
  const int strip = blockIdx.x % nstrip, split = blockIdx.x / nstrip;
  if (ep.ss_zero != nullptr && blockIdx.x == 0 && tid < M) ep.ss_zero[tid] = 0.f;
  const int nkk = K / 32;
  // k-steps (of 32) of this wave and where they start
  const int nsteps = chunks_per_split * KC;
  const int kk0 = KIN ? (split * 4 + w) * nsteps : split * nsteps;
  const int nt0 = KIN ? strip * R : (strip * 4 + w) * R;  // first 16-row tile of this wave
  const WFrag<W8>* wp = (const WFrag<W8>*)wpv;
  const WFrag<W8>* wrow[R];
  float wsc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    wrow[r] = wp + ((long)(nt0 + r) * nkk + kk0) * 64 + lane;
    wsc[r] = W8 ? ep.wscale[16 * (nt0 + r) + (lane & 15)] : 1.f;
  }
  // EROPE: per (column tile c, row tile r) the lane's 4 cos / sin values and its
  // row's cache slot, fetched now so their latency hides under the main loop
  float rcs[EROPE ? MT : 1][EROPE ? R : 1][4], rsn[EROPE ? MT : 1][EROPE ? R : 1][4];
  int rslot[EROPE ? MT : 1];
  if constexpr (EROPE) {
    const int gq = lane >> 4;
#pragma unroll
    for (int c = 0; c < MT; ++c) {
      const int mr = min(16 * c + (lane & 15), M - 1);
      const int p = ep.pos[mr];
      rslot[c] = 16 * c + (lane & 15) < M ? ep.slot[mr] : -1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int T = nt0 + r, t = T & 7;
        const int dd = gq < 2 ? 8 * t + 4 * gq : 8 * t + 4 * (gq - 2);  // dim within the rotated half
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          rcs[c][r][i] = ep.cosv[(long)p * (HD / 2) + dd + i];
          rsn[c][r][i] = ep.sinv[(long)p * (HD / 2) + dd + i];
        }
      }
    }
  }

  // x chunk staging: element e = tid + 256 i of the chunk, row-major over
  // (row m, 16-B column q) so global reads are whole-row runs; the LDS position
  // is the fragment slot ((kk*MT + ct)*64 + g*16 + r). Rows >= M re-read row
  // M-1 (their output columns are never stored).
  constexpr int QPR = KC * 4;  // 16-B columns per row per chunk
  bf16x8 xstage[C::LOADS];
  auto load_x = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int e = tid + 256 * i, m = e / QPR, q = e - m * QPR;
      const int mr = m < M ? m : M - 1;
      xstage[i] = *(const bf16x8*)(x + (long)mr * ldx + (long)(kk0 + chunk * KC) * 32 + 8 * q);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int e = tid + 256 * i, m = e / QPR, q = e - m * QPR;
      const int kk = q >> 2, g = q & 3, ct = m >> 4, r = m & 15;
      xs[buf][(kk * MT + ct) * 64 + g * 16 + r] = xstage[i];
    }
  };

  f32x4v acc[R][MT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < MT; ++c) acc[r][c] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // Every load below is unconditional (indices clamped to the last step /
  // chunk: a few redundant L2-hit reloads at the tail) so hipcc can count
  // vmcnt through the loop instead of draining the ring before each MFMA.
  WFrag<W8> wf[PF][R];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int r = 0; r < R; ++r) wf[p][r] = __builtin_nontemporal_load(wrow[r] + (long)min(p, nsteps - 1) * 64);

  if constexpr (KIN) {
    // B fragment of k-step s: lane (column m = lane & 15, k = 8 (lane >> 4) ..)
    const unsigned short* xr = x + (long)min(lane & 15, M - 1) * ldx + (long)kk0 * 32 + 8 * (lane >> 4);
    bf16x8 xf[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) xf[p] = *(const bf16x8*)(xr + p * 32);
    for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          bf16x8 wdq;
          if constexpr (W8) wdq = dequant8(wf[p][r], wsc[r]);
          else wdq = wf[p][r];
          acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wdq, xf[p], acc[r][0], 0, 0, 0);
        }
        const int sn = min(s0 + p + PF, nsteps - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) wf[p][r] = __builtin_nontemporal_load(wrow[r] + (long)sn * 64);
        xf[p] = *(const bf16x8*)(xr + sn * 32);
      }
    }
    // the four K quarters of the strip: waves 1-3 hand theirs to wave 0 (slot 0
    // of xs stays free for the split-K flag); summed in wave order
    f32x4v* red = (f32x4v*)&xs[0][1];
    if (w > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) red[((w - 1) * R + r) * 64 + lane] = acc[r][0];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        f32x4v t = acc[r][0];
#pragma unroll
        for (int v = 0; v < 3; ++v) t += red[(v * R + r) * 64 + lane];
        acc[r][0] = t;
      }
    }
  } else {
  load_x(0);
  store_x(0);
  __syncthreads();
  const int nchunks = chunks_per_split;
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    load_x(min(chunk + 1, nchunks - 1));
    const bf16x8* xb = xs[chunk & 1] + lane;
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const int p = kk % PF;
      bf16x8 wdq[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (W8) wdq[r] = dequant8(wf[p][r], wsc[r]);
        else wdq[r] = wf[p][r];
      }
#pragma unroll
      for (int c = 0; c < MT; ++c) {
        const bf16x8 bfrag = xb[(kk * MT + c) * 64];
#pragma unroll
        for (int r = 0; r < R; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wdq[r], bfrag, acc[r][c], 0, 0, 0);
      }
      const long sn = min(chunk * KC + kk + PF, nsteps - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) wf[p][r] = __builtin_nontemporal_load(wrow[r] + sn * 64);
    }
    store_x((chunk + 1) & 1);
    __syncthreads();
  }
  }  // !KIN

  // C^T tile (r, c): lane holds column m = 16c + (lane & 15), rows n = 16*(nt0+r) + 4*(lane>>4) + i
  const int g = lane >> 4, mc = lane & 15;
  // store one lane's 4 consecutive outputs; every lane of the wave calls it
  // (the SWIGLU / RESID exchanges are cross-lane)
  auto emit = [&](f32x4v v, int m, int r) {
    const int ms = m < M ? m : M - 1;
    if (ep.mode & EPI_RMS) v *= rsqrtf(ep.ss_in[ms] * ep.inv_k + ep.eps);
    if (ep.mode & EPI_SWIGLU) {
      f32x4v u;
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = lane_xor32(v[i]);
      if (m < M && g < 2) {
        f32x4v o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = v[i] / (1.0f + __expf(-v[i])) * u[i];
        uint2 pk;
        pk.x = pack_bf16x2(o[0], o[1]);
        pk.y = pack_bf16x2(o[2], o[3]);
        *(uint2*)(y + (long)m * ldy + 8 * (nt0 + r) + 4 * g) = pk;
      }
    } else if (ep.mode & EPI_RESID) {
      float sq = 0.f;
      if (m < M) {
        uint2* yp = (uint2*)(y + (long)m * ldy + 16 * (nt0 + r) + 4 * g);
        const uint2 old = *yp;
        float o[4] = {bf2f(old.x & 0xffff) + v[0], bf2f(old.x >> 16) + v[1], bf2f(old.y & 0xffff) + v[2],
                      bf2f(old.y >> 16) + v[3]};
        uint2 pk;
        pk.x = pack_bf16x2(o[0], o[1]);
        pk.y = pack_bf16x2(o[2], o[3]);
        *yp = pk;
        // statistic of the stored (bf16-rounded) values, as add_rmsnorm computes it
        const float r0 = bf2f(pk.x & 0xffff), r1 = bf2f(pk.x >> 16), r2 = bf2f(pk.y & 0xffff), r3 = bf2f(pk.y >> 16);
        sq = r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
      }
      sq = wsum16(sq);  // lanes of one column m (g = 0..3)
      if (m < M && g == 0) atomicAdd(ep.ss_out + m, sq);
    } else if (EROPE) {
      const int c = m >> 4;
      const int T = nt0 + r, hh = T >> 3, t = T & 7;  // head and 16-row tile within it
      const bool rot = hh < ep.H + ep.HKV;
      f32x4v vb, pb;  // this lane's and its partner's (lane ^ 32) values, bf16-rounded
#pragma unroll
      for (int i = 0; i < 4; ++i) vb[i] = bf2f(f2bf(v[i]));
#pragma unroll
      for (int i = 0; i < 4; ++i) pb[i] = lane_xor32(vb[i]);
      // original dim of element 0: rotated heads hold (d, d + 64) pairs in a tile
      const int d0 = rot ? (g < 2 ? 8 * t + 4 * g : 64 + 8 * t + 4 * (g - 2)) : 16 * t + 4 * g;
      if (m < M) {
        f32x4v o = vb;
        if (rot) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float cs = rcs[c][r][i], sn = rsn[c][r][i];
            o[i] = g < 2 ? rope_lo(vb[i], pb[i], cs, sn) : rope_hi(pb[i], vb[i], cs, sn);
          }
        }
        uint2 pk;
        pk.x = pack_bf16x2(o[0], o[1]);
        pk.y = pack_bf16x2(o[2], o[3]);
        *(uint2*)(y + (long)m * ldy + hh * HD + d0) = pk;
        const int sl = hh >= ep.H ? rslot[c] : -1;
        if (sl >= 0) {
          const int page = sl / PAGE, tau = sl - page * PAGE;
          const bool isv = hh >= ep.H + ep.HKV;
          const int kvh = isv ? hh - ep.H - ep.HKV : hh - ep.H;
          unsigned short* pg = ep.cache + (((long)page * ep.HKV + kvh) * 2 + (isv ? 1 : 0)) * PAGE_ELEMS;
          if (!isv) {
            *(uint2*)(pg + kv_k_index(tau, d0)) = pk;  // 4 consecutive dims: one 8-B run of the K fragment
          } else {
            pg[kv_v_index(tau, d0 + 0)] = (unsigned short)(pk.x & 0xffff);
            pg[kv_v_index(tau, d0 + 1)] = (unsigned short)(pk.x >> 16);
            pg[kv_v_index(tau, d0 + 2)] = (unsigned short)(pk.y & 0xffff);
            pg[kv_v_index(tau, d0 + 3)] = (unsigned short)(pk.y >> 16);
          }
        }
      }
    } else if (m < M) {
      uint2 pk;
      pk.x = pack_bf16x2(v[0], v[1]);
      pk.y = pack_bf16x2(v[2], v[3]);
      *(uint2*)(y + (long)m * ldy + 16 * (nt0 + r) + 4 * g) = pk;
    }
  };
  if (ksplit == 1) {
    if (KIN && w != 0) return;
#pragma unroll
    for (int c = 0; c < MT; ++c)
#pragma unroll
      for (int r = 0; r < R; ++r) emit(acc[r][c], 16 * c + mc, r);
    return;
  }
  // split-K: fp32 slabs ws[split][m][n] stored write-through (sc1); every wave
  // drains, the workgroup takes a ticket; the last arriver of the strip reads
  // every slab with sc1 loads and reduces -- no release/acquire fences.
  const long mstride = N, sstride = (long)16 * MT * N;
  const __amdgpu_buffer_rsrc_t wr = rsrc(ws, (unsigned)(ksplit * sstride * 4));
#pragma unroll
  for (int c = 0; c < MT; ++c) {
    const int m = 16 * c + mc;
    if (m < M && (!KIN || w == 0)) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int n = 16 * (nt0 + r) + 4 * g;
        st_sc1(wr, (unsigned)((split * sstride + m * mstride + n) * 4), acc[r][c]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = (int*)&xs[0][0];
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(cnt + strip, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == ksplit - 1;
    if (last) {
      __hip_atomic_store(cnt + strip, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag || (KIN && w != 0)) return;
#pragma unroll
  for (int c = 0; c < MT; ++c) {
    const int m = 16 * c + mc;
    const int ms = m < M ? m : M - 1;  // every lane joins the epilogue exchanges
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int n = 16 * (nt0 + r) + 4 * g;
      f32x4v t = f32x4v{0.f, 0.f, 0.f, 0.f};
      // four slabs' loads in flight at a time (a load-add chain pays one L2
      // round trip per slab); summed in slab order as before
      for (int sp0 = 0; sp0 < ksplit; sp0 += 4) {
        f32x4v pv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sp0 + j < ksplit) pv[j] = ld_sc1(wr, (unsigned)(((sp0 + j) * sstride + ms * mstride + n) * 4));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sp0 + j < ksplit) t += pv[j];
      }
      emit(t, m, r);
    }
  }
}

// ---------------------------------------------------------------------------
// RoPE + KV-cache write
// ---------------------------------------------------------------------------
// k / v head h (H <= h < H + 2 HKV), dims (8c.., 64+8c..) = (a, b), into cache
// slot sl (page sl / 32, offset sl % 32) in the MFMA operand order of the pages
template <bool KV8>
__device__ __forceinline__ void kv_write(void* __restrict__ cache, int sl, int h, int H, int HKV, int c, bf16x8 a,
                                         bf16x8 b) {
  const int page = sl / PAGE, tau = sl - page * PAGE;
  const bool isv = h >= H + HKV;
  const int kvh = isv ? h - H - HKV : h - H;
  const long region = (((long)page * HKV + kvh) * 2 + (isv ? 1 : 0)) * PAGE_ELEMS;
  const int d1 = 8 * c, d2 = HD / 2 + 8 * c;
  if constexpr (KV8) {
    unsigned char* pg = (unsigned char*)cache + region;
    float fa[8], fb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fa[e] = bf2f((unsigned short)a[e]);
      fb[e] = bf2f((unsigned short)b[e]);
    }
    if (!isv) {
      *(uint2*)(pg + kv_k_index(tau, d1)) = tfm_e4m3x8(fa);
      *(uint2*)(pg + kv_k_index(tau, d2)) = tfm_e4m3x8(fb);
    } else {
      const uint2 qa = tfm_e4m3x8(fa), qb = tfm_e4m3x8(fb);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pg[kv_v_index(tau, d1 + e)] = (unsigned char)(((e < 4 ? qa.x : qa.y) >> (8 * (e & 3))) & 0xff);
        pg[kv_v_index(tau, d2 + e)] = (unsigned char)(((e < 4 ? qb.x : qb.y) >> (8 * (e & 3))) & 0xff);
      }
    }
  } else {
    unsigned short* pg = (unsigned short*)cache + region;
    if (!isv) {
      *(bf16x8*)(pg + kv_k_index(tau, d1)) = a;
      *(bf16x8*)(pg + kv_k_index(tau, d2)) = b;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pg[kv_v_index(tau, d1 + e)] = (unsigned short)a[e];
        pg[kv_v_index(tau, d2 + e)] = (unsigned short)b[e];
      }
    }
  }
}

// qkv row t: [H q heads | HKV k heads | HKV v heads] x 128. Thread = (token,
// head among H + 2 HKV, chunk c < 8): q/k heads rotate dims (8c.., 64+8c..) in
// place; k and v heads are also written into page slot[t] (skipped when < 0).
// KV8: the cache holds OCP e4m3 bytes (scale 1, saturating) in the same
// element order -- a page region is 4 KB instead of 8 KB.
// SK: the projection arrives as nslice fp32 split-K partials P[s][t][nh * 128]
// (gemm_nt_w4x without its reduce); they are summed in slice order and rounded
// to bf16 exactly as kgs::splitk_reduce would, then rotated and stored to qkv
// and the cache -- one launch instead of reduce + rope_cache. NSL > 0: the
// slice count at compile time (all partial loads issued before the first add).
template <bool KV8, bool SK = false, int NSL = 0>
__global__ __launch_bounds__(256) void rope_cache(unsigned short* __restrict__ qkv, const float* __restrict__ cosv,
                                                  const float* __restrict__ sinv, const int* __restrict__ pos,
                                                  const int* __restrict__ slot, void* __restrict__ cache,
                                                  long tokens, int H, int HKV, long ld,
                                                  const float* __restrict__ P = nullptr, int nslice = 0) {
  const int nh = H + 2 * HKV;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= tokens * nh * 8) return;
  const long t = idx / (nh * 8);
  const int rem = (int)(idx - t * nh * 8);
  const int h = rem >> 3, c = rem & 7;
  unsigned short* base = qkv + t * ld + (long)h * HD + 8 * c;
  bf16x8* p1 = (bf16x8*)base;
  bf16x8* p2 = (bf16x8*)(base + HD / 2);
  // position and cache slot first: the cos/sin loads hang off pos[t], so its
  // latency overlaps the qkv / partial loads instead of following them
  const int p = pos[t];
  const int sl = slot[t];
  bf16x8 a, b;
  if constexpr (SK) {
    const long MN = tokens * nh * HD, e = t * nh * HD + (long)h * HD + 8 * c;
    f32x4 s[4];
    if constexpr (NSL > 0) {
      f32x4 ps[NSL][4];
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
        for (int q = 0; q < 4; ++q) ps[sl][q] = *(const f32x4*)(P + sl * MN + e + (q >> 1) * (HD / 2) + (q & 1) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s[q] = ps[0][q];
#pragma unroll
        for (int sl = 1; sl < NSL; ++sl) s[q] += ps[sl][q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) s[q] = *(const f32x4*)(P + e + (q >> 1) * (HD / 2) + (q & 1) * 4);
      for (int sl = 1; sl < nslice; ++sl)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] += *(const f32x4*)(P + sl * MN + e + (q >> 1) * (HD / 2) + (q & 1) * 4);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[k] = (short)f2bf(s[k >> 2][k & 3]);
      b[k] = (short)f2bf(s[2 + (k >> 2)][k & 3]);
    }
    if (h >= H + HKV) {  // v heads are not rotated: store them here
      *p1 = a;
      *p2 = b;
    }
  } else {
    a = *p1;
    b = *p2;
  }
  if (h < H + HKV) {
    const f32x4* cp = (const f32x4*)(cosv + (long)p * (HD / 2) + 8 * c);
    const f32x4* sp = (const f32x4*)(sinv + (long)p * (HD / 2) + 8 * c);
    const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
    bf16x8 o1, o2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float cs = e < 4 ? c0[e] : c1[e - 4];
      const float sn = e < 4 ? s0[e] : s1[e - 4];
      const float x1 = bf2f((unsigned short)a[e]), x2 = bf2f((unsigned short)b[e]);
      o1[e] = (short)f2bf(rope_lo(x1, x2, cs, sn));
      o2[e] = (short)f2bf(rope_hi(x1, x2, cs, sn));
    }
    *p1 = o1;
    *p2 = o2;
    a = o1;
    b = o2;
  }
  if (h < H) return;
  if (sl < 0) return;
  kv_write<KV8>(cache, sl, h, H, HKV, c, a, b);
}

// Prompt-pass form (the projection in qkv, (H + 2 HKV) % 8 == 0): thread =
// (token, group of 8 heads, chunk c). The cos / sin of (pos[t], c) are loaded
// once for the 8 heads -- the per-head form above loads them once per head, as
// many bytes again as the qkv rows, all through L1 -- and the 8 heads' 16 row
// loads are issued before the first rotation. Same arithmetic per element
// (bitwise the per-head form's result).
// VSEP: the v heads are left to v_cache_pages (below): this kernel neither
// loads nor writes them.
template <bool KV8, bool VSEP = false>
__global__ __launch_bounds__(256) void rope_cache_g8(unsigned short* __restrict__ qkv, const float* __restrict__ cosv,
                                                     const float* __restrict__ sinv, const int* __restrict__ pos,
                                                     const int* __restrict__ slot, void* __restrict__ cache,
                                                     long tokens, int H, int HKV, long ld) {
  const int ng = (H + 2 * HKV) >> 3;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= tokens * ng * 8) return;
  const long t = idx / (ng * 8);
  const int rem = (int)(idx - t * ng * 8);
  const int g = rem >> 3, c = rem & 7;
  if (VSEP && g * 8 >= H + HKV) return;  // a group of v heads only
  const int p = pos[t];
  const int sl = slot[t];
  unsigned short* base = qkv + t * ld + (long)g * 8 * HD + 8 * c;
  bf16x8 a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = *(const bf16x8*)(base + j * HD);
    b[j] = *(const bf16x8*)(base + j * HD + HD / 2);
  }
  const f32x4* cp = (const f32x4*)(cosv + (long)p * (HD / 2) + 8 * c);
  const f32x4* sp = (const f32x4*)(sinv + (long)p * (HD / 2) + 8 * c);
  const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int h = g * 8 + j;
    if (h < H + HKV) {
      bf16x8 o1, o2;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float cs = e < 4 ? c0[e] : c1[e - 4];
        const float sn = e < 4 ? s0[e] : s1[e - 4];
        const float x1 = bf2f((unsigned short)a[j][e]), x2 = bf2f((unsigned short)b[j][e]);
        o1[e] = (short)f2bf(rope_lo(x1, x2, cs, sn));
        o2[e] = (short)f2bf(rope_hi(x1, x2, cs, sn));
      }
      *(bf16x8*)(base + j * HD) = o1;
      *(bf16x8*)(base + j * HD + HD / 2) = o2;
      a[j] = o1;
      b[j] = o2;
    }
    if (h >= H && sl >= 0 && !(VSEP && h >= H + HKV)) kv_write<KV8>(cache, sl, h, H, HKV, c, a[j], b[j]);
  }
}

// The prompt pass's V rows into the paged bf16 cache, one (run of 32 tokens,
// KV head) per workgroup. The V page layout is transposed (kv_v_index: a 16-B
// chunk holds one dim of 8 tokens), so a per-token writer stores 2 bytes at a
// time. Here the run's 32 x 128 values are staged in LDS and, when its slots
// fill one page in order (a prompt written from a page boundary), written as
// the page's 512 whole chunks; any other run goes element by element, exactly
// as kv_write.
__global__ __launch_bounds__(256) void v_cache_pages(const unsigned short* __restrict__ qkv,
                                                     const int* __restrict__ slot, unsigned short* __restrict__ cache,
                                                     long tokens, int H, int HKV, long ld) {
  __shared__ unsigned short vs[PAGE][HD + 8];
  __shared__ int sl[PAGE];
  __shared__ int fast;
  const long t0 = (long)blockIdx.x * PAGE;
  const int kvh = blockIdx.y, tid = threadIdx.x;
  if (tid < PAGE) sl[tid] = t0 + tid < tokens ? slot[t0 + tid] : -1;
  for (int k = tid; k < PAGE * (HD / 8); k += 256) {
    const int r = k / (HD / 8), ch = k % (HD / 8);
    const long t = t0 + r;
    const uint4 v = t < tokens ? *(const uint4*)(qkv + t * ld + (long)(H + HKV + kvh) * HD + ch * 8)
                               : make_uint4(0, 0, 0, 0);
    *(uint4*)&vs[r][ch * 8] = v;
  }
  __syncthreads();
  if (tid == 0) {
    int ok = sl[0] >= 0 && sl[0] % PAGE == 0;
    for (int i = 1; i < PAGE && ok; ++i) ok = sl[i] == sl[0] + i;
    fast = ok;
  }
  __syncthreads();
  if (fast) {
    unsigned short* pg = cache + (((long)(sl[0] / PAGE) * HKV + kvh) * 2 + 1) * PAGE_ELEMS;
    for (int k = tid; k < PAGE_ELEMS / 8; k += 256) {  // chunk k = dt * 64 + g * 16 + m
      const int d = (k >> 6) * 16 + (k & 15), g = (k >> 4) & 3;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)vs[4 * g + (j & 3) + 16 * (j >> 2)][d];
      *(bf16x8*)(pg + k * 8) = o;
    }
  } else {
    for (int k = tid; k < PAGE * HD; k += 256) {
      const int r = k / HD, d = k % HD, s = sl[r];
      if (s < 0) continue;
      unsigned short* pg = cache + (((long)(s / PAGE) * HKV + kvh) * 2 + 1) * PAGE_ELEMS;
      pg[kv_v_index(s % PAGE, d)] = vs[r][d];
    }
  }
}

// ---------------------------------------------------------------------------
// paged decode attention
// ---------------------------------------------------------------------------
struct AttnArgs {
  const unsigned short* q;      // [B, ldq]: head h at q + h*128
  const unsigned short* cache;  // layer base: [pages][HKV][2][4096]
  const int* block_tables;      // [B, max_pages]
  const int* ctx_lens;          // [B] tokens in the cache (incl. the new one)
  unsigned short* o;            // [B, ldo]
  float* po;                    // [B, H, nsplit, 128] (nsplit > 1)
  float* pml;                   // [B, H, nsplit, 2]
  int* cnt;                     // [B * HKV] split tickets (in-launch merge), zero / re-armed
  long ldq, ldo;
  int B, H, HKV, max_pages, pages_per_split, nsplit;
  int merge;                    // nsplit > 1: 1 = last split merges in-launch, 0 = paged_reduce follows
  float sl2;                    // scale * log2(e)
  // RP (rope prologue): q / k / v arrive as nslice fp32 split-K partials of the
  // fused qkv projection, P[s][B][(H + 2 HKV) * 128]; the wave reduces, rotates
  // and caches its own (sequence, KV head) rows -- rope_cache folded in
  const float* P;
  int nslice;
  const float* cosv;            // [max_pos, 64]
  const float* sinv;
  const int* pos;               // [B]
  const int* slot;              // [B] cache slot of the new token (< 0: no write)
  void* cache_w;                // the same layer base as cache, writable
};

// store O^T[dim 16dt + 4g + i][head] * inv for the lane's head
__device__ __forceinline__ void store_o(unsigned short* op, const f32x4v* acc, float inv) {
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    uint2 pk;
    pk.x = pack_bf16x2(acc[dt][0] * inv, acc[dt][1] * inv);
    pk.y = pack_bf16x2(acc[dt][2] * inv, acc[dt][3] * inv);
    *(uint2*)(op + 16 * dt) = pk;
  }
}

// One wave per (sequence, KV head, context split). With nsplit > 1 the partial (m, l, O)
// go to a workspace and the split that arrives last (agent-scope ticket per
// (sequence, KV head)) merges them -- no separate reduction launch.
// PIPE (small grids, e.g. batch 1-16): the next page's loads are issued before
// the current page is computed. With a few dozen waves on the chip no other wave
// hides a page's HBM latency, so a split otherwise pays it once per page.
//
// RP: the rope_cache work of this (sequence, KV head) runs first, in the wave:
// lane (hs = lane / 8, c = lane % 8) takes head slot hs (G q heads, then the k
// and the v head) and dims (8c.., 64+8c..), reduces the nslice partials in
// slice order, rounds to bf16 and rotates exactly as rope_cache does. The q
// heads go to LDS (the q fragments below are read from there), k and v to the
// cache slot -- written by the split whose pages hold the new token, which
// reads them back after its own stores have drained (vmcnt(0) before that
// page's loads only; nothing on this CU has that line in L1). Every split
// rotates q for itself. RP = the slice count (2, 4 or 8): all partial loads
// are issued before the first add, next to the position / slot loads.
template <bool KV8, bool PIPE = false, int RP = 0>
__global__ __launch_bounds__(64) void paged_decode(AttnArgs a) {
  const int lane = threadIdx.x;
  const int G = a.H / a.HKV;
  int id = blockIdx.x;
  const int sp = id % a.nsplit;
  id /= a.nsplit;
  const int kvh = id % a.HKV, b = id / a.HKV;
  const int g = lane >> 4, n = lane & 15;
  const int ctx = a.ctx_lens[b];
  const int npages = (ctx + PAGE - 1) / PAGE;
  const int p0 = sp * a.pages_per_split, p1 = min(npages, p0 + a.pages_per_split);
  const int h = kvh * G + n;
  __shared__ __attribute__((aligned(16))) unsigned short qs[RP ? 6 * HD : 8];  // RP: G <= 6 (host check)

  if constexpr (RP) {
    const int hs = lane >> 3, c = lane & 7;
    if (p0 < p1 && hs < G + 2) {
      const int nh = a.H + 2 * a.HKV;
      const int hh = hs < G ? kvh * G + hs : (hs == G ? a.H + kvh : a.H + a.HKV + kvh);
      const int p = a.pos[b];
      const int sl = a.slot[b];
      const long MN = (long)a.B * nh * HD, e = (long)b * nh * HD + (long)hh * HD + 8 * c;
      f32x4 ps[RP][4];
#pragma unroll
      for (int si = 0; si < RP; ++si)
#pragma unroll
        for (int q = 0; q < 4; ++q) ps[si][q] = *(const f32x4*)(a.P + si * MN + e + (q >> 1) * (HD / 2) + (q & 1) * 4);
      f32x4 s4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s4[q] = ps[0][q];
#pragma unroll
        for (int si = 1; si < RP; ++si) s4[q] += ps[si][q];
      }
      bf16x8 ra, rb;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ra[k] = (short)f2bf(s4[k >> 2][k & 3]);
        rb[k] = (short)f2bf(s4[2 + (k >> 2)][k & 3]);
      }
      if (hs <= G) {  // q and k heads: rotate-half RoPE at position p
        const f32x4* cp = (const f32x4*)(a.cosv + (long)p * (HD / 2) + 8 * c);
        const f32x4* spp = (const f32x4*)(a.sinv + (long)p * (HD / 2) + 8 * c);
        const f32x4 c0 = cp[0], c1 = cp[1], s0 = spp[0], s1 = spp[1];
        bf16x8 o1, o2;
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) {
          const float cs = e2 < 4 ? c0[e2] : c1[e2 - 4];
          const float sn = e2 < 4 ? s0[e2] : s1[e2 - 4];
          const float x1 = bf2f((unsigned short)ra[e2]), x2 = bf2f((unsigned short)rb[e2]);
          o1[e2] = (short)f2bf(rope_lo(x1, x2, cs, sn));
          o2[e2] = (short)f2bf(rope_hi(x1, x2, cs, sn));
        }
        ra = o1;
        rb = o2;
      }
      if (hs < G) {
        *(bf16x8*)(qs + hs * HD + 8 * c) = ra;
        *(bf16x8*)(qs + hs * HD + HD / 2 + 8 * c) = rb;
      } else if (sl >= 0 && (ctx - 1) / PAGE >= p0 && (ctx - 1) / PAGE < p1) {
        kv_write<KV8>(a.cache_w, sl, hh, a.H, a.HKV, c, ra, rb);
      }
    }
    __syncthreads();  // q in LDS (the cache stores drain before the last page's loads)
  }
  const int last_page = (ctx - 1) / PAGE;  // RP: the page that holds the new token

  float m = -INFINITY, lsum = 0.f;
  f32x4v acc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) acc[dt] = f32x4v{0.f, 0.f, 0.f, 0.f};

  if (p0 < p1) {
    bf16x8 qf[4];
    if constexpr (RP) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = n < G ? *(const bf16x8*)(qs + n * HD + 8 * g + 32 * ks) : bf16x8{};
    } else {
      const unsigned short* qp = a.q + (long)b * a.ldq + (long)h * HD + 8 * g;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = n < G ? *(const bf16x8*)(qp + 32 * ks) : bf16x8{};
    }
    const int* bt = a.block_tables + (long)b * a.max_pages;
    auto load_page = [&](bf16x8 (&kf)[8], bf16x8 (&vf)[8], int pi) {
      if constexpr (RP != 0)
        if (pi == last_page) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own k / v stores landed
      const long region = ((long)bt[pi] * a.HKV + kvh) * 2 * PAGE_ELEMS;  // elements of the K region
      if constexpr (KV8) {  // e4m3 pages: 8 B per lane per fragment, dequantised in registers
        const u32x2* kp = (const u32x2*)((const unsigned char*)a.cache + region) + lane;
        u32x2 kr[8], vr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kr[i] = __builtin_nontemporal_load(kp + 64 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) vr[i] = __builtin_nontemporal_load(kp + PAGE_ELEMS / 8 + 64 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          kf[i] = dequant8(kr[i], 1.f);
          vf[i] = dequant8(vr[i], 1.f);
        }
      } else {
        const bf16x8* kp = (const bf16x8*)(a.cache + region) + lane;
#pragma unroll
        for (int i = 0; i < 8; ++i) kf[i] = __builtin_nontemporal_load(kp + 64 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) vf[i] = __builtin_nontemporal_load(kp + PAGE_ELEMS / 8 + 64 * i);
      }
    };
    auto page = [&](const bf16x8 (&kf)[8], const bf16x8 (&vf)[8], int pi) {
      f32x4v s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t * 4 + ks], qf[ks], s[t], 0, 0, 0);
      }
      // lane holds S^T[token 16t + 4g + i][head n]
      const int tok0 = pi * PAGE + 4 * g;
      float bm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = (tok0 + 16 * t + i) < ctx ? s[t][i] * a.sl2 : -INFINITY;
          s[t][i] = v;
          bm = fmaxf(bm, v);
        }
      bm = wmax16(bm);
      const float mn = fmaxf(m, bm);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      bf16x8 pf;
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(s[t][i] - mn);
          ps += p;
          pf[4 * t + i] = (short)f2bf(p);
        }
      lsum = lsum * alpha + ps;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        acc[dt] *= alpha;
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pf, acc[dt], 0, 0, 0);
      }
    };
    if constexpr (PIPE) {
      // two register sets: page pi + 1 is in flight while page pi is computed
      bf16x8 ka[8], va[8], kb[8], vb[8];
      load_page(ka, va, p0);
      for (int pi = p0; pi < p1; pi += 2) {
        if (pi + 1 < p1) load_page(kb, vb, pi + 1);
        page(ka, va, pi);
        if (pi + 1 < p1) {
          if (pi + 2 < p1) load_page(ka, va, pi + 2);
          page(kb, vb, pi + 1);
        }
      }
    } else {
      // one page at a time: the loads of other waves on the SIMD hide this one's
      // latency (a two-register-set pipeline measured slower here: 208 VGPRs cost
      // a wave of occupancy, 47 -> 59 us at batch 64 x 1024)
      for (int pi = p0; pi < p1; ++pi) {
        bf16x8 kf[8], vf[8];
        load_page(kf, vf, pi);
        page(kf, vf, pi);
      }
    }
  }
  lsum = wsum16(lsum);
  // lane holds O^T[dim 16dt + 4g + i][head n]
  unsigned short* op = a.o + (long)b * a.ldo + (long)h * HD + 4 * g;
  if (a.nsplit == 1) {
    if (n < G) store_o(op, acc, lsum > 0.f ? 1.f / lsum : 0.f);
    return;
  }
  const long row = ((long)b * a.H + h) * a.nsplit;  // this head's first split slot
  const long nrows = (long)a.B * a.H * a.nsplit;
  const __amdgpu_buffer_rsrc_t por = rsrc(a.po, (unsigned)(nrows * HD * 4));
  const __amdgpu_buffer_rsrc_t mlr = rsrc(a.pml, (unsigned)(nrows * 8));
  if (n < G) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) st_sc1(por, (unsigned)(((row + sp) * HD + 16 * dt + 4 * g) * 4), acc[dt]);
    if (g == 0) {
      st1_sc1(mlr, (unsigned)((row + sp) * 8), m);
      st1_sc1(mlr, (unsigned)((row + sp) * 8 + 4), lsum);
    }
  }
  if (!a.merge) return;  // paged_reduce merges after the kernel boundary
  // publish (write-through stores drained), take a ticket; the last split of
  // (b, kvh) merges with sc1 loads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int last = 0;
  if (lane == 0) {
    int* c = a.cnt + (long)b * a.HKV + kvh;
    last = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.nsplit - 1;
    if (last) {
      __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  if constexpr (PIPE) {
    // one pass with an online rescale (as over pages), the (m, l, O) loads of
    // four splits in flight together: the serial two-pass loop below pays an
    // L2 round trip per split (it stays for the large-grid variant, whose
    // occupancy the 128 extra VGPRs would cost)
    if (n >= G) return;
    float M = -INFINITY, L = 0.f;
    f32x4v o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4v{0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < a.nsplit; s0 += 4) {
      float mv[4], lv[4];
      f32x4v part[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mv[j] = -INFINITY;
        lv[j] = 0.f;
        if (s0 + j < a.nsplit) {
          mv[j] = ld1_sc1(mlr, (unsigned)((row + s0 + j) * 8));
          lv[j] = ld1_sc1(mlr, (unsigned)((row + s0 + j) * 8 + 4));
#pragma unroll
          for (int dt = 0; dt < 8; ++dt)
            part[j][dt] = ld_sc1(por, (unsigned)(((row + s0 + j) * HD + 16 * dt + 4 * g) * 4));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (lv[j] <= 0.f) continue;
        const float mn = fmaxf(M, mv[j]);
        const float sc = __builtin_amdgcn_exp2f(M - mn), f = __builtin_amdgcn_exp2f(mv[j] - mn);
        L = L * sc + f * lv[j];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[dt] = o[dt] * sc + f * part[j][dt];
        M = mn;
      }
    }
    store_o(op, o, L > 0.f ? 1.f / L : 0.f);
    return;
  }
  if (n >= G) return;
  float M = -INFINITY;
  for (int s2 = 0; s2 < a.nsplit; ++s2) M = fmaxf(M, ld1_sc1(mlr, (unsigned)((row + s2) * 8)));
  float L = 0.f;
  f32x4v o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4v{0.f, 0.f, 0.f, 0.f};
  for (int s2 = 0; s2 < a.nsplit; ++s2) {
    const float ms = ld1_sc1(mlr, (unsigned)((row + s2) * 8));
    const float ls = ld1_sc1(mlr, (unsigned)((row + s2) * 8 + 4));
    if (ls <= 0.f) continue;
    const float f = __builtin_amdgcn_exp2f(ms - M);
    L += f * ls;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] += f * ld_sc1(por, (unsigned)(((row + s2) * HD + 16 * dt + 4 * g) * 4));
  }
  store_o(op, o, L > 0.f ? 1.f / L : 0.f);
}

// merge nsplit partials (m in log2 units, l, unnormalised O) of one (b, h):
// the launch-boundary variant, for batches with many (sequence, KV head)
// groups -- there an in-launch last-arriver merge costs one L2-invalidating
// acquire per group (measured 47 -> 58 us at batch 64 x 1024)
__global__ __launch_bounds__(64) void paged_reduce(const float* __restrict__ po, const float* __restrict__ pml,
                                                   unsigned short* __restrict__ o, int H, int nsplit, long ldo) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const int b = bh / H, h = bh - b * H;
  const float* ml = pml + (long)bh * nsplit * 2;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f, o0 = 0.f, o1 = 0.f;
  // the writer stores O^T in 16-dim tiles: lane's dims d = 2*lane, 2*lane + 1
  const float* pb = po + (long)bh * nsplit * HD + 2 * lane;
#pragma unroll 4
  for (int s = 0; s < nsplit; ++s) {
    const float l = ml[2 * s + 1];
    if (l <= 0.f) continue;
    const float f = __builtin_amdgcn_exp2f(ml[2 * s] - M);
    L += f * l;
    const float2 v = *(const float2*)(pb + (long)s * HD);
    o0 += f * v.x;
    o1 += f * v.y;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  *(unsigned*)(o + (long)b * ldo + (long)h * HD + 2 * lane) = pack_bf16x2(o0 * inv, o1 * inv);
}

}  // namespace dec
}  // namespace kgs

namespace {
inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Tile variants (R = 16-row W tiles per wave, MT = 16-column x tiles, KC =
// k-steps per x chunk). 0 = the measured default for the batch size.
struct SkinnyVariant {
  int r, mt, kc, kin;
};
constexpr SkinnyVariant kVariants[] = {
    {0, 0, 0},                                      // 0: auto
    {1, 1, 16}, {1, 1, 8}, {2, 1, 16},              // 1-3:  M <= 16
    {1, 2, 16}, {1, 2, 8}, {2, 2, 8}, {2, 2, 16},   // 4-7:  M <= 32
    {1, 4, 16}, {1, 4, 4}, {1, 4, 8}, {2, 4, 4}, {2, 4, 8},  // 8-12: M <= 64
    {2, 8, 2}, {2, 8, 4}, {4, 8, 2}, {1, 8, 4},     // 13-16: M <= 128
    {2, 16, 2}, {1, 16, 4}, {1, 16, 2},             // 17-19: M <= 256
    {1, 1, 8, 1}, {2, 1, 8, 1},                     // 20-21: M <= 16, K split inside the workgroup
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

int mt_for(int M) { return M <= 16 ? 1 : M <= 32 ? 2 : M <= 64 ? 4 : M <= 128 ? 8 : 16; }
int default_variant(int mt) { return mt == 1 ? 1 : mt == 2 ? 4 : mt == 4 ? 8 : mt == 8 ? 13 : 17; }

template <int R, int MT, int KC, bool W8, bool KIN = false>
hipError_t launch_skinny(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N, int K, long ldx,
                         long ldy, int ksplit, int cps, const kgs::dec::SkinnyEpi& ep, hipStream_t s) {
  const int nstrip = N / ((KIN ? 16 : 64) * R);
  if constexpr (!W8 && MT <= 4 && R == 1) {  // the fused layer's qkv variants (kgs/ops/decode.py rope_variant)
    if (ep.mode & kgs::dec::EPI_ROPE) {
      hipLaunchKernelGGL((kgs::dec::skinny<R, MT, KC, false, true, KIN>), dim3(nstrip * ksplit), dim3(256), 0, s, wp,
                         (const unsigned short*)x, (unsigned short*)y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep);
      return hipGetLastError();
    }
  }
  if (ep.mode & kgs::dec::EPI_ROPE) return hipErrorInvalidValue;  // no RoPE instantiation for this variant
  hipLaunchKernelGGL((kgs::dec::skinny<R, MT, KC, W8, false, KIN>), dim3(nstrip * ksplit), dim3(256), 0, s, wp,
                     (const unsigned short*)x, (unsigned short*)y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep);
  return hipGetLastError();
}
}  // namespace

// Geometry of tile variant `variant` (0 = default) for a batch of M rows:
// rows of W per workgroup strip, k elements per x chunk, padded batch. Lets the
// host size split-K and the workspace (kgs/ops/decode.py). Returns
// KGS_ERR_ARG when the variant does not cover M's column-tile count.
KGS_EXPORT int kgs_skinny_variant_geometry(int variant, int M, int* rows_per_strip, int* k_per_chunk, int* mpad) {
  if (M <= 0 || M > 256) return KGS_ERR_SHAPE;
  const int mt = mt_for(M);
  if (variant == 0) variant = default_variant(mt);
  if (variant < 0 || variant >= kNumVariants || kVariants[variant].mt != mt) return KGS_ERR_ARG;
  *mpad = 16 * mt;
  const int kin = kVariants[variant].kin;
  *rows_per_strip = (kin ? 16 : 64) * kVariants[variant].r;
  *k_per_chunk = (kin ? 4 : 1) * 32 * kVariants[variant].kc;
  return 0;
}

KGS_EXPORT int kgs_skinny_geometry(int M, int* rows_per_strip, int* k_per_chunk, int* mpad) {
  return kgs_skinny_variant_geometry(0, M, rows_per_strip, k_per_chunk, mpad);
}

// y[M, N] (bf16, row stride ldy) = x[M, K] (row stride ldx) . W^T with W
// prepacked ([N/16][K/32][64][8] bf16). ksplit must divide K / k_per_chunk;
// with ksplit > 1, ws holds ksplit * mpad * N floats and cnt N / rows_per_strip
// zero-initialised ints (left zeroed on return). epi: EPI_* flags (SWIGLU: y is
// [M, N/2]; RMS needs ss_in[M]; RESID accumulates into y and ss_out[M]);
// ss_zero (optional, [M] floats) is cleared at kernel start.
namespace {
int skinny_fused(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N, int K, long ldx, long ldy,
                 int ksplit, int variant, int epi, const float* ss_in, float* ss_out, float* ss_zero, float inv_k,
                 float eps, const float* wscale, const kgs::dec::SkinnyEpi* rope, hipStream_t s);
}

KGS_EXPORT int kgs_skinny_gemm_bf16_fused(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N,
                                         int K, long ldx, long ldy, int ksplit, int variant, int epi,
                                         const float* ss_in, float* ss_out, float* ss_zero, float inv_k, float eps,
                                         const float* wscale, hipStream_t s) {
  if (epi & kgs::dec::EPI_ROPE) return KGS_ERR_ARG;  // kgs_skinny_gemm_bf16_rope
  return skinny_fused(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, variant, epi, ss_in, ss_out, ss_zero, inv_k, eps,
                      wscale, nullptr, s);
}

// The fused qkv projection with RoPE + the KV-cache write in its epilogue
// (EPI_ROPE; W packed with kgs/ops/decode.py rope_rows): y [M, (H + 2 HKV) 128]
// gets the rotated q, k and the v rows in the original order, and k / v land
// in the bf16 cache slot slot[m] (< 0: no write). cos / sin: fp32 [max_pos, 64].
// epi may add EPI_RMS (ss_in, inv_k, eps as in kgs_skinny_gemm_bf16_fused).
KGS_EXPORT int kgs_skinny_gemm_bf16_rope(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N,
                                        int K, long ldx, long ldy, int ksplit, int variant, int epi,
                                        const float* ss_in, float inv_k, float eps, const float* cosv,
                                        const float* sinv, const int* pos, const int* slot, void* cache, int H,
                                        int HKV, hipStream_t s) {
  using namespace kgs::dec;
  if (epi & ~EPI_RMS) return KGS_ERR_ARG;
  if (H <= 0 || HKV <= 0 || H % HKV || N != (H + 2 * HKV) * HD) return KGS_ERR_SHAPE;
  if (!cosv || !sinv || !pos || !slot || !al16(cache)) return KGS_ERR_ARG;
  SkinnyEpi r{};
  r.cosv = cosv;
  r.sinv = sinv;
  r.pos = pos;
  r.slot = slot;
  r.cache = (unsigned short*)cache;
  r.H = H;
  r.HKV = HKV;
  return skinny_fused(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, variant, epi | EPI_ROPE, ss_in, nullptr, nullptr,
                      inv_k, eps, nullptr, &r, s);
}

namespace {
int skinny_fused(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N, int K, long ldx, long ldy,
                 int ksplit, int variant, int epi, const float* ss_in, float* ss_out, float* ss_zero, float inv_k,
                 float eps, const float* wscale, const kgs::dec::SkinnyEpi* rope, hipStream_t s) {
  using namespace kgs::dec;
  int rps, kpc, mpad;
  const int rc = kgs_skinny_variant_geometry(variant, M, &rps, &kpc, &mpad);
  if (rc) return rc;
  if (variant == 0) variant = default_variant(mt_for(M));
  if (epi & ~(EPI_SWIGLU | EPI_RMS | EPI_RESID | EPI_ROPE) || ((epi & EPI_SWIGLU) && (epi & EPI_RESID)))
    return KGS_ERR_ARG;
  if ((epi & EPI_ROPE) && (rope == nullptr || (epi & (EPI_SWIGLU | EPI_RESID)) || wscale != nullptr))
    return KGS_ERR_ARG;
  if (((epi & EPI_RMS) && ss_in == nullptr) || ((epi & EPI_RESID) && ss_out == nullptr)) return KGS_ERR_ARG;
  if (N <= 0 || K <= 0 || N % rps || K % kpc || ldx < K || ldy < ((epi & EPI_SWIGLU) ? N / 2 : N))
    return KGS_ERR_SHAPE;
  const int nchunks = K / kpc;
  if (ksplit <= 0 || nchunks % ksplit) return KGS_ERR_ARG;
  if (ksplit > 1 && (ws == nullptr || cnt == nullptr)) return KGS_ERR_ARG;
  if (!al16(wp) || !al16(x) || ((uintptr_t)y & 7) || ((uintptr_t)ws & 15) || ldx % 8 || ldy % 4) return KGS_ERR_ALIGN;
  const int cps = nchunks / ksplit;
  SkinnyEpi ep = rope ? *rope : SkinnyEpi{};
  ep.mode = epi;
  ep.ss_in = ss_in;
  ep.ss_out = ss_out;
  ep.ss_zero = ss_zero;
  ep.inv_k = inv_k;
  ep.eps = eps;
  ep.wscale = wscale;
  const bool w8 = wscale != nullptr;
  if (w8 && variant > 12 && variant < 20) return KGS_ERR_ARG;  // fp8 weights: batch buckets <= 64
  switch (variant * 2 + (w8 ? 1 : 0)) {
#define KGS_SKV(id, R, MT, KC)                                                                                       \
  case 2 * id: return (int)launch_skinny<R, MT, KC, false>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep, s); \
  case 2 * id + 1:                                                                                                    \
    if constexpr (id <= 12) return (int)launch_skinny<R, MT, KC, true>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit,  \
                                                                        cps, ep, s);                                  \
    return KGS_ERR_ARG;
    KGS_SKV(1, 1, 1, 16) KGS_SKV(2, 1, 1, 8) KGS_SKV(3, 2, 1, 16)
    KGS_SKV(4, 1, 2, 16) KGS_SKV(5, 1, 2, 8) KGS_SKV(6, 2, 2, 8) KGS_SKV(7, 2, 2, 16)
    KGS_SKV(8, 1, 4, 16) KGS_SKV(9, 1, 4, 4) KGS_SKV(10, 1, 4, 8) KGS_SKV(11, 2, 4, 4) KGS_SKV(12, 2, 4, 8)
    KGS_SKV(13, 2, 8, 2) KGS_SKV(14, 2, 8, 4) KGS_SKV(15, 4, 8, 2) KGS_SKV(16, 1, 8, 4)
    KGS_SKV(17, 2, 16, 2) KGS_SKV(18, 1, 16, 4) KGS_SKV(19, 1, 16, 2)
#undef KGS_SKV
    case 2 * 20: return (int)launch_skinny<1, 1, 8, false, true>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep, s);
    case 2 * 20 + 1: return (int)launch_skinny<1, 1, 8, true, true>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep, s);
    case 2 * 21: return (int)launch_skinny<2, 1, 8, false, true>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep, s);
    case 2 * 21 + 1: return (int)launch_skinny<2, 1, 8, true, true>(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, cps, ep, s);
    default: return KGS_ERR_ARG;
  }
}
}  // namespace

KGS_EXPORT int kgs_skinny_gemm_bf16_ex(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N,
                                      int K, long ldx, long ldy, int ksplit, int variant, int epi, hipStream_t s) {
  return kgs_skinny_gemm_bf16_fused(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, variant, epi, nullptr, nullptr,
                                    nullptr, 0.f, 0.f, nullptr, s);
}

KGS_EXPORT int kgs_skinny_gemm_bf16_v(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N, int K,
                                     long ldx, long ldy, int ksplit, int variant, hipStream_t s) {
  return kgs_skinny_gemm_bf16_ex(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, variant, 0, s);
}

KGS_EXPORT int kgs_skinny_gemm_bf16(const void* wp, const void* x, void* y, float* ws, int* cnt, int M, int N, int K,
                                   long ldx, long ldy, int ksplit, hipStream_t s) {
  return kgs_skinny_gemm_bf16_v(wp, x, y, ws, cnt, M, N, K, ldx, ldy, ksplit, 0, s);
}

// qkv: [tokens, ld] fused projection rows (H q heads, HKV k heads, HKV v heads
// of 128); pos/slot: int32 [tokens]; cache: this layer's pages
// [pages][HKV][2][4096] bf16. q and k are rotated in place; k, v land in the cache.
// kv8: the cache holds e4m3 bytes ([pages][HKV][2][4096] B) instead of bf16.
// P != nullptr: the projection is given as nslice fp32 split-K partials
// [nslice][tokens][(H + 2 HKV) * hd] instead of in qkv; the reduced, rotated
// rows are written to qkv (which is then output only).
KGS_EXPORT int kgs_rope_cache_bf16(void* qkv, const float* cosv, const float* sinv, const int* pos, const int* slot,
                                  void* cache, long tokens, int H, int HKV, int hd, long ld, int kv8, const float* P,
                                  int nslice, hipStream_t s) {
  if (tokens < 0 || H <= 0 || HKV <= 0 || H % HKV || hd != kgs::dec::HD) return KGS_ERR_SHAPE;
  if (ld < (long)(H + 2 * HKV) * hd) return KGS_ERR_SHAPE;
  if (!al16(qkv) || !al16(cosv) || !al16(sinv) || !al16(cache) || ld % 8) return KGS_ERR_ALIGN;
  if (P != nullptr && (nslice <= 0 || !al16(P))) return KGS_ERR_ARG;
  const long n = tokens * (H + 2 * HKV) * 8;
  if (n == 0) return 0;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  auto q = (unsigned short*)qkv;
  if (P != nullptr) {
#define KGS_RCS(KV, NSL)                                                                                           \
  hipLaunchKernelGGL((kgs::dec::rope_cache<KV, true, NSL>), g, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H, \
                     HKV, ld, P, nslice)
#define KGS_RCS_KV(KV)                \
  switch (nslice) {                   \
    case 2: KGS_RCS(KV, 2); break;    \
    case 4: KGS_RCS(KV, 4); break;    \
    case 8: KGS_RCS(KV, 8); break;    \
    default: KGS_RCS(KV, 0); break;   \
  }
    if (kv8) {
      KGS_RCS_KV(true);
    } else {
      KGS_RCS_KV(false);
    }
#undef KGS_RCS_KV
#undef KGS_RCS
  } else if ((H + 2 * HKV) % 8 == 0 && !kv8 && tokens >= 1024) {
    // prompt-sized: the v heads go through the page-run writer
    const dim3 g8((unsigned)((n / 8 + 255) / 256));
    hipLaunchKernelGGL((kgs::dec::rope_cache_g8<false, true>), g8, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H,
                       HKV, ld);
    const dim3 gv((unsigned)((tokens + kgs::dec::PAGE - 1) / kgs::dec::PAGE), (unsigned)HKV);
    hipLaunchKernelGGL(kgs::dec::v_cache_pages, gv, b, 0, s, (const unsigned short*)q, slot, (unsigned short*)cache,
                       tokens, H, HKV, ld);
  } else if ((H + 2 * HKV) % 8 == 0) {
    const dim3 g8((unsigned)((n / 8 + 255) / 256));
    if (kv8)
      hipLaunchKernelGGL(kgs::dec::rope_cache_g8<true>, g8, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H, HKV,
                         ld);
    else
      hipLaunchKernelGGL(kgs::dec::rope_cache_g8<false>, g8, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H, HKV,
                         ld);
  } else if (kv8) {
    hipLaunchKernelGGL(kgs::dec::rope_cache<true>, g, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H, HKV, ld,
                       nullptr, 0);
  } else {
    hipLaunchKernelGGL(kgs::dec::rope_cache<false>, g, b, 0, s, q, cosv, sinv, pos, slot, cache, tokens, H, HKV, ld,
                       nullptr, 0);
  }
  return (int)hipGetLastError();
}

// Paged decode attention for one new query token per sequence. q: [B, ldq]
// (query heads at 128-element blocks); cache: layer base; block_tables
// [B, max_pages] int32; ctx_lens [B] int32 (>= 1). nsplit > 1 needs po
// (B*H*nsplit*128 f32), pml (B*H*nsplit*2 f32) and cnt (B*HKV zeroed ints, left
// zeroed); the splits are merged in the same launch.
KGS_EXPORT int kgs_paged_decode_bf16_ex(const void* q, const void* cache, const int* block_tables,
                                       const int* ctx_lens, void* o, float* po, float* pml, int* cnt, int B, int H,
                                       int HKV, int hd, int max_pages, int pages_per_split, int nsplit, long ldq,
                                       long ldo, float scale, int kv8, int pipe_mode, hipStream_t s);

KGS_EXPORT int kgs_paged_decode_bf16(const void* q, const void* cache, const int* block_tables, const int* ctx_lens,
                                    void* o, float* po, float* pml, int* cnt, int B, int H, int HKV, int hd,
                                    int max_pages, int pages_per_split, int nsplit, long ldq, long ldo, float scale,
                                    int kv8, hipStream_t s) {
  return kgs_paged_decode_bf16_ex(q, cache, block_tables, ctx_lens, o, po, pml, cnt, B, H, HKV, hd, max_pages,
                                  pages_per_split, nsplit, ldq, ldo, scale, kv8, -1, s);
}

// pipe_mode: -1 = automatic (the two-page register pipeline for small grids),
// 0 / 1 = force it off / on (measurement)
KGS_EXPORT int kgs_paged_decode_bf16_ex(const void* q, const void* cache, const int* block_tables,
                                       const int* ctx_lens, void* o, float* po, float* pml, int* cnt, int B, int H,
                                       int HKV, int hd, int max_pages, int pages_per_split, int nsplit, long ldq,
                                       long ldo, float scale, int kv8, int pipe_mode, hipStream_t s) {
  using namespace kgs::dec;
  if (B <= 0 || H <= 0 || HKV <= 0 || H % HKV || H / HKV > 16 || hd != HD) return KGS_ERR_SHAPE;
  if (max_pages <= 0 || pages_per_split <= 0 || nsplit <= 0) return KGS_ERR_SHAPE;
  if ((long)pages_per_split * nsplit < max_pages) return KGS_ERR_ARG;
  if (ldq < (long)H * HD || ldo < (long)H * HD) return KGS_ERR_SHAPE;
  if (!al16(q) || !al16(cache) || !al16(o) || ldq % 8 || ldo % 8) return KGS_ERR_ALIGN;
  if (nsplit > 1 && (po == nullptr || pml == nullptr || !al16(po))) return KGS_ERR_ARG;
  const long nwg = (long)B * HKV * nsplit;
  if (nwg > 0x7fffffff) return KGS_ERR_SHAPE;
  // in-launch merge only when there are few (sequence, KV head) groups: it saves
  // the reduce launch but costs each group's last split an acquire
  const int merge = nsplit > 1 && cnt != nullptr && (long)B * HKV <= 32;
  AttnArgs a{(const unsigned short*)q, (const unsigned short*)cache, block_tables, ctx_lens, (unsigned short*)o, po,
             pml, cnt, ldq, ldo, B, H, HKV, max_pages, pages_per_split, nsplit, merge, scale * 1.4426950408889634f,
             nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
  // up to 4 waves per CU (1024 on the chip) other waves cannot hide a page's
  // latency: pipeline inside the wave there. Round 3 measured the pipeline at
  // 1.2-1.9x for 512-1024-wave grids (batch 64-128 at 528-2000 cached
  // tokens) and +-2 % at 2048 waves (profiles/r3/decode/paged_sweep_ctx*.log)
  const bool pipe = pipe_mode < 0 ? nwg <= 1024 : pipe_mode != 0;
  if (kv8) {
    if (pipe) hipLaunchKernelGGL((paged_decode<true, true>), dim3((unsigned)nwg), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((paged_decode<true, false>), dim3((unsigned)nwg), dim3(64), 0, s, a);
  } else {
    if (pipe) hipLaunchKernelGGL((paged_decode<false, true>), dim3((unsigned)nwg), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((paged_decode<false, false>), dim3((unsigned)nwg), dim3(64), 0, s, a);
  }
  if (nsplit > 1 && !merge)
    hipLaunchKernelGGL(paged_reduce, dim3((unsigned)(B * H)), dim3(64), 0, s, po, pml, (unsigned short*)o, H, nsplit,
                       ldo);
  return (int)hipGetLastError();
}

// rope_cache + paged decode attention in one launch: the fused qkv projection
// arrives as nslice fp32 split-K partials P [nslice][B][(H + 2 HKV) * 128]
// (gemm_nt_w4x_partials); each attention wave reduces, rotates and caches its
// own (sequence, KV head) rows (paged_decode RP) -- the same bits as
// kgs_rope_cache_bf16(P) followed by kgs_paged_decode_bf16 on the rotated q.
// slot[b]: the new token's cache slot; its page must be the last one of
// ctx_lens[b] in block_tables (as the engine assigns it).
KGS_EXPORT int kgs_paged_decode_rope_bf16(const float* P, int nslice, const float* cosv, const float* sinv,
                                         const int* pos, const int* slot, void* cache, const int* block_tables,
                                         const int* ctx_lens, void* o, float* po, float* pml, int* cnt, int B, int H,
                                         int HKV, int hd, int max_pages, int pages_per_split, int nsplit, long ldo,
                                         float scale, int kv8, int pipe_mode, hipStream_t s) {
  using namespace kgs::dec;
  if (B <= 0 || H <= 0 || HKV <= 0 || H % HKV || H / HKV > 6 || hd != HD) return KGS_ERR_SHAPE;
  if (max_pages <= 0 || pages_per_split <= 0 || nsplit <= 0) return KGS_ERR_SHAPE;
  if (nslice != 2 && nslice != 4 && nslice != 8) return KGS_ERR_ARG;  // compile-time slice counts
  if ((long)pages_per_split * nsplit < max_pages) return KGS_ERR_ARG;
  if (ldo < (long)H * HD || ldo % 8) return KGS_ERR_SHAPE;
  if (P == nullptr || pos == nullptr || slot == nullptr) return KGS_ERR_ARG;
  if (!al16(P) || !al16(cosv) || !al16(sinv) || !al16(cache) || !al16(o)) return KGS_ERR_ALIGN;
  if (nsplit > 1 && (po == nullptr || pml == nullptr || !al16(po))) return KGS_ERR_ARG;
  const long nwg = (long)B * HKV * nsplit;
  if (nwg > 0x7fffffff) return KGS_ERR_SHAPE;
  const int merge = nsplit > 1 && cnt != nullptr && (long)B * HKV <= 32;
  AttnArgs a{nullptr, (const unsigned short*)cache, block_tables, ctx_lens, (unsigned short*)o, po, pml, cnt, 0, ldo,
             B, H, HKV, max_pages, pages_per_split, nsplit, merge, scale * 1.4426950408889634f,
             P, nslice, cosv, sinv, pos, slot, cache};
  const bool pipe = pipe_mode < 0 ? nwg <= 1024 : pipe_mode != 0;
#define KGS_PDR(KV, PP, NS) hipLaunchKernelGGL((paged_decode<KV, PP, NS>), dim3((unsigned)nwg), dim3(64), 0, s, a)
#define KGS_PDR_NS(KV, PP)         \
  switch (nslice) {                \
    case 2: KGS_PDR(KV, PP, 2); break; \
    case 4: KGS_PDR(KV, PP, 4); break; \
    default: KGS_PDR(KV, PP, 8); break; \
  }
  if (kv8) {
    if (pipe) { KGS_PDR_NS(true, true); } else { KGS_PDR_NS(true, false); }
  } else {
    if (pipe) { KGS_PDR_NS(false, true); } else { KGS_PDR_NS(false, false); }
  }
#undef KGS_PDR_NS
#undef KGS_PDR
  if (nsplit > 1 && !merge)
    hipLaunchKernelGGL(paged_reduce, dim3((unsigned)(B * H)), dim3(64), 0, s, po, pml, (unsigned short*)o, H, nsplit,
                       ldo);
  return (int)hipGetLastError();
}
