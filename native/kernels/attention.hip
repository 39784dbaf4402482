// Flash-attention forward for gfx950 (bf16 in/out, fp32 softmax/accumulate),
// head_dim 128, causal or full, GQA -- the prefill attention of the Llama
// stand-in (kgs/models/llama.py). Q, K and V are read in place from the fused
// QKV projection output ([tokens, (H + 2 HKV) * 128], any row stride) and O is
// written as [tokens, H * 128], the layout the O projection consumes: no
// transposes around the kernel.
//
// Structure (one workgroup = 4 waves = 128 query rows of one (batch, head);
// 2 workgroups per CU; K/V tiles of 64 keys):
//   * swapped QK^T on v_mfma_f32_32x32x16_bf16: S^T = K . Q^T, so a lane owns
//     ONE query row (lane & 31) and 32 of the tile's 64 scores -- the row max /
//     row sum are in-lane plus one xor-32 exchange, and the per-row rescale of
//     O is a lane scalar;
//   * the S^T accumulator is the B operand of P.V with no data movement
//     (O^T = V^T . P^T): registers 8s..8s+7 of each 32x32 tile are k-step s,
//     in the permuted key order kv = 16s + 8(j>>2) + 4(lane>>5) + (j&3) that
//     the V fragments are read in;
//   * V fragments via ds_read_b64_tr_b16 (a free transpose out of the
//     row-major tile), K fragments via ds_read_b128; both tiles use the
//     256-B-row XOR image off(r, c) = 256 r + 16 (c ^ ((r&3)<<2 | (r>>2)&3)),
//     conflict-free for the 16-lane groups of ds_read_b128 and the 32-lane
//     halves of the transposed read;
//   * double buffer filled by LDS-DMA: the next K/V tile's global_load_lds
//     are issued before the current tile's MFMAs (no staging registers),
//     vmcnt(0) + one barrier per tile;
//   * causal: fully-masked tiles are skipped per wave, the diagonal tiles are
//     masked in registers; q-blocks are dispatched heaviest first, and the four
//     query heads sharing a KV head are dealt to the same XCD back to back so
//     the K/V tiles they share are L2 hits.
#include "kgs_common.h"

namespace kgs {
namespace attn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x4s __attribute__((ext_vector_type(4)));

constexpr int HD = 128;
constexpr int QB = 128;  // query rows per workgroup (4 waves x 32)
constexpr int KB = 64;   // keys per tile
constexpr int TILE_BYTES = KB * HD * 2;  // 16 KB
constexpr float NEG = -1.0e30f;
constexpr float RESCALE = 8.0f;  // deferred-max threshold, log2 units: P <= 256

struct Args {
  const unsigned short* q;
  const unsigned short* k;
  const unsigned short* v;
  unsigned short* o;
  long ldq, ldk, ldv, ldo;  // row strides (elements)
  int B, S, H, HKV;
  float sl2;  // softmax scale * log2(e)
  int causal;
  int Sk;    // keys per sequence (= S, or S + qoff for a chunk over a cached context)
  int qoff;  // position of query row 0 among the keys: causal row i sees keys <= qoff + i
};

__device__ __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int off(int r, int c) { return 256 * r + 16 * (c ^ swz(r)); }

__device__ __forceinline__ bf16x8 tr_frag(const char* lo, const char* hi) {
  const bf16x4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((KGS_LDS bf16x4s*)lo);
  const bf16x4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((KGS_LDS bf16x4s*)hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& s, int base) { return pack_bf16x8(s, base); }

__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void fwd(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE_BYTES];  // [buf][K, V]

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hh = lane >> 5;
  const int nqb = a.S / QB;
  const int nwg = gridDim.x;
  // XCD-aware order: 8 consecutive dispatch slots of one XCD take 4 heads of
  // one KV group; work ids stay heaviest-first in dispatch time.
  int lid = blockIdx.x;
  if ((nwg & 31) == 0) {
    const int t = lid >> 3, x = lid & 7;
    lid = ((t >> 2) << 5) | (x << 2) | (t & 3);
  }
  const int per = a.B * a.H;
  const int qi = lid / per, rem = lid - qi * per;
  const int qb = a.causal ? nqb - 1 - qi : qi;
  const int b = rem / a.H, h = rem - b * a.H;
  const int kvh = h / (a.H / a.HKV);

  const int q0 = qb * QB;
  const int qw = q0 + 32 * w;       // this wave's first query row
  const int qrow = qw + l32;        // this lane's query row
  const long tok0 = (long)b * a.S;     // first query token of the sequence
  const long ktok0 = (long)b * a.Sk;   // its first key token
  const int qoff = a.qoff;

  // Q fragments (B operand of S^T = K.Q^T): lane holds Q[qrow][16ks + 8hh .. +7]
  bf16x8 qf[8];
  {
    const bf16x8* qp = (const bf16x8*)(a.q + (tok0 + qrow) * a.ldq + (long)h * HD + 8 * hh);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = qp[2 * ks];
  }

  const unsigned short* kbase = a.k + ktok0 * a.ldk + (long)kvh * HD;
  const unsigned short* vbase = a.v + ktok0 * a.ldv + (long)kvh * HD;
  // K/V tile jn -> LDS buffer sb by LDS-DMA (global_load_lds, no staging
  // registers): a 16 KB tile is 16 chunks of 1 KB = 4 rows of 256 B; wave w
  // issues chunks 4w .. 4w+3 of K and of V. Lane l lands at chunk + 16 l, i.e.
  // at slot (r, c') of the XOR image, so it fetches column c = c' ^ swz(r).
  auto dma_tiles = [&](int jn, int sb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = 4 * w + i;
      const int r = 4 * ch + (lane >> 4), c = (lane & 15) ^ swz(r);
      const long row = (long)jn * KB + r;
      glds16(kbase + row * a.ldk + 8 * c, smem[sb][0] + 1024 * ch);
      glds16(vbase + row * a.ldv + 8 * c, smem[sb][1] + 1024 * ch);
    }
  };

  const int ntile = a.causal ? (qoff + q0 + QB) / KB : a.Sk / KB;
  dma_tiles(0, 0);
  // Q fragments and tile 0 complete before the loop (a vmcnt the waitcnt pass
  // sees, so it does not carry the Q loads into the loop header)
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  __syncthreads();

  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x16{};
  float m = NEG, l = 0.f;
  const float sl2 = a.sl2;

  // tr-read lane address pieces: group g = lane >> 4, lane 4q + p in it
  const int g = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;

  for (int j = 0; j < ntile; ++j) {
    const int buf = j & 1;
    // the other buffer was released by the previous tile's barrier
    if (j + 1 < ntile) dma_tiles(j + 1, buf ^ 1);
    const int kv0 = j * KB;
    if (!a.causal || kv0 <= qoff + qw + 31) {
      const char* Ks = smem[buf][0];
      const char* Vs = smem[buf][1];
      // all 16 K fragments of the tile are read up front (the registers the
      // LDS-DMA staging freed), so the QK^T MFMAs never wait on one LDS read
      bf16x8 kf[2][8];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) kf[t][ks] = *(const bf16x8*)(Ks + off(32 * t + l32, 2 * ks + hh));
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them otherwise)
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[t][ks], qf[ks], s[t], 0, 0, 0);
      }
      // the first half of the tile's V fragments is read now, so its LDS
      // latency hides under the softmax below (all 16 would spill at 2 waves
      // per SIMD); the second half is read under the first half's P.V MFMAs
      bf16x8 vfr[4][2][2];
      auto read_v = [&](int d) {
        const int c0 = 4 * d + 2 * (g & 1) + (tp >> 1);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            const int kvb = 32 * t + 16 * sp + 4 * hh + tq;
            vfr[d][t][sp] = tr_frag(Vs + off(kvb, c0) + 8 * (tp & 1), Vs + off(kvb + 8, c0) + 8 * (tp & 1));
          }
      };
      read_v(0);
      read_v(1);
      __builtin_amdgcn_sched_barrier(0);
      if (a.causal && kv0 + KB - 1 > qoff + qw) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kv = kv0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (kv > qoff + qrow) s[t][r] = NEG;
          }
      }
      float mx = m;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[t][r]);
      mx = xor32_max(mx);  // v_permlane32_swap (kgs_common.h), not an LDS round trip
      // deferred rescale (guide T13): the running max m only moves when a row's
      // new max exceeds it by more than RESCALE (log2 units after sl2), so most
      // tiles skip the 64-multiply O rescale; p = exp2(s sl2 - m sl2) then stays
      // <= 2^RESCALE (fp32 sums and bf16 P are scale-free). Both l and O see the
      // same alpha, and the decision is wave-uniform, so no pending P.V is split.
      const bool grow = (mx - m) * sl2 > RESCALE;
      if (__any(grow)) {
        const float mn = grow ? mx : m;
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * sl2);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] *= alpha;
      }
      const float msl = m * sl2;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[t][r], sl2, -msl));
          s[t][r] = p;
          l += p;
        }
      bf16x8 pf[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        pf[t][0] = pack8(s[t], 0);
        pf[t][1] = pack8(s[t], 8);
      }
      read_v(2);
      read_v(3);
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[d][t][sp], pf[t][sp], o[d], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the next tile has landed
    __syncthreads();
  }

  l = xor32_sum(l);
  const float inv = 1.0f / l;
  unsigned short* op = a.o + (tok0 + qrow) * a.ldo + (long)h * HD;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int dcol = 32 * d + 8 * r4 + 4 * hh;
      uint2 pk;
      pk.x = pack_bf16x2(o[d][4 * r4 + 0] * inv, o[d][4 * r4 + 1] * inv);
      pk.y = pack_bf16x2(o[d][4 * r4 + 2] * inv, o[d][4 * r4 + 3] * inv);
      *(uint2*)(op + dcol) = pk;
    }
}

}  // namespace attn
}  // namespace kgs

// q/k/v/o point at head 0 of token 0 ([B*S, ld] token-major); heads of one
// token are contiguous 128-element blocks. Requires head_dim 128, S % 128 == 0,
// H % HKV == 0, 16-B aligned pointers and ld % 8 == 0.
//
// _ex: Sk keys per sequence ([B*Sk, ld] k/v), Sk >= S, Sk - S a multiple of 64:
// the S query rows are the LAST S positions of the sequence (a prefill chunk
// over Sk - S cached tokens), so causal row i sees keys 0 .. Sk - S + i.
KGS_EXPORT int kgs_attn_fwd_bf16_ex(const void* q, const void* k, const void* v, void* o, int B, int S, int Sk, int H,
                                   int HKV, int hd, long ldq, long ldk, long ldv, long ldo, float scale, int causal,
                                   hipStream_t s) {
  using namespace kgs::attn;
  if (B <= 0 || S <= 0 || H <= 0 || HKV <= 0 || H % HKV) return KGS_ERR_SHAPE;
  if (hd != HD || S % QB || Sk < S || (Sk - S) % KB) return KGS_ERR_SHAPE;
  if (ldq < (long)H * HD || ldk < (long)HKV * HD || ldv < (long)HKV * HD || ldo < (long)H * HD) return KGS_ERR_SHAPE;
  const uintptr_t al = (uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o;
  if ((al & 15) || (ldq | ldk | ldv | ldo) & 7) return KGS_ERR_ALIGN;
  const long nwg = (long)B * H * (S / QB);
  if (nwg > 0x7fffffff) return KGS_ERR_SHAPE;
  Args a{(const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o,
         ldq, ldk, ldv, ldo, B, S, H, HKV, scale * 1.4426950408889634f, causal ? 1 : 0, Sk, Sk - S};
  hipLaunchKernelGGL(fwd, dim3((unsigned)nwg), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

KGS_EXPORT int kgs_attn_fwd_bf16(const void* q, const void* k, const void* v, void* o, int B, int S, int H, int HKV,
                                int hd, long ldq, long ldk, long ldv, long ldo, float scale, int causal,
                                hipStream_t s) {
  return kgs_attn_fwd_bf16_ex(q, k, v, o, B, S, S, H, HKV, hd, ldq, ldk, ldv, ldo, scale, causal, s);
}
