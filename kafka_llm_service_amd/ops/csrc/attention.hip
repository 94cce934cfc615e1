// Paged attention for gfx950 on v_mfma_f32_32x32x16_bf16.
//
// KV page layout (page = 16 tokens, one layer):
//   K: [num_blocks, Hkv, 16, D]   stored as D/8 chunk planes [16][16 keys][8]: (key o, d) at ((d>>3)*16 + o)*8 + (d&7)
//                                 (see rope_kv.hip): a wave's K fragment load is two contiguous 512-B runs
//   V: [num_blocks, Hkv, D, 16]   V^T per page, key offset o stored at swap_bits_2_3(o)   (see rope_kv.hip)
//
// One wave processes 32 query rows x 32 keys per step, entirely in registers:
//   S^T[key][q] = K . Q^T      A = K rows (16-B loads straight from the page), B = Q^T (kept in VGPRs)
//   softmax per q column: each lane owns one q column (lane & 31), so row max / row sum are lane-local plus one
//                         exchange with lane ^ 32; the online-softmax rescale of O is lane-local too.
//   O^T[d][q] += V^T . P      A = V^T page rows (one 16-B load per lane thanks to the page permutation),
//                             B = P taken from the S^T accumulator registers (regs 8s..8s+7 -> k-step s), no LDS.
// Scores use the exp2 domain (scale * log2 e folded in); lse outputs are log2-domain.
//
// Kernels:
//   attn_decode_kernel   grid (splits, Hkv, B): one query token per sequence, its G = Hq/Hkv heads packed in the
//                        q columns, the sequence's keys split over `splits` workgroups and over the 4 waves of each
//                        (flash-decoding); waves combine through LDS, splits through attn_merge_kernel.
//   attn_prefill_kernel  grid (Hkv, work items): a tile of up to 128 (token, head) query rows against a paged key
//                        range; per-row causal limit; writes bf16 output directly or an (O, lse) partial. Used for
//                        chunked prefill and for the cascade pass where the rows are the decode sequences of a
//                        batch and the keys are the shared system-prompt prefix (read once for all sequences).
//   attn_merge_kernel    log-sum-exp merge of S partials per (row, head) -> bf16.
//   (attn_prefill_kernel variants: 0 = 8 waves / 256 rows per item, K/V staged once per workgroup in LDS;
//    1 = 4 waves / 128 rows, LDS; 2 = 4 waves / 128 rows, per-wave register loads. ops.tile_rows(variant).)
//
// fp8 KV cache (FP8 template flag; page layout in rope_kv.hip): e4m3 pages with one power-of-two exponent per
// (token, kv head) for K and for V. Register path (decode, variant 2): a lane's 16-B K load is the A-fragments of
// two k-steps of ONE key, so the key's exponent is the scale operand of v_cvt_scalef32_pk_bf16_fp8 (dequant is one
// VALU op per 2 elements); V^T fragments dequantize unscaled and the per-key V exponent goes into P instead
// (v_ldexp on the 16 probabilities of the lane after the row sum — P . diag(2^e) . V). LDS path (tile kernel):
// the staging threads dequantize K (scaled) and V (unscaled) into the same bf16 LDS tiles, and the two pages' V
// exponents ride along in 32 B at the end of the stage. MFMA stays bf16: QK^T with an fp8 Q would add a second
// quantization error for no gain in a kernel that is bound by bytes (decode) or by staging (tile).
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace kafka {

constexpr int PAGE = 16;

struct AttnWorkItem {
  int q_start;  // first query token (row of q / out)
  int q_count;  // tokens in this tile
  int bt_row;   // block-table row used for the keys
  int kv_lo;    // first key position (inclusive)
  int kv_hi;    // last key position (exclusive)
  int split;    // -1: write normalized bf16 to out; >= 0: write partial #split
  int pad0, pad1;
};

// Reductions with the partner lane l ^ 32 on gfx950's v_permlane32_swap (one VALU op, no LDS crossbar round trip
// through ds_bpermute — which also queued behind the K/V fragment reads): swapping a register with itself leaves
// x[l] in one result and x[l ^ 32] in the other, so a symmetric op of the two is the xor-32 reduction on every lane.
// max as llvm.maximum (gfx950 v_maximum3_f32, 3 inputs, no NaN-quieting v_max x, x of each MFMA result that fmaxf
// costs in IEEE mode; attn_tile.hip t3_max)
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int KPAGE8 = PAGE * 128 + 32;  // fp8 K page bytes per (block, kv head): data + K/V exponents
constexpr int VPAGE8 = PAGE * 128;
constexpr int KEXP8 = PAGE * 128, VEXP8 = PAGE * 128 + 16;

__device__ __forceinline__ float exp2i(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }

// 8 e4m3 bytes (two dwords) -> bf16x8 times `sc` (a power of two)
__device__ __forceinline__ bf16x8 dq8(uint32_t lo, uint32_t hi, float sc) {
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, sc, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, sc, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, sc, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, sc, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

template <int D>
struct WaveAcc {
  f32x16 o[D / 32];
  float m;
  float l;
};

// K/V fragments of one 32-key block for one wave (register-staged; the next block is prefetched while the
// current one is computed: loads for block i+1 are issued before the MFMAs of block i, so HBM/L2 latency hides
// under the QK^T / softmax / PV work instead of stalling every 32-key step).
template <int D>
struct KVFrag {
  bf16x8 k[D / 16];
  bf16x8 v[2][D / 32];
};

// fp8: 16-B unit j of the lane's key = A-fragments of k-steps 2j, 2j + 1; V^T rows as 8-B loads; the lane's key
// exponent (K) and its 8 keys' exponents per page (V)
template <int D>
struct KVFrag8 {
  u32x4 k[D / 32];
  u32x2 v[2][D / 32];
  int kexp;
  u32x2 vexp[2];
};

template <int D>
__device__ __forceinline__ void load_kv8(KVFrag8<D>& f, const uint8_t* __restrict__ k_cache,
                                         const uint8_t* __restrict__ v_cache, int Hkv, int kvh, int page0,
                                         int page1, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int kp = (r >> 4) ? page1 : page0;
  const uint8_t* kb = k_cache + ((int64_t)kp * Hkv + kvh) * KPAGE8;
#pragma unroll
  for (int j = 0; j < D / 32; ++j)
    f.k[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kb + ((2 * j + h) * PAGE + (r & 15)) * 16));
  f.kexp = (int)*reinterpret_cast<const int8_t*>(kb + KEXP8 + (r & 15));
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int vp = s2 ? page1 : page0;
    const uint8_t* vb = v_cache + ((int64_t)vp * Hkv + kvh) * VPAGE8 + r * PAGE + 8 * h;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) f.v[s2][t] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(vb + 32 * t * PAGE));
    f.vexp[s2] = *reinterpret_cast<const u32x2*>(k_cache + ((int64_t)vp * Hkv + kvh) * KPAGE8 + VEXP8 + 8 * h);
  }
}

template <int D>
__device__ __forceinline__ void load_kv(KVFrag<D>& f, const bf16* __restrict__ k_cache,
                                        const bf16* __restrict__ v_cache, int Hkv, int kvh, int page0, int page1,
                                        int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int kp = (r >> 4) ? page1 : page0;
  // chunk plane 2kk + h, key r & 15
  const bf16* kptr = k_cache + ((int64_t)kp * Hkv + kvh) * (PAGE * D) + (r & 15) * 8 + h * (PAGE * 8);
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) f.k[kk] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kptr + kk * (2 * PAGE * 8)));
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int vp = s2 ? page1 : page0;
    const bf16* vptr = v_cache + ((int64_t)vp * Hkv + kvh) * (D * PAGE) + r * PAGE + 8 * h;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) f.v[s2][t] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(vptr + 32 * t * PAGE));
  }
}

// Page ids of a decode piece staged in LDS: page i of the row at pages[i - pg0] (one ds_read instead of an L2 round
// trip in front of every K/V block load — the decode loop is bound by that dependent chain per wave, not by HBM)
struct LdsPages {
  const int* p;
  int pg0;
  __device__ __forceinline__ int operator[](int i) const { return p[i - pg0]; }
};

// Pages holding keys [key0, key0 + 32) (key0 32-aligned); the second page is only dereferenced below `end`.
template <typename BT>
__device__ __forceinline__ void block_pages(const BT& bt, int key0, int end, int& p0, int& p1) {
  p0 = bt[key0 >> 4];
  p1 = (key0 + 16 < end) ? bt[(key0 >> 4) + 1] : p0;
}

// Online softmax of one 32-key S^T tile (raw scores, lane = query column) + the P.V MFMAs.
//   * `masked` (wave-uniform) is false for interior blocks: no per-element range / causal test at all;
//   * the O / l rescale runs only when some row's running max moved (wave vote) — exact, and after the first few
//     blocks of a row it almost never fires;
//   * the softmax scale is folded into one FMA in front of exp2.
// acc.m is kept in the scaled log2 domain.
// VS (fp8 cache): P column scaled by the per-key V exponents vexp (lane half h: keys of page s2 in register order)
template <int D, bool VS = false>
__device__ __forceinline__ void softmax_pv(f32x16& s, bool masked, int key0, int lo, int hi, int limit,
                                           float scale_log2, const bf16x8 (&vf)[2][D / 32], WaveAcc<D>& acc,
                                           int lane, u32x2 ve0 = {0u, 0u}, u32x2 ve1 = {0u, 0u}) {
  const int h = lane >> 5;
  if (masked) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = key0 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (!((key >= lo) & (key < hi) & (key <= limit))) s[i] = -INFINITY;
    }
  }
  float ma = vmax(s[0], s[1]), mb = vmax(s[2], s[3]);
#pragma unroll
  for (int i = 4; i < 16; i += 4) {
    ma = vmax(vmax(ma, s[i]), s[i + 1]);
    mb = vmax(vmax(mb, s[i + 2]), s[i + 3]);
  }
  const float mx = xor32_max(vmax(ma, mb));
  const float m_new = vmax(acc.m, mx * scale_log2);
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  if (!__all(m_new == acc.m)) {
    const float alpha = exp2f(acc.m - m_use);
    acc.l *= alpha;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) acc.o[t] *= alpha;
  }
  acc.m = m_new;
  float psum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float p = fast_exp2(fmaf(s[i], scale_log2, -m_use));
    s[i] = p;
    psum += p;
  }
  psum = xor32_sum(psum);
  acc.l += psum;
  if constexpr (VS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t w0 = j < 4 ? ve0[0] : ve0[1], w1 = j < 4 ? ve1[0] : ve1[1];
      s[j] = ldexpf(s[j], __builtin_amdgcn_sbfe(w0, 8 * (j & 3), 8));
      s[8 + j] = ldexpf(s[8 + j], __builtin_amdgcn_sbfe(w1, 8 * (j & 3), 8));
    }
  }
  bf16x8 pf[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pf[0][j] = (bf16)s[j];
    pf[1][j] = (bf16)s[8 + j];
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < D / 32; ++t) acc.o[t] = mfma32(vf[s2][t], pf[s2], acc.o[t]);
}

// One 32-key step for one wave on already-loaded fragments.
template <int D>
__device__ __forceinline__ void attn_compute(const KVFrag<D>& f, int key0, int lo, int hi, int limit,
                                             const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                             int lane, bool masked = true) {
  f32x16 s = {};
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) s = mfma32(f.k[kk], qf[kk], s);
  softmax_pv<D>(s, masked, key0, lo, hi, limit, scale_log2, f.v, acc, lane);
}

template <int D>
__device__ __forceinline__ void attn_compute8(const KVFrag8<D>& f, int key0, int lo, int hi, int limit,
                                              const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                              int lane, bool masked) {
  const float ks = exp2i(f.kexp);
  f32x16 s = {};
#pragma unroll
  for (int j = 0; j < D / 32; ++j) {
    s = mfma32(dq8(f.k[j][0], f.k[j][1], ks), qf[2 * j], s);
    s = mfma32(dq8(f.k[j][2], f.k[j][3], ks), qf[2 * j + 1], s);
  }
  bf16x8 vf[2][D / 32];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < D / 32; ++t) vf[s2][t] = dq8(f.v[s2][t][0], f.v[s2][t][1], 1.f);
  softmax_pv<D, true>(s, masked, key0, lo, hi, limit, scale_log2, vf, acc, lane, f.vexp[0], f.vexp[1]);
}

// Key blocks first, first+stride, ... < nblk (block b covers keys [base + 32 b, base + 32 b + 32)), software
// pipelined one block deep. The prefetch of the block after the last one is clamped to the last block (pad, don't
// branch: no divergent load, no extra waitcnt).
template <int D, bool FP8, typename BT = const int*>
__device__ __forceinline__ void attn_blocks(const void* __restrict__ k_cache, const void* __restrict__ v_cache,
                                            int Hkv, int kvh, const BT bt, int base, int first,
                                            int nblk, int stride, int end, int lo, int hi, int limit,
                                            const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                            int lane) {
  if (first >= nblk) return;
  using Frag = std::conditional_t<FP8, KVFrag8<D>, KVFrag<D>>;
  auto load = [&](Frag& f, int p0, int p1) {
    if constexpr (FP8)
      load_kv8<D>(f, static_cast<const uint8_t*>(k_cache), static_cast<const uint8_t*>(v_cache), Hkv, kvh, p0, p1,
                  lane);
    else
      load_kv<D>(f, static_cast<const bf16*>(k_cache), static_cast<const bf16*>(v_cache), Hkv, kvh, p0, p1, lane);
  };
  auto compute = [&](const Frag& f, int b) {
    const int key0 = base + 32 * b;
    const bool masked = (key0 < lo) | (key0 + 32 > hi) | (key0 + 31 > limit);
    if constexpr (FP8)
      attn_compute8<D>(f, key0, lo, hi, limit, qf, scale_log2, acc, lane, masked);
    else
      attn_compute<D>(f, key0, lo, hi, limit, qf, scale_log2, acc, lane, masked);
  };
  int p0, p1;
  Frag cur;
  block_pages(bt, base + 32 * first, end, p0, p1);
  load(cur, p0, p1);
  // (fp8: keeping two blocks in flight measured slower — 55.6 vs 52.0 us on the attn_bench decode case)
  for (int b = first; b < nblk; b += stride) {
    const int nb = (b + stride < nblk) ? b + stride : b;
    Frag nxt;
    block_pages(bt, base + 32 * nb, end, p0, p1);
    load(nxt, p0, p1);
    compute(cur, b);
    cur = nxt;
  }
}

template <int D>
__device__ __forceinline__ void load_q_frags(bf16x8 (&qf)[D / 16], const bf16* qrow, bool valid, int h) {
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) {
    if (valid) {
      qf[kk] = load_bf16x8(qrow + 16 * kk + 8 * h);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[kk][j] = (bf16)0.f;
    }
  }
}

template <int D>
__device__ __forceinline__ void init_acc(WaveAcc<D>& acc) {
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc.o[t][i] = 0.f;
  acc.m = -INFINITY;
  acc.l = 0.f;
}

// ------------------------------------------------------------------------------------------------------------------
// Decode: grid (work items, Hkv), 256 threads. Requires G <= 8.
// A work item is one decode row's key range [lo, hi) — the whole per-thread suffix, or one of `nsplit` pieces of a
// long one (the host sizes pieces so every workgroup streams about the same bytes: one 3k-token history no longer
// holds the whole launch while the short ones have finished). Row b's partials live at slots [0, npre) (cascade
// prefix partials written by the tile kernel, for the row's prefix group) and npre + split (this piece).
struct DecodeItem {
  int b, lo, hi, split, nsplit, npre, pad0, pad1;
};

// LDS of one decode piece (4 waves' partial results + the fused merge's per-split weights)
constexpr int DEC_MAXPG = 2048;  // page ids of one decode piece staged in LDS (longer pieces read the table)
template <int D>
struct DecodeSmem {
  int pages[DEC_MAXPG];
  bf16 qs[8][D];  // bf16: the unit's G <= 8 query heads (B operand rows), read per block instead of held in VGPRs
  float sO[4][8][D];
  float sM[4][8];
  float sL[4][8];
  float sW[8][65];
  float sWt[8];
  int s_last;
  bf16 so[8][D];  // OST: the final bf16 rows, stored from here as 16-B sc1 stores
};

// the workgroup's G final rows from sm.so to out (every thread of the workgroup calls it)
template <int D>
__device__ __forceinline__ void store_rows_sc1(DecodeSmem<D>& sm, bf16* __restrict__ out, int64_t out_stride, int b,
                                               int kvh, int G) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < G * (D / 8)) {
    const int g = t / (D / 8), c = (t % (D / 8)) * 8;
    store16_slab(reinterpret_cast<float*>(out + (int64_t)b * out_stride + (int64_t)(kvh * G + g) * D + c),
                 *reinterpret_cast<const f32x4*>(&sm.so[g][c]));
  }
}

// One decode piece: keys [lo, hi) of row b, kv head kvh, piece `split` of S, partial slots from split_offset. Every
// thread of the workgroup calls it with the same arguments (it synchronises the workgroup); returns when the
// piece's partial or final rows are written.
// OST: the final bf16 rows leave through LDS as 16-B sc1 stores (one instruction per 16 B of a row instead of one
// 8-B plain store per thread: the lines leave this XCD's L2, so the launch ends with no dirty output lines to write
// back; the o GEMM reads them on every XCD). Needs 16-B aligned rows (host-checked).
template <int D, bool FP8, bool OST = false>
__device__ __forceinline__ void decode_piece(DecodeSmem<D>& sm, const bf16* __restrict__ q, int64_t q_stride,
                                             const void* __restrict__ k_cache, const void* __restrict__ v_cache,
                                             int Hkv, int G, const int* __restrict__ block_tables, int bt_stride,
                                             int b, int kvh, int lo, int hi, int split, int S, int split_offset,
                                             float* __restrict__ out_part, float* __restrict__ lse_part, int S_total,
                                             float scale_log2, bf16* __restrict__ out, int64_t out_stride,
                                             int* __restrict__ tickets, const bf16* __restrict__ pre_bf16) {
  constexpr bool OCC3 = !FP8;  // bf16: three workgroups per CU, Q in LDS, one K/V block per wave in flight
  constexpr int MG = 32;       // prefix partials per load round trip of the fused merge
  auto& sO = sm.sO;
  auto& sM = sm.sM;
  auto& sL = sm.sL;
  auto& sW = sm.sW;
  auto& sWt = sm.sWt;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int Hq = Hkv * G;
  const int a0 = lo & ~31;
  const int nb = hi > lo ? (hi - a0 + 31) >> 5 : 0;
  const int* bt = block_tables + (int64_t)b * bt_stride;

  // the piece's page ids -> LDS (pages covering [a0, hi))
  const int pg0 = a0 >> 4;
  const int npg = nb > 0 ? ((hi - 1) >> 4) - pg0 + 1 : 0;
  const bool lds_pt = npg <= DEC_MAXPG;
  if (lds_pt)
    for (int i = threadIdx.x; i < npg; i += 256) sm.pages[i] = bt[pg0 + i];
  if constexpr (OCC3) {
    for (int i = threadIdx.x; i < G * (D / 8); i += 256) {
      const int g = i / (D / 8), c = i % (D / 8);
      *reinterpret_cast<bf16x8*>(&sm.qs[g][8 * c]) = load_bf16x8(q + (int64_t)b * q_stride + (int64_t)(kvh * G + g) * D + 8 * c);
    }
  }
  __syncthreads();
  WaveAcc<D> acc;
  init_acc<D>(acc);
  if constexpr (OCC3) {
    // Three waves per SIMD (VGPR budget 168): no Q fragments and no second K/V block in registers — each wave
    // has its one block in flight at a time, and 12 waves per CU (3 workgroups) keep the memory system fed;
    // more resident workgroups also cover each other's piece start / end.
    if (w < nb && !FP8) {
      const bool qrow = r < G;
      for (int bk = w; bk < nb; bk += 4) {
        const int key0 = a0 + 32 * bk;
        int p0, p1;
        if (lds_pt)
          block_pages(LdsPages{sm.pages, pg0}, key0, hi, p0, p1);
        else
          block_pages(bt, key0, hi, p0, p1);
        KVFrag<D> f;
        load_kv<D>(f, static_cast<const bf16*>(k_cache), static_cast<const bf16*>(v_cache), Hkv, kvh, p0, p1, lane);
        f32x16 sacc = {};
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
          bf16x8 qv = *reinterpret_cast<const bf16x8*>(&sm.qs[qrow ? r : 0][16 * kk + 8 * h]);
          if (!qrow) qv = bf16x8{};
          sacc = mfma32(f.k[kk], qv, sacc);
        }
        const bool masked = (key0 < lo) | (key0 + 32 > hi);
        softmax_pv<D>(sacc, masked, key0, lo, hi, 0x7fffffff, scale_log2, f.v, acc, lane);
      }
    }
  } else if (w < nb) {
    bf16x8 qf[D / 16];
    load_q_frags<D>(qf, q + (int64_t)b * q_stride + (int64_t)(kvh * G + r) * D, r < G, h);
    if (lds_pt)
      attn_blocks<D, FP8>(k_cache, v_cache, Hkv, kvh, LdsPages{sm.pages, pg0}, a0, w, nb, 4, hi, lo, hi, 0x7fffffff,
                          qf, scale_log2, acc, lane);
    else
      attn_blocks<D, FP8>(k_cache, v_cache, Hkv, kvh, bt, a0, w, nb, 4, hi, lo, hi, 0x7fffffff, qf, scale_log2, acc,
                          lane);
  }
  // cross-wave combine
  if (r < G) {
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int d = 32 * t + 8 * i4 + 4 * h;
        f32x4 v = {acc.o[t][4 * i4 + 0], acc.o[t][4 * i4 + 1], acc.o[t][4 * i4 + 2], acc.o[t][4 * i4 + 3]};
        *reinterpret_cast<f32x4*>(&sO[w][r][d]) = v;
      }
    if (h == 0) {
      sM[w][r] = acc.m;
      sL[w][r] = acc.l;
    }
  }
  __syncthreads();
  if (out != nullptr && S == 1) {
    // Fused merge (one split per sequence): fold in the cascade-prefix partials [0, split_offset) written earlier
    // on the stream and write the final bf16 rows — no merge kernel, no partial round trip of this split.
    // Phase 1: wave w owns heads w, w + 4: lanes load the prefix lse values in parallel, wave-reduce the max and
    // the weight sum, and publish per-split weights in LDS. Phase 2: thread (g, 4 dims) sums weight x partial over
    // the splits with all loads of a group of 8 in flight.
    for (int g = w; g < G; g += 4) {
      float Ms = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) Ms = fmaxf(Ms, sM[i][g]);
      float Ls = 0.f;
      if (Ms != -INFINITY) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Ls += exp2f(sM[i][g] - Ms) * sL[i][g];
      }
      const float ls = Ls > 0.f ? Ms + log2f(Ls) : -INFINITY;
      const int64_t pbase = ((int64_t)b * Hq + kvh * G + g) * S_total;
      float lp = -INFINITY;
      if (lane < split_offset) lp = lse_part[pbase + lane];
      const float lv = lane < split_offset ? lp : (lane == split_offset ? ls : -INFINITY);
      float mx = lv;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float wv = mx == -INFINITY ? 0.f : exp2f(lv - mx);
      float ws = wv;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
      if (lane <= split_offset) sW[g][lane] = wv;
      if (lane == 0) sWt[g] = ws;
    }
    __syncthreads();
    const int g = threadIdx.x >> 5, c = (threadIdx.x & 31) * 4;
    if (g < G) {
      // this workgroup's own (normalised) result for dims c..c+3
      float Ms = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) Ms = fmaxf(Ms, sM[i][g]);
      f32x4 os = {0.f, 0.f, 0.f, 0.f};
      float Ls = 0.f;
      if (Ms != -INFINITY) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float f = exp2f(sM[i][g] - Ms);
          Ls += f * sL[i][g];
          os += *reinterpret_cast<const f32x4*>(&sO[i][g][c]) * f;
        }
      }
      f32x4 acc4 = Ls > 0.f ? os * (sW[g][split_offset] / Ls) : f32x4{0.f, 0.f, 0.f, 0.f};
      const int64_t pbase = ((int64_t)b * Hq + kvh * G + g) * S_total * D + c;
      int s2 = 0;
      // MG prefix partials per round trip (the cascade writes 32 per row: 2 round trips at MG = 16, 4 at 8)
      if (pre_bf16 != nullptr) {  // bf16 cascade partials (tile v3): half the bytes of the fp32 round trip
        const bf16* pb = pre_bf16 + pbase;
        for (; s2 + MG <= split_offset; s2 += MG) {
          bf16x4 v[MG];
#pragma unroll
          for (int j = 0; j < MG; ++j) v[j] = *reinterpret_cast<const bf16x4*>(pb + (s2 + j) * D);
#pragma unroll
          for (int j = 0; j < MG; ++j) {
            const float wj = sW[g][s2 + j];
            acc4 += f32x4{(float)v[j][0], (float)v[j][1], (float)v[j][2], (float)v[j][3]} * wj;
          }
        }
        for (; s2 < split_offset; ++s2) {
          const bf16x4 v = *reinterpret_cast<const bf16x4*>(pb + s2 * D);
          acc4 += f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]} * sW[g][s2];
        }
      } else {
        const float* pp = out_part + pbase;
        for (; s2 + MG <= split_offset; s2 += MG) {
          f32x4 v[MG];
#pragma unroll
          for (int j = 0; j < MG; ++j) v[j] = *reinterpret_cast<const f32x4*>(pp + (s2 + j) * D);
#pragma unroll
          for (int j = 0; j < MG; ++j) acc4 += v[j] * sW[g][s2 + j];
        }
        for (; s2 < split_offset; ++s2) {
          acc4 += *reinterpret_cast<const f32x4*>(pp + s2 * D) * sW[g][s2];
        }
      }
      const float inv = sWt[g] > 0.f ? 1.f / sWt[g] : 0.f;
      bf16x4 o4;
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = (bf16)(acc4[j] * inv);
      if constexpr (OST)
        *reinterpret_cast<bf16x4*>(&sm.so[g][c]) = o4;
      else
        *reinterpret_cast<bf16x4*>(out + (int64_t)b * out_stride + (int64_t)(kvh * G + g) * D + c) = o4;
    }
    if constexpr (OST) store_rows_sc1<D>(sm, out, out_stride, b, kvh, G);
    return;
  }
  if (out != nullptr) {
    // ticket merge: each split's partial row leaves as 16-B write-through (sc1, agent-coherent) stores — 4-B ones
    // cost several times more per byte — and the last workgroup reads it back with 16-B sc1 loads (ld4 below)
    for (int idx4 = threadIdx.x; idx4 < G * D / 4; idx4 += 256) {
      const int g = idx4 / (D / 4), d0 = (idx4 % (D / 4)) * 4;
      float M = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) M = fmaxf(M, sM[i][g]);
      float L = 0.f;
      f32x4 O4 = {0.f, 0.f, 0.f, 0.f};
      if (M != -INFINITY) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float f = exp2f(sM[i][g] - M);
          L += f * sL[i][g];
#pragma unroll
          for (int j = 0; j < 4; ++j) O4[j] += f * sO[i][g][d0 + j];
        }
      }
      const int64_t pidx = ((int64_t)b * Hq + kvh * G + g) * S_total + split_offset + split;
      const float inv = L > 0.f ? 1.f / L : 0.f, lv = L > 0.f ? M + log2f(L) : -INFINITY;
      f32x4 ov4;
#pragma unroll
      for (int j = 0; j < 4; ++j) ov4[j] = L > 0.f ? O4[j] * inv : 0.f;
      store16_slab(out_part + pidx * D + d0, ov4);
      if (d0 == 0) __hip_atomic_store(lse_part + pidx, lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) M = fmaxf(M, sM[i][g]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float f = exp2f(sM[i][g] - M);
        L += f * sL[i][g];
        O += f * sO[i][g][d];
      }
    }
    const int64_t pidx = ((int64_t)b * Hq + kvh * G + g) * S_total + split_offset + split;
    const float ov = L > 0.f ? O / L : 0.f, lv = L > 0.f ? M + log2f(L) : -INFINITY;
    if (out == nullptr) {
      out_part[pidx * D + d] = ov;
      if (d == 0) lse_part[pidx] = lv;
    } else {  // ticket merge: write-through (agent-coherent) stores, no L2-wide write-back fence needed
      __hip_atomic_store(out_part + pidx * D + d, ov, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) __hip_atomic_store(lse_part + pidx, lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (out == nullptr) return;
  // Ticket merge (S > 1, e.g. one long sequence spread over many workgroups): every split publishes its partial
  // with agent-coherent write-through stores (another XCD's workgroup may read it; a __threadfence release here
  // would write back the whole L2 from every workgroup), waits for them, takes a ticket, and the LAST of the S
  // workgroups of (b, kvh) merges all split_offset + S partials (agent-coherent loads) and writes the bf16 rows —
  // no merge kernel launch. The last one also re-arms the counter for the next launch.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* tk = tickets + b * Hkv + kvh;
    const int t = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm.s_last = t == S - 1;
    if (t == S - 1) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!sm.s_last) return;
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  // 16-B agent-coherent loads (sc1: not served from this XCD's possibly stale L2) as compiler builtins over a buffer
  // of out_part, so hipcc's waitcnt pass tracks them (out_part < 2 GiB: host-checked)
  const auto prs = buf_rsrc(out_part);
  auto ld4 = [&](const float* p) { return load16_sc1(prs, (int)((p - out_part) * 4)); };
  const int n = split_offset + S;  // <= 64 (host-checked)
  for (int g = w; g < G; g += 4) {
    const int64_t pbase = ((int64_t)b * Hq + kvh * G + g) * S_total;
    const float lv = lane < n ? ld(lse_part + pbase + lane) : -INFINITY;
    float mx = lv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const float wv = mx == -INFINITY ? 0.f : exp2f(lv - mx);
    float ws = wv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
    if (lane < n) sW[g][lane] = wv;
    if (lane == 0) sWt[g] = ws;
  }
  __syncthreads();
  const int g = threadIdx.x >> 5, c = (threadIdx.x & 31) * 4;
  if (g < G) {
    f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
    const float* pp = out_part + ((int64_t)b * Hq + kvh * G + g) * S_total * D + c;
    const int p0 = pre_bf16 != nullptr ? split_offset : 0;  // first fp32 slot (the pieces, or every slot)
    // one round trip for the common row: the first PQ fp32 slots (agent-coherent loads) and MG bf16 prefix slots
    // are all in flight before the first wait (was: the prefix batch, then the pieces batch — two tail latencies)
    constexpr int PQ = 8;
    f32x4 pv[PQ];
#pragma unroll
    for (int j = 0; j < PQ; ++j) pv[j] = ld4(pp + min(p0 + j, n - 1) * D);
    int s0 = 0;
    if (pre_bf16 != nullptr) {  // the cascade's bf16 prefix partials, MG loads per round trip (as the one-piece path)
      const bf16* pb = pre_bf16 + ((int64_t)b * Hq + kvh * G + g) * S_total * D + c;
      for (; s0 + MG <= split_offset; s0 += MG) {
        bf16x4 v[MG];
#pragma unroll
        for (int j = 0; j < MG; ++j) v[j] = *reinterpret_cast<const bf16x4*>(pb + (s0 + j) * D);
#pragma unroll
        for (int j = 0; j < MG; ++j) {
          const float wj = sW[g][s0 + j];
          acc4 += f32x4{(float)v[j][0], (float)v[j][1], (float)v[j][2], (float)v[j][3]} * wj;
        }
      }
      for (; s0 < split_offset; ++s0) {
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(pb + s0 * D);
        acc4 += f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]} * sW[g][s0];
      }
    }
#pragma unroll
    for (int j = 0; j < PQ; ++j)
      if (p0 + j < n) acc4 += pv[j] * sW[g][p0 + j];
    // rows with more pieces: groups of 16 with all loads in flight (the tail of the kernel: latency, not bandwidth)
    for (int s2 = p0 + PQ; s2 < n; s2 += 16) {
      f32x4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = ld4(pp + min(s2 + j, n - 1) * D);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (s2 + j < n) acc4 += v[j] * sW[g][s2 + j];
    }
    const float inv = sWt[g] > 0.f ? 1.f / sWt[g] : 0.f;
    bf16x4 o4;
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = (bf16)(acc4[j] * inv);
    if constexpr (OST)
      *reinterpret_cast<bf16x4*>(&sm.so[g][c]) = o4;
    else
      *reinterpret_cast<bf16x4*>(out + (int64_t)b * out_stride + (int64_t)(kvh * G + g) * D + c) = o4;
  }
  if constexpr (OST) store_rows_sc1<D>(sm, out, out_stride, b, kvh, G);
}

// Prefill rows merged by the decode launch (grid rows past the decode items): a step whose new-turn rows rode in the
// cascade launch (prefix AND own keys, model_runner join_suffix) has no prefill launch left, only the log-sum-exp
// merge of those rows' fp32 partials — done by extra workgroups of this launch instead of an attn_merge launch of its
// own (one kernel boundary and ramp less per layer). Workgroup (kvh, n_items + m): rows RPW m .. RPW m + RPW - 1,
// heads kvh G .. kvh G + G - 1, 32 lanes x float4 columns per (row, head) as attn_merge_kernel.
struct FusedMerge {
  const float* part = nullptr;  // [rows, Hq, S, 128]
  const float* lse = nullptr;   // [rows, Hq, S]
  int S = 0;
  int rows = 0;
  bf16* out = nullptr;          // row r at out + r * out_stride
  int64_t out_stride = 0;
};

__device__ __forceinline__ void fused_merge_rows(const FusedMerge& fm, int m, int kvh, int G, int Hq) {
  constexpr int D = 128;
  const int t = threadIdx.x >> 5, rpw = (8 % G == 0) ? 8 / G : 1;
  const int rr = t / G, row = m * rpw + rr;
  if (rr >= rpw || row >= fm.rows) return;
  const int hh = kvh * G + t % G, c = (threadIdx.x & 31) * 4, S = fm.S;
  const float* l = fm.lse + ((int64_t)row * Hq + hh) * S;
  const float* p = fm.part + ((int64_t)row * Hq + hh) * S * D + c;
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, l[s]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float L = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < S; ++s) {
      const float w = exp2f(l[s] - M);
      if (w > 0.f) acc += *reinterpret_cast<const f32x4*>(p + s * D) * w;  // (an unwritten slot has lse -inf)
      L += w;
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  bf16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (bf16)(acc[j] * inv);
  *reinterpret_cast<bf16x4*>(fm.out + (int64_t)row * fm.out_stride + (int64_t)hh * D + c) = o;
}

// grid (Hkv, items [+ merge workgroups]): the Hkv heads of an item are consecutive workgroups, dealt to different
// XCDs, reading one page row together (heads-fast: +7 % over items-fast, three workgroups per CU +5 % over two,
// profiles/r04/bench_ab_decode_placement_occ.jsonl)
template <int D, bool FP8, bool OST = false>
__global__ __launch_bounds__(256, FP8 ? 2 : 3) void attn_decode_kernel(const bf16* __restrict__ q, int64_t q_stride,
                                                                      const void* __restrict__ k_cache,
                                                                      const void* __restrict__ v_cache, int Hkv, int G,
                                                                      const int* __restrict__ block_tables,
                                                                      int bt_stride,
                                                                      const DecodeItem* __restrict__ items, int B,
                                                                      float* __restrict__ out_part,
                                                                      float* __restrict__ lse_part, int S_total,
                                                                      float scale_log2, bf16* __restrict__ out,
                                                                      int64_t out_stride, int* __restrict__ tickets,
                                                                      const bf16* __restrict__ pre_bf16, int n_items,
                                                                      FusedMerge fm) {
  __shared__ DecodeSmem<D> sm;
  if ((int)blockIdx.y >= n_items) {  // (workgroup-uniform)
    fused_merge_rows(fm, blockIdx.y - n_items, blockIdx.x, G, Hkv * G);
    return;
  }
  const DecodeItem it = items[blockIdx.y];
  const int b = it.b, kvh = blockIdx.x, split = it.split, S = it.nsplit, split_offset = it.npre;
  // a malformed item (host bug) is dropped instead of indexing out of bounds (workgroup-uniform)
  if (b < 0 || b >= B || split < 0 || split >= S || split_offset < 0 || split_offset + S > S_total ||
      (out != nullptr && split_offset + S > 64))
    return;
  decode_piece<D, FP8, OST>(sm, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, b, kvh, it.lo, it.hi,
                       split, S, split_offset, out_part, lse_part, S_total, scale_log2, out, out_stride, tickets,
                       pre_bf16);
}

// ------------------------------------------------------------------------------------------------------------------
// Prefill / cascade: grid (Hkv, num_items), 256 or 512 threads; wave w owns tile rows [32w, 32w+32), row R -> token R / G,
// head kvh*G + R % G.
// LDS staging for the tile kernel: every 32-key block is loaded ONCE per workgroup (256 threads x 4 x 16 B) and
// read by all 4 waves from LDS, instead of once per wave from L2 (the 4 waves own different query rows but need the
// same keys). Two 16 KB buffers; the global loads of block b+1 are issued before the MFMAs of block b and written to
// LDS after them (issue-early / write-late), one barrier per block.
//   K tile  [32 keys][128 d] bf16, 256-B rows, 16-B chunk c of key k stored at chunk c ^ (k & 15) (XOR swizzle:
//           the A-fragment reads of 16 lanes on 16 different keys hit 16 different bank groups)
//   V tile  [2 pages][128 d][16 pos] bf16, 32-B rows, 16-B half j of row d stored at half j ^ ((d >> 3) & 1)
constexpr int KT_BYTES = 32 * 128 * 2;
constexpr int VT_BYTES = 2 * 128 * 16 * 2;
constexpr int STAGE_BYTES = KT_BYTES + VT_BYTES;
constexpr int MAX_STAGED_PAGES = 2048;
#ifndef ATTN_PREFETCH
#define ATTN_PREFETCH 2  // K/V blocks in flight per workgroup (4 measured no faster: not latency-bound)
#endif  // keys [base, base + 32k) have their page ids staged in LDS

// NT threads stage one block: K 512 chunks + V 512 chunks of 16 B -> 1024 / NT chunks of each per thread.
template <int NT>
struct StageRegs {
  bf16x8 k[512 / NT];
  bf16x8 v[512 / NT];
};

// Staging loads are issued with inline asm so hipcc's waitcnt pass does not see them: it would otherwise drain
// vmcnt(0) before the LDS store of the OLDER register stage and collapse the 2-deep prefetch to 1 (ROCm 7.2). The
// loop waits for them itself with a counted `s_waitcnt vmcnt(N)` (N = loads of the younger stage still in flight).
__device__ __forceinline__ bf16x8 asm_load16(const bf16* p) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  i32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return __builtin_bit_cast(bf16x8, r);
}

template <int NT>
__device__ __forceinline__ void stage_load(StageRegs<NT>& sr, const bf16* __restrict__ k_cache,
                                           const bf16* __restrict__ v_cache, int Hkv, int kvh, int p0, int p1,
                                           int tid) {
  constexpr int D = 128;
#pragma unroll
  for (int i = 0; i < 512 / NT; ++i) {
    const int qd = tid + NT * i;
    // K: 16-B piece qd & 255 of page qd >> 8 (= chunk plane (qd >> 4) & 15, key qd & 15): contiguous per wave
    const int page = (qd >> 8) ? p1 : p0;
    sr.k[i] = asm_load16(k_cache + ((int64_t)page * Hkv + kvh) * (PAGE * D) + (qd & 255) * 8);
    const int vp = (qd >> 8) ? p1 : p0;
    sr.v[i] = asm_load16(v_cache + ((int64_t)vp * Hkv + kvh) * (D * PAGE) + (qd & 255) * 8);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n * L) for a wave-uniform runtime n in [0, MAXN] (the count must be an immediate)
template <int L, int MAXN>
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  if constexpr (MAXN >= 5) if (n >= 5) { wait_vmcnt<5 * L>(); return; }
  if constexpr (MAXN >= 4) if (n == 4) { wait_vmcnt<4 * L>(); return; }
  if constexpr (MAXN >= 3) if (n == 3) { wait_vmcnt<3 * L>(); return; }
  if constexpr (MAXN >= 2) if (n == 2) { wait_vmcnt<2 * L>(); return; }
  if constexpr (MAXN >= 1) if (n == 1) { wait_vmcnt<1 * L>(); return; }
  wait_vmcnt<0>();
}

// fp8 staging: 512 16-B chunks per 32-key block — K units [0, 256) (page qd >> 7, unit qd & 127 = plane p, key o)
// and V^T rows [256, 512) (page (qd - 256) >> 7, d = qd & 127) — plus one aux load each (the dword holding the K
// unit's key exponent; the page's 16 V exponents), so every thread issues the same 2 * 512 / NT loads as bf16.
template <int NT>
struct StageRegs8 {
  u32x4 c[512 / NT];
  u32x4 aux[512 / NT];
};

__device__ __forceinline__ uint32_t asm_load4(const uint8_t* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

template <int NT>
__device__ __forceinline__ void stage_load8(StageRegs8<NT>& sr, const uint8_t* __restrict__ k_cache,
                                            const uint8_t* __restrict__ v_cache, int Hkv, int kvh, int p0, int p1,
                                            int tid) {
#pragma unroll
  for (int i = 0; i < 512 / NT; ++i) {
    const int qd = tid + NT * i;
    if (qd < 256) {  // wave-uniform (NT = 512: waves 0-3; NT = 256: i == 0)
      const uint8_t* kb = k_cache + ((int64_t)((qd >> 7) ? p1 : p0) * Hkv + kvh) * KPAGE8;
      sr.c[i] = __builtin_bit_cast(u32x4, asm_load16(reinterpret_cast<const bf16*>(kb + (qd & 127) * 16)));
      sr.aux[i][0] = asm_load4(kb + KEXP8 + (qd & 12));
    } else {
      const int vq = qd - 256, page = (vq >> 7) ? p1 : p0;
      sr.c[i] = __builtin_bit_cast(
          u32x4, asm_load16(reinterpret_cast<const bf16*>(v_cache + ((int64_t)page * Hkv + kvh) * VPAGE8 + (vq & 127) * 16)));
      sr.aux[i] = __builtin_bit_cast(
          u32x4, asm_load16(reinterpret_cast<const bf16*>(k_cache + ((int64_t)page * Hkv + kvh) * KPAGE8 + VEXP8)));
    }
  }
}

template <int NT>
__device__ __forceinline__ void stage_store8(const StageRegs8<NT>& sr, char* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 512 / NT; ++i) {
    const int qd = tid + NT * i;
    const u32x4 w = sr.c[i];
    if (qd < 256) {
      const int pc = qd & 127, p = pc >> 4, o = pc & 15, key = ((qd >> 7) << 4) | o;
      const float sc = exp2i(__builtin_amdgcn_sbfe(sr.aux[i][0], 8 * (o & 3), 8));
      const int c1 = 4 * (p >> 1) + (p & 1);  // d chunk (8 elements) of the unit's first half; second = c1 + 2
      *reinterpret_cast<bf16x8*>(lds + key * 256 + 16 * (c1 ^ (key & 15))) = dq8(w[0], w[1], sc);
      *reinterpret_cast<bf16x8*>(lds + key * 256 + 16 * ((c1 + 2) ^ (key & 15))) = dq8(w[2], w[3], sc);
    } else {
      const int vq = qd - 256, pg = vq >> 7, d = vq & 127;
      char* row = lds + KT_BYTES + pg * 4096 + d * 32;
      *reinterpret_cast<bf16x8*>(row + 16 * (0 ^ ((d >> 3) & 1))) = dq8(w[0], w[1], 1.f);
      *reinterpret_cast<bf16x8*>(row + 16 * (1 ^ ((d >> 3) & 1))) = dq8(w[2], w[3], 1.f);
      if (d == 0) *reinterpret_cast<u32x4*>(lds + KT_BYTES + VT_BYTES + pg * 16) = sr.aux[i];
    }
  }
}

template <int NT>
__device__ __forceinline__ void stage_store(const StageRegs<NT>& sr, char* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 512 / NT; ++i) {
    const int qd = tid + NT * i;
    const int key = ((qd >> 8) << 4) | (qd & 15), c = (qd >> 4) & 15;
    *reinterpret_cast<bf16x8*>(lds + key * 256 + 16 * (c ^ (key & 15))) = sr.k[i];
    const int vq = qd & 255, d = vq >> 1, half = vq & 1;
    *reinterpret_cast<bf16x8*>(lds + KT_BYTES + (qd >> 8) * 4096 + d * 32 + 16 * (half ^ ((d >> 3) & 1))) =
        sr.v[i];
  }
}

// One 32-key step reading K/V fragments from an LDS stage. All 8 K-fragment reads are issued before the first
// QK^T MFMA and all 8 V-fragment reads right behind the QK^T MFMAs (sched_barrier pins the order; left alone hipcc
// issues one ds_read at a time, each waited with lgkmcnt(0) before its MFMA).
template <int D, bool FP8>
__device__ __forceinline__ void attn_compute_lds(const char* lds, int key0, int lo, int hi, int limit,
                                                 const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                                 int lane, bool masked) {
  const int r = lane & 31, h = lane >> 5;
  bf16x8 kf[D / 16];
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk)
    kf[kk] = *reinterpret_cast<const bf16x8*>(lds + r * 256 + 16 * ((2 * kk + h) ^ (r & 15)));
  __builtin_amdgcn_sched_barrier(0);
  f32x16 s = {};
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) s = mfma32(kf[kk], qf[kk], s);
  bf16x8 vf[2][D / 32];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < D / 32; ++t) {
      const int d = 32 * t + r;
      vf[s2][t] = *reinterpret_cast<const bf16x8*>(lds + KT_BYTES + s2 * 4096 + d * 32 + 16 * (h ^ ((d >> 3) & 1)));
    }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (FP8) {
    const char* ve = lds + KT_BYTES + VT_BYTES + 8 * h;
    softmax_pv<D, true>(s, masked, key0, lo, hi, limit, scale_log2, vf, acc, lane,
                        *reinterpret_cast<const u32x2*>(ve), *reinterpret_cast<const u32x2*>(ve + 16));
  } else {
    softmax_pv<D>(s, masked, key0, lo, hi, limit, scale_log2, vf, acc, lane);
  }
}

template <int D, int NW, bool LDS, bool FP8>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_prefill_kernel(const AttnWorkItem* __restrict__ items,
                                                            const bf16* __restrict__ q, int64_t q_stride,
                                                            const void* __restrict__ k_cache,
                                                            const void* __restrict__ v_cache, int Hkv, int G,
                                                            const int* __restrict__ block_tables, int bt_stride,
                                                            const int* __restrict__ q_limit, bf16* __restrict__ out,
                                                            int64_t out_stride, float* __restrict__ out_part,
                                                            float* __restrict__ lse_part, int S_total,
                                                            float scale_log2) {
  // grid (Hkv, items): the Hkv heads of an item are consecutive workgroups, so a launch longer than one round of the
  // CUs starts the host's longest-first items on every head before any short one (and an item's heads read the same
  // pages together)
  const AttnWorkItem it = items[blockIdx.y];
  const int kvh = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int Hq = Hkv * G;
  const int R = w * 32 + r;
  const int tok = R / G, g = R % G;
  const bool valid = tok < it.q_count;
  const int token = it.q_start + tok;
  const int limit = valid ? q_limit[token] : -1;
  const int* bt = block_tables + (int64_t)it.bt_row * bt_stride;
  // LDS variant: the Q fragments and the page ids of the item's key range are requested here, together with
  // q_limit, so the prologue pays one memory round trip for all three instead of one each
  constexpr int SB = FP8 ? STAGE_BYTES + 32 : STAGE_BYTES;  // fp8: + the two pages' V exponents
  __shared__ __attribute__((aligned(16))) char lds[LDS ? 2 * SB : 16];
  __shared__ int s_hi[NW];
  __shared__ int s_pages[LDS ? MAX_STAGED_PAGES : 1];
  bf16x8 qf[D / 16];
  if constexpr (LDS) {
    load_q_frags<D>(qf, q + (int64_t)token * q_stride + (int64_t)(kvh * G + g) * D, valid, h);
    // (the host never builds an LDS-variant item spanning more than MAX_STAGED_PAGES pages: model_runner splits
    // longer key ranges; a violating item produces NaN instead of reading out of bounds)
    const int pg0 = (it.kv_lo & ~31) >> 4;
    const int npg = min(((it.kv_hi + 15) >> 4) - pg0, MAX_STAGED_PAGES);
    for (int i = threadIdx.x; i < npg; i += NW * 64) s_pages[i] = bt[pg0 + i];
  }
  // wave-uniform key range
  int wmax = limit;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o, 64));
  int wmin = valid ? limit : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmin = min(wmin, __shfl_xor(wmin, o, 64));
  const int lo = it.kv_lo;
  const int hi = min(it.kv_hi, wmax + 1);

  WaveAcc<D> acc;
  init_acc<D>(acc);
  if constexpr (!LDS) {
    if (hi > lo) {
      load_q_frags<D>(qf, q + (int64_t)token * q_stride + (int64_t)(kvh * G + g) * D, valid, h);
      const int base = lo & ~31;
      attn_blocks<D, FP8>(k_cache, v_cache, Hkv, kvh, bt, base, 0, (hi - base + 31) >> 5, 1, hi, lo, hi, limit,
                          qf, scale_log2, acc, lane);
    }
  } else {
    if (lane == 0) s_hi[w] = hi;
    __syncthreads();
    int hi_wg = s_hi[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) hi_wg = max(hi_wg, s_hi[i]);
    if (hi_wg > lo) {  // workgroup-uniform
      // retire the Q loads here: otherwise hipcc keeps a vmcnt(0) for them inside the loop, which would also
      // drain the (compiler-invisible) staging loads every block
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) asm volatile("" ::"v"(qf[kk]));
      const int base = lo & ~31;
      const int nblk = (hi_wg - base + 31) >> 5;
      const int tid = threadIdx.x;
      constexpr int LOADS = 2 * (512 / (NW * 64));  // asm loads per register stage per thread
      // page indices of the item's key range were staged in LDS in the prologue (published by the s_hi barrier):
      // no scalar global load (and no lgkmcnt(0) on it) inside the block loop
      const int pg0 = base >> 4;
      const int npg = ((hi_wg + 15) >> 4) - pg0;
      const bool fits = npg <= MAX_STAGED_PAGES;
      auto pages_of = [&](int key0, int& a, int& b2) {
        const int i0 = min((key0 >> 4) - pg0, MAX_STAGED_PAGES - 2);
        a = s_pages[i0];
        b2 = (key0 + 16 < hi_wg) ? s_pages[i0 + 1] : a;
      };
      if (!fits) acc.m = acc.l = __builtin_nanf("");
      // PF register stages in flight: block j is loaded into stage j % PF, PF blocks ahead of the one being
      // computed, and written to LDS (double buffer) right before it is needed. (PF = 4 measured the same as 2 on
      // the cascade pass, profiles/README.md: the kernel is not waiting on HBM latency.)
      constexpr int PF = ATTN_PREFETCH;
      using Regs = std::conditional_t<FP8, StageRegs8<NW * 64>, StageRegs<NW * 64>>;
      auto sload = [&](Regs& r2, int a, int b2) {
        if constexpr (FP8)
          stage_load8<NW * 64>(r2, static_cast<const uint8_t*>(k_cache), static_cast<const uint8_t*>(v_cache), Hkv,
                               kvh, a, b2, tid);
        else
          stage_load<NW * 64>(r2, static_cast<const bf16*>(k_cache), static_cast<const bf16*>(v_cache), Hkv, kvh, a,
                              b2, tid);
      };
      auto sstore = [&](const Regs& r2, char* dst) {
        if constexpr (FP8)
          stage_store8<NW * 64>(r2, dst, tid);
        else
          stage_store<NW * 64>(r2, dst, tid);
      };
      Regs rs[PF];
      int p0, p1;
      pages_of(base, p0, p1);
      sload(rs[0], p0, p1);
      wait_vmcnt<0>();
      sstore(rs[0], lds);
#pragma unroll
      for (int j = 1; j <= PF; ++j) {
        if (j < nblk) {
          pages_of(base + 32 * j, p0, p1);
          sload(rs[j % PF], p0, p1);
        }
      }
      __syncthreads();
      // J = b % PF (compile time, so the stage registers are statically indexed)
      auto body = [&](auto Jc, int b) {
        constexpr int J = decltype(Jc)::value;
        const int key0 = base + 32 * b;
        if (key0 < hi) {  // wave-uniform: skip blocks past this wave's causal limit
          const bool masked = (key0 < lo) | (key0 + 32 > hi) | (key0 + 31 > wmin);
          attn_compute_lds<D, FP8>(lds + (b & 1) * SB, key0, lo, hi, limit, qf, scale_log2, acc, lane, masked);
        }
        if (b + 1 < nblk) {
          // stage (J+1) % PF holds block b+1; blocks b+2 .. min(b+PF, nblk-1) may still be in flight behind it
          const int younger = min(PF - 1, nblk - 2 - b);
          wait_vmcnt_dyn<LOADS, PF - 1>(younger);
          sstore(rs[(J + 1) % PF], lds + ((b + 1) & 1) * SB);
          if (b + 1 + PF < nblk) {
            pages_of(key0 + 32 * (1 + PF), p0, p1);
            sload(rs[(J + 1) % PF], p0, p1);
          }
        }
        __syncthreads();
      };
      for (int b = 0; b < (fits ? nblk : 0); b += PF) {
        body(std::integral_constant<int, 0>{}, b);
        if constexpr (PF > 1) if (b + 1 < nblk) body(std::integral_constant<int, 1 % PF>{}, b + 1);
        if constexpr (PF > 2) if (b + 2 < nblk) body(std::integral_constant<int, 2 % PF>{}, b + 2);
        if constexpr (PF > 3) if (b + 3 < nblk) body(std::integral_constant<int, 3 % PF>{}, b + 3);
        if constexpr (PF > 4) if (b + 4 < nblk) body(std::integral_constant<int, 4 % PF>{}, b + 4);
        if constexpr (PF > 5) if (b + 5 < nblk) body(std::integral_constant<int, 5 % PF>{}, b + 5);
      }
    }
  }
  const int head = kvh * G + g;
  if constexpr (LDS && D == 128) {
    // Output through a per-wave LDS transpose. The accumulators hold one (token, head) row per lane pair, 16 B per
    // lane per d-chunk, and consecutive rows lie a whole partial slab apart ((token * Hq + head) * S_total): stored
    // straight from registers every instruction writes 32 B into 32 different lines (the cascade pass's 32 MB of
    // partials then took ~10 us of its ~39). Through LDS each store instruction writes 8 whole 128-B row lines.
    // Every wave has its own 4 KB slice of the (now idle) stage buffers; rows are 128 B with 16-B chunks XOR-swizzled
    // by row. fp32 partials: 4 rounds of 32 d; bf16 output: 2 rounds of 64 d.
    if (!__any(valid)) return;  // wave-uniform
    const bool part = it.split >= 0;
    const float inv = acc.l > 0.f ? 1.f / acc.l : 0.f;
    if (part && valid && h == 0)
      lse_part[((int64_t)token * Hq + head) * S_total + it.split] = acc.l > 0.f ? acc.m + log2f(acc.l) : -INFINITY;
    char* slab = lds + w * 4096;
    const int nvalid = it.q_count * G - w * 32;  // rows of this wave below it (uniform)
    const int cc = lane & 7;
    // read back 4 rows x 16 B per lane (8 lanes = one 128-B row line) and store them
    auto flush = [&](int rd) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = (lane >> 3) + 8 * k;
        const f32x4 v = *reinterpret_cast<const f32x4*>(slab + row * 128 + 16 * (cc ^ (row & 7)));
        if (row < nvalid) {
          const int R2 = w * 32 + row, tok2 = it.q_start + R2 / G, head2 = kvh * G + R2 % G;
          if (part)
            *reinterpret_cast<f32x4*>(out_part + (((int64_t)tok2 * Hq + head2) * S_total + it.split) * D + 32 * rd +
                                      4 * cc) = v;
          else
            *reinterpret_cast<f32x4*>(out + (int64_t)tok2 * out_stride + (int64_t)head2 * D + 64 * rd + 8 * cc) = v;
        }
      }
    };
    if (part) {
#pragma unroll
      for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int c = 2 * i4 + h;
          f32x4 v = {acc.o[rd][4 * i4] * inv, acc.o[rd][4 * i4 + 1] * inv, acc.o[rd][4 * i4 + 2] * inv,
                     acc.o[rd][4 * i4 + 3] * inv};
          *reinterpret_cast<f32x4*>(slab + r * 128 + 16 * (c ^ (r & 7))) = v;
        }
        flush(rd);
      }
    } else {
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int i4 = 0; i4 < 4; ++i4) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(acc.o[2 * rd + tt][4 * i4 + j] * inv);
            *reinterpret_cast<bf16x4*>(slab + r * 128 + 16 * ((4 * tt + i4) ^ (r & 7)) + 8 * h) = v;
          }
        flush(rd);
      }
    }
    return;
  }
  if (!valid) return;
  if (it.split < 0) {
    const float inv = acc.l > 0.f ? 1.f / acc.l : 0.f;
    bf16* orow = out + (int64_t)token * out_stride + (int64_t)head * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int d = 32 * t + 8 * i4 + 4 * h;
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (bf16)(acc.o[t][4 * i4 + j] * inv);
        *reinterpret_cast<bf16x4*>(orow + d) = v;
      }
  } else {
    const int64_t pidx = ((int64_t)token * Hq + head) * S_total + it.split;
    const float inv = acc.l > 0.f ? 1.f / acc.l : 0.f;
    float* prow = out_part + pidx * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const int d = 32 * t + 8 * i4 + 4 * h;
        f32x4 v = {acc.o[t][4 * i4] * inv, acc.o[t][4 * i4 + 1] * inv, acc.o[t][4 * i4 + 2] * inv,
                   acc.o[t][4 * i4 + 3] * inv};
        *reinterpret_cast<f32x4*>(prow + d) = v;
      }
    if (h == 0) lse_part[pidx] = acc.l > 0.f ? acc.m + log2f(acc.l) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------------------------------------------
// Merge S partials: grid (rows, ceil(Hq / 8)), 256 threads = 8 heads x 32 lanes x float4 columns. Each lane
// recomputes its head's max / sum over the S lse values (L1-resident broadcast reads), then accumulates its 4 columns.
constexpr int MERGE_MAX_S = 256;
// pre (optional): slots [0, npre) are read from this bf16 buffer of part's layout instead (the cascade's prefix
// partials, tile v3 part_bf16)
template <int D>
__global__ __launch_bounds__(256) void attn_merge_kernel(const float* __restrict__ part, const float* __restrict__ lse,
                                                          int S, bf16* __restrict__ out, int64_t out_stride, int Hq,
                                                          float* __restrict__ lse_out, const bf16* __restrict__ pre,
                                                          int npre) {
  static_assert(D == 128, "merge maps 32 lanes x float4 onto one head");
  const int64_t row = blockIdx.x;
  const int hh = blockIdx.y * 8 + (threadIdx.x >> 5);
  if (hh >= Hq) return;
  const int c = (threadIdx.x & 31) * 4;
  const float* l = lse + (row * Hq + hh) * S;
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, l[s]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float L = 0.f;
  if (M != -INFINITY) {
    const float* p = part + ((row * Hq + hh) * S) * D + c;
    int s = 0;
    // a slot with lse = -inf (a row with fewer pieces than S) has weight 0 and was never written: select it away
    // instead of multiplying (0 x a stale NaN is NaN)
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if (pre != nullptr) {
      const bf16* pb = pre + ((row * Hq + hh) * S) * D + c;
      auto pre_at = [&](int s2, float w) {
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(pb + s2 * D);
        return w > 0.f ? f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]} * w : z;
      };
      for (; s + 4 <= npre; s += 4) {
        const float w0 = exp2f(l[s] - M), w1 = exp2f(l[s + 1] - M), w2 = exp2f(l[s + 2] - M),
                    w3 = exp2f(l[s + 3] - M);
        acc += pre_at(s, w0) + pre_at(s + 1, w1) + pre_at(s + 2, w2) + pre_at(s + 3, w3);
        L += (w0 + w1) + (w2 + w3);
      }
      for (; s < npre; ++s) {
        const float w0 = exp2f(l[s] - M);
        acc += pre_at(s, w0);
        L += w0;
      }
    }
    auto part_at = [&](int s2, float w) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(p + s2 * D);
      return w > 0.f ? a * w : z;
    };
    for (; s + 4 <= S; s += 4) {
      const float w0 = exp2f(l[s] - M), w1 = exp2f(l[s + 1] - M), w2 = exp2f(l[s + 2] - M),
                  w3 = exp2f(l[s + 3] - M);
      acc += part_at(s, w0) + part_at(s + 1, w1) + part_at(s + 2, w2) + part_at(s + 3, w3);
      L += (w0 + w1) + (w2 + w3);
    }
    for (; s < S; ++s) {
      const float w0 = exp2f(l[s] - M);
      acc += part_at(s, w0);
      L += w0;
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  bf16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (bf16)(acc[j] * inv);
  *reinterpret_cast<bf16x4*>(out + row * out_stride + (int64_t)hh * D + c) = o;
  if (lse_out && (threadIdx.x & 31) == 0) lse_out[row * Hq + hh] = L > 0.f ? M + log2f(L) : -INFINITY;
}

// ------------------------------------------------------------------------------------------------------------------
// items: int32 [n_items, 8] DecodeItem records (host-checked: npre + nsplit <= S_total, and <= 64 with `out` — the
// fused merge gives one wave lane per partial; items with nsplit > 1 merge through the ticket counters
// ([B * Hkv] int32, zero, re-armed by the kernel)).
extern "C" hipError_t kafka_launch_attn_decode(const bf16* q, int64_t q_stride, const void* k_cache,
                                              const void* v_cache, int fp8, int n_items, int B, int Hkv, int G, int D,
                                              const int* block_tables, int bt_stride, const int* items,
                                              float* out_part, float* lse_part, int S_total, float scale, bf16* out,
                                              int64_t out_stride, int* tickets, const bf16* pre_bf16,
                                              const float* m_part, const float* m_lse, int m_S, int m_rows,
                                              bf16* m_out, int64_t m_out_stride, hipStream_t st) {
  if (n_items == 0) return hipSuccess;
  if (D != 128 || G > 8 || G < 1) return hipErrorInvalidValue;
  if (out != nullptr && tickets == nullptr) return hipErrorInvalidValue;
  if (m_rows > 0 && (m_part == nullptr || m_lse == nullptr || m_out == nullptr || m_S < 1)) return hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  const auto* di = reinterpret_cast<const DecodeItem*>(items);
  const int rpw = (8 % G == 0) ? 8 / G : 1;
  const int n_mwg = m_rows > 0 ? (m_rows + rpw - 1) / rpw : 0;
  if (n_items + n_mwg > 65535) return hipErrorInvalidValue;
  const FusedMerge fm{m_part, m_lse, m_S, m_rows, m_out, m_out_stride};
  const dim3 grid(Hkv, n_items + n_mwg);
  // KAFKA_SC1_ATTN (default 1): the bf16 rows as 16-B sc1 stores through LDS (decode_piece OST)
  static const bool sc1 = [] {
    const char* e = getenv("KAFKA_SC1_ATTN");
    return e == nullptr || e[0] != '0';
  }();
  const bool ost = sc1 && out != nullptr && out_stride % 8 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
  if (ost && !fp8)
    attn_decode_kernel<128, false, true><<<grid, 256, 0, st>>>(q, q_stride, k_cache, v_cache, Hkv, G, block_tables,
                                                                bt_stride, di, B, out_part, lse_part, S_total,
                                                                scale_log2, out, out_stride, tickets, pre_bf16,
                                                                n_items, fm);
  else if (fp8)
    attn_decode_kernel<128, true><<<grid, 256, 0, st>>>(q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride,
                                                         di, B, out_part, lse_part, S_total, scale_log2, out,
                                                         out_stride, tickets, pre_bf16, n_items, fm);
  else
    attn_decode_kernel<128, false><<<grid, 256, 0, st>>>(q, q_stride, k_cache, v_cache, Hkv, G, block_tables,
                                                          bt_stride, di, B, out_part, lse_part, S_total, scale_log2,
                                                          out, out_stride, tickets, pre_bf16, n_items, fm);
  return hipGetLastError();
}

template <bool FP8>
static void launch_prefill(const AttnWorkItem* it, int n_items, const bf16* q, int64_t q_stride,
                           const void* k_cache, const void* v_cache, int Hkv, int G, const int* block_tables,
                           int bt_stride, const int* q_limit, bf16* out, int64_t out_stride, float* out_part,
                           float* lse_part, int S_total, float scale_log2, int variant, hipStream_t st) {
  if (variant == 0)  // 8 waves, 256 query rows per item, K/V staged in LDS
    attn_prefill_kernel<128, 8, true, FP8><<<dim3(Hkv, n_items), 512, 0, st>>>(
        it, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, q_limit, out, out_stride, out_part,
        lse_part, S_total, scale_log2);
  else if (variant == 1)  // 4 waves, 128 rows, LDS
    attn_prefill_kernel<128, 4, true, FP8><<<dim3(Hkv, n_items), 256, 0, st>>>(
        it, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, q_limit, out, out_stride, out_part,
        lse_part, S_total, scale_log2);
  else  // 4 waves, 128 rows, per-wave register loads
    attn_prefill_kernel<128, 4, false, FP8><<<dim3(Hkv, n_items), 256, 0, st>>>(
        it, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, q_limit, out, out_stride, out_part,
        lse_part, S_total, scale_log2);
}

extern "C" hipError_t kafka_launch_attn_tile(const void* items, int n_items, const bf16* q, int64_t q_stride,
                                            const void* k_cache, const void* v_cache, int Hkv, int G, int D,
                                            const int* block_tables, int bt_stride, const int* q_limit, bf16* out,
                                            int64_t out_stride, float* out_part, float* lse_part, int S_total,
                                            float scale, int part_bf16, float* alt_part, float* alt_lse, int alt_S,
                                            int alt_tok_off, hipStream_t st);

extern "C" hipError_t kafka_launch_attn_prefill(const void* items, int n_items, const bf16* q, int64_t q_stride,
                                               const void* k_cache, const void* v_cache, int fp8, int Hkv, int G,
                                               int D, const int* block_tables, int bt_stride, const int* q_limit,
                                               bf16* out, int64_t out_stride, float* out_part, float* lse_part,
                                               int S_total, float scale, int variant, int part_bf16, float* alt_part,
                                               float* alt_lse, int alt_S, int alt_tok_off, hipStream_t st) {
  if (n_items == 0) return hipSuccess;
  if (variant == 3) {  // LDS-DMA ring, 8 waves, 256 rows (attn_tile.hip); bf16 pages only
    if (fp8) return hipErrorInvalidValue;
    return kafka_launch_attn_tile(items, n_items, q, q_stride, k_cache, v_cache, Hkv, G, D, block_tables, bt_stride,
                                  q_limit, out, out_stride, out_part, lse_part, S_total, scale, part_bf16, alt_part,
                                  alt_lse, alt_S, alt_tok_off, st);
  }
  if (part_bf16 || alt_part != nullptr) return hipErrorInvalidValue;  // tile v3 only
  if (D != 128 || G < 1 || G > 32 || (128 % G) != 0 || n_items > 65535) return hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  const auto* it = reinterpret_cast<const AttnWorkItem*>(items);
  if (fp8)
    launch_prefill<true>(it, n_items, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, q_limit, out,
                         out_stride, out_part, lse_part, S_total, scale_log2, variant, st);
  else
    launch_prefill<false>(it, n_items, q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride, q_limit, out,
                          out_stride, out_part, lse_part, S_total, scale_log2, variant, st);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_attn_merge(const float* part, const float* lse, int rows, int Hq, int S, int D, bf16* out,
                             int64_t out_stride, float* lse_out, const bf16* pre, int npre, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (D != 128 || S > MERGE_MAX_S || npre < 0 || npre > S) return hipErrorInvalidValue;
  attn_merge_kernel<128><<<dim3(rows, (Hq + 7) / 8), 256, 0, st>>>(part, lse, S, out, out_stride, Hq, lse_out, pre,
                                                                    pre != nullptr ? npre : 0);
  return hipGetLastError();
}

}  // namespace kafka
