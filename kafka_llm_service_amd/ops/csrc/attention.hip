// Paged attention for gfx950 on v_mfma_f32_32x32x16_bf16.
//
// KV page layout (page = 16 tokens, one layer):
//   K: [num_blocks, Hkv, 16, D]   key-major, 256 B per key row (D = 128)
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
//   attn_prefill_kernel  grid (work items, Hkv): a tile of up to 128 (token, head) query rows against a paged key
//                        range; per-row causal limit; writes bf16 output directly or an (O, lse) partial. Used for
//                        chunked prefill and for the cascade pass where the rows are the decode sequences of a
//                        batch and the keys are the shared system-prompt prefix (read once for all sequences).
//   attn_merge_kernel    log-sum-exp merge of S partials per (row, head) -> bf16.
#include "common.h"

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

template <int D>
__device__ __forceinline__ void load_kv(KVFrag<D>& f, const bf16* __restrict__ k_cache,
                                        const bf16* __restrict__ v_cache, int Hkv, int kvh, int page0, int page1,
                                        int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int kp = (r >> 4) ? page1 : page0;
  const bf16* kptr = k_cache + ((int64_t)kp * Hkv + kvh) * (PAGE * D) + (r & 15) * D + 8 * h;
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) f.k[kk] = load_bf16x8(kptr + 16 * kk);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int vp = s2 ? page1 : page0;
    const bf16* vptr = v_cache + ((int64_t)vp * Hkv + kvh) * (D * PAGE) + r * PAGE + 8 * h;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) f.v[s2][t] = load_bf16x8(vptr + 32 * t * PAGE);
  }
}

// Pages holding keys [key0, key0 + 32) (key0 32-aligned); the second page is only dereferenced below `end`.
__device__ __forceinline__ void block_pages(const int* __restrict__ bt, int key0, int end, int& p0, int& p1) {
  p0 = bt[key0 >> 4];
  p1 = (key0 + 16 < end) ? bt[(key0 >> 4) + 1] : p0;
}

// One 32-key step for one wave on already-loaded fragments.
template <int D>
__device__ __forceinline__ void attn_compute(const KVFrag<D>& f, int key0, int lo, int hi, int limit,
                                             const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                             int lane) {
  const int h = lane >> 5;
  f32x16 s = {};
#pragma unroll
  for (int kk = 0; kk < D / 16; ++kk) s = mfma32(f.k[kk], qf[kk], s);

  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int key = key0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    const bool ok = (key >= lo) & (key < hi) & (key <= limit);
    const float v = ok ? s[i] * scale_log2 : -INFINITY;
    s[i] = v;
    mx = fmaxf(mx, v);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float m_new = fmaxf(acc.m, mx);
  const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
  const float alpha = exp2f(acc.m - m_use);
  float psum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float p = exp2f(s[i] - m_use);
    s[i] = p;
    psum += p;
  }
  psum += __shfl_xor(psum, 32, 64);
  acc.l = acc.l * alpha + psum;
  acc.m = m_new;
#pragma unroll
  for (int t = 0; t < D / 32; ++t) acc.o[t] *= alpha;
  bf16x8 pf[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pf[0][j] = (bf16)s[j];
    pf[1][j] = (bf16)s[8 + j];
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < D / 32; ++t) acc.o[t] = mfma32(f.v[s2][t], pf[s2], acc.o[t]);
}

// Key blocks first, first+stride, ... < nblk (block b covers keys [base + 32 b, base + 32 b + 32)), software
// pipelined one block deep. The prefetch of the block after the last one is clamped to the last block (pad, don't
// branch: no divergent load, no extra waitcnt).
template <int D>
__device__ __forceinline__ void attn_blocks(const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
                                            int Hkv, int kvh, const int* __restrict__ bt, int base, int first,
                                            int nblk, int stride, int end, int lo, int hi, int limit,
                                            const bf16x8 (&qf)[D / 16], float scale_log2, WaveAcc<D>& acc,
                                            int lane) {
  if (first >= nblk) return;
  int p0, p1;
  KVFrag<D> cur;
  block_pages(bt, base + 32 * first, end, p0, p1);
  load_kv<D>(cur, k_cache, v_cache, Hkv, kvh, p0, p1, lane);
  for (int b = first; b < nblk; b += stride) {
    const int nb = (b + stride < nblk) ? b + stride : b;
    KVFrag<D> nxt;
    block_pages(bt, base + 32 * nb, end, p0, p1);
    load_kv<D>(nxt, k_cache, v_cache, Hkv, kvh, p0, p1, lane);
    attn_compute<D>(cur, base + 32 * b, lo, hi, limit, qf, scale_log2, acc, lane);
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
// Decode: grid (S, Hkv, B), 256 threads. Requires G <= 8.
template <int D>
__global__ __launch_bounds__(256) void attn_decode_kernel(const bf16* __restrict__ q, int64_t q_stride,
                                                           const bf16* __restrict__ k_cache,
                                                           const bf16* __restrict__ v_cache, int Hkv, int G,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ seq_lens,
                                                           const int* __restrict__ kv_start,
                                                           float* __restrict__ out_part, float* __restrict__ lse_part,
                                                           int S_total, int split_offset, float scale_log2) {
  __shared__ float sO[4][8][D];
  __shared__ float sM[4][8];
  __shared__ float sL[4][8];
  const int b = blockIdx.z, kvh = blockIdx.y, split = blockIdx.x, S = gridDim.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int Hq = Hkv * G;
  const int len = seq_lens[b];
  const int start = kv_start ? kv_start[b] : 0;
  const int a0 = start & ~31;
  const int nb = len > a0 ? (len - a0 + 31) >> 5 : 0;
  const int bps = (nb + S - 1) / S;
  const int blo = split * bps, bhi = min(nb, blo + bps);
  const int lo = max(start, a0 + blo * 32), hi = min(len, a0 + bhi * 32);
  const int* bt = block_tables + (int64_t)b * bt_stride;

  WaveAcc<D> acc;
  init_acc<D>(acc);
  if (blo + w < bhi) {
    bf16x8 qf[D / 16];
    load_q_frags<D>(qf, q + (int64_t)b * q_stride + (int64_t)(kvh * G + r) * D, r < G, h);
    attn_blocks<D>(k_cache, v_cache, Hkv, kvh, bt, a0, blo + w, bhi, 4, len, lo, hi, 0x7fffffff, qf, scale_log2,
                   acc, lane);
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
    out_part[pidx * D + d] = L > 0.f ? O / L : 0.f;
    if (d == 0) lse_part[pidx] = L > 0.f ? M + log2f(L) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------------------------------------------
// Prefill / cascade: grid (num_items, Hkv), 256 threads; wave w owns tile rows [32w, 32w+32), row R -> token R / G,
// head kvh*G + R % G.
template <int D>
__global__ __launch_bounds__(256) void attn_prefill_kernel(const AttnWorkItem* __restrict__ items,
                                                            const bf16* __restrict__ q, int64_t q_stride,
                                                            const bf16* __restrict__ k_cache,
                                                            const bf16* __restrict__ v_cache, int Hkv, int G,
                                                            const int* __restrict__ block_tables, int bt_stride,
                                                            const int* __restrict__ q_limit, bf16* __restrict__ out,
                                                            int64_t out_stride, float* __restrict__ out_part,
                                                            float* __restrict__ lse_part, int S_total,
                                                            float scale_log2) {
  const AttnWorkItem it = items[blockIdx.x];
  const int kvh = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int Hq = Hkv * G;
  const int R = w * 32 + r;
  const int tok = R / G, g = R % G;
  const bool valid = tok < it.q_count;
  const int token = it.q_start + tok;
  const int limit = valid ? q_limit[token] : -1;
  // wave-uniform key range
  int wmax = limit;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o, 64));
  const int lo = it.kv_lo;
  const int hi = min(it.kv_hi, wmax + 1);
  const int* bt = block_tables + (int64_t)it.bt_row * bt_stride;

  WaveAcc<D> acc;
  init_acc<D>(acc);
  if (hi > lo) {
    bf16x8 qf[D / 16];
    load_q_frags<D>(qf, q + (int64_t)token * q_stride + (int64_t)(kvh * G + g) * D, valid, h);
    const int base = lo & ~31;
    attn_blocks<D>(k_cache, v_cache, Hkv, kvh, bt, base, 0, (hi - base + 31) >> 5, 1, hi, lo, hi, limit, qf,
                   scale_log2, acc, lane);
  }
  if (!valid) return;
  const int head = kvh * G + g;
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
// Merge S partials of every head of one row: grid (rows), 256 threads. The per-(head, split) merge weights
// exp2(lse - M) / L are computed once into LDS; then every thread combines float4 columns of its heads.
constexpr int MERGE_MAX_HS = 4096;  // Hq * S
template <int D>
__global__ __launch_bounds__(256) void attn_merge_kernel(const float* __restrict__ part, const float* __restrict__ lse,
                                                          int S, bf16* __restrict__ out, int64_t out_stride, int Hq,
                                                          float* __restrict__ lse_out) {
  __shared__ float wgt[MERGE_MAX_HS];
  __shared__ float sM[64], sL[64];
  const int64_t row = blockIdx.x;
  const float* l = lse + row * Hq * S;
  for (int hh = threadIdx.x; hh < Hq; hh += 256) {
    float M = -INFINITY;
    for (int s = 0; s < S; ++s) M = fmaxf(M, l[hh * S + s]);
    float L = 0.f;
    if (M != -INFINITY)
      for (int s = 0; s < S; ++s) L += exp2f(l[hh * S + s] - M);
    sM[hh] = M;
    sL[hh] = L;
    if (lse_out) lse_out[row * Hq + hh] = L > 0.f ? M + log2f(L) : -INFINITY;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Hq * S; i += 256) {
    const int hh = i / S;
    const float L = sL[hh];
    wgt[i] = L > 0.f ? exp2f(l[i] - sM[hh]) / L : 0.f;
  }
  __syncthreads();
  constexpr int D4 = D / 4;
  for (int i = threadIdx.x; i < Hq * D4; i += 256) {
    const int hh = i / D4, c = (i % D4) * 4;
    const float* p = part + ((row * Hq + hh) * S) * D + c;
    const float* w = wgt + hh * S;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 4 <= S; s += 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(p + (s + 0) * D);
      const f32x4 b = *reinterpret_cast<const f32x4*>(p + (s + 1) * D);
      const f32x4 cc = *reinterpret_cast<const f32x4*>(p + (s + 2) * D);
      const f32x4 d = *reinterpret_cast<const f32x4*>(p + (s + 3) * D);
      acc += a * w[s] + b * w[s + 1] + cc * w[s + 2] + d * w[s + 3];
    }
    for (; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(p + s * D) * w[s];
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)acc[j];
    *reinterpret_cast<bf16x4*>(out + row * out_stride + (int64_t)hh * D + c) = o;
  }
}

// ------------------------------------------------------------------------------------------------------------------
extern "C" hipError_t kafka_launch_attn_decode(const bf16* q, int64_t q_stride, const bf16* k_cache, const bf16* v_cache, int B,
                              int Hkv, int G, int D, const int* block_tables, int bt_stride, const int* seq_lens,
                              const int* kv_start, float* out_part, float* lse_part, int S, int S_total,
                              int split_offset, float scale, hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (D != 128 || G > 8 || G < 1) return hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  attn_decode_kernel<128><<<dim3(S, Hkv, B), 256, 0, st>>>(q, q_stride, k_cache, v_cache, Hkv, G, block_tables,
                                                           bt_stride, seq_lens, kv_start, out_part, lse_part, S_total,
                                                           split_offset, scale_log2);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_attn_prefill(const void* items, int n_items, const bf16* q, int64_t q_stride, const bf16* k_cache,
                               const bf16* v_cache, int Hkv, int G, int D, const int* block_tables, int bt_stride,
                               const int* q_limit, bf16* out, int64_t out_stride, float* out_part, float* lse_part,
                               int S_total, float scale, hipStream_t st) {
  if (n_items == 0) return hipSuccess;
  if (D != 128 || G < 1 || G > 32 || (128 % G) != 0) return hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  attn_prefill_kernel<128><<<dim3(n_items, Hkv), 256, 0, st>>>(
      reinterpret_cast<const AttnWorkItem*>(items), q, q_stride, k_cache, v_cache, Hkv, G, block_tables, bt_stride,
      q_limit, out, out_stride, out_part, lse_part, S_total, scale_log2);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_attn_merge(const float* part, const float* lse, int rows, int Hq, int S, int D, bf16* out,
                             int64_t out_stride, float* lse_out, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (D != 128 || Hq > 64 || Hq * S > MERGE_MAX_HS) return hipErrorInvalidValue;
  attn_merge_kernel<128><<<rows, 256, 0, st>>>(part, lse, S, out, out_stride, Hq, lse_out);
  return hipGetLastError();
}

}  // namespace kafka
