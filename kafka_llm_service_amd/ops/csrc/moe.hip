// Sparse-MoE kernels for gfx950 (Mixtral: E = 8 experts, top-2; SURVEY.md §2.6 `moe_router_topk`, `grouped_gemm`).
//
// moe_route_kernel — ONE workgroup of 1024 threads does the whole routing of a step (T <= 32k tokens):
//   softmax over the E router logits -> top-k -> renormalise (Mixtral), then a stable expert sort of the T*k
//   (token, slot) entries: per expert, a block-wide exclusive scan of the per-thread counts gives every entry its
//   position, so the permutation is deterministic (token order inside each expert). Outputs:
//     topk_w f32 [T, k], topk_e i32 [T, k], perm_tok i32 [T*k] (token of the sorted entry), perm_w f32 [T*k],
//     expert_off i32 [E+1] (row segment of each expert), tile_off i32 [E+1] (BM-row tiles before each expert).
//   The grouped GEMM reads tile_off / expert_off on the device: no host synchronisation between router and experts.
//
// grouped_gemm_kernel — Y = X_e . W_e^T for every expert segment, MFMA 32x32x16 bf16, fp32 accumulate.
//   Workgroup tile = BM 64 rows (one expert's segment) x BN 128 columns, 4 waves as 2 (rows) x 2 (cols), each wave a
//   32 x 64 block = 2 MFMA tiles. K is consumed in BK = 64 steps staged through LDS (A 8 KB + B 16 KB per stage,
//   XOR-swizzled 16-B chunks so the ds_read_b128 fragment reads of 32 rows spread over the banks), two stages:
//   the next step's global loads are issued into registers before the current step's MFMAs.
//   Grid = (upper bound on row tiles, N / 128); workgroups past the last tile of the local experts exit at once.
//   Expert parallelism: only experts [e_lo, e_lo + e_n) are resident (W = their weights). Modes:
//     * gather:  A row r = X[perm_tok[r]]            (the first expert GEMM reads the un-permuted activations),
//     * direct:  A row r = X[r]                       (the second GEMM reads the expert-sorted intermediate),
//     * output:  bf16 Y[r, :] through an LDS transpose (16-B coalesced row stores), or
//     * combine: out_f32[perm_tok[r], :] += perm_w[r] * Y[r, :] with float atomics — a token receives exactly k
//                contributions onto a zeroed buffer, and for k = 2 IEEE addition makes the order irrelevant.
//
// Expert-parallel all-to-all (models/moe.py MoEBlock._a2a; transport: parallel/custom_allreduce.py all_to_all over
// the IPC-mapped buffers, or all_to_all_single): everything that used to be bincount / one_hot / argsort / index_add
// on the host-visible path is a kernel here, so a dispatch + combine never synchronises with the host and captures
// into a hipGraph. The send image of a rank is [ep][C + MR][d] bf16: block q holds, for destination rank q, C row
// slots (the activations of the owned (token, expert) pairs routed to q's experts, packed in pair order) and MR
// metadata rows, read as int32: [count, 0, 0, 0, local expert of slot 0, ..., of slot C-1] (C = capacity).
//   ep_dispatch_kernel   grid (pairs + ep): block i < pairs places pair i (its slot = the number of earlier pairs
//                        with the same destination, a block-wide count — pairs <= a few thousand), copies the row
//                        and records slot_map[i] = q (C + MR) + slot; block pairs + q writes q's count and marks its
//                        unused slots -1.
//   ep_recv_route_kernel one workgroup: the received image's valid slots sorted stably by local expert -> the
//                        MoERouting arrays of the grouped GEMMs (perm_tok = slot row, perm_w = 1; invalid slots past
//                        expert_off[El]).
//   ep_combine_kernel    grid (owned tokens): out[t] = sum_j w[t, j] * back[slot_map[t k + j]] (fp32, bf16 store).
#include "common.h"

namespace kafka {

constexpr int MOE_MAXE = 16;
constexpr int MOE_MAXK = 4;
constexpr int MOE_NT = 1024;

__global__ __launch_bounds__(MOE_NT) void moe_route_kernel(const bf16* __restrict__ logits, int64_t ld, int T, int E,
                                                            int K, int BM, float* __restrict__ topk_w,
                                                            int* __restrict__ topk_e, int* __restrict__ perm_tok,
                                                            float* __restrict__ perm_w, int* __restrict__ expert_off,
                                                            int* __restrict__ tile_off) {
  __shared__ int wsum[MOE_NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (T + MOE_NT - 1) / MOE_NT;  // tokens owned by this thread: [t0, t1)
  const int t0 = min(T, tid * per), t1 = min(T, t0 + per);
  // ---- phase 1: softmax + top-k + renormalise for the owned tokens
  for (int t = t0; t < t1; ++t) {
    float p[MOE_MAXE];
    float m = -INFINITY;
    for (int e = 0; e < E; ++e) {
      p[e] = (float)logits[(int64_t)t * ld + e];
      m = fmaxf(m, p[e]);
    }
    float s = 0.f;
    for (int e = 0; e < E; ++e) {
      p[e] = __expf(p[e] - m);
      s += p[e];
    }
    float tot = 0.f;
    int sel[MOE_MAXK];
    float sw[MOE_MAXK];
    for (int j = 0; j < K; ++j) {
      int best = 0;
      float bv = -1.f;
      for (int e = 0; e < E; ++e)
        if (p[e] > bv) {  // strict: lowest index wins ties (torch.topk order on equal values is unspecified)
          bv = p[e];
          best = e;
        }
      sel[j] = best;
      sw[j] = bv / s;
      tot += sw[j];
      p[best] = -2.f;
    }
    for (int j = 0; j < K; ++j) {
      topk_w[(int64_t)t * K + j] = sw[j] / tot;
      topk_e[(int64_t)t * K + j] = sel[j];
    }
  }
  // ---- phase 2: stable sort of the entries [t0*K, t1*K) by expert (each thread re-reads its own writes)
  int base = 0, tbase = 0;
  for (int e = 0; e < E; ++e) {
    int c = 0;
    for (int i = t0 * K; i < t1 * K; ++i) c += topk_e[i] == e;
    // block exclusive scan of c
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int wpre = 0, total = 0;
    for (int i = 0; i < MOE_NT / 64; ++i) {
      const int v = wsum[i];
      wpre += i < w ? v : 0;
      total += v;
    }
    int pos = base + wpre + incl - c;
    for (int i = t0 * K; i < t1 * K; ++i)
      if (topk_e[i] == e) {
        perm_tok[pos] = i / K;
        perm_w[pos] = topk_w[i];
        ++pos;
      }
    base += total;
    tbase += (total + BM - 1) / BM;
    if (tid == 0) {
      expert_off[e + 1] = base;
      tile_off[e + 1] = tbase;
    }
    __syncthreads();  // wsum is reused by the next expert
  }
  if (tid == 0) {
    expert_off[0] = 0;
    tile_off[0] = 0;
  }
}

// ------------------------------------------------------------------------------------------------------------------
constexpr int GG_BM = 64, GG_BN = 128, GG_BK = 64;
constexpr int GG_A_BYTES = GG_BM * GG_BK * 2;  // 8 KB
constexpr int GG_B_BYTES = GG_BN * GG_BK * 2;  // 16 KB
constexpr int GG_STAGE = GG_A_BYTES + GG_B_BYTES;

// 16-B chunk c (0..7) of a 128-B LDS row r lives at chunk c ^ (r & 7)
__device__ __forceinline__ int gg_off(int r, int c) { return r * 128 + 16 * (c ^ (r & 7)); }

template <bool GATHER, bool COMBINE>
__global__ __launch_bounds__(256) void grouped_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                            const bf16* __restrict__ W, int N, int Kd,
                                                            const int* __restrict__ perm_tok,
                                                            const float* __restrict__ perm_w,
                                                            const int* __restrict__ expert_off,
                                                            const int* __restrict__ tile_off, int e_lo, int e_n,
                                                            bf16* __restrict__ Y, int64_t ldy,
                                                            float* __restrict__ out, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) char lds[2 * GG_STAGE];
  // experts [e_lo, e_lo + e_n) are local (expert parallelism: W holds only those)
  const int tile = blockIdx.x + tile_off[e_lo];
  if (tile >= tile_off[e_lo + e_n]) return;
  int e = e_lo;
  while (e + 1 < e_lo + e_n && tile_off[e + 1] <= tile) ++e;
  const int seg0 = expert_off[e], cnt = expert_off[e + 1] - seg0;
  const int r0 = (tile - tile_off[e]) * GG_BM;  // first row of this tile inside the expert segment
  const int n0 = blockIdx.y * GG_BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16* We = W + (int64_t)(e - e_lo) * N * Kd;

  // per-thread staging addresses: A = 64 rows x 8 chunks (2 per thread), B = 128 rows x 8 chunks (4 per thread)
  const bf16* a_src[2];
  int a_dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i, r = q >> 3, c = q & 7;
    const int rr = min(r0 + r, cnt - 1);  // rows past the segment load a valid row; their outputs are dropped
    const int64_t src_row = GATHER ? (int64_t)perm_tok[seg0 + rr] : (int64_t)(seg0 + rr);
    a_src[i] = X + src_row * ldx + c * 8;
    a_dst[i] = gg_off(r, c);
  }
  const bf16* b_src[4];
  int b_dst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i, r = q >> 3, c = q & 7;
    b_src[i] = We + (int64_t)(n0 + r) * Kd + c * 8;
    b_dst[i] = GG_A_BYTES + gg_off(r, c);
  }
  bf16x8 ra[2], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = load_bf16x8(a_src[i] + k0);
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(b_src[i] + k0));
  };
  auto store = [&](char* st) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8*>(st + a_dst[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<bf16x8*>(st + b_dst[i]) = rb[i];
  };

  const int wr = (w & 1) * 32, wc = (w >> 1) * 64;  // this wave's 32 x 64 block
  const int fr = lane & 31, fh = lane >> 5;
  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  const int nk = Kd / GG_BK;
  load(0);
  store(lds);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    char* cur = lds + (ks & 1) * GG_STAGE;
    if (ks + 1 < nk) load((ks + 1) * GG_BK);
#pragma unroll
    for (int s = 0; s < GG_BK / 16; ++s) {
      const int c = 2 * s + fh;
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(cur + gg_off(wr + fr, c));
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(cur + GG_A_BYTES + gg_off(wc + fr, c));
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(cur + GG_A_BYTES + gg_off(wc + 32 + fr, c));
      acc[0] = mfma32(a, b0, acc[0]);
      acc[1] = mfma32(a, b1, acc[1]);
    }
    if (ks + 1 < nk) {
      store(lds + ((ks + 1) & 1) * GG_STAGE);
      __syncthreads();
    }
  }

  if (COMBINE) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = r0 + wr + (i & 3) + 8 * (i >> 2) + 4 * fh;
        if (r < cnt) {
          const int n = n0 + wc + 32 * j + fr;
          atomicAdd(out + (int64_t)perm_tok[seg0 + r] * ldo + n, perm_w[seg0 + r] * acc[j][i]);
        }
      }
    return;
  }
  // bf16 tile through LDS (64 x 128 x 2 B = 16 KB, reusing stage 0) -> 16-B row stores
  __syncthreads();
  bf16* ct = reinterpret_cast<bf16*>(lds);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = wr + (i & 3) + 8 * (i >> 2) + 4 * fh;
      ct[r * GG_BN + wc + 32 * j + fr] = (bf16)acc[j][i];
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i, r = q >> 4, c = q & 15;
    if (r0 + r < cnt)
      store_bf16x8(Y + (int64_t)(seg0 + r0 + r) * ldy + n0 + c * 8,
                   *reinterpret_cast<const bf16x8*>(ct + r * GG_BN + c * 8));
  }
}

extern "C" hipError_t kafka_launch_moe_route(const bf16* logits, int64_t ld, int T, int E, int K, int BM,
                                            float* topk_w, int* topk_e, int* perm_tok, float* perm_w,
                                            int* expert_off, int* tile_off, hipStream_t st) {
  if (E > MOE_MAXE || K > MOE_MAXK || K > E) return hipErrorInvalidValue;
  moe_route_kernel<<<1, MOE_NT, 0, st>>>(logits, ld, T, E, K, BM, topk_w, topk_e, perm_tok, perm_w, expert_off,
                                         tile_off);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_grouped_gemm(const bf16* X, int64_t ldx, const bf16* W, int N, int Kd,
                                               const int* perm_tok, const float* perm_w, const int* expert_off,
                                               const int* tile_off, int e_lo, int e_n, int max_tiles, int gather,
                                               bf16* Y,
                                               int64_t ldy, float* out, int64_t ldo, hipStream_t st) {
  if (N % GG_BN || Kd % GG_BK) return hipErrorInvalidValue;
  dim3 grid(max_tiles, N / GG_BN);
  if (out) {
    if (gather)
      grouped_gemm_kernel<true, true><<<grid, 256, 0, st>>>(X, ldx, W, N, Kd, perm_tok, perm_w, expert_off,
                                                            tile_off, e_lo, e_n, Y, ldy, out, ldo);
    else
      grouped_gemm_kernel<false, true><<<grid, 256, 0, st>>>(X, ldx, W, N, Kd, perm_tok, perm_w, expert_off,
                                                             tile_off, e_lo, e_n, Y, ldy, out, ldo);
  } else {
    if (gather)
      grouped_gemm_kernel<true, false><<<grid, 256, 0, st>>>(X, ldx, W, N, Kd, perm_tok, perm_w, expert_off,
                                                             tile_off, e_lo, e_n, Y, ldy, out, ldo);
    else
      grouped_gemm_kernel<false, false><<<grid, 256, 0, st>>>(X, ldx, W, N, Kd, perm_tok, perm_w, expert_off,
                                                              tile_off, e_lo, e_n, Y, ldy, out, ldo);
  }
  return hipGetLastError();
}


// ------------------------------------------------------------------------------------------------------------------
// Expert-parallel dispatch / receive routing / combine (see the header).
__device__ __forceinline__ int block_sum_i(int v, int* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(256) void ep_dispatch_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                          const int* __restrict__ topk_e, int lo, int n_pairs, int k,
                                                          int El, int ep, int C, int MR, int d,
                                                          bf16* __restrict__ img, int* __restrict__ slot_map) {
  __shared__ int red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t blk = (int64_t)(C + MR) * d;  // elements per destination block
  const int* te = topk_e + (int64_t)lo * k;
  if (b < n_pairs) {
    const int e = te[b], q = e / El;
    int c = 0;
    for (int i = tid; i < b; i += 256) c += te[i] / El == q;
    const int pos = block_sum_i(c, red);  // block-uniform
    if (pos >= C) return;                   // cannot happen for C = Tl * min(k, El) (host-checked); never overflow
    int* meta = reinterpret_cast<int*>(img + q * blk + (int64_t)C * d);
    if (tid == 0) {
      slot_map[b] = q * (C + MR) + pos;
      meta[4 + pos] = e - q * El;
    }
    const bf16* src = x + (int64_t)(lo + b / k) * ldx;
    bf16* dst = img + q * blk + (int64_t)pos * d;
    for (int c8 = tid; c8 < (d >> 3); c8 += 256) store_bf16x8(dst + c8 * 8, load_bf16x8(src + c8 * 8));
  } else {
    const int q = b - n_pairs;
    int c = 0;
    for (int i = tid; i < n_pairs; i += 256) c += te[i] / El == q;
    const int n = block_sum_i(c, red);
    int* meta = reinterpret_cast<int*>(img + q * blk + (int64_t)C * d);
    if (tid < 4) meta[tid] = tid == 0 ? n : 0;
    for (int s = n + tid; s < C; s += 256) meta[4 + s] = -1;
  }
}

__global__ __launch_bounds__(256) void ep_recv_route_kernel(const bf16* __restrict__ img, int ep, int C, int MR,
                                                            int d, int El, int BM, int* __restrict__ perm_tok,
                                                            float* __restrict__ perm_w, int* __restrict__ expert_off,
                                                            int* __restrict__ tile_off) {
  __shared__ int wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int S = ep * C;                       // candidate slots, flattened (source p, slot s) -> p * C + s
  const int per = (S + 255) / 256;
  const int s0 = min(S, tid * per), s1 = min(S, s0 + per);
  const int64_t blk = (int64_t)(C + MR) * d;
  auto expert_of = [&](int f) {               // local expert of flattened slot f, -1 if unused
    const int p = f / C, s = f % C;
    const int* meta = reinterpret_cast<const int*>(img + p * blk + (int64_t)C * d);
    return s < meta[0] ? meta[4 + s] : -1;
  };
  int base = 0, tbase = 0;
  for (int e = 0; e < El; ++e) {
    int c = 0;
    for (int f = s0; f < s1; ++f) c += expert_of(f) == e;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int wpre = 0, total = 0;
    for (int i = 0; i < 4; ++i) {
      wpre += i < w ? wsum[i] : 0;
      total += wsum[i];
    }
    int pos = base + wpre + incl - c;
    for (int f = s0; f < s1; ++f)
      if (expert_of(f) == e) {
        perm_tok[pos] = (f / C) * (C + MR) + f % C;  // row of the slot in the received image
        perm_w[pos] = 1.f;
        ++pos;
      }
    base += total;
    tbase += (total + BM - 1) / BM;
    if (tid == 0) {
      expert_off[e + 1] = base;
      tile_off[e + 1] = tbase;
    }
  }
  if (tid == 0) {
    expert_off[0] = 0;
    tile_off[0] = 0;
  }
  // entries past the last segment: a valid row, weight 0 (no kernel reads them; keeps every index in range)
  for (int i = base + tid; i < S; i += 256) {
    perm_tok[i] = 0;
    perm_w[i] = 0.f;
  }
}

__global__ __launch_bounds__(256) void ep_combine_kernel(const bf16* __restrict__ back, const int* __restrict__ slot_map,
                                                         const float* __restrict__ topk_w, int lo, int k, int d,
                                                         bf16* __restrict__ out, int64_t ldo) {
  const int i = blockIdx.x;
  const float* w = topk_w + (int64_t)(lo + i) * k;
  const int* sm = slot_map + (int64_t)i * k;
  for (int c8 = threadIdx.x; c8 < (d >> 3); c8 += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {  // the token's k expert outputs, in routing order (deterministic)
      const bf16x8 v = load_bf16x8(back + (int64_t)sm[j] * d + c8 * 8);
      const float wj = w[j];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] += wj * (float)v[t];
    }
    bf16x8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] = (bf16)acc[t];
    store_bf16x8(out + (int64_t)i * ldo + c8 * 8, o);
  }
}

extern "C" hipError_t kafka_launch_ep_dispatch(const bf16* x, int64_t ldx, const int* topk_e, int lo, int n_pairs,
                                              int k, int El, int ep, int C, int MR, int d, bf16* img, int* slot_map,
                                              hipStream_t st) {
  if (ep < 1 || El < 1 || d % 8 != 0 || (int64_t)(16 + 4 * (int64_t)C) > (int64_t)MR * d * 2) return hipErrorInvalidValue;
  ep_dispatch_kernel<<<n_pairs + ep, 256, 0, st>>>(x, ldx, topk_e, lo, n_pairs, k, El, ep, C, MR, d, img, slot_map);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_ep_recv_route(const bf16* img, int ep, int C, int MR, int d, int El, int BM,
                                                int* perm_tok, float* perm_w, int* expert_off, int* tile_off,
                                                hipStream_t st) {
  if (ep < 1 || El < 1 || El > MOE_MAXE) return hipErrorInvalidValue;
  ep_recv_route_kernel<<<1, 256, 0, st>>>(img, ep, C, MR, d, El, BM, perm_tok, perm_w, expert_off, tile_off);
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_ep_combine(const bf16* back, const int* slot_map, const float* topk_w, int lo,
                                             int n_own, int k, int d, bf16* out, int64_t ldo, hipStream_t st) {
  if (n_own < 1) return hipSuccess;
  if (d % 8 != 0) return hipErrorInvalidValue;
  ep_combine_kernel<<<n_own, 256, 0, st>>>(back, slot_map, topk_w, lo, k, d, out, ldo);
  return hipGetLastError();
}

}  // namespace kafka
