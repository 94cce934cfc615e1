// Weight-streaming decode GEMM on pre-tiled weights (gfx950):   Y[M, N] = X[M, K] . W[N, K]^T,  M <= 128.
//
// At decode the weights are read exactly once per step and M (running sequences) is small, so this GEMM is an HBM
// stream of W with just enough MFMA work riding on it. Two layout decisions make the stream full-rate:
//
//   * W is stored "wave-tiled" (done once at load time, ops.tile_weight):  Wt[N/32][K/16][64 lanes][8] bf16 with
//     lane l = (r = l & 31, h = l >> 5) holding W[32 nb + r][16 kb + 8 h + j]. That is exactly the B fragment of
//     v_mfma_f32_32x32x16_bf16 for a 32-column tile, so every wave-instruction of the stream is ONE contiguous 1 KB
//     read (16 B per lane, non-temporal: each byte is used once), and one wave's whole K slice is a single
//     contiguous run. (A row-major [N, K] weight read as MFMA fragments touches 32 rows x 32 B per instruction.)
//   * X (the activations, <= 128 x K bf16, L2-resident) is staged per 128/256-deep K chunk into LDS with full-line
//     coalesced loads and read back as A fragments with ds_read_b128 from an XOR-swizzled image (chunk c of row m
//     at c ^ (m & 15): the 16 lanes of one LDS cycle hit 16 different bank groups). The 4 waves of a workgroup own 4
//     different 32-column tiles and share each X chunk, so X costs 1/4 of the W traffic on-chip and nothing in HBM.
//
// Work decomposition: workgroup = 4 waves = 128 output columns x one K split; grid (ceil(N / 128), S). S (1..8)
// is chosen on the host so the grid has >= 256 workgroups when N is small. S == 1 writes bf16 Y directly; S > 1
// writes fp32 partial slabs P[S][M][N] that the NEXT kernel sums while reading its input (rope_kv, fused
// add+RMSNorm, SwiGLU all accept slabs), so split-K costs no extra launch and no extra bf16 round trip.
// Pipelining: X chunk c+1 and the W fragments of chunk c+1 are issued before the MFMAs of chunk c; the LDS image of
// chunk c+1 is written after them (issue-early / write-late, one barrier per chunk).
// C = X . W^T comes out with lanes along N (col = lane & 31), so every epilogue store instruction writes two
// 128-B row segments.
#include "common.h"

#include <cstdlib>

namespace kafka {

// ---- Fused decode-layer epilogues (FIN template argument) -------------------------------------------------------
// A pure decode layer used to be 9 launches: add+RMSNorm -> qkv -> RoPE/KV write -> cascade -> decode -> o ->
// add+RMSNorm -> gate_up -> down. With FIN the GEMMs absorb the three small kernels (VERDICT r05 "Next" #1):
//
//   * deferred RMSNorm: rmsnorm(h) . W^T = r (.) ((h (.) w) . W^T) with r[m] = rsqrt(mean_k h[m,k]^2 + eps). The
//     producer of h (the residual stream) writes X' = bf16(h (.) w) and, per 128-column block, the partial sums of
//     h^2 (ss [N/128][M]); the consumer GEMM streams X' as its A operand and applies r in its epilogue.
//   * split-K finisher: every split writes its fp32 tile as 16-B sc1 (write-through, agent-coherent) stores, waits
//     for them (vmcnt 0), takes a per-column-block ticket (relaxed agent-scope atomic), and the LAST split of the
//     column block sums the other S - 1 slabs with sc1 loads (compiler-tracked buffer loads, policy bit sc1) plus its
//     own tile from LDS, then runs the fused epilogue and re-arms the ticket. No fence: a release fence at agent scope
//     would write back this XCD's whole L2 from every workgroup (see attention.hip's ticket merge).
//       FIN_RES  (o, down):  h = resid + sum; resid <- bf16(h); xn <- bf16(h (.) nw); ss_out[cb][m] = sum_cols h^2
//       FIN_ROPE (qkv):      y = r (.) sum; rotate-half RoPE on q / k heads; q -> q_out, k / v -> the paged caches
//   * FIN_GLU (gate_up, one split): silu(r g) * (r u) in the SwiGLU epilogue; r from ss_in, whose loads are issued
//     at kernel start (their latency hides under the weight stream).
// One 128-column workgroup tile is exactly one head (D = 128), so the RoPE partner d +- 64 is in the same
// workgroup. Memory-model notes: common.h "Store / load scopes".
enum { FIN_NONE = 0, FIN_RES = 1, FIN_ROPE = 2, FIN_GLU = 3 };

struct FinArgs {
  int* tickets;                 // [N / 128] zeroed once, re-armed by each column block's finisher
  const float* ss_in;           // [nss][ss_ld] partial sums of h^2 of X's rows (nullptr: X is already normalised)
  int nss, ss_ld;
  float inv_d, eps;
  bf16* resid;                  // FIN_RES: residual stream [M, N] (row stride ldr), updated in place
  int64_t ldr;
  const bf16* nw;               // FIN_RES: the next RMSNorm's weight [N]
  bf16* xn;                     // FIN_RES: bf16(h (.) nw) [M, N] (row stride ldxn): the next GEMM's A operand
  int64_t ldxn;
  float* ss_out;                // FIN_RES: [N / 128][ss_out_ld]
  int ss_out_ld;
  const int64_t* positions;     // FIN_ROPE
  const float* cos_sin;         // [max_pos, 128]: cos in [0, 64), sin in [64, 128)
  bf16* q_out;                  // [M, Hq, 128] (row stride q_stride)
  int64_t q_stride;
  bf16* k_cache;                // [blocks, Hkv, 16, 128] in D/8 chunk planes (rope_kv.hip)
  bf16* v_cache;                // [blocks, Hkv, 128, 16] V^T, key o at vt_pos(o)
  const int64_t* slots;         // [M] (-1: no KV write) or nullptr
  int Hq, Hkv;
  uint64_t* stamps;             // optional phase stamps [grid][8] (100 MHz clock; benchmarks/fused_bench.py)
  int* err;                     // bit 0 set if a finisher could not reach a split's slab (see "home XCD" below)
};

// split s's 16 B: from this XCD's L2 (the split stored it there: same XCD) or, flagged, agent-coherent (sc1)
template <bool MIXED>
__device__ __forceinline__ f32x4 load16_split(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned flags, int s) {
  if constexpr (MIXED) {
    if ((flags >> s) & 1u) return load16_sc1(rs, byte_off);
  }
  return load16_plain(rs, byte_off);
}

__device__ __forceinline__ int vt_pos16(int o) { return (o & ~15) | (o & 3) | ((o & 4) << 1) | ((o & 8) >> 1); }

// tp: this split's tile [4 column tiles][ROWS][32] fp32 in LDS; own column c of row m at tp[((c >> 5) * ROWS + m) * 32
// + (c & 31)]. P: slabs [S][Mtot][N]; the finisher is split `by`.
template <int S, int ROWS, int NTH, bool MIXED>
__device__ __forceinline__ void fin_res(const float* tp, const float* P, int by, int M, int Mtot, int N, int cb,
                                        const FinArgs& fa, int tid, unsigned flags) {
  constexpr int O = S - 1;                                  // the other splits' slabs
  constexpr int UB = O == 0 ? 8 : (28 / O >= 8 ? 8 : (28 / O < 1 ? 1 : 28 / O));  // <= 28 loads in flight
  const auto rs = buf_rsrc(P);
  const int c0 = cb * 128, nunits = M * 32;                 // unit = (row, 4 columns); a row = 32 consecutive lanes
  for (int q0 = tid; q0 < nunits; q0 += NTH * UB) {
    f32x4 pv[UB][O > 0 ? O : 1];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int q = min(q0 + u * NTH, nunits - 1);
      const int row = q >> 5, g = q & 31;
#pragma unroll
      for (int j = 0; j < O; ++j) {
        const int s = j < by ? j : j + 1;
        pv[u][j] = load16_split<MIXED>(rs, (int)((((int64_t)s * Mtot + row) * N + c0 + 4 * g) * 4), flags, s);
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int q = q0 + u * NTH;
      const bool valid = q < nunits;  // whole 32-lane rows are valid or not (nunits = 32 M)
      const int row = min(q, nunits - 1) >> 5, g = q & 31;
      f32x4 v = *reinterpret_cast<const f32x4*>(tp + ((g >> 3) * ROWS + row) * 32 + 4 * (g & 7));
#pragma unroll
      for (int j = 0; j < O; ++j) v += pv[u][j];
      const int64_t col = c0 + 4 * g;
      const bf16x4 rb = *reinterpret_cast<const bf16x4*>(fa.resid + row * fa.ldr + col);
      const bf16x4 wb = *reinterpret_cast<const bf16x4*>(fa.nw + col);
      bf16x4 hs, xo;
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hs[j] = (bf16)(v[j] + (float)rb[j]);  // the residual stream is bf16 (as fused_add_rmsnorm)
        const float hf = (float)hs[j];
        ss += hf * hf;
        xo[j] = (bf16)(hf * (float)wb[j]);
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      if (valid) {
        *reinterpret_cast<bf16x4*>(fa.resid + row * fa.ldr + col) = hs;
        *reinterpret_cast<bf16x4*>(fa.xn + row * fa.ldxn + col) = xo;
        if (g == 0) fa.ss_out[(int64_t)cb * fa.ss_out_ld + row] = ss;
      }
    }
  }
}

template <int S, int ROWS, int NTH, bool MIXED>
__device__ __forceinline__ void fin_rope(const float* tp, const float* P, int by, int M, int Mtot, int N, int cb,
                                         const FinArgs& fa, int tid, const float* s_r, const int* s_pos,
                                         const int64_t* s_slot, unsigned flags) {
  constexpr int O = S - 1;
  const auto rs = buf_rsrc(P);
  const int head = cb, c0 = cb * 128;
  const bool is_q = head < fa.Hq, is_k = !is_q && head < fa.Hq + fa.Hkv;  // workgroup-uniform
  if (is_q || is_k) {
    // unit = (row, g < 16): columns 4g..4g+3 and their rotate-half partners 64 + 4g..
    constexpr int UB = O == 0 ? 4 : (14 / O >= 4 ? 4 : (14 / O < 1 ? 1 : 14 / O));
    const int nunits = M * 16;
    for (int q0 = tid; q0 < nunits; q0 += NTH * UB) {
      f32x4 pa[UB][O > 0 ? O : 1], pb[UB][O > 0 ? O : 1];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = min(q0 + u * NTH, nunits - 1);
        const int row = q >> 4, g = q & 15;
#pragma unroll
        for (int j = 0; j < O; ++j) {
          const int s = j < by ? j : j + 1;
          const int64_t base = ((int64_t)s * Mtot + row) * N + c0 + 4 * g;
          pa[u][j] = load16_split<MIXED>(rs, (int)(base * 4), flags, s);
          pb[u][j] = load16_split<MIXED>(rs, (int)((base + 64) * 4), flags, s);
        }
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = q0 + u * NTH;
        if (q >= nunits) continue;
        const int row = q >> 4, g = q & 15;
        f32x4 x1 = *reinterpret_cast<const f32x4*>(tp + ((g >> 3) * ROWS + row) * 32 + 4 * (g & 7));
        f32x4 x2 = *reinterpret_cast<const f32x4*>(tp + ((2 + (g >> 3)) * ROWS + row) * 32 + 4 * (g & 7));
#pragma unroll
        for (int j = 0; j < O; ++j) {
          x1 += pa[u][j];
          x2 += pb[u][j];
        }
        const float rr = s_r[row];
        const float* cs = fa.cos_sin + (int64_t)s_pos[row] * 128;
        const f32x4 cv = *reinterpret_cast<const f32x4*>(cs + 4 * g);
        const f32x4 sv = *reinterpret_cast<const f32x4*>(cs + 64 + 4 * g);
        bf16x4 o1, o2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = x1[j] * rr, b = x2[j] * rr;
          o1[j] = (bf16)(a * cv[j] - b * sv[j]);
          o2[j] = (bf16)(b * cv[j] + a * sv[j]);
        }
        if (is_q) {
          bf16* dst = fa.q_out + row * fa.q_stride + head * 128 + 4 * g;
          *reinterpret_cast<bf16x4*>(dst) = o1;
          *reinterpret_cast<bf16x4*>(dst + 64) = o2;
        } else {
          const int64_t slot = s_slot[row];
          if (slot >= 0) {
            // element (key o, d) of a page at ((d >> 3) * 16 + o) * 8 + (d & 7): d = 4g..4g+3 is one 8-B run
            bf16* dst = fa.k_cache + ((slot >> 4) * fa.Hkv + (head - fa.Hq)) * 2048 + (slot & 15) * 8 +
                        (g >> 1) * 128 + 4 * (g & 1);
            *reinterpret_cast<bf16x4*>(dst) = o1;
            *reinterpret_cast<bf16x4*>(dst + 8 * 128) = o2;  // d + 64: 8 chunk planes further
          }
        }
      }
    }
  } else {
    // V head: unit = (row, g < 32), columns 4g..4g+3, scaled and transposed into the V^T page
    constexpr int UB = O == 0 ? 8 : (28 / O >= 8 ? 8 : (28 / O < 1 ? 1 : 28 / O));
    const int nunits = M * 32, vh = head - fa.Hq - fa.Hkv;
    for (int q0 = tid; q0 < nunits; q0 += NTH * UB) {
      f32x4 pv[UB][O > 0 ? O : 1];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = min(q0 + u * NTH, nunits - 1);
        const int row = q >> 5, g = q & 31;
#pragma unroll
        for (int j = 0; j < O; ++j) {
          const int s = j < by ? j : j + 1;
          pv[u][j] = load16_split<MIXED>(rs, (int)((((int64_t)s * Mtot + row) * N + c0 + 4 * g) * 4), flags, s);
        }
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = q0 + u * NTH;
        if (q >= nunits) continue;
        const int row = q >> 5, g = q & 31;
        const int64_t slot = s_slot[row];
        if (slot < 0) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(tp + ((g >> 3) * ROWS + row) * 32 + 4 * (g & 7));
#pragma unroll
        for (int j = 0; j < O; ++j) v += pv[u][j];
        const float rr = s_r[row];
        bf16* dst = fa.v_cache + ((slot >> 4) * fa.Hkv + vh) * 2048 + vt_pos16((int)(slot & 15)) + (4 * g) * 16;
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j * 16] = (bf16)(v[j] * rr);
      }
    }
  }
}

template <int MT, int KC, bool NT, int KW, bool PIN, int FIN = FIN_NONE>
__global__ __launch_bounds__(256 * KW) void wstream_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                                 const bf16x8* __restrict__ Wt, int M, int N, int K,
                                                                 int ks, bf16* __restrict__ Y, int64_t ldy,
                                                                 float* __restrict__ P, int glu, int row_tiles,
                                                                 int slab16, FinArgs fa) {
  constexpr int NTH = 256 * KW;
  constexpr int ROWS = 32 * MT;
  constexpr int CPR = KC / 8;             // 16-B chunks per X row of one K chunk
  constexpr int XL = ROWS * CPR / NTH;    // X chunks staged per thread
  constexpr int KSTEP = KC / 16;          // MFMA k-steps per K chunk
  constexpr int KSW = KSTEP / KW;         // k-steps of one wave (KW waves split each chunk along K)
  static_assert(CPR >= 16 && XL >= 1 && KSW >= 1, "chunk too small");
  static_assert(2 * ROWS * KC * 2 >= 4 * (KW - 1) * MT * 16 * 64 * 4, "LDS too small for the K-half reduction");
  __shared__ __attribute__((aligned(16))) bf16 xs[2][ROWS * KC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ct = w & 3, kh = w >> 2;  // column tile of the workgroup, K part of the chunk
  const int r = lane & 31, h = lane >> 5;
  // row tiles (M > 32 MT): the row_tiles workgroups of one weight slice are placed on ONE XCD — workgroups b, b + 8,
  // ... under round-robin placement (blockIdx.x % 8 picks the XCD) — so the slice streams from HBM once and the other
  // row tiles read it from that XCD's L2 (the launch pads the column blocks to a multiple of 8; padding workgroups
  // exit); P stays [S][M_total][N]
  int cb = blockIdx.x, rti = 0;
  if (row_tiles > 1) {
    const int grp = blockIdx.x / (8 * row_tiles), rem = blockIdx.x % (8 * row_tiles);
    cb = grp * 8 + rem % 8;
    rti = rem / 8;
    if (cb >= (N + 127) / 128) return;  // padding workgroup (workgroup-uniform)
  }
  const int row0 = rti * ROWS;
  const int Mtot = M;
  M = min(ROWS, Mtot - row0);
  X += (int64_t)row0 * ldx;
  if (Y != nullptr) Y += (int64_t)row0 * ldy;
  if (P != nullptr) P += (int64_t)row0 * N;
  const int nb = cb * 4 + ct;
  // wave-uniform: a tail wave past the last column tile streams a valid tile and skips only its stores — every
  // load and MFMA stays unconditional, so hipcc's waitcnt pass sees straight-line code and keeps counted vmcnt
  // waits (a divergent `if` around the loads collapses them to vmcnt(0..1) at the join)
  const bool active = nb < (N >> 5);
  const int k0 = blockIdx.y * ks;
  const int nchunks = ks / KC;
  const bf16x8* wp =
      Wt + ((int64_t)(active ? nb : (N >> 5) - 1) * (K >> 4) + (k0 >> 4) + kh * KSW) * 64 + lane;

  // phase stamps (FinArgs::stamps, benchmarks only): 0 start, 1 main loop done, 2 slab stores drained, 3 ticket
  // taken (finisher), 4 finisher done
  auto stamp = [&](int k) {
    if constexpr (FIN != FIN_NONE)
      if (fa.stamps != nullptr && tid == 0)
        fa.stamps[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // FIN_GLU: this thread's share of the row-scale partials ss_in[j][row], issued before the stream (host-checked:
  // tpr = a power of two >= nss / SSL threads per row, M * tpr <= NTH)
  constexpr int SSL = FIN == FIN_GLU ? 4096 / NTH : 1;
  float ssv[SSL];
  int tpr = 1;
  if constexpr (FIN == FIN_GLU) {
    while (tpr * SSL < fa.nss) tpr <<= 1;
    const int row = tid / tpr, j0 = (tid % tpr) * SSL;
#pragma unroll
    for (int i = 0; i < SSL; ++i)
      ssv[i] = (fa.ss_in != nullptr && row < M && j0 + i < fa.nss) ? fa.ss_in[(int64_t)(j0 + i) * fa.ss_ld + row] : 0.f;
  }

  bf16x8 xr[XL];
  auto load_x = [&](int ch) {
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx / CPR, c = idx % CPR;
      const int m = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
      xr[i] = load_bf16x8(X + (int64_t)m * ldx + k0 + ch * KC + c * 8);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx / CPR, c = idx % CPR;
      *reinterpret_cast<bf16x8*>(&xs[buf][row * KC + 8 * (c ^ (row & 15))]) = xr[i];
    }
  };
  auto load_w = [&](bf16x8(&wv)[KSW], int ch) {
#pragma unroll
    for (int t = 0; t < KSW; ++t) {
      const bf16x8* p = wp + (int64_t)(ch * KSTEP + t) * 64;
      wv[t] = NT ? __builtin_nontemporal_load(p) : *p;
    }
    // PIN keeps the prefetch where it is issued: left alone, the machine scheduler sinks these loads (and the X
    // loads before them) below the MFMAs of the current chunk (shorter register live ranges), which leaves the next
    // chunk a prefetch distance of ~0, so every chunk waits out the full HBM latency
    if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
  };
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
  auto compute = [&](int buf, const bf16x8(&wv)[KSW]) {
#pragma unroll
    for (int t = 0; t < KSW; ++t) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = mt * 32 + r, c = 2 * (kh * KSW + t) + h;
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(&xs[buf][m * KC + 8 * (c ^ (m & 15))]);
        acc[mt] = mfma32(xf, wv[t], acc[mt]);
      }
    }
  };

  bf16x8 wa[KSW], wb[KSW];
  // X first: its LDS image is written while the first weight chunk is still in flight (loads return in order)
  load_x(0);
  load_w(wa, 0);
  store_x(0);
  __syncthreads();
  int ch = 0;
  // steady state: two chunks per trip, both prefetches in range (no conditional loads inside the trip); chunk ch is
  // in buffer 0 / wa
  for (; ch + 2 < nchunks; ch += 2) {
    load_x(ch + 1);
    load_w(wb, ch + 1);
    compute(0, wa);
    store_x(1);
    __syncthreads();
    load_x(ch + 2);
    load_w(wa, ch + 2);
    compute(1, wb);
    store_x(0);
    __syncthreads();
  }
  // tail: one or two chunks left (chunk ch is in buffer 0 / wa)
  if (ch + 1 < nchunks) {
    load_x(ch + 1);
    load_w(wb, ch + 1);
    compute(0, wa);
    store_x(1);
    __syncthreads();
    compute(1, wb);
  } else {
    compute(0, wa);
  }

  if constexpr (KW > 1) {
    // the KW waves of a column tile hold partial sums over different k-steps: fold them through LDS (the X stage
    // is dead now), every wave reaches both barriers
    float* red = reinterpret_cast<float*>(&xs[0][0]);
    __syncthreads();
    if (kh > 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[((((kh - 1) * 4 + ct) * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int j = 1; j < KW; ++j)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[mt][i] += red[((((j - 1) * 4 + ct) * MT + mt) * 16 + i) * 64 + lane];
    }
  }
  if constexpr (FIN == FIN_RES || FIN == FIN_ROPE) {
    __shared__ int s_last;
    __shared__ float s_r[FIN == FIN_ROPE ? ROWS : 1];
    __shared__ int s_pos[FIN == FIN_ROPE ? ROWS : 1];
    __shared__ int64_t s_slot[FIN == FIN_ROPE ? ROWS : 1];
    const int S = gridDim.y, by = blockIdx.y;
    float* tp = reinterpret_cast<float*>(&xs[0][0]);  // [4][ROWS][32] fp32: this split's tile (the X stage is dead)
    // Home XCD: workgroups are dealt to the 8 XCDs round-robin (linear id % 8), so with N / 128 a multiple of 8 every
    // split of column block cb runs on XCD cb % 8 and the finisher is one of them: the slabs can go through that XCD's
    // L2 (plain stores, L2-hit loads) instead of the agent-coherent level. Each split CHECKS it (hardware XCC_ID);
    // one that is not home stores sc1 and flags its bit in the ticket (bits 8 + s), so the finisher loads that slab
    // sc1. A finisher that is itself not home cannot reach the home L2 of the others: it sets fa.err.
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xfu;  // hwreg(HW_REG_XCC_ID, 0, 4)
    const bool home = (gridDim.x & 7) == 0 && (int)xcc == (lin & 7);
    __shared__ unsigned s_flags;
    stamp(1);
    // FIN_ROPE: every split loads the per-row partials / position / slot (the finisher is not known yet) into
    // registers before its slab stores and parks them in LDS after issuing them, so the load round trip overlaps the
    // store drain. Thread (row = tid % ROWS, part = tid / ROWS) sums partials part, part + PARTS, ... (nss <= 32,
    // host-checked); the PARTS sums of a row are added in a fixed order (deterministic).
    constexpr int PARTS = NTH / ROWS >= 8 ? 8 : (NTH / ROWS >= 4 ? 4 : (NTH / ROWS >= 2 ? 2 : 1));
    constexpr int JL = FIN == FIN_ROPE ? 32 / PARTS : 1;
    __shared__ float s_ssp[FIN == FIN_ROPE ? PARTS : 1][FIN == FIN_ROPE ? ROWS : 1];
    const int prow = tid % ROWS, ppart = tid / ROWS;
    const bool pact = FIN == FIN_ROPE && ppart < PARTS && prow < M;
    float ssv2[JL];
    int posv = 0;
    int64_t slotv = -1;
    if constexpr (FIN == FIN_ROPE) {
      if (pact) {
#pragma unroll
        for (int u = 0; u < JL; ++u) {
          const int j = ppart + PARTS * u;
          ssv2[u] = (fa.ss_in != nullptr && j < fa.nss) ? fa.ss_in[(int64_t)j * fa.ss_ld + prow] : 0.f;
        }
        if (ppart == 0) {
          posv = (int)fa.positions[prow];
          slotv = fa.slots != nullptr ? fa.slots[prow] : -1;
        }
      }
    }
    __syncthreads();  // (the K-part fold's LDS reads are done)
    if (kh == 0) {
      float* tw = tp + ct * (ROWS * 32);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) tw[(mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[mt][i];
      if (S > 1) {
        // (one wave's LDS accesses complete in order: the reads below see its writes)
#pragma unroll
        for (int j = 0; j < ROWS / 8; ++j) {
          const int q = j * 64 + lane, row = q >> 3, c4 = q & 7;
          const f32x4 v = *reinterpret_cast<const f32x4*>(tw + row * 32 + 4 * c4);
          if (row < M) {
            float* dst = P + ((int64_t)by * Mtot + row) * N + cb * 128 + ct * 32 + 4 * c4;
            if (home)
              *reinterpret_cast<f32x4*>(dst) = v;  // into this XCD's L2, where the finisher will read it
            else
              store16_slab(dst, v);
          }
        }
      }
    }
    if constexpr (FIN == FIN_ROPE) {
      if (pact) {
        float sacc = 0.f;
#pragma unroll
        for (int u = 0; u < JL; ++u) sacc += ssv2[u];
        s_ssp[ppart][prow] = sacc;
        if (ppart == 0) {
          s_pos[prow] = posv;
          s_slot[prow] = slotv;
        }
      }
      __syncthreads();
      if (tid < M) {
        float sacc = 0.f;
#pragma unroll
        for (int p = 0; p < PARTS; ++p) sacc += s_ssp[p][tid];
        s_r[tid] = fa.ss_in != nullptr ? rsqrtf(sacc * fa.inv_d + fa.eps) : 1.f;
      }
    }
    if (S > 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this split's slab has reached the coherent level
      stamp(2);
      __syncthreads();
      if (tid == 0) {
        int* tk = fa.tickets + cb;
        const int add = 1 + (home ? 0 : (256 << by));
        const int t = __hip_atomic_fetch_add(tk, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int tot = t + add;
        s_last = (tot & 255) == S;
        s_flags = (unsigned)(tot >> 8) & 255u;
        if ((tot & 255) == S) {
          __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
          const unsigned others = ((1u << S) - 1u) & ~(1u << by);
          if (!home && (s_flags & others) != others && fa.err != nullptr) atomicOr(fa.err, 1);
        }
      }
      __syncthreads();
      if (!s_last) return;  // workgroup-uniform
      stamp(3);
    } else {
      if (tid == 0) s_flags = 0;
      __syncthreads();
    }
    const unsigned flags = s_flags;
#define KAFKA_FIN_S(S_)                                                                                     \
  case S_:                                                                                                  \
    if constexpr (FIN == FIN_RES) {                                                                         \
      if (flags == 0)                                                                                       \
        fin_res<S_, ROWS, NTH, false>(tp, P, by, M, Mtot, N, cb, fa, tid, 0u);                              \
      else                                                                                                  \
        fin_res<S_, ROWS, NTH, true>(tp, P, by, M, Mtot, N, cb, fa, tid, flags);                            \
    } else {                                                                                                \
      if (flags == 0)                                                                                       \
        fin_rope<S_, ROWS, NTH, false>(tp, P, by, M, Mtot, N, cb, fa, tid, s_r, s_pos, s_slot, 0u);         \
      else                                                                                                  \
        fin_rope<S_, ROWS, NTH, true>(tp, P, by, M, Mtot, N, cb, fa, tid, s_r, s_pos, s_slot, flags);       \
    }                                                                                                       \
    break;
    switch (S) {
      KAFKA_FIN_S(1)
      KAFKA_FIN_S(2)
      KAFKA_FIN_S(4)
      KAFKA_FIN_S(8)
      default: break;  // (host-checked: S in {1, 2, 4, 8})
    }
#undef KAFKA_FIN_S
    if (fa.stamps != nullptr) {
      __syncthreads();
      stamp(4);
    }
    return;
  }
  if (glu && P == nullptr) {
    // fused SwiGLU epilogue (weight tiles GLU-interleaved: tile 2j = gate rows [32j, 32j+32), tile 2j+1 = the
    // matching up rows): odd waves hand their up tile to the even wave of the pair through LDS, which writes
    // silu(gate) * up straight from the fp32 accumulators into Y [M, N/2]
    float* red = reinterpret_cast<float*>(&xs[0][0]);
    // FIN_GLU: deferred RMSNorm of X, r[row] from the partials loaded at kernel start (1 without ss_in)
    __shared__ float s_rg[FIN == FIN_GLU ? ROWS : 1];
    if constexpr (FIN == FIN_GLU) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < SSL; ++i) s += ssv[i];
      for (int o = tpr >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const int row = tid / tpr;
      if (tid % tpr == 0 && row < ROWS) s_rg[row] = fa.ss_in != nullptr ? rsqrtf(s * fa.inv_d + fa.eps) : 1.f;
    }
    auto rrow = [&](int m) { return FIN == FIN_GLU ? s_rg[m < ROWS ? m : ROWS - 1] : 1.f; };
    __syncthreads();
    if (kh == 0 && (ct & 1)) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(((ct >> 1) * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
    }
    __syncthreads();
    if (slab16 & 2) {
      // the workgroup's 64 output columns (128 B per row) through an LDS tile, then 16-B sc1 stores: 8 lanes per row
      bf16* ty = reinterpret_cast<bf16*>(red + 2 * MT * 16 * 64);  // [ROWS][64], after the up-tile exchange
      if (active && kh == 0 && !(ct & 1)) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int m = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const float rr = rrow(m);
            const float g = acc[mt][i] * rr, u = red[(((ct >> 1) * MT + mt) * 16 + i) * 64 + lane] * rr;
            ty[m * 64 + (ct >> 1) * 32 + r] = (bf16)(g / (1.0f + __expf(-g)) * u);
          }
      }
      __syncthreads();
      const int c0 = cb * 64, W2 = N >> 1;
      for (int q = tid; q < ROWS * 8; q += NTH) {
        const int row = q >> 3, c = q & 7;
        if (row < M && c0 + 8 * c < W2)
          store16_slab(reinterpret_cast<float*>(Y + (int64_t)row * ldy + c0 + 8 * c),
                       *reinterpret_cast<const f32x4*>(ty + row * 64 + 8 * c));
      }
    } else if (active && kh == 0 && !(ct & 1)) {
      const int n = (nb >> 1) * 32 + r;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m < M) {
            const float rr = rrow(m);
            const float g = acc[mt][i] * rr, u = red[(((ct >> 1) * MT + mt) * 16 + i) * 64 + lane] * rr;
            Y[(int64_t)m * ldy + n] = (bf16)(g / (1.0f + __expf(-g)) * u);
          }
        }
    }
  } else if (P == nullptr && !glu && (slab16 & 2)) {
    // un-split bf16 output (the lm_head): the workgroup's 128 columns (256 B per row) through an LDS tile, then
    // 16-B sc1 stores, 8 lanes per 128-B line
    bf16* ty = reinterpret_cast<bf16*>(&xs[0][0]);  // [ROWS][128]
    __syncthreads();  // (workgroup-uniform: P, glu and slab16 are kernel arguments)
    if (active && kh == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) ty[(mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 128 + ct * 32 + r] = (bf16)acc[mt][i];
    }
    __syncthreads();
    const int c0 = cb * 128;
    for (int q = tid; q < ROWS * 16; q += NTH) {
      const int row = q >> 4, c = q & 15;
      if (row < M && c0 + 8 * c < N)
        store16_slab(reinterpret_cast<float*>(Y + (int64_t)row * ldy + c0 + 8 * c),
                     *reinterpret_cast<const f32x4*>(ty + row * 128 + 8 * c));
    }
  } else if (P != nullptr && (slab16 & 1)) {
    // split-K slab through a per-wave LDS transpose (the X stage is dead): each lane then holds 4 consecutive columns
    // of a row and writes them with one 16-B sc1 store (the line leaves this XCD's L2 — the consumer kernel runs on
    // every XCD — and the launch ends with fewer dirty lines to write back)
    float* tp = reinterpret_cast<float*>(&xs[0][0]) + ct * (ROWS * 32);
    __syncthreads();  // (workgroup-uniform: P and slab16 are kernel arguments)
    if (active && kh == 0) {
      const int cbase = glu ? ((nb & 1) ? (N >> 1) : 0) + (nb >> 1) * 32 : nb * 32;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) tp[(mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[mt][i];
      // (one wave's LDS accesses complete in order: the reads below see its writes)
#pragma unroll
      for (int j = 0; j < ROWS / 8; ++j) {
        const int q = j * 64 + lane, row = q >> 3, c4 = q & 7;
        const f32x4 v = *reinterpret_cast<const f32x4*>(tp + row * 32 + 4 * c4);
        if (row < M) {
          store16_slab(P + ((int64_t)blockIdx.y * Mtot + row) * N + cbase + 4 * c4, v);
        }
      }
    }
  } else if (active && kh == 0) {
    // GLU-interleaved tiles written un-split: tile 2j -> gate columns [32j, +32), tile 2j+1 -> up columns N/2 + 32j
    const int n = glu ? ((nb & 1) ? (N >> 1) : 0) + (nb >> 1) * 32 + r : nb * 32 + r;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < M) {
          if (P)
            P[((int64_t)blockIdx.y * Mtot + m) * N + n] = acc[mt][i];
          else
            Y[(int64_t)m * ldy + n] = (bf16)acc[mt][i];
        }
      }
  }
}

// Grouped (MoE) variant: one weight stream per expert over wave-tiled expert weights Wt[E_local][N/32][K/16][64][8].
// Grid (ceil(N / 128), E_local, row tiles of 32 * MT); expert e's rows are the routing segment
// [expert_off[e], expert_off[e + 1]) read on the device (no host sync after the router); workgroups past the end
// of their expert's segment exit at once, and row tiles past it skip their MFMAs (wave-uniform).
//   GATHER: A row = X[perm_tok[entry]] (token activations), else X[entry] (expert-sorted intermediate).
//   Epilogue GLU (GLU-interleaved tiles): Y[entry, :N/2] = silu(gate) * up, bf16 — the SwiGLU of the expert MLP.
//   Epilogue COMBINE: out_f32[perm_tok[entry], n] += perm_w[entry] * y (a token gets exactly k contributions).
// (MT = 4: at most 256 registers so two workgroups share a CU — left free the compiler took 316, one wave per SIMD:
// the 128-row expert tiles streamed 8 % slower, Mixtral 128 threads 5,155 vs 5,234 tok/s, profiles/r06/mixtral/;
// MT = 2 spills 32+ registers under the same bound and keeps its 324)
template <int MT, int KC, bool GATHER, bool COMBINE, bool PIN>
__global__ __launch_bounds__(256, MT == 4 ? 2 : 1) void wstream_grouped_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                               const bf16x8* __restrict__ Wt, int N, int K,
                                                               const int* __restrict__ perm_tok,
                                                               const float* __restrict__ perm_w,
                                                               const int* __restrict__ expert_off, int e_lo,
                                                               bf16* __restrict__ Y, int64_t ldy,
                                                               float* __restrict__ out, int64_t ldo) {
  constexpr int ROWS = 32 * MT;
  constexpr int CPR = KC / 8;
  constexpr int XL = ROWS * CPR / 256;
  constexpr int KSTEP = KC / 16;
  static_assert(CPR >= 16 && XL >= 1, "chunk too small");
  __shared__ __attribute__((aligned(16))) bf16 xs[2][ROWS * KC];
  const int el = blockIdx.y, e = e_lo + el;
  const int seg0 = expert_off[e];
  const int cnt = expert_off[e + 1] - seg0;
  const int row0 = blockIdx.z * ROWS;
  if (row0 >= cnt) return;  // workgroup-uniform
  const int rows = min(ROWS, cnt - row0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nb = blockIdx.x * 4 + w;
  const bool active = nb < (N >> 5);
  const bf16x8* wp = Wt + ((int64_t)el * (N >> 5) + (active ? nb : (N >> 5) - 1)) * (K >> 4) * 64 + lane;
  const int nchunks = K / KC;

  // A-row sources of this thread's staged chunks (fixed over K)
  const bf16* xsrc[XL];
#pragma unroll
  for (int i = 0; i < XL; ++i) {
    const int idx = tid + 256 * i;
    const int row = idx / CPR, c = idx % CPR;
    const int ent = seg0 + row0 + min(row, rows - 1);  // rows past the segment reload a valid row, never stored
    const int64_t src = GATHER ? (int64_t)perm_tok[ent] : (int64_t)ent;
    xsrc[i] = X + src * ldx + c * 8;
  }
  bf16x8 xr[XL];
  auto load_x = [&](int ch) {
#pragma unroll
    for (int i = 0; i < XL; ++i) xr[i] = load_bf16x8(xsrc[i] + ch * KC);
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / CPR, c = idx % CPR;
      *reinterpret_cast<bf16x8*>(&xs[buf][row * KC + 8 * (c ^ (row & 15))]) = xr[i];
    }
  };
  auto load_w = [&](bf16x8(&wv)[KSTEP], int ch) {
#pragma unroll
    for (int t = 0; t < KSTEP; ++t) wv[t] = __builtin_nontemporal_load(wp + (int64_t)(ch * KSTEP + t) * 64);
    if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);  // (prefetch kept ahead of the MFMAs, as wstream_gemm)
  };
  const int mt_used = (rows + 31) >> 5;  // row tiles with live rows (uniform)
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
  auto compute = [&](int buf, const bf16x8(&wv)[KSTEP]) {
#pragma unroll
    for (int t = 0; t < KSTEP; ++t) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // MT = 4 computes every row tile (rows past the segment hold a valid row, never stored): with the MFMAs of
        // unused tiles skipped behind a branch, the last accumulator register of tile 0 was read before its final
        // MFMA had written it (row 27 / 31 of a 28..32-row expert wrong at K = 512; the 128-row tile's MFMAs are
        // cheap next to its weight stream)
        if (MT == 4 || mt < mt_used) {
          const int m = mt * 32 + r, c = 2 * t + h;
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(&xs[buf][m * KC + 8 * (c ^ (m & 15))]);
          acc[mt] = mfma32(xf, wv[t], acc[mt]);
        }
      }
    }
  };
  bf16x8 wa[KSTEP], wb[KSTEP];
  load_x(0);
  load_w(wa, 0);
  store_x(0);
  __syncthreads();
  int ch = 0;
  for (; ch + 2 < nchunks; ch += 2) {
    load_x(ch + 1);
    load_w(wb, ch + 1);
    compute(0, wa);
    store_x(1);
    __syncthreads();
    load_x(ch + 2);
    load_w(wa, ch + 2);
    compute(1, wb);
    store_x(0);
    __syncthreads();
  }
  if (ch + 1 < nchunks) {
    load_x(ch + 1);
    load_w(wb, ch + 1);
    compute(0, wa);
    store_x(1);
    __syncthreads();
    compute(1, wb);
  } else {
    compute(0, wa);
  }

  if constexpr (!COMBINE) {
    // SwiGLU epilogue: odd waves hand their up tile to the even wave of the pair through LDS
    float* red = reinterpret_cast<float*>(&xs[0][0]);
    __syncthreads();
    if (w & 1) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(((w >> 1) * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
    }
    __syncthreads();
    if (!active || (w & 1)) return;
    const int n = (nb >> 1) * 32 + r;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < rows) {
          const float g = acc[mt][i], u = red[(((w >> 1) * MT + mt) * 16 + i) * 64 + lane];
          Y[(int64_t)(seg0 + row0 + m) * ldy + n] = (bf16)(g / (1.0f + __expf(-g)) * u);
        }
      }
  } else {
    if (!active) return;
    const int n = nb * 32 + r;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < rows) {
          const int ent = seg0 + row0 + m;
          atomicAdd(out + (int64_t)perm_tok[ent] * ldo + n, perm_w[ent] * acc[mt][i]);
        }
      }
  }
}

// Y[m, n] = sum_s P[s, m, n] (bf16), 8 columns per thread: the standalone combine for callers without a
// slab-aware consumer (TP all-reduce inputs, tests).
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ P, int S, int M, int N,
                                                          bf16* __restrict__ Y, int64_t ldy) {
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (idx >= (int64_t)M * N) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  const int64_t ps = (int64_t)M * N;
  float v[8];
  load_in8(v, nullptr, P, S, ps, idx);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  store_bf16x8(Y + (int64_t)m * ldy + n, o);
}

// Host plan: row tiles MT, K chunk KC and split count S for a shape; returns 0 if supported (mirrored by
// ops.stream_plan). max_splits caps S (1 forces a direct bf16 output).
//   MT: 1 tile up to 32 rows, 2 up to 64, 3 up to 96 (a decode batch plus a short new-turn chunk: three 32-row tiles
//   on 256-deep chunks, 96 KB X stage; +0.24 % over four on 128-deep ones, profiles/r04/bench_ab_wstream_mt3.jsonl),
//   4 up to 128 (128-deep chunks: 256-deep ones lose 1.9 %, profiles/r04/bench_ab_wstream_mt4_kc256.jsonl), 6 up to
//   192 (a decode batch plus a ~100-token new turn: one 192-row tile on 128-deep chunks, 96 KB X stage, ~210
//   registers at one wave per SIMD; two 128-row tiles sharing the weight slice lost to hipBLASLt, r02/r05). Beyond
//   192 rows (tiled-only models) the rows are split over row tiles of 128.
//   Measured and rejected (profiles/r04/): 64-row tiles sharing a weight slice in one XCD's L2 beyond 64 rows (-0.6 %)
//   and 33..64 rows as two 32-row tiles (-4.8 %).
extern "C" int kafka_wstream_plan(int M, int N, int K, int max_splits, int* mt, int* kc, int* splits) {
  if (M < 1 || M > 256 || N % 32 != 0 || N <= 0) return 1;
  const int MT = M <= 32 ? 1 : (M <= 64 ? 2 : (M <= 96 ? 3 : (M <= 128 || M > 192 ? 4 : 6)));
  const int KC = MT >= 4 ? 128 : 256;
  if (K % KC != 0 || K <= 0) return 2;
  const int nx = (N + 127) / 128 * ((M + 32 * MT - 1) / (32 * MT));  // workgroups per split (x row tiles)
  const int chunks = K / KC;
  // split until the grid reaches ~192 workgroups: measured on MI355X (benchmarks/wstream_sweep.py,
  // profiles/wstream_sweep_r01.log; split targets 96..384 re-checked in profiles/r04/bench_ab_split_target_*.jsonl)
  // — every extra split adds 2 x M x N x 4 B of slab traffic, so e.g. gate_up (N = 28672) at M = 64 runs fastest
  // unsplit and qkv (N = 6144) with S = 4. With the pinned prefetch, gate_up at 97..128 rows also runs fastest
  // unsplit (53.3 us at 114 rows with its fused SwiGLU vs 60.4 + a SwiGLU pass split in two;
  // profiles/r05/wstream_sweep_pin.jsonl), so MT = 4 shares the target (it was 256).
  const int target = 192;
  int s = 1;
  while (s * 2 <= max_splits && s * 2 <= 8 && chunks % (s * 2) == 0 && nx * s < target) s *= 2;
  *mt = MT;
  *kc = KC;
  *splits = s;
  return 0;
}

extern "C" hipError_t kafka_launch_wstream_gemm(const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K,
                                               int mt, int kc, int splits, int nt, int kw, int pin, int glu, bf16* Y,
                                               int64_t ldy, float* P, hipStream_t st) {
  if (M < 1) return hipSuccess;
  if (glu && (N % 64 != 0 || kw > 2)) return hipErrorInvalidValue;  // (the SwiGLU epilogue runs after the KW fold)
  if (K % (kc * splits) != 0 || (splits > 1 && P == nullptr) || (splits == 1 && P == nullptr && Y == nullptr))
    return hipErrorInvalidValue;
  const int rt = (M + 32 * mt - 1) / (32 * mt);  // row tiles of 32 * mt rows
  const int nblk = (N + 127) / 128;
  const dim3 grid((rt > 1 ? (nblk + 7) / 8 * 8 : nblk) * rt, splits);  // (row tiles: column blocks padded to 8)
  const int ks = K / splits;
  const auto* wt = reinterpret_cast<const bf16x8*>(Wt);
  float* p = splits > 1 ? P : nullptr;
  // split-K slabs leave as 16-B sc1 stores through an LDS transpose (was one 4-B store per accumulator, the lines
  // kept dirty in the XCD's L2): +2.0 % on the headline, in-step GPU time 7.50 vs 7.65 ms
  // (profiles/r05/bench_ab_wstream_slab16_sc1.jsonl); KAFKA_WSTREAM_SLAB16=0 restores the old epilogue
  // bit 1: the un-split bf16 outputs (fused SwiGLU, lm_head) the same way through a workgroup LDS tile, whole 128-B
  // lines per store instruction (was one 2-B store per accumulator, half lines): +1.1..2.1 %, in-step GPU time 7.37
  // vs 7.45-7.49 ms (profiles/r05/bench_ab_wstream_wide_y.jsonl)
  static const int slab16 = [] {
    const char* e = getenv("KAFKA_WSTREAM_SLAB16");
    return e ? atoi(e) : 3;
  }();
  // (16-B stores of Y need 16-B aligned rows)
  const int wide = (Y != nullptr && (ldy % 8 != 0 || reinterpret_cast<uintptr_t>(Y) % 16 != 0)) ? (slab16 & 1) : slab16;
#define KAFKA_WS(MT_, KC_, KW_, PIN_)                                                                            \
  do {                                                                                                          \
    if (nt)                                                                                                     \
      wstream_gemm_kernel<MT_, KC_, true, KW_, PIN_><<<grid, 256 * KW_, 0, st>>>(X, ldx, wt, M, N, K, ks, Y, ldy, p, \
                                                                              glu, rt, wide, FinArgs{});        \
    else                                                                                                        \
      wstream_gemm_kernel<MT_, KC_, false, KW_, PIN_><<<grid, 256 * KW_, 0, st>>>(X, ldx, wt, M, N, K, ks, Y, ldy, p, \
                                                                               glu, rt, wide, FinArgs{});       \
  } while (0)
#define KAFKA_WS_IF(MT_, KC_, KW_)                                      \
  if (mt == MT_ && kc == KC_ && kw == KW_) {                           \
    if (pin)                                                           \
      KAFKA_WS(MT_, KC_, KW_, true);                                   \
    else                                                               \
      KAFKA_WS(MT_, KC_, KW_, false);                                  \
  }
  KAFKA_WS_IF(1, 256, 1)
  else KAFKA_WS_IF(1, 256, 2)
  else KAFKA_WS_IF(2, 256, 1)
  else KAFKA_WS_IF(2, 256, 2)
  else KAFKA_WS_IF(3, 256, 1)
  else KAFKA_WS_IF(4, 128, 1)
  else KAFKA_WS_IF(4, 128, 2)
  else KAFKA_WS_IF(6, 128, 1)
  else return hipErrorInvalidValue;
#undef KAFKA_WS_IF
#undef KAFKA_WS
  return hipGetLastError();
}

extern "C" int kafka_fin_args_size() { return (int)sizeof(FinArgs); }

// Fused decode-layer GEMMs (FIN_RES / FIN_ROPE / FIN_GLU above): one row tile (M <= 128), N % 128 == 0, S in
// {1, 2, 4, 8}; P = [S][M][N] fp32 scratch (unused for S == 1); FIN_GLU needs S == 1.
extern "C" hipError_t kafka_launch_wstream_fin(int fin, const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K,
                                              int mt, int kc, int splits, int kw, int pin, bf16* Y, int64_t ldy,
                                              float* P, const FinArgs* fa_in, hipStream_t st) {
  if (M < 1) return hipSuccess;
  const FinArgs fa = *fa_in;
  if (M > 32 * mt || M > 128 || N % 128 != 0 || K % (kc * splits) != 0) return hipErrorInvalidValue;
  if (!(splits == 1 || splits == 2 || splits == 4 || splits == 8)) return hipErrorInvalidValue;
  if (fin == FIN_GLU) {
    const int ssl = 4096 / (256 * kw);
    int tpr = 1;
    while (tpr * ssl < fa.nss) tpr <<= 1;
    if (splits != 1 || Y == nullptr || tpr > 64 || M * tpr > 256 * kw) return hipErrorInvalidValue;
  } else if (fin == FIN_RES) {
    if (fa.resid == nullptr || fa.nw == nullptr || fa.xn == nullptr || fa.ss_out == nullptr) return hipErrorInvalidValue;
  } else if (fin == FIN_ROPE) {
    if (fa.nss > 32 || fa.positions == nullptr || fa.cos_sin == nullptr || fa.q_out == nullptr || N != (fa.Hq + 2 * fa.Hkv) * 128 ||
        (fa.slots != nullptr && (fa.k_cache == nullptr || fa.v_cache == nullptr)))
      return hipErrorInvalidValue;
  } else {
    return hipErrorInvalidValue;
  }
  if (fin != FIN_GLU && ((splits > 1 && (P == nullptr || fa.tickets == nullptr))))
    return hipErrorInvalidValue;
  const dim3 grid(N / 128, splits);
  const int ks = K / splits;
  const auto* wt = reinterpret_cast<const bf16x8*>(Wt);
  float* p = splits > 1 ? P : nullptr;
  static const int slab16 = [] {
    const char* e = getenv("KAFKA_WSTREAM_SLAB16");
    return e ? atoi(e) : 3;
  }();
  const int wide = (Y != nullptr && (ldy % 8 != 0 || reinterpret_cast<uintptr_t>(Y) % 16 != 0)) ? 0 : (slab16 & 2);
  const int glu = fin == FIN_GLU ? 1 : 0;
#define KAFKA_WF(MT_, KC_, KW_, PIN_, FIN_)                                                                      \
  wstream_gemm_kernel<MT_, KC_, true, KW_, PIN_, FIN_><<<grid, 256 * KW_, 0, st>>>(X, ldx, wt, M, N, K, ks, Y, ldy, p, \
                                                                                  glu, 1, wide, fa)
#define KAFKA_WF_FIN(MT_, KC_, KW_, PIN_)                                    \
  do {                                                                       \
    if (fin == FIN_RES) KAFKA_WF(MT_, KC_, KW_, PIN_, FIN_RES);              \
    else if (fin == FIN_ROPE) KAFKA_WF(MT_, KC_, KW_, PIN_, FIN_ROPE);       \
    else KAFKA_WF(MT_, KC_, KW_, PIN_, FIN_GLU);                             \
  } while (0)
#define KAFKA_WF_IF(MT_, KC_, KW_)                                \
  if (mt == MT_ && kc == KC_ && kw == KW_) {                      \
    if (pin)                                                      \
      KAFKA_WF_FIN(MT_, KC_, KW_, true);                          \
    else                                                          \
      KAFKA_WF_FIN(MT_, KC_, KW_, false);                         \
  }
  KAFKA_WF_IF(1, 256, 1)
  else KAFKA_WF_IF(1, 256, 2)
  else KAFKA_WF_IF(2, 256, 1)
  else KAFKA_WF_IF(2, 256, 2)
  else KAFKA_WF_IF(3, 256, 1)
  else KAFKA_WF_IF(4, 128, 1)
  else KAFKA_WF_IF(4, 128, 2)
  else return hipErrorInvalidValue;
#undef KAFKA_WF_IF
#undef KAFKA_WF_FIN
#undef KAFKA_WF
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_slab_reduce(const float* P, int S, int M, int N, bf16* Y, int64_t ldy,
                                              hipStream_t st) {
  if (M < 1) return hipSuccess;
  if (N % 8 != 0) return hipErrorInvalidValue;
  const int64_t total = (int64_t)M * N / 8;
  slab_reduce_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(P, S, M, N, Y, ldy);
  return hipGetLastError();
}

}  // namespace kafka

namespace kafka {
// Grouped streaming GEMM for the expert MLP (see wstream_grouped_kernel). max_rows bounds any expert's segment
// (the token count T: a token picks an expert at most once); glu: gate_up with fused SwiGLU into Y [n_ent, N/2];
// else combine into out_f32 [T, N].
extern "C" hipError_t kafka_launch_wstream_grouped(const bf16* X, int64_t ldx, const bf16* Wt, int e_local, int N,
                                                  int K, const int* perm_tok, const float* perm_w,
                                                  const int* expert_off, int e_lo, int max_rows, int gather,
                                                  bf16* Y, int64_t ldy, float* out, int64_t ldo, int pin,
                                                  hipStream_t st) {
  if (max_rows < 1 || e_local < 1) return hipSuccess;
  if (N % 64 != 0 || K % 256 != 0 || (out == nullptr) == (Y == nullptr)) return hipErrorInvalidValue;
  // MT = 4 (128-row tiles on 128-deep K chunks) for large steps: with 64-row tiles every
  // row tile of an expert re-streams its weights, and those tiles run far apart in dispatch order (blockIdx.z is the
  // slowest dimension), so no cache keeps the slice between them — an expert with 65..128 rows read its 352 MB twice.
  // KAFKA_MOE_MT4=0 keeps 64-row tiles (A/B).
  static const bool mt4 = [] {
    const char* e = getenv("KAFKA_MOE_MT4");
    return e == nullptr || e[0] != '0';
  }();
  // (64-row tiles stay below 193 rows: an expert then rarely fills a second tile, and they stream faster there —
  // benchmarks/moe_bench.py T = 128 / 192: 493 / 522 vs 517 / 551 us per layer; T = 256 / 384 / 512: 761 / 1002 /
  // 1303 vs 601 / 691 / 1004, profiles/r06/mixtral/)
  const int MT = max_rows <= 32 ? 1 : ((max_rows <= 192 || !mt4) ? 2 : 4);
  const dim3 grid((N + 127) / 128, e_local, (max_rows + 32 * MT - 1) / (32 * MT));
  const auto* wt = reinterpret_cast<const bf16x8*>(Wt);
#define KAFKA_WG(MT_, G_, C_)                                                                                   \
  do {                                                                                                         \
    constexpr int KC_ = MT_ == 4 ? 128 : 256;                                                                  \
    if (pin)                                                                                                   \
      wstream_grouped_kernel<MT_, KC_, G_, C_, true><<<grid, 256, 0, st>>>(X, ldx, wt, N, K, perm_tok, perm_w,      \
                                                                           expert_off, e_lo, Y, ldy, out, ldo);  \
    else                                                                                                       \
      wstream_grouped_kernel<MT_, KC_, G_, C_, false><<<grid, 256, 0, st>>>(X, ldx, wt, N, K, perm_tok, perm_w,     \
                                                                            expert_off, e_lo, Y, ldy, out, ldo); \
  } while (0)
  const bool comb = out != nullptr;
  if (MT == 1) {
    if (gather) { if (comb) KAFKA_WG(1, true, true); else KAFKA_WG(1, true, false); }
    else { if (comb) KAFKA_WG(1, false, true); else KAFKA_WG(1, false, false); }
  } else if (MT == 2) {
    if (gather) { if (comb) KAFKA_WG(2, true, true); else KAFKA_WG(2, true, false); }
    else { if (comb) KAFKA_WG(2, false, true); else KAFKA_WG(2, false, false); }
  } else {
    if (gather) { if (comb) KAFKA_WG(4, true, true); else KAFKA_WG(4, true, false); }
    else { if (comb) KAFKA_WG(4, false, true); else KAFKA_WG(4, false, false); }
  }
#undef KAFKA_WG
  return hipGetLastError();
}
}  // namespace kafka
