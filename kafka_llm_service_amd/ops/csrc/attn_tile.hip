// Tile attention v3 for gfx950: the cascade prefix pass (all decode rows of a batch against the shared system
// prompt's KV, SURVEY.md §2.6 `shared_prefix_decode_attention`) and chunked / causal prefill
// (`prefill_flash_attention`). Same work items, page layouts and outputs as attn_prefill_kernel (attention.hip);
// selected as tile variant 3 (ops.tile_rows(3) = 256 rows).
//
// Structure (one workgroup = 8 waves = two waves per SIMD, 256 query rows of one KV head):
//   * each wave owns 32 query rows (one 32-row MFMA block); the partner wave's MFMAs run beside this wave's softmax
//     VALU (a 4-wave / 64-row layout with one wave per SIMD halves the LDS reads but hides no latency: -3.8 % on the
//     headline, profiles/r04/bench_ab_tile_prologue.jsonl);
//   * K/V arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction) in 64-key tiles (4 pages: 16 KB
//     K + 16 KB V) into a 3-slot ring: tile j+2 is issued right after the barrier that retires tile j, so two
//     tiles (64 KB per CU) stay in flight across every barrier. No register round trip, no ds_write pass, and one
//     counted `s_waitcnt vmcnt(8)` + one `s_barrier` per 64 keys (v2: a vmcnt + ds_write pass + barrier per 32);
//   * the DMA destination is lane-linear, so layouts are chosen on the SOURCE side: a K page (plane-major, see
//     rope_kv.hip) is copied verbatim — its plane-major order already makes the A-fragment reads of a 16-lane
//     ds_read_b128 group hit 16 distinct bank slots; the V^T page is copied with the 16-B halves of rows 8..15 of
//     every 16-row group swapped (source lane permutation L ^ ((L >> 4) & 1)), which makes the V^T fragment reads
//     conflict-free too (cdna_hip_programming.md §5.4 rule 21: linear destination, permuted source, same
//     permutation on the read);
//   * softmax in the S^T layout (lane = query column: row max / sum are lane-local plus one permlane32 swap) with a
//     deferred rescale (T13): O and l are rescaled only when some row's max grew by more than 2^THR, so the 64-wide
//     O rescale almost never runs; the row sums run on the matrix pipe (an MFMA against a ones operand).
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace kafka {

namespace tile3 {
constexpr int PAGE = 16;
constexpr int D = 128;
constexpr int TK = 64;                  // keys per tile (4 pages)
constexpr int KBYTES = TK * D * 2;      // K part of a ring slot
constexpr int SLOT = 2 * KBYTES;        // K + V
constexpr int MAXPG = 2048;             // page ids of an item's key range staged in LDS
template <int NSLOT>
constexpr int lds_bytes() { return NSLOT * SLOT + MAXPG * 4 + 64; }
constexpr float THR = 24.f;             // deferred-rescale threshold (log2 domain): P <= 2^THR, fp32-safe
}  // namespace tile3

struct TileItem {
  int q_start, q_count, bt_row, kv_lo, kv_hi, split, alt, pad1;
};

// Second partial buffer of a launch (fp32 [rows, Hq, S, D] + lse [rows, Hq, S]) for the items flagged `alt`: the
// cascade's prefix pass also serves the new-turn prefill rows of the step, whose prefix partials join their own
// suffix tiles' partials (merged by attn_merge) instead of the decode rows' bf16 slots. Row = token - tok_off.
struct AltPart {
  float* part = nullptr;
  float* lse = nullptr;
  int S = 0;
  int tok_off = 0;
};

typedef __attribute__((address_space(3))) void lds_void_t;

template <int AUX = 0>
__device__ __forceinline__ void dma16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds, 16, 0, AUX);
}

// max without fmaxf's NaN-quieting: IEEE-mode v_max_f32 needs each MFMA result canonicalised first (a v_max x, x
// per value: 3 VALU ops per pair of scores); llvm.maximum lowers to gfx950's v_maximum3_f32, 3 inputs per op, no
// canonicalisation (it propagates NaN instead of dropping it: a NaN score poisons its row either way)
__device__ __forceinline__ float t3_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float t3_xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return t3_max(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float t3_xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int N>
__device__ __forceinline__ void t3_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// raw barrier, opaque to the compiler's memory model: no vmcnt(0) drain of the DMAs in flight (a __syncthreads()
// would emit one), and no LDS access is moved across it
__device__ __forceinline__ void t3_barrier() { asm volatile("s_barrier" ::: "memory"); }

// diagnostic-build stamp (ABL == 8): the 100 MHz constant clock, comparable across CUs and XCDs
__device__ __forceinline__ uint64_t t3_rt() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// s_waitcnt vmcnt(n * DPT) for a wave-uniform n in [0, 2] (the count is an immediate)
template <int DPT>
__device__ __forceinline__ void t3_wait_tiles(int n) {
  if (n >= 2)
    t3_wait_vmcnt<2 * DPT>();
  else if (n == 1)
    t3_wait_vmcnt<DPT>();
  else
    t3_wait_vmcnt<0>();
}

// ABL = 8 (diagnostic build, KAFKA_TILE_ABL=8, benchmarks/attn_tile_stamps.py): workgroup phase stamps on the 100 MHz
// clock; the full kernel runs and lse_part is overwritten with u64 [entry, prologue done, first tile landed, loop
// done, epilogue done, 0, 0, 0] per workgroup blockIdx.y * Hkv + blockIdx.x.
// PST = 1: the bf16 prefix partials are stored sc1 (16-B stores whose lines leave this XCD's L2: the reader, the
// suffix decode's merge, runs on any XCD, and the launch ends with fewer dirty lines to write back)
template <int ABL = 0, int KVAUX = 0, int PST = 0>
__global__ __launch_bounds__(512, 2) void attn_tile_kernel(const TileItem* __restrict__ items,
                                                           const bf16* __restrict__ q, int64_t q_stride,
                                                           const bf16* __restrict__ k_cache,
                                                           const bf16* __restrict__ v_cache, int Hkv, int G,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ q_limit, bf16* __restrict__ out,
                                                           int64_t out_stride, float* __restrict__ out_part,
                                                           float* __restrict__ lse_part, int S_total,
                                                           float scale_log2, int part_bf16, AltPart ap) {
  using namespace tile3;
  constexpr int RB = 1;                   // 32-row MFMA blocks per wave
  constexpr int NSLOT = 3;                // ring slots (4: 30.9 vs 29.9 us per cascade launch,
                                          // profiles/r05/cascade/cascade_nslot_*.jsonl)
  constexpr int NW = 8;                   // waves
  constexpr int DPT = 32 / NW;            // LDS-DMA instructions per wave per tile (16 K + 16 V pieces per tile)
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes<NSLOT>()];
  int* s_pages = reinterpret_cast<int*>(smem + NSLOT * SLOT);
  int* s_hi = s_pages + MAXPG;

  uint64_t ph[5] = {0, 0, 0, 0, 0};
  if constexpr (ABL == 8) ph[0] = t3_rt();
  const TileItem it = items[blockIdx.y];
  // an item flagged alt without an alt buffer (host bug) would write row B + q of the main buffer, past its end:
  // dropped (workgroup-uniform), as the decode kernel drops malformed items
  if (it.alt != 0 && ap.part == nullptr) return;
  const int kvh = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int Hq = Hkv * G;

  // ---- rows of this wave: R = 64 w + 32 rb + r -> token R / G, head kvh G + R % G
  int token[RB], head[RB], limit[RB];
  bool valid[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int R = 32 * RB * w + 32 * rb + r;
    const int tok = R / G;
    valid[rb] = tok < it.q_count;
    token[rb] = it.q_start + tok;
    head[rb] = kvh * G + R % G;
  }
  // prologue loads that depend only on the work item go out together (one round trip): the item's page ids and the
  // causal limits; Q fragments (B operand of S^T = K . Q^T: lane (r, h) holds Q[row r][16 kk + 8 h + j]) follow the
  // first DMAs
  const int lo0 = it.kv_lo;
  const int pg00 = (lo0 & ~63) >> 4;
  const int npg_all0 = ((it.kv_hi + 15) >> 4) - pg00;
  const int npg0 = min(npg_all0, 2048);
  const int* bt0 = block_tables + (int64_t)it.bt_row * bt_stride;
  constexpr int PPT = 2048 / (512 / RB);  // page ids per thread (MAXPG / threads)
  int pgv[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int i = tid + k * (512 / RB);
    pgv[k] = i < npg0 ? bt0[pg00 + i] : 0;
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) limit[rb] = valid[rb] ? q_limit[token[rb]] : -1;
  bf16x8 qf[RB][D / 16];
  auto load_q = [&]() {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const bf16* qrow = q + (int64_t)token[rb] * q_stride + (int64_t)head[rb] * D + 8 * h;
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        if (valid[rb]) {
          qf[rb][kk] = load_bf16x8(qrow + 16 * kk);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) qf[rb][kk][j] = (bf16)0.f;
        }
      }
    }
  };
  // (Q fragments are loaded after the first K/V tiles' DMAs are issued: those are the critical path — Q loads issued
  // ahead of them delayed the first tile, -0.6 % on the headline, profiles/r04/bench_ab_tile_prologue.jsonl)
  // per-block wave-uniform bounds: keys past hi_b are masked for every row of the block, keys <= wmin_b for none
  int hi_b[2], wmin_b[2];  // (RB == 1: block 1 mirrors block 0)
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    int mx = limit[rb], mn = valid[rb] ? limit[rb] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mx = max(mx, __shfl_xor(mx, o, 64));
      mn = min(mn, __shfl_xor(mn, o, 64));
    }
    hi_b[rb] = min(it.kv_hi, mx + 1);
    wmin_b[rb] = mn;
  }
  if constexpr (RB == 1) {
    hi_b[1] = hi_b[0];
    wmin_b[1] = wmin_b[0];
  }
  // (a block without valid rows does not make tiles edges: its rows are never written)
  const int hi_e = min(hi_b[0] > 0 ? hi_b[0] : 0x7fffffff, hi_b[1] > 0 ? hi_b[1] : 0x7fffffff);
  const int lo = it.kv_lo;
  const int base = lo & ~(TK - 1);
  const int pg0 = base >> 4;
  const int npg_all = ((it.kv_hi + 15) >> 4) - pg0;
  const int npg = min(npg_all, MAXPG);
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int i = tid + k * (512 / RB);
    if (i < npg) s_pages[i] = pgv[k];
  }
  if (lane == 0) s_hi[w] = max(hi_b[0], hi_b[1]);
  __syncthreads();
  if constexpr (ABL == 8) ph[1] = t3_rt();
  int hi_wg = s_hi[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) hi_wg = max(hi_wg, s_hi[i]);
  // (the host never builds an item spanning more than MAXPG pages; a violating item yields NaN rows)
  const bool fits = npg_all <= MAXPG;
  const int ntiles = (fits && hi_wg > lo) ? (hi_wg - base + TK - 1) / TK : 0;

  const int jf = (lo > base && ntiles > 0) ? 1 : 0;  // (= j0 below)
  auto tile_of = [&](int i) { return i < ntiles - jf ? i + jf : 0; };
  // ---- DMA of processing index i (tile t(i)) into ring slot i % NSLOT: wave w copies page w of the tile
  auto issue = [&](int i) {
    const int j = i;
    // wave w: page (w * 4) / NW of the tile, its 1-KiB pieces c0 .. c0 + DPT/2 - 1 of K and of V
    const int pw = (w * 4) / NW, c0 = (w % (NW / 4)) * (DPT / 2);
    const int pg = s_pages[min(4 * tile_of(i) + pw, npg - 1)];
    const int64_t poff = ((int64_t)pg * Hkv + kvh) * (PAGE * D);
    const bf16* kp = k_cache + poff;
    const bf16* vp = v_cache + poff;
    char* kd = smem + (j % NSLOT) * SLOT + pw * 4096;
    char* vd = kd + KBYTES;
#pragma unroll
    for (int cc = 0; cc < DPT / 2; ++cc) {
      const int c = c0 + cc;
      const int L = c * 64 + lane;
      dma16<KVAUX>(kp + L * 8, kd + c * 1024);
      dma16<KVAUX>(vp + (L ^ ((L >> 4) & 1)) * 8, vd + c * 1024);
    }
  };
#pragma unroll
  for (int j = 0; j < NSLOT - 1; ++j)
    if (j < ntiles) issue(j);
  load_q();

  // Running state per row block: O^T accumulators; row sums `ls` as an MFMA accumulator (every register of a lane
  // holds its column's sum ones . P: 8 MFMAs per tile instead of 64 adds); the running max m (exp2 domain).
  // (Folding -m into the QK^T accumulator init would save the per-score FMA too, but needs Q prescaled by
  // scale * log2(e) in bf16: +0.4 % relative score error, 0.037 abs on a peaked row vs 0.02 tolerance — rejected.)
  f32x16 o[RB][D / 32], ls[RB];
  float m[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[rb][t][i] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) ls[rb][i] = 0.f;
    m[rb] = -INFINITY;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;

  // ---- one 64-key tile (processing index j) from ring slot j % NSLOT
  auto tile_body = [&](auto masked_c, int j, int key0) {
    constexpr bool MASKED = decltype(masked_c)::value;
    const char* Ks = smem + (j % NSLOT) * SLOT;  // [page 4][plane 16][key 16][16 B]
    const char* Vs = Ks + KBYTES;                // [page 4][d 128][2 x 16 B] (halves swapped on rows 8..15 of 16)
    // S^T = K . Q^T for both 32-key halves (kb) and both row blocks
    f32x16 s[RB][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8 kf[D / 16];
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk)
        kf[kk] = *reinterpret_cast<const bf16x8*>(Ks + (2 * kb + (r >> 4)) * 4096 + ((2 * kk + h) * 16 + (r & 15)) * 16);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        f32x16 acc = {};
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) acc = mfma32(kf[kk], qf[rb][kk], acc);
        s[rb][kb] = acc;
      }
    }
    if constexpr (MASKED) {  // wave-uniform per 32-key half: range edges and the causal diagonal
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int k0 = key0 + 32 * kb;
          if ((k0 < lo) | (k0 + 32 > hi_b[rb]) | (k0 + 31 > wmin_b[rb])) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
              if (!((key >= lo) & (key < hi_b[rb]) & (key <= limit[rb]))) s[rb][kb][i] = -INFINITY;
            }
          }
        }
    }
    // row max; deferred rescale, rare: only when a row's max passed m + THR (or at its first finite scores)
    float smax[2];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      // two chains of v_maximum3_f32 (m = max3(m, a, b)): 16 VALU ops for the 32 scores of a lane
      float ma = t3_max(s[rb][0][0], s[rb][1][0]), mb = t3_max(s[rb][0][1], s[rb][1][1]);
#pragma unroll
      for (int i = 2; i < 16; i += 2) {
        ma = t3_max(t3_max(ma, s[rb][0][i]), s[rb][1][i]);
        mb = t3_max(t3_max(mb, s[rb][0][i + 1]), s[rb][1][i + 1]);
      }
      smax[rb] = t3_xor32_max(t3_max(ma, mb)) * scale_log2;
    }
    bool need = false;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) need = need | !(smax[rb] <= m[rb] + THR);
    if (__any(need)) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const float mn = fmaxf(m[rb], smax[rb]);
        const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m[rb] - mn);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) o[rb][t] *= alpha;
        ls[rb] *= alpha;
        m[rb] = mn;
      }
    }
    // P = exp2(S scale - m) (<= 2^THR), O^T += V^T . P, row sums += ones . P (both on the matrix pipe). V^T fragments (A
    // operand: lane (r, h) = row d = 32 t + r, keys 8h .. 8h+7 of a page) are read per 32-key half (32 VGPRs live).
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8 vf[2][D / 32];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          const int d = 32 * t + r;
          vf[s2][t] = *reinterpret_cast<const bf16x8*>(Vs + (2 * kb + s2) * 4096 + d * 32 + 16 * (h ^ ((d >> 3) & 1)));
        }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const float mu = (m[rb] == -INFINITY) ? 0.f : m[rb];
        bf16x8 pf[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float x = fmaf(s[rb][kb][i], scale_log2, -mu);
          pf[i >> 3][i & 7] = (bf16)fast_exp2(x);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int t = 0; t < D / 32; ++t) o[rb][t] = mfma32(vf[s2][t], pf[s2], o[rb][t]);
          ls[rb] = mfma32(ones, pf[s2], ls[rb]);
        }
      }
    }
  };

  // Processing order: the interior tiles first, then the edge tiles (range ends, causal diagonal), so each kind runs
  // in a loop of its own with its own body — interior tiles without any masking code (one straight-line block up to
  // the rare rescale branch and one after it: the scheduler can put the max of one row block beside the other's QK^T
  // MFMAs and the exp of one beside the other's PV MFMAs). Online softmax does not care about key order; the DMA
  // ring streams in processing order. Index i -> tile t(i): tiles j0 .. ntiles-1, then tile 0 when it starts below lo.
  const int j0 = (lo > base && ntiles > 0) ? 1 : 0;
  const int wmin_all = min(wmin_b[0], wmin_b[1]);
  const int clean_end = min(hi_e, wmin_all == 0x7fffffff ? 0x7fffffff : wmin_all + 1);  // keys below: no mask
  const int j_e = clean_end > base ? min(ntiles, (clean_end - base) / TK) : 0;
  const int n_int = max(0, j_e - j0);
  auto step = [&](int i) {
    // tile i landed (this wave's pieces; the NSLOT - 2 younger tiles stay in flight), then every wave's: the
    // barrier also retires every read of slot (i + NSLOT - 1) % NSLOT (index i - 1's)
    t3_wait_tiles<DPT>(min(NSLOT - 2, ntiles - 1 - i));
    t3_barrier();
    if (i + NSLOT - 1 < ntiles) issue(i + NSLOT - 1);
  };
  for (int i = 0; i < n_int; ++i) {
    step(i);
    if constexpr (ABL == 8)
      if (i == 0) ph[2] = t3_rt();
    tile_body(std::false_type{}, i, base + TK * tile_of(i));
  }
  for (int i = n_int; i < ntiles; ++i) {
    step(i);
    tile_body(std::true_type{}, i, base + TK * tile_of(i));
  }

  if constexpr (ABL == 8) ph[3] = t3_rt();
  // ---- epilogue: through a per-wave LDS transpose (slot ntiles % NSLOT is idle: its last tile was read before the
  // barrier every wave passed NSLOT - 1 tiles ago), so every store instruction writes whole 128-B lines
  const bool part = it.split >= 0;
  const bool alt = part && it.alt != 0 && ap.part != nullptr;  // (workgroup-uniform)
  float* const opart = alt ? ap.part : out_part;
  float* const lpart = alt ? ap.lse : lse_part;
  const int Sx = alt ? ap.S : S_total, toff = alt ? ap.tok_off : 0;
  const bool pbf = part_bf16 && !alt;
  char* slab = smem + (ntiles % NSLOT) * SLOT + w * (4096 * RB);
  const int cc = lane & 7;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    if (!__any(valid[rb])) continue;  // wave-uniform
    const float ll = fits ? ls[rb][0] : __builtin_nanf("");
    const float inv = ll > 0.f ? 1.f / ll : (fits ? 0.f : ll);
    if (ABL != 8 && part && valid[rb] && h == 0) {
      float* lp = lpart + ((int64_t)(token[rb] - toff) * Hq + head[rb]) * Sx + it.split;
      *lp = ll > 0.f ? m[rb] + log2f(ll) : (fits ? -INFINITY : ll);
    }
    const int R0 = 32 * RB * w + 32 * rb;
    const int nvalid = it.q_count * G - R0;
    char* sl = slab + rb * 4096;
    auto flush = [&](int rd) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = (lane >> 3) + 8 * k;
        const f32x4 v = *reinterpret_cast<const f32x4*>(sl + row * 128 + 16 * (cc ^ (row & 7)));
        if (row < nvalid) {
          const int R2 = R0 + row, tok2 = it.q_start + R2 / G, head2 = kvh * G + R2 % G;
          f32x4* dst;
          if (PST && pbf) {
            float* d = reinterpret_cast<float*>(reinterpret_cast<bf16*>(out_part) +
                                                (((int64_t)tok2 * Hq + head2) * S_total + it.split) * D + 64 * rd + 8 * cc);
            store16_slab(d, v);  // (common.h: asm store + its hazard wait state)
            continue;
          }
          if (part && !pbf)
            dst = reinterpret_cast<f32x4*>(opart + (((int64_t)(tok2 - toff) * Hq + head2) * Sx + it.split) * D +
                                           32 * rd + 4 * cc);
          else if (part)  // bf16 partial (O / l in [-max|v|, max|v|]: half the bytes of the cascade round trip)
            dst = reinterpret_cast<f32x4*>(reinterpret_cast<bf16*>(out_part) +
                                           (((int64_t)tok2 * Hq + head2) * S_total + it.split) * D + 64 * rd + 8 * cc);
          else
            dst = reinterpret_cast<f32x4*>(out + (int64_t)tok2 * out_stride + (int64_t)head2 * D + 64 * rd + 8 * cc);
          *dst = v;
        }
      }
    };
    if (part && !pbf) {
#pragma unroll
      for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int c = 2 * i4 + h;
          const f32x4 v = {o[rb][rd][4 * i4] * inv, o[rb][rd][4 * i4 + 1] * inv, o[rb][rd][4 * i4 + 2] * inv,
                           o[rb][rd][4 * i4 + 3] * inv};
          *reinterpret_cast<f32x4*>(sl + r * 128 + 16 * (c ^ (r & 7))) = v;
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
            for (int jj = 0; jj < 4; ++jj) v[jj] = (bf16)(o[rb][2 * rd + tt][4 * i4 + jj] * inv);
            *reinterpret_cast<bf16x4*>(sl + r * 128 + 16 * ((4 * tt + i4) ^ (r & 7)) + 8 * h) = v;
          }
        flush(rd);
      }
    }
  }
  if constexpr (ABL == 8) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ph[4] = t3_rt();
    if (tid == 0) {
      uint64_t* dst = reinterpret_cast<uint64_t*>(lse_part) + ((int64_t)blockIdx.y * Hkv + blockIdx.x) * 8;
#pragma unroll
      for (int k = 0; k < 5; ++k) dst[k] = ph[k];
    }
  }
}

// Host launcher (bf16 KV only; the fp8 cache keeps tile variant 0). Items: int32 [n, 8] as attn_prefill_kernel.
extern "C" hipError_t kafka_launch_attn_tile(const void* items, int n_items, const bf16* q, int64_t q_stride,
                                            const void* k_cache, const void* v_cache, int Hkv, int G, int D,
                                            const int* block_tables, int bt_stride, const int* q_limit, bf16* out,
                                            int64_t out_stride, float* out_part, float* lse_part, int S_total,
                                            float scale, int part_bf16, float* alt_part, float* alt_lse, int alt_S,
                                            int alt_tok_off, hipStream_t st) {
  if (n_items == 0) return hipSuccess;
  if (D != 128 || G < 1 || G > 32 || (256 % G) != 0 || n_items > 65535) return hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  static const bool stamps = [] {  // diagnostic build (benchmarks/attn_tile_stamps.py)
    const char* e = getenv("KAFKA_TILE_ABL");
    return e && atoi(e) == 8;
  }();
  // The cascade prefix pass (bf16 partials) reads each K / V tile of the shared prefix once per KV head and 256 query
  // rows (one workgroup at the headline's 64 streams): its DMAs go nt (aux = 2), +0.9 % on the headline
  // (profiles/r05/cascade/bench_ab_kv_nt.jsonl). Prefill launches keep the default policy: their query tiles re-read
  // the same keys.
  // Its bf16 partials are stored sc1 (16-B stores that leave this XCD's L2: +0.2..0.6 %, bench_ab_part_sc1.jsonl).
  auto kern = stamps ? attn_tile_kernel<8> : part_bf16 ? attn_tile_kernel<0, 2, 1> : attn_tile_kernel<0>;
  kern<<<dim3(Hkv, n_items), 512, 0, st>>>(reinterpret_cast<const TileItem*>(items), q, q_stride,
                                           static_cast<const bf16*>(k_cache), static_cast<const bf16*>(v_cache), Hkv,
                                           G, block_tables, bt_stride, q_limit, out, out_stride, out_part, lse_part,
                                           S_total, scale_log2, part_bf16, AltPart{alt_part, alt_lse, alt_S, alt_tok_off});
  return hipGetLastError();
}

}  // namespace kafka
