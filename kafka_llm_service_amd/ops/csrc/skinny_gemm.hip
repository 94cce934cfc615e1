// Skinny MFMA GEMM for mixed decode + prefill steps (129..256 rows) on the wave-tiled weights (gfx950).
//     Y[M, N] = X[M, K] . W[N, K]^T,   128 < M <= 256,  W in the wave-tiled layout of wstream_gemm.hip
//
// Between the weight-streaming decode GEMM (M <= 128: one MFMA B-fragment per 1 KB weight load, X from LDS) and
// hipBLASLt (large M) sit the steps that carry 64 decodes plus a new turn's prompt: 130-300 rows, where hipBLASLt
// runs at 1.3-2 TB/s (profiles/r02/gemm_sweep_M129_320.log) although the shape is still weight-bound: at 256 rows a
// workgroup that keeps every operand fragment busy on two MFMAs streams its weights at HBM rate.
//
//   * workgroup = 8 waves, tile 256 rows x 128 columns; wave w owns rows 64 (w & 3) .. + 64 and the column-tile
//     pair (cb * 4 + 2 (w >> 2), + 1): a 2 x 2 block of 32 x 32 MFMA tiles, so each A fragment (X) and each B
//     fragment (W) read from LDS feeds TWO v_mfma_f32_32x32x16_bf16 — the operand traffic per MFMA of the decode
//     kernel halved;
//   * both operands arrive by LDS-DMA (global_load_lds_dwordx4: no register round trip) into a 3-stage ring of
//     64-deep K stages (X 32 KB + W 16 KB per stage, 144 KB): per wave and stage 4 X + 2 W instructions, a counted
//     `s_waitcnt vmcnt` and one raw `s_barrier` per stage. W instructions are whole 1 KB B fragments (the tiled
//     layout is lane-linear already); X rows are 128 B with 16-B chunk c of row m at chunk c ^ (m & 7) — the DMA
//     writes lane-linear, so each lane LOADS the chunk that belongs at its LDS slot (source-side permutation) and the
//     A-fragment reads of 32 rows spread over the banks;
//   * split-K over gridDim.y for small N (fp32 slabs [S, M, N], summed by the consumer kernels like the decode
//     GEMM's); one split writes bf16, or with GLU-interleaved weights (tile 2j = gate, 2j + 1 = up: a wave's pair)
//     the activated silu(gate) * up [M, N / 2] straight from the accumulators.
// Rows >= M load row M - 1 (finite garbage, never stored).
#include "common.h"

namespace kafka {

namespace skg {
constexpr int BM = 256, BN = 128;
constexpr int NW = 8;  // waves
template <int BK>
struct Cfg {
  static constexpr int XB = BM * BK * 2;     // X bytes per stage (32 KB at BK = 64)
  static constexpr int WB = BN * BK * 2;     // W bytes per stage (16 KB at BK = 64)
  static constexpr int STAGE = XB + WB;
  static constexpr int DX = XB / 1024 / NW;  // X DMA instructions per wave per stage
  static constexpr int DW = WB / 1024 / NW;  // W DMA instructions per wave per stage
  static constexpr int DPS = DX + DW;
  static constexpr int RB = BK * 2;          // LDS bytes of one X row per stage
  static constexpr int CPR = BK / 8;         // 16-B chunks per X row per stage
};
}  // namespace skg

typedef __attribute__((address_space(3))) void skg_lds_t;

__device__ __forceinline__ void skg_dma16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (skg_lds_t*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void skg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BK, int NS, int OCC>
__global__ __launch_bounds__(512, OCC) void skinny_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                               const bf16x8* __restrict__ Wt, int M, int N, int K,
                                                               int ks, bf16* __restrict__ Y, int64_t ldy,
                                                               float* __restrict__ P, int glu) {
  using namespace skg;
  using C = Cfg<BK>;
  constexpr int XB = C::XB, STAGE = C::STAGE, DX = C::DX, DW = C::DW, DPS = C::DPS, RB = C::RB, CPR = C::CPR;
  static_assert(DX >= 1 && DW >= 1 && (CPR == 8 || CPR == 4), "stage shape");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int rg = w & 3, cg = w >> 2;
  const int cb = blockIdx.x;
  const int k0 = blockIdx.y * ks;
  const int nst = ks / BK;
  const int K16 = K >> 4;

  // per-lane DMA sources of this wave's share of a stage (stage s adds s * BK to the K offset)
  // X: instruction j = DX w + u covers LDS bytes [1024 j, +1024) = 1024 / RB rows; lane -> row, slot (chunk c of row
  // m stored at slot c ^ (m % CPR))
  const bf16* xsrc[DX];
#pragma unroll
  for (int u = 0; u < DX; ++u) {
    const int j = DX * w + u, row = (1024 / RB) * j + lane / CPR, slot = lane % CPR;
    const int m = row < M ? row : M - 1;
    xsrc[u] = X + (int64_t)m * ldx + k0 + 8 * (slot ^ (row % CPR));
  }
  // W: instruction j = DW w + u = (tile t = j / KB, k-block kk = j % KB): one B fragment of column tile cb * 4 + t
  constexpr int KB = BK / 16;
  const bf16x8* wsrc[DW];
#pragma unroll
  for (int u = 0; u < DW; ++u) {
    const int j = DW * w + u, t = j / KB, kk = j % KB;
    wsrc[u] = Wt + ((int64_t)(cb * 4 + t) * K16 + (k0 >> 4) + kk) * 64 + lane;
  }
  auto issue = [&](int s) {
    char* base = smem + (s % NS) * STAGE;
#pragma unroll
    for (int u = 0; u < DX; ++u) skg_dma16(xsrc[u] + s * BK, base + (DX * w + u) * 1024);
#pragma unroll
    for (int u = 0; u < DW; ++u) skg_dma16(wsrc[u] + (int64_t)s * (BK / 16) * 64, base + XB + (DW * w + u) * 1024);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  // s_waitcnt vmcnt(n * DPS) for a wave-uniform n in [0, NS - 2] (the count is an immediate)
  auto wait_stage = [&](int n) {
    if (NS > 5 && n >= 4) skg_vmcnt<(NS > 5 ? 4 : 0) * DPS>();
    else if (NS > 4 && n >= 3) skg_vmcnt<(NS > 4 ? 3 : 0) * DPS>();
    else if (NS > 3 && n >= 2) skg_vmcnt<(NS > 3 ? 2 : 0) * DPS>();
    else if (n >= 1) skg_vmcnt<DPS>();
    else skg_vmcnt<0>();
  };
  for (int s = 0; s < NS - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    // this wave's DMAs of stage s have landed (the NS - 2 later stages may still be in flight), then every wave's
    // have, and every wave is done reading slot (s + NS - 1) % NS (stage s - 1)
    wait_stage(min(NS - 2, nst - 1 - s));
    asm volatile("s_barrier" ::: "memory");
    if (s + NS - 1 < nst) issue(s + NS - 1);
    const char* xs = smem + (s % NS) * STAGE;
    const char* ws = xs + XB;
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int c = 2 * kk + h;
      const int m0 = 64 * rg + r, m1 = m0 + 32;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(xs + m0 * RB + 16 * (c ^ (m0 % CPR)));
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(xs + m1 * RB + 16 * (c ^ (m1 % CPR)));
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(ws + ((2 * cg) * KB + kk) * 1024 + lane * 16);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(ws + ((2 * cg + 1) * KB + kk) * 1024 + lane * 16);
      acc[0][0] = mfma32(a0, b0, acc[0][0]);
      acc[0][1] = mfma32(a0, b1, acc[0][1]);
      acc[1][0] = mfma32(a1, b0, acc[1][0]);
      acc[1][1] = mfma32(a1, b1, acc[1][1]);
    }
  }

  // epilogue: C lane layout (lanes along N): acc[a][b][i] -> row 64 rg + 32 a + (i & 3) + 8 (i >> 2) + 4 h,
  // column (cb * 4 + 2 cg + b) * 32 + r
  const int nb0 = cb * 4 + 2 * cg;
  if (glu && P == nullptr) {  // (gate, up) = (tile nb0, tile nb0 + 1): output column block nb0 / 2
    const int n = (nb0 >> 1) * 32 + r;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 64 * rg + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < M) {
          const float g = acc[a][0][i], u = acc[a][1][i];
          Y[(int64_t)m * ldy + n] = (bf16)(g / (1.0f + __expf(-g)) * u);
        }
      }
    return;
  }
  if (P) {
    // split-K slab through a per-wave LDS transpose (the ring is dead once every wave is past its last stage): each
    // lane then writes 4 consecutive columns of a row with one 16-B sc1 store, 16 lanes per 256-B row (as the decode
    // GEMM's slabs)
    __syncthreads();  // (workgroup-uniform: P is a kernel argument)
    float* tp = reinterpret_cast<float*>(smem) + w * 64 * 64;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) tp[(32 * a + (i & 3) + 8 * (i >> 2) + 4 * h) * 64 + 32 * b + r] = acc[a][b][i];
    // (one wave's LDS accesses complete in order: the reads below see its writes)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int q = j * 64 + lane, row = q >> 4, c4 = q & 15;
      const f32x4 v = *reinterpret_cast<const f32x4*>(tp + row * 64 + 4 * c4);
      const int m = 64 * rg + row;
      // GLU-interleaved pair: tile nb0 -> gate columns, nb0 + 1 -> up columns N/2 + ...
      const int n = glu ? ((c4 >> 3) ? (N >> 1) : 0) + (nb0 >> 1) * 32 + 4 * (c4 & 7) : nb0 * 32 + 4 * c4;
      if (m < M) store16_slab(P + ((int64_t)blockIdx.y * M + m) * N + n, v);
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int nb = nb0 + b;
    // GLU-interleaved tiles written un-split or as slabs: tile 2j -> gate columns [32 j, +32), 2j + 1 -> up N/2 + 32 j
    const int n = glu ? ((nb & 1) ? (N >> 1) : 0) + (nb >> 1) * 32 + r : nb * 32 + r;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 64 * rg + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < M) {
          if (P)
            P[((int64_t)blockIdx.y * M + m) * N + n] = acc[a][b][i];
          else
            Y[(int64_t)m * ldy + n] = (bf16)acc[a][b][i];
        }
      }
  }
}

// Split plan for a shape (mirrored by ops.skinny_plan): the fewest power-of-two splits that give >= 192 workgroups
// while every split keeps >= 4 K stages of 64.
extern "C" int kafka_skinny_plan(int M, int N, int K, int max_splits, int* splits) {
  using namespace skg;
  if (M <= 128 || M > BM || N % BN != 0 || K % 64 != 0) return 1;
  const int nx = N / BN;
  int s = 1;
  while (s * 2 <= max_splits && nx * s < 192 && K % (64 * s * 2) == 0 && K / (s * 2) >= 256) s *= 2;
  *splits = s;
  return 0;
}

// BK 64 x 3 stages (144 KB of LDS, one workgroup per CU; BK 32 x 6 stages and BK 32 x 3 stages at two workgroups
// per CU measured slower, profiles/r03/skinny_gemm/)
extern "C" hipError_t kafka_launch_skinny_gemm(const bf16* X, int64_t ldx, const bf16* Wt, int M, int N, int K,
                                              int splits, int glu, bf16* Y, int64_t ldy, float* P, hipStream_t st) {
  using namespace skg;
  if (M <= 0 || M > BM || N % BN != 0 || splits < 1 || K % (64 * splits) != 0 || ldx % 8 != 0) return hipErrorInvalidValue;
  if ((splits > 1) != (P != nullptr) || (splits == 1 && Y == nullptr) || (glu && N % 64 != 0))
    return hipErrorInvalidValue;
  const dim3 grid(N / BN, splits);
  const auto* wt = reinterpret_cast<const bf16x8*>(Wt);
  const int ks = K / splits;
  skinny_gemm_kernel<64, 3, 1><<<grid, NW * 64, 0, st>>>(X, ldx, wt, M, N, K, ks, Y, ldy, P, glu);
  return hipGetLastError();
}

}  // namespace kafka
