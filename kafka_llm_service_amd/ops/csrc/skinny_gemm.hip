// Weight-streaming "skinny" GEMM for decode batches on gfx950:  Y[M, N] = X[M, K] . W[N, K]^T   (bf16 in / out,
// fp32 accumulate, M <= 64).
//
// At decode the weights are read exactly once per step and M (the number of running sequences) is small, so the
// kernel is an HBM stream of W with just enough MFMA work riding on it. hipBLASLt's tilings for these shapes stream
// W at 1.8-3.4 TB/s (o_proj / qkv / down at M = 64, benchmarks/gemm_bench.py); this kernel is built for the stream:
//   * wave tile = 32 output columns (n) x M rows, computed as C^T = W_tile . X^T with v_mfma_f32_32x32x16_bf16:
//       A fragment = 16 B of one W row (lane n = l & 31, k = 8 (l >> 5) + j)  -> W is read straight from HBM into
//                    VGPRs, non-temporal (each byte is used once), never staged through LDS;
//       B fragment = 16 B of one X row (lane m = l & 31)                      -> X (<= 512 KB) is L2-resident;
//   * the 4 waves of a workgroup split K four ways and combine through LDS (so a workgroup = 32 columns x K slice),
//     the grid's second dimension splits K again (SPLITK) when N/32 is too small to fill 256 CUs; split partials are
//     written as fp32 slabs and summed by a small reduce kernel;
//   * the K loop is unrolled by U k-steps with two named register sets (loads of group g+1 issued before the MFMAs
//     of group g), so every wave keeps U * (1 + MT) 16-B loads in flight.
#include "common.h"

namespace kafka {

template <int MT, int U>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                           const bf16* __restrict__ W, int64_t ldw,
                                                           bf16* __restrict__ Y, int64_t ldy,
                                                           float* __restrict__ slab, int M, int N, int K,
                                                           int k_per_wave) {
  __shared__ float red[4][MT * 16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  const int split = blockIdx.y;
  const int k0 = (split * 4 + w) * k_per_wave;
  const bf16* wrow = W + (int64_t)(n0 + r) * ldw + k0 + 8 * h;
  const bf16* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xrow[mt] = X + (int64_t)min(mt * 32 + r, M - 1) * ldx + k0 + 8 * h;

  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;

  bf16x8 wa[U], xa[U][MT], wb[U], xb[U][MT];
  auto load = [&](bf16x8(&wv)[U], bf16x8(&xv)[U][MT], int kk) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wv[u] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wrow + kk + 16 * u));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xv[u][mt] = load_bf16x8(xrow[mt] + kk + 16 * u);
    }
  };
  auto compute = [&](const bf16x8(&wv)[U], const bf16x8(&xv)[U][MT]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32(wv[u], xv[u][mt], acc[mt]);
  };
  constexpr int G = 16 * U;  // k per group
  const int ngroups = k_per_wave / G;
  load(wa, xa, 0);
  int g = 0;
  for (; g + 2 <= ngroups; g += 2) {
    load(wb, xb, (g + 1) * G);
    compute(wa, xa);
    if (g + 2 < ngroups) load(wa, xa, (g + 2) * G);
    compute(wb, xb);
  }
  if (g < ngroups) compute(wa, xa);

  // combine the 4 K-slices of the workgroup through LDS
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[w][mt * 16 + i][lane] = acc[mt][i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < MT * 16 * 64; idx += 256) {
    const int ri = idx >> 6, l = idx & 63;
    const float v = red[0][ri][l] + red[1][ri][l] + red[2][ri][l] + red[3][ri][l];
    const int mt = ri >> 4, i = ri & 15;
    const int m = mt * 32 + (l & 31);
    const int n = n0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    if (m < M) {
      if (slab)
        slab[((int64_t)split * M + m) * N + n] = v;
      else
        Y[(int64_t)m * ldy + n] = (bf16)v;
    }
  }
}

// Y[m, n] = sum_s slab[s, m, n]  (bf16 out), 8 columns per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int S, int M, int N,
                                                             bf16* __restrict__ Y, int64_t ldy) {
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (idx >= (int64_t)M * N) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float* p = slab + ((int64_t)s * M + m) * N + n;
    a += *reinterpret_cast<const f32x4*>(p);
    b += *reinterpret_cast<const f32x4*>(p + 4);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (bf16)a[j];
    o[4 + j] = (bf16)b[j];
  }
  store_bf16x8(Y + (int64_t)m * ldy + n, o);
}

// Host-side plan: returns 0 and fills splitk / k_per_wave, or an error if the shape is not supported.
extern "C" int kafka_skinny_gemm_plan(int M, int N, int K, int U, int* splitk, int* k_per_wave) {
  if (M < 1 || M > 64 || N % 32 != 0 || K % 16 != 0) return 1;
  const int G = 16 * U;
  const int tiles = N / 32;
  int s = 1;
  // grow split-K until the grid has ~2 workgroups per CU, keeping >= 2 groups of K per wave
  while (tiles * s < 512 && K % (4 * (s * 2) * G) == 0 && K / (4 * (s * 2)) >= 2 * G) s *= 2;
  if (K % (4 * s * G) != 0) return 2;
  *splitk = s;
  *k_per_wave = K / (4 * s);
  return 0;
}

extern "C" hipError_t kafka_launch_skinny_gemm(const bf16* X, int64_t ldx, const bf16* W, int64_t ldw, bf16* Y,
                                              int64_t ldy, float* slab, int M, int N, int K, int U, int splitk,
                                              int k_per_wave, hipStream_t st) {
  dim3 grid(N / 32, splitk);
  float* sl = splitk > 1 ? slab : nullptr;
  const bool two = M > 32;
  if (U == 4) {
    if (two) skinny_gemm_kernel<2, 4><<<grid, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, sl, M, N, K, k_per_wave);
    else skinny_gemm_kernel<1, 4><<<grid, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, sl, M, N, K, k_per_wave);
  } else if (U == 8) {
    if (two) skinny_gemm_kernel<2, 8><<<grid, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, sl, M, N, K, k_per_wave);
    else skinny_gemm_kernel<1, 8><<<grid, 256, 0, st>>>(X, ldx, W, ldw, Y, ldy, sl, M, N, K, k_per_wave);
  } else {
    return hipErrorInvalidValue;
  }
  if (splitk > 1) {
    const int64_t total = (int64_t)M * N / 8;
    splitk_reduce_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(slab, splitk, M, N, Y, ldy);
  }
  return hipGetLastError();
}

}  // namespace kafka
