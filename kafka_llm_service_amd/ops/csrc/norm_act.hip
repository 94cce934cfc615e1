// RMSNorm, fused residual-add + RMSNorm, and SwiGLU activation for gfx950.
//
// All three are HBM-bound streaming ops: one workgroup per token row, 16-byte (bf16x8) loads per lane, the
// row kept in registers between the reduction and the scale pass (one HBM read + one write per element),
// fp32 accumulation. The residual add is fused into the norm so the decoder layer reads the residual
// stream once per sub-block instead of three times.
//
// Split-K slab inputs: the decode GEMM (wstream_gemm.hip) leaves its output as S fp32 partial slabs
// P[S][T][n]; every kernel here can take such a slab instead of a bf16 input and sums the S partials while
// loading (load_in8 in common.h), so the split-K combine costs no launch of its own.
#include <cstdlib>

#include "common.h"

namespace kafka {

// y = x * rsqrt(mean(x^2) + eps) * w     (x: [T, d] with row stride, out: [T, d] contiguous)
// If RESID: r = x + r (rounded to bf16, written back to r), y = norm(r) * w.
template <int NV, bool RESID, int NT = 256, bool SC1 = false>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(bf16* __restrict__ out, int64_t out_stride,
                                                       const bf16* __restrict__ x, const float* __restrict__ xp,
                                                       int S, int64_t ps, int64_t x_stride,
                                                       bf16* __restrict__ resid, int64_t r_stride,
                                                       const bf16* __restrict__ w, int d, float eps) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  const int nvec = d >> 3;
  float v[NV][8];
  float ss = 0.f;
  // the weight loads go out with the row loads (not after the reduction: one HBM round trip instead of two)
  bf16x8 wv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) wv[i] = load_bf16x8(w + vi * 8);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      load_in8(v[i], x, xp, S, ps, row * x_stride + vi * 8);
      if constexpr (RESID) {
        const bf16x8 b = load_bf16x8(resid + row * r_stride + vi * 8);
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = (bf16)(v[i][j] + (float)b[j]);
          v[i][j] = (float)s[j];
        }
        if constexpr (SC1)
          store16_slab(reinterpret_cast<float*>(resid + row * r_stride + vi * 8), __builtin_bit_cast(f32x4, s));
        else
          store_bf16x8(resid + row * r_stride + vi * 8, s);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum<NT>(ss, red);
  const float r = rsqrtf(ss / (float)d + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[i][j] * r * (float)wv[i][j]);
      if constexpr (SC1)
        store16_slab(reinterpret_cast<float*>(out + row * out_stride + vi * 8), __builtin_bit_cast(f32x4, o));
      else
        store_bf16x8(out + row * out_stride + vi * 8, o);
    }
  }
}

// out[t, :] = silu(x[t, :F]) * x[t, F:]   (x: [T, 2F] row stride xs (bf16 or slabs), out: [T, F] contiguous)
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                        const float* __restrict__ xp, int S, int64_t ps,
                                                        int64_t xs, int F) {
  const int64_t row = blockIdx.y;
  const int nvec = F >> 3;
  for (int vi = blockIdx.x * 256 + threadIdx.x; vi < nvec; vi += gridDim.x * 256) {
    float g[8], u[8];
    load_in8(g, x, xp, S, ps, row * xs + vi * 8);
    load_in8(u, x, xp, S, ps, row * xs + F + vi * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)(g[j] / (1.0f + __expf(-g[j])) * u[j]);
    store_bf16x8(out + row * (int64_t)F + vi * 8, o);
  }
}

template <bool RESID>
static hipError_t launch_rmsnorm_t(bf16* out, int64_t os, const bf16* x, const float* xp, int S, int64_t ps,
                                   int64_t xs, bf16* r, int64_t rs, const bf16* w, int T, int d, float eps,
                                   hipStream_t st) {
  const int nvec = d / 8;
  const int nv = (nvec + 255) / 256;
  dim3 grid(T), block(256);
  if (T == 0) return hipSuccess;
  // outputs (normalised rows and the in-place residual) as 16-B sc1 stores — the lines leave this XCD's L2, so the
  // launch ends with none of them dirty (+2.1 % on the headline with RoPE's, profiles/r06/ab/); KAFKA_SC1_NORM=0 keeps
  // plain stores. Needs 16-B aligned rows. common.h "Store / load scopes"
  static const bool sc1 = [] {
    const char* e = getenv("KAFKA_SC1_NORM");
    return e == nullptr || e[0] != '0';
  }();
  if (nvec <= 512 && nvec > 256) {  // e.g. d = 4096: one 16-B vector per thread, twice the loads in flight per row
    if (sc1 && os % 8 == 0 && rs % 8 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
        (!RESID || reinterpret_cast<uintptr_t>(r) % 16 == 0))
      rmsnorm_kernel<1, RESID, 512, true><<<grid, 512, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps);
    else
      rmsnorm_kernel<1, RESID, 512><<<grid, 512, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps);
    return hipGetLastError();
  }
  switch (nv) {
    case 1: rmsnorm_kernel<1, RESID><<<grid, block, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps); break;
    case 2: rmsnorm_kernel<2, RESID><<<grid, block, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps); break;
    case 3:
    case 4: rmsnorm_kernel<4, RESID><<<grid, block, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps); break;
    default: rmsnorm_kernel<8, RESID><<<grid, block, 0, st>>>(out, os, x, xp, S, ps, xs, r, rs, w, d, eps); break;
  }
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_rmsnorm(bf16* out, int64_t os, const bf16* x, int64_t xs, const bf16* w, int T, int d,
                          float eps, hipStream_t st) {
  return launch_rmsnorm_t<false>(out, os, x, nullptr, 0, 0, xs, nullptr, 0, w, T, d, eps, st);
}

extern "C" hipError_t kafka_launch_fused_add_rmsnorm(bf16* out, int64_t os, const bf16* x, int64_t xs, bf16* resid, int64_t rs,
                                    const bf16* w, int T, int d, float eps, hipStream_t st) {
  return launch_rmsnorm_t<true>(out, os, x, nullptr, 0, 0, xs, resid, rs, w, T, d, eps, st);
}

// fused add + RMSNorm whose x input is S fp32 split-K slabs [S][T][d] (row stride d, slab stride ps)
extern "C" hipError_t kafka_launch_fused_add_rmsnorm_slab(bf16* out, int64_t os, const float* xp, int S, int64_t ps,
                                                         bf16* resid, int64_t rs, const bf16* w, int T, int d,
                                                         float eps, hipStream_t st) {
  return launch_rmsnorm_t<true>(out, os, nullptr, xp, S, ps, d, resid, rs, w, T, d, eps, st);
}

extern "C" hipError_t kafka_launch_silu_mul(bf16* out, const bf16* x, int64_t xs, int T, int F, hipStream_t st) {
  if (T == 0) return hipSuccess;
  const int nvec = F / 8;
  int gx = (nvec + 255) / 256;
  if (gx > 64) gx = 64;
  silu_mul_kernel<<<dim3(gx, T), dim3(256), 0, st>>>(out, x, nullptr, 0, 0, xs, F);
  return hipGetLastError();
}

// SwiGLU over S fp32 split-K slabs [S][T][2F]
extern "C" hipError_t kafka_launch_silu_mul_slab(bf16* out, const float* xp, int S, int64_t ps, int T, int F,
                                                hipStream_t st) {
  if (T == 0) return hipSuccess;
  const int nvec = F / 8;
  int gx = (nvec + 255) / 256;
  if (gx > 64) gx = 64;
  silu_mul_kernel<<<dim3(gx, T), dim3(256), 0, st>>>(out, nullptr, xp, S, ps, 2 * (int64_t)F, F);
  return hipGetLastError();
}

}  // namespace kafka
