// Token sampler for gfx950: greedy / temperature / top-k / top-p in one kernel, one 1024-thread workgroup per row.
//
//   temperature == 0       -> argmax (first maximal index)
//   otherwise              -> Gumbel-max over x = logits / T with counter-based uniforms (seed, step, index):
//                             an exact sample of softmax(x) in one pass, no sort, no normalisation pass.
//   top_k > 0 or top_p < 1 -> rejection on a pivot: draw c from the tokens strictly above the pivot, accept iff
//                             (#tokens with x > x_c) < k and (mass of tokens with x > x_c) < p; otherwise raise the
//                             pivot to x_c and redraw. Accepted draws are exactly distributed as the renormalised
//                             top-k/top-p distribution; rounds are bounded (fallback: argmax).
// All reads are 16-byte vectors; every pass is one streaming read of the row (bf16 or fp32 logits).
// Greedy and plain-temperature rows (no top-k / top-p) are split over `nsplit` workgroups (grid (B, nsplit)): each
// takes a slice of the vocabulary, publishes its (value, index) winner, and the last of a row's workgroups to take
// its ticket reduces them — the noise of index i is the same in every split, so the token is the one-workgroup
// result. A 64-row decode batch then runs 512 workgroups instead of 64 (128k-entry rows: 62 -> ~10 us).
#include "common.h"

namespace kafka {

template <typename T>
struct Vec8;
template <>
struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[8]) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
  }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
};

constexpr int SNT = 1024;
constexpr int SAMPLE_MAX_ROWS = 65536;  // ws: tickets [SAMPLE_MAX_ROWS] | partials [B][nsplit][2]

struct ArgMax {
  float v;
  int i;
};

__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ __forceinline__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = better(a, b);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = a.v;
    si[w] = a.i;
  }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  for (int k = 1; k < SNT / 64; ++k) r = better(r, ArgMax{sv[k], si[k]});
  __syncthreads();
  return r;
}

__device__ __forceinline__ float gumbel(uint64_t seed, uint64_t stream, uint64_t idx) {
  const float u = uniform01(seed, stream, idx);  // (0, 1]
  return -__logf(-__logf(fminf(u, 0.99999994f)));
}

// Plain-temperature rows: the per-element noise from a per-row 64-bit key (two splitmix64 rounds, once per thread)
// and a 32-bit integer hash of the index (two lowbias32 rounds: 4 v_mul_lo_u32 instead of the ~16 32-bit multiplies
// two 64-bit splitmix rounds cost per element) — the noise stream is still a pure function of (seed, step, index),
// so every split of a row draws the same noise for an index and the token is the one-workgroup result.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float gumbel_fast(uint64_t key, uint32_t idx) {
  const uint32_t h = lowbias32(lowbias32(idx + (uint32_t)key) ^ (uint32_t)(key >> 32));
  const float u = ((float)(h >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  return -__logf(-__logf(fminf(u, 0.99999994f)));
}

template <typename T>
__global__ __launch_bounds__(SNT) void sample_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                      const float* __restrict__ temperature,
                                                      const float* __restrict__ top_p, const int* __restrict__ top_k,
                                                      const int64_t* __restrict__ seeds, const int64_t* __restrict__ step_ptr,
                                                      int64_t* __restrict__ out_tokens, int max_rounds,
                                                      int* __restrict__ ws) {
  __shared__ float sv[SNT / 64];
  __shared__ int si[SNT / 64];
  __shared__ float red[SNT / 64];
  const int row = blockIdx.x, sp = blockIdx.y, nsplit = gridDim.y;
  const T* x = logits + (int64_t)row * stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const int nvec = V >> 3;
  const int tail0 = nvec << 3;
  const float tp = top_p ? top_p[row] : 1.f;
  const int tk = top_k ? top_k[row] : 0;
  const bool filtered = temp > 0.f && ((tp < 1.f) || (tk > 0 && tk < V));

  if (!filtered) {
    // argmax of x (greedy) or of x / T + Gumbel noise over this workgroup's slice of the row
    const bool greedy = !(temp > 0.f);
    const float inv_t = greedy ? 1.f : 1.f / temp;
    const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0x1234ull;
    const uint64_t stream = (uint64_t)(step_ptr ? step_ptr[0] : 0) << 8;  // round 0 of the filtered path
    const uint64_t key = mix64(seed ^ mix64(stream * 0x632BE59BD9B4E019ull));
    const int per = (nvec + nsplit - 1) / nsplit;
    const int v0 = sp * per, v1 = min(nvec, v0 + per);
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int vi = v0 + threadIdx.x; vi < v1; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = v[j] * inv_t;
        a = better(a, ArgMax{greedy ? xv : xv + gumbel_fast(key, vi * 8 + j), vi * 8 + j});
      }
    }
    if (sp == nsplit - 1)
      for (int i = tail0 + threadIdx.x; i < V; i += SNT) {
        const float xv = (float)x[i] * inv_t;
        a = better(a, ArgMax{greedy ? xv : xv + gumbel_fast(key, i), i});
      }
    a = block_argmax(a, sv, si);
    if (threadIdx.x != 0) return;
    if (nsplit == 1) {
      out_tokens[row] = a.i < V ? a.i : 0;  // an all-NaN row (a broken upstream kernel) must not yield an id >= V
      return;
    }
    // ws: tickets (zero, re-armed here) | [B][nsplit][2] (value bits, index)
    int* tk_row = ws + row;
    int* part = ws + SAMPLE_MAX_ROWS + ((int64_t)row * nsplit + sp) * 2;
    __hip_atomic_store(part, __float_as_int(a.v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + 1, a.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int t = __hip_atomic_fetch_add(tk_row, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t != nsplit - 1) return;
    __hip_atomic_store(tk_row, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int* p0 = ws + SAMPLE_MAX_ROWS + (int64_t)row * nsplit * 2;
    ArgMax r{-INFINITY, 0x7fffffff};
    for (int k = 0; k < nsplit; ++k)
      r = better(r, ArgMax{__int_as_float(__hip_atomic_load(p0 + 2 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                           __hip_atomic_load(p0 + 2 * k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)});
    out_tokens[row] = r.i < V ? r.i : 0;
    return;
  }
  if (sp != 0) return;  // top-k / top-p rows: one workgroup runs the whole-row rejection sampler
  const float inv_t = 1.f / temp;
  const int64_t step = step_ptr ? step_ptr[0] : 0;
  const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0x1234ull;

  // pass 1: max of x (needed for the mass test only)
  float mx = -INFINITY;
  float z = 0.f;
  if (filtered) {
    for (int vi = threadIdx.x; vi < nvec; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j] * inv_t);
    }
    for (int i = tail0 + threadIdx.x; i < V; i += SNT) mx = fmaxf(mx, (float)x[i] * inv_t);
    mx = block_max<SNT>(mx, red);
    for (int vi = threadIdx.x; vi < nvec; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) z += __expf(v[j] * inv_t - mx);
    }
    for (int i = tail0 + threadIdx.x; i < V; i += SNT) z += __expf((float)x[i] * inv_t - mx);
    z = block_sum<SNT>(z, red);
  }

  float pivot = -INFINITY;
  int result = -1;
  for (int round = 0; round < max_rounds; ++round) {
    const uint64_t stream = ((uint64_t)step << 8) ^ (uint64_t)round;
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int vi = threadIdx.x; vi < nvec; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = v[j] * inv_t;
        if (xv > pivot) a = better(a, ArgMax{xv + gumbel(seed, stream, vi * 8 + j), vi * 8 + j});
      }
    }
    for (int i = tail0 + threadIdx.x; i < V; i += SNT) {
      const float xv = (float)x[i] * inv_t;
      if (xv > pivot) a = better(a, ArgMax{xv + gumbel(seed, stream, i), i});
    }
    a = block_argmax(a, sv, si);
    if (a.i == 0x7fffffff) break;
    if (!filtered) {
      result = a.i;
      break;
    }
    const float xc = (float)x[a.i] * inv_t;
    float mass = 0.f, cnt = 0.f;
    for (int vi = threadIdx.x; vi < nvec; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = v[j] * inv_t;
        if (xv > xc) {
          mass += __expf(xv - mx);
          cnt += 1.f;
        }
      }
    }
    for (int i = tail0 + threadIdx.x; i < V; i += SNT) {
      const float xv = (float)x[i] * inv_t;
      if (xv > xc) {
        mass += __expf(xv - mx);
        cnt += 1.f;
      }
    }
    mass = block_sum<SNT>(mass, red) / z;
    cnt = block_sum<SNT>(cnt, red);
    const bool ok_p = mass < tp;
    const bool ok_k = (tk <= 0) || (cnt < (float)tk);
    if (ok_p && ok_k) {
      result = a.i;
      break;
    }
    pivot = xc;
  }
  if (result < 0) {  // fallback: argmax
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int vi = threadIdx.x; vi < nvec; vi += SNT) {
      float v[8];
      Vec8<T>::load(x + vi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) a = better(a, ArgMax{v[j], vi * 8 + j});
    }
    for (int i = tail0 + threadIdx.x; i < V; i += SNT) a = better(a, ArgMax{(float)x[i], i});
    a = block_argmax(a, sv, si);
    result = a.i;
  }
  if (threadIdx.x == 0) out_tokens[row] = result >= 0 && result < V ? result : 0;
}

// ws (optional): int32 workspace of >= SAMPLE_MAX_ROWS + 2 * B * nsplit entries whose first SAMPLE_MAX_ROWS are zero
// (tickets, re-armed by the kernel); without it every row is one workgroup.
extern "C" hipError_t kafka_launch_sample(const void* logits, bool is_bf16, int64_t stride, int B, int V, const float* temperature,
                         const float* top_p, const int* top_k, const int64_t* seeds, const int64_t* step,
                         int64_t* out_tokens, int* ws, int nsplit, hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (ws == nullptr || nsplit < 1) nsplit = 1;
  if (B > SAMPLE_MAX_ROWS || nsplit > 64) return hipErrorInvalidValue;
  const dim3 grid(B, nsplit);
  if (is_bf16)
    sample_kernel<bf16><<<grid, SNT, 0, st>>>(reinterpret_cast<const bf16*>(logits), stride, V, temperature, top_p,
                                              top_k, seeds, step, out_tokens, 32, ws);
  else
    sample_kernel<float><<<grid, SNT, 0, st>>>(reinterpret_cast<const float*>(logits), stride, V, temperature, top_p,
                                               top_k, seeds, step, out_tokens, 32, ws);
  return hipGetLastError();
}

}  // namespace kafka
