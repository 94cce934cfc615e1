// Shared device helpers for the CDNA4 (gfx950) kernels of kafka_llm_service_amd.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * bf16 is the clang `__bf16` scalar type; casts f32->bf16 lower to v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
//   * bf16/f32 global traffic is vectorised to 16 B per lane (bf16x8 / f32x4).
//   * MFMA fragments follow the gfx950 maps of v_mfma_f32_32x32x16_bf16:
//       A: lane l holds A[row l&31][k = 8*(l>>5) + j], j = 0..7
//       B: lane l holds B[k = 8*(l>>5) + j][col l&31]
//       C/D: lane l, reg i -> row (i&3) + 8*(i>>2) + 4*(l>>5), col l&31
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define KAFKA_WAVE 64

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ bf16x8 load_bf16x8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void store_bf16x8(bf16* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }

// 8 consecutive fp32 values at element offset `off` of a bf16 tensor x, or — when xp is set — the sum of S fp32
// split-K slabs (slab stride ps elements, same element offset): the decode GEMM (wstream_gemm.hip) leaves its output
// as slabs and the consuming kernel combines them while loading.
template <int S>
__device__ __forceinline__ void sum_slabs8(f32x4& a, f32x4& b, const float* __restrict__ p, int64_t ps) {
  f32x4 va[S], vb[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {  // every slab load in flight before the first add (one HBM latency, not S)
    va[s] = *reinterpret_cast<const f32x4*>(p + s * ps);
    vb[s] = *reinterpret_cast<const f32x4*>(p + s * ps + 4);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    a += va[s];
    b += vb[s];
  }
}

// 8 consecutive inputs as fp32: from bf16 x, or summed over S fp32 split-K slabs xp (slab stride ps)
__device__ __forceinline__ void load_in8(float (&v)[8], const bf16* __restrict__ x, const float* __restrict__ xp,
                                         int S, int64_t ps, int64_t off) {
  if (xp) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
    const float* p = xp + off;
    switch (S) {  // uniform branch; each case fully unrolled
      case 1: sum_slabs8<1>(a, b, p, ps); break;
      case 2: sum_slabs8<2>(a, b, p, ps); break;
      case 4: sum_slabs8<4>(a, b, p, ps); break;
      case 8: sum_slabs8<8>(a, b, p, ps); break;
      default:
        for (int s = 0; s < S; ++s) {
          a += *reinterpret_cast<const f32x4*>(p + s * ps);
          b += *reinterpret_cast<const f32x4*>(p + s * ps + 4);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a[j];
      v[4 + j] = b[j];
    }
  } else {
    const bf16x8 a = load_bf16x8(x + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
  }
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---- device gates: early-launched consumers ---------------------------------------------------------------------
// A consumer kernel launched WITHOUT the AQL barrier bit (hipExtAnyOrderLaunch) is dispatched as soon as its
// predecessor's last workgroup has been dispatched, so it runs its producer-independent prologue (the weight stream
// of a projection, page tables, first K/V tiles) while the producer's tail still runs, then waits on a gate. Dispatch
// order within a queue guarantees every producer workgroup is resident before any consumer workgroup, so a waiting
// consumer can never starve its producer.
// A gate is 17 cache lines (no line is hot): lines 0..7 are arrival counters (a producer unit u arrives on line
// u & 7), line 8 the top counter (+ error word), lines 9..16 per-XCD "done" flags. The last arrival of a line bumps
// the top counter; the last of those raises all 8 flags. A consumer workgroup polls ONE flag (line 9 + its id & 7),
// so each line sees a handful of same-address accesses instead of every workgroup of both kernels.
// The producer's arrivals are agent-scope acq_rel RMWs after a workgroup barrier (release cumulativity carries the
// whole workgroup's writes), the flags release stores, the consumer's wait ends with an agent-scope acquire.
// Rule for callers (ops.GateSet / models): a gated consumer writes nothing to global memory before its wait, and it
// waits on the kernel launched immediately before it (gates then chain transitively, and the caching allocator's
// stream-order reuse stays safe).
constexpr int GATE_LINE = 16;                // int32 per 64-B line
constexpr int GATE_INTS = 17 * GATE_LINE;
struct Gates {
  int* wait = nullptr;   // wait until this gate's producer has fully arrived (nullptr: no wait)
  int expect = 0;        // (unused: the producer counts its own arrivals)
  int* sig = nullptr;    // arrive on this gate when the unit's outputs are written (nullptr: none)
  int* wait2 = nullptr;  // a second gate (decode attention: the cascade partials, before the merge)
  int expect2 = 0;
  int mode = 0;          // diagnostics: bit 0 (KAFKA_GATE_MODE=1/3) = no release / acquire (timing only: unordered
                         // reads); bits 4.. (KAFKA_GATE_SLEEP) = poll back-off level
};

__device__ __forceinline__ int gate_block_id() {
  return (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
}

// ONE thread, after a __syncthreads() that follows every global write of arrival unit `unit` (0 <= unit < total; a
// launch arrives `total` times, each unit once)
__device__ __forceinline__ void gate_arrive(int* g, int unit, int total, int mode = 0) {
  if (g == nullptr) return;
  const int s = unit & 7;
  const int n_s = total / 8 + (s < total % 8 ? 1 : 0);
  const int lines = total < 8 ? total : 8;
  const bool rlx = mode & 1;
  const int old = rlx ? __hip_atomic_fetch_add(g + s * GATE_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : __hip_atomic_fetch_add(g + s * GATE_LINE, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old != n_s - 1) return;
  const int top = rlx ? __hip_atomic_fetch_add(g + 8 * GATE_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : __hip_atomic_fetch_add(g + 8 * GATE_LINE, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (top != lines - 1) return;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    if (rlx)
      __hip_atomic_store(g + (9 + x) * GATE_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_store(g + (9 + x) * GATE_LINE, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// every thread of the workgroup (workgroup-uniform arguments); bounded: after 2 s the error word is raised and the
// wait gives up (the host fails the step instead of hanging the GPU)
__device__ __forceinline__ void gate_wait(int* g, int mode = 0) {
  if (g == nullptr) return;
  if (threadIdx.x == 0) {
    const int* flag = g + (9 + (gate_block_id() & 7)) * GATE_LINE;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        __hip_atomic_store(g + 8 * GATE_LINE + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      switch (mode >> 4) {  // uniform
        case 0: __builtin_amdgcn_s_sleep(1); break;
        case 1: __builtin_amdgcn_s_sleep(8); break;
        default: __builtin_amdgcn_s_sleep(32); break;
      }
    }
  }
  __syncthreads();
  if (!(mode & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Write-through hand-off (the cascade -> suffix-decode overlap): the producer writes its outputs with agent-coherent
// stores (sc1: through to memory, not parked dirty in its XCD's L2), waits for them (vmcnt), and arrives RELAXED; the
// consumer waits RELAXED and reads them with agent-coherent loads (sc1: not served from its XCD's possibly stale L2)
// — neither side needs the L2-wide write-back / invalidate of a release / acquire fence.
__device__ __forceinline__ void st_wt16(void* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4 ld_wt16(const void* p) {  // the caller waits (s_waitcnt vmcnt) before using it
  f32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ f32x2 ld_wt8(const void* p) {
  f32x2 r;
  asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// after every write-through store of the workgroup: all of them complete, then ONE relaxed arrival
__device__ __forceinline__ void gate_arrive_wt(int* g, int unit, int total) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) gate_arrive(g, unit, total, 1);
}

// Launch `kernel`; `early`: without the AQL barrier bit (the kernel waits on a gate before reading its inputs)
template <typename F, typename... Args>
inline void launch_maybe_early(F kernel, dim3 grid, dim3 block, hipStream_t st, bool early, Args... args) {
  static const bool ordered = [] {  // diagnostics: KAFKA_GATE_MODE=2 keeps the barrier bit (gates without overlap)
    const char* e = getenv("KAFKA_GATE_MODE");
    return e && (e[0] == '2' || e[0] == '3');
  }();
  if (early && !ordered)
    hipExtLaunchKernelGGL(kernel, grid, block, 0, st, nullptr, nullptr, hipExtAnyOrderLaunch, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
}

// Counter-based RNG (splitmix64 finaliser): deterministic given (seed, stream, index).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Uniform in (0, 1].
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t stream, uint64_t idx) {
  uint64_t r = mix64(seed ^ mix64(stream * 0x632BE59BD9B4E019ull + idx));
  return ((float)(r >> 40) + 1.0f) * (1.0f / 16777216.0f);
}
