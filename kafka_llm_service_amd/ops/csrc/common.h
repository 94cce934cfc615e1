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
// ---- Store / load scopes on gfx950 (8 XCDs, one L2 each; the MALL and HBM behind them are shared) ---------------
// What the kernels here rely on, and the evidence for it:
//   * plain store  -> the writer XCD's L2 (write-back). Visible to other XCDs in LATER kernels (the kernel-end release
//     writes dirty lines back, a kernel start drops other XCDs' stale copies). Within one launch it is visible to
//     workgroups of the SAME XCD only (they share the L2): the fused finishers in wstream_gemm.hip rely on this and
//     check it (hardware XCC_ID, flagged fallback).
//   * sc1 store (agent scope) -> written through to the coherent level. Readable in the same launch by sc1 loads
//     from any XCD once the writer's vmcnt reached 0 (decode ticket merge, GEMM finishers' flagged slabs; the ticket
//     itself is a relaxed agent-scope atomic issued after that wait — no release fence, which would write back the
//     writer's whole L2). In later kernels it is read with plain loads like any other data (decode-GEMM slabs, GEMM
//     bf16 outputs, cascade bf16 partials: tests/test_sc1_reuse_gpu.py rewrites each buffer after readers on every
//     XCD cached it).
//   * sc1 load -> not served from this XCD's (possibly stale) L2.
// Round 5 saw sc1 stores at other sites (RMSNorm / RoPE / tile outputs) leave wrong data (21 GPU tests, NaN in
// test_rope_kv_write). The cause was the STORE INSTRUCTION, not the scope: an inline-asm global_store_dwordx4 is
// opaque to hipcc's hazard recognizer, and on gfx9 a VMEM store of more than 8 bytes followed by a VALU write of its
// data VGPRs needs one wait state — hipcc inserts it for its own stores, never after an asm one, so a loop that
// reuses the data registers at once stored garbage. The same blindness holds on the way in: a VALU result read by
// the store too early (gfx950 forwarding hazards after dst_sel / op_sel writes such as the bf16 packs of a
// conversion, or after a transcendental) needs wait states hipcc does not insert in front of an asm consumer —
// round 6 measured garbage (1e30) in RMSNorm's in-place residual stored this way. Every asm store below therefore
// carries wait states on both sides — and FIVE after it, not the one hipcc itself puts behind a compiler-emitted
// dwordx4 store: with `s_nop 0` after the sc1 store the residual row (whose data VGPRs the next instruction, a
// v_pk_mul_f32 of the sum of squares, overwrites) still came out as garbage in 8 GPU tests; with `s_nop 4` all 60
// store-scope tests pass (profiles/r06/sc1/). The sites that passed with one wait state never rewrote the data
// registers right after the store.
__device__ __forceinline__ void store16_slab(float* p, f32x4 v) {
  asm volatile("s_nop 4\n\tglobal_store_dwordx4 %0, %1, off sc1\n\ts_nop 4" ::"v"(p), "v"(v) : "memory");
}

// raw buffer over 2 GiB from a wave-uniform base (gfx9 dword3: untyped 32-bit data); loads through it are compiler
// builtins, so hipcc's waitcnt and hazard passes see them (unlike inline asm)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// 16-B agent-coherent load (cache policy sc1)
__device__ __forceinline__ f32x4 load16_sc1(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16));
}
__device__ __forceinline__ f32x4 load16_plain(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 0));
}

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

// 2^x as the single v_exp_f32: exp2f() adds a denormal range fix-up (compare, select, add, ldexp: 6 VALU ops per
// value) that softmax does not need — its arguments are <= a small bound and results below 2^-126 may flush to 0.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
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
