// Rotary embedding on Q/K fused with the paged KV-cache write (gfx950).
// Input is the fused QKV projection output [T, (Hq + 2*Hkv) * D] — bf16, or S fp32 split-K slabs of the decode
// GEMM (wstream_gemm.hip) summed while loading. One workgroup per token, one thread per 8-element unit:
//   * Q heads: rotate-half RoPE -> q_out[T, Hq, D]
//   * K heads: rotate-half RoPE -> k_cache page  [num_blocks, Hkv, 16, D]   as D/8 chunk planes [D/8][16 keys][8]:
//              element (key o, d) at ((d >> 3) * 16 + o) * 8 + (d & 7). The MFMA A fragment of a 16-key page for
//              k-step kk (lanes: 16 keys x 2 halves of 8 d) is then ONE contiguous 512-B run (chunks 2kk, 2kk+1),
//              where a key-major page gives 16 rows x 32 B per wave-instruction.
//   * V heads: copy            -> v_cache page  [num_blocks, Hkv, D, 16]   (d-major: V^T per page)
// The V^T page stores key offset o at position swap_bits_2_3(o). With that permutation the PV step of the
// attention kernels (O^T = V^T . P, P taken straight from the S^T accumulator registers of
// v_mfma_f32_32x32x16_bf16) reads each lane's 8-key A-fragment as ONE contiguous 16-byte load:
// accumulator element j of lane-half h holds key 8*(j>>2) + 4*h + (j&3) of a 16-key page, which lands at
// page position 8*h + j.
// cos/sin come from a host-built table [max_pos, D] (cos in [0, D/2), sin in [D/2, D)) so the kernel does no
// transcendental math (llama3 / linear / none scaling is folded into the table on the host).
//
// fp8 KV cache (kv_dtype="fp8", OCP e4m3, D = 128): rope_kv_fp8_kernel quantizes each (token, kv head) vector of K
// and of V with its own power-of-two scale 2^e (e = exponent of amax / 448, so the largest element lands in
// [224, 448]; a power of two loses no mantissa and dequantizes with an exponent add). Per (block, kv head):
//   K page  KPAGE8 = 2080 B: 2048 B e4m3 data in 16-B units [8 planes p = 2j + h][16 keys o]; unit (p, o) holds
//           d = 32j + 8h + {0..7} followed by d = 32j + 16 + 8h + {0..7} — the bf16 MFMA A-fragments of k-steps 2j
//           and 2j + 1 of lane (key o, half h), i.e. ONE 16-B load per two k-steps; then int8 exponents: K of key
//           o at byte 2048 + o, V of key o at byte 2064 + vt_pos(o) (the order in which the PV step's P registers
//           hold the keys, so a lane's 8 V exponents of a page are one 8-B load).
//   V page  2048 B: V^T [D][16] e4m3, key o at position vt_pos(o) (as the bf16 layout).
#include <cstdlib>

#include "common.h"

namespace kafka {

__device__ __forceinline__ int vt_pos(int o) { return (o & ~15) | (o & 3) | ((o & 4) << 1) | ((o & 8) >> 1); }

template <int D, bool SC1 = false>
__global__ __launch_bounds__(1024) void rope_kv_kernel(const bf16* __restrict__ qkv, const float* __restrict__ qp,
                                                       int S, int64_t ps, int64_t qkv_stride,
                                                       const int64_t* __restrict__ positions,
                                                       const float* __restrict__ cos_sin,
                                                       bf16* __restrict__ q_out, int64_t q_stride,
                                                       bf16* __restrict__ k_cache, bf16* __restrict__ v_cache,
                                                       const int64_t* __restrict__ slot_mapping, int Hq, int Hkv,
                                                       int block_size) {
  constexpr int HALF = D / 2;
  constexpr int RU = HALF / 8;  // rope units (8 rotation pairs each) per head
  constexpr int VU = D / 8;     // v copy units (8 elements) per head
  const int64_t t = blockIdx.x;
  const int64_t pos = positions[t];
  const int64_t slot = slot_mapping ? slot_mapping[t] : -1;
  const int64_t row = t * qkv_stride;
  const float* cs = cos_sin + pos * D;
  const int n_rope = (Hq + Hkv) * RU;
  const int n_total = n_rope + Hkv * VU;
  const int64_t blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? (int)(slot % block_size) : 0;
  for (int u = blockIdx.y * blockDim.x + threadIdx.x; u < n_total; u += gridDim.y * blockDim.x) {
    if (u < n_rope) {
      const int head = u / RU;
      const int c = (u % RU) * 8;
      float x1[8], x2[8];
      load_in8(x1, qkv, qp, S, ps, row + head * D + c);
      load_in8(x2, qkv, qp, S, ps, row + head * D + HALF + c);
      f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + c);
      f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + c + 4);
      f32x4 s0 = *reinterpret_cast<const f32x4*>(cs + HALF + c);
      f32x4 s1 = *reinterpret_cast<const f32x4*>(cs + HALF + c + 4);
      float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      bf16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = x1[j], b = x2[j];
        o1[j] = (bf16)(a * cv[j] - b * sv[j]);
        o2[j] = (bf16)(b * cv[j] + a * sv[j]);
      }
      auto st16 = [](bf16* p, bf16x8 v) {
        if constexpr (SC1)
          store16_slab(reinterpret_cast<float*>(p), __builtin_bit_cast(f32x4, v));
        else
          store_bf16x8(p, v);
      };
      if (head < Hq) {
        bf16* dst = q_out + t * q_stride + head * D;
        st16(dst + c, o1);
        st16(dst + HALF + c, o2);
      } else if (slot >= 0) {
        const int kh = head - Hq;
        bf16* dst = k_cache + (blk * Hkv + kh) * (int64_t)block_size * D + off * 8;
        st16(dst + (c >> 3) * block_size * 8, o1);
        st16(dst + ((HALF + c) >> 3) * block_size * 8, o2);
      }
    } else if (slot >= 0) {
      const int v = u - n_rope;
      const int vh = v / VU;
      const int c = (v % VU) * 8;
      float x[8];
      load_in8(x, qkv, qp, S, ps, row + (Hq + Hkv + vh) * D + c);
      bf16* dst = v_cache + (blk * Hkv + vh) * (int64_t)D * block_size + vt_pos(off);
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[(int64_t)(c + j) * block_size] = (bf16)x[j];
    }
  }
}

constexpr int KPAGE8 = 16 * 128 + 32;
constexpr int MAX_HKV8 = 64;

// e such that amax * 2^-e <= 448 (frexp of amax / 448); 0 for an all-zero vector
__device__ __forceinline__ int fp8_exponent(float amax) {
  int e = 0;
  frexpf(amax / 448.f, &e);
  return amax > 0.f ? e : 0;
}

// 8 fp32 (already scaled) -> 8 e4m3 bytes, RNE, saturated to +-448
__device__ __forceinline__ uint2 pack_fp8x8(const float (&x)[8]) {
  int w[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_fmed3f(x[4 * i + j], 448.f, -448.f);
    int v = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    w[i] = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], v, true);
  }
  return make_uint2((unsigned)w[0], (unsigned)w[1]);
}

// One workgroup per token, one pass (host-checked: every unit has its own thread). K/V amax per (token, head) is
// reduced through LDS (atomicMax on the float bits: non-negative floats order like their bit patterns).
__global__ __launch_bounds__(1024) void rope_kv_fp8_kernel(const bf16* __restrict__ qkv, const float* __restrict__ qp,
                                                           int S, int64_t ps, int64_t qkv_stride,
                                                           const int64_t* __restrict__ positions,
                                                           const float* __restrict__ cos_sin,
                                                           bf16* __restrict__ q_out, int64_t q_stride,
                                                           uint8_t* __restrict__ k_cache, uint8_t* __restrict__ v_cache,
                                                           const int64_t* __restrict__ slot_mapping, int Hq, int Hkv) {
  constexpr int D = 128, HALF = 64, RU = HALF / 8, VU = D / 8;
  __shared__ unsigned s_amax[2 * MAX_HKV8];
  const int64_t t = blockIdx.x;
  const int64_t pos = positions[t];
  const int64_t slot = slot_mapping ? slot_mapping[t] : -1;
  const int64_t row = t * qkv_stride;
  const float* cs = cos_sin + pos * D;
  const int n_rope = (Hq + Hkv) * RU;
  const int n_total = n_rope + Hkv * VU;
  const int64_t blk = slot >= 0 ? slot / 16 : 0;
  const int off = slot >= 0 ? (int)(slot % 16) : 0;
  const int u = threadIdx.x;
  for (int i = u; i < 2 * Hkv; i += blockDim.x) s_amax[i] = 0u;
  __syncthreads();
  float y1[8], y2[8];
  int kind = 0, head = 0, c = 0;  // kind 1: K unit (y1 = d c.., y2 = d 64 + c..), 2: V unit (y1 = d c..)
  float amax = 0.f;
  if (u < n_rope) {
    head = u / RU;
    c = (u % RU) * 8;
    float x1[8], x2[8];
    load_in8(x1, qkv, qp, S, ps, row + head * D + c);
    load_in8(x2, qkv, qp, S, ps, row + head * D + HALF + c);
    f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + c);
    f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + c + 4);
    f32x4 s0 = *reinterpret_cast<const f32x4*>(cs + HALF + c);
    f32x4 s1 = *reinterpret_cast<const f32x4*>(cs + HALF + c + 4);
    float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = x1[j], b = x2[j];
      y1[j] = a * cv[j] - b * sv[j];
      y2[j] = b * cv[j] + a * sv[j];
    }
    if (head < Hq) {
      bf16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = (bf16)y1[j];
        o2[j] = (bf16)y2[j];
      }
      bf16* dst = q_out + t * q_stride + head * D;
      store_bf16x8(dst + c, o1);
      store_bf16x8(dst + HALF + c, o2);
    } else if (slot >= 0) {
      kind = 1;
      head -= Hq;
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fmaxf(fabsf(y1[j]), fabsf(y2[j])));
      atomicMax(&s_amax[head], __float_as_uint(amax));
    }
  } else if (u < n_total && slot >= 0) {
    kind = 2;
    const int v = u - n_rope;
    head = v / VU;
    c = (v % VU) * 8;
    load_in8(y1, qkv, qp, S, ps, row + (Hq + Hkv + head) * D + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(y1[j]));
    atomicMax(&s_amax[Hkv + head], __float_as_uint(amax));
  }
  __syncthreads();
  if (kind == 0) return;
  uint8_t* kpage = k_cache + (blk * Hkv + head) * (int64_t)KPAGE8;
  const int e = fp8_exponent(__uint_as_float(s_amax[(kind == 2 ? Hkv : 0) + head]));
  const float inv = ldexpf(1.f, -e);
  if (kind == 1) {
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      float z[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = (part ? y2[j] : y1[j]) * inv;
      const int q8 = ((part ? HALF : 0) + c) >> 3;  // 8-element chunk of d
      const int p = 2 * (q8 >> 2) + (q8 & 1), second = (q8 >> 1) & 1;
      *reinterpret_cast<uint2*>(kpage + (p * 16 + off) * 16 + 8 * second) = pack_fp8x8(z);
    }
    if (c == 0) kpage[2048 + off] = (uint8_t)(int8_t)e;
  } else {
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = y1[j] * inv;
    const uint2 w = pack_fp8x8(z);
    uint8_t* dst = v_cache + (blk * Hkv + head) * (int64_t)(D * 16) + vt_pos(off);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[(c + j) * 16] = (uint8_t)(((j < 4 ? w.x : w.y) >> (8 * (j & 3))) & 0xff);
    if (c == 0) kpage[2064 + vt_pos(off)] = (uint8_t)(int8_t)e;
  }
}

extern "C" hipError_t kafka_launch_rope_kv_fp8(const bf16* qkv, const float* qp, int S, int64_t ps,
                                              int64_t qkv_stride, const int64_t* positions, const float* cos_sin,
                                              bf16* q_out, int64_t q_stride, uint8_t* k_cache, uint8_t* v_cache,
                                              const int64_t* slot_mapping, int T, int Hq, int Hkv, int D,
                                              hipStream_t st) {
  if (T == 0) return hipSuccess;
  const int units = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  if (D != 128 || Hkv > MAX_HKV8 || units > 1024) return hipErrorInvalidValue;
  const int nt = ((units + 63) / 64) * 64;
  rope_kv_fp8_kernel<<<T, nt, 0, st>>>(qkv, qp, S, ps, qkv_stride, positions, cos_sin, q_out, q_stride, k_cache,
                                       v_cache, slot_mapping, Hq, Hkv);
  return hipGetLastError();
}

// qp != nullptr: the input is S fp32 slabs [S][T][(Hq + 2 Hkv) D] (slab stride ps) instead of bf16 qkv
extern "C" hipError_t kafka_launch_rope_kv(const bf16* qkv, const float* qp, int S, int64_t ps, int64_t qkv_stride,
                                          const int64_t* positions, const float* cos_sin, bf16* q_out,
                                          int64_t q_stride, bf16* k_cache, bf16* v_cache,
                                          const int64_t* slot_mapping, int T, int Hq, int Hkv, int D,
                                          int block_size, hipStream_t st) {
  if (T == 0) return hipSuccess;
  if (D != 128 && D != 64) return hipErrorInvalidValue;
  // one thread per work unit (8 rotation pairs of a Q/K head, or 8 V elements), so a token's whole row is one
  // round of loads instead of a strided loop paying the HBM latency twice (448 units for Llama-3-8B), spread over
  // workgroups of 64 threads: at decode T is the batch (64), and one workgroup per token leaves 3/4 of the CUs idle
  // while each busy CU pulls the token's S slabs (~100 KB) through its own L2 port (+0.5 % tok/s over one workgroup
  // per token, profiles/r02/rope_wg_ab.jsonl)
  const int units = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  const int nt = 64, ny = (units + nt - 1) / nt;
  const dim3 grid(T, ny);
  // q and K rows as 16-B sc1 stores (KAFKA_SC1_ROPE=0: plain; with the RMSNorm outputs +2.1 %, common.h)
  static const bool sc1 = [] {
    const char* e = getenv("KAFKA_SC1_ROPE");
    return e == nullptr || e[0] != '0';
  }();
  if (D == 128 && sc1 && q_stride % 8 == 0)
    rope_kv_kernel<128, true><<<grid, nt, 0, st>>>(qkv, qp, S, ps, qkv_stride, positions, cos_sin, q_out, q_stride,
                                                k_cache, v_cache, slot_mapping, Hq, Hkv, block_size);
  else if (D == 128)
    rope_kv_kernel<128><<<grid, nt, 0, st>>>(qkv, qp, S, ps, qkv_stride, positions, cos_sin, q_out, q_stride, k_cache,
                                          v_cache, slot_mapping, Hq, Hkv, block_size);
  else
    rope_kv_kernel<64><<<grid, nt, 0, st>>>(qkv, qp, S, ps, qkv_stride, positions, cos_sin, q_out, q_stride, k_cache,
                                         v_cache, slot_mapping, Hq, Hkv, block_size);
  return hipGetLastError();
}

}  // namespace kafka
