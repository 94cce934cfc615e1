// One-shot all-reduce over xGMI for decode-sized TP messages (SURVEY.md §2.6 `custom_allreduce_oneshot`, §5.8).
//
// Every rank owns ONE fine-grained, uncached device allocation, IPC-mapped into every peer of its TP group:
//     [ flags: MAX_RANKS x MAX_BLOCKS int32 | err int32 | epochs: MAX_BLOCKS int32 | pad to 8 KB | data: 2 halves ]
// Block b of every rank owns the same slice of the message and keeps its own call counter (epoch) in device memory
// (epochs[b] of its rank's allocation: read + advanced by the block itself, so a captured hipGraph replays with
// fresh epochs — nothing host-side is baked into the launch). A call with epoch e uses data half (e & 1):
//   1. stage its slice of the input into its OWN data half: the input is bf16, or fp32 split-K slabs of the decode
//      GEMM (summed while loading, rounded to bf16 once: half the xGMI bytes of fp32),
//   2. publish: every staging wave waits for its stores, the block barriers, one wave releases system-wide and
//      stores e into flags[my_rank][b] of EVERY peer,
//   3. wait until flags[p][b] >= e for every peer p in its own flag block (relaxed polls, one system acquire;
//      bounded: after ~2 s it sets err and proceeds, so a lost peer can never hang the GPU; once err is set every
//      later call skips its waits — garbage fast instead of 2 s per call — and the engine, which copies err back
//      with every step's sampled ids (car_error_async), fails the replica: 503 + respawn, never silent tokens),
//   4. read slice b from all peers' data halves at once (each MI355X reads its 7 peers over its 7 xGMI links in
//      parallel: one hop, vs a ring's 2(N-1) hops) and sum in fp32 in a fixed rank order (bit-identical on every
//      rank). Plain mode writes the bf16 sum; the fused mode (slices = whole rows) also adds the residual (updated in
//      place, bf16) and writes rmsnorm(residual) * w — the all-reduce, the residual add and the next layer's
//      RMSNorm in ONE launch (replaces slab-reduce + all-reduce + fused_add_rmsnorm).
// Double-buffering by epoch parity makes a trailing barrier unnecessary: a peer can only still be reading half
// (e & 1) during call e-2, and this block started call e only after every peer's block b had entered call e-1,
// i.e. after every peer's launch of call e-2 had completed (stream order). Epochs advance together on all blocks
// (every block takes part in every call, with or without rows), so e is the same for the whole call.
// Loads of peer data use sc0 sc1 (system-coherent) so no stale line of an older call is returned.
//
// The same buffers, epochs and exchange carry the expert-parallel all-to-all and all-gather of the MoE layers
// (a2a_pull_kernel): every rank stages its whole send image (per-destination parts of `bpd` bytes, or ONE part for
// every destination in all-gather mode) into its data half, publishes, and then pulls from each peer the part
// addressed to it. Block b stages image chunks [c0, c1) and pulls only chunks of that same range from the peers —
// exactly what the peers' block b staged before releasing flag (p, b) — so the per-block flags order every read.
#include "common.h"

namespace kafka {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 128;
constexpr int AR_ERR_OFF = AR_MAX_RANKS * AR_MAX_BLOCKS * 4;  // 4096
constexpr int AR_EPOCH_OFF = AR_ERR_OFF + 256;
// collective timing ring (SURVEY §5.5 "all-reduce time"): block 0 of every call stamps the 100 MHz constant clock at
// entry and exit into slot (epoch & 127) — [start, end] uint64 pairs, read by the host on /metrics requests only
constexpr int AR_TIME_OFF = 5120;
constexpr int AR_TIME_SLOTS = 128;
constexpr int AR_HEADER = 8192;
static_assert(AR_EPOCH_OFF + AR_MAX_BLOCKS * 4 <= AR_TIME_OFF && AR_TIME_OFF + AR_TIME_SLOTS * 16 <= AR_HEADER, "hdr");

struct ARPtrs {
  char* base[AR_MAX_RANKS];  // every rank's allocation, mapped into this process (base[rank] = own)
};

typedef int ar_i32x4 __attribute__((ext_vector_type(4)));

// system-coherent 16-B load, issued without a wait (the caller waits once for all peers' loads)
__device__ __forceinline__ ar_i32x4 load_sys16_nowait(const bf16* p) {
  ar_i32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// This block's epoch for this call: its device counter + 1 (advanced here; one block per counter, stream-ordered
// between launches). `s_e` is the block's broadcast slot in LDS.
__device__ __forceinline__ int ar_epoch(const ARPtrs& ptrs, int rank, int* s_e) {
  if (threadIdx.x == 0) {
    int* ep = reinterpret_cast<int*>(ptrs.base[rank] + AR_EPOCH_OFF) + blockIdx.x;
    // vector memory ops (atomic forms) on purpose: never the scalar cache for this read-modify-write
    const int e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(ep, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_e = e;
    if (blockIdx.x == 0) {
      uint64_t* ts = reinterpret_cast<uint64_t*>(ptrs.base[rank] + AR_TIME_OFF) + (e & (AR_TIME_SLOTS - 1)) * 2;
      __hip_atomic_store(ts, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *s_e;
}

// Exit stamp of the call's timing slot (block 0, thread 0; vector store like the epoch update)
__device__ __forceinline__ void ar_stamp_end(const ARPtrs& ptrs, int rank, int e) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t* ts = reinterpret_cast<uint64_t*>(ptrs.base[rank] + AR_TIME_OFF) + (e & (AR_TIME_SLOTS - 1)) * 2 + 1;
    __hip_atomic_store(ts, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Steps 2 + 3: publish this block's staged slice to every peer and wait for theirs.
template <int NR>
__device__ __forceinline__ void ar_exchange(const ARPtrs& ptrs, int rank, int e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's staging stores have completed
  __syncthreads();                                    // ... and every other wave's
  if (threadIdx.x < 64) {
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x < NR) {
      const int p = threadIdx.x;
      int* pf = reinterpret_cast<int*>(ptrs.base[p]) + rank * AR_MAX_BLOCKS + blockIdx.x;
      __hip_atomic_store(pf, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      int* my = reinterpret_cast<int*>(ptrs.base[rank]) + p * AR_MAX_BLOCKS + blockIdx.x;
      int* err = reinterpret_cast<int*>(ptrs.base[rank] + AR_ERR_OFF);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
      while (__hip_atomic_load(my, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
        // a group that already lost a peer does not wait again (the engine is failing the replica)
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s: report instead of hanging the queue
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
  }
  __syncthreads();
}

// Sum of chunk c (8 bf16) over all ranks' data halves, in rank order.
template <int NR>
__device__ __forceinline__ void ar_sum8(const ARPtrs& ptrs, int64_t half, int64_t c, float (&v)[8]) {
  ar_i32x4 raw[NR];
#pragma unroll
  for (int p = 0; p < NR; ++p)  // all peers' loads in flight at once (one per xGMI link)
    raw[p] = load_sys16_nowait(reinterpret_cast<const bf16*>(ptrs.base[p] + AR_HEADER + half) + c * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    const bf16x8 b = __builtin_bit_cast(bf16x8, raw[p]);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += (float)b[j];
  }
}

__device__ __forceinline__ void stage8(bf16* mine, const bf16* x, const float* xp, int S, int64_t ps, int64_t c) {
  float v[8];
  load_in8(v, x, xp, S, ps, c * 8);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  store_bf16x8(mine + c * 8, o);
}

// Plain all-reduce of n8 16-B chunks: y = sum over ranks of (x or the slab sum), bf16. y may alias x.
template <int NR>
__global__ __launch_bounds__(256) void allreduce_oneshot_kernel(ARPtrs ptrs, int rank, const bf16* x,
                                                                 const float* __restrict__ xp, int S, int64_t ps,
                                                                 bf16* y, int64_t n8, int64_t max_bytes) {
  __shared__ int s_e;
  const int e = ar_epoch(ptrs, rank, &s_e);
  const int b = blockIdx.x, nb = gridDim.x;
  const int64_t per = (n8 + nb - 1) / nb;
  const int64_t c0 = min(n8, (int64_t)b * per), c1 = min(n8, c0 + per);
  const int64_t half = (int64_t)(e & 1) * max_bytes;
  bf16* mine = reinterpret_cast<bf16*>(ptrs.base[rank] + AR_HEADER + half);
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) stage8(mine, x, xp, S, ps, c);
  ar_exchange<NR>(ptrs, rank, e);
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    float v[8];
    ar_sum8<NR>(ptrs, half, c, v);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    store_bf16x8(y + c * 8, o);
  }
  ar_stamp_end(ptrs, rank, e);
}

// Fused: rows r of [T, d] are owned by block r % nblocks (d <= 8 * 256 * CPT). Per row: s = bf16(allreduce(x) +
// resid); resid = s; out = bf16(s * rsqrt(mean(s^2) + eps) * w) — the fused_add_rmsnorm of the same inputs.
// With `pre` (dpre > 0 columns): the row's first dpre columns are ALREADY all-reduced (bf16 [T, dpre], row stride
// pre_s: the first column half of an overlapped TP seam, reduced on a side stream while the second half's GEMM
// streamed) and only the last d - dpre columns (x: [T, d - dpre] or its slabs) go through this exchange — the
// half's all-reduce, the join, the residual add and the RMSNorm of the full row in one launch, no concatenation.
template <int NR, int CPT>
__global__ __launch_bounds__(256) void allreduce_add_rmsnorm_kernel(ARPtrs ptrs, int rank, const bf16* x,
                                                                     const float* __restrict__ xp, int S,
                                                                     int64_t ps, int T, int d,
                                                                     bf16* __restrict__ resid, int64_t rs,
                                                                     const bf16* __restrict__ w, float eps,
                                                                     bf16* __restrict__ out, int64_t os,
                                                                     int64_t max_bytes, const bf16* __restrict__ pre,
                                                                     int64_t pre_s, int dpre) {
  __shared__ int s_e;
  __shared__ float red[4];
  const int e = ar_epoch(ptrs, rank, &s_e);
  const int64_t half = (int64_t)(e & 1) * max_bytes;
  bf16* mine = reinterpret_cast<bf16*>(ptrs.base[rank] + AR_HEADER + half);
  const int n8 = d >> 3, np8 = dpre >> 3, nx8 = n8 - np8;  // chunks per row: all / pre-reduced / exchanged
  for (int r = blockIdx.x; r < T; r += gridDim.x)
    for (int c = threadIdx.x; c < nx8; c += 256) stage8(mine, x, xp, S, ps, (int64_t)r * nx8 + c);
  ar_exchange<NR>(ptrs, rank, e);
  for (int r = blockIdx.x; r < T; r += gridDim.x) {  // block-uniform
    float v[CPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (c < n8) {
        if (c < np8) {
          const bf16x8 pv = load_bf16x8(pre + (int64_t)r * pre_s + c * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = (float)pv[j];
        } else {
          ar_sum8<NR>(ptrs, half, (int64_t)r * nx8 + (c - np8), v[i]);
        }
        const bf16x8 rv = load_bf16x8(resid + (int64_t)r * rs + c * 8);
        bf16x8 sv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sv[j] = (bf16)(v[i][j] + (float)rv[j]);
          v[i][j] = (float)sv[j];
          ss += v[i][j] * v[i][j];
        }
        store_bf16x8(resid + (int64_t)r * rs + c * 8, sv);
      }
    }
    const float inv = rsqrtf(block_sum<256>(ss, red) / (float)d + eps);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (c < n8) {
        const bf16x8 wv = load_bf16x8(w + c * 8);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[i][j] * inv * (float)wv[j]);
        store_bf16x8(out + (int64_t)r * os + c * 8, o);
      }
    }
  }
  ar_stamp_end(ptrs, rank, e);
}

extern "C" hipError_t kafka_car_alloc(int64_t bytes, void** out) {
  hipError_t e = hipExtMallocWithFlags(out, (size_t)(AR_HEADER + bytes), hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  return hipMemset(*out, 0, AR_HEADER);
}

extern "C" int64_t kafka_car_header_bytes() { return AR_HEADER; }

// Host copy of the timing ring ([AR_TIME_SLOTS][2] uint64 = 2 KB) and of block 0's epoch (the call count), on a
// private stream so a /metrics request never waits behind the engine's queued steps.
extern "C" hipError_t kafka_car_timing(const void* own, uint64_t* ring_out, int* epoch_out) {
  hipStream_t s;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  const char* b = static_cast<const char*>(own);
  e = hipMemcpyAsync(ring_out, b + AR_TIME_OFF, AR_TIME_SLOTS * 16, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(epoch_out, b + AR_EPOCH_OFF, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  hipStreamDestroy(s);
  return e;
}

extern "C" hipError_t kafka_car_ipc_handle(void* p, hipIpcMemHandle_t* h) { return hipIpcGetMemHandle(h, p); }

extern "C" hipError_t kafka_car_open(const hipIpcMemHandle_t* h, void** out) {
  return hipIpcOpenMemHandle(out, *h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" hipError_t kafka_car_close(void* p) { return hipIpcCloseMemHandle(p); }

extern "C" hipError_t kafka_car_free(void* p) { return hipFree(p); }

// x: bf16 input (or nullptr with xp = S fp32 slabs of stride ps elements); y: bf16 output (may alias x).
// Every call of a group must use the same nblocks (the per-block epochs advance together).
extern "C" hipError_t kafka_launch_car_allreduce(char* const* bases, int nranks, int rank, const bf16* x,
                                                const float* xp, int S, int64_t ps, bf16* y, int64_t n8,
                                                int64_t max_bytes, int nblocks, hipStream_t st) {
  if (nranks < 2 || nranks > AR_MAX_RANKS || nblocks < 1 || nblocks > AR_MAX_BLOCKS || n8 * 16 > max_bytes ||
      (x == nullptr) == (xp == nullptr))
    return hipErrorInvalidValue;
  ARPtrs p{};
  for (int i = 0; i < nranks; ++i) p.base[i] = bases[i];
  switch (nranks) {
    case 2: allreduce_oneshot_kernel<2><<<nblocks, 256, 0, st>>>(p, rank, x, xp, S, ps, y, n8, max_bytes); break;
    case 4: allreduce_oneshot_kernel<4><<<nblocks, 256, 0, st>>>(p, rank, x, xp, S, ps, y, n8, max_bytes); break;
    case 8: allreduce_oneshot_kernel<8><<<nblocks, 256, 0, st>>>(p, rank, x, xp, S, ps, y, n8, max_bytes); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t kafka_launch_car_allreduce_add_rmsnorm(char* const* bases, int nranks, int rank,
                                                            const bf16* x, const float* xp, int S, int64_t ps,
                                                            int T, int d, bf16* resid, int64_t rs, const bf16* w,
                                                            float eps, bf16* out, int64_t os, int64_t max_bytes,
                                                            int nblocks, const bf16* pre, int64_t pre_s, int dpre,
                                                            hipStream_t st) {
  if (nranks < 2 || nranks > AR_MAX_RANKS || nblocks < 1 || nblocks > AR_MAX_BLOCKS || d % 8 != 0 ||
      dpre % 8 != 0 || dpre < 0 || dpre >= d || (dpre > 0) != (pre != nullptr) ||
      (int64_t)T * (d - dpre) * 2 > max_bytes || (x == nullptr) == (xp == nullptr))
    return hipErrorInvalidValue;
  const int cpt = (d / 8 + 255) / 256;
  ARPtrs p{};
  for (int i = 0; i < nranks; ++i) p.base[i] = bases[i];
#define KAFKA_CARN(NR_, CPT_)                                                                                    \
  allreduce_add_rmsnorm_kernel<NR_, CPT_><<<nblocks, 256, 0, st>>>(p, rank, x, xp, S, ps, T, d, resid, rs, w, eps, \
                                                                   out, os, max_bytes, pre, pre_s, dpre)
#define KAFKA_CARN_R(CPT_)                          \
  switch (nranks) {                                 \
    case 2: KAFKA_CARN(2, CPT_); break;             \
    case 4: KAFKA_CARN(4, CPT_); break;             \
    case 8: KAFKA_CARN(8, CPT_); break;             \
    default: return hipErrorInvalidValue;           \
  }
  if (cpt <= 1) { KAFKA_CARN_R(1) }
  else if (cpt <= 2) { KAFKA_CARN_R(2) }
  else if (cpt <= 4) { KAFKA_CARN_R(4) }
  else if (cpt <= 8) { KAFKA_CARN_R(8) }
  else return hipErrorInvalidValue;
#undef KAFKA_CARN_R
#undef KAFKA_CARN
  return hipGetLastError();
}


// Pull-mode all-to-all (bcast = 0: part q of the image, at q * bpd, goes to rank q; recv part p = peer p's part for
// this rank) or all-gather (bcast = 1: the image is one part of bpd bytes; recv part p = peer p's image).
// nbytes = image bytes (ep * bpd, or bpd); bpd % 16 == 0.
template <int NR>
__global__ __launch_bounds__(256) void a2a_pull_kernel(ARPtrs ptrs, int rank, const ar_i32x4* __restrict__ send,
                                                       int64_t n16, ar_i32x4* __restrict__ recv, int64_t bpd16,
                                                       int bcast, int64_t max_bytes) {
  __shared__ int s_e;
  const int e = ar_epoch(ptrs, rank, &s_e);
  const int b = blockIdx.x, nb = gridDim.x;
  const int64_t per = (n16 + nb - 1) / nb;
  const int64_t c0 = min(n16, (int64_t)b * per), c1 = min(n16, c0 + per);
  const int64_t half = (int64_t)(e & 1) * max_bytes;
  ar_i32x4* mine = reinterpret_cast<ar_i32x4*>(ptrs.base[rank] + AR_HEADER + half);
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) mine[c] = send[c];
  ar_exchange<NR>(ptrs, rank, e);
  // the part addressed to this rank, clipped to this block's staged range
  const int64_t lo = bcast ? 0 : rank * bpd16, hi = lo + bpd16;
  const int64_t a = max(lo, c0), z = min(hi, c1);
  constexpr int U = 4;  // loads in flight per thread and peer
  for (int64_t c = a + threadIdx.x; c < z; c += (int64_t)blockDim.x * U) {
    ar_i32x4 v[NR][U];
#pragma unroll
    for (int p = 0; p < NR; ++p)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t cc = min(c + (int64_t)u * blockDim.x, z - 1);  // clamp, don't branch (stores are guarded)
        v[p][u] = load_sys16_nowait(reinterpret_cast<const bf16*>(ptrs.base[p] + AR_HEADER + half) + cc * 8);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NR; ++p)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t cc = c + (int64_t)u * blockDim.x;
        if (cc < z) recv[p * bpd16 + (cc - lo)] = v[p][u];
      }
  }
  ar_stamp_end(ptrs, rank, e);
}

extern "C" hipError_t kafka_launch_car_a2a(char* const* bases, int nranks, int rank, const void* send, int64_t nbytes,
                                          void* recv, int64_t bpd, int bcast, int64_t max_bytes, int nblocks,
                                          hipStream_t st) {
  if (nranks < 2 || nranks > AR_MAX_RANKS || nblocks < 1 || nblocks > AR_MAX_BLOCKS || nbytes > max_bytes ||
      nbytes % 16 != 0 || bpd % 16 != 0 || (bcast ? nbytes != bpd : nbytes != bpd * nranks))
    return hipErrorInvalidValue;
  ARPtrs p{};
  for (int i = 0; i < nranks; ++i) p.base[i] = bases[i];
  const auto* s = reinterpret_cast<const ar_i32x4*>(send);
  auto* r = reinterpret_cast<ar_i32x4*>(recv);
  switch (nranks) {
    case 2: a2a_pull_kernel<2><<<nblocks, 256, 0, st>>>(p, rank, s, nbytes / 16, r, bpd / 16, bcast, max_bytes); break;
    case 4: a2a_pull_kernel<4><<<nblocks, 256, 0, st>>>(p, rank, s, nbytes / 16, r, bpd / 16, bcast, max_bytes); break;
    case 8: a2a_pull_kernel<8><<<nblocks, 256, 0, st>>>(p, rank, s, nbytes / 16, r, bpd / 16, bcast, max_bytes); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kafka
