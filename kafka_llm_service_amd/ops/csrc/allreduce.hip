// One-shot all-reduce over xGMI for decode-sized TP messages (SURVEY.md §2.6 `custom_allreduce_oneshot`, §5.8).
//
// Every rank owns ONE fine-grained, uncached device allocation, IPC-mapped into every peer of its TP group:
//     [ flags: MAX_RANKS x MAX_BLOCKS int32 | err: int32 | pad to 8 KB | data: 2 x max_bytes ]
// A call with epoch e (host counter, +1 per call) uses data half (e & 1). Block b of every rank handles the same
// slice b of the tensor:
//   1. copy its slice of x into its OWN data half (uncached -> straight to HBM),
//   2. publish: store e into flags[my_rank][b] of EVERY peer (system-scope release),
//   3. wait until flags[p][b] >= e for every peer p in its own flag block (system-scope acquire, bounded spin:
//      after ~2 s it sets err and proceeds, so a lost peer can never hang the GPU),
//   4. read slice b from all peers' data halves at once (each MI355X reads its 7 peers over its 7 xGMI links in
//      parallel: one hop, vs a ring's 2(N-1) hops), sum in fp32, write the result back into x.
// Double-buffering by epoch parity makes a trailing barrier unnecessary: a peer can only still be reading half
// (e & 1) of call e-2 before it signals call e-1, and this rank passed call e-1's barrier before starting call e.
// Loads of peer data use sc0 sc1 (system-coherent) so no stale line from call e-2 can be returned.
#include "common.h"

namespace kafka {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 128;
constexpr int AR_HEADER = 8192;  // flags (4 KB) + err, padded

struct ARPtrs {
  char* base[AR_MAX_RANKS];  // every rank's allocation, mapped into this process (base[rank] = own)
};

__device__ __forceinline__ f32x4 bf16x8_lo(bf16x8 v) { return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; }
__device__ __forceinline__ f32x4 bf16x8_hi(bf16x8 v) { return f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]}; }

typedef int ar_i32x4 __attribute__((ext_vector_type(4)));

// system-coherent 16-B load, issued without a wait (the caller waits once for all peers' loads)
__device__ __forceinline__ ar_i32x4 load_sys16_nowait(const bf16* p) {
  ar_i32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}

template <int NR>
__global__ __launch_bounds__(256) void allreduce_oneshot_kernel(ARPtrs ptrs, int rank, int epoch, bf16* __restrict__ x,
                                                                 int64_t n8, int64_t max_bytes) {
  const int b = blockIdx.x, nb = gridDim.x;
  const int64_t per = (n8 + nb - 1) / nb;  // 16-B chunks of this block's slice
  const int64_t c0 = min(n8, (int64_t)b * per), c1 = min(n8, c0 + per);
  const int64_t half = (int64_t)(epoch & 1) * max_bytes;
  bf16* mine = reinterpret_cast<bf16*>(ptrs.base[rank] + AR_HEADER + half);
  // 1. stage my slice
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) store_bf16x8(mine + c * 8, load_bf16x8(x + c * 8));
  __threadfence_system();  // every thread's staging stores are visible system-wide before the flag goes out
  __syncthreads();
  // 2. publish to every peer, 3. wait for every peer
  if (threadIdx.x < NR) {
    const int p = threadIdx.x;
    int* pf = reinterpret_cast<int*>(ptrs.base[p]) + rank * AR_MAX_BLOCKS + b;
    __hip_atomic_store(pf, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    int* my = reinterpret_cast<int*>(ptrs.base[rank]) + p * AR_MAX_BLOCKS + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
    while (__hip_atomic_load(my, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s: report instead of hanging the queue
        int* err = reinterpret_cast<int*>(ptrs.base[rank] + AR_MAX_RANKS * AR_MAX_BLOCKS * 4);
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  // 4. reduce slice b over all ranks (fixed rank order: every rank computes bit-identical sums)
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    ar_i32x4 raw[NR];
#pragma unroll
    for (int p = 0; p < NR; ++p)  // all peers' loads in flight at once (one per xGMI link)
      raw[p] = load_sys16_nowait(reinterpret_cast<const bf16*>(ptrs.base[p] + AR_HEADER + half) + c * 8);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const bf16x8 v = __builtin_bit_cast(bf16x8, raw[p]);
      lo += bf16x8_lo(v);
      hi += bf16x8_hi(v);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)lo[j];
      o[4 + j] = (bf16)hi[j];
    }
    store_bf16x8(x + c * 8, o);
  }
}

extern "C" hipError_t kafka_car_alloc(int64_t bytes, void** out) {
  hipError_t e = hipExtMallocWithFlags(out, (size_t)(AR_HEADER + bytes), hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  return hipMemset(*out, 0, AR_HEADER);
}

extern "C" int64_t kafka_car_header_bytes() { return AR_HEADER; }

extern "C" hipError_t kafka_car_ipc_handle(void* p, hipIpcMemHandle_t* h) { return hipIpcGetMemHandle(h, p); }

extern "C" hipError_t kafka_car_open(const hipIpcMemHandle_t* h, void** out) {
  return hipIpcOpenMemHandle(out, *h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" hipError_t kafka_car_close(void* p) { return hipIpcCloseMemHandle(p); }

extern "C" hipError_t kafka_car_free(void* p) { return hipFree(p); }

extern "C" hipError_t kafka_launch_car_allreduce(char* const* bases, int nranks, int rank, int epoch, bf16* x,
                                                int64_t n8, int64_t max_bytes, int nblocks, hipStream_t st) {
  if (nranks < 2 || nranks > AR_MAX_RANKS || nblocks < 1 || nblocks > AR_MAX_BLOCKS || n8 * 16 > max_bytes)
    return hipErrorInvalidValue;
  ARPtrs p{};
  for (int i = 0; i < nranks; ++i) p.base[i] = bases[i];
  switch (nranks) {
    case 2: allreduce_oneshot_kernel<2><<<nblocks, 256, 0, st>>>(p, rank, epoch, x, n8, max_bytes); break;
    case 4: allreduce_oneshot_kernel<4><<<nblocks, 256, 0, st>>>(p, rank, epoch, x, n8, max_bytes); break;
    case 8: allreduce_oneshot_kernel<8><<<nblocks, 256, 0, st>>>(p, rank, epoch, x, n8, max_bytes); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kafka
