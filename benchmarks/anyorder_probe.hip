// Probe: does a kernel launched with hipExtAnyOrderLaunch on the SAME stream start before its predecessor has
// finished on gfx950 (the AQL barrier bit cleared), and what does a device-counter hand-off between the two cost?
//
// producer: W workgroups stream a buffer (imbalanced: workgroup i reads (1 + i % 4) slices, so CUs free up at
// different times), stamp start / end on the 100 MHz clock, then arrive on a device counter.
// consumer: W workgroups stamp their start, wait (bounded: 20 ms) until the counter reaches W, stamp again.
// Printed per mode (ordered / any-order): consumer start relative to the producer's first and last end, and the
// hand-off (consumer released - last producer end).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o anyorder_probe benchmarks/anyorder_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void producer(const float4* __restrict__ buf, size_t slice, float* out, int* ctr,
                                                unsigned long long* st) {
  const unsigned long long t0 = rt();
  const int wg = blockIdx.x;
  const int reps = 1 + wg % 4;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r) {
    const float4* p = buf + ((size_t)wg * 4 + r) * slice;
    for (size_t i = threadIdx.x; i < slice; i += 256) {
      const float4 v = p[i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  out[wg * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    st[wg * 2] = t0;
    st[wg * 2 + 1] = rt();
  }
}

__global__ __launch_bounds__(256) void consumer(int* ctr, int expect, unsigned long long* st) {
  const unsigned long long t0 = rt();
  unsigned long long t1 = t0;
  if (threadIdx.x == 0) {
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < expect) {
      __builtin_amdgcn_s_sleep(2);
      t1 = rt();
      if (t1 - t0 > 2000000ull) break;  // 20 ms: never hang the box on a failed hand-off
    }
    t1 = rt();
    st[blockIdx.x * 2] = t0;
    st[blockIdx.x * 2 + 1] = t1;
  }
  __syncthreads();
}

int main() {
  const int W = 256;
  const size_t slice = (size_t)1 << 16;  // float4 per slice: 1 MiB
  float4* buf;
  float* out;
  int* ctr;
  unsigned long long *sp, *sc;
  CK(hipMalloc(&buf, (size_t)W * 4 * slice * sizeof(float4)));
  CK(hipMemset(buf, 0, (size_t)W * 4 * slice * sizeof(float4)));
  CK(hipMalloc(&out, W * 256 * sizeof(float)));
  CK(hipMalloc(&ctr, sizeof(int)));
  CK(hipMalloc(&sp, W * 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&sc, W * 2 * sizeof(unsigned long long)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<unsigned long long> hp(W * 2), hc(W * 2);
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipMemsetAsync(ctr, 0, sizeof(int), s));
      hipLaunchKernelGGL(producer, dim3(W), dim3(256), 0, s, buf, slice, out, ctr, sp);
      int expect = W;
      void* args[] = {&ctr, &expect, &sc};
      CK(hipExtLaunchKernel((const void*)consumer, dim3(W), dim3(256), args, 0, s, nullptr, nullptr, mode));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(hp.data(), sp, hp.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hc.data(), sc, hc.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long p0 = ~0ull, pe_min = ~0ull, pe_max = 0, c0 = ~0ull, c0max = 0, crel = 0;
      for (int i = 0; i < W; ++i) {
        p0 = std::min(p0, hp[2 * i]);
        pe_min = std::min(pe_min, hp[2 * i + 1]);
        pe_max = std::max(pe_max, hp[2 * i + 1]);
        c0 = std::min(c0, hc[2 * i]);
        c0max = std::max(c0max, hc[2 * i]);
        crel = std::max(crel, hc[2 * i + 1]);
      }
      auto us = [&](unsigned long long a, unsigned long long b) { return ((double)a - (double)b) * 0.01; };
      if (rep > 0)
        printf("{\"mode\": \"%s\", \"producer_span_us\": %.2f, \"first_producer_end_us\": %.2f, "
               "\"consumer_first_start_vs_last_end_us\": %.2f, \"consumer_last_start_vs_last_end_us\": %.2f, "
               "\"released_vs_last_end_us\": %.2f}\n",
               mode ? "any_order" : "ordered", us(pe_max, p0), us(pe_min, p0), us(c0, pe_max), us(c0max, pe_max),
               us(crel, pe_max));
    }
  }
  return 0;
}
