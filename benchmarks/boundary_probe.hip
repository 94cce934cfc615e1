// Probe: what a kernel boundary costs on gfx950, eager vs hipGraph replay, and how it depends on the dirty L2
// lines the previous kernel leaves (plain vs sc1 stores) and on L2 reuse across the boundary.
//
// A chain of N dependent launches on one stream, each kernel = 256 workgroups x 256 threads that
//   mode 0 "nop"     : do nothing
//   mode 1 "plain"   : write BYTES (default 512 KiB) with plain 16-B stores   (lines stay dirty in the writer XCD's L2)
//   mode 2 "sc1"     : write BYTES with 16-B sc1 stores                       (lines leave the L2)
//   mode 3 "reread"  : read BYTES written by the previous kernel (plain) and write them back plain (the engine's
//                      producer -> consumer pattern: is the consumer's read an L2 hit after the boundary?)
// (argv: N, BYTES, SPIN = 100 MHz ticks each kernel idles first so an eager chain is GPU-bound, not host-bound)
// timed with hipEvents around the whole chain; us per kernel printed as one JSON line per (mode, eager|graph).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/boundary_probe benchmarks/boundary_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void step(f32x4* __restrict__ a, f32x4* __restrict__ b, int n4, int mode, float k,
                                            int spin) {
  const int i0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  if (spin > 0) {  // every workgroup busy for `spin` ticks of the 100 MHz clock (keeps the eager chain GPU-bound)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(1);
  }
  if (mode == 0) return;
  for (int i = i0; i < n4; i += stride) {
    if (mode == 1) {
      a[i] = f32x4{k, k, k, k};
    } else if (mode == 2) {
      f32x4 v = {k, k, k, k};
      asm volatile("s_nop 4\n\tglobal_store_dwordx4 %0, %1, off sc1\n\ts_nop 4" ::"v"(a + i), "v"(v) : "memory");
    } else {
      f32x4 v = b[i];
      a[i] = v + k;
    }
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 400;
  const size_t bytes = argc > 2 ? (size_t)atol(argv[2]) : (512 << 10);
  const int n4 = (int)(bytes / 16);
  const int spin = argc > 3 ? atoi(argv[3]) : 0;  // 100 MHz ticks per kernel (e.g. 1000 = 10 us)
  f32x4 *A, *B;
  CK(hipMalloc(&A, bytes));
  CK(hipMalloc(&B, bytes));
  CK(hipMemset(A, 0, bytes));
  CK(hipMemset(B, 0, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"nop", "plain", "sc1", "reread"};
  for (int mode = 0; mode < 4; ++mode) {
    auto chain = [&]() {
      for (int i = 0; i < N; ++i) {
        if (mode == 3)  // ping-pong: kernel i reads what kernel i - 1 wrote
          step<<<256, 256, 0, st>>>((i & 1) ? A : B, (i & 1) ? B : A, n4, mode, 1.f, spin);
        else
          step<<<256, 256, 0, st>>>(A, B, n4, mode, (float)i, spin);
      }
    };
    for (int g = 0; g < 2; ++g) {
      hipGraphExec_t ex = nullptr;
      if (g) {
        hipGraph_t graph;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        chain();
        CK(hipStreamEndCapture(st, &graph));
        CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
        CK(hipGraphDestroy(graph));
      }
      float best = 1e30f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0, st));
        if (g)
          CK(hipGraphLaunch(ex, st));
        else
          chain();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("{\"mode\": \"%s\", \"launch\": \"%s\", \"kernels\": %d, \"bytes\": %zu, \"spin_us\": %.2f, \"us_per_kernel\": %.3f}\n",
             names[mode], g ? "graph" : "eager", N, bytes, spin / 100.f, best * 1e3f / N);
      if (ex) CK(hipGraphExecDestroy(ex));
    }
  }
  return 0;
}
