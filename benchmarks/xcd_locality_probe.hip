// XCD <-> HBM locality probe (gfx950): does a workgroup read faster from addresses whose interleave unit maps to
// "its" XCD? Workgroup w runs on XCD w % 8 (round-robin dispatch). Each workgroup streams `per_wg` bytes as
// `unit`-byte chunks; chunk ids are chosen so that chunk_id % 8 == (w % 8 + shift) % 8 (shift 0 = "matching",
// 1..7 = the other residues) or contiguous (shift = -1). If HBM interleaves `unit`-sized chunks over 8 stacks and
// each XCD is closer to one stack, shift 0 reads locally. Prints GB/s per (unit, shift).
// Build: hipcc -O3 --offload-arch=gfx950 -o xcd_locality_probe xcd_locality_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe(const f32x4* __restrict__ buf, size_t n_units, int unit_vec,
                                             int per_wg_units, int shift, float* __restrict__ sink) {
  const int w = blockIdx.x;
  const int x = w % 8;
  const int grp = w / 8;  // workgroups of one XCD: grp = 0 .. gridDim / 8
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < per_wg_units; ++i) {
    size_t c;
    if (shift < 0) {
      c = (size_t)w * per_wg_units + i;  // contiguous per workgroup
    } else {
      const size_t k = (size_t)grp * per_wg_units + i;  // k-th chunk of residue r
      c = k * 8 + (size_t)((x + shift) & 7);
    }
    c %= n_units;
    const f32x4* p = buf + c * unit_vec;
    for (int j = threadIdx.x; j < unit_vec; j += 256) acc += __builtin_nontemporal_load(p + j);
  }
  if (acc[0] == 12345.f) sink[w] = acc[1] + acc[2] + acc[3];
}

int main() {
  const size_t bytes = (size_t)4 << 30;  // 4 GB: far beyond the MALL
  f32x4* buf;
  float* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int nwg = 2048;
  for (int unit : {1024, 2048, 4096, 8192, 16384, 65536}) {
    const int unit_vec = unit / 16;
    const size_t n_units = bytes / unit;
    const int per_wg = (int)((size_t)(1 << 30) / unit / nwg);  // 1 GB per launch
    for (int shift : {-1, 0, 1, 2, 4}) {
      probe<<<nwg, 256>>>(buf, n_units, unit_vec, per_wg, shift, sink);
      hipDeviceSynchronize();
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(a);
        probe<<<nwg, 256>>>(buf, n_units, unit_vec, per_wg, shift, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      const double gb = (double)per_wg * nwg * unit / 1e9;
      printf("{\"unit\": %d, \"shift\": %d, \"ms\": %.3f, \"GB/s\": %.0f}\n", unit, shift, best, gb / best * 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
