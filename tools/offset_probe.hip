// offset_probe.hip — does the distance between a streaming kernel's input and output buffers
// change its HBM rate?  One allocation; in = base, out = base + span + delta for a sweep of
// deltas; a frame-mode-shaped pass (16 B read + 16 B written per point, float4 lanes, nt loads,
// sc1 nt stores, one 1024-point sub-tile per workgroup) timed with HIP events per delta.
//   hipcc -O3 --offload-arch=gfx950 tools/offset_probe.hip -o /tmp/offset_probe && /tmp/offset_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1nt(float* p, v4f v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// C input columns per 256-point block, 4 output columns (blocked layout of the batch)
template <int CI>
__global__ __launch_bounds__(256) void k_pass(const float* __restrict__ in, float* __restrict__ out, long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;   // float4 group
  if (4 * g >= n) return;
  const long blk = g >> 6, off = 4 * (g & 63);
  const float* bi = in + blk * CI * 256 + off;
  float* bo = out + blk * 4 * 256 + off;
  v4f v[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
#pragma unroll
  for (int c = 0; c < 4; ++c) st_sc1nt(bo + c * 256, v[c] * 1.0001f + (CI > 4 ? v[CI - 1] : v[0]));
}

int main() {
  const long n = 60'000'000 / 1024 * 1024;
  const size_t in_bytes = 5 * n * sizeof(float), out_bytes = 4 * n * sizeof(float);
  const size_t max_delta = 64ul << 20;
  char* base = nullptr;
  if (hipMalloc(&base, in_bytes + out_bytes + max_delta + (4ul << 20)) != hipSuccess) return 1;
  hipMemset(base, 0, in_bytes + out_bytes + max_delta + (4ul << 20));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<size_t> deltas = {0, 256, 1024, 2048, 4096, 8192, 12288, 16384, 32768, 65536, 131072, 262144,
                                524288, 1u << 20, 2u << 20, 3u << 20, 4u << 20, 8u << 20, 16u << 20, 64u << 20};
  const int grid = (int)(n / 1024);
  for (int ci = 4; ci <= 5; ++ci) {
    const size_t span = (ci == 4 ? 4 : 5) * n * sizeof(float);
    for (int round = 0; round < 2; ++round) {
      for (size_t d : deltas) {
        const float* in = reinterpret_cast<const float*>(base);
        float* out = reinterpret_cast<float*>(base + span + d);
        auto launch = [&] {
          if (ci == 4) hipLaunchKernelGGL(k_pass<4>, dim3(grid), dim3(256), 0, 0, in, out, n);
          else hipLaunchKernelGGL(k_pass<5>, dim3(grid), dim3(256), 0, 0, in, out, n);
        };
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0, 0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        const double bytes = (ci * 4.0 + 16.0) * n;
        std::printf("{\"in_cols\": %d, \"round\": %d, \"delta\": %zu, \"us\": %.1f, \"TBs\": %.3f}\n", ci, round, d, us,
                    bytes / (us * 1e-6) / 1e12);
        std::fflush(stdout);
      }
    }
  }
  hipFree(base);
  return 0;
}
