// layout_probe.hip — does the column layout of a batch matter for a 5-in / 4-out streaming pass?
// Compares (a) columns a whole batch apart (the padded-CSR layout: stride = cap) with (b) the same
// columns blocked per 2048-point tile (tile-local SoA).  Pure copy-like traffic: 20 B read, 16 B
// written per point, float4 lanes, nt loads / sc1 stores like the deskew kernels.
//   hipcc -O3 --offload-arch=gfx950 tools/layout_probe.hip -o /tmp/layout_probe && /tmp/layout_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1(float* p, v4f v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// layout A: column c of point p at c*cap + p; one workgroup per 1024-point sub-tile
__global__ __launch_bounds__(256) void k_cols(const float* __restrict__ in, float* __restrict__ out, long cap,
                                              long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;     // float4 group
  if (4 * g >= n) return;
  v4f v[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(in + c * cap) + g);
  v4f o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = v[c] * 1.0001f + v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) st_sc1(out + c * cap + 4 * g, o[c]);
}

// layout B: tile t (2048 points) holds its 5 (in) / 4 (out) columns contiguously
__global__ __launch_bounds__(256) void k_tiles(const float* __restrict__ in, float* __restrict__ out, long n) {
  const long sub = blockIdx.x;                      // 1024-point sub-tile
  const long tile = sub >> 1, half = sub & 1;
  const float* ti = in + tile * 5 * 2048 + half * 1024;
  float* to = out + tile * 4 * 2048 + half * 1024;
  const int g = threadIdx.x;
  if (sub * 1024 + 4 * g >= n) return;
  v4f v[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(ti + c * 2048) + g);
  v4f o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = v[c] * 1.0001f + v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) st_sc1(to + c * 2048 + 4 * g, o[c]);
}

// layout C: 256-point blocks, block b holds its 5 (in) / 4 (out) columns of 256 floats
template <int B>
__global__ __launch_bounds__(256) void k_blocks(const float* __restrict__ in, float* __restrict__ out, long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;     // float4 group
  if (4 * g >= n) return;
  const long p = 4 * g, blk = p / B, off = p % B;
  const float* bi = in + blk * 5 * B + off;
  float* bo = out + blk * 4 * B + off;
  v4f v[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * B));
  v4f o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) o[c] = v[c] * 1.0001f + v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) st_sc1(bo + c * B, o[c]);
}

int main() {
  const long n = 60'000'000 / 2048 * 2048;          // whole tiles
  float *in, *out;
  hipMalloc(&in, 5 * n * sizeof(float));
  hipMalloc(&out, 4 * n * sizeof(float));
  hipMemset(in, 0, 5 * n * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  for (int round = 0; round < 3; ++round) {
    for (int which = 0; which < 4; ++which) {
      auto launch = [&] {
        if (which == 0) hipLaunchKernelGGL(k_cols, dim3(grid), dim3(256), 0, 0, in, out, n, n);
        else if (which == 1) hipLaunchKernelGGL(k_tiles, dim3(grid), dim3(256), 0, 0, in, out, n);
        else if (which == 2) hipLaunchKernelGGL(k_blocks<256>, dim3(grid), dim3(256), 0, 0, in, out, n);
        else hipLaunchKernelGGL(k_blocks<1024>, dim3(grid), dim3(256), 0, 0, in, out, n);
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
      std::printf("{\"layout\": \"%s\", \"round\": %d, \"us\": %.1f, \"TBs\": %.3f}\n", which == 0 ? "columns" : which == 1 ? "tiles2048" : which == 2 ? "blocks256" : "blocks1024",
                  round, us, 36.0 * n / (us * 1e-6) / 1e12);
    }
  }
  hipFree(in);
  hipFree(out);
  return 0;
}
