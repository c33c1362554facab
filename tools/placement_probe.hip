// placement_probe.hip — how much does WHERE a streaming kernel's buffers land matter?  K separate
// (input, output) allocation pairs of the SLERP kernel's size (60 M points: 5 input columns, 4
// output columns, blocked), the same 5-in / 4-out pass (float4 lanes, nt loads, sc1 stores, one
// 1024-point sub-tile per workgroup) timed on each pair.  Launch order is fixed (per pair: 2 warm-up
// + 10 timed launches), so a rocprofv3 --pmc run's dispatches map to pairs by index (12 per pair).
//   hipcc -O3 --offload-arch=gfx950 tools/placement_probe.hip -o tools/placement_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_pass(const float* __restrict__ in, float* __restrict__ out, long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (4 * g >= n) return;
  const long blk = g >> 6, off = 4 * (g & 63);
  const float* bi = in + blk * 5 * 256 + off;
  float* bo = out + blk * 4 * 256 + off;
  v4f v[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const v4f r = v[c] * 1.0001f + v[4];
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(bo + c * 256), "v"(r) : "memory");
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 6;
  const long n = 60'000'000 / 1024 * 1024;
  float* in[16];
  float* out[16];
  for (int k = 0; k < K; ++k) {
    if (hipMalloc(&in[k], 5 * n * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&out[k], 4 * n * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(in[k], 0, 5 * n * sizeof(float));
    (void)hipMemset(out[k], 0, 4 * n * sizeof(float));
  }
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  for (int k = 0; k < K; ++k) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, 0, in[k], out[k], n);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_pass, dim3(grid), dim3(256), 0, 0, in[k], out[k], n);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 10;
    std::printf("{\"pair\": %d, \"in\": \"%p\", \"out\": \"%p\", \"us\": %.1f, \"TBs\": %.3f}\n", k, (void*)in[k],
                (void*)out[k], us, 36.0 * n / (us * 1e-6) / 1e12);
    std::fflush(stdout);
  }
  return 0;
}
