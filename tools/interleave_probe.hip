// interleave_probe.hip — does placing a block's output next to its input (one allocation, 256-point
// blocks of CI input columns followed by the 4 output columns of the same block) stream faster than
// separate input and output buffers?  A frame-/SLERP-shaped pass (float4 lanes, nt loads, sc1 nt
// stores, one 1024-point sub-tile per workgroup), HIP events over 20 launches per arm, arms
// interleaved over rounds.  Output: one JSON line per (arm, round).
//   hipcc -O3 --offload-arch=gfx950 tools/interleave_probe.hip -o tools/interleave_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1nt(float* p, v4f v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// in block pitch PI floats, out block pitch PO floats, out at out_base (same or another buffer)
template <int CI>
__global__ __launch_bounds__(256) void k_pass(const float* __restrict__ in, long pi, float* __restrict__ out, long po,
                                              long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;   // float4 group
  if (4 * g >= n) return;
  const long blk = g >> 6, off = 4 * (g & 63);
  const float* bi = in + blk * pi + off;
  float* bo = out + blk * po + off;
  v4f v[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
#pragma unroll
  for (int c = 0; c < 4; ++c) st_sc1nt(bo + c * 256, v[c] * 1.0001f + (CI > 4 ? v[CI - 1] : v[0]));
}

int main() {
  const long n = 60'000'000 / 1024 * 1024;
  const long blocks = n / 256;
  float *sep_in[2], *sep_out[2], *il[2];
  for (int k = 0; k < 2; ++k) {
    if (hipMalloc(&sep_in[k], 5 * n * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&sep_out[k], 4 * n * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&il[k], 9 * n * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(sep_in[k], 0, 5 * n * sizeof(float));
    (void)hipMemset(il[k], 0, 9 * n * sizeof(float));
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  (void)blocks;
  for (int ci = 4; ci <= 5; ++ci) {
    for (int round = 0; round < 3; ++round) {
      for (int arm = 0; arm < 4; ++arm) {   // 0,1: separate buffers (two allocations each); 2,3: interleaved
        const int k = arm & 1;
        const bool inter = arm >= 2;
        const float* in = inter ? il[k] : sep_in[k];
        float* out = inter ? il[k] + ci * 256 : sep_out[k];
        const long pi = inter ? (ci + 4) * 256 : ci * 256;
        const long po = inter ? (ci + 4) * 256 : 4 * 256;
        auto launch = [&] {
          if (ci == 4) hipLaunchKernelGGL(k_pass<4>, dim3(grid), dim3(256), 0, 0, in, pi, out, po, n);
          else hipLaunchKernelGGL(k_pass<5>, dim3(grid), dim3(256), 0, 0, in, pi, out, po, n);
        };
        for (int w = 0; w < 3; ++w) launch();
        (void)hipEventRecord(e0, 0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        const double bytes = (ci * 4.0 + 16.0) * n;
        std::printf("{\"in_cols\": %d, \"round\": %d, \"arm\": \"%s%d\", \"us\": %.1f, \"TBs\": %.3f}\n", ci, round,
                    inter ? "interleaved" : "separate", k, us, bytes / (us * 1e-6) / 1e12);
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
