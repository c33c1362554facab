// stage_probe.hip — the stager's ceiling: how fast does a bare stream with the stager's read:write
// byte ratio run?  k_soa_to_aos reads 16 B and writes 32 B per point (float32 in, float64 out);
// k_aos_to_soa the reverse.  Each variant moves 60 M points' worth of bytes, one 16-byte load or
// store per lane instruction, non-temporal loads, stores with each cache policy; median of 20 runs.
//   hipcc -O3 --offload-arch=gfx950 tools/stage_probe.hip -o tools/stage_probe && tools/stage_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// RI 16-byte loads and WO 16-byte stores per lane, consecutive lanes on consecutive 16-byte slots
template <int RI, int WO, int POL>
__global__ __launch_bounds__(256) void k_stream(const v4f* __restrict__ in, v4f* __restrict__ out, long units) {
  const long u = (long)blockIdx.x * 256 + threadIdx.x;
  if (u >= units) return;
  const long b = (long)blockIdx.x * 256;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < RI; ++r) acc += __builtin_nontemporal_load(in + b * RI + r * 256 + threadIdx.x);
#pragma unroll
  for (int w = 0; w < WO; ++w) st<POL>(out + b * WO + w * 256 + threadIdx.x, acc + (float)w);
}

template <int RI, int WO, int POL>
static void run(const char* name, v4f* in, v4f* out, long units) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned grid = (unsigned)((units + 255) / 256);
  std::vector<float> ms;
  for (int i = 0; i < 25; ++i) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_stream<RI, WO, POL>), dim3(grid), dim3(256), 0, 0, in, out, units);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t;
    hipEventElapsedTime(&t, e0, e1);
    if (i >= 5) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double bytes = 16.0 * (RI + WO) * units;
  const double med = ms[ms.size() / 2];
  printf("{\"variant\": \"%s\", \"read_B\": %.0f, \"write_B\": %.0f, \"median_us\": %.1f, \"min_us\": %.1f, "
         "\"TBs\": %.3f, \"frac_of_8TBs\": %.3f}\n",
         name, 16.0 * RI * units, 16.0 * WO * units, med * 1e3, ms[0] * 1e3, bytes / (med * 1e-3) / 1e12,
         bytes / (med * 1e-3) / 8e12);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  const long pts = 60000000;     // the bench batch: 60 M points
  const long units = pts / 4;    // one float4 (4 f32 points of a column, or 2 f64 values) per lane per load
  v4f *in, *out;
  if (hipMalloc(&in, 32 * pts) != hipSuccess || hipMalloc(&out, 32 * pts) != hipSuccess) return 1;
  hipMemset(in, 0, 32 * pts);
  hipMemset(out, 0, 32 * pts);
  hipDeviceSynchronize();
  // soa_to_aos shape: 16 B read, 32 B written per point (pts / 4 lanes x 4 loads + 8 stores)
  run<4, 8, 0>("r16w32 default", in, out, units);
  run<4, 8, 1>("r16w32 sc1", in, out, units);
  run<4, 8, 2>("r16w32 nt", in, out, units);
  run<1, 2, 2>("r16w32 nt (1 load / 2 stores)", in, out, 4 * units);
  // aos_to_soa shape: 32 B read, 16 B written per point
  run<8, 4, 0>("r32w16 default", in, out, units);
  run<8, 4, 2>("r32w16 nt", in, out, units);
  // 1:1 copy
  run<4, 4, 2>("r16w16 nt", in, out, units);
  run<4, 4, 0>("r16w16 default", in, out, units);
  // write only
  run<0, 8, 2>("w32 nt (write only)", in, out, units);
  run<0, 8, 0>("w32 default (write only)", in, out, units);
  hipFree(in);
  hipFree(out);
  return 0;
}
