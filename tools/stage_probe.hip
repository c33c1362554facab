// stage_probe.hip — the stager's ceiling: how fast does a bare stream with the stager's read:write
// byte ratio run?  k_soa_to_aos reads 16 B and writes 32 B per point (float32 in, float64 out);
// k_aos_to_soa the reverse.  Each variant moves 60 M points' worth of bytes, one 16-byte load or
// store per lane instruction, non-temporal loads, stores with each cache policy; median of 20 runs.
//   hipcc -O3 --offload-arch=gfx950 tools/stage_probe.hip -o tools/stage_probe && tools/stage_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
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

// The per-point kernels' blocked layout (5 columns x 256 points per block: x|y|z|i|t, 4 columns
// out): LPG lanes per float4 group (1: one lane loads all 5 columns and stores 4; 2: lane h loads
// columns 2h, 2h+1 and t and stores 2; 4: lane c loads column c and t and stores 1), with K
// dependent FMAs per value between the loads and the stores (the per-point math's spacing).
template <int LPG, int K, int POL>
__global__ __launch_bounds__(256) void k_blocked(const v4f* __restrict__ in, v4f* __restrict__ out, long groups) {
  const long lane = (long)blockIdx.x * 256 + threadIdx.x;
  const long g = lane / LPG;
  const int part = (int)(lane % LPG);
  if (g >= groups) return;
  const long blk = g >> 6, off = g & 63;                   // 64 float4 groups per 256-point block
  const v4f* bi = in + blk * 5 * 64 + off;
  v4f* bo = out + blk * 4 * 64 + off;
  constexpr int NC = 4 / LPG;                               // columns per lane
  v4f v[NC];
  const v4f t = __builtin_nontemporal_load(bi + 4 * 64);
#pragma unroll
  for (int j = 0; j < NC; ++j) v[j] = __builtin_nontemporal_load(bi + (part * NC + j) * 64);
  v4f a = t;
#pragma unroll
  for (int k = 0; k < K; ++k) a = a * 1.0000001f + 0.5f;
#pragma unroll
  for (int j = 0; j < NC; ++j) st<POL>(bo + (part * NC + j) * 64, v[j] + a);
}

template <int LPG, int K, int POL>
static void run_blocked(const char* name, v4f* in, v4f* out, long groups, unsigned lds = 0) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned grid = (unsigned)((groups * LPG + 255) / 256);
  std::vector<float> ms;
  for (int i = 0; i < 25; ++i) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_blocked<LPG, K, POL>), dim3(grid), dim3(256), lds, 0, in, out, groups);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t;
    hipEventElapsedTime(&t, e0, e1);
    if (i >= 5) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double bytes = 36.0 * 4 * groups, med = ms[ms.size() / 2];
  printf("{\"variant\": \"%s\", \"median_us\": %.1f, \"min_us\": %.1f, \"TBs\": %.3f, \"frac_of_8TBs\": %.3f}\n", name,
         med * 1e3, ms[0] * 1e3, bytes / (med * 1e-3) / 1e12, bytes / (med * 1e-3) / 8e12);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
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

int main(int argc, char** argv) {
  const long pts = argc > 1 ? atol(argv[1]) : 60000000;   // default: the bench batch, 60 M points
  const bool blocked_only = argc > 2;
  const long units = pts / 4;    // one float4 (4 f32 points of a column, or 2 f64 values) per lane per load
  v4f *in, *out;
  if (hipMalloc(&in, 32 * pts) != hipSuccess || hipMalloc(&out, 32 * pts) != hipSuccess) return 1;
  hipMemset(in, 0, 32 * pts);
  hipMemset(out, 0, 32 * pts);
  hipDeviceSynchronize();
  if (blocked_only) goto blocked;
  // soa_to_aos shape: 16 B read, 32 B written per point (pts / 4 lanes x 4 loads + 8 stores)
  run<4, 8, 0>("r16w32 default", in, out, units);
  run<4, 8, 1>("r16w32 sc1", in, out, units);
  run<4, 8, 2>("r16w32 nt", in, out, units);
  run<1, 2, 2>("r16w32 nt (1 load / 2 stores)", in, out, 4 * units);
  run<1, 2, 0>("r16w32 default (1 load / 2 stores)", in, out, 4 * units);
  run<2, 4, 2>("r16w32 nt (2 loads / 4 stores)", in, out, 2 * units);
  // aos_to_soa shape: 32 B read, 16 B written per point
  run<8, 4, 0>("r32w16 default", in, out, units);
  run<8, 4, 2>("r32w16 nt", in, out, units);
  run<2, 1, 2>("r32w16 nt (2 loads / 1 store)", in, out, 4 * units);
  // 1:1 copy (the frame kernel's 16 B in / 16 B out)
  run<4, 4, 2>("r16w16 nt", in, out, units);
  run<4, 4, 0>("r16w16 default", in, out, units);
  run<1, 1, 2>("r16w16 nt (1 load / 1 store)", in, out, 4 * units);
  run<1, 1, 1>("r16w16 sc1 (1 load / 1 store)", in, out, 4 * units);
  // 5:4 (the per-point kernels' 20 B in / 16 B out)
  run<5, 4, 2>("r20w16 nt", in, out, units);
  run<5, 4, 1>("r20w16 sc1", in, out, units);
  // write only
  run<0, 8, 2>("w32 nt (write only)", in, out, units);
  run<0, 8, 0>("w32 default (write only)", in, out, units);
  // 5-in / 4-out blocked (the per-point kernels' 20 B in / 16 B out per point)
blocked:
  const long groups = pts / 4;
  run<1, 1, 1>("r16w16 sc1 (1 load / 1 store)", in, out, pts);
  run<4, 4, 2>("r16w16 nt", in, out, pts / 4);
  run_blocked<1, 0, 2>("blocked5x4 1 lane/group nt K0", in, out, groups);
  run_blocked<2, 0, 2>("blocked5x4 2 lanes/group nt K0", in, out, groups);
  run_blocked<4, 0, 2>("blocked5x4 4 lanes/group nt K0", in, out, groups);
  run_blocked<1, 16, 2>("blocked5x4 1 lane/group nt K16", in, out, groups);
  run_blocked<2, 16, 2>("blocked5x4 2 lanes/group nt K16", in, out, groups);
  run_blocked<4, 16, 2>("blocked5x4 4 lanes/group nt K16", in, out, groups);
  run_blocked<1, 16, 1>("blocked5x4 1 lane/group sc1 K16", in, out, groups);
  run_blocked<4, 16, 1>("blocked5x4 4 lanes/group sc1 K16", in, out, groups);
  run_blocked<1, 48, 1>("blocked5x4 1 lane/group sc1 K48", in, out, groups);
  run_blocked<4, 48, 1>("blocked5x4 4 lanes/group sc1 K48", in, out, groups);
  // occupancy caps through reserved LDS (160 KB per CU; 4-wave workgroups): waves / SIMD = WGs / CU
  run_blocked<1, 16, 1>("blocked5x4 1 lane/group sc1 K16 occ<=6", in, out, groups, 26 * 1024);
  run_blocked<1, 16, 1>("blocked5x4 1 lane/group sc1 K16 occ<=4", in, out, groups, 40 * 1024);
  run_blocked<1, 16, 1>("blocked5x4 1 lane/group sc1 K16 occ<=3", in, out, groups, 52 * 1024);
  run_blocked<1, 16, 1>("blocked5x4 1 lane/group sc1 K16 occ<=2", in, out, groups, 64 * 1024);
  hipFree(in);
  hipFree(out);
  return 0;
}
