// pacing_probe.hip — why does the SLERP kernel (5 columns in, 4 out, ~60 FLOP per point) stream
// faster than a bare 5-in / 4-out pass?  Adds K dependent FMAs per value between each wave's
// loads and stores (and, separately, an s_sleep) to the bare blocked-layout pass, then times it.
//   hipcc -O3 --offload-arch=gfx950 tools/pacing_probe.hip -o tools/pacing_probe && tools/pacing_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(float* p, v4f v) {
  if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  else __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
}

template <int CI, int K, int SLEEP, int POL, int TFIRST = 0>
__global__ __launch_bounds__(256) void k_pass(const float* __restrict__ in, float* __restrict__ out, long n) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;   // float4 group
  if (4 * g >= n) return;
  const long blk = g >> 6, off = 4 * (g & 63);
  const float* bi = in + blk * CI * 256 + off;
  float* bo = out + blk * 4 * 256 + off;
  v4f v[CI];
#pragma unroll
  for (int j = 0; j < CI; ++j) {
    const int c = TFIRST ? (j + CI - 1) % CI : j;   // TFIRST: the last column is loaded first
    v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
  }
  if constexpr (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
  v4f a = v[CI - 1];
#pragma unroll
  for (int k = 0; k < K; ++k) a = a * 1.0000001f + 0.5f;   // dependent chain on the t column
#pragma unroll
  for (int c = 0; c < 4; ++c) st<POL>(bo + c * 256, v[c] + a);
}

// the deskew kernels' start: a scalar load of the workgroup's tile record, then the data loads at
// addresses taken from it (DEP = 1), vs addresses straight from blockIdx (DEP = 0, as k_pass)
template <typename T>
__device__ __forceinline__ T ldu(const T* p) {
  struct Raw { int v[sizeof(T) / 4]; };
  typedef __attribute__((address_space(4))) const int CI;
  CI* q = (CI*)(p);
  Raw r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) r.v[i] = q[i];
  return __builtin_bit_cast(T, r);
}
struct TileRec { long pstart; int frame; int ngroups; };
template <int CI, int DEP, int POL>
__global__ __launch_bounds__(256) void k_tiled(const float* __restrict__ in, float* __restrict__ out, long n,
                                               const TileRec* __restrict__ tiles, const float4* __restrict__ tbl) {
  long p0 = (long)blockIdx.x * 1024;
  float4 r = make_float4(1.f, 1.f, 1.f, 0.f);
  if constexpr (DEP) {
    const TileRec t = ldu(tiles + blockIdx.x);
    p0 = t.pstart;
    r = ldu(tbl + t.frame);
  }
  const long p = p0 + 4 * threadIdx.x;
  const float* bi = in + ((p >> 8) * CI) * 256 + (p & 255);
  float* bo = out + ((p >> 8) * 4) * 256 + (p & 255);
  v4f v[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
  v4f a = v[CI - 1];
#pragma unroll
  for (int k = 0; k < 32; ++k) a = a * 1.0000001f + 0.5f;
#pragma unroll
  for (int c = 0; c < 4; ++c) st<POL>(bo + c * 256, v[c] * r.x + a + r.w);
}

static size_t g_lds = 0;   // dynamic LDS per workgroup (caps workgroups per CU)
template <typename Kern>
static double time_it(Kern k, const float* in, float* out, long n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(256), g_lds, 0, in, out, n);
  hipEventRecord(e0, 0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), g_lds, 0, in, out, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1e3 / reps;
}

#define RUN(CI, K, S, P, TF, LDS)                                                                          \
  {                                                                                                        \
    g_lds = LDS;                                                                                           \
    const double us = time_it(k_pass<CI, K, S, P, TF>, in, out, n);                                        \
    std::printf("{\"in_cols\": %d, \"fma_chain\": %d, \"sleep\": %d, \"store_pol\": %d, \"t_first\": %d, "  \
                "\"lds\": %d, \"round\": %d, \"us\": %.1f, \"TBs\": %.3f}\n",                               \
                CI, K, S, P, TF, LDS, round, us, (CI * 4.0 + 16.0) * n / (us * 1e-6) / 1e12);              \
    std::fflush(stdout);                                                                                   \
  }

template <typename Kern>
static double time_tiled(Kern k, const float* in, float* out, long n, const TileRec* tiles, const float4* tbl) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, in, out, n, tiles, tbl);
  hipEventRecord(e0, 0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, in, out, n, tiles, tbl);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps;
}

#define RUNT(CI, DEP, P)                                                                                    \
  {                                                                                                         \
    const double us = time_tiled(k_tiled<CI, DEP, P>, in, out, n, tiles, tbl);                              \
    std::printf("{\"tiled\": 1, \"in_cols\": %d, \"dep_lookup\": %d, \"store_pol\": %d, \"round\": %d, "     \
                "\"us\": %.1f, \"TBs\": %.3f}\n", CI, DEP, P, round, us, (CI * 4.0 + 16.0) * n / (us * 1e-6) / 1e12); \
    std::fflush(stdout);                                                                                    \
  }

int main(int argc, char** argv) {
  const long n = 60'000'000 / 1024 * 1024;
  float *in, *out;
  if (hipMalloc(&in, 5 * n * sizeof(float)) != hipSuccess || hipMalloc(&out, 4 * n * sizeof(float)) != hipSuccess)
    return 1;
  hipMemset(in, 0, 5 * n * sizeof(float));
  if (argc > 1) {   // dependent-lookup comparison only
    const int nt = (int)(n / 1024);
    std::vector<TileRec> h(nt);
    for (int i = 0; i < nt; ++i) h[i] = TileRec{(long)i * 1024, i / 100, 256};
    TileRec* tiles;
    float4* tbl;
    hipMalloc(&tiles, nt * sizeof(TileRec));
    hipMalloc(&tbl, (nt / 100 + 1) * sizeof(float4));
    hipMemcpy(tiles, h.data(), nt * sizeof(TileRec), hipMemcpyHostToDevice);
    std::vector<float4> ht(nt / 100 + 1, make_float4(1.f, 1.f, 1.f, 0.f));
    hipMemcpy(tbl, ht.data(), ht.size() * sizeof(float4), hipMemcpyHostToDevice);
    for (int round = 0; round < 3; ++round) {
      RUNT(4, 0, 4) RUNT(4, 1, 4) RUNT(5, 0, 2) RUNT(5, 1, 2) RUNT(5, 0, 1) RUNT(5, 1, 1)
    }
    return 0;
  }
  for (int round = 0; round < 2; ++round) {
    RUN(5, 0, 0, 2, 0, 0) RUN(5, 32, 0, 2, 0, 0) RUN(5, 64, 0, 1, 0, 0)
    RUN(5, 0, 0, 2, 1, 0) RUN(5, 32, 0, 2, 1, 0) RUN(5, 64, 0, 1, 1, 0) RUN(5, 32, 0, 4, 1, 0)
    RUN(5, 0, 0, 2, 0, 40000) RUN(5, 32, 0, 2, 0, 40000) RUN(5, 64, 0, 1, 0, 40000)
    RUN(5, 0, 0, 2, 1, 40000) RUN(5, 32, 0, 2, 1, 40000) RUN(5, 64, 0, 1, 1, 40000) RUN(5, 32, 0, 4, 1, 40000)
    RUN(5, 32, 0, 2, 1, 26000) RUN(5, 32, 0, 2, 1, 20000)
    RUN(4, 32, 0, 4, 0, 0) RUN(4, 32, 0, 4, 1, 0) RUN(4, 32, 0, 4, 0, 40000) RUN(4, 32, 0, 2, 0, 40000)
    RUN(4, 32, 0, 4, 1, 40000)
  }
  hipFree(in);
  hipFree(out);
  return 0;
}
