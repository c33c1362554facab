// anyorder_probe.hip — can the per-step prep run on the kernel's own queue without a kernel
// boundary of its own?  The AQL packet of a kernel launched with hipExtAnyOrderLaunch has its
// barrier bit clear: the packet processor may start it while earlier packets still run, and the
// next ordinary packet (barrier bit set) still waits for it.  A 60 M-point 5-in / 4-out blocked
// pass (the deskew kernel's traffic) is stepped 50 times with:
//   A0  the streaming kernel alone, back to back on one stream;
//   A1  a small latency-bound "prep" kernel, then the streaming kernel, both ordinary packets;
//   A2  the prep with hipExtAnyOrderLaunch, then the streaming kernel (ordinary);
//   A3  A2 with hipExtLaunchKernel start/stop events on every 5th streaming kernel (the bench's
//       sampled kernel timing without extra marker packets);
//   A4  A1 with those events (a baseline for what A3 costs).
// Per-step time = wall of the 50 steps (events on the stream) / 50.  The overlap check stamps
// the prep's first wave start and the previous streaming kernel's last wave end (s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 tools/anyorder_probe.hip -o tools/anyorder_probe && tools/anyorder_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream(const float* __restrict__ in, float* __restrict__ out, long n,
                                                unsigned long long* end_clk) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (4 * g >= n) return;
  const long blk = g >> 6, off = 4 * (g & 63);
  const float* bi = in + blk * 5 * 256 + off;
  float* bo = out + blk * 4 * 256 + off;
  v4f v[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) v[c] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(bi + c * 256));
#pragma unroll
  for (int c = 0; c < 4; ++c) __builtin_nontemporal_store(v[c] * 1.0001f + v[4], reinterpret_cast<v4f*>(bo + c * 256));
  if (end_clk && (threadIdx.x & 63) == 0) atomicMax(end_clk, (unsigned long long)wall_clock64());
}

// latency-bound prep: a short dependent chain of loads per lane, one store per lane
__global__ __launch_bounds__(256) void k_prep(const double* __restrict__ tbl, double* __restrict__ out, int n, int chain,
                                              unsigned long long* start_clk) {
  if (start_clk && threadIdx.x == 0) atomicMin(start_clk, (unsigned long long)wall_clock64());
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int k = i;
  double acc = 0.0;
  for (int j = 0; j < chain; ++j) {
    acc += tbl[k];
    k = ((int)acc * 7 + k * 13 + j) & (n - 1);
  }
  out[i] = acc;
}

int main() {
  const long n = 60'000'000 / 1024 * 1024;
  float *in, *out;
  double *tbl, *pout;
  unsigned long long* clk;
  const int pn = 600 * 64;   // one wave per frame of a 600-frame batch
  if (hipMalloc(&in, 5 * n * sizeof(float)) != hipSuccess || hipMalloc(&out, 4 * n * sizeof(float)) != hipSuccess ||
      hipMalloc(&tbl, 65536 * sizeof(double)) != hipSuccess || hipMalloc(&pout, pn * sizeof(double)) != hipSuccess ||
      hipMalloc(&clk, 2 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  hipMemset(in, 0, 5 * n * sizeof(float));
  hipMemset(tbl, 0, 65536 * sizeof(double));
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEvent_t ks[10], ke[10];
  for (int i = 0; i < 10; ++i) {
    hipEventCreate(&ks[i]);
    hipEventCreate(&ke[i]);
  }
  const int grid = (int)(n / 1024);
  const int steps = 50;
  const int chain = 16;
  for (int round = 0; round < 3; ++round) {
    for (int pat = 0; pat < 5; ++pat) {
      int nk = 0;
      auto step = [&](int it, bool timed) {
        if (pat >= 1) {
          const unsigned fl = (pat == 2 || pat == 3) ? hipExtAnyOrderLaunch : 0;
          hipExtLaunchKernelGGL(k_prep, dim3((pn + 255) / 256), dim3(256), 0, s, nullptr, nullptr, fl, tbl, pout, pn,
                                chain, (unsigned long long*)nullptr);
        }
        const bool ev = timed && (pat == 3 || pat == 4) && it % 5 == 2 && nk < 10;
        hipExtLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, ev ? ks[nk] : nullptr, ev ? ke[nk] : nullptr, 0u,
                              (const float*)in, out, n, (unsigned long long*)nullptr);
        if (ev) ++nk;
      };
      for (int w = 0; w < 5; ++w) step(w, false);
      hipEventRecord(e0, s);
      for (int it = 0; it < steps; ++it) step(it, true);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      double kus = 0.0;
      for (int i = 0; i < nk; ++i) {
        float k = 0;
        if (hipEventElapsedTime(&k, ks[i], ke[i]) != hipSuccess) k = -1.f;
        kus += k * 1e3 / nk;
      }
      std::printf("{\"pattern\": \"A%d\", \"round\": %d, \"step_us\": %.2f, \"ext_event_kernel_us\": %.2f, \"ext_events\": %d}\n",
                  pat, round, ms * 1e3 / steps, kus, nk);
      std::fflush(stdout);
    }
  }
  // overlap check: stream(i) ; prep (any-order or not) ; stream(i+1)
  for (int any = 0; any < 2; ++any) {
    for (int round = 0; round < 3; ++round) {
      unsigned long long h[2] = {~0ull, 0ull};
      hipMemcpy(clk, h, sizeof(h), hipMemcpyHostToDevice);   // [0] prep start (min), [1] stream end (max)
      hipExtLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, nullptr, nullptr, 0u, (const float*)in, out, n,
                            clk + 1);
      hipExtLaunchKernelGGL(k_prep, dim3((pn + 255) / 256), dim3(256), 0, s, nullptr, nullptr,
                            any ? (unsigned)hipExtAnyOrderLaunch : 0u, tbl, pout, pn, chain, clk);
      hipExtLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, nullptr, nullptr, 0u, (const float*)in, out, n,
                            (unsigned long long*)nullptr);
      hipStreamSynchronize(s);
      hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
      int khz = 0;
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
      const double us = ((double)(long long)(h[0] - h[1])) / (khz * 1e-3);
      std::printf("{\"overlap_check\": true, \"any_order\": %d, \"round\": %d, \"prep_start_minus_stream_end_us\": %.2f}\n",
                  any, round, us);
      std::fflush(stdout);
    }
  }
  return 0;
}
