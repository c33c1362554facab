// gap_probe.hip — what does the per-step pattern around a streaming kernel cost?  A 60 M-point
// 5-in / 4-out blocked pass (the deskew kernel's traffic) is stepped 50 times with:
//   P0  the streaming kernel alone, back to back on one stream;
//   P1  the library's pattern: a small "prep" kernel on a second stream (waiting on the event of
//       the main kernel two steps back), an event, the main stream waiting on it, the main kernel;
//   P2  the prep kernel on the main stream right before the streaming kernel;
//   P3  P1 with the prep launched before the previous step's streaming kernel has finished only in
//       host order (no wait on main_done), i.e. the cheapest cross-stream ordering.
// Per-step time = wall of the 50 steps (events on the main stream) / 50.
//   hipcc -O3 --offload-arch=gfx950 tools/gap_probe.hip -o tools/gap_probe && tools/gap_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream(const float* __restrict__ in, float* __restrict__ out, long n) {
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
}

// a latency-bound prep: 150 blocks, a short dependent chain of loads per lane, one store per lane
__global__ __launch_bounds__(256) void k_prep(const double* __restrict__ tbl, double* __restrict__ out, int n, int chain) {
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
  const int pn = 1 << 15;
  if (hipMalloc(&in, 5 * n * sizeof(float)) != hipSuccess || hipMalloc(&out, 4 * n * sizeof(float)) != hipSuccess ||
      hipMalloc(&tbl, pn * sizeof(double)) != hipSuccess || hipMalloc(&pout, pn * sizeof(double)) != hipSuccess)
    return 1;
  hipMemset(in, 0, 5 * n * sizeof(float));
  hipMemset(tbl, 0, pn * sizeof(double));
  hipStream_t s, sd;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&sd, hipStreamNonBlocking);
  const unsigned fl = hipEventDisableTiming | hipEventReleaseToDevice;
  hipEvent_t main_done[2], prep_done[2], e0, e1;
  for (int i = 0; i < 2; ++i) {
    hipEventCreateWithFlags(&main_done[i], fl);
    hipEventCreateWithFlags(&prep_done[i], fl);
  }
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)(n / 1024);
  const int steps = 50;
  for (int chain : {4, 16}) {
    for (int round = 0; round < 3; ++round) {
      for (int pat = 0; pat < 4; ++pat) {
        auto step = [&](int it) {
          const int h = it & 1;
          if (pat == 1 || pat == 3) {
            if (pat == 1) hipStreamWaitEvent(sd, main_done[h], 0);
            hipLaunchKernelGGL(k_prep, dim3(pn / 256), dim3(256), 0, sd, tbl, pout, pn, chain);
            hipEventRecord(prep_done[h], sd);
            hipStreamWaitEvent(s, prep_done[h], 0);
          } else if (pat == 2) {
            hipLaunchKernelGGL(k_prep, dim3(pn / 256), dim3(256), 0, s, tbl, pout, pn, chain);
          }
          hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, in, out, n);
          if (pat == 1 || pat == 3) hipEventRecord(main_done[h], s);
        };
        for (int w = 0; w < 5; ++w) step(w);
        hipEventRecord(e0, s);
        for (int it = 0; it < steps; ++it) step(it);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("{\"pattern\": %d, \"prep_chain\": %d, \"round\": %d, \"step_us\": %.1f}\n", pat, chain, round,
                    ms * 1e3 / steps);
        std::fflush(stdout);
      }
    }
  }
  // P4 / P5: the P1 / P2 step sequence captured once as a hipGraph of `steps` steps and replayed
  // (the prep of step i+1 is a graph branch parallel to step i's streaming kernel in P4)
  for (int pat : {4, 5}) {
    for (int round = 0; round < 3; ++round) {
      hipGraph_t graph;
      hipGraphExec_t exec;
      hipEvent_t fork, join;
      hipEventCreateWithFlags(&fork, hipEventDisableTiming);
      hipEventCreateWithFlags(&join, hipEventDisableTiming);
      hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
      if (pat == 4) {
        hipEventRecord(fork, s);
        hipStreamWaitEvent(sd, fork, 0);
      }
      for (int it = 0; it < steps; ++it) {
        const int h = it & 1;
        if (pat == 4) {
          if (it >= 2) hipStreamWaitEvent(sd, main_done[h], 0);
          hipLaunchKernelGGL(k_prep, dim3(pn / 256), dim3(256), 0, sd, tbl, pout, pn, 16);
          hipEventRecord(prep_done[h], sd);
          hipStreamWaitEvent(s, prep_done[h], 0);
        } else {
          hipLaunchKernelGGL(k_prep, dim3(pn / 256), dim3(256), 0, s, tbl, pout, pn, 16);
        }
        hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, in, out, n);
        if (pat == 4) hipEventRecord(main_done[h], s);
      }
      if (pat == 4) {
        hipEventRecord(join, sd);
        hipStreamWaitEvent(s, join, 0);
      }
      if (hipStreamEndCapture(s, &graph) != hipSuccess ||
          hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) {
        std::printf("{\"pattern\": %d, \"error\": \"capture/instantiate failed\"}\n", pat);
        return 2;
      }
      hipGraphLaunch(exec, s);   // warm
      hipStreamSynchronize(s);
      hipEventRecord(e0, s);
      hipGraphLaunch(exec, s);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float gms = 0;
      hipEventElapsedTime(&gms, e0, e1);
      std::printf("{\"pattern\": %d, \"graph\": true, \"prep_chain\": 16, \"round\": %d, \"step_us\": %.1f}\n", pat,
                  round, gms * 1e3 / steps);
      std::fflush(stdout);
      hipGraphExecDestroy(exec);
      hipGraphDestroy(graph);
      hipEventDestroy(fork);
      hipEventDestroy(join);
    }
  }
  // the prep kernel alone
  hipEventRecord(e0, s);
  for (int it = 0; it < steps; ++it) hipLaunchKernelGGL(k_prep, dim3(pn / 256), dim3(256), 0, s, tbl, pout, pn, 16);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::printf("{\"prep_alone_us\": %.1f}\n", ms * 1e3 / steps);
  // the streaming kernel alone: per launch (an event pair around every launch, serialised by a
  // host sync) vs back to back (one event pair around `steps` launches) -> the kernel-to-kernel gap
  for (int round = 0; round < 3; ++round) {
    double one = 0.0;
    for (int it = 0; it < 20; ++it) {
      hipEventRecord(e0, s);
      hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, in, out, n);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      one += ms * 1e3 / 20;
    }
    hipEventRecord(e0, s);
    for (int it = 0; it < steps; ++it) hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, s, in, out, n);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    std::printf("{\"round\": %d, \"kernel_alone_us\": %.1f, \"back_to_back_step_us\": %.1f}\n", round, one,
                ms * 1e3 / steps);
    std::fflush(stdout);
  }
  return 0;
}
