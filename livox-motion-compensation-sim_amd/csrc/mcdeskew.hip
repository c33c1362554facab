// mcdeskew.hip — host side of the C-ABI declared in include/mcdeskew.h.
//
// Owns the per-context HIP stream, the device copies of the pose sources (trajectory / IMU),
// the padded-CSR batches and the launch of the kernels in kernels.hpp.  No torch, no numpy:
// plain pointers and sizes in, status codes out (thread-local message in mc_last_error()).
#include "../../include/mcdeskew.h"
#include "kernels.hpp"
#include <hip/hip_ext.h>
#include "scan.hpp"
#include "internal.hpp"
#include "hostutil.hpp"
#include "plan.hpp"
#include "rot.hpp"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

using namespace mc;

namespace mcimpl {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace mcimpl
static int launch_grid(const mc_ctx* c, int32_t n_tiles) {
  int g = n_tiles;
  if (c->max_grid > 0 && g > c->max_grid) g = c->max_grid;
  return g < 1 ? 1 : g;
}

static_assert(mcimpl::kBatchBlock == kBlkPts && mcplan::kBlk == kBlkPts, "batch block size");

// workgroups of a stager launch over n_tiles tiles (256-point units; ld: AoS columns)
static int32_t stage_units(int32_t n_tiles, int64_t ld) { return ld == 4 ? n_tiles * kStageQuarters : n_tiles; }
// ... of the SoA -> AoS launch
static int32_t fetch_units(int32_t n_tiles) { return n_tiles * kStageQuarters; }
static_assert(sizeof(mcplan::TileRec) == sizeof(Tile) && offsetof(mcplan::TileRec, frame) == offsetof(Tile, frame) &&
                  offsetof(mcplan::TileRec, ngroups) == offsetof(Tile, ngroups),
              "host tile records are uploaded as mc::Tile");

static LayoutArgs layout_of(const mc_batch* b) {
  LayoutArgs a;
  a.tiles = b->d_tiles; a.n_tiles = b->n_tiles;
  a.poff = b->d_poff; a.doff = b->d_doff; a.counts = b->d_counts;
  a.cols = b->d_cols; a.C = b->C;
  a.dbase = 0;
  a.pcd_len = nullptr;
  return a;
}

template <typename T>
static int upload_column(mc_batch* b, const T* src, int col) {
  mc_ctx* c = b->ctx;
  void* st = nullptr;
  if (int r = ctx_stage(c, (size_t)b->N * sizeof(T), &st)) return r;
  HIPCHK(hipMemcpyAsync(st, src, (size_t)b->N * sizeof(T), hipMemcpyHostToDevice, c->stream));
  if (col < 4) b->wrote(false);
  hipLaunchKernelGGL((k_column<T, 0>), dim3(launch_grid(c, b->n_tiles)), dim3(kBlock), 0, c->stream,
                     layout_of(b), col, static_cast<const T*>(st), static_cast<T*>(nullptr));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}
template <typename T>
static int download_column(mc_batch* b, int col, T* dst) {
  mc_ctx* c = b->ctx;
  void* st = nullptr;
  if (int r = ctx_stage(c, (size_t)b->N * sizeof(T), &st)) return r;
  hipLaunchKernelGGL((k_column<T, 1>), dim3(launch_grid(c, b->n_tiles)), dim3(kBlock), 0, c->stream,
                     layout_of(b), col, static_cast<const T*>(nullptr), static_cast<T*>(st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(dst, st, (size_t)b->N * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

// per-frame t_ns span, recomputed whenever the t column is written (staging time, not per step)
static int compute_trange(mc_batch* b) {
  mc_ctx* c = b->ctx;
  if (b->F == 0 || !b->has_t()) { b->trange_valid = true; return MC_OK; }
  hipLaunchKernelGGL(k_trange_init, dim3((b->F + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, b->d_trange, b->F);
  if (b->n_tiles > 0)
    hipLaunchKernelGGL(k_trange, dim3(launch_grid(c, b->n_tiles)), dim3(kBlock), 0, c->stream, layout_of(b),
                       b->d_trange, b->d_strange);
  HIPCHK(hipGetLastError());
  b->trange_valid = true;
  ++b->prep_ver;
  return MC_OK;
}

// ------------------------------------------------------------------------------------------------
extern "C" {

int mc_abi_version(void) { return MC_ABI_VERSION; }

const char* mc_last_error(void) { return mcimpl::g_err.c_str(); }

int mc_device_count(int* count) {
  CHECK_ARG(count, "count is NULL");
  *count = 0;
  HIPCHK(hipGetDeviceCount(count));
  return MC_OK;
}

int mc_device_pci_bus_id(int device, char* out, int len) {
  CHECK_ARG(out && len >= 16, "output buffer needs >= 16 bytes");
  HIPCHK(hipDeviceGetPCIBusId(out, len, device));
  return MC_OK;
}

// launch-span pool (DeskewArgs::span): slots of 1 + kSpanTail wall-clock stamps
constexpr int32_t kSpanSlots = 64;
constexpr size_t kSpanWords = 1 + kSpanTail;

int mc_create(int device, mc_ctx** out) {
  CHECK_ARG(out, "out is NULL");
  *out = nullptr;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  CHECK_ARG(device >= 0 && device < n, "device %d out of range (%d visible)", device, n);
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MC_ERR_STATE, "device %d is %s; this library is built for gfx950 (MI355X) only",
                device, prop.gcnArchName);
  mc_ctx* c = new mc_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    // stream-ordering events between two queues of the same device: device-scope release only
    const unsigned fl = hipEventDisableTiming | hipEventReleaseToDevice;
    e = hipEventCreateWithFlags(&c->ev_main_done[i], fl);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_prep_done[i], fl);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming | hipEventReleaseToDevice);
  // the launch-span pool (span_take), zeroed
  if (e == hipSuccess) e = hipMalloc(&c->d_span, kSpanSlots * kSpanWords * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->d_span, 0, kSpanSlots * kSpanWords * sizeof(unsigned long long));
  if (e != hipSuccess) {
    if (c->d_span) (void)hipFree(c->d_span);
    delete c;
    return fail(MC_ERR_HIP, "stream/event creation: %s", hipGetErrorString(e));
  }
  *out = c;
  return MC_OK;
}

int mc_destroy(mc_ctx* c) {
  if (!c) return MC_OK;
  DeviceGuard g(c->device);
  (void)sync_all(c);
  dev_free(c->d_time); dev_free(c->d_pos); dev_free(c->d_rpy); dev_free(c->d_pose_seg);
  dev_free(c->d_imu_ts); dev_free(c->d_gyro); dev_free(c->d_imu_seg);
  dev_free(c->d_env); dev_free(c->d_scan_pose); dev_free(c->d_scan_tcount);
  dev_free(c->d_scan_toff); dev_free(c->d_scan_nvis); dev_free(c->d_scan_bits);
  if (c->d_codec) (void)hipFree(c->d_codec);
  if (c->d_span) (void)hipFree(c->d_span);
  dev_free(c->d_codec_err);
  dev_free(c->d_pcd_len);
  if (c->d_seg64) (void)hipFree(c->d_seg64);
  if (c->h_pin) (void)hipHostFree(c->h_pin);
  if (c->h_pipe) (void)hipHostFree(c->h_pipe);
  if (c->d_pipe) (void)hipFree(c->d_pipe);
  for (auto& p : c->codec_ev) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  if (c->d_stage) (void)hipFree(c->d_stage);
  for (auto& p : c->main_ev) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  for (auto& p : c->scan_ev) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  for (auto& p : c->prep_ev) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  for (auto& p : c->layout_ev) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; ++i) { (void)hipEventDestroy(c->ev_main_done[i]); (void)hipEventDestroy(c->ev_prep_done[i]); }
  (void)hipEventDestroy(c->ev_order);
  (void)hipStreamDestroy(c->side);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return MC_OK;
}

int mc_sync(mc_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  DeviceGuard g(c->device);
  return sync_all(c);
}

int mc_set_launch(mc_ctx* c, int32_t max_grid) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(max_grid >= 0, "max_grid must be >= 0");
  c->max_grid = max_grid;
  return MC_OK;
}

// ---- pose sources -------------------------------------------------------------------------
int mc_set_trajectory(mc_ctx* c, int64_t T, const double* time, const double* pos, const double* rpy) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(T >= 1, "trajectory needs at least one pose (got %lld)", (long long)T);
  CHECK_ARG(time && pos && rpy, "trajectory arrays must not be NULL");
  for (int64_t i = 1; i < T; ++i)
    CHECK_ARG(time[i] >= time[i - 1], "trajectory time must be non-decreasing (index %lld)", (long long)i);
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  ++c->traj_ver;   // before anything changes (a failed upload must not leave a matching key)
  if (T > c->T_cap) {
    dev_free(c->d_time); dev_free(c->d_pos); dev_free(c->d_rpy); dev_free(c->d_pose_seg);
    c->T_cap = 0;
    if (int r = dev_alloc(&c->d_time, T)) return r;
    if (int r = dev_alloc(&c->d_pos, 3 * T)) return r;
    if (int r = dev_alloc(&c->d_rpy, 3 * T)) return r;
    if (int r = dev_alloc(&c->d_pose_seg, 2 * T)) return r;
    c->T_cap = T;
  }
  HIPCHK(hipMemcpyAsync(c->d_time, time, T * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_pos, pos, 3 * T * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_rpy, rpy, 3 * T * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->h_time.assign(time, time + T);
  c->h_pos.assign(pos, pos + 3 * T);
  c->h_rpy.assign(rpy, rpy + 3 * T);
  c->T = T;
  return MC_OK;
}

int mc_set_imu(mc_ctx* c, int64_t M, const int64_t* ts, const double* gyro) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(M >= 1, "IMU table needs at least one sample (got %lld)", (long long)M);
  CHECK_ARG(ts && gyro, "IMU arrays must not be NULL");
  for (int64_t i = 1; i < M; ++i)
    CHECK_ARG(ts[i] >= ts[i - 1], "IMU timestamps must be non-decreasing (index %lld)", (long long)i);
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  ++c->imu_ver;
  if (M > c->M_cap) {
    dev_free(c->d_imu_ts); dev_free(c->d_gyro); dev_free(c->d_imu_seg);
    c->M_cap = 0;
    if (int r = dev_alloc(&c->d_imu_ts, M)) return r;
    if (int r = dev_alloc(&c->d_gyro, 3 * M)) return r;
    if (int r = dev_alloc(&c->d_imu_seg, 2 * M)) return r;
    c->M_cap = M;
  }
  HIPCHK(hipMemcpyAsync(c->d_imu_ts, ts, M * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_gyro, gyro, 3 * M * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->M = M;
  return MC_OK;
}

// ---- batches ------------------------------------------------------------------------------
int mc_batch_create(mc_ctx* c, int32_t F, const int64_t* counts, uint32_t flags, mc_batch** out) {
  CHECK_ARG(c && out, "NULL argument");
  *out = nullptr;
  CHECK_ARG(F >= 0, "n_frames must be >= 0");
  CHECK_ARG(F == 0 || counts, "counts is NULL");
  // host-side layout planning (plan.cpp; sanitizer-tested on the CPU, tests/test_sanitizers.py)
  mcplan::BatchLayout L;
  const std::string perr = mcplan::plan_batch(counts, F, kTileGroups, kSub, &L);
  if (!perr.empty()) return fail(MC_ERR_INVALID, "%s", perr.c_str());
  mc_batch* b = new mc_batch();
  static std::atomic<uint64_t> next_uid{1};
  b->ctx = c;
  b->uid = next_uid.fetch_add(1);
  b->F = F;
  b->counts.assign(counts, counts + F);
  b->poff = std::move(L.poff);
  b->doff = std::move(L.doff);
  b->ftile = std::move(L.ftile);
  const std::vector<mcplan::TileRec>& tiles = L.tiles;
  const std::vector<int32_t>& ftile = b->ftile;
  b->N = b->doff[F];
  b->P = b->poff[F];
  b->C = (flags & MC_BATCH_WITH_TIME) ? 5 : 4;
  const size_t col_vals = (size_t)b->C * (size_t)std::max<int64_t>(b->P, kBlkPts);
  b->n_tiles = (int32_t)tiles.size();
  DeviceGuard g(c->device);
  int r = MC_OK;
  auto bail = [&](int code) { mc_batch_destroy(b); return code; };
  if ((r = dev_alloc(&b->d_cols, col_vals))) return bail(r);
  if ((r = dev_alloc(&b->d_counts, F + 1))) return bail(r);
  if ((r = dev_alloc(&b->d_poff, F + 1))) return bail(r);
  if ((r = dev_alloc(&b->d_doff, F + 1))) return bail(r);
  if ((r = dev_alloc(&b->d_tiles, tiles.size()))) return bail(r);
  if ((r = dev_alloc(&b->d_frame_time, F))) return bail(r);
  if ((r = dev_alloc(&b->d_frame_start, F))) return bail(r);
  // k_prep outputs: two halves (double buffer, see mc_deskew)
  if ((r = dev_alloc(&b->d_frame_tbl, 2 * 3 * (size_t)F))) return bail(r);
  if ((r = dev_alloc(&b->d_trange, F))) return bail(r);
  if ((r = dev_alloc(&b->d_fwin, 2 * (size_t)F))) return bail(r);
  b->frec_half = 2 * (size_t)std::max<int>(F, 1) * std::max(sizeof(PoseWin), sizeof(ImuSeg));
  if ((r = dev_alloc(reinterpret_cast<char**>(&b->d_frec), 2 * b->frec_half))) return bail(r);
  const size_t n_sub = std::max<size_t>(tiles.size(), 1) * kSub;
  if (b->has_t()) {
    if ((r = dev_alloc(&b->d_ftile, F + 1))) return bail(r);
    if ((r = dev_alloc(&b->d_strange, n_sub))) return bail(r);
    if ((r = dev_alloc(&b->d_swin, 2 * n_sub))) return bail(r);
  }
  if ((r = dev_alloc(&b->d_partial, 5 * (size_t)b->n_tiles))) return bail(r);
  if ((flags & MC_BATCH_WITH_PCD_LEN) && (r = dev_alloc(&b->d_pcd_len, std::max<int64_t>(b->P / kBlkPts, 1))))
    return bail(r);
  hipStream_t s = c->stream;
  auto cpy = [&](void* d, const void* h, size_t n) { return hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s); };
  if (F > 0) {
    if (cpy(b->d_counts, b->counts.data(), F * sizeof(int64_t)) != hipSuccess ||
        cpy(b->d_poff, b->poff.data(), (F + 1) * sizeof(int64_t)) != hipSuccess ||
        cpy(b->d_doff, b->doff.data(), (F + 1) * sizeof(int64_t)) != hipSuccess)
      return bail(fail(MC_ERR_HIP, "batch metadata upload failed"));
    if (!tiles.empty() && cpy(b->d_tiles, tiles.data(), tiles.size() * sizeof(Tile)) != hipSuccess)
      return bail(fail(MC_ERR_HIP, "tile table upload failed"));
    if (b->d_ftile && cpy(b->d_ftile, ftile.data(), (F + 1) * sizeof(int32_t)) != hipSuccess)
      return bail(fail(MC_ERR_HIP, "frame tile table upload failed"));
  }
  // zero the columns so padding slots are defined even before the first upload
  if (hipMemsetAsync(b->d_cols, 0, col_vals * sizeof(float), s) != hipSuccess)
    return bail(fail(MC_ERR_HIP, "memset failed"));
  if (hipStreamSynchronize(s) != hipSuccess) return bail(fail(MC_ERR_HIP, "sync failed"));
  *out = b;
  return MC_OK;
}

int mc_batch_destroy(mc_batch* b) {
  if (!b) return MC_OK;
  DeviceGuard g(b->ctx->device);
  (void)sync_all(b->ctx);
  dev_free(b->d_cols); dev_free(b->d_counts); dev_free(b->d_poff); dev_free(b->d_doff);
  dev_free(b->d_tiles); dev_free(b->d_frame_time); dev_free(b->d_frame_start); dev_free(b->d_frame_tbl);
  dev_free(b->d_trange); dev_free(b->d_fwin); dev_free(b->d_partial);
  if (b->d_frec) (void)hipFree(b->d_frec);
  b->d_frec = nullptr;
  dev_free(b->d_ftile); dev_free(b->d_strange); dev_free(b->d_swin);
  dev_free(b->d_pcd_len);
  delete b;
  return MC_OK;
}

int mc_batch_info(const mc_batch* b, int64_t* n, int64_t* padded, int32_t* F, int32_t* n_tiles) {
  CHECK_ARG(b, "batch is NULL");
  if (n) *n = b->N;
  if (padded) *padded = b->P;
  if (F) *F = b->F;
  if (n_tiles) *n_tiles = b->n_tiles;
  return MC_OK;
}

int mc_batch_padded_offsets(const mc_batch* b, int64_t* poff) {
  CHECK_ARG(b && poff, "NULL argument");
  std::memcpy(poff, b->poff.data(), (b->F + 1) * sizeof(int64_t));
  return MC_OK;
}

int mc_batch_pcd_len_current(const mc_batch* b, int32_t* current) {
  CHECK_ARG(b && current, "NULL argument");
  *current = b->pcd_current() ? 1 : 0;
  return MC_OK;
}

int mc_batch_set_frame_times(mc_batch* b, const double* t) {
  CHECK_ARG(b, "batch is NULL");
  CHECK_ARG(b->F == 0 || t, "frame times are NULL");
  DeviceGuard g(b->ctx->device);
  if (b->F) {
    HIPCHK(hipMemcpyAsync(b->d_frame_time, t, b->F * sizeof(double), hipMemcpyHostToDevice, b->ctx->stream));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
  }
  b->has_times = true;
  ++b->prep_ver;
  return MC_OK;
}

int mc_batch_set_frame_start_ns(mc_batch* b, const int64_t* s) {
  CHECK_ARG(b, "batch is NULL");
  CHECK_ARG(b->F == 0 || s, "frame starts are NULL");
  DeviceGuard g(b->ctx->device);
  if (b->F) {
    HIPCHK(hipMemcpyAsync(b->d_frame_start, s, b->F * sizeof(int64_t), hipMemcpyHostToDevice, b->ctx->stream));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
  }
  b->has_starts = true;
  ++b->prep_ver;
  return MC_OK;
}

// Work this context queues on its stream and leaves running when the call returns must keep the next
// mc_deskew's prep from being issued any-order: that prep may only overtake this
// context's own deskew kernel.  Every API that returns with work in flight calls this.
static inline void queued_async(mc_ctx* c) { c->prep_fence = true; }

// device AoS -> batch columns (async, timed as a layout kernel)
static int launch_stage(mc_batch* b, const double* d_aos, int64_t ld) {
  mc_ctx* c = b->ctx;
  if (b->n_tiles == 0) return MC_OK;
  queued_async(c);
  LayoutArgs a = layout_of(b);
  a.pcd_len = b->d_pcd_len;   // MC_BATCH_WITH_PCD_LEN: the stager sums each block's text bytes
  {
    TimedRegion tr(c, &c->layout_ev, c->stream);
    hipLaunchKernelGGL(k_aos_to_soa, dim3(launch_grid(c, stage_units(b->n_tiles, ld))), dim3(kBlock), 0, c->stream,
                       a, d_aos, ld);
  }
  b->wrote(false);
  HIPCHK(hipGetLastError());
  b->wrote(true);
  return MC_OK;
}
// batch columns -> device AoS (N,4) f64 (async, timed as a layout kernel)
static int launch_fetch(mc_batch* b, double* d_aos) {
  mc_ctx* c = b->ctx;
  if (b->n_tiles == 0) return MC_OK;
  queued_async(c);
  {
    TimedRegion tr(c, &c->layout_ev, c->stream);
    hipLaunchKernelGGL(k_soa_to_aos, dim3(launch_grid(c, fetch_units(b->n_tiles))), dim3(kBlock), 0, c->stream,
                       layout_of(b), d_aos);
  }
  HIPCHK(hipGetLastError());
  return MC_OK;
}

int mc_batch_upload_aos_f64(mc_batch* b, const double* aos, int64_t ld) {
  CHECK_ARG(b, "batch is NULL");
  if (ld < 4) return fail(MC_ERR_INDEX, "points need at least 4 columns (x,y,z,intensity); got %lld", (long long)ld);
  if (b->N == 0) return MC_OK;
  CHECK_ARG(aos, "points pointer is NULL");
  mc_ctx* c = b->ctx;
  DeviceGuard g(c->device);
  void* st = nullptr;
  if (int r = ctx_stage(c, (size_t)b->N * ld * sizeof(double), &st)) return r;
  HIPCHK(hipMemcpyAsync(st, aos, (size_t)b->N * ld * sizeof(double), hipMemcpyHostToDevice, c->stream));
  if (int r = launch_stage(b, static_cast<const double*>(st), ld)) return r;
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_batch_stage_aos_f64_device(mc_batch* b, const double* d_aos, int64_t ld) {
  CHECK_ARG(b, "batch is NULL");
  if (ld < 4) return fail(MC_ERR_INDEX, "points need at least 4 columns (x,y,z,intensity); got %lld", (long long)ld);
  if (b->N == 0) return MC_OK;
  CHECK_ARG(d_aos, "device points pointer is NULL");
  DeviceGuard g(b->ctx->device);
  return launch_stage(b, d_aos, ld);
}

int mc_batch_fetch_aos_f64_device(mc_batch* b, double* d_aos) {
  CHECK_ARG(b, "batch is NULL");
  if (b->N == 0) return MC_OK;
  CHECK_ARG(d_aos, "device output pointer is NULL");
  DeviceGuard g(b->ctx->device);
  return launch_fetch(b, d_aos);
}

int mc_device_alloc(mc_ctx* c, int64_t bytes, void** dptr) {
  CHECK_ARG(c && dptr, "NULL argument");
  CHECK_ARG(bytes >= 0, "negative size");
  DeviceGuard g(c->device);
  *dptr = nullptr;
  HIPCHK(hipMalloc(dptr, bytes > 0 ? (size_t)bytes : 1));
  return MC_OK;
}

int mc_device_free(mc_ctx* c, void* dptr) {
  CHECK_ARG(c, "ctx is NULL");
  if (!dptr) return MC_OK;
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  HIPCHK(hipFree(dptr));
  return MC_OK;
}

int mc_memcpy_h2d(mc_ctx* c, void* dptr, const void* host, int64_t bytes) {
  CHECK_ARG(c && dptr && host && bytes >= 0, "bad argument");
  DeviceGuard g(c->device);
  HIPCHK(hipMemcpyAsync(dptr, host, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_memcpy_d2h(mc_ctx* c, void* host, const void* dptr, int64_t bytes) {
  CHECK_ARG(c && dptr && host && bytes >= 0, "bad argument");
  DeviceGuard g(c->device);
  HIPCHK(hipMemcpyAsync(host, dptr, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_memcpy_d2d(mc_ctx* c, void* dst, const void* src, int64_t bytes) {
  CHECK_ARG(c && (bytes == 0 || (dst && src)), "NULL argument");
  CHECK_ARG(bytes >= 0, "negative size");
  if (bytes == 0) return MC_OK;
  DeviceGuard g(c->device);
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_batch_upload_columns_f32(mc_batch* b, const float* x, const float* y, const float* z, const float* in) {
  CHECK_ARG(b, "batch is NULL");
  if (b->N == 0) return MC_OK;
  DeviceGuard g(b->ctx->device);
  const float* src[4] = {x, y, z, in};
  for (int k = 0; k < 4; ++k)
    if (src[k])
      if (int r = upload_column<float>(b, src[k], k)) return r;
  return MC_OK;
}

int mc_batch_upload_time_ns(mc_batch* b, const int32_t* t) {
  CHECK_ARG(b, "batch is NULL");
  if (!b->has_t()) return fail(MC_ERR_STATE, "batch was created without MC_BATCH_WITH_TIME");
  if (b->N == 0) return MC_OK;
  CHECK_ARG(t, "t_ns is NULL");
  DeviceGuard g(b->ctx->device);
  if (int r = upload_column<int32_t>(b, t, 4)) return r;
  if (int r = compute_trange(b)) return r;
  HIPCHK(hipStreamSynchronize(b->ctx->stream));
  return MC_OK;
}

int mc_batch_download_aos_f64(mc_batch* b, double* aos) {
  CHECK_ARG(b, "batch is NULL");
  if (b->N == 0) return MC_OK;
  CHECK_ARG(aos, "output pointer is NULL");
  mc_ctx* c = b->ctx;
  DeviceGuard g(c->device);
  void* st = nullptr;
  if (int r = ctx_stage(c, (size_t)b->N * 4 * sizeof(double), &st)) return r;
  if (int r = launch_fetch(b, static_cast<double*>(st))) return r;
  HIPCHK(hipMemcpyAsync(aos, st, (size_t)b->N * 4 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_batch_download_frames_aos_f64(mc_batch* b, int32_t f0, int32_t f1, double* aos) {
  CHECK_ARG(b, "batch is NULL");
  CHECK_ARG(0 <= f0 && f0 <= f1 && f1 <= b->F, "frame range [%d, %d) outside [0, %d)", f0, f1, b->F);
  const int64_t rows = b->doff[f1] - b->doff[f0];
  if (rows == 0) return MC_OK;
  CHECK_ARG(aos, "output pointer is NULL");
  mc_ctx* c = b->ctx;
  DeviceGuard g(c->device);
  void* st = nullptr;
  if (int r = ctx_stage(c, (size_t)rows * 4 * sizeof(double), &st)) return r;
  // the stager over the tiles of frames [f0, f1) only, writing rows from doff[f0] on
  LayoutArgs a = layout_of(b);
  a.tiles = b->d_tiles + b->ftile[f0];
  a.n_tiles = b->ftile[f1] - b->ftile[f0];
  a.dbase = b->doff[f0];
  if (a.n_tiles > 0)
    hipLaunchKernelGGL(k_soa_to_aos, dim3(launch_grid(c, fetch_units(a.n_tiles))), dim3(kBlock), 0, c->stream, a,
                       static_cast<double*>(st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(aos, st, (size_t)rows * 4 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_batch_download_columns_f32(mc_batch* b, float* x, float* y, float* z, float* in) {
  CHECK_ARG(b, "batch is NULL");
  if (b->N == 0) return MC_OK;
  DeviceGuard g(b->ctx->device);
  float* dst[4] = {x, y, z, in};
  for (int k = 0; k < 4; ++k)
    if (dst[k])
      if (int r = download_column<float>(b, k, dst[k])) return r;
  return MC_OK;
}

int mc_batch_download_time_ns(mc_batch* b, int32_t* t) {
  CHECK_ARG(b, "batch is NULL");
  if (!b->has_t()) return fail(MC_ERR_STATE, "batch was created without MC_BATCH_WITH_TIME");
  if (b->N == 0) return MC_OK;
  CHECK_ARG(t, "t_ns is NULL");
  DeviceGuard g(b->ctx->device);
  return download_column<int32_t>(b, 4, t);
}

int mc_batch_synth(mc_batch* b, uint64_t seed, int64_t frame_id_base) {
  CHECK_ARG(b, "batch is NULL");
  if (b->n_tiles == 0) return MC_OK;
  mc_ctx* c = b->ctx;
  DeviceGuard g(c->device);
  b->wrote(false);
  hipLaunchKernelGGL(k_synth, dim3(launch_grid(c, b->n_tiles)), dim3(kBlock), 0, c->stream, layout_of(b), seed,
                     frame_id_base);
  HIPCHK(hipGetLastError());
  if (int r = compute_trange(b)) return r;
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

int mc_batch_checksum(mc_batch* b, double* sums) {
  CHECK_ARG(b && sums, "NULL argument");
  for (int k = 0; k < 5; ++k) sums[k] = 0.0;
  if (b->n_tiles == 0) return MC_OK;
  mc_ctx* c = b->ctx;
  DeviceGuard g(c->device);
  hipLaunchKernelGGL(k_checksum, dim3(launch_grid(c, b->n_tiles)), dim3(kBlock), 0, c->stream, layout_of(b),
                     b->d_partial);
  HIPCHK(hipGetLastError());
  std::vector<double> part(5 * (size_t)b->n_tiles);
  HIPCHK(hipMemcpyAsync(part.data(), b->d_partial, part.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int32_t t = 0; t < b->n_tiles; ++t)
    for (int k = 0; k < 5; ++k) sums[k] += part[5 * (size_t)t + k];
  return MC_OK;
}

// ---- the hot path ---------------------------------------------------------------------------
// How mc_deskew issues a step's k_prep (tools/anyorder_probe.hip, tools/ab.py): on the main stream as
// an any-order packet (hipExtAnyOrderLaunch: AQL barrier bit clear) right behind the previous step's
// deskew kernel, so it runs beside that kernel's tail without a second queue; the deskew kernel after
// it is an ordinary packet and waits for both.  (Rejected in rounds 1-2: the prep on a side stream one
// step ahead with cross-queue events, ~7-10 us per step; serial on the main stream, +2 to +6 us.)
// Identical consecutive calls are speculated (mc_ctx::PrepKey): a call's launch also runs the next
// identical call's prep in its first workgroups (k_deskew_points<MODE, true> / k_deskew_frame_next,
// the same fused launch mc_deskew_steps' pipeline issues; for SLERP step wall 320.2-328.3 vs
// 329.5-329.6 us with the prep as a separate packet, profiles/round3/s19).
namespace {

// Table halves written outside mc_deskew's key bookkeeping: no speculated tables stay valid, and the
// next mc_deskew does not speculate from a key seen before this call.
void forget_speculation(mc_ctx* c) {
  c->spec_valid = false;
  c->last_call = mc_ctx::PrepKey{};
}

int deskew_check(mc_ctx* c, const mc_batch* in, const mc_batch* out, int mode, int pose_select) {
  CHECK_ARG(c && in && out, "NULL argument");
  CHECK_ARG(in->ctx == c && out->ctx == c, "batches belong to another context");
  CHECK_ARG(mode >= MC_MODE_FRAME && mode <= MC_MODE_IMU, "unknown mode %d", mode);
  CHECK_ARG(in->counts == out->counts, "input and output batches have different frame counts");
  if (mode == MC_MODE_FRAME) {
    CHECK_ARG(pose_select == MC_POSE_SEARCHSORTED || pose_select == MC_POSE_DIRECT, "unknown pose_select %d",
              pose_select);
    if (c->T < 1) return fail(MC_ERR_STATE, "no trajectory uploaded (mc_set_trajectory)");
    if (pose_select == MC_POSE_DIRECT && c->T != in->F)
      return fail(MC_ERR_INVALID, "MC_POSE_DIRECT needs one pose per frame (T=%lld, frames=%d)", (long long)c->T,
                  in->F);
    if (pose_select == MC_POSE_SEARCHSORTED && !in->has_times)
      return fail(MC_ERR_STATE, "frame times not set (mc_batch_set_frame_times)");
  } else if (mode == MC_MODE_POSE_SLERP) {
    if (c->T < 1) return fail(MC_ERR_STATE, "no trajectory uploaded (mc_set_trajectory)");
    if (!in->has_times) return fail(MC_ERR_STATE, "frame times not set (mc_batch_set_frame_times)");
    if (!in->has_t()) return fail(MC_ERR_STATE, "input batch has no t_ns column");
  } else {
    if (c->M < 1) return fail(MC_ERR_STATE, "no IMU samples uploaded (mc_set_imu)");
    if (!in->has_starts) return fail(MC_ERR_STATE, "frame start times not set (mc_batch_set_frame_start_ns)");
    if (!in->has_t()) return fail(MC_ERR_STATE, "input batch has no t_ns column");
  }
  return MC_OK;
}

// Everything one step launches, for table half h: k_prep's and the deskew kernel's arguments and
// grids.  Plain old data, zero-filled first, so two plans compare bytewise (the graph cache key).
struct StepPlan {
  PrepArgs pa;
  DeskewArgs da;
  uint32_t prep_blocks;
  uint32_t grid;
  int32_t kernel;   // -1: no deskew launch (no tiles); else the mode
};

constexpr int64_t kSlerpXcdMinPoints = 200000000;

// sub-tile order of a mode's kernel without a tuned choice (MC_XCD_*, kernels.hpp): XCD-contiguous
// for the frame kernel; dealt for IMU and for SLERP below kSlerpXcdMinPoints padded points
int32_t default_order(int mode, int64_t P) {
  if (mode == MC_MODE_FRAME) return MC_XCD_FRAME;
  if (mode == MC_MODE_IMU) return MC_XCD_IMU;
  return (MC_XCD_SLERP || P >= kSlerpXcdMinPoints) ? 1 : 0;
}

void deskew_plan(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, int h, StepPlan* sp) {
  std::memset(sp, 0, sizeof(*sp));
  const mc_batch* pb = in;  // per-frame tables live with the input batch
  FrameRow* frame_tbl = pb->d_frame_tbl + 3 * (size_t)in->F * h;
  FrameWin* fwin = pb->d_fwin + (size_t)in->F * h;
  void* frec = static_cast<char*>(pb->d_frec) + pb->frec_half * h;
  PoseSeg* pose_seg = c->d_pose_seg ? c->d_pose_seg + (size_t)c->T_cap * h : nullptr;
  ImuSeg* imu_seg = c->d_imu_seg ? c->d_imu_seg + (size_t)c->M_cap * h : nullptr;

  PrepArgs& pa = sp->pa;
  pa.mode = mode;
  pa.pose_select = pose_select;
  pa.n_frames = in->F;
  pa.time = c->d_time; pa.pos = c->d_pos; pa.rpy = c->d_rpy; pa.T = c->T;
  pa.imu_ts = c->d_imu_ts; pa.gyro = c->d_gyro; pa.M = c->M;
  pa.frame_time = pb->d_frame_time; pa.frame_start = pb->d_frame_start; pa.trange = pb->d_trange;
  pa.frame_tbl = frame_tbl; pa.pose_seg = pose_seg; pa.imu_seg = imu_seg;
  pa.fwin = fwin; pa.frec = frec;
  FrameWin* swin = pb->d_swin ? pb->d_swin + (size_t)in->n_tiles * kSub * h : nullptr;
  pa.ftile = pb->d_ftile; pa.strange = pb->d_strange; pa.swin = swin;
  // one wave per frame, then one lane per pose segment / IMU sample
  int64_t table = 0;
  if (mode == MC_MODE_POSE_SLERP) { pa.nseg = std::max<int64_t>(c->T - 1, 1); table = pa.nseg; }
  if (mode == MC_MODE_IMU) { pa.nseg = c->M; table = c->M; }
  const int64_t waves = in->F + (table + 63) / 64;
  sp->prep_blocks = (uint32_t)((waves + 3) / 4);
  sp->kernel = -1;
  if (in->n_tiles == 0) return;

  DeskewArgs& da = sp->da;
  da.in = in->d_cols; da.in_C = in->C;
  da.out = out->d_cols; da.out_C = out->C;
  // per-point modes pass the timestamps through (CSIM:1472) when out is another batch with t_ns
  da.copy_t = mode != MC_MODE_FRAME && out != in && out->has_t();
  da.tiles = in->d_tiles; da.n_tiles = in->n_tiles;
  da.fpoff = out->d_poff; da.fcount = out->d_counts;   // (the PCD kernels' valid-point test)
  da.frame_tbl = frame_tbl;
  da.frame_time = pb->d_frame_time; da.frame_start = pb->d_frame_start;
  da.fwin = fwin; da.frec = frec;
  da.swin = swin;
  da.pose_time = c->d_time; da.pose_seg = pose_seg;
  da.imu_ts = c->d_imu_ts; da.imu_seg = imu_seg;
  if (mode == MC_MODE_POSE_SLERP) { da.nseg = pa.nseg; da.ntab = c->T; }
  if (mode == MC_MODE_IMU) { da.nseg = c->M; da.ntab = c->M; }
  // frame mode: one workgroup per tile (2 float4 groups per thread); per-point modes: one per
  // kBlock-group sub-tile (1 group per thread, kSub sub-tiles per tile)
  int32_t units = in->n_tiles * kSub;
  if (mode == MC_MODE_FRAME) units = in->n_tiles * kSub * kQuadUnitsPerSub;   // the quad decomposition
  sp->grid = (uint32_t)launch_grid(c, units);
  sp->kernel = mode;
  da.xcd_order = mcimpl::deskew_order(c, in, mode);
  in->hot_order = out->hot_order = da.xcd_order ? 2 : 0;   // (the deskew kernels run forward)
}


// A span slot for a timed deskew launch (null when the pool is spent: that launch has events only).
// The pool is allocated and zeroed by mc_create: allocating it at the first timed launch idled the
// device for ~11 ms right before the timed steps, and the launches after such a pause run through a
// power transient (SLERP 341 -> 353 -> 327 us, profiles/round4/s15 kernel trace).
unsigned long long* span_take(mc_ctx* c) {
  if (!c->d_span || c->span_used >= kSpanSlots) return nullptr;
  return c->d_span + (size_t)c->span_used++ * kSpanWords;
}

// Launches with optional hipExtLaunchKernel timing events (e0/e1 null: untimed) and AQL flags.
void launch_prep(const StepPlan& sp, hipStream_t sd, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr,
                 unsigned flags = 0) {
  if (!e0 && !flags) hipLaunchKernelGGL(k_prep, dim3(sp.prep_blocks), dim3(kBlock), 0, sd, sp.pa);
  else hipExtLaunchKernelGGL(k_prep, dim3(sp.prep_blocks), dim3(kBlock), 0, sd, e0, e1, flags, sp.pa);
}

void launch_main(const StepPlan& sp, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
  const dim3 grid(sp.grid), block(kBlock);
  if (sp.da.pcd_len) {   // mc_deskew_pcd
    if (sp.kernel == MC_MODE_FRAME) hipExtLaunchKernelGGL(k_deskew_frame_pcd, grid, block, 0, s, e0, e1, 0u, sp.da);
    else if (sp.kernel == MC_MODE_POSE_SLERP)
      hipExtLaunchKernelGGL((k_deskew_points<1, false, true>), grid, block, 0, s, e0, e1, 0u, sp.da, sp.pa, 0u);
    else hipExtLaunchKernelGGL((k_deskew_points<2, false, true>), grid, block, 0, s, e0, e1, 0u, sp.da, sp.pa, 0u);
    return;
  }
  if (!e0) {
    if (sp.kernel == MC_MODE_FRAME) hipLaunchKernelGGL(k_deskew_frame, grid, block, 0, s, sp.da);
    else if (sp.kernel == MC_MODE_POSE_SLERP) hipLaunchKernelGGL((k_deskew_points<1>), grid, block, 0, s, sp.da, sp.pa, 0u);
    else hipLaunchKernelGGL((k_deskew_points<2>), grid, block, 0, s, sp.da, sp.pa, 0u);
    return;
  }
  if (sp.kernel == MC_MODE_FRAME) hipExtLaunchKernelGGL(k_deskew_frame, grid, block, 0, s, e0, e1, 0u, sp.da);
  else if (sp.kernel == MC_MODE_POSE_SLERP)
    hipExtLaunchKernelGGL((k_deskew_points<1>), grid, block, 0, s, e0, e1, 0u, sp.da, sp.pa, 0u);
  else hipExtLaunchKernelGGL((k_deskew_points<2>), grid, block, 0, s, e0, e1, 0u, sp.da, sp.pa, 0u);
}

// This step's deskew (sp) with the NEXT step's prep (nx) in the first workgroups of the same launch
// (k_deskew_points<MODE, true> / k_deskew_frame_next): pre = nx's prep workgroups rounded up to the
// XCD count.  sp reads one table half, nx writes the other.
void launch_fused(const StepPlan& sp, const StepPlan& nx, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const uint32_t pre = (nx.prep_blocks + kXcds - 1) / kXcds * kXcds;
  const dim3 grid(sp.grid + pre), block(kBlock);
  if (sp.kernel == MC_MODE_FRAME)
    hipExtLaunchKernelGGL(k_deskew_frame_next, grid, block, 0, s, e0, e1, 0u, sp.da, nx.pa, pre);
  else if (sp.kernel == MC_MODE_POSE_SLERP)
    hipExtLaunchKernelGGL((k_deskew_points<1, true>), grid, block, 0, s, e0, e1, 0u, sp.da, nx.pa, pre);
  else hipExtLaunchKernelGGL((k_deskew_points<2, true>), grid, block, 0, s, e0, e1, 0u, sp.da, nx.pa, pre);
}

// frame time spans derived lazily from t_ns (queued on the main stream)
int ensure_trange(mc_batch* in, int mode) {
  if (mode != MC_MODE_FRAME && !in->trange_valid) return compute_trange(in);
  return MC_OK;
}
}  // namespace

int mc_deskew(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select) {
  return mcimpl::deskew_call(c, in, out, mode, pose_select, nullptr);
}

}  // extern "C"

// sub-tile order: default_order, or a device-measured choice for this mode and batch size
// (mc_tune_order)
int mcimpl::deskew_order(const mc_ctx* c, const mc_batch* in, int mode) {
  const mc_ctx::OrderTune& ot = c->order_tune[mode];
  return ot.order >= 0 && ot.P == in->P ? ot.order : default_order(mode, in->P);
}

int mcimpl::deskew_call(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t* pcd_len) {
  if (int r = deskew_check(c, in, out, mode, pose_select)) return r;
  if (in->F == 0) return MC_OK;
  if (!pcd_len) pcd_len = out->d_pcd_len;   // MC_BATCH_WITH_PCD_LEN: the *_pcd kernels keep its sums
  out->wrote(false);
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  if (mode != MC_MODE_FRAME && !in->trange_valid) {
    // the spans are queued on the main stream: order the prep after them
    if (int r = ensure_trange(const_cast<mc_batch*>(in), mode)) return r;
    c->prep_fence = true;
  }
  // Per-step tables come in two halves: this step's prep writes half h, which the deskew kernel
  // two calls back read; the previous call's kernel reads the other half.
  const int h = c->buf;
  c->buf ^= 1;
  StepPlan sp;
  deskew_plan(c, in, out, mode, pose_select, h, &sp);
  sp.da.pcd_len = pcd_len;
  // a per-point deskew that carries t_ns into another batch rewrites that batch's time column:
  // its cached [min, max] spans no longer describe it
  if (sp.kernel >= 0 && sp.da.copy_t) out->trange_valid = false;
  // Speculation (see mc_ctx::PrepKey): h is the half the previous call's launch prepared for this
  // key, if it did; then this call needs no k_prep at all.
  const mc_ctx::PrepKey key{in->uid, c->traj_ver, c->imu_ver, in->prep_ver, mode, pose_select};
  const bool hit = c->spec_valid && c->spec_half == h && c->spec_key == key;
  // (the fused next-call launch has no PCD variant: a PCD call never speculates, it may hit)
  const bool speculate = sp.kernel >= 0 && c->last_call == key && !pcd_len;
  c->last_call = key;
  c->spec_valid = false;
  if (!hit) {
    // One queue.  Any-order prep only right behind this context's own deskew
    // kernel (prep_fence clear): the packets before it are then that kernel — still reading the
    // other half — and, before it, work the kernel's barrier already waited for.  Everything else
    // that could precede it either finished before its API call returned (trajectory / IMU / frame
    // tables are uploaded synchronously) or set the fence (t_ns spans queued above, graph replays,
    // a speculative launch whose prep workgroups write this very half).  The deskew kernel's own
    // packet keeps the barrier bit, so it waits for this prep, and anything queued after it waits
    // for both.  With no kernel to follow (no tiles) the prep is ordinary.
    const unsigned fl = (!c->prep_fence && sp.kernel >= 0) ? hipExtAnyOrderLaunch : 0u;
    {
      LaunchEvents ev(c);
      launch_prep(sp, s, ev.e0, ev.e1, fl);
      ev.keep(&c->prep_ev);
    }
    HIPCHK(hipGetLastError());
  }
  if (sp.kernel >= 0) {
    LaunchEvents ev(c);
    if (ev.e0) sp.da.span = span_take(c);
    if (speculate) {
      // this call's deskew with an identical next call's prep in the first workgroups (half h ^ 1,
      // which no queued work reads: the previous kernel read it and has finished before this launch)
      StepPlan nx;
      deskew_plan(c, in, out, mode, pose_select, h ^ 1, &nx);
      launch_fused(sp, nx, s, ev.e0, ev.e1);
      c->spec_valid = true;
      c->spec_half = h ^ 1;
      c->spec_key = key;
    } else {
      launch_main(sp, s, ev.e0, ev.e1);
    }
    ev.keep(&c->main_ev);
    HIPCHK(hipGetLastError());
    out->wrote(pcd_len != nullptr && pcd_len == out->d_pcd_len);
    // after a speculative launch the next prep (on a miss) writes the half its prep workgroups write
    c->prep_fence = speculate;
  } else {
    c->prep_fence = true;
  }
  // No event records here: a marker packet between this kernel and the next step's any-order prep
  // would hold that prep until this kernel completes.  Everything is on one queue, so the stream
  // order is the only ordering the halves need (a graph replay forks its prep branch from s).
  return MC_OK;
}

extern "C" {

namespace {
// The launches of n steps over the two table halves of `plan` (step i reads half i & 1 of plan):
// step 0's k_prep, then n deskew launches of which the first n - 1 carry the next step's prep.
// Every `every`-th step's kernel (and prep) is timed.
// last_pcd: the last step's launch also writes the output blocks' PCD text bytes there (its output is
// what the batch keeps; the launches before it have no PCD variant of the fused next-prep kernel).
void issue_steps(mc_ctx* c, const StepPlan* plan, int mode, int32_t n_steps, int32_t every, int32_t* last_pcd) {
  hipStream_t s = c->stream;
  (void)mode;
  auto sampled = [&](int32_t i) { return every > 0 && i % every == every / 2; };
  for (int32_t i = 0; i < n_steps; ++i) {
    if (i == 0) {
      // any-order right behind this context's own deskew kernel, as in mc_deskew
      const bool ao = !c->prep_fence;
      LaunchEvents ev(c, sampled(i));
      launch_prep(plan[i & 1], s, ev.e0, ev.e1, ao ? hipExtAnyOrderLaunch : 0u);
      ev.keep(&c->prep_ev);
    }
    LaunchEvents ev(c, sampled(i));
    StepPlan sp = plan[i & 1];
    if (ev.e0) sp.da.span = span_take(c);
    if (i + 1 < n_steps) {
      launch_fused(sp, plan[(i + 1) & 1], s, ev.e0, ev.e1);
    } else {
      sp.da.pcd_len = last_pcd;
      launch_main(sp, s, ev.e0, ev.e1);
    }
    ev.keep(&c->main_ev);
  }
}

// n steps as n launches, step i's launch carrying step i+1's prep: one
// standalone k_prep for step 0, then n deskew launches; the kernel boundaries order each prep
// before the step that reads it, as in mc_deskew.  Step i reads half h0 ^ (i & 1).
int deskew_steps_pipelined(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select,
                           int32_t n_steps, int32_t every) {
  forget_speculation(c);
  if (mode != MC_MODE_FRAME && !in->trange_valid) {
    if (int r = ensure_trange(const_cast<mc_batch*>(in), mode)) return r;
    c->prep_fence = true;
  }
  const int h0 = c->buf;
  StepPlan plan[2];
  deskew_plan(c, in, out, mode, pose_select, h0, &plan[0]);
  deskew_plan(c, in, out, mode, pose_select, h0 ^ 1, &plan[1]);
  if (plan[0].da.copy_t) out->trange_valid = false;
  out->wrote(false);
  issue_steps(c, plan, mode, n_steps, every, plan[0].kernel >= 0 ? out->d_pcd_len : nullptr);
  HIPCHK(hipGetLastError());
  if (plan[0].kernel >= 0 && n_steps > 0) out->wrote(true);
  c->buf = h0 ^ (n_steps & 1);   // the half the last launch did not read
  c->prep_fence = false;
  return MC_OK;
}
}  // namespace

// Which sub-tile order streams faster depends on the device, not only on the kernel: with the float64
// math the dealt order measured 318-370 us for the same SLERP step on different MI355X boxes, the
// XCD-contiguous one 327-347 us (profiles/round3/s04-s13).  The candidates run back to back, rounds
// alternating between them (drift hits both), each round after a few untimed launches of its own
// order (a kernel's speed depends on what the previous one left in the caches, profiles/round3/s09
// pingpong); the median per-launch time decides.
int mc_tune_order(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t launches,
                  int32_t rounds, double* us_out, int32_t* chosen) {
  if (int r = deskew_check(c, in, out, mode, pose_select)) return r;
  CHECK_ARG(out != in, "mc_tune_order runs the kernel repeatedly: it needs an output batch other than the input");
  CHECK_ARG(launches >= 1 && launches <= 1000 && rounds >= 1 && rounds <= 100, "launches / rounds out of range");
  c->order_tune[mode] = mc_ctx::OrderTune{};
  if (in->n_tiles == 0) {
    if (us_out) us_out[0] = us_out[1] = 0.0;
    if (chosen) *chosen = -1;
    return MC_OK;
  }
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  if (int r = ensure_trange(const_cast<mc_batch*>(in), mode)) return r;
  forget_speculation(c);
  // the candidates run as the steps of mc_deskew_steps do (issue_steps: fused next-step launches)
  const int h0 = c->buf;
  StepPlan plan[2];
  deskew_plan(c, in, out, mode, pose_select, h0, &plan[0]);
  deskew_plan(c, in, out, mode, pose_select, h0 ^ 1, &plan[1]);
  if (plan[0].da.copy_t) out->trange_valid = false;
  out->wrote(false);      // plain kernels only: any PCD text sums of out go stale
  c->prep_fence = true;   // the first prep is an ordinary packet: waits for everything queued before it
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPCHK(hipEventCreate(&e0));
  if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return fail(MC_ERR_HIP, "event create"); }
  std::vector<double> t[2];
  hipError_t e = hipSuccess;
  const bool timing = c->timing;
  c->timing = false;
  for (int32_t r = 0; r < rounds && e == hipSuccess; ++r)
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
      const int cand = (r & 1) ? 1 - k : k;
      plan[0].da.xcd_order = plan[1].da.xcd_order = cand;
      // the previous round's last launch may read either half (odd `launches`): the warm-up's first
      // prep is an ordinary packet, so it waits for that launch
      c->prep_fence = true;
      issue_steps(c, plan, mode, 2, 0, nullptr);   // untimed: this order's own steady state
      c->prep_fence = false;
      e = hipEventRecord(e0, s);
      issue_steps(c, plan, mode, launches, 0, nullptr);
      if (e == hipSuccess) e = hipEventRecord(e1, s);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      float ms = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
      t[cand].push_back(1e3 * ms / launches);
    }
  c->timing = timing;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (e != hipSuccess) return fail(MC_ERR_HIP, "tune_order: %s", hipGetErrorString(e));
  double med[2];
  for (int k = 0; k < 2; ++k) {
    std::sort(t[k].begin(), t[k].end());
    med[k] = t[k][t[k].size() / 2];
  }
  // the other order replaces the mode's default only when it is at least kTuneMargin faster: closer
  // than that the two are within the tuner's noise, and the default is the order that measured best
  // across boxes (profiles/round4/s26: frame dealt 303.5 vs XCD 305.9 us in the tuner, then 314.3 us
  // in the timed steps, where XCD ran 297.9 us on the box of s21)
  constexpr double kTuneMargin = 0.01;
  const int def = default_order(mode, in->P), other = 1 - def;
  const int best = med[other] < med[def] * (1.0 - kTuneMargin) ? other : def;
  c->order_tune[mode] = mc_ctx::OrderTune{in->P, best};
  c->prep_fence = true;   // the next prep is an ordinary packet
  if (us_out) { us_out[0] = med[0]; us_out[1] = med[1]; }
  if (chosen) *chosen = best;
  return MC_OK;
}

int mc_deskew_steps(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t n_steps,
                    int32_t sample_every) {
  if (int r = deskew_check(c, in, out, mode, pose_select)) return r;
  CHECK_ARG(n_steps >= 1 && n_steps <= (1 << 16), "n_steps %d outside [1, 65536]", n_steps);
  CHECK_ARG(sample_every >= 0, "sample_every %d < 0", sample_every);
  if (in->F == 0 || in->n_tiles == 0) {
    // no deskew launch to carry a prep: the plain calls
    for (int32_t i = 0; i < n_steps; ++i)
      if (int r = mc_deskew(c, in, out, mode, pose_select)) return r;
    return MC_OK;
  }
  DeviceGuard g(c->device);
  return deskew_steps_pipelined(c, in, out, mode, pose_select, n_steps, sample_every);
}

constexpr int64_t kPipeRows = 1 << 21;                                 // 64 MB of (n,4) float64 (max chunk)
constexpr size_t kPipeBytes = (size_t)kPipeRows * 4 * sizeof(double);
constexpr int64_t kZeroCopyRows = 1 << 15;                             // below: zero-copy kernels
constexpr int kPoolThreads = 16;                                       // the box's CPU share per GPU
constexpr int64_t kJobRows = 8192;                                     // rows per host copy job (256 KB)
static int row_pipeline(mc_ctx* c, const double* const* frames, const int64_t* lds, const std::vector<int64_t>& doff,
                        const int64_t* d_doff, const double* d_pose, double* const* outs);

// pinned, device-mapped host scratch of at least `bytes` (the zero-copy path of the single calls)
static int ctx_pin(mc_ctx* c, size_t bytes, char** out) {
  if (bytes > c->pin_bytes) {
    if (c->h_pin) { (void)hipStreamSynchronize(c->stream); (void)hipHostFree(c->h_pin); c->h_pin = nullptr; }
    c->pin_bytes = 0;
    HIPCHK(hipHostMalloc(&c->h_pin, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    c->pin_bytes = bytes;
  }
  *out = static_cast<char*>(c->h_pin);
  return MC_OK;
}

// Frames of host float64 rows through k_align_rows_f64 with the per-frame poses pose12 (F x 12,
// host): below kZeroCopyRows rows the kernel reads and writes pinned, device-mapped host memory
// (no DMA round trips for the reference's per-frame calls); above, the DMA row pipeline.
static int align_host_rows(mc_ctx* c, const double* const* frames, const int64_t* lds, const std::vector<int64_t>& doff,
                           const std::vector<double>& pose12, double* const* outs) {
  const int32_t F = (int32_t)doff.size() - 1;
  const int64_t n = doff[F];
  if (n >= kZeroCopyRows) {
    void* st = nullptr;
    const size_t tab_b = doff.size() * sizeof(int64_t) + pose12.size() * sizeof(double);
    if (int r = ctx_stage(c, tab_b, &st)) return r;
    int64_t* d_doff = static_cast<int64_t*>(st);
    double* d_pose = reinterpret_cast<double*>(d_doff + doff.size());
    HIPCHK(hipMemcpyAsync(d_doff, doff.data(), doff.size() * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_pose, pose12.data(), pose12.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return row_pipeline(c, frames, lds, doff, d_doff, d_pose, outs);
  }
  // pinned [doff (F+1) | poses (12 F) | rows (n, 4) | out (n, 4)], 8-byte words
  const size_t w_pose = doff.size(), w_rows = w_pose + pose12.size(), w_out = w_rows + 4 * (size_t)n;
  char* base = nullptr;
  if (int r = ctx_pin(c, (w_out + 4 * (size_t)n) * 8, &base)) return r;
  double* pin = reinterpret_cast<double*>(base);
  std::memcpy(pin, doff.data(), doff.size() * 8);
  std::memcpy(pin + w_pose, pose12.data(), pose12.size() * 8);
  for (int32_t f = 0; f < F; ++f) {
    const int64_t m = doff[f + 1] - doff[f], ld = lds[f];
    double* dst = pin + w_rows + 4 * doff[f];
    if (ld == 4) std::memcpy(dst, frames[f], (size_t)m * 4 * sizeof(double));
    else for (int64_t i = 0; i < m; ++i) std::memcpy(dst + 4 * i, frames[f] + i * ld, 4 * sizeof(double));
  }
  {
    TimedRegion tr(c, &c->main_ev, c->stream);
    const int grid = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, 1024);
    hipLaunchKernelGGL(k_align_rows_f64, dim3(grid), dim3(kBlock), 0, c->stream, pin + w_rows, (int64_t)4, n,
                       (int64_t)0, reinterpret_cast<const int64_t*>(pin), F, pin + w_pose, pin + w_out);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int32_t f = 0; f < F; ++f)
    if (doff[f + 1] > doff[f])
      std::memcpy(outs[f], pin + w_out + 4 * doff[f], (size_t)(doff[f + 1] - doff[f]) * 4 * sizeof(double));
  return MC_OK;
}

int mc_transform_pointcloud_f64(mc_ctx* c, const double* points, int64_t n, int64_t ld, const double* rpy,
                                const double* translation, double* out) {
  CHECK_ARG(c && rpy && translation, "NULL argument");
  CHECK_ARG(n >= 0, "negative point count");
  if (ld < 4) return fail(MC_ERR_INDEX, "index 3 is out of bounds for axis 1 with size %lld", (long long)ld);
  if (n == 0) return MC_OK;
  CHECK_ARG(points && out, "NULL points / out");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  // LMC:774: R = Rotation.from_euler('xyz', rotation).as_matrix(), scipy's arithmetic (rot.cpp)
  std::vector<double> pose(12);
  mcrot::euler_xyz_scipy(rpy, pose.data());
  for (int k = 0; k < 3; ++k) pose[9 + k] = translation[k];
  const std::vector<int64_t> doff{0, n};
  const double* fr[1] = {points};
  const int64_t lds[1] = {ld};
  double* const outs[1] = {out};
  return align_host_rows(c, fr, lds, doff, pose, outs);
}

// ---- per-point modes on host float64 rows (k_points_f64) --------------------------------------

int mc_deskew_points_f64(mc_ctx* c, int mode, int32_t F, const int64_t* counts, const double* points, int64_t ld,
                         const int64_t* t_ns, const double* frame_times, const int64_t* frame_start_ns, double* out) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(mode == MC_MODE_POSE_SLERP || mode == MC_MODE_IMU, "mode %d: MC_MODE_POSE_SLERP or MC_MODE_IMU expected",
            mode);
  CHECK_ARG(F >= 0, "n_frames must be >= 0");
  CHECK_ARG(F == 0 || counts, "counts is NULL");
  if (ld < 3) return fail(MC_ERR_INDEX, "points need at least 3 columns (x, y, z); got %lld", (long long)ld);
  std::vector<int64_t> doff((size_t)F + 1, 0);
  for (int32_t f = 0; f < F; ++f) {
    CHECK_ARG(counts[f] >= 0, "negative frame size at frame %d", f);
    doff[f + 1] = doff[f] + counts[f];
  }
  if (mode == MC_MODE_POSE_SLERP) {
    if (c->T < 1) return fail(MC_ERR_STATE, "no trajectory uploaded (mc_set_trajectory)");
    CHECK_ARG(F == 0 || frame_times, "frame times are NULL");
  } else {
    if (c->M < 1) return fail(MC_ERR_STATE, "no IMU samples uploaded (mc_set_imu)");
    CHECK_ARG(F == 0 || frame_start_ns, "frame start times are NULL");
  }
  const int64_t n = doff[F];
  if (n == 0) return MC_OK;
  CHECK_ARG(points && t_ns && out, "NULL points / t_ns / out");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  hipStream_t s = c->stream;
  // the segment table of the uploaded trajectory / IMU samples (k_prep's table lanes, no frames)
  const uint64_t ver = mode == MC_MODE_POSE_SLERP ? c->traj_ver : c->imu_ver;
  const int64_t nseg = mode == MC_MODE_POSE_SLERP ? std::max<int64_t>(c->T - 1, 1) : c->M;
  const size_t seg_b = (size_t)nseg * (mode == MC_MODE_POSE_SLERP ? sizeof(PoseSeg) : sizeof(ImuSeg));
  if (!(c->d_seg64 && c->seg64_mode == mode && c->seg64_ver == ver)) {
    c->seg64_mode = -1;
    if (seg_b > c->seg64_bytes) {
      if (c->d_seg64) (void)hipFree(c->d_seg64);
      c->d_seg64 = nullptr;
      c->seg64_bytes = 0;
      HIPCHK(hipMalloc(&c->d_seg64, seg_b));
      c->seg64_bytes = seg_b;
    }
    PrepArgs pa;
    std::memset(&pa, 0, sizeof(pa));
    pa.mode = mode;
    pa.n_frames = 0;
    pa.time = c->d_time; pa.pos = c->d_pos; pa.rpy = c->d_rpy; pa.T = c->T;
    pa.imu_ts = c->d_imu_ts; pa.gyro = c->d_gyro; pa.M = c->M;
    pa.pose_seg = static_cast<PoseSeg*>(c->d_seg64);
    pa.imu_seg = static_cast<ImuSeg*>(c->d_seg64);
    pa.nseg = nseg;
    const uint32_t blocks = (uint32_t)(((nseg + 63) / 64 + 3) / 4);
    hipLaunchKernelGGL(k_prep, dim3(blocks), dim3(kBlock), 0, s, pa);
    HIPCHK(hipGetLastError());
    c->seg64_mode = mode;
    c->seg64_ver = ver;
  }
  // scratch: [doff (F+1) | per-frame value (F) | t_ns (n) | points (n, ld) | out (n, 4)], 8-byte words;
  // pinned and device-mapped below kZeroCopyRows rows (the kernel reads and writes host memory: no
  // DMA round trips for the reference's per-frame calls), a device staging buffer above
  const size_t w_doff = 0, w_fv = (size_t)F + 1, w_t = w_fv + (size_t)F, w_pts = w_t + (size_t)n,
               w_out = w_pts + (size_t)n * (size_t)ld, words = w_out + 4 * (size_t)n;
  const bool zero_copy = n < kZeroCopyRows;
  char* base = nullptr;
  if (zero_copy) {
    if (int r = ctx_pin(c, words * 8, &base)) return r;
    std::memcpy(base + 8 * w_doff, doff.data(), doff.size() * 8);
    std::memcpy(base + 8 * w_fv, mode == MC_MODE_POSE_SLERP ? static_cast<const void*>(frame_times)
                                                            : static_cast<const void*>(frame_start_ns), (size_t)F * 8);
    std::memcpy(base + 8 * w_t, t_ns, (size_t)n * 8);
    std::memcpy(base + 8 * w_pts, points, (size_t)n * (size_t)ld * 8);
  } else {
    void* st = nullptr;
    if (int r = ctx_stage(c, words * 8, &st)) return r;
    base = static_cast<char*>(st);
    HIPCHK(hipMemcpyAsync(base + 8 * w_doff, doff.data(), doff.size() * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(base + 8 * w_fv, mode == MC_MODE_POSE_SLERP ? static_cast<const void*>(frame_times)
                                                                      : static_cast<const void*>(frame_start_ns),
                          (size_t)F * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(base + 8 * w_t, t_ns, (size_t)n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(base + 8 * w_pts, points, (size_t)n * (size_t)ld * 8, hipMemcpyHostToDevice, s));
  }
  PointsF64Args a;
  std::memset(&a, 0, sizeof(a));
  a.pts = reinterpret_cast<const double*>(base + 8 * w_pts); a.ld = ld; a.n = n;
  a.t_ns = reinterpret_cast<const int64_t*>(base + 8 * w_t);
  a.doff = reinterpret_cast<const int64_t*>(base + 8 * w_doff); a.F = F;
  a.ftime = reinterpret_cast<const double*>(base + 8 * w_fv);
  a.fstart = reinterpret_cast<const int64_t*>(base + 8 * w_fv);
  a.pose_time = c->d_time; a.pose_seg = static_cast<const PoseSeg*>(c->d_seg64); a.nseg = nseg;
  a.imu_ts = c->d_imu_ts; a.imu_seg = static_cast<const ImuSeg*>(c->d_seg64);
  a.ntab = mode == MC_MODE_POSE_SLERP ? c->T : c->M;
  a.out = reinterpret_cast<double*>(base + 8 * w_out);
  const int grid = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, zero_copy ? 1024 : 65536);
  {
    TimedRegion tr(c, &c->main_ev, s);
    if (mode == MC_MODE_POSE_SLERP) hipLaunchKernelGGL(k_points_f64<1>, dim3(grid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL(k_points_f64<2>, dim3(grid), dim3(kBlock), 0, s, a);
  }
  HIPCHK(hipGetLastError());
  if (!zero_copy) HIPCHK(hipMemcpyAsync(out, a.out, (size_t)n * 32, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (zero_copy) std::memcpy(out, a.out, (size_t)n * 32);
  return MC_OK;
}

// ---- host arrays <-> device: the row pipeline ------------------------------------------------
// Rows of the concatenated frames travel in chunks: the host pool copies a chunk into pinned
// memory (compacting rows to 4 columns), DMA to HBM, k_align_rows_f64, DMA back, the pool copies
// the rows out to the caller's arrays — chunk k's host copies overlap chunk k±1's DMA and kernel.

static void host_rows(mc_ctx* c, const std::vector<int64_t>& doff, int64_t r0, int64_t r1,
                      const std::function<void(int32_t, int64_t, int64_t)>& seg) {
  // segments (frame, row_a, row_b) of [r0, r1), at most kJobRows rows each, run on the pool
  std::vector<std::array<int64_t, 3>> jobs;
  int32_t f = (int32_t)(std::upper_bound(doff.begin(), doff.end(), r0) - doff.begin()) - 1;
  for (; f < (int32_t)doff.size() - 1 && doff[f] < r1; ++f)
    for (int64_t a = std::max(doff[f], r0), e = std::min(doff[f + 1], r1); a < e; a += kJobRows)
      jobs.push_back({f, a, std::min(a + kJobRows, e)});
  if (!c->pool) c->pool.reset(new mcimpl::HostPool(kPoolThreads));
  c->pool->run((int64_t)jobs.size(), [&](int64_t j) { seg((int32_t)jobs[j][0], jobs[j][1], jobs[j][2]); });
}

// Chunk k's H2D (main stream) runs beside chunk k-1's D2H (side stream), and the host pool copies
// chunk k into pinned memory, and chunk k-1's rows out of it, while the DMA engines move the chunks
// around them.  For 600 x 100k rows (profiles/round6/s04, s06, s18): one stream for both directions
// 79-84 ms, two streams 58-66 ms into an already-faulted output (3.84 GB over PCIe; both directions
// at once carry 55-97 GB/s together depending on the box, s16 / s18), DMA straight from the caller's
// pageable frames 157-248 ms, D2H straight into page-locked outputs 59-74 ms (no gain over the
// staged copy-out).  MCDESKEW_ROWPIPE_TRACE=1 prints the phase times.

static int row_pipeline(mc_ctx* c, const double* const* frames, const int64_t* lds, const std::vector<int64_t>& doff,
                        const int64_t* d_doff, const double* d_pose, double* const* outs) {
  const int32_t F = (int32_t)doff.size() - 1;
  const int64_t n = doff[F];
  const int64_t rows_per = kPipeRows;   // 2 M rows (64 MB) per chunk: 58-61 vs 64 ms at 1 M (round 6, s04 / s06)
  const bool trace = std::getenv("MCDESKEW_ROWPIPE_TRACE") != nullptr;
  double t_in = 0, t_out = 0, t_wait_in = 0, t_wait_out = 0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = now();
  if (!c->h_pipe) HIPCHK(hipHostMalloc(&c->h_pipe, 4 * kPipeBytes, hipHostMallocDefault));
  if (!c->d_pipe) HIPCHK(hipMalloc(&c->d_pipe, 4 * kPipeBytes));
  double* pin[4];
  double* dev[4];
  for (int k = 0; k < 4; ++k) {
    pin[k] = reinterpret_cast<double*>(static_cast<char*>(c->h_pipe) + k * kPipeBytes);
    dev[k] = reinterpret_cast<double*>(static_cast<char*>(c->d_pipe) + k * kPipeBytes);
  }
  hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_out[2] = {nullptr, nullptr}, ev_k[2] = {nullptr, nullptr};
  for (int b = 0; b < 2; ++b) {
    HIPCHK(hipEventCreateWithFlags(&ev_in[b], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_out[b], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_k[b], hipEventDisableTiming));
  }
  hipStream_t s = c->stream, so = c->side;   // H2D + kernel | D2H
  auto copy_out = [&](int64_t k) {
    const double t0 = now();
    const int64_t r0 = k * rows_per, r1 = std::min(n, r0 + rows_per);
    const double* src = pin[2 + (k & 1)];
    host_rows(c, doff, r0, r1, [&](int32_t f, int64_t a, int64_t e) {
      std::memcpy(outs[f] + 4 * (a - doff[f]), src + 4 * (a - r0), (size_t)(e - a) * 4 * sizeof(double));
    });
    t_out += now() - t0;
  };
  const int64_t K = (n + rows_per - 1) / rows_per;
  int rc = MC_OK;
  for (int64_t k = 0; k < K && rc == MC_OK; ++k) {
    const int b = (int)(k & 1);
    const int64_t r0 = k * rows_per, r1 = std::min(n, r0 + rows_per), m = r1 - r0;
    const double tw = now();
    if (k >= 2) (void)hipEventSynchronize(ev_in[b]);                 // pinned input b is free again
    const double t0 = now();
    t_wait_in += t0 - tw;
    double* dst = pin[b];
    host_rows(c, doff, r0, r1, [&](int32_t f, int64_t a, int64_t z) {
      const int64_t ld = lds[f];
      const double* sp = frames[f] + (a - doff[f]) * ld;
      double* dp = dst + 4 * (a - r0);
      if (ld == 4) {
        std::memcpy(dp, sp, (size_t)(z - a) * 4 * sizeof(double));
      } else {
        for (int64_t i = 0; i < z - a; ++i) std::memcpy(dp + 4 * i, sp + i * ld, 4 * sizeof(double));
      }
    });
    t_in += now() - t0;
    hipError_t e = hipMemcpyAsync(dev[b], pin[b], (size_t)m * 32, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(ev_in[b], s);
    // dev[2 + b] is free once chunk k-2's D2H (side stream) has finished
    if (e == hipSuccess && k >= 2) e = hipStreamWaitEvent(s, ev_out[b], 0);
    if (e == hipSuccess) {
      TimedRegion tr(c, &c->main_ev, s);
      hipLaunchKernelGGL(k_align_rows_f64, dim3((unsigned)std::min<int64_t>((m + kBlock - 1) / kBlock, 4096)),
                         dim3(kBlock), 0, s, dev[b], (int64_t)4, m, r0, d_doff, F, d_pose, dev[2 + b]);
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(ev_k[b], s);
    if (e == hipSuccess) e = hipStreamWaitEvent(so, ev_k[b], 0);
    if (e == hipSuccess && k >= 1) {                                // chunk k-1's rows are back: copy out
      const double tw2 = now();
      e = hipEventSynchronize(ev_out[b ^ 1]);
      t_wait_out += now() - tw2;
      if (e == hipSuccess) copy_out(k - 1);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(pin[2 + b], dev[2 + b], (size_t)m * 32, hipMemcpyDeviceToHost, so);
    if (e == hipSuccess) e = hipEventRecord(ev_out[b], so);
    if (e != hipSuccess) rc = fail(MC_ERR_HIP, "row pipeline: %s", hipGetErrorString(e));
  }
  if (rc == MC_OK && K > 0) {
    const double tw = now();
    const hipError_t e = hipEventSynchronize(ev_out[(K - 1) & 1]);
    t_wait_out += now() - tw;
    if (e != hipSuccess) rc = fail(MC_ERR_HIP, "row pipeline: %s", hipGetErrorString(e));
    else copy_out(K - 1);
  }
  (void)hipStreamSynchronize(so);
  (void)hipStreamSynchronize(s);
  for (int b = 0; b < 2; ++b) {
    (void)hipEventDestroy(ev_in[b]); (void)hipEventDestroy(ev_out[b]); (void)hipEventDestroy(ev_k[b]);
  }
  if (trace)
    std::fprintf(stderr, "rowpipe rows %lld chunks %lld: total %.2f ms, copy-in %.2f, copy-out %.2f, wait-in %.2f, "
                 "wait-out %.2f ms\n", (long long)rows_per, (long long)K,
                 1e3 * (now() - t_start), 1e3 * t_in, 1e3 * t_out, 1e3 * t_wait_in, 1e3 * t_wait_out);
  return rc;
}

int mc_align_frames_host_f64(mc_ctx* c, int32_t F, const double* const* frames, const int64_t* counts,
                             const int64_t* lds, const double* frame_times, int pose_select, double* const* outs) {
  CHECK_ARG(c && (F == 0 || (frames && counts && lds && outs)), "NULL argument");
  CHECK_ARG(F >= 0, "n_frames must be >= 0");
  CHECK_ARG(pose_select == MC_POSE_SEARCHSORTED || pose_select == MC_POSE_DIRECT, "unknown pose_select");
  if (c->T < 1) return fail(MC_ERR_STATE, "no trajectory uploaded (mc_set_trajectory)");
  if (pose_select == MC_POSE_DIRECT && c->T != F)
    return fail(MC_ERR_INVALID, "MC_POSE_DIRECT needs one pose per frame (T=%lld, frames=%d)", (long long)c->T, F);
  CHECK_ARG(pose_select == MC_POSE_DIRECT || F == 0 || frame_times, "frame times are NULL");
  std::vector<int64_t> doff((size_t)F + 1, 0);
  for (int32_t f = 0; f < F; ++f) {
    CHECK_ARG(counts[f] >= 0, "negative frame size at frame %d", f);
    if (counts[f] > 0 && lds[f] < 4)
      return fail(MC_ERR_INDEX, "index 3 is out of bounds for axis 1 with size %lld", (long long)lds[f]);
    CHECK_ARG(counts[f] == 0 || (frames[f] && outs[f]), "NULL frame pointer at frame %d", f);
    doff[f + 1] = doff[f] + counts[f];
  }
  const int64_t n = doff[F];
  if (n == 0) return MC_OK;
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  // per-frame float64 pose {R | t}: pose selection LMC:804-812 and scipy's R (LMC:774), host-side
  std::vector<double> pose(12 * (size_t)F);
  mcrot::frame_poses(c->h_time.data(), c->h_pos.data(), c->h_rpy.data(), c->T, frame_times, F, pose_select,
                     pose.data());
  return align_host_rows(c, frames, lds, doff, pose, outs);
}

int mc_affine_rows_f64(mc_ctx* c, int32_t F, const int64_t* counts, const double* rows, int64_t ld, int32_t n_mats,
                       const double* mats, int per_row, double* out) {
  CHECK_ARG(c && (F == 0 || counts) && mats, "NULL argument");
  CHECK_ARG(F >= 0, "n_frames must be >= 0");
  CHECK_ARG(ld == 3 || ld == 4, "rows need 3 or 4 columns (got %lld)", (long long)ld);
  CHECK_ARG(n_mats == 1 || n_mats == F, "need 1 or n_frames matrices (got %d for %d frames)", n_mats, F);
  CHECK_ARG(per_row >= MC_AFFINE_PER_FRAME && per_row <= MC_AFFINE_TRANSLATE, "unknown per_row mode %d", per_row);
  std::vector<int64_t> doff((size_t)F + 1, 0);
  for (int32_t f = 0; f < F; ++f) {
    CHECK_ARG(counts[f] >= 0, "negative frame size at frame %d", f);
    doff[f + 1] = doff[f] + counts[f];
  }
  const int64_t n = doff[F];
  if (n == 0) return MC_OK;
  CHECK_ARG(rows && out, "NULL rows / out");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  // [doff (F+1) | mats (12 n_mats) | rows (n, ld) | out (n, 3)] in 8-byte words: pinned and
  // device-mapped below kZeroCopyRows rows, device staging with DMA above
  const size_t w_mat = doff.size(), w_rows = w_mat + 12 * (size_t)n_mats, w_out = w_rows + (size_t)n * ld,
               words = w_out + 3 * (size_t)n;
  const bool zero_copy = n < kZeroCopyRows;
  char* base = nullptr;
  hipStream_t s = c->stream;
  if (zero_copy) {
    if (int r = ctx_pin(c, words * 8, &base)) return r;
    std::memcpy(base, doff.data(), doff.size() * 8);
    std::memcpy(base + 8 * w_mat, mats, 12 * (size_t)n_mats * 8);
    std::memcpy(base + 8 * w_rows, rows, (size_t)n * ld * 8);
  } else {
    void* st = nullptr;
    if (int r = ctx_stage(c, words * 8, &st)) return r;
    base = static_cast<char*>(st);
    HIPCHK(hipMemcpyAsync(base, doff.data(), doff.size() * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(base + 8 * w_mat, mats, 12 * (size_t)n_mats * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(base + 8 * w_rows, rows, (size_t)n * ld * 8, hipMemcpyHostToDevice, s));
  }
  double* d_out = reinterpret_cast<double*>(base + 8 * w_out);
  {
    TimedRegion tr(c, &c->main_ev, s);
    const int grid = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, zero_copy ? 1024 : 65536);
    hipLaunchKernelGGL(k_affine_rows_f64, dim3(grid), dim3(kBlock), 0, s,
                       reinterpret_cast<const double*>(base + 8 * w_rows), ld, n, reinterpret_cast<const int64_t*>(base),
                       F, reinterpret_cast<const double*>(base + 8 * w_mat), n_mats, per_row, d_out);
  }
  HIPCHK(hipGetLastError());
  if (!zero_copy) HIPCHK(hipMemcpyAsync(out, d_out, (size_t)n * 24, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (zero_copy) std::memcpy(out, d_out, (size_t)n * 24);
  return MC_OK;
}

int mc_transform_affine(mc_ctx* c, const mc_batch* in, mc_batch* out, int32_t n_mats, const double* mats,
                        int w_column) {
  CHECK_ARG(c && in && out && mats, "NULL argument");
  CHECK_ARG(in->ctx == c && out->ctx == c, "batches belong to another context");
  CHECK_ARG(in->counts == out->counts, "input and output batches have different frame counts");
  CHECK_ARG(n_mats == 1 || n_mats == in->F, "need 1 or n_frames matrices (got %d for %d frames)", n_mats, in->F);
  if (in->F == 0) return MC_OK;
  DeviceGuard g(c->device);
  hipStream_t s = c->stream;
  // the frame table half not used by the last mc_deskew; main-stream order protects the previous
  // reader of this half, the event hands it back to the next pipelined prep
  const int h = c->buf;
  c->buf ^= 1;
  forget_speculation(c);   // half h is overwritten below
  std::vector<FrameRow> tbl(3 * (size_t)in->F);
  for (int32_t f = 0; f < in->F; ++f) {
    const double* m = mats + 12 * (size_t)(n_mats == 1 ? 0 : f);
    for (int r = 0; r < 3; ++r) tbl[3 * (size_t)f + r] = FrameRow{m[4 * r], m[4 * r + 1], m[4 * r + 2], m[4 * r + 3]};
  }
  FrameRow* frame_tbl = in->d_frame_tbl + 3 * (size_t)in->F * h;
  queued_async(c);
  HIPCHK(hipMemcpyAsync(frame_tbl, tbl.data(), tbl.size() * sizeof(FrameRow), hipMemcpyHostToDevice, s));
  if (in->n_tiles > 0) {
    out->wrote(false);
    DeskewArgs da;
    std::memset(&da, 0, sizeof(da));
    da.in = in->d_cols; da.in_C = in->C;
    da.out = out->d_cols; da.out_C = out->C;
    da.tiles = in->d_tiles; da.n_tiles = in->n_tiles;
    da.frame_tbl = frame_tbl;
    da.xcd_order = MC_XCD_FRAME;
    const dim3 grid(launch_grid(c, in->n_tiles)), block(kBlock);
    TimedRegion tr(c, &c->main_ev, s);
    if (w_column) hipLaunchKernelGGL(k_affine_w, grid, block, 0, s, da);
    else hipLaunchKernelGGL(k_deskew_frame, grid, block, 0, s, da);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_main_done[h], s));
  // the host table must outlive the (possibly pageable-staged) copy
  HIPCHK(hipStreamSynchronize(s));
  return MC_OK;
}

int mc_timing_enable(mc_ctx* c, int enable) {
  CHECK_ARG(c, "ctx is NULL");
  c->timing = enable != 0;
  return MC_OK;
}


int mc_timing_read_each(mc_ctx* c, double* ms, int64_t cap, int64_t* n) {
  CHECK_ARG(c && n && (cap == 0 || ms), "NULL argument");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  *n = (int64_t)c->main_ev.size();
  for (int64_t k = 0; k < *n && k < cap; ++k) {
    float m = 0.f;
    HIPCHK(hipEventElapsedTime(&m, c->main_ev[k].first, c->main_ev[k].second));
    ms[k] = m;
  }
  return sum_events(c, c->main_ev, nullptr, nullptr);   // the main events only (the rest stays pending)
}

int mc_timing_read_spans(mc_ctx* c, double* us, int64_t cap, int64_t* n) {
  CHECK_ARG(c && n && (cap == 0 || us), "NULL argument");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  *n = 0;
  if (!c->d_span || c->span_used == 0) return MC_OK;
  if (c->wall_khz <= 0.0) {
    int khz = 0;
    HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    if (khz <= 0) return fail(MC_ERR_HIP, "wall clock rate %d kHz", khz);
    c->wall_khz = khz;
  }
  std::vector<unsigned long long> h((size_t)c->span_used * kSpanWords);
  HIPCHK(hipMemcpy(h.data(), c->d_span, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (int32_t k = 0; k < c->span_used; ++k) {
    const unsigned long long* w = h.data() + (size_t)k * kSpanWords;
    unsigned long long end = 0;
    for (size_t j = 1; j < kSpanWords; ++j) end = w[j] > end ? w[j] : end;
    if (w[0] == 0 || end < w[0]) continue;   // a launch without deskew workgroups
    if (*n < cap) us[*n] = (double)(end - w[0]) / c->wall_khz * 1e3;   // ticks / kHz = ms
    ++*n;
  }
  HIPCHK(hipMemset(c->d_span, 0, (size_t)c->span_used * kSpanWords * sizeof(unsigned long long)));
  c->span_used = 0;
  return MC_OK;
}

int mc_timing_read(mc_ctx* c, double* main_ms, int64_t* main_n, double* prep_ms, int64_t* prep_n) {
  CHECK_ARG(c, "ctx is NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  if (int r = sum_events(c, c->main_ev, main_ms, main_n)) return r;
  if (int r = sum_events(c, c->prep_ev, prep_ms, prep_n)) return r;
  return MC_OK;
}

// ---- scan_environment (LMC:701-770) --------------------------------------------------------
int mc_set_environment(mc_ctx* c, int64_t n, const double* env, int64_t ld) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(n >= 0, "negative scene size");
  if (ld < 4) return fail(MC_ERR_INDEX, "scene points need at least 4 columns; got %lld", (long long)ld);
  CHECK_ARG(n == 0 || env, "scene pointer is NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  ++c->env_ver;              // any earlier mc_scan_count's state is now stale
  c->scan_valid = false;
  dev_free(c->d_env);
  c->E = 0;
  // scan.hpp's column layout: x, y, z, intensity float64, transposed here once per scene
  const size_t words = scene_words(n);
  if (int r = dev_alloc(&c->d_env, std::max<size_t>(words, 1))) return r;
  if (n > 0) {
    std::vector<double> h(words);
    for (int64_t i = 0; i < n; ++i) {
      const double* q = env + i * ld;
      h[i] = q[0]; h[n + i] = q[1]; h[2 * n + i] = q[2]; h[3 * n + i] = q[3];
    }
    HIPCHK(hipMemcpyAsync(c->d_env, h.data(), words * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  c->E = n;
  return MC_OK;
}

int mc_scan_count(mc_ctx* c, int32_t F, const double* frame_times, int pose_select, const double* params,
                  int64_t cap, int64_t* counts_out) {
  CHECK_ARG(c && params && counts_out, "NULL argument");
  CHECK_ARG(F >= 0 && F <= 65535 * kScanFrames, "n_frames must be in [0, %d]", 65535 * kScanFrames);
  CHECK_ARG(cap >= 1, "points_per_frame must be >= 1");
  CHECK_ARG(pose_select == MC_POSE_SEARCHSORTED || pose_select == MC_POSE_DIRECT, "unknown pose_select");
  if (c->T < 1) return fail(MC_ERR_STATE, "no trajectory uploaded (mc_set_trajectory)");
  if (pose_select == MC_POSE_DIRECT && c->T != F)
    return fail(MC_ERR_INVALID, "MC_POSE_DIRECT needs one pose per frame (T=%lld, frames=%d)", (long long)c->T, F);
  CHECK_ARG(pose_select == MC_POSE_DIRECT || F == 0 || frame_times, "frame times are NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  const int32_t tiles = (int32_t)((c->E + kScanTile - 1) / kScanTile);
  dev_free(c->d_scan_pose); dev_free(c->d_scan_tcount); dev_free(c->d_scan_toff);
  dev_free(c->d_scan_nvis);
  c->scan_F = 0;
  c->scan_valid = false;
  if (int r = dev_alloc(&c->d_scan_pose, 12 * (size_t)std::max(F, 1))) return r;
  const int32_t Fp = scan_fpad(F);   // per-tile rows of counts / offsets, frames padded to kScanFrames
  if (int r = dev_alloc(&c->d_scan_tcount, (size_t)std::max(Fp, 1) * std::max(tiles, 1))) return r;
  if (int r = dev_alloc(&c->d_scan_toff, (size_t)std::max(Fp, 1) * std::max(tiles, 1))) return r;
  if (int r = dev_alloc(&c->d_scan_nvis, std::max(F, 1))) return r;
  c->scan_par[0] = params[0];
  c->scan_par[1] = params[1] * params[1];   // LMC:715 max_range_sq
  c->scan_par[2] = params[2] / 2;           // LMC:740
  c->scan_par[3] = params[3] / 2;           // LMC:741
  c->scan_cap = cap;
  c->scan_counts.assign(F, 0);
  c->scan_F = F;
  c->scan_tiles = tiles;
  c->scan_env_ver = c->env_ver;
  if (F == 0) {
    c->scan_valid = true;
    return MC_OK;
  }
  // per-frame sensor pose {R | t} (LMC:804-812; R as scipy computes it, LMC:726), host-side
  std::vector<double> pose(12 * (size_t)F);
  mcrot::frame_poses(c->h_time.data(), c->h_pos.data(), c->h_rpy.data(), c->T, frame_times, F, pose_select,
                     pose.data());
  HIPCHK(hipMemcpyAsync(c->d_scan_pose, pose.data(), pose.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
  std::vector<int64_t> nvis(F, 0), toff((size_t)Fp * std::max(tiles, 1), 0);
  if (tiles > 0) {
    const ScanParams sp = make_scan_params(c->scan_par, cap);
    const size_t words = (size_t)tiles * ((F + kScanFrames - 1) / kScanFrames) * kBlock;
    if (words > c->scan_bits_cap) {
      dev_free(c->d_scan_bits);
      c->scan_bits_cap = 0;
      if (int r = dev_alloc(&c->d_scan_bits, words)) return r;
      c->scan_bits_cap = words;
    }
    {
      TimedRegion tr(c, &c->scan_ev, c->stream);
      const uint32_t units = (uint32_t)tiles * (uint32_t)((F + kScanFrames - 1) / kScanFrames);
      hipLaunchKernelGGL(k_scan_count, dim3(units), dim3(kBlock), 0, c->stream, c->d_env, c->E, tiles,
                         c->d_scan_pose, F, sp, c->d_scan_tcount, c->d_scan_bits);
    }
    HIPCHK(hipGetLastError());
    std::vector<int32_t> tc((size_t)Fp * tiles);
    HIPCHK(hipMemcpyAsync(tc.data(), c->d_scan_tcount, tc.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int32_t t = 0; t < tiles; ++t) {   // tile-major rows: the frames' running sums side by side
      const size_t row = (size_t)t * Fp;
      for (int32_t f = 0; f < F; ++f) { toff[row + f] = nvis[f]; nvis[f] += tc[row + f]; }
    }
    HIPCHK(hipMemcpyAsync(c->d_scan_toff, toff.data(), toff.size() * sizeof(int64_t), hipMemcpyHostToDevice,
                          c->stream));
  }
  HIPCHK(hipMemcpyAsync(c->d_scan_nvis, nvis.data(), F * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int32_t f = 0; f < F; ++f) {
    // LMC:757-762: every (n // cap)-th visible point, at most cap of them
    const int64_t n = nvis[f];
    int64_t k = n;
    if (n > cap) {
      const int64_t step = n / cap;
      k = std::min<int64_t>(cap, (n + step - 1) / step);
    }
    c->scan_counts[f] = k;
    counts_out[f] = k;
  }
  c->scan_valid = true;
  return MC_OK;
}

// pass 2 of the last mc_scan_count: the batch's float32 columns (out != nullptr) or the reference's
// float64 rows (local, aligned: device (N, 4) arrays, aligned may be nullptr)
static int scan_emit(mc_ctx* c, mc_batch* out, const double* noise, double* d_local, double* d_aligned) {
  if (!c->scan_valid || c->scan_env_ver != c->env_ver)
    return fail(MC_ERR_STATE, "no mc_scan_count for the current scene (mc_set_environment since the count?)");
  int64_t N = 0;
  for (int64_t k : c->scan_counts) N += k;
  if (c->scan_F == 0 || N == 0 || c->scan_tiles == 0) return MC_OK;
  DeviceGuard g(c->device);
  // staging: [noise (N, 3) | doff (F + 1)] (the rows path has no batch offsets of its own)
  const size_t noise_w = noise ? 3 * (size_t)N : 0;
  void* st = nullptr;
  if (int r = ctx_stage(c, (noise_w + (size_t)c->scan_F + 1) * 8, &st)) return r;
  double* d_noise = noise ? static_cast<double*>(st) : nullptr;
  int64_t* d_doff = reinterpret_cast<int64_t*>(static_cast<double*>(st) + noise_w);
  if (noise) HIPCHK(hipMemcpyAsync(d_noise, noise, noise_w * sizeof(double), hipMemcpyHostToDevice, c->stream));
  std::vector<int64_t> doff((size_t)c->scan_F + 1, 0);
  for (int32_t f = 0; f < c->scan_F; ++f) doff[f + 1] = doff[f] + c->scan_counts[f];
  if (!out) HIPCHK(hipMemcpyAsync(d_doff, doff.data(), doff.size() * 8, hipMemcpyHostToDevice, c->stream));
  ScanEmitArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.env = c->d_env; ea.E = c->E; ea.n_tiles = c->scan_tiles;
  ea.pose = c->d_scan_pose; ea.F = c->scan_F;
  ea.sp = make_scan_params(c->scan_par, c->scan_cap);
  ea.tile_off = c->d_scan_toff; ea.nvis = c->d_scan_nvis; ea.vis_bits = c->d_scan_bits; ea.noise = d_noise;
  if (out) {
    ea.poff = out->d_poff; ea.doff = out->d_doff; ea.cols = out->d_cols; ea.C = out->C;
    out->wrote(false);
    ea.pcd_len = out->d_pcd_len;   // MC_BATCH_WITH_PCD_LEN: per-point atomic adds into zeroed slots
    if (ea.pcd_len) HIPCHK(hipMemsetAsync(ea.pcd_len, 0, (size_t)(out->P / kBlkPts) * sizeof(int32_t), c->stream));
  } else {
    ea.doff = d_doff; ea.local = d_local; ea.aligned = d_aligned;
  }
  {
    TimedRegion tr(c, &c->scan_ev, c->stream);
    const uint32_t units = (uint32_t)c->scan_tiles * (uint32_t)((c->scan_F + kScanFrames - 1) / kScanFrames);
    if (out) hipLaunchKernelGGL(k_scan_emit<false>, dim3(units), dim3(kBlock), 0, c->stream, ea);
    else hipLaunchKernelGGL(k_scan_emit<true>, dim3(units), dim3(kBlock), 0, c->stream, ea);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  if (out) out->wrote(true);
  return MC_OK;
}

int mc_scan_emit(mc_ctx* c, mc_batch* out, const double* noise) {
  CHECK_ARG(c && out, "NULL argument");
  CHECK_ARG(out->ctx == c, "batch belongs to another context");
  if (out->counts != c->scan_counts)
    return fail(MC_ERR_INVALID, "output batch frame counts differ from the last mc_scan_count");
  return scan_emit(c, out, noise, nullptr, nullptr);
}

int mc_scan_emit_f64(mc_ctx* c, const double* noise, double* d_local, double* d_aligned) {
  CHECK_ARG(c && d_local, "NULL argument");
  return scan_emit(c, nullptr, noise, d_local, d_aligned);
}

int mc_timing_read_scan(mc_ctx* c, double* ms, int64_t* n) {
  CHECK_ARG(c, "ctx is NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  return sum_events(c, c->scan_ev, ms, n);
}

int mc_timing_read_layout(mc_ctx* c, double* ms, int64_t* n) {
  CHECK_ARG(c, "ctx is NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  return sum_events(c, c->layout_ev, ms, n);
}

}  // extern "C"
