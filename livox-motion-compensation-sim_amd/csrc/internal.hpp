// internal.hpp — the opaque handles of include/mcdeskew.h (shared by mcdeskew.hip and comm.cpp).
#pragma once
#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <stdint.h>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mc {
struct Tile;
struct PoseSeg;
struct FrameRow;
struct ImuSeg;
struct FrameWin;
}  // namespace mc

namespace mcimpl {
int fail(int code, const char* fmt, ...);
constexpr int64_t kBatchBlock = 256;   // points per block of the blocked batch layout (= mc::kBlkPts)

// Persistent host worker pool for the host-side row copies of the host<->device pipeline.
class HostPool {
 public:
  explicit HostPool(int threads) {
    for (int k = 0; k < threads; ++k) th_.emplace_back([this] { work(); });
  }
  ~HostPool() {
    { std::lock_guard<std::mutex> l(m_); stop_ = true; }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(i) for i in [0, n) on the pool's threads; returns when all are done
  void run(int64_t n, const std::function<void(int64_t)>& fn) {
    if (n <= 0) return;
    std::unique_lock<std::mutex> l(m_);
    fn_ = &fn; n_ = n; next_ = 0; busy_ = (int)th_.size(); ++gen_;
    cv_.notify_all();
    done_.wait(l, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> l(m_);
      cv_.wait(l, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(int64_t)>* fn = fn_;
      const int64_t n = n_;
      l.unlock();
      for (int64_t i = next_++; i < n; i = next_++) (*fn)(i);
      l.lock();
      if (--busy_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};
}  // namespace mcimpl

struct mc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;   // main stream: staging + the deskew kernels
  hipStream_t side = nullptr;     // per-step pose prep, pipelined one step ahead of `stream`
  // per-step tables are double-buffered: prep of step i+1 (side) overlaps the kernel of step i
  int buf = 0;
  // true until the next k_prep must wait for everything queued before it (an ordinary, barrier
  // launch): set by async writers of the prep's inputs (t_ns spans) and by step-graph replays;
  // cleared by mc_deskew, whose deskew kernel then ends the queue (see mc_deskew)
  bool prep_fence = true;
  // Per-call speculation (mc_deskew): a call whose inputs equal the previous call's launches its
  // deskew fused with the prep of an identical next call into the other table half (the pipelined
  // launch of mc_deskew_steps); the next call, if its key still matches, finds its tables ready and
  // issues no k_prep.  Keys: the input batch's uid, mode, pose selection and the versions of every
  // prep input (trajectory, IMU, the batch's frame times / starts / t_ns spans).
  struct PrepKey {
    uint64_t batch = 0, traj = 0, imu = 0, frames = 0;
    int mode = -1, pose_select = -1;
    bool operator==(const PrepKey& o) const {
      return batch == o.batch && traj == o.traj && imu == o.imu && frames == o.frames && mode == o.mode &&
             pose_select == o.pose_select;
    }
  };
  PrepKey last_call;            // the previous mc_deskew's key (batch 0: none)
  PrepKey spec_key;             // what the tables in half spec_half were prepared for
  bool spec_valid = false;
  int spec_half = 0;
  uint64_t traj_ver = 0, imu_ver = 0;   // bumped by mc_set_trajectory / mc_set_imu
  // sub-tile order per mode measured by mc_tune_order for batches of P padded points (-1: none)
  struct OrderTune {
    int64_t P = -1;
    int32_t order = -1;
  };
  OrderTune order_tune[3];
  hipEvent_t ev_main_done[2] = {nullptr, nullptr};
  hipEvent_t ev_prep_done[2] = {nullptr, nullptr};
  hipEvent_t ev_order = nullptr;  // orders side-stream prep after async main-stream staging
  // trajectory (LMC:361-428): time, position_gps, orientation_imu; host copies for the float64
  // paths' per-frame poses (rot.cpp frame_poses)
  int64_t T = 0, T_cap = 0;
  std::vector<double> h_time, h_pos, h_rpy;
  double* d_time = nullptr;
  double* d_pos = nullptr;
  double* d_rpy = nullptr;
  mc::PoseSeg* d_pose_seg = nullptr;   // 2 * T_cap (double buffer)
  // IMU (CSIM:1191-1240)
  int64_t M = 0, M_cap = 0;
  int64_t* d_imu_ts = nullptr;
  double* d_gyro = nullptr;
  mc::ImuSeg* d_imu_seg = nullptr;     // 2 * M_cap (double buffer)
  // scan_environment state (LMC:701-770): scene, per-frame f64 poses, per-(frame, tile) counts
  int64_t E = 0;
  double* d_env = nullptr;   // the scene as columns (scan.hpp scene_cols)
  int32_t scan_F = 0, scan_tiles = 0;
  double* d_scan_pose = nullptr;
  int32_t* d_scan_tcount = nullptr;
  int64_t* d_scan_toff = nullptr;
  int64_t* d_scan_nvis = nullptr;
  uint32_t* d_scan_bits = nullptr;    // pass-1 visibility words
  size_t scan_bits_cap = 0;
  std::vector<int64_t> scan_counts;   // final per-frame counts of the last mc_scan_count
  double scan_par[4] = {0, 0, 0, 0};  // range_min, range_max^2, fov_h/2, fov_v/2
  int64_t scan_cap = 0;
  // the visibility words / tile offsets above describe the scene of version scan_env_ver; a pass 2
  // on any other scene is refused (the poses were copied to d_scan_pose by the count itself)
  uint64_t env_ver = 0, scan_env_ver = 0;
  bool scan_valid = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> scan_ev;
  // output codecs: per-call frame / unit tables carved from one scratch buffer, error flag
  void* d_codec = nullptr;
  size_t codec_bytes = 0;
  int* d_codec_err = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> codec_ev;
  // mc_deskew_pcd: ASCII PCD text bytes per 256-point output block, written by the deskew kernel
  int32_t* d_pcd_len = nullptr;
  int64_t pcd_len_cap = 0;
  // segment table of the float64 per-point path (mc_deskew_points_f64): built by k_prep for one mode
  // and the trajectory / IMU upload it came from (seg64_ver), rebuilt when either changes
  void* d_seg64 = nullptr;
  size_t seg64_bytes = 0;
  int seg64_mode = -1;
  uint64_t seg64_ver = 0;
  // pinned, device-mapped host buffer of the single-call drop-in path
  void* h_pin = nullptr;
  size_t pin_bytes = 0;
  // host <-> device row pipeline (double-buffered pinned and device chunks, in + out)
  void* h_pipe = nullptr;
  void* d_pipe = nullptr;
  std::unique_ptr<mcimpl::HostPool> pool;
  // staging buffer for host<->device layout conversion
  void* d_stage = nullptr;
  size_t stage_bytes = 0;
  // launch knobs / timing
  int32_t max_grid = 0;
  bool timing = false;
  double wall_khz = 0.0;   // wall_clock64() rate
  // workgroup spans of timed deskew launches (DeskewArgs::span): kSpanSlots slots of 1 + kSpanTail
  // wall-clock stamps, zeroed, handed out in launch order until mc_timing_read_spans
  unsigned long long* d_span = nullptr;
  int32_t span_used = 0;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> main_ev, prep_ev, layout_ev;
};

struct mc_batch {
  mc_ctx* ctx = nullptr;
  uint64_t uid = 0;         // unique per batch ever created (a key can never match a new batch)
  uint64_t prep_ver = 0;    // bumped whenever frame times, frame starts or the t_ns spans change
  int32_t F = 0;
  int64_t N = 0;    // valid points
  int64_t P = 0;    // padded points (poff[F]; every frame starts on a kBlkPts boundary)
  int32_t C = 4;    // columns per block: x | y | z | intensity [| t_ns]
  std::vector<int64_t> counts, poff, doff;
  std::vector<int32_t> ftile;      // first tile of each frame (F+1), host copy
  int32_t n_tiles = 0;
  // stream_unit order (layout.hpp) of the last kernel that went over the batch's points: its last
  // units may still be in the Infinity Cache, so the codec kernels run the opposite direction
  // (a hint for speed only; kernels that do not record it leave it stale)
  mutable int hot_order = 0;
  // blocked columns: block k (points 256k .. 256k+255) holds its C columns of 256 values back to
  // back, C * P values in all (mc::bidx); t_ns, when present, is column 4 (int32 bits)
  float* d_cols = nullptr;
  bool has_t() const { return C == 5; }
  int64_t* d_counts = nullptr;
  int64_t* d_poff = nullptr;
  int64_t* d_doff = nullptr;
  mc::Tile* d_tiles = nullptr;
  double* d_frame_time = nullptr;
  int64_t* d_frame_start = nullptr;
  // k_prep outputs, double-buffered (ctx->buf selects the half): F entries per half
  mc::FrameRow* d_frame_tbl = nullptr;   // 3 float64 rows per frame (R row, t)
  int2* d_trange = nullptr;        // per-frame [min, max] t_ns (valid when trange_valid)
  mc::FrameWin* d_fwin = nullptr;  // per-frame segment window
  void* d_frec = nullptr;          // 2 frame-specialised pose/IMU records per frame
  size_t frec_half = 0;            // bytes per half of d_frec
  // per sub-tile windows (batches with t_ns): frames wider than the SGPR path use these
  int32_t* d_ftile = nullptr;      // first tile of each frame (F+1)
  int2* d_strange = nullptr;       // per sub-tile [min, max] t_ns
  mc::FrameWin* d_swin = nullptr;  // per sub-tile window, double-buffered (2 * n_sub)
  double* d_partial = nullptr;
  bool has_times = false, has_starts = false, trange_valid = false;
  // MC_BATCH_WITH_PCD_LEN: ASCII PCD text bytes per 256-point block (layout.hpp PcdCount sums).
  // data_ver counts the writes of the x|y|z|intensity columns; pcd_ver is the data_ver the sums
  // were written with (current iff equal).
  int32_t* d_pcd_len = nullptr;
  uint64_t data_ver = 1, pcd_ver = 0;
  void wrote(bool with_sums) {                               // after queueing a write of the columns
    ++data_ver;
    if (with_sums && d_pcd_len) pcd_ver = data_ver;
  }
  bool pcd_current() const { return d_pcd_len && pcd_ver == data_ver; }
};

namespace mcimpl {
// mc_deskew's body; pcd_len != nullptr: the *_pcd deskew kernels also write each output block's
// ASCII PCD text bytes there (mc_deskew_pcd)
int deskew_call(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t* pcd_len);
// the sub-tile order (0 dealt, 1 XCD-contiguous) mc_deskew's kernel takes for this mode and batch
int deskew_order(const mc_ctx* c, const mc_batch* in, int mode);
}  // namespace mcimpl
