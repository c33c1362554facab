// internal.hpp — the opaque handles of include/mcdeskew.h (shared by mcdeskew.hip and comm.cpp).
#pragma once
#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <stdint.h>
#include <string>
#include <utility>
#include <vector>

namespace mc {
struct Tile;
struct PoseSeg;
struct ImuSeg;
struct FrameWin;
}  // namespace mc

namespace mcimpl {
int fail(int code, const char* fmt, ...);
}

struct mc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // trajectory (LMC:361-428): time, position_gps, orientation_imu
  int64_t T = 0, T_cap = 0;
  double* d_time = nullptr;
  double* d_pos = nullptr;
  double* d_rpy = nullptr;
  mc::PoseSeg* d_pose_seg = nullptr;
  // IMU (CSIM:1191-1240)
  int64_t M = 0, M_cap = 0;
  int64_t* d_imu_ts = nullptr;
  double* d_gyro = nullptr;
  mc::ImuSeg* d_imu_seg = nullptr;
  // staging buffer for host<->device layout conversion
  void* d_stage = nullptr;
  size_t stage_bytes = 0;
  // launch knobs / timing
  int32_t max_grid = 0;
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> main_ev, prep_ev;
};

struct mc_batch {
  mc_ctx* ctx = nullptr;
  int32_t F = 0;
  int64_t N = 0;    // valid points
  int64_t P = 0;    // padded points (poff[F])
  int64_t cap = 0;  // column stride (>= P, multiple of 64)
  std::vector<int64_t> counts, poff, doff;
  int32_t n_tiles = 0;
  float* d_cols = nullptr;    // x | y | z | intensity, each `cap` floats
  int32_t* d_t = nullptr;     // t_ns (optional)
  int64_t* d_counts = nullptr;
  int64_t* d_poff = nullptr;
  int64_t* d_doff = nullptr;
  mc::Tile* d_tiles = nullptr;
  double* d_frame_time = nullptr;
  int64_t* d_frame_start = nullptr;
  float4* d_frame_tbl = nullptr;   // 3 float4 per frame (R row, t)
  int2* d_trange = nullptr;        // per-frame [min, max] t_ns (valid when trange_valid)
  mc::FrameWin* d_fwin = nullptr;  // per-frame segment window (k_prep output)
  void* d_frec = nullptr;          // 2 frame-specialised pose/IMU records per frame
  double* d_partial = nullptr;
  bool has_times = false, has_starts = false, trange_valid = false;
};
