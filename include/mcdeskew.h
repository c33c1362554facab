/*
 * mcdeskew.h — C-ABI of the MI355X (gfx950) LiDAR motion-compensation library.
 *
 * This is the drop-in boundary for the reference's hot path.
 * The reference is pure Python, so the "FFI" a maintainer binds is ctypes:
 * every entry point takes plain pointers, sizes and ints, never a torch or
 * numpy type.  The Python host layer (livox-motion-compensation-sim_amd/)
 * mirrors the reference's own methods on top of these calls:
 *
 *   reference (file:line)                                      replaced by
 *   ---------------------------------------------------------  -----------------------------
 *   LiDARMotionSimulator.transform_pointcloud  LMC:772-776     mc_transform_pointcloud_f64 (one
 *                                                              call, host arrays, float64), or
 *                                                              mc_batch_upload_aos_f64 +
 *                                                              mc_deskew(MC_MODE_FRAME,
 *                                                              MC_POSE_DIRECT) +
 *                                                              mc_batch_download_aos_f64
 *   run_simulation pose selection + hot loop   LMC:802-832     mc_set_trajectory +
 *                                                              mc_batch_set_frame_times +
 *                                                              mc_deskew(MC_MODE_FRAME,
 *                                                              MC_POSE_SEARCHSORTED)
 *   save_results merge (np.vstack)             LMC:887-889     blocked-CSR batch layout;
 *                                                              mc_comm_gather_batch (multi-GPU)
 *   MotionCompensator.compensate_point_cloud   CSIM:1435-1480  mc_set_imu + mc_deskew_points_f64(MC_MODE_IMU)
 *                                                              (host float64 rows), or mc_deskew(MC_MODE_IMU)
 *                                                              on a device batch
 *     _interpolate_imu_data                    CSIM:1482-1516    (per-point gyro LERP in-kernel)
 *     _create_rotation_matrix                  CSIM:1518-1536    (R_xyz(theta)^T in-kernel)
 *   (build-added)                          mc_deskew(MC_MODE_POSE_SLERP)
 *
 * LMC = lidar_motion_compensation.py, CSIM = livox_mid70_complete_simulator.py.
 *
 * Conventions
 *  - Every function returns int: 0 = MC_OK, < 0 = error code; the message of the
 *    last failure on the calling thread is returned by mc_last_error().
 *  - The caller owns host buffers; a context owns device buffers; no host
 *    pointer is retained after a call returns.
 *  - All device work of a context is ordered on the context's own HIP stream.
 *    Calls that return host data synchronise that stream before returning;
 *    mc_deskew is asynchronous (mc_sync() waits for it).
 *  - One context per thread and device.
 *
 * Device layout of a batch ("blocked CSR"): n_frames ragged
 * frames; frame f holds count[f] points at padded indices [poff[f], poff[f]+count[f]);
 * poff[f] is a multiple of 256, so every frame starts on a block.  Block k holds
 * points 256k..256k+255 as C runs of 256 values: x, y, z, intensity (float32) and,
 * with MC_BATCH_WITH_TIME, t_ns (int32, nanoseconds since the frame start).
 */
#ifndef MCDESKEW_H_
#define MCDESKEW_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_ABI_VERSION 1

/* status codes */
#define MC_OK 0
#define MC_ERR_INVALID -1   /* bad argument / shape: Python maps to ValueError   */
#define MC_ERR_HIP -2       /* HIP runtime failure                                */
#define MC_ERR_NOMEM -3     /* device allocation failed                           */
#define MC_ERR_STATE -4     /* missing prerequisite (e.g. no trajectory uploaded) */
#define MC_ERR_INDEX -5     /* column count < 4: Python maps to IndexError (LMC:776) */
#define MC_ERR_COMM -6      /* RCCL failure                                       */
#define MC_ERR_SPACE -7     /* output buffer too small (the size needed is reported) */

/* deskew modes */
#define MC_MODE_FRAME 0      /* Path A: one SE(3) pose per frame, p' = R(rpy) p + t   (LMC:772-776)    */
#define MC_MODE_POSE_SLERP 1 /* per point: quaternion SLERP + position LERP of the pose table at
                                t_frame + t_ns*1e-9, then p' = R(q) p + pos       */
#define MC_MODE_IMU 2        /* Path B: per point gyro LERP, theta = w*dt, p' = R_xyz(theta)^T p
                                                                                 (CSIM:1435-1536) */

/* pose selection for MC_MODE_FRAME */
#define MC_POSE_SEARCHSORTED 0 /* idx = clamp(searchsorted(time, t_frame, 'left'), 0, T-1)  LMC:804-806 */
#define MC_POSE_DIRECT 1       /* frame f uses trajectory row f (explicit per-frame transformation)   */

/* batch creation flags */
#define MC_BATCH_WITH_TIME 1u  /* allocate the t_ns column (needed by SLERP / IMU modes) */
/* Keep the ASCII PCD text length (LMC:948) of every 256-point block beside the columns: the
 * kernels that write the batch's x|y|z|intensity (mc_deskew / mc_deskew_steps into it, the stager
 * mc_batch_upload_aos_f64 / mc_batch_stage_aos_f64_device, mc_scan_emit) also write those sums, so
 * mc_pcd_encode_batch skips its measure pass.  Any other write of the columns (column uploads,
 * synth, affine, gathers, mc_tune_order) marks the sums stale and the encoder measures again. */
#define MC_BATCH_WITH_PCD_LEN 2u

typedef struct mc_ctx mc_ctx;
typedef struct mc_batch mc_batch;
typedef struct mc_comm mc_comm;

/* ---- library / context ------------------------------------------------- */
int mc_abi_version(void);
const char* mc_last_error(void);
int mc_device_count(int* count);
/* PCI bus id ("dddd:bb:dd.f") of a visible device: tells ranks that share one GPU apart from
 * ranks on distinct GPUs (bench.py counts devices, not ranks) */
int mc_device_pci_bus_id(int device, char* out, int len);
int mc_create(int device, mc_ctx** out);
int mc_destroy(mc_ctx* ctx);
int mc_sync(mc_ctx* ctx);

/* ---- pose sources (copied to device; replace any previous table) ------- */
/* trajectory table of LMC:361-428: time (T,), position_gps (T,3), orientation_imu (T,3) rad,
 * all float64 C-contiguous.  time must be non-decreasing. */
int mc_set_trajectory(mc_ctx* ctx, int64_t n_poses, const double* time, const double* position,
                      const double* rpy);
/* IMU samples of CSIM:1191-1240: timestamp (M,) int64 ns, gyro (M,3) rad/s float64.
 * timestamps must be non-decreasing (duplicates allowed). */
int mc_set_imu(mc_ctx* ctx, int64_t n_samples, const int64_t* timestamp_ns, const double* gyro);

/* ---- batches ------------------------------------------------------------ */
int mc_batch_create(mc_ctx* ctx, int32_t n_frames, const int64_t* counts, uint32_t flags,
                    mc_batch** out);
int mc_batch_destroy(mc_batch* b);
int mc_batch_info(const mc_batch* b, int64_t* n_points, int64_t* padded_points, int32_t* n_frames,
                  int32_t* n_tiles);
/* padded frame offsets (n_frames+1 entries) as laid out on the device */
int mc_batch_padded_offsets(const mc_batch* b, int64_t* poff_out);
/* 1 when the batch's per-block PCD text sums describe its current columns (MC_BATCH_WITH_PCD_LEN
 * and the last write of the columns produced them), else 0 */
int mc_batch_pcd_len_current(const mc_batch* b, int32_t* current);
/* per-frame reference time in seconds (LMC:792-793 lidar_times) for SEARCHSORTED / SLERP */
int mc_batch_set_frame_times(mc_batch* b, const double* t_frame);
/* per-frame start timestamp in ns (CSIM:2049 frame['timestamp']) for MC_MODE_IMU */
int mc_batch_set_frame_start_ns(mc_batch* b, const int64_t* start_ns);

/* host dense AoS (N, ld) float64, columns 0..3 = x,y,z,intensity  ->  device SoA float32.
 * ld < 4 -> MC_ERR_INDEX (mirrors points[:, 3] in LMC:776). */
int mc_batch_upload_aos_f64(mc_batch* b, const double* aos, int64_t ld);
/* host dense columns (float32, N each); any pointer may be NULL to leave that column */
int mc_batch_upload_columns_f32(mc_batch* b, const float* x, const float* y, const float* z,
                                const float* intensity);
int mc_batch_upload_time_ns(mc_batch* b, const int32_t* t_ns);
/* device SoA float32 -> host dense AoS (N,4) float64 (the (N,4) f64 layout LMC:776 returns) */
int mc_batch_download_aos_f64(mc_batch* b, double* aos_out);
/* frames [f0, f1) only: (doff[f1] - doff[f0], 4) float64 rows (spot checks of batches too large
 * to bring back whole, e.g. BASELINE config 5's 1.2 G points) */
int mc_batch_download_frames_aos_f64(mc_batch* b, int32_t f0, int32_t f1, double* aos_out);
int mc_batch_download_columns_f32(mc_batch* b, float* x, float* y, float* z, float* intensity);
int mc_batch_download_time_ns(mc_batch* b, int32_t* t_ns);

/* ---- device buffers and the device-side stager ---------------------- */
/* The stager pair converts the reference's (N,4) float64 AoS (LMC:770 in, LMC:776 out) to and
 * from the batch's float32 SoA columns without leaving HBM; both are asynchronous on the ctx
 * stream and timed under mc_timing_read_layout. */
int mc_device_alloc(mc_ctx* ctx, int64_t bytes, void** dptr);
int mc_device_free(mc_ctx* ctx, void* dptr);
int mc_memcpy_h2d(mc_ctx* ctx, void* dptr, const void* host, int64_t bytes);
int mc_memcpy_d2h(mc_ctx* ctx, void* host, const void* dptr, int64_t bytes);
int mc_memcpy_d2d(mc_ctx* ctx, void* dst, const void* src, int64_t bytes);
int mc_batch_stage_aos_f64_device(mc_batch* b, const double* d_aos, int64_t ld);
int mc_batch_fetch_aos_f64_device(mc_batch* b, double* d_aos);
int mc_timing_read_layout(mc_ctx* ctx, double* ms_total, int64_t* launches);

/* ---- scan_environment, the step before the path (LMC:701-770) ----------- */
/* scene points (n, ld>=4) float64 [x, y, z, intensity, ...], copied to the device */
int mc_set_environment(mc_ctx* ctx, int64_t n, const double* env, int64_t ld);
/* Pass 1 for F frames: sensor pose per frame from the trajectory (pose_select as mc_deskew's
 * frame mode; frame_times used by MC_POSE_SEARCHSORTED), visibility of every scene point,
 * params = {range_min, range_max, fov_horizontal, fov_vertical} (degrees, full angles),
 * systematic subsample to points_per_frame.  counts_out[F] = points each frame's scan keeps. */
int mc_scan_count(mc_ctx* ctx, int32_t n_frames, const double* frame_times, int pose_select,
                  const double* params, int64_t points_per_frame, int64_t* counts_out);
/* Pass 2: writes the scans into `out` (created with counts_out as frame counts) as sensor-frame
 * x,y,z + noise, intensity.  noise: (sum(counts), 3) float64 drawn by the caller in frame order
 * (LMC:767 np.random.normal), or NULL for noise-free scans. */
int mc_scan_emit(mc_ctx* ctx, mc_batch* out, const double* noise);
/* Pass 2 into the reference's own float64 arrays instead of a float32 batch: d_local receives every
 * frame's scan_environment output (LMC:770: sensor-frame x, y, z + noise, intensity) and d_aligned
 * (may be NULL) the frame loop's transform_pointcloud of it with the same pose (LMC:826-831), as
 * device (N, 4) float64 rows, frames back to back (N = sum of counts_out).  Bit-identical to the
 * reference's values: the pose's R is scipy's (mc_rotation_from_euler_xyz) and every product sum
 * accumulates as numpy's matmul does.  Synchronous. */
int mc_scan_emit_f64(mc_ctx* ctx, const double* noise, double* d_local, double* d_aligned);
int mc_timing_read_scan(mc_ctx* ctx, double* ms_total, int64_t* launches);

/* ---- output codecs, encoded from a device (N, ld) float64 AoS cloud whose
 * frames lie back to back (counts[f] rows each): the array layout the reference hands its writers.
 * Both are synchronous and timed under mc_timing_read_codec. ------------------------------------ */
/* LVX v1.1 layout (LMC:113-132): byte offset of every frame; frame_pos[F] = file size. Host only. */
int mc_lvx_layout(int32_t n_frames, const int64_t* counts, int64_t* frame_pos);
/* The whole LVX v1.1 file of LivoxLVXWriter.write_compatible_lvx (LMC:57-272) into d_out
 * (>= frame_pos[F] bytes, 2-byte aligned): 88-byte file header, per frame a 24-byte header
 * (offset, next offset, frame_ids[f]) and 96-point packages stamped timestamp_ns[f]
 * (= int(timestamp * 1e9), LMC:176).  ld >= 3; has_intensity[f] == 0 gives reflectivity 128
 * (LMC:268); has_intensity NULL means (ld > 3).  A NaN coordinate or intensity -> MC_ERR_INVALID
 * (the reference's int(nan) fails its write). */
int mc_lvx_encode(mc_ctx* ctx, const double* d_aos, int64_t ld, int32_t n_frames, const int64_t* counts,
                  const uint64_t* frame_ids, const uint64_t* timestamp_ns, const uint8_t* has_intensity,
                  void* d_out, int64_t out_bytes);
/* ASCII PCD point lines of save_pcd (LMC:946-948, "%.6f %.6f %.6f %.6f\n", Python's correctly
 * rounded formatting) for F clouds, back to back in d_out; body_pos[F+1] receives each cloud's byte
 * offset (body_pos[F] = total).  If out_bytes < total: MC_ERR_SPACE, body_pos filled, nothing
 * written.  |value| >= 2^107 -> MC_ERR_INVALID (beyond the device formatter). */
int mc_pcd_encode(mc_ctx* ctx, const double* d_aos, int64_t ld, int32_t n_frames, const int64_t* counts,
                  void* d_out, int64_t out_bytes, int64_t* body_pos);
/* The same two encoders reading a batch's own float32 columns in HBM (frames = the batch's frames,
 * 4 columns, intensity present): the bytes mc_lvx_encode / mc_pcd_encode produce from the batch's
 * values widened to float64 (mc_batch_fetch_aos_f64_device), without that 48 B/point pass and
 * with 16 instead of 32 B/point read.  The writers behind save_results (LMC:887-921) and the
 * LVX export (LMC:24-272) on a device-resident, deskewed batch. */
int mc_lvx_encode_batch(mc_ctx* ctx, const mc_batch* b, const uint64_t* frame_ids, const uint64_t* timestamp_ns,
                        void* d_out, int64_t out_bytes);
int mc_pcd_encode_batch(mc_ctx* ctx, const mc_batch* b, void* d_out, int64_t out_bytes, int64_t* body_pos);
/* Deskew -> ASCII PCD in one call: mc_deskew(in -> out) (out != in), whose kernel also sums each
 * output block's text bytes, then the PCD lines of out as mc_pcd_encode_batch writes them, with no
 * separate measure pass over out (the reference's LMC:831 -> 887-889 -> 932-948 sequence on
 * device-resident frames; a block holding a value beyond the packed formatter, |v| >= 4294 / NaN /
 * inf, falls back to the measure pass).  MC_ERR_SPACE as mc_pcd_encode_batch: out is deskewed and
 * body_pos filled, no text written.  The deskew kernel is timed under mc_timing_read, the writer
 * under mc_timing_read_codec. */
int mc_deskew_pcd(mc_ctx* ctx, const mc_batch* in, mc_batch* out, int mode, int pose_select, void* d_out,
                  int64_t out_bytes, int64_t* body_pos);
int mc_timing_read_codec(mc_ctx* ctx, double* ms_total, int64_t* launches);

/* Synthetic Mid-70 frames generated on the device (counter-hash RNG, bit-identical to
 * oracle/synth.py): frame f uses seed  seed + frame_id_base + f. */
int mc_batch_synth(mc_batch* b, uint64_t seed, int64_t frame_id_base);
/* float64 sums of x, y, z, intensity, t_ns over the valid points (deterministic order) */
int mc_batch_checksum(mc_batch* b, double* sums5);

/* ---- the hot path --------------------------------------------------------- */
/* out must have the same frame counts as in (it may be the same batch: in-place). */
int mc_deskew(mc_ctx* ctx, const mc_batch* in, mc_batch* out, int mode, int pose_select);

/* Measure, on this device, which sub-tile order streams the mode's deskew kernel faster for batches
 * shaped like `in` (dealt over the 8 XCDs vs XCD-contiguous: the faster one differs between MI355X
 * boxes by up to 7 %) and use it for every later launch of that mode on batches of the same padded
 * size.  Runs the kernel `launches` times per order and round (in -> out, out != in; the results do
 * not depend on the order), alternating the orders over `rounds`.  us_out[2] (may be NULL) receives
 * the median microseconds per launch of {dealt, XCD-contiguous}; *chosen (may be NULL) the order
 * kept (0 / 1; -1 for an empty batch): the mode's default order unless the other one is at least
 * 1 % faster.  Synchronous. */
int mc_tune_order(mc_ctx* ctx, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t launches,
                  int32_t rounds, double* us_out, int32_t* chosen);
/* n_steps consecutive mc_deskew calls (same arguments), LMC:802-832 n times over one batch, as
 * n + 1 launches: step 0's pose prep, then n deskew launches of which the first n - 1 also run the
 * next step's prep in their first workgroups (every step runs its own prep, one launch ahead, into
 * the other table half).  sample_every > 0 puts timing events around the kernels of every
 * sample_every-th step (read by mc_timing_read).  Asynchronous. */
int mc_deskew_steps(mc_ctx* ctx, const mc_batch* in, mc_batch* out, int mode, int pose_select, int32_t n_steps,
                    int32_t sample_every);

/* One call of transform_pointcloud (LMC:772-776) on host arrays: points (n, ld>=4) float64 rows,
 * rpy / translation (3,) float64 -> out (n, 4) float64 = [R p + t, intensity], bit-identical to the
 * reference's float64 result (R as scipy's from_euler('xyz').as_matrix(), numpy's matmul
 * accumulation).  Below 32768 rows the kernel reads and writes pinned, device-mapped host memory (no
 * DMA round trips); a lone ~1.6k-row call still costs ~14 us against numpy's ~9.5 (INTEGRATION.md:
 * batch the frames).  ld < 4 -> MC_ERR_INDEX. */
int mc_transform_pointcloud_f64(mc_ctx* ctx, const double* points, int64_t n, int64_t ld, const double* rpy,
                                const double* translation, double* out);

/* Host only (no device): R (n, 3, 3) row-major of Rotation.from_euler('xyz', rpy[i]).as_matrix() for
 * each rpy (n, 3) — scipy 1.15's arithmetic repeated operation for operation, equal bit for bit.  The
 * per-frame rotation basis of every float64 path (LMC:726, 774). */
int mc_rotation_from_euler_xyz(int64_t n, const double* rpy, double* R);

/* The per-point modes on the reference's own float64 data (no float32 staging): MotionCompensator.
 * compensate_point_cloud / apply_motion_compensation (CSIM:1435-1480, 2086-2105) for MC_MODE_IMU,
 * the per-point SLERP deskew for MC_MODE_POSE_SLERP.  points (N, ld >= 3) float64 rows, frames back
 * to back (counts[f] rows each); t_ns (N,) int64 = each point's time minus its frame's start (any
 * int64: no int32 limit here); frame_times[F] (s, SLERP: t = frame_times[f] + t_ns * 1e-9) or
 * frame_start_ns[F] (IMU: the point's timestamp = frame_start_ns[f] + t_ns, CSIM:1447, 1454).  out
 * (N, 4) float64 = x', y', z' computed in float64 end to end, column 3 = points[:, 3] (0 when ld == 3).
 * Pose / IMU tables from mc_set_trajectory / mc_set_imu.  ld < 3 -> MC_ERR_INDEX.  Synchronous. */
int mc_deskew_points_f64(mc_ctx* ctx, int mode, int32_t n_frames, const int64_t* counts, const double* points,
                         int64_t ld, const int64_t* t_ns, const double* frame_times, const int64_t* frame_start_ns,
                         double* out);

/* The frame loop (LMC:802-832) on host arrays: frames[f] (counts[f], lds[f] >= 4) float64 rows
 * -> outs[f] (counts[f], 4) float64, pose per frame from the uploaded trajectory (pose_select as
 * mc_deskew's frame mode; frame_times for MC_POSE_SEARCHSORTED), float64 math, one launch over
 * all frames on pinned, device-mapped host memory (host copies on 16 threads above 8 MB). */
int mc_align_frames_host_f64(mc_ctx* ctx, int32_t n_frames, const double* const* frames, const int64_t* counts,
                             const int64_t* lds, const double* frame_times, int pose_select, double* const* outs);

/* CoordinateTransformer.transform_points (CSIM:153-233) / _transform_coordinates (CSIM:2107-2163):
 * p' = A p + b with one 3x4 [A | b] matrix (row-major float64, 12 values) for all frames
 * (n_mats == 1) or one per frame (n_mats == n_frames).  w_column != 0: the intensity column is the
 * homogeneous w of (N,4) input (p' = A p + b w, CSIM:226-229).  The 4th column passes through.
 * Synchronous; timed with the deskew kernels (mc_timing_read main). */
int mc_transform_affine(mc_ctx* ctx, const mc_batch* in, mc_batch* out, int32_t n_mats, const double* mats,
                        int w_column);
/* The same on the caller's float64 rows, bit-identical to the reference (numpy's accumulation of
 * (T @ points_h.T).T, CSIM:230): rows (N, ld) with ld 3 (w = 1, CSIM:223-225) or 4 (the 4th column is
 * w, CSIM:227), frames back to back (counts[f] rows); mats = 3x4 [A | b] row-major, 1 or n_frames of
 * them; out (N, 3) float64 (CSIM:233).  A frame is one transform_points call: numpy sums a one-row
 * call (a matrix-vector product) in another order than a larger one, and both are repeated.  per_row
 * = MC_AFFINE_PER_ROW treats every row as its own call — _transform_coordinates' per-point loop
 * (CSIM:2117-2141); MC_AFFINE_TRANSLATE adds b to each row's x, y, z and ignores A — that loop's UTM
 * branch, point + [utm_x, utm_y, 0] (CSIM:2132), one rounding per coordinate (no products, so a
 * non-finite coordinate does not spread to the others).  Synchronous. */
#define MC_AFFINE_PER_FRAME 0
#define MC_AFFINE_PER_ROW 1
#define MC_AFFINE_TRANSLATE 2
int mc_affine_rows_f64(mc_ctx* ctx, int32_t n_frames, const int64_t* counts, const double* rows, int64_t ld,
                       int32_t n_mats, const double* mats, int per_row, double* out);

/* HIP-event timing of the hot kernels (main deskew kernel and the pose-prep kernel) */
int mc_timing_enable(mc_ctx* ctx, int enable);
int mc_timing_read(mc_ctx* ctx, double* main_ms_total, int64_t* main_launches,
                   double* prep_ms_total, int64_t* prep_launches);
/* the main kernels' event times one by one (ms, in launch order; up to cap of them, *n = how many
 * were pending); those events are released (the prep / layout / codec ones stay for mc_timing_read) */
int mc_timing_read_each(mc_ctx* ctx, double* main_ms, int64_t cap, int64_t* n);
/* the same timed deskew launches' own execution spans (us, launch order; up to cap, *n = how many):
 * first workgroup start to last workgroup end on the wall clock, without the dispatch gap a start
 * event ahead of a launch includes; released */
int mc_timing_read_spans(mc_ctx* ctx, double* us, int64_t cap, int64_t* n);
/* kernel tuning knobs: 0 keeps the default */
int mc_set_launch(mc_ctx* ctx, int32_t max_grid);

/* ---- multi-GPU merged-cloud gather over RCCL/xGMI (LMC:887-889 vstack) ---- */
int mc_comm_unique_id(char id_out[128]);
int mc_comm_init(mc_ctx* ctx, int nranks, int rank, const char id[128], mc_comm** out);
int mc_comm_destroy(mc_comm* comm);
/* ragged gather of every rank's batch columns (x,y,z,intensity; blocked layout) into `merged`
 * on `root`, in rank order (== np.vstack of the frame-ordered shards).  `merged` is ignored on
 * non-root ranks and on root must have been created with the concatenated frame counts. */
int mc_comm_gather_batch(mc_comm* comm, const mc_batch* local, int root, mc_batch* merged);
int mc_comm_allreduce_max_f64(mc_comm* comm, double* values, int64_t n);
/* Host only (no device work): the plan mc_comm_gather_batch follows for n ranks whose shards hold
 * padded[q] points of columns[q] (4 or 5) values per block into a merged batch of merged_padded
 * points and merged_columns columns: offset_out[q] = the shard's first padded point in the merged
 * batch (rank order == np.vstack order, LMC:887-889), stage_offset_out[q] = its value offset in the
 * root's staging area (-1: received in place), *stage_values_out = staging size.  Invalid plans
 * (sizes that do not add up, a shard with fewer columns than the merged batch) -> MC_ERR_INVALID. */
int mc_gather_plan(int32_t nranks, int32_t root, const int64_t* padded, const int64_t* columns, int64_t merged_padded,
                   int32_t merged_columns, int64_t* offset_out, int64_t* stage_offset_out, int64_t* stage_values_out);
/* The same merge inside one process: n shard batches of one context into `merged` (created with the
 * concatenated frame counts), shard `root` playing the root's own batch and device copies standing
 * in for the RCCL receives — the plan, staging and re-pitch of mc_comm_gather_batch.  Synchronous. */
int mc_gather_batches(mc_ctx* ctx, int32_t n, const mc_batch* const* shards, int32_t root, mc_batch* merged);

#ifdef __cplusplus
}
#endif
#endif /* MCDESKEW_H_ */
