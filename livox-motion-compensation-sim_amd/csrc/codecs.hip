// codecs.hip — host side of the output codecs in include/mcdeskew.h:
// LVX v1.1 files (LMC:24-272) and ASCII PCD bodies (LMC:932-948) encoded on the device from a
// device-resident (N, ld) float64 AoS cloud.
#include "codecs.hpp"
#include "hostutil.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace mc;

namespace {

int codec_scratch(mc_ctx* c, size_t bytes, char** out) {
  if (bytes > c->codec_bytes) {
    if (c->d_codec) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->d_codec); c->d_codec = nullptr; }
    c->codec_bytes = 0;
    HIPCHK(hipMalloc(&c->d_codec, bytes));
    c->codec_bytes = bytes;
  }
  if (!c->d_codec_err) {
    if (int r = dev_alloc(&c->d_codec_err, 1)) return r;
  }
  *out = static_cast<char*>(c->d_codec);
  return MC_OK;
}

// the 88 bytes ahead of the first frame: public header (LMC:86-101), private header (LMC:104-110),
// device info block (LMC:146-172)
void lvx_file_header(uint8_t h[kLvxFileHdr]) {
  std::memset(h, 0, kLvxFileHdr);
  std::memcpy(h, "livox_tech", 10);
  h[16] = 1; h[17] = 1;
  const uint32_t magic = 0xAC0EA767u, dur = 50;
  std::memcpy(h + 20, &magic, 4);
  std::memcpy(h + 24, &dur, 4);
  h[28] = 1;                                       // device count
  std::memcpy(h + 29, "3GGDJ6K00200101", 15);      // LiDAR SN (16 B, NUL-terminated)
  h[29 + 33] = 1;                                  // device type
}

int check_frames(int32_t F, const int64_t* counts, std::vector<int64_t>& doff) {
  CHECK_ARG(F >= 0, "n_frames must be >= 0");
  CHECK_ARG(F == 0 || counts, "counts is NULL");
  doff.assign((size_t)F + 1, 0);
  for (int32_t f = 0; f < F; ++f) {
    CHECK_ARG(counts[f] >= 0, "negative frame size at frame %d", f);
    CHECK_ARG(counts[f] < ((int64_t)1 << 31), "frame %d has %lld points (the encoders take < 2^31 per frame)", f,
              (long long)counts[f]);
    doff[f + 1] = doff[f] + counts[f];
  }
  return MC_OK;
}

template <typename T>
size_t put(std::vector<uint8_t>& blob, const T* src, size_t n) {
  const size_t at = (blob.size() + 7) & ~size_t(7);
  blob.resize(at + n * sizeof(T));
  if (n) std::memcpy(blob.data() + at, src, n * sizeof(T));
  return at;
}

// where the points come from: a device (N, ld) float64 AoS array or a batch's blocked columns
struct Source {
  const double* aos = nullptr;
  int64_t ld = 4;
  const mc_batch* batch = nullptr;
};

CodecFrames frames_of(const Source& src, const int64_t* d_doff, const int64_t* d_units, int32_t F, int64_t n_units) {
  CodecFrames cf;
  cf.aos = src.aos;
  cf.ld = src.batch ? 4 : src.ld;
  cf.cols = src.batch ? src.batch->d_cols : nullptr;
  cf.C = src.batch ? src.batch->C : 0;
  cf.poff = src.batch ? src.batch->d_poff : nullptr;
  cf.doff = d_doff;
  cf.unit_off = d_units;
  cf.F = F;
  cf.n_units = n_units;
  cf.frames_per_unit = n_units > 0 ? (double)F / (double)n_units : 0.0;
  return cf;
}

int lvx_encode(mc_ctx* c, const Source& src, int32_t F, const int64_t* counts, const uint64_t* frame_ids,
               const uint64_t* ts_ns, const uint8_t* has_int, void* d_out, int64_t out_bytes);
int pcd_encode(mc_ctx* c, const Source& src, int32_t F, const int64_t* counts, void* d_out, int64_t out_bytes,
               int64_t* body_pos, const int32_t* d_measured = nullptr);

}  // namespace

extern "C" {

int mc_lvx_layout(int32_t F, const int64_t* counts, int64_t* pos) {
  CHECK_ARG(pos, "frame_pos is NULL");
  std::vector<int64_t> doff;
  if (int r = check_frames(F, counts, doff)) return r;
  pos[0] = kLvxFileHdr;
  for (int32_t f = 0; f < F; ++f)
    pos[f + 1] = pos[f] + kLvxFrameHdr + (counts[f] + kLvxPkgPoints - 1) / kLvxPkgPoints * kLvxPkg;
  return MC_OK;
}

int mc_lvx_encode(mc_ctx* c, const double* d_aos, int64_t ld, int32_t F, const int64_t* counts,
                  const uint64_t* frame_ids, const uint64_t* ts_ns, const uint8_t* has_int, void* d_out,
                  int64_t out_bytes) {
  CHECK_ARG(c && d_out, "NULL argument");
  if (ld < 3) return fail(MC_ERR_INDEX, "LVX points need at least 3 columns; got %lld", (long long)ld);
  Source src;
  src.aos = d_aos;
  src.ld = ld;
  return lvx_encode(c, src, F, counts, frame_ids, ts_ns, has_int, d_out, out_bytes);
}

int mc_lvx_encode_batch(mc_ctx* c, const mc_batch* b, const uint64_t* frame_ids, const uint64_t* ts_ns, void* d_out,
                        int64_t out_bytes) {
  CHECK_ARG(c && b && d_out, "NULL argument");
  CHECK_ARG(b->ctx == c, "batch belongs to another context");
  Source src;
  src.batch = b;
  return lvx_encode(c, src, b->F, b->counts.data(), frame_ids, ts_ns, nullptr, d_out, out_bytes);
}

}  // extern "C"

namespace {

int lvx_encode(mc_ctx* c, const Source& src, int32_t F, const int64_t* counts, const uint64_t* frame_ids,
               const uint64_t* ts_ns, const uint8_t* has_int, void* d_out, int64_t out_bytes) {
  std::vector<int64_t> doff;
  if (int r = check_frames(F, counts, doff)) return r;
  CHECK_ARG(F == 0 || (frame_ids && ts_ns), "frame_ids / timestamp_ns are NULL");
  CHECK_ARG(doff[F] == 0 || src.aos || src.batch, "points pointer is NULL");
  CHECK_ARG(((uintptr_t)d_out & 1) == 0, "d_out must be 2-byte aligned");
  std::vector<int64_t> pos((size_t)F + 1), units((size_t)F + 1, 0);
  mc_lvx_layout(F, counts, pos.data());
  if (out_bytes < pos[F])
    return fail(MC_ERR_SPACE, "LVX output needs %lld bytes, buffer has %lld", (long long)pos[F], (long long)out_bytes);
  for (int32_t f = 0; f < F; ++f) units[f + 1] = units[f] + (counts[f] + kLvxUnitPoints - 1) / kLvxUnitPoints;
  const int64_t n_pkg = units[F];   // units of up to kLvxPkgPerWG packages
  CHECK_ARG(n_pkg < (int64_t)INT32_MAX, "too many packages for one launch");
  DeviceGuard g(c->device);

  std::vector<uint8_t> blob;
  const size_t o_doff = put(blob, doff.data(), doff.size());
  const size_t o_unit = put(blob, units.data(), units.size());
  const size_t o_pos = put(blob, pos.data(), (size_t)F + 1);
  const size_t o_ids = put(blob, frame_ids, (size_t)F);
  const size_t o_ts = put(blob, ts_ns, (size_t)F);
  const size_t o_hi = has_int ? put(blob, has_int, (size_t)F) : 0;
  char* d = nullptr;
  if (int r = codec_scratch(c, blob.size(), &d)) return r;
  HIPCHK(hipMemcpyAsync(d, blob.data(), blob.size(), hipMemcpyHostToDevice, c->stream));
  uint8_t hdr[kLvxFileHdr];
  lvx_file_header(hdr);
  HIPCHK(hipMemcpyAsync(d_out, hdr, kLvxFileHdr, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_codec_err, 0, sizeof(int), c->stream));

  LvxArgs a;
  a.src = frames_of(src, reinterpret_cast<const int64_t*>(d + o_doff), reinterpret_cast<const int64_t*>(d + o_unit),
                    F, n_pkg);
  a.frame_pos = reinterpret_cast<const int64_t*>(d + o_pos);
  a.frame_id = reinterpret_cast<const uint64_t*>(d + o_ids);
  a.ts_ns = reinterpret_cast<const uint64_t*>(d + o_ts);
  a.has_int = has_int ? reinterpret_cast<const uint8_t*>(d + o_hi) : nullptr;
  a.out = static_cast<char*>(d_out);
  a.err = c->d_codec_err;
  a.order = src.batch ? src.batch->hot_order ^ 1 : 0;   // start where the last kernel over the batch ended
  {
    TimedRegion tr(c, &c->codec_ev, c->stream);
    // frame headers: each frame's first unit writes its own, so this launch only when a frame has no
    // points (and therefore no unit)
    const bool empty_frame = std::any_of(counts, counts + F, [](int64_t n) { return n == 0; });
    if (F > 0 && empty_frame)
      hipLaunchKernelGGL(k_lvx_frames, dim3((F + kCodecBlock - 1) / kCodecBlock), dim3(kCodecBlock), 0, c->stream,
                         a, (int64_t)0);
    if (n_pkg > 0) {
      hipLaunchKernelGGL(k_lvx_packages, dim3((uint32_t)n_pkg), dim3(kCodecBlock), 0, c->stream, a);
      if (src.batch) src.batch->hot_order = a.order;
    }
  }
  HIPCHK(hipGetLastError());
  int err = 0;
  HIPCHK(hipMemcpyAsync(&err, c->d_codec_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (err) return fail(MC_ERR_INVALID, "cannot convert float NaN to integer (NaN coordinate or intensity)");
  return MC_OK;
}

}  // namespace

extern "C" {

int mc_pcd_encode(mc_ctx* c, const double* d_aos, int64_t ld, int32_t F, const int64_t* counts, void* d_out,
                  int64_t out_bytes, int64_t* body_pos) {
  CHECK_ARG(c && body_pos, "NULL argument");
  if (ld < 4) return fail(MC_ERR_INDEX, "index 3 is out of bounds for axis 0 with size %lld", (long long)ld);
  Source src;
  src.aos = d_aos;
  src.ld = ld;
  return pcd_encode(c, src, F, counts, d_out, out_bytes, body_pos);
}

int mc_pcd_encode_batch(mc_ctx* c, const mc_batch* b, void* d_out, int64_t out_bytes, int64_t* body_pos) {
  CHECK_ARG(c && b && body_pos, "NULL argument");
  CHECK_ARG(b->ctx == c, "batch belongs to another context");
  Source src;
  src.batch = b;
  // MC_BATCH_WITH_PCD_LEN: the kernel that last wrote the columns left their text sums (no measure pass)
  return pcd_encode(c, src, b->F, b->counts.data(), d_out, out_bytes, body_pos,
                    b->pcd_current() ? b->d_pcd_len : nullptr);
}

int mc_deskew_pcd(mc_ctx* c, const mc_batch* in, mc_batch* out, int mode, int pose_select, void* d_out,
                  int64_t out_bytes, int64_t* body_pos) {
  CHECK_ARG(c && in && out && body_pos, "NULL argument");
  CHECK_ARG(out != in, "mc_deskew_pcd needs an output batch other than the input");
  CHECK_ARG(out->ctx == c, "batch belongs to another context");
  DeviceGuard g(c->device);
  if (out->d_pcd_len) {   // MC_BATCH_WITH_PCD_LEN: the deskew writes the batch's own sums
    if (int r = mcimpl::deskew_call(c, in, out, mode, pose_select, nullptr)) return r;
    return mc_pcd_encode_batch(c, out, d_out, out_bytes, body_pos);
  }
  // one text-byte slot per 256-point block of the output batch (= one PCD tile)
  const int64_t blocks = out->P / kBlkPts;
  if (blocks > c->pcd_len_cap) {
    if (c->d_pcd_len) { (void)hipStreamSynchronize(c->stream); dev_free(c->d_pcd_len); c->d_pcd_len = nullptr; }
    c->pcd_len_cap = 0;
    if (int r = dev_alloc(&c->d_pcd_len, (size_t)blocks)) return r;
    c->pcd_len_cap = blocks;
  }
  if (int r = mcimpl::deskew_call(c, in, out, mode, pose_select, blocks > 0 ? c->d_pcd_len : nullptr)) return r;
  Source src;
  src.batch = out;
  return pcd_encode(c, src, out->F, out->counts.data(), d_out, out_bytes, body_pos, c->d_pcd_len);
}

}  // extern "C"

namespace {

// d_measured (mc_deskew_pcd): the tiles' text bytes already written by the deskew kernel that
// produced the batch (pcd_value_len sums per 256-point block = per tile); the measure pass is then
// skipped unless a tile holds a value outside the packed path, whose exact length only the measure
// pass forms.
int pcd_encode(mc_ctx* c, const Source& src, int32_t F, const int64_t* counts, void* d_out, int64_t out_bytes,
               int64_t* body_pos, const int32_t* d_measured) {
  std::vector<int64_t> doff;
  if (int r = check_frames(F, counts, doff)) return r;
  CHECK_ARG(doff[F] == 0 || src.aos || src.batch, "points pointer is NULL");
  std::vector<int64_t> units((size_t)F + 1, 0);
  for (int32_t f = 0; f < F; ++f) units[f + 1] = units[f] + (counts[f] + kPcdBlock - 1) / kPcdBlock;
  const int64_t n_tiles = units[F];
  CHECK_ARG(n_tiles < (int64_t)INT32_MAX, "too many tiles for one launch");
  if (n_tiles == 0) {
    std::fill(body_pos, body_pos + F + 1, (int64_t)0);
    return MC_OK;
  }
  DeviceGuard g(c->device);
  std::vector<uint8_t> blob;
  const size_t o_doff = put(blob, doff.data(), doff.size());
  const size_t o_unit = put(blob, units.data(), units.size());
  const size_t o_tb = put(blob, (const int32_t*)nullptr, 0);
  blob.resize(o_tb + (size_t)n_tiles * sizeof(int32_t));
  const size_t o_tp = put(blob, (const int64_t*)nullptr, 0);
  blob.resize(o_tp + (size_t)n_tiles * sizeof(int64_t));
  char* d = nullptr;
  if (int r = codec_scratch(c, blob.size(), &d)) return r;
  HIPCHK(hipMemcpyAsync(d, blob.data(), o_tb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_codec_err, 0, sizeof(int), c->stream));
  PcdArgs a;
  a.src = frames_of(src, reinterpret_cast<const int64_t*>(d + o_doff), reinterpret_cast<const int64_t*>(d + o_unit),
                    F, n_tiles);
  a.tile_bytes = reinterpret_cast<int32_t*>(d + o_tb);
  a.tile_pos = reinterpret_cast<const int64_t*>(d + o_tp);
  a.out = static_cast<char*>(d_out);
  a.err = c->d_codec_err;
  // batch source: each pass starts where the previous kernel over the batch ended (stream_unit);
  // fused (d_measured): the write pass follows the deskew kernel directly
  const int hot = src.batch ? src.batch->hot_order : 1;
  a.morder = hot ^ 1;
  a.worder = hot ^ 1;
  std::vector<int32_t> tb((size_t)n_tiles);
  bool measured = false;
  if (d_measured) {
    HIPCHK(hipMemcpyAsync(tb.data(), d_measured, tb.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    measured = std::all_of(tb.begin(), tb.end(), [](int32_t v) { return v >= 0 && v < kPcdSlowValue; });
    if (measured) a.tile_bytes = const_cast<int32_t*>(d_measured);   // the write pass reads it (no slow flags)
  }
  if (!measured) {
    a.worder = a.morder ^ 1;
    {
      TimedRegion tr(c, &c->codec_ev, c->stream);
      const int per = a.src.cols ? kPcdMeasureTiles : kPcdTilesPerWG;   // tiles per measure workgroup
      const dim3 mgrid((uint32_t)((n_tiles + per - 1) / per));
      if (a.src.cols) hipLaunchKernelGGL(k_pcd_measure<true>, mgrid, dim3(kPcdBlock), 0, c->stream, a);
      else hipLaunchKernelGGL(k_pcd_measure<false>, mgrid, dim3(kPcdBlock), 0, c->stream, a);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(tb.data(), a.tile_bytes, tb.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (a.src.cols) {
      // the float32 measure pass only flags tiles with lines outside the packed path: their exact
      // bytes from k_pcd_measure_list (the list rides in the tile-position slots, not yet written)
      HIPCHK(hipStreamSynchronize(c->stream));
      std::vector<int32_t> flagged;
      for (int64_t t = 0; t < n_tiles; ++t)
        if (tb[t] & kPcdSlowTile) flagged.push_back((int32_t)t);
      if (!flagged.empty()) {
        int32_t* d_list = reinterpret_cast<int32_t*>(d + o_tp);
        HIPCHK(hipMemcpyAsync(d_list, flagged.data(), flagged.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                              c->stream));
        {
          TimedRegion tr(c, &c->codec_ev, c->stream);
          hipLaunchKernelGGL(k_pcd_measure_list, dim3((uint32_t)flagged.size()), dim3(kPcdBlock), 0, c->stream, a,
                             (const int32_t*)d_list);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(tb.data(), a.tile_bytes, tb.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                              c->stream));
      }
    }
  }
  int err = 0;
  HIPCHK(hipMemcpyAsync(&err, c->d_codec_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (err) return fail(MC_ERR_INVALID, "a value has |v| >= 2^107, beyond the device %%.6f formatter");
  // tiles holding a line outside the packed path (kPcdSlowTile) go to the byte-path kernel
  std::vector<int64_t> tpos((size_t)n_tiles);
  std::vector<int32_t> slow;
  int64_t run = 0;
  for (int32_t f = 0; f < F; ++f) {
    body_pos[f] = run;
    for (int64_t t = units[f]; t < units[f + 1]; ++t) {
      if (tb[t] & kPcdSlowTile) slow.push_back((int32_t)t);
      tpos[t] = run;
      run += tb[t] & ~kPcdSlowTile;
    }
  }
  body_pos[F] = run;
  if (out_bytes < run)
    return fail(MC_ERR_SPACE, "PCD text needs %lld bytes, buffer has %lld", (long long)run, (long long)out_bytes);
  CHECK_ARG(d_out, "d_out is NULL");
  HIPCHK(hipMemcpyAsync(d + o_tp, tpos.data(), tpos.size() * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  const dim3 grid((uint32_t)((n_tiles + kPcdWriteTiles - 1) / kPcdWriteTiles));
  {
    TimedRegion tr(c, &c->codec_ev, c->stream);
    if (a.src.cols) hipLaunchKernelGGL(k_pcd_write<true>, grid, dim3(kPcdBlock), 0, c->stream, a);
    else hipLaunchKernelGGL(k_pcd_write<false>, grid, dim3(kPcdBlock), 0, c->stream, a);
  }
  if (src.batch) src.batch->hot_order = a.worder;
  HIPCHK(hipGetLastError());
  if (!slow.empty()) {
    // the list rides in the scratch blob's tile-byte slots, which k_pcd_write has finished reading
    // (same stream); the byte path reads no tile bytes
    HIPCHK(hipMemcpyAsync(a.tile_bytes, slow.data(), slow.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                          c->stream));
    TimedRegion tr(c, &c->codec_ev, c->stream);
    hipLaunchKernelGGL(k_pcd_write_bytes, dim3((uint32_t)slow.size()), dim3(kPcdBlock), 0, c->stream, a,
                       (const int32_t*)a.tile_bytes);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

}  // namespace

extern "C" {

int mc_timing_read_codec(mc_ctx* c, double* ms, int64_t* n) {
  CHECK_ARG(c, "ctx is NULL");
  DeviceGuard g(c->device);
  if (int r = sync_all(c)) return r;
  return sum_events(c, c->codec_ev, ms, n);
}

}  // extern "C"
