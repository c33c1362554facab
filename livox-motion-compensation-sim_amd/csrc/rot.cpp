// rot.cpp — see rot.hpp.  Built with -ffp-contract=off -fno-builtin (Makefile): every product and
// sum below is rounded on its own, and sin / cos stay separate glibc calls.
#include "rot.hpp"

#include <algorithm>
#include <cmath>

#include "../../include/mcdeskew.h"

namespace mcrot {
namespace {

// r = p * q (quaternions, scalar last): scipy's _compose_quat_single — cross product first, then
// p.w q.xyz + q.w p.xyz + p x q and p.w q.w - p.xyz . q.xyz, summed left to right
void compose(const double p[4], const double q[4], double r[4]) {
  const double c0 = p[1] * q[2] - p[2] * q[1];
  const double c1 = p[2] * q[0] - p[0] * q[2];
  const double c2 = p[0] * q[1] - p[1] * q[0];
  r[0] = p[3] * q[0] + q[3] * p[0] + c0;
  r[1] = p[3] * q[1] + q[3] * p[1] + c1;
  r[2] = p[3] * q[2] + q[3] * p[2] + c2;
  r[3] = p[3] * q[3] - p[0] * q[0] - p[1] * q[1] - p[2] * q[2];
}

}  // namespace

void euler_xyz_scipy(const double rpy[3], double R[9]) {
  // elementary quaternion of axis 0 (scipy's _make_elementary_quat: cos(a/2) scalar, sin(a/2) on the axis)
  double q[4] = {std::sin(rpy[0] / 2), 0.0, 0.0, std::cos(rpy[0] / 2)};
  for (int ax = 1; ax < 3; ++ax) {
    double e[4] = {0.0, 0.0, 0.0, std::cos(rpy[ax] / 2)};
    e[ax] = std::sin(rpy[ax] / 2);
    double r[4];
    compose(e, q, r);   // extrinsic: the new axis multiplies from the left
    for (int k = 0; k < 4; ++k) q[k] = r[k];
  }
  // scipy's as_matrix on the (unnormalised) quaternion
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
  const double xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
  R[0] = x2 - y2 - z2 + w2;
  R[3] = 2 * (xy + zw);
  R[6] = 2 * (xz - yw);
  R[1] = 2 * (xy - zw);
  R[4] = -x2 + y2 - z2 + w2;
  R[7] = 2 * (yz + xw);
  R[2] = 2 * (xz + yw);
  R[5] = 2 * (yz - xw);
  R[8] = -x2 - y2 + z2 + w2;
}

void frame_poses(const double* time, const double* pos, const double* rpy, int64_t T, const double* frame_time,
                 int32_t F, int pose_select, double* pose12) {
  for (int32_t f = 0; f < F; ++f) {
    int64_t idx = f;
    if (pose_select == 0) {
      // np.searchsorted(time, t, 'left'): the first index whose time is not below t (LMC:804-806)
      // (NaN sorts last in numpy: past the end, then clamped)
      idx = std::isnan(frame_time[f]) ? T : std::lower_bound(time, time + T, frame_time[f]) - time;
      if (idx > T - 1) idx = T - 1;
    }
    double* P = pose12 + 12 * (int64_t)f;
    euler_xyz_scipy(rpy + 3 * idx, P);
    for (int k = 0; k < 3; ++k) P[9 + k] = pos[3 * idx + k];
  }
}

}  // namespace mcrot

namespace mcimpl {
int fail(int code, const char* fmt, ...);
}

extern "C" int mc_rotation_from_euler_xyz(int64_t n, const double* rpy, double* R) {
  if (n < 0) return mcimpl::fail(MC_ERR_INVALID, "negative count %lld", (long long)n);
  if (n > 0 && (!rpy || !R)) return mcimpl::fail(MC_ERR_INVALID, "NULL argument");
  for (int64_t i = 0; i < n; ++i) mcrot::euler_xyz_scipy(rpy + 3 * i, R + 9 * i);
  return MC_OK;
}
