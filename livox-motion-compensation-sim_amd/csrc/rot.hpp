// rot.hpp — host-only rotation bases, bit-identical to what the reference computes.
//
// The reference builds every frame's rotation with scipy (LMC:726, LMC:774:
// Rotation.from_euler('xyz', rpy).as_matrix(); scipy 1.15.3, the version in this image).  scipy
// composes three elementary quaternions (extrinsic x -> y -> z: q = qz * qy * qx, scalar last) and
// converts the unnormalised product to a matrix.  euler_xyz_scipy repeats that arithmetic operation
// for operation (glibc sin / cos, no fused multiply-add, rot.cpp is built with -ffp-contract=off
// and -fno-builtin so the compiler neither contracts nor merges sin / cos into sincos, which
// rounds differently), so R is equal bit for bit to scipy's for any angles
// (tests/test_host.py::test_rotation_basis_bitwise_equals_scipy).
//
// With that R, the float64 row kernels reproduce numpy's matmul accumulation (an ascending FMA
// chain per output, then the translation added separately) and their outputs equal the
// reference's float64 values exactly ("Float64 rows").
#pragma once
#include <cstdint>

namespace mcrot {

// R (row-major 3x3) of Rotation.from_euler('xyz', [roll, pitch, yaw]).as_matrix()
void euler_xyz_scipy(const double rpy[3], double R[9]);

// per-frame 12-double pose rows {R row-major (9) | t (3)} of the reference's frame loop
// (LMC:804-812): idx = clamp(searchsorted(time, t_frame, 'left'), 0, T-1) for
// pose_select 0, idx = f for pose_select 1; R of rpy[idx], t = pos[idx]
void frame_poses(const double* time, const double* pos, const double* rpy, int64_t T, const double* frame_time,
                 int32_t F, int pose_select, double* pose12);

}  // namespace mcrot
