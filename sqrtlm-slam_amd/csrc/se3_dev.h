// se3_dev.h — SE3 / quaternion arithmetic of the g2o pose vertex, usable on
// host and device. Semantics (not code) follow the reference:
//   SE3Quat::exp           Thirdparty/g2o/g2o/types/se3quat.h:223-257
//   SE3Quat::operator*     se3quat.h:104-110, normalizeRotation :280-285
//   VertexSE3Expmap::oplus types_six_dof_expmap.h:73-76 (left update)
// Quaternion layout x, y, z, w (Eigen coeffs order).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace sqlm {

#define SQLM_HD __host__ __device__ __forceinline__

// The pose algebra and the LiDAR numeric Jacobian (central differences with
// delta = 1e-9 amplify one-ulp differences by 5e8) are evaluated without FMA
// contraction so host, device and the reference's x86 build round alike.
#pragma clang fp contract(off)

SQLM_HD void q_normalize_rot(double q[4]) {
  if (q[3] < 0.0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
  const double z = (q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]);
  if (z > 0.0) {
    const double n = sqrt(z);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
  }
}

SQLM_HD void q_mul(const double a[4], const double b[4], double o[4]) {
  const double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  const double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  const double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  const double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

// q * v via uv = 2 (q.vec x v); v + w uv + q.vec x uv
SQLM_HD void q_rotate(const double q[4], const double v[3], double o[3]) {
  double u0 = q[1] * v[2] - q[2] * v[1];
  double u1 = q[2] * v[0] - q[0] * v[2];
  double u2 = q[0] * v[1] - q[1] * v[0];
  u0 += u0; u1 += u1; u2 += u2;
  const double c0 = q[1] * u2 - q[2] * u1;
  const double c1 = q[2] * u0 - q[0] * u2;
  const double c2 = q[0] * u1 - q[1] * u0;
  o[0] = v[0] + q[3] * u0 + c0;
  o[1] = v[1] + q[3] * u1 + c1;
  o[2] = v[2] + q[3] * u2 + c2;
}

SQLM_HD void q_to_mat(const double q[4], double R[9]) {
  const double tx = 2.0 * q[0], ty = 2.0 * q[1], tz = 2.0 * q[2];
  const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
  const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
  const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1.0 - (txx + tyy);
}

SQLM_HD void q_from_mat(const double m[9], double q[4]) {
  double t = (m[0] + m[4]) + m[8];
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m[7] - m[5]) * t;
    q[1] = (m[2] - m[6]) * t;
    q[2] = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[i * 4]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[k * 3 + j] - m[j * 3 + k]) * t;
    q[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
    q[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
  }
}

SQLM_HD void mat3_mul(const double A[9], const double B[9], double C[9]) {
  double T[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) T[r * 3 + c] = A[r * 3] * B[c] + A[r * 3 + 1] * B[3 + c] + A[r * 3 + 2] * B[6 + c];
#pragma unroll
  for (int i = 0; i < 9; ++i) C[i] = T[i];
}

// exp([omega; upsilon]) -> (q, t)
SQLM_HD void se3_exp(const double d[6], double q[4], double t[3]) {
  const double w0 = d[0], w1 = d[1], w2 = d[2];
  const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double Om[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
  double Om2[9], R[9], V[9];
  mat3_mul(Om, Om, Om2);
  if (theta < 0.00001) {
#pragma unroll
    for (int i = 0; i < 9; ++i) { R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + Om[i] + Om2[i]; V[i] = R[i]; }
  } else {
    const double st = sin(theta), ct = cos(theta);
    const double a = st / theta, b = (1.0 - ct) / (theta * theta), c = (theta - st) / (theta * theta * theta);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const double I = (i % 4 == 0) ? 1.0 : 0.0;
      R[i] = (I + a * Om[i]) + b * Om2[i];
      V[i] = (I + b * Om[i]) + c * Om2[i];
    }
  }
  q_from_mat(R, q);
  q_normalize_rot(q);
#pragma unroll
  for (int r = 0; r < 3; ++r) t[r] = V[r * 3] * d[3] + V[r * 3 + 1] * d[4] + V[r * 3 + 2] * d[5];
}

// (q,t) <- exp(d) * (q,t)
SQLM_HD void se3_oplus(double q[4], double t[3], const double d[6]) {
  double qe[4], te[3], rt[3], qn[4];
  se3_exp(d, qe, te);
  q_rotate(qe, t, rt);
  t[0] = te[0] + rt[0]; t[1] = te[1] + rt[1]; t[2] = te[2] + rt[2];
  q_mul(qe, q, qn);
  q_normalize_rot(qn);
  q[0] = qn[0]; q[1] = qn[1]; q[2] = qn[2]; q[3] = qn[3];
}

// EdgeLidarFlatPoint error restated as (T_cw p_w - p_c) . n
SQLM_HD double lidar_error(const double q[4], const double t[3], const double *pc, const double *pw,
                           const double *n) {
  double c[3];
  q_rotate(q, pw, c);
  const double d0 = (c[0] + t[0]) - pc[0], d1 = (c[1] + t[1]) - pc[1], d2 = (c[2] + t[2]) - pc[2];
  return (d0 * n[0] + d1 * n[1]) + d2 * n[2];
}

// numeric central-difference Jacobian, delta = 1e-9 through oplus
SQLM_HD void lidar_jacobian(const double q[4], const double t[3], const double *pc, const double *pw,
                            const double *n, double J[6]) {
  const double delta = 1e-9, scalar = 1.0 / (2 * delta);
  for (int k = 0; k < 6; ++k) {
    double add[6] = {0, 0, 0, 0, 0, 0};
    double qa[4] = {q[0], q[1], q[2], q[3]}, ta[3] = {t[0], t[1], t[2]};
    add[k] = delta;
    se3_oplus(qa, ta, add);
    const double e1 = lidar_error(qa, ta, pc, pw, n);
    double qb[4] = {q[0], q[1], q[2], q[3]}, tb[3] = {t[0], t[1], t[2]};
    add[k] = -delta;
    se3_oplus(qb, tb, add);
    const double e2 = lidar_error(qb, tb, pc, pw, n);
    J[k] = scalar * (e1 - e2);
  }
}

#pragma clang fp contract(on)

}  // namespace sqlm
