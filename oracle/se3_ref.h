/*
 * se3_ref.h — TEST INFRASTRUCTURE (oracle). Not part of the shipped product.
 *
 * Eigen-free restatement of the fixed-size Lie-group arithmetic that g2o's
 * SE3Quat performs through Eigen 3, written so each formula follows the
 * reference (and Eigen's documented implementation) operation for operation.
 *
 *   SE3Quat ctor / normalizeRotation  Thirdparty/g2o/g2o/types/se3quat.h:58-60, :280-285
 *   SE3Quat::operator*(SE3Quat)        se3quat.h:104-110
 *   SE3Quat::map                       se3quat.h:217-220
 *   SE3Quat::exp (small-angle branch)  se3quat.h:223-257
 *   skew                               Thirdparty/g2o/g2o/types/se3_ops.hpp
 *   Eigen::Quaterniond(Matrix3d)       Eigen quaternionbase_assign_impl<Matrix3>
 *   Quaterniond::toRotationMatrix      Eigen QuaternionBase::toRotationMatrix
 *   Quaterniond * Vector3d             Eigen QuaternionBase::_transformVector
 *   Quaterniond * Quaterniond          Eigen quat_product (generic form)
 *   Matrix3d::inverse                  Eigen compute_inverse<...,3> (cofactors)
 *
 * Quaternion storage follows Eigen's coeffs() order: q[0..3] = x, y, z, w.
 * Compiled with -ffp-contract=off so no FMA contraction changes rounding.
 */
#ifndef SQLM_ORACLE_SE3_REF_H
#define SQLM_ORACLE_SE3_REF_H

#include <math.h>

/* Eigen squaredNorm of a Vector4d reduces pairwise: (x^2+z^2)+(y^2+w^2). */
static inline double oq_sqnorm(const double q[4]) {
  return (q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]);
}

/* Eigen normalize(): divide every coefficient by sqrt(squaredNorm) when > 0. */
static inline void oq_normalize(double q[4]) {
  double z = oq_sqnorm(q);
  if (z > 0.0) {
    double n = sqrt(z);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
  }
}

/* SE3Quat::normalizeRotation (se3quat.h:280-285): flip to w >= 0, normalise. */
static inline void oq_normalize_rotation(double q[4]) {
  if (q[3] < 0.0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
  oq_normalize(q);
}

/* a*b, Eigen quat_product. */
static inline void oq_mul(const double a[4], const double b[4], double out[4]) {
  double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
  out[0] = x; out[1] = y; out[2] = z; out[3] = w;
}

static inline void o3_cross(const double a[3], const double b[3], double o[3]) {
  double x = a[1] * b[2] - a[2] * b[1];
  double y = a[2] * b[0] - a[0] * b[2];
  double z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

/* q*v, Eigen _transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv. */
static inline void oq_rotate(const double q[4], const double v[3], double o[3]) {
  double uv[3], c2[3];
  o3_cross(q, v, uv);
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  o3_cross(q, uv, c2);
  o[0] = v[0] + q[3] * uv[0] + c2[0];
  o[1] = v[1] + q[3] * uv[1] + c2[1];
  o[2] = v[2] + q[3] * uv[2] + c2[2];
}

/* Eigen QuaternionBase::toRotationMatrix, row-major R[3][3]. */
static inline void oq_to_mat(const double q[4], double R[9]) {
  const double tx = 2.0 * q[0], ty = 2.0 * q[1], tz = 2.0 * q[2];
  const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
  const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
  const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
  R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

/* Eigen Quaterniond(const Matrix3d&) (quaternionbase_assign_impl, 3x3). */
static inline void oq_from_mat(const double m[9], double q[4]) {
#define M_(r, c) m[(r) * 3 + (c)]
  double t = (M_(0, 0) + M_(1, 1)) + M_(2, 2);
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (M_(2, 1) - M_(1, 2)) * t;
    q[1] = (M_(0, 2) - M_(2, 0)) * t;
    q[2] = (M_(1, 0) - M_(0, 1)) * t;
  } else {
    int i = 0;
    if (M_(1, 1) > M_(0, 0)) i = 1;
    if (M_(2, 2) > M_(i, i)) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(M_(i, i) - M_(j, j) - M_(k, k) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (M_(k, j) - M_(j, k)) * t;
    q[j] = (M_(j, i) + M_(i, j)) * t;
    q[k] = (M_(k, i) + M_(i, k)) * t;
  }
#undef M_
}

/* 3x3 row-major product C = A*B (Eigen lazy product, k ascending). */
static inline void o3_matmul(const double A[9], const double B[9], double C[9]) {
  double T[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      T[r * 3 + c] = A[r * 3 + 0] * B[0 * 3 + c] + A[r * 3 + 1] * B[1 * 3 + c] + A[r * 3 + 2] * B[2 * 3 + c];
  for (int i = 0; i < 9; ++i) C[i] = T[i];
}

/* SE3Quat::exp (se3quat.h:223-257). upd = [omega(3); upsilon(3)]. */
static inline void ose3_exp(const double upd[6], double q[4], double t[3]) {
  const double *w = upd, *u = upd + 3;
  double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double Om[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
  double Om2[9], R[9], V[9];
  o3_matmul(Om, Om, Om2);
  if (theta < 0.00001) {
    for (int i = 0; i < 9; ++i) R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + Om[i] + Om2[i];
    for (int i = 0; i < 9; ++i) V[i] = R[i];
  } else {
    double a = sin(theta) / theta;
    double b = (1.0 - cos(theta)) / (theta * theta);
    double c = (theta - sin(theta)) / pow(theta, 3);
    for (int i = 0; i < 9; ++i) R[i] = (((i % 4 == 0) ? 1.0 : 0.0) + a * Om[i]) + b * Om2[i];
    for (int i = 0; i < 9; ++i) V[i] = (((i % 4 == 0) ? 1.0 : 0.0) + b * Om[i]) + c * Om2[i];
  }
  oq_from_mat(R, q);
  oq_normalize_rotation(q);
  for (int r = 0; r < 3; ++r) t[r] = V[r * 3 + 0] * u[0] + V[r * 3 + 1] * u[1] + V[r * 3 + 2] * u[2];
}

/* (qa,ta) <- (qa,ta) * (qb,tb) as SE3Quat::operator* (se3quat.h:104-110). */
static inline void ose3_compose(const double qa[4], const double ta[3], const double qb[4],
                                const double tb[3], double qo[4], double to[3]) {
  double rt[3], q[4];
  oq_rotate(qa, tb, rt);
  to[0] = ta[0] + rt[0]; to[1] = ta[1] + rt[1]; to[2] = ta[2] + rt[2];
  oq_mul(qa, qb, q);
  oq_normalize_rotation(q);
  qo[0] = q[0]; qo[1] = q[1]; qo[2] = q[2]; qo[3] = q[3];
}

/* VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:73-76): T <- exp(d) * T. */
static inline void ose3_oplus(double q[4], double t[3], const double d[6]) {
  double qe[4], te[3];
  ose3_exp(d, qe, te);
  ose3_compose(qe, te, q, t, q, t);
}

/* Eigen 3x3 inverse via cofactors (compute_inverse_size3_helper). */
static inline void o3_inverse(const double m[9], double out[9]) {
#define C_(i, j)                                                                       \
  (m[(((i) + 1) % 3) * 3 + (((j) + 1) % 3)] * m[(((i) + 2) % 3) * 3 + (((j) + 2) % 3)] - \
   m[(((i) + 1) % 3) * 3 + (((j) + 2) % 3)] * m[(((i) + 2) % 3) * 3 + (((j) + 1) % 3)])
  double c00 = C_(0, 0), c10 = C_(1, 0), c20 = C_(2, 0);
  double det = (c00 * m[0] + c10 * m[3]) + c20 * m[6];
  double invdet = 1.0 / det;
  out[5] = C_(2, 1) * invdet;
  out[7] = C_(1, 2) * invdet;
  out[8] = C_(2, 2) * invdet;
  out[3] = C_(0, 1) * invdet;
  out[4] = C_(1, 1) * invdet;
  out[6] = C_(0, 2) * invdet;
  out[0] = c00 * invdet; out[1] = c10 * invdet; out[2] = c20 * invdet;
#undef C_
}

#endif
