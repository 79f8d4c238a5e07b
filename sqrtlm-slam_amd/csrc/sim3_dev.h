// sim3_dev.h — Sim3 algebra of the essential graph, usable on host and
// device. Semantics (not code) follow the reference:
//   Sim3(update) / log / inverse / operator*   Thirdparty/g2o/g2o/types/sim3.h
//   VertexSim3Expmap::oplusImpl                types_seven_dof_expmap.h:60-66
//   EdgeSim3::computeError                     types_seven_dof_expmap.h:106-114
//   numeric Jacobian (delta = 1e-9, central)   core/base_binary_edge.hpp:131-205
// S = [qx qy qz qw tx ty tz s]. Like se3_dev.h, evaluated without FMA
// contraction: the numeric Jacobians divide error differences by 2e-9. The
// transcendental functions are sqlm_libm.h's, shared with the oracle, so the
// Jacobians are the oracle's bit for bit.
#pragma once
#include "se3_dev.h"
#include "../../include/sqlm_libm.h"

namespace sqlm {

#pragma clang fp contract(off)

SQLM_HD void skew3(const double w[3], double O[9]) {
  O[0] = 0.0; O[1] = -w[2]; O[2] = w[1];
  O[3] = w[2]; O[4] = 0.0; O[5] = -w[0];
  O[6] = -w[1]; O[7] = w[0]; O[8] = 0.0;
}

SQLM_HD void sim3_from_update(const double u[7], double S[8]) {
  const double omega[3] = {u[0], u[1], u[2]}, sigma = u[6];
  const double theta = sqrt((omega[0] * omega[0] + omega[1] * omega[1]) + omega[2] * omega[2]);
  double O[9], O2[9], R[9];
  skew3(omega, O);
  const double s = sqlm_exp(sigma);
  mat3_mul(O, O, O2);
  const double eps = 0.00001;
  double A, B, C;
  if (fabs(sigma) < eps) {
    C = 1;
    if (theta < eps) {
      A = 1. / 2.;
      B = 1. / 6.;
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + O[k]) + O2[k];
    } else {
      const double theta2 = theta * theta;
      A = (1 - sqlm_cos(theta)) / (theta2);
      B = (theta - sqlm_sin(theta)) / (theta2 * theta);
      const double a = sqlm_sin(theta) / theta, b = (1 - sqlm_cos(theta)) / (theta * theta);
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + a * O[k]) + b * O2[k];
    }
  } else {
    C = (s - 1) / sigma;
    if (theta < eps) {
      const double sigma2 = sigma * sigma;
      A = ((sigma - 1) * s + 1) / sigma2;
      B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + O[k]) + O2[k];
    } else {
      const double ra = sqlm_sin(theta) / theta, rb = (1 - sqlm_cos(theta)) / (theta * theta);
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + ra * O[k]) + rb * O2[k];
      const double a = s * sqlm_sin(theta), b = s * sqlm_cos(theta);
      const double theta2 = theta * theta, sigma2 = sigma * sigma, c = theta2 + sigma2;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  q_from_mat(R, S);
  double W[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) W[k] = (A * O[k] + B * O2[k]) + C * (k % 4 == 0 ? 1.0 : 0.0);
#pragma unroll
  for (int r = 0; r < 3; ++r) S[4 + r] = (W[3 * r] * u[3] + W[3 * r + 1] * u[4]) + W[3 * r + 2] * u[5];
  S[7] = s;
}

// W.lu().solve(t): partial pivoting, first maximum as pivot (Eigen PartialPivLU)
SQLM_HD void lu_solve3(const double Win[9], const double b[3], double x[3]) {
  double a[9];
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 9; ++k) a[k] = Win[k];
  for (int k = 0; k < 3; ++k) {
    int piv = k;
    double big = fabs(a[3 * k + k]);
    for (int i = k + 1; i < 3; ++i)
      if (fabs(a[3 * i + k]) > big) { big = fabs(a[3 * i + k]); piv = i; }
    if (big != 0.0) {
      if (piv != k) {
        for (int c = 0; c < 3; ++c) { const double t = a[3 * k + c]; a[3 * k + c] = a[3 * piv + c]; a[3 * piv + c] = t; }
        const int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
      }
      for (int i = k + 1; i < 3; ++i) a[3 * i + k] /= a[3 * k + k];
    }
    for (int i = k + 1; i < 3; ++i)
      for (int c = k + 1; c < 3; ++c) a[3 * i + c] -= a[3 * i + k] * a[3 * k + c];
  }
  double y[3];
  for (int i = 0; i < 3; ++i) {
    double v = b[perm[i]];
    for (int j = 0; j < i; ++j) v -= a[3 * i + j] * y[j];
    y[i] = v;
  }
  for (int i = 2; i >= 0; --i) {
    double v = y[i];
    for (int j = i + 1; j < 3; ++j) v -= a[3 * i + j] * x[j];
    x[i] = v / a[3 * i + i];
  }
}

SQLM_HD void sim3_log(const double S[8], double out[7]) {
  const double s = S[7];
  const double sigma = sqlm_log(s);
  double R[9], omega[3], O[9], dr[3];
  q_to_mat(S, R);
  const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
  const double eps = 0.00001;
  double A, B, C;
  dr[0] = R[7] - R[5];
  dr[1] = R[2] - R[6];
  dr[2] = R[3] - R[1];
  if (fabs(sigma) < eps) {
    C = 1;
    if (d > 1 - eps) {
#pragma unroll
      for (int k = 0; k < 3; ++k) omega[k] = 0.5 * dr[k];
      A = 1. / 2.;
      B = 1. / 6.;
    } else {
      const double theta = sqlm_acos(d), theta2 = theta * theta;
      const double f = theta / (2 * sqrt(1 - d * d));
#pragma unroll
      for (int k = 0; k < 3; ++k) omega[k] = f * dr[k];
      A = (1 - sqlm_cos(theta)) / (theta2);
      B = (theta - sqlm_sin(theta)) / (theta2 * theta);
    }
  } else {
    C = (s - 1) / sigma;
    if (d > 1 - eps) {
      const double sigma2 = sigma * sigma;
#pragma unroll
      for (int k = 0; k < 3; ++k) omega[k] = 0.5 * dr[k];
      A = ((sigma - 1) * s + 1) / (sigma2);
      B = ((0.5 * sigma2 - sigma + 1) * s) / (sigma2 * sigma);
    } else {
      const double theta = sqlm_acos(d);
      const double f = theta / (2 * sqrt(1 - d * d));
#pragma unroll
      for (int k = 0; k < 3; ++k) omega[k] = f * dr[k];
      const double theta2 = theta * theta;
      const double a = s * sqlm_sin(theta), b = s * sqlm_cos(theta);
      const double c = theta2 + sigma * sigma;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  skew3(omega, O);
  double O2[9], W[9];
  mat3_mul(O, O, O2);
#pragma unroll
  for (int k = 0; k < 9; ++k) W[k] = (A * O[k] + B * O2[k]) + C * (k % 4 == 0 ? 1.0 : 0.0);
  double ups[3];
  lu_solve3(W, S + 4, ups);
#pragma unroll
  for (int k = 0; k < 3; ++k) { out[k] = omega[k]; out[3 + k] = ups[k]; }
  out[6] = sigma;
}

SQLM_HD void sim3_mul(const double a[8], const double b[8], double o[8]) {
  double q[4], rt[3];
  q_mul(a, b, q);
  q_rotate(a, b + 4, rt);
  o[4] = a[7] * rt[0] + a[4];
  o[5] = a[7] * rt[1] + a[5];
  o[6] = a[7] * rt[2] + a[6];
  o[7] = a[7] * b[7];
  o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3];
}

SQLM_HD void sim3_inverse(const double a[8], double o[8]) {
  const double qc[4] = {-a[0], -a[1], -a[2], a[3]};
  const double k = -1. / a[7];
  const double v[3] = {k * a[4], k * a[5], k * a[6]};
  q_rotate(qc, v, o + 4);
  o[0] = qc[0]; o[1] = qc[1]; o[2] = qc[2]; o[3] = qc[3];
  o[7] = 1. / a[7];
}

// S <- Sim3(u) * S, the scale update zeroed when the scale is fixed
SQLM_HD void sim3_oplus(double S[8], const double upd[7], bool fix_scale) {
  double u[7], E[8], o[8];
#pragma unroll
  for (int k = 0; k < 7; ++k) u[k] = upd[k];
  if (fix_scale) u[6] = 0;
  sim3_from_update(u, E);
  sim3_mul(E, S, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) S[k] = o[k];
}

// EdgeSim3 error: sqlm_log(C * Si * Sj^-1)
SQLM_HD void eg_edge_error(const double Si[8], const double Sj[8], const double C[8], double e[7]) {
  double a[8], b[8], jinv[8];
  sim3_mul(C, Si, a);
  sim3_inverse(Sj, jinv);
  sim3_mul(a, jinv, b);
  sim3_log(b, e);
}

#pragma clang fp contract(on)

}  // namespace sqlm
