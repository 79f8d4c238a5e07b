/*
 * skyline_ref.h — TEST INFRASTRUCTURE (oracle). Column-profile LDL^T shared by
 * the BA oracle (g2o_ref.c) and the essential-graph oracle (eg_ref.c).
 */
#ifndef SQLM_SKYLINE_REF_H
#define SQLM_SKYLINE_REF_H

#include <stdint.h>

/* ------------------------------------------------------- skyline LDL^T */

/* Column-profile LDL^T of the upper triangle (natural block order). Stands in
 * for Eigen::SimplicialLDLT<Upper> + AMD (linear_solver_eigen.h:60-75,94-124):
 * the same factorisation up to rounding; fails only on an exact zero pivot,
 * as SimplicialLDLT does. */
typedef struct {
  int n;
  int *first;      /* first row in column c */
  int64_t *cptr;   /* column start in val */
  double *val;
} skyline;

static inline double *sky_at(skyline *s, int r, int c) { return s->val + s->cptr[c] + (r - s->first[c]); }

static inline int sky_factor(skyline *s) {
  for (int j = 0; j < s->n; ++j) {
    const int fj = s->first[j];
    double *cj = s->val + s->cptr[j] - fj; /* cj[r] for r in [fj, j] */
    for (int i = fj; i < j; ++i) {
      const int fi = s->first[i];
      const double *ci = s->val + s->cptr[i] - fi;
      int k0 = fi > fj ? fi : fj;
      double acc = cj[i];
      for (int k = k0; k < i; ++k) acc -= ci[k] * cj[k];
      cj[i] = acc;
    }
    double d = cj[j];
    for (int i = fj; i < j; ++i) {
      const double gi = cj[i];
      const double u = gi / s->val[s->cptr[i] + (i - s->first[i])];
      d -= u * gi;
      cj[i] = u;
    }
    if (d == 0.0) return 0;
    cj[j] = d;
  }
  return 1;
}

static inline void sky_solve(skyline *s, const double *b, double *x) {
  const int n = s->n;
  for (int j = 0; j < n; ++j) {
    const int fj = s->first[j];
    const double *cj = s->val + s->cptr[j] - fj;
    double acc = b[j];
    for (int k = fj; k < j; ++k) acc -= cj[k] * x[k];
    x[j] = acc;
  }
  for (int j = 0; j < n; ++j) x[j] /= s->val[s->cptr[j] + (j - s->first[j])];
  for (int j = n - 1; j >= 0; --j) {
    const int fj = s->first[j];
    const double *cj = s->val + s->cptr[j] - fj;
    const double xj = x[j];
    for (int k = fj; k < j; ++k) x[k] -= cj[k] * xj;
  }
}

#endif
