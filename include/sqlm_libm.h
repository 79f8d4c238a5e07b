/* sqlm_libm.h — exp, log, sin, cos, acos in double precision from IEEE +, -,
 * *, / and sqrt alone (no FMA contraction), so that the host and the GPU compute
 * them to the same bits.
 *
 * The essential graph's numeric Jacobians (g2o base_binary_edge.hpp:131-205,
 * central differences with delta = 1e-9) divide error differences by 2e-9:
 * any difference between two libm's sin / cos / exp / log / acos, one ulp of
 * 1 being 2.2e-16, becomes a 1e-7 relative difference of a Jacobian entry.
 * With these functions on both sides (sim3_dev.h on the GPU, the oracle's
 * eg_ref.c on the CPU) the Jacobians agree bit for bit
 * (tests/test_eg_gpu.py::test_eg_numeric_jacobians_bitwise).
 *
 * The algorithms are the classic freely distributable fdlibm ones (Sun
 * Microsystems, 1993: e_exp.c, e_log.c, k_sin.c, k_cos.c, e_rem_pio2.c medium
 * range, e_acos.c), errors below one ulp; they differ from glibc's by at most
 * one ulp. Plain C11 and HIP: the oracle (gcc -ffp-contract=off) and the
 * library (hipcc, contraction off per function below) include the same text.
 * sin / cos reduce arguments with the three-part pi/2 of fdlibm's medium case,
 * exact for |x| < 2^19 pi/2 (the Sim3 angles here are in [0, pi]). */
#ifndef SQLM_LIBM_H
#define SQLM_LIBM_H

#if defined(__HIPCC__)
#define SQLM_LM static inline __host__ __device__
#else
#include <math.h>
#define SQLM_LM static inline
#endif

#if defined(__clang__)
#define SQLM_LM_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define SQLM_LM_NOCONTRACT
#endif

typedef union {
  double d;
  unsigned long long u;
} sqlm_lm_bits;

SQLM_LM int sqlm_lm_hi(double x) {
  sqlm_lm_bits b;
  b.d = x;
  return (int)(unsigned)(b.u >> 32);
}
SQLM_LM unsigned sqlm_lm_lo(double x) {
  sqlm_lm_bits b;
  b.d = x;
  return (unsigned)b.u;
}
SQLM_LM double sqlm_lm_make(int hi, unsigned lo) {
  sqlm_lm_bits b;
  b.u = ((unsigned long long)(unsigned)hi << 32) | lo;
  return b.d;
}
/* x * 2^k for a normal result (|k| < 1023 here) */
SQLM_LM double sqlm_lm_scale(double x, int k) {
  if (k > 1023) return x * sqlm_lm_make(0x7fe00000, 0) * sqlm_lm_make((k - 1023 + 1023) << 20, 0);
  if (k < -1022) return x * sqlm_lm_make((k + 54 + 1023) << 20, 0) * sqlm_lm_make((1023 - 54) << 20, 0);
  return x * sqlm_lm_make((k + 1023) << 20, 0);
}

SQLM_LM double sqlm_exp(double x) {
  SQLM_LM_NOCONTRACT
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
  const int hx = sqlm_lm_hi(x), xsb = (hx >> 31) & 1, ix = hx & 0x7fffffff;
  if (ix >= 0x40862E42) { /* |x| >= 709.78 */
    if (ix >= 0x7ff00000) return (((unsigned)ix & 0xfffff) | sqlm_lm_lo(x)) ? x + x : (xsb ? 0.0 : x);
    if (x > 7.09782712893383973096e+02) return sqlm_lm_make(0x7ff00000, 0); /* overflow */
    if (x < -7.45133219101941108420e+02) return 0.0;                         /* underflow */
  }
  double hi = 0.0, lo = 0.0;
  int k = 0;
  if (ix > 0x3fd62e42) { /* |x| > 0.5 ln2 */
    if (ix < 0x3FF0A2B2) { /* |x| < 1.5 ln2 */
      hi = xsb ? x + ln2HI : x - ln2HI;
      lo = xsb ? -ln2LO : ln2LO;
      k = xsb ? -1 : 1;
    } else {
      k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
      const double t = k;
      hi = x - t * ln2HI;
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (ix < 0x3e300000) { /* |x| < 2^-28 */
    return 1.0 + x;
  }
  const double t = x * x;
  const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  return sqlm_lm_scale(y, k);
}

SQLM_LM double sqlm_log(double x) {
  SQLM_LM_NOCONTRACT
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10, two54 = 1.80143985094819840000e+16;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int hx = sqlm_lm_hi(x);
  const unsigned lx = sqlm_lm_lo(x);
  int k = 0;
  if (hx < 0x00100000) { /* x < 2^-1022 */
    if (((hx & 0x7fffffff) | (int)lx) == 0) return -two54 / 0.0; /* log(+-0) = -inf */
    if (hx < 0) return (x - x) / 0.0;                          /* log(-#) = NaN */
    k -= 54;
    x *= two54;
    hx = sqlm_lm_hi(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int i = (hx + 0x95f64) & 0x100000;
  x = sqlm_lm_make(hx | (i ^ 0x3ff00000), sqlm_lm_lo(x)); /* normalise x or x / 2 */
  k += (i >> 20);
  const double f = x - 1.0;
  const double dk = (double)k;
  if ((0x000fffff & (2 + hx)) < 3) { /* -2^-20 <= f < 2^-20 */
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f), z = s * s, w = z * z;
  int ii = hx - 0x6147a;
  const int j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  ii |= j;
  const double R = t2 + t1;
  if (ii > 0) {
    const double hfsq = 0.5 * f * f;
    return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* sin on [-pi/4, pi/4]: x + y the reduced argument (iy = 0: y is zero) */
SQLM_LM double sqlm_lm_ksin(double x, double y, int iy) {
  SQLM_LM_NOCONTRACT
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
               S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  if ((sqlm_lm_hi(x) & 0x7fffffff) < 0x3e400000) return x; /* |x| < 2^-27 */
  const double z = x * x, v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

/* cos on [-pi/4, pi/4] */
SQLM_LM double sqlm_lm_kcos(double x, double y) {
  SQLM_LM_NOCONTRACT
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
               C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const int ix = sqlm_lm_hi(x) & 0x7fffffff;
  if (ix < 0x3e400000) return 1.0; /* |x| < 2^-27 */
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y)); /* |x| < 0.3 */
  const double qx = ix > 0x3fe90000 ? 0.28125 : sqlm_lm_make(ix - 0x00200000, 0u);
  const double hz = 0.5 * z - qx, a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}

/* x = n pi/2 + y[0] + y[1], |y| <= pi/4; returns n. fdlibm's medium-range
   reduction only: exact for |x| <= 2^20 pi/2 (SQLM_LM_PIO2_MAX). Beyond it
   (fdlibm's Payne-Hanek range) y = NaN: sin / cos return NaN, so a wild LM
   step (a rotation of more than 1.6e6 rad) yields a NaN chi2 and is rejected
   cleanly instead of meeting the undefined int conversion below. */
#define SQLM_LM_PIO2_MAX 0x413921fb
SQLM_LM int sqlm_lm_rem_pio2(double x, double *y) {
  SQLM_LM_NOCONTRACT
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const int hx = sqlm_lm_hi(x), ix = hx & 0x7fffffff;
  if (ix <= 0x3fe921fb) { /* |x| <= pi/4 */
    y[0] = x;
    y[1] = 0.0;
    return 0;
  }
  if (ix > SQLM_LM_PIO2_MAX) { /* outside the medium range (and inf / NaN) */
    y[0] = y[1] = __builtin_nan("");
    return 0;
  }
  double t = hx < 0 ? -x : x;
  const int n = (int)(t * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t - fn * pio2_1, w = fn * pio2_1t;
  const int j = ix >> 20;
  y[0] = r - w;
  int i = j - ((sqlm_lm_hi(y[0]) >> 20) & 0x7ff);
  if (i > 16) { /* second iteration: 118 bits */
    t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y[0] = r - w;
    i = j - ((sqlm_lm_hi(y[0]) >> 20) & 0x7ff);
    if (i > 49) { /* third iteration: 151 bits */
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y[0] = r - w;
    }
  }
  y[1] = (r - y[0]) - w;
  if (hx < 0) {
    y[0] = -y[0];
    y[1] = -y[1];
    return -n;
  }
  return n;
}

SQLM_LM double sqlm_sin(double x) {
  const int ix = sqlm_lm_hi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return sqlm_lm_ksin(x, 0.0, 0);
  if (ix >= 0x7ff00000) return x - x;
  double y[2];
  const int n = sqlm_lm_rem_pio2(x, y);
  switch (n & 3) {
    case 0: return sqlm_lm_ksin(y[0], y[1], 1);
    case 1: return sqlm_lm_kcos(y[0], y[1]);
    case 2: return -sqlm_lm_ksin(y[0], y[1], 1);
    default: return -sqlm_lm_kcos(y[0], y[1]);
  }
}

SQLM_LM double sqlm_cos(double x) {
  const int ix = sqlm_lm_hi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return sqlm_lm_kcos(x, 0.0);
  if (ix >= 0x7ff00000) return x - x;
  double y[2];
  const int n = sqlm_lm_rem_pio2(x, y);
  switch (n & 3) {
    case 0: return sqlm_lm_kcos(y[0], y[1]);
    case 1: return -sqlm_lm_ksin(y[0], y[1], 1);
    case 2: return -sqlm_lm_kcos(y[0], y[1]);
    default: return sqlm_lm_ksin(y[0], y[1], 1);
  }
}

SQLM_LM double sqlm_acos(double x) {
  SQLM_LM_NOCONTRACT
  const double pi = 3.14159265358979311600e+00, pio2_hi = 1.57079632679489655800e+00,
               pio2_lo = 6.12323399573676603587e-17;
  const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01,
               pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
               qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01,
               qS4 = 7.70381505559019352791e-02;
  const int hx = sqlm_lm_hi(x), ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) { /* |x| >= 1 */
    if (((ix - 0x3ff00000) | (int)sqlm_lm_lo(x)) == 0) return hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
    return (x - x) / (x - x); /* NaN */
  }
  if (ix < 0x3fe00000) { /* |x| < 0.5 */
    if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
    const double z = x * x;
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const double r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if (hx < 0) { /* x < -0.5 */
    const double z = (1.0 + x) * 0.5;
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const double s = sqrt(z), r = p / q, w = r * s - pio2_lo;
    return pi - 2.0 * (s + w);
  }
  /* x > 0.5 */
  const double z = (1.0 - x) * 0.5, s = sqrt(z);
  const double df = sqlm_lm_make(sqlm_lm_hi(s), 0u);
  const double c = (z - df * df) / (s + df);
  const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const double r = p / q, w = r * s + c;
  return 2.0 * (df + w);
}

#endif /* SQLM_LIBM_H */
