/*
 * pmo.c — CPU ORACLE (test infrastructure only; see pmo.h).
 * Instantiates pmo_dense.inc / pmo_impl.inc for T = double and T = float.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "pmo.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#if defined(__FP_FAST_FMA) && !defined(PMO_ALLOW_FMA)
/* contraction must stay off: distances are ((dx*dx + dy*dy) + dz*dz) */
#endif

#include <time.h>
static double pmo_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ---- T = double ---- */
#define T double
#define SUF(x) x##_f64
static inline double tmin_f64(void) { return DBL_MIN; }
static inline double teps_f64(void) { return DBL_EPSILON; }
static inline double tpow_f64(double a, double b) { return pow(a, b); }
#include "pmo_dense.inc"
#include "pmo_impl.inc"
#undef T
#undef SUF

/* ---- T = float ---- */
#define T float
#define SUF(x) x##_f32
static inline float tmin_f32(void) { return FLT_MIN; }
static inline float teps_f32(void) { return FLT_EPSILON; }
static inline float tpow_f32(float a, float b) { return powf(a, b); }
#include "pmo_dense.inc"
#include "pmo_impl.inc"
#undef T
#undef SUF
