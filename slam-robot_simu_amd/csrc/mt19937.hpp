// mt19937.hpp -- NumPy's legacy RandomState stream (MT19937 + polar
// Box-Muller with the cached second normal), host and device.
//
// The reference draws every noise sample from np.random's global RandomState
// (particle_filter.py:152, :165, :214; motion_model.py:46-48).  NumPy's legacy
// generator (numpy/random/src/mt19937/mt19937.c, legacy-distributions.c):
//   word      = temper(key[pos++]), the 624-word key regenerated when pos = 624
//   double    = ((w0 >> 5) * 67108864.0 + (w1 >> 6)) / 9007199254740992.0
//   gauss     = a cached value if one is held, otherwise: draw x1 = 2 d - 1,
//               x2 = 2 d - 1 until 0 < r2 = x1^2 + x2^2 < 1, f = sqrt(-2 log(r2)
//               / r2), cache f x1, return f x2
// The key obeys X[n + 624] = X[n + 397] ^ twist(X[n], X[n + 1]) over the whole
// stream, so the device generates the untempered sequence block by block and
// every later pass reads it as one array.
//
// log is the C library's (NumPy calls libm here, not its SIMD loops), and
// glibc's log is not correctly rounded: it differs from the correctly rounded
// logarithm in ~0.3 % of the polar draws.  glibc_log() restates glibc 2.35's
// algorithm (sysdeps/ieee754/dbl-64/e_log.c, the ARM optimized-routines log:
// a 128-entry table of (1/c, log c) and two polynomials) operation by
// operation, with the fused multiply-adds of its FMA build (the x86-64 ifunc
// variant selected on FMA-capable CPUs) or the plain operations of its SSE2
// build.  The table is glibc's own data, read from the process's libm at run
// time (rng_api.hip) and checked against log() before it is used.
#pragma once

#include <stdint.h>

namespace slam {

constexpr int kMtN = 624;
constexpr int kMtM = 397;

struct GlibcLogTable {
    double ln2hi, ln2lo;
    double poly[5];       // A[0..4]: log1p(r) - r ~ r^2 A0 + r^3 (A1 + ...)
    double poly1[11];     // B[0..10]: the |x - 1| < 2^-4 polynomial
    double tab[256];      // (invc, logc) x 128
    double tab2[256];     // (chi, clo) x 128 (the build without FMA)
    int32_t fma_build;    // 1: __log_fma's operation order
    int32_t pad;
};

__host__ __device__ inline uint64_t mt_bits(double x) {
    union {
        double d;
        uint64_t u;
    } v;
    v.d = x;
    return v.u;
}

__host__ __device__ inline double mt_double(uint64_t x) {
    union {
        double d;
        uint64_t u;
    } v;
    v.u = x;
    return v.d;
}

// glibc 2.35 __log for finite x > 0 (the polar method's r2 is in (2^-104, 1)).
__host__ __device__ inline double glibc_log(const double x, const GlibcLogTable& T) {
    const uint64_t ix = mt_bits(x);
    const uint64_t lo_b = 0x3fee000000000000ULL;          // asuint64(1.0 - 0x1p-4)
    const uint64_t hi_b = 0x3ff1090000000000ULL;          // asuint64(1.0 + 0x1.09p-4)
    const double* B = T.poly1;
    const double* A = T.poly;
    if (ix - lo_b < hi_b - lo_b) {                        // close to 1.0
        if (ix == 0x3ff0000000000000ULL) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        double y;
        if (T.fma_build) {
            double p3 = fma(r, B[8], B[7]);
            p3 = fma(r2, B[9], p3);
            p3 = fma(r3, B[10], p3);
            double p2 = fma(r, B[5], B[4]);
            p2 = fma(r2, B[6], p2);
            p2 = fma(r3, p3, p2);
            double p1 = fma(r, B[2], B[1]);
            p1 = fma(r2, B[3], p1);
            p1 = fma(r3, p2, p1);
            const double w = r * 0x1p27;
            const double rhi = r + w - w;
            const double rlo = r - rhi;
            const double ww = rhi * rhi * B[0];
            const double hi = r + ww;
            double lo = r - hi + ww;
            lo = fma(B[0] * rlo, rhi + r, lo);
            y = fma(r3, p1, lo);
            return y + hi;
        }
        y = r3 * (B[1] + r * B[2] + r2 * B[3] +
                  r3 * (B[4] + r * B[5] + r2 * B[6] + r3 * (B[7] + r * B[8] + r2 * B[9] + r3 * B[10])));
        const double w = r * 0x1p27;
        const double rhi = r + w - w;
        const double rlo = r - rhi;
        const double ww = rhi * rhi * B[0];
        const double hi = r + ww;
        double lo = r - hi + ww;
        lo += B[0] * rlo * (rhi + r);
        y += lo;
        y += hi;
        return y;
    }
    uint64_t jx = ix;
    if (ix < 0x0010000000000000ULL) {                     // subnormal: normalise
        jx = mt_bits(x * 0x1p52);
        jx -= 52ULL << 52;
    }
    const uint64_t tmp = jx - 0x3fe6000000000000ULL;
    const int i = (int)((tmp >> 45) % 128);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = jx - (tmp & (0xfffULL << 52));
    const double invc = T.tab[2 * i], logc = T.tab[2 * i + 1], z = mt_double(iz);
    const double kd = (double)k;
    if (T.fma_build) {
        const double r = fma(z, invc, -1.0);
        const double w = fma(kd, T.ln2hi, logc);
        const double hi = w + r;
        const double lo = fma(kd, T.ln2lo, w - hi + r);
        const double r2 = r * r;
        const double p = fma(r2, fma(r, A[4], A[3]), fma(r, A[2], A[1]));
        return fma(r * r2, p, fma(r2, A[0], lo)) + hi;
    }
    const double r = (z - T.tab2[2 * i] - T.tab2[2 * i + 1]) * invc;
    const double w = kd * T.ln2hi + logc;
    const double hi = w + r;
    const double lo = w - hi + r + kd * T.ln2lo;
    const double r2 = r * r;
    return lo + r2 * A[0] + r * r2 * (A[1] + r * A[2] + r2 * (A[3] + r * A[4])) + hi;
}

__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// X[n + 624] from X[n] (upper bit), X[n + 1] (lower bits) and X[n + 397]
__host__ __device__ inline uint32_t mt_next(uint32_t xn, uint32_t xn1, uint32_t xm) {
    const uint32_t y = (xn & 0x80000000u) | (xn1 & 0x7fffffffu);
    return xm ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// mt19937_next_double from two tempered words
__host__ __device__ inline double mt_legacy_double(uint32_t w0, uint32_t w1) {
    const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

}  // namespace slam
