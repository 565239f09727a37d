// fastmath.hpp -- fp64 sin/cos, exp, log and sqrt specialised for the
// particle-filter step (gfx950).  The per-particle transcendentals of the
// fused kernel (motion_model.py:50-56, mylib/transform.py:31-33, the one exp
// of the log-sum likelihood, the device RNG) cost as much VALU issue as 100
// landmark updates when taken from the general-purpose device library, whose
// sin/cos carry a Payne-Hanek path and whose exp/log/sqrt cover every IEEE
// class.  These routines cover the ranges the step produces and hand anything
// else to the library routine (a divergent, practically never taken branch),
// so the results stay within 1 ulp everywhere.
//
// Issue cost: gfx950 VOP3 has no literal operands, so a polynomial
// coefficient must sit in a register.  Left to itself the compiler copies each
// Horner addend into the tied VGPR of v_fmac_f64 with two v_mov_b32 (three
// VALU issues per step; 300 of the fused kernel's 1,840 per-wave VALU issues
// outside the landmark loop were such copies).  fma_k() keeps the constant in
// an SGPR pair (s_mov on the scalar pipe) and issues ONE v_fma_f64; the
// arithmetic is the same single-rounding fma.
#pragma once
#include <hip/hip_runtime.h>

namespace slam {

// fma(a, b, k), k a constant held in an SGPR pair: one VALU issue
__device__ __forceinline__ double fma_k(const double a, const double b, const double k) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
// fma(x, a, b), a and b constants: v_mov_b64 + v_fmac_f64 (two issues, not three)
__device__ __forceinline__ double fma_kk(const double x, const double a, const double b) {
    double r;
    asm("v_mov_b64 %0, %3\n\tv_fmac_f64 %0, %2, %1" : "=&v"(r) : "v"(x), "s"(a), "s"(b));
    return r;
}

// ---- sin/cos ------------------------------------------------------------
// Cody-Waite reduction by pi/2 with FMA (the first step is exact for
// |x| < 2^19, see below) and the fdlibm kernel polynomials with the tail of the
// reduced argument (__kernel_sin / __kernel_cos, |r| <= pi/4, < 1 ulp).
namespace fm {
constexpr double kInvPio2 = 6.36619772367581382433e-01;
constexpr double kPio2Hi = 1.57079632679489655800e+00;   // RN(pi/2)
constexpr double kPio2Mid = 6.12323399573676603587e-17;  // RN(pi/2 - kPio2Hi)
constexpr double kPio2Lo = -1.49738490485916983e-33;     // next part
constexpr double kPio4 = 7.85398163397448278999e-01;     // RN(pi/4)
constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;

// sin(x + y), |x| <= pi/4, |y| <= ulp(x)/2 (fdlibm __kernel_sin, iy = 1)
__device__ __forceinline__ double ksin(const double x, const double y) {
    const double z = x * x;
    const double v = z * x;
    const double r = fma_k(z, fma_k(z, fma_k(z, fma_kk(z, S6, S5), S4), S3), S2);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
// sin(x), |x| <= pi/4 (fdlibm __kernel_sin, iy = 0)
__device__ __forceinline__ double ksin0(const double x) {
    const double z = x * x;
    const double v = z * x;
    const double r = fma_k(z, fma_k(z, fma_k(z, fma_kk(z, S6, S5), S4), S3), S2);
    return x + v * fma_k(z, r, S1);
}

// cos(x + y) (musl __cos)
__device__ __forceinline__ double kcos(const double x, const double y) {
    const double z = x * x;
    const double w2 = z * z;
    const double r = z * fma_k(z, fma_kk(z, C3, C2), C1) + w2 * w2 * fma_k(z, fma_kk(z, C6, C5), C4);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}
}  // namespace fm

// sincos for |x| < 2^19 (every angle of the step: wrapped headings plus one
// turn increment); other arguments (and NaN/inf) take the library routine.
// Exactness of r1 = fma(-n, kPio2Hi, x): kPio2Hi is a multiple of 2^-52 and
// |r1| < 2, so for |x| >= 1 (ulp(x) >= 2^-52) the exact difference has at
// most 53 significant bits; for |x| < 1 either n = 0 or ulp(x) = 2^-53 and
// |r1| < 1/4.
__device__ __forceinline__ void fast_sincos(const double x, double* sp, double* cp) {
    if (!(fabs(x) < 0x1p19)) {
        sincos(x, sp, cp);
        return;
    }
    const double n = rint(x * fm::kInvPio2);
    const double r1 = fma(-n, fm::kPio2Hi, x);
    const double r = fma(-n, fm::kPio2Mid, r1);
    double y = fma(-n, fm::kPio2Mid, r1 - r);
    y = fma(-n, fm::kPio2Lo, y);
    const double s = fm::ksin(r, y);
    const double c = fm::kcos(r, y);
    const int q = (int)n & 3;
    const double sa = (q & 1) ? c : s;
    const double ca = (q & 1) ? s : c;
    *sp = (q & 2) ? -sa : sa;
    *cp = ((q + 1) & 2) ? -ca : ca;
}

// sin/cos of a turn increment: |x| <= pi/4 goes straight to the kernels (no
// reduction, no quadrant selects), anything larger to fast_sincos.
__device__ __forceinline__ void small_sincos(const double x, double* sp, double* cp) {
    if (fabs(x) <= fm::kPio4) {
        *sp = fm::ksin0(x);
        *cp = fm::kcos(x, 0.0);
    } else {
        fast_sincos(x, sp, cp);
    }
}

// (sin, cos)(a + d) from (sin, cos)(a) and (sin, cos)(d): the angle-addition
// rotation, two roundings per component.
__device__ __forceinline__ void rotate_sc(const double s, const double c, const double sd,
                                          const double cd, double* so, double* co) {
    *so = fma(s, cd, c * sd);
    *co = fma(c, cd, -(s * sd));
}

// ---- exp ----------------------------------------------------------------
// exp(x) = 2^n exp(r), n = rint(x / ln 2), r = x - n ln 2 (Cody-Waite with the
// fdlibm split: ln2_hi has 21 trailing zero bits, so n ln2_hi is exact), exp(r)
// by its degree-13 Taylor polynomial on |r| <= ln2/2 (truncation < 6e-18
// relative), 2^n by v_ldexp_f64 (correctly rounded, subnormal results
// included).  Below -746 the result is +0, above 710 +inf, NaN stays NaN.
__device__ __forceinline__ double exp_lean(const double x) {
    constexpr double kLog2e = 1.44269504088896338700e+00;
    constexpr double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;
    const double n = rint(x * kLog2e);
    const double r = fma(-n, kLn2Lo, fma(-n, kLn2Hi, x));
    double p = fma_kk(r, 1.6059043836821613e-10, 2.08767569878681e-09);
    p = fma_k(r, p, 2.505210838544172e-08);
    p = fma_k(r, p, 2.755731922398589e-07);
    p = fma_k(r, p, 2.7557319223985893e-06);
    p = fma_k(r, p, 2.48015873015873e-05);
    p = fma_k(r, p, 1.984126984126984e-04);
    p = fma_k(r, p, 1.388888888888889e-03);
    p = fma_k(r, p, 8.333333333333333e-03);
    p = fma_k(r, p, 4.1666666666666664e-02);
    p = fma_k(r, p, 1.6666666666666666e-01);
    p = fma(r, p, 0.5);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    const double e = ldexp(p, (int)fmax(fmin(n, 2000.0), -2000.0));
    return (x < -746.0) ? 0.0 : (x > 710.0 ? __builtin_inf() : e);
}

// ---- sqrt of a non-negative, non-subnormal argument ----------------------
// v_rsq_f64 seed and the Goldschmidt/Newton refinement of the device library's
// sqrt (without its subnormal scaling); sqrt(0) = 0.
__device__ __forceinline__ double sqrt_pos(const double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    g = fma(d, h, g);
    return x > 0.0 ? g : 0.0;
}

// ---- device-RNG transcendentals (Box-Muller on 32-bit uniforms) ----------
// log(d 2^e) for d in [1, 2^32] (an integer-valued double): fdlibm e_log on
// the reduced mantissa (< 1 ulp); the quotient f / (2 + f) is refined from the
// hardware reciprocal by two Newton steps.
__device__ __forceinline__ double rng_log_scaled(const double d, const int e) {
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                     Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                     Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    int k = __builtin_amdgcn_frexp_exp(d) + e;        // d = m 2^k, m in [0.5, 1)
    double m = __builtin_amdgcn_frexp_mant(d);
    if (m < 0.70710678118654752440) {                 // m in [sqrt(2)/2, sqrt(2))
        m = m + m;
        k -= 1;
    }
    const double f = m - 1.0;                         // exact (Sterbenz)
    const double den = 2.0 + f;
    double rcp = __builtin_amdgcn_rcp(den);
    rcp = fma(fma(-den, rcp, 1.0), rcp, rcp);
    rcp = fma(fma(-den, rcp, 1.0), rcp, rcp);
    const double s = f * rcp;
    const double z = s * s, w = z * z;
    const double t1 = w * fma_k(w, fma_kk(w, Lg6, Lg4), Lg2);
    const double t2 = z * fma_k(w, fma_k(w, fma_kk(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// sin(2 pi u), cos(2 pi u) for u = k 2^-32, k in [1, 2^32]: the turn fraction is
// reduced exactly to the nearest quarter turn, |t| <= pi/4 is one rounding of
// pi * r, then the fdlibm kernels (the RNG only needs a few ulp).
__device__ __forceinline__ void rng_sincos2pi(const double u, double* sp, double* cp) {
    const double x = 4.0 * u;                         // quarter turns, exact
    const double n = rint(x);
    const double r = x - n;                           // exact, |r| <= 1/2
    const double t = r * 1.57079632679489661923;      // quarter turn = pi/2 rad
    const double s = fm::ksin0(t);
    const double c = fm::kcos(t, 0.0);
    const int q = (int)n & 3;
    const double sa = (q & 1) ? c : s;
    const double ca = (q & 1) ? s : c;
    *sp = (q & 2) ? -sa : sa;
    *cp = ((q + 1) & 2) ? -ca : ca;
}

}  // namespace slam
