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

// sin/cos of a turn increment: |x| <= 1/16 (every increment of the bench's
// motion model) by the Taylor polynomials in z = x^2 (truncation below
// 3e-19 relative; cos as 1 + z q(z), so the only rounding of note is the last
// one: < 1 ulp, and sin to x^9); |x| <= pi/4 straight to the kernels (no
// reduction, no quadrant selects); anything larger to fast_sincos.
__device__ __forceinline__ void small_sincos(const double x, double* sp, double* cp) {
    if (fabs(x) <= 0.0625) {
        const double z = x * x;
        const double ps = fma_k(z, fma_k(z, fma_kk(z, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0),
                                -1.0 / 6.0);
        *sp = fma(x * z, ps, x);
        const double pc = fma_k(z, fma_k(z, fma_kk(z, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5);
        *cp = fma(z, pc, 1.0);
    } else if (fabs(x) <= fm::kPio4) {
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

// exp(x) from a 64-entry table of 2^(j/64) (each entry the rounded value and
// its rounding error), held in LDS by the caller: x = (64 k + j) ln2/64 + r,
// |r| <= ln2/128, exp(r) - 1 by its degree-6 Taylor polynomial (truncation
// < 3e-20), exp(x) = 2^k (T_j + (T_j p + T_lo_j)) -- under 0.51 ulp, with six
// polynomial fmas against exp_lean's thirteen.  ln2/64 is split so that
// kd ln2hi/64 is exact for |kd| < 2^24.  Below -746 the result is +0, above
// 710 +inf, NaN stays NaN (as exp_lean).
__device__ __constant__ const double2 kExpTab64[64] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56},
    {0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55},
    {0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57},
    {0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54},
    {0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59},
    {0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54},
    {0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54},
    {0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55},
    {0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55},
    {0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54},
    {0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55},
    {0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54},
    {0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55},
    {0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55},
    {0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54},
    {0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55},
    {0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54},
    {0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54},
    {0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56},
    {0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55},
    {0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58},
    {0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59},
    {0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56},
    {0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56},
    {0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54},
    {0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55},
    {0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54},
    {0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54},
    {0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54},
    {0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54},
    {0x1.6623882552225p+0, -0x1.bb60987591c34p-54},
    {0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54},
    {0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57},
    {0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55},
    {0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54},
    {0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55},
    {0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56},
    {0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54},
    {0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54},
    {0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54},
    {0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55},
    {0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57},
    {0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54},
    {0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56},
    {0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54},
    {0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54},
    {0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54},
    {0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54},
    {0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57},
    {0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56},
    {0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55},
    {0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55},
    {0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54},
    {0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56},
    {0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54},
    {0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55},
    {0x1.da9e603db3285p+0, 0x1.c2300696db532p-54},
    {0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54},
    {0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55},
    {0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54},
    {0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54},
    {0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54},
    {0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55},
};

// NONPOS: the caller guarantees x <= 0 or NaN (no overflow test).
template <bool NONPOS = false>
__device__ __forceinline__ double exp_tab(const double x, const double2* __restrict__ tab) {
    constexpr double kInvLn2N = 0x1.71547652b82fep+6;       // 64 / ln2
    constexpr double kNegLn2HiN = -0x1.62e42ff000000p-7;    // -(ln2/64), 29 significant bits
    constexpr double kNegLn2LoN = 0x1.718432a1b0e26p-41;    // -(ln2/64 - ln2hi/64)
    const double kd = rint(x * kInvLn2N);
    const double r = fma(kd, kNegLn2LoN, fma(kd, kNegLn2HiN, x));
    const int ki = (int)kd;
    const double2 t = tab[ki & 63];
    const double r2 = r * r;
    const double c46 = fma(r2, 1.0 / 720.0, fma_kk(r, 1.0 / 120.0, 1.0 / 24.0));   // 1/24 + r/120 + r^2/720
    const double c23 = fma_kk(r, 1.0 / 6.0, 0.5);                                 // 1/2 + r/6
    const double p = fma(r2, fma(r2, c46, c23), r);                               // exp(r) - 1
    const double v = t.x + fma(t.x, p, t.y);
    const double e = ldexp(v, ki >> 6);
    if (NONPOS) return (x < -746.0) ? 0.0 : e;
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
