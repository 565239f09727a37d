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
// |r| <= ln2/128, exp(r) - 1 by its degree-5 Taylor polynomial (truncation
// < 3.5e-17, round 3: degree 6 before), exp(x) = 2^k (T_j + (T_j p + T_lo_j))
// -- under 0.9 ulp, with five polynomial fmas against exp_lean's thirteen (the
// parity bar is the weights' 1e-12, not the last ulp).  ln2/64 is split so that
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
    // k = round(x 64/ln2) by the 1.5 2^52 shift: the integer sits in the low
    // word of kdm (no rint / convert); |x 64/ln2| >= 2^51 only where the range
    // select below decides
    const double kdm = fma(x, kInvLn2N, 0x1.8p52);
    const double kd = kdm - 0x1.8p52;
    const double r = fma(kd, kNegLn2LoN, fma(kd, kNegLn2HiN, x));
    const int ki = (int)(uint32_t)__double_as_longlong(kdm);
    const double2 t = tab[ki & 63];
    const double r2 = r * r;
    const double c45 = fma_kk(r, 1.0 / 120.0, 1.0 / 24.0);                      // 1/24 + r/120
    const double c23 = fma_kk(r, 1.0 / 6.0, 0.5);                                 // 1/2 + r/6
    const double p = fma(r2, fma(r2, c45, c23), r);      // exp(r) - 1 to degree 5 (r^6/720 < 3.5e-17)
    const double v = t.x + fma(t.x, p, t.y);
    const double e = ldexp(v, ki >> 6);
    if (NONPOS) return (x < -746.0) ? 0.0 : e;
    return (x < -746.0) ? 0.0 : (x > 710.0 ? __builtin_inf() : e);
}

// exp(-y/2) with exactly the bits of exp_tab(-y/2) -- the product
// likelihood's exp(-q/2) without forming q/2 (one fp64 multiply less per
// factor).  Every quantity is held at a power-of-two multiple of exp_tab's:
// the reduction yields 2r, the polynomial's coefficients are scaled so that it
// yields 2p, and the table htab holds (t.x/2, t.y).  Scaling by a power of two
// commutes with rounding in the normal range; where y/2 would be subnormal the
// result is 1 either way (tests/test_exp_tab.py checks the bits on the host).
template <bool NONPOS = false>
__device__ __forceinline__ double exp_nhalf(const double y, const double2* __restrict__ htab) {
    constexpr double kInvLn2N = 0x1.71547652b82fep+6;       // exp_tab's constants
    constexpr double kNegLn2HiN = -0x1.62e42ff000000p-7;
    constexpr double kNegLn2LoN = 0x1.718432a1b0e26p-41;
    const double kdm = fma(y, -0.5 * kInvLn2N, 0x1.8p52);   // = fma(-y/2, 64/ln2, shift)
    const double kd = kdm - 0x1.8p52;
    const double r = fma(kd, 2.0 * kNegLn2LoN, fma(kd, 2.0 * kNegLn2HiN, -y));   // 2 r
    const int ki = (int)(uint32_t)__double_as_longlong(kdm);
    const double2 t = htab[ki & 63];                         // (t.x / 2, t.y)
    const double r2 = r * r;                                 // 4 r^2
    // c45's addend from a VGPR (the asm hides the constant: hoisted out of the
    // loop, one v_fma instead of v_mov_b64 + v_fmac); c23's is an inline constant
    double k24 = (1.0 / 24.0) / 8.0;
    asm("" : "+v"(k24));
    double c45;                                                                   // c45 / 8
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(c45) : "v"(r), "s"((1.0 / 120.0) / 16.0), "v"(k24));
    const double c23 = fma(r, (1.0 / 6.0) / 4.0, 0.25);                           // c23 / 2
    const double p = fma(r2, fma(r2, c45, c23), r);          // 2 p
    const double v = fma(t.x, 2.0, fma(t.x, p, t.y));        // t.x + fma(t.x, p, t.y)
    const double e = ldexp(v, ki >> 6);
    if (NONPOS) return (y > 1492.0) ? 0.0 : e;
    return (y > 1492.0) ? 0.0 : (y < -1420.0 ? __builtin_inf() : e);
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

// ---- device-RNG transcendentals from LDS tables (round 3) ---------------
// sin/cos(2 pi j / 256) correctly rounded; for the log, per 256 slots of the
// reduced mantissa m in [sqrt(1/2), sqrt(2)) (exponent bit, top 7 fraction
// bits): invc = 1/c, c the slot's midpoint, rounded to 2^-10 (exactly 1 for
// the two slots beside m = 1, so that log(m) = log1p(m - 1) with m - 1 exact
// there) and -log(invc) as a double-double (hi, lo); tools/gen_rng_tables.py
// generates them (tests/test_rng_tables.py checks these copies).
__device__ __constant__ const double2 kRngSinCos256[256] = {
    {0x0.0p+0, 0x1.0000000000000p+0},
    {0x1.92155f7a3667ep-6, 0x1.ffd886084cd0dp-1},
    {0x1.91f65f10dd814p-5, 0x1.ff621e3796d7ep-1},
    {0x1.2d52092ce19f6p-4, 0x1.fe9cdad01883ap-1},
    {0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1},
    {0x1.f564e56a9730ep-4, 0x1.fc26470e19fd3p-1},
    {0x1.2c8106e8e613ap-3, 0x1.fa7557f08a517p-1},
    {0x1.5e214448b3fc6p-3, 0x1.f8764fa714ba9p-1},
    {0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1},
    {0x1.c0b826a7e4f63p-3, 0x1.f38f3ac64e589p-1},
    {0x1.f19f97b215f1bp-3, 0x1.f0a7efb9230d7p-1},
    {0x1.111d262b1f677p-2, 0x1.ed740e7684963p-1},
    {0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1},
    {0x1.4135c94176601p-2, 0x1.e6288ec48e112p-1},
    {0x1.58f9a75ab1fddp-2, 0x1.e212104f686e5p-1},
    {0x1.7088530fa459fp-2, 0x1.ddb13b6ccc23cp-1},
    {0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1},
    {0x1.9ef7943a8ed8ap-2, 0x1.d4134d14dc93ap-1},
    {0x1.b5d1009e15cc0p-2, 0x1.ced7af43cc773p-1},
    {0x1.cc66e9931c45ep-2, 0x1.c954b213411f5p-1},
    {0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1},
    {0x1.f8ba4dbf89abap-2, 0x1.bd7c0ac6f952ap-1},
    {0x1.073879922ffeep-1, 0x1.b728345196e3ep-1},
    {0x1.11eb3541b4b23p-1, 0x1.b090a58150200p-1},
    {0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1},
    {0x1.26d054cdd12dfp-1, 0x1.a29a7a0462782p-1},
    {0x1.30ff7fce17035p-1, 0x1.9b3e047f38741p-1},
    {0x1.3affa292050b9p-1, 0x1.93a22499263fbp-1},
    {0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1},
    {0x1.4e6cabbe3e5e9p-1, 0x1.83b0e0bff976ep-1},
    {0x1.57d69348ceca0p-1, 0x1.7b5df226aafafp-1},
    {0x1.610b7551d2cdfp-1, 0x1.72d0837efff96p-1},
    {0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1},
    {0x1.72d0837efff96p-1, 0x1.610b7551d2cdfp-1},
    {0x1.7b5df226aafafp-1, 0x1.57d69348ceca0p-1},
    {0x1.83b0e0bff976ep-1, 0x1.4e6cabbe3e5e9p-1},
    {0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1},
    {0x1.93a22499263fbp-1, 0x1.3affa292050b9p-1},
    {0x1.9b3e047f38741p-1, 0x1.30ff7fce17035p-1},
    {0x1.a29a7a0462782p-1, 0x1.26d054cdd12dfp-1},
    {0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1},
    {0x1.b090a58150200p-1, 0x1.11eb3541b4b23p-1},
    {0x1.b728345196e3ep-1, 0x1.073879922ffeep-1},
    {0x1.bd7c0ac6f952ap-1, 0x1.f8ba4dbf89abap-2},
    {0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2},
    {0x1.c954b213411f5p-1, 0x1.cc66e9931c45ep-2},
    {0x1.ced7af43cc773p-1, 0x1.b5d1009e15cc0p-2},
    {0x1.d4134d14dc93ap-1, 0x1.9ef7943a8ed8ap-2},
    {0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2},
    {0x1.ddb13b6ccc23cp-1, 0x1.7088530fa459fp-2},
    {0x1.e212104f686e5p-1, 0x1.58f9a75ab1fddp-2},
    {0x1.e6288ec48e112p-1, 0x1.4135c94176601p-2},
    {0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2},
    {0x1.ed740e7684963p-1, 0x1.111d262b1f677p-2},
    {0x1.f0a7efb9230d7p-1, 0x1.f19f97b215f1bp-3},
    {0x1.f38f3ac64e589p-1, 0x1.c0b826a7e4f63p-3},
    {0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3},
    {0x1.f8764fa714ba9p-1, 0x1.5e214448b3fc6p-3},
    {0x1.fa7557f08a517p-1, 0x1.2c8106e8e613ap-3},
    {0x1.fc26470e19fd3p-1, 0x1.f564e56a9730ep-4},
    {0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4},
    {0x1.fe9cdad01883ap-1, 0x1.2d52092ce19f6p-4},
    {0x1.ff621e3796d7ep-1, 0x1.91f65f10dd814p-5},
    {0x1.ffd886084cd0dp-1, 0x1.92155f7a3667ep-6},
    {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.ffd886084cd0dp-1, -0x1.92155f7a3667ep-6},
    {0x1.ff621e3796d7ep-1, -0x1.91f65f10dd814p-5},
    {0x1.fe9cdad01883ap-1, -0x1.2d52092ce19f6p-4},
    {0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4},
    {0x1.fc26470e19fd3p-1, -0x1.f564e56a9730ep-4},
    {0x1.fa7557f08a517p-1, -0x1.2c8106e8e613ap-3},
    {0x1.f8764fa714ba9p-1, -0x1.5e214448b3fc6p-3},
    {0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3},
    {0x1.f38f3ac64e589p-1, -0x1.c0b826a7e4f63p-3},
    {0x1.f0a7efb9230d7p-1, -0x1.f19f97b215f1bp-3},
    {0x1.ed740e7684963p-1, -0x1.111d262b1f677p-2},
    {0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2},
    {0x1.e6288ec48e112p-1, -0x1.4135c94176601p-2},
    {0x1.e212104f686e5p-1, -0x1.58f9a75ab1fddp-2},
    {0x1.ddb13b6ccc23cp-1, -0x1.7088530fa459fp-2},
    {0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2},
    {0x1.d4134d14dc93ap-1, -0x1.9ef7943a8ed8ap-2},
    {0x1.ced7af43cc773p-1, -0x1.b5d1009e15cc0p-2},
    {0x1.c954b213411f5p-1, -0x1.cc66e9931c45ep-2},
    {0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2},
    {0x1.bd7c0ac6f952ap-1, -0x1.f8ba4dbf89abap-2},
    {0x1.b728345196e3ep-1, -0x1.073879922ffeep-1},
    {0x1.b090a58150200p-1, -0x1.11eb3541b4b23p-1},
    {0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1},
    {0x1.a29a7a0462782p-1, -0x1.26d054cdd12dfp-1},
    {0x1.9b3e047f38741p-1, -0x1.30ff7fce17035p-1},
    {0x1.93a22499263fbp-1, -0x1.3affa292050b9p-1},
    {0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1},
    {0x1.83b0e0bff976ep-1, -0x1.4e6cabbe3e5e9p-1},
    {0x1.7b5df226aafafp-1, -0x1.57d69348ceca0p-1},
    {0x1.72d0837efff96p-1, -0x1.610b7551d2cdfp-1},
    {0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1},
    {0x1.610b7551d2cdfp-1, -0x1.72d0837efff96p-1},
    {0x1.57d69348ceca0p-1, -0x1.7b5df226aafafp-1},
    {0x1.4e6cabbe3e5e9p-1, -0x1.83b0e0bff976ep-1},
    {0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1},
    {0x1.3affa292050b9p-1, -0x1.93a22499263fbp-1},
    {0x1.30ff7fce17035p-1, -0x1.9b3e047f38741p-1},
    {0x1.26d054cdd12dfp-1, -0x1.a29a7a0462782p-1},
    {0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1},
    {0x1.11eb3541b4b23p-1, -0x1.b090a58150200p-1},
    {0x1.073879922ffeep-1, -0x1.b728345196e3ep-1},
    {0x1.f8ba4dbf89abap-2, -0x1.bd7c0ac6f952ap-1},
    {0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1},
    {0x1.cc66e9931c45ep-2, -0x1.c954b213411f5p-1},
    {0x1.b5d1009e15cc0p-2, -0x1.ced7af43cc773p-1},
    {0x1.9ef7943a8ed8ap-2, -0x1.d4134d14dc93ap-1},
    {0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1},
    {0x1.7088530fa459fp-2, -0x1.ddb13b6ccc23cp-1},
    {0x1.58f9a75ab1fddp-2, -0x1.e212104f686e5p-1},
    {0x1.4135c94176601p-2, -0x1.e6288ec48e112p-1},
    {0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1},
    {0x1.111d262b1f677p-2, -0x1.ed740e7684963p-1},
    {0x1.f19f97b215f1bp-3, -0x1.f0a7efb9230d7p-1},
    {0x1.c0b826a7e4f63p-3, -0x1.f38f3ac64e589p-1},
    {0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1},
    {0x1.5e214448b3fc6p-3, -0x1.f8764fa714ba9p-1},
    {0x1.2c8106e8e613ap-3, -0x1.fa7557f08a517p-1},
    {0x1.f564e56a9730ep-4, -0x1.fc26470e19fd3p-1},
    {0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1},
    {0x1.2d52092ce19f6p-4, -0x1.fe9cdad01883ap-1},
    {0x1.91f65f10dd814p-5, -0x1.ff621e3796d7ep-1},
    {0x1.92155f7a3667ep-6, -0x1.ffd886084cd0dp-1},
    {0x0.0p+0, -0x1.0000000000000p+0},
    {-0x1.92155f7a3667ep-6, -0x1.ffd886084cd0dp-1},
    {-0x1.91f65f10dd814p-5, -0x1.ff621e3796d7ep-1},
    {-0x1.2d52092ce19f6p-4, -0x1.fe9cdad01883ap-1},
    {-0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1},
    {-0x1.f564e56a9730ep-4, -0x1.fc26470e19fd3p-1},
    {-0x1.2c8106e8e613ap-3, -0x1.fa7557f08a517p-1},
    {-0x1.5e214448b3fc6p-3, -0x1.f8764fa714ba9p-1},
    {-0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1},
    {-0x1.c0b826a7e4f63p-3, -0x1.f38f3ac64e589p-1},
    {-0x1.f19f97b215f1bp-3, -0x1.f0a7efb9230d7p-1},
    {-0x1.111d262b1f677p-2, -0x1.ed740e7684963p-1},
    {-0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1},
    {-0x1.4135c94176601p-2, -0x1.e6288ec48e112p-1},
    {-0x1.58f9a75ab1fddp-2, -0x1.e212104f686e5p-1},
    {-0x1.7088530fa459fp-2, -0x1.ddb13b6ccc23cp-1},
    {-0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1},
    {-0x1.9ef7943a8ed8ap-2, -0x1.d4134d14dc93ap-1},
    {-0x1.b5d1009e15cc0p-2, -0x1.ced7af43cc773p-1},
    {-0x1.cc66e9931c45ep-2, -0x1.c954b213411f5p-1},
    {-0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1},
    {-0x1.f8ba4dbf89abap-2, -0x1.bd7c0ac6f952ap-1},
    {-0x1.073879922ffeep-1, -0x1.b728345196e3ep-1},
    {-0x1.11eb3541b4b23p-1, -0x1.b090a58150200p-1},
    {-0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1},
    {-0x1.26d054cdd12dfp-1, -0x1.a29a7a0462782p-1},
    {-0x1.30ff7fce17035p-1, -0x1.9b3e047f38741p-1},
    {-0x1.3affa292050b9p-1, -0x1.93a22499263fbp-1},
    {-0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1},
    {-0x1.4e6cabbe3e5e9p-1, -0x1.83b0e0bff976ep-1},
    {-0x1.57d69348ceca0p-1, -0x1.7b5df226aafafp-1},
    {-0x1.610b7551d2cdfp-1, -0x1.72d0837efff96p-1},
    {-0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1},
    {-0x1.72d0837efff96p-1, -0x1.610b7551d2cdfp-1},
    {-0x1.7b5df226aafafp-1, -0x1.57d69348ceca0p-1},
    {-0x1.83b0e0bff976ep-1, -0x1.4e6cabbe3e5e9p-1},
    {-0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1},
    {-0x1.93a22499263fbp-1, -0x1.3affa292050b9p-1},
    {-0x1.9b3e047f38741p-1, -0x1.30ff7fce17035p-1},
    {-0x1.a29a7a0462782p-1, -0x1.26d054cdd12dfp-1},
    {-0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1},
    {-0x1.b090a58150200p-1, -0x1.11eb3541b4b23p-1},
    {-0x1.b728345196e3ep-1, -0x1.073879922ffeep-1},
    {-0x1.bd7c0ac6f952ap-1, -0x1.f8ba4dbf89abap-2},
    {-0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2},
    {-0x1.c954b213411f5p-1, -0x1.cc66e9931c45ep-2},
    {-0x1.ced7af43cc773p-1, -0x1.b5d1009e15cc0p-2},
    {-0x1.d4134d14dc93ap-1, -0x1.9ef7943a8ed8ap-2},
    {-0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2},
    {-0x1.ddb13b6ccc23cp-1, -0x1.7088530fa459fp-2},
    {-0x1.e212104f686e5p-1, -0x1.58f9a75ab1fddp-2},
    {-0x1.e6288ec48e112p-1, -0x1.4135c94176601p-2},
    {-0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2},
    {-0x1.ed740e7684963p-1, -0x1.111d262b1f677p-2},
    {-0x1.f0a7efb9230d7p-1, -0x1.f19f97b215f1bp-3},
    {-0x1.f38f3ac64e589p-1, -0x1.c0b826a7e4f63p-3},
    {-0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3},
    {-0x1.f8764fa714ba9p-1, -0x1.5e214448b3fc6p-3},
    {-0x1.fa7557f08a517p-1, -0x1.2c8106e8e613ap-3},
    {-0x1.fc26470e19fd3p-1, -0x1.f564e56a9730ep-4},
    {-0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4},
    {-0x1.fe9cdad01883ap-1, -0x1.2d52092ce19f6p-4},
    {-0x1.ff621e3796d7ep-1, -0x1.91f65f10dd814p-5},
    {-0x1.ffd886084cd0dp-1, -0x1.92155f7a3667ep-6},
    {-0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.ffd886084cd0dp-1, 0x1.92155f7a3667ep-6},
    {-0x1.ff621e3796d7ep-1, 0x1.91f65f10dd814p-5},
    {-0x1.fe9cdad01883ap-1, 0x1.2d52092ce19f6p-4},
    {-0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4},
    {-0x1.fc26470e19fd3p-1, 0x1.f564e56a9730ep-4},
    {-0x1.fa7557f08a517p-1, 0x1.2c8106e8e613ap-3},
    {-0x1.f8764fa714ba9p-1, 0x1.5e214448b3fc6p-3},
    {-0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3},
    {-0x1.f38f3ac64e589p-1, 0x1.c0b826a7e4f63p-3},
    {-0x1.f0a7efb9230d7p-1, 0x1.f19f97b215f1bp-3},
    {-0x1.ed740e7684963p-1, 0x1.111d262b1f677p-2},
    {-0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2},
    {-0x1.e6288ec48e112p-1, 0x1.4135c94176601p-2},
    {-0x1.e212104f686e5p-1, 0x1.58f9a75ab1fddp-2},
    {-0x1.ddb13b6ccc23cp-1, 0x1.7088530fa459fp-2},
    {-0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2},
    {-0x1.d4134d14dc93ap-1, 0x1.9ef7943a8ed8ap-2},
    {-0x1.ced7af43cc773p-1, 0x1.b5d1009e15cc0p-2},
    {-0x1.c954b213411f5p-1, 0x1.cc66e9931c45ep-2},
    {-0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2},
    {-0x1.bd7c0ac6f952ap-1, 0x1.f8ba4dbf89abap-2},
    {-0x1.b728345196e3ep-1, 0x1.073879922ffeep-1},
    {-0x1.b090a58150200p-1, 0x1.11eb3541b4b23p-1},
    {-0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1},
    {-0x1.a29a7a0462782p-1, 0x1.26d054cdd12dfp-1},
    {-0x1.9b3e047f38741p-1, 0x1.30ff7fce17035p-1},
    {-0x1.93a22499263fbp-1, 0x1.3affa292050b9p-1},
    {-0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1},
    {-0x1.83b0e0bff976ep-1, 0x1.4e6cabbe3e5e9p-1},
    {-0x1.7b5df226aafafp-1, 0x1.57d69348ceca0p-1},
    {-0x1.72d0837efff96p-1, 0x1.610b7551d2cdfp-1},
    {-0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1},
    {-0x1.610b7551d2cdfp-1, 0x1.72d0837efff96p-1},
    {-0x1.57d69348ceca0p-1, 0x1.7b5df226aafafp-1},
    {-0x1.4e6cabbe3e5e9p-1, 0x1.83b0e0bff976ep-1},
    {-0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1},
    {-0x1.3affa292050b9p-1, 0x1.93a22499263fbp-1},
    {-0x1.30ff7fce17035p-1, 0x1.9b3e047f38741p-1},
    {-0x1.26d054cdd12dfp-1, 0x1.a29a7a0462782p-1},
    {-0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1},
    {-0x1.11eb3541b4b23p-1, 0x1.b090a58150200p-1},
    {-0x1.073879922ffeep-1, 0x1.b728345196e3ep-1},
    {-0x1.f8ba4dbf89abap-2, 0x1.bd7c0ac6f952ap-1},
    {-0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1},
    {-0x1.cc66e9931c45ep-2, 0x1.c954b213411f5p-1},
    {-0x1.b5d1009e15cc0p-2, 0x1.ced7af43cc773p-1},
    {-0x1.9ef7943a8ed8ap-2, 0x1.d4134d14dc93ap-1},
    {-0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1},
    {-0x1.7088530fa459fp-2, 0x1.ddb13b6ccc23cp-1},
    {-0x1.58f9a75ab1fddp-2, 0x1.e212104f686e5p-1},
    {-0x1.4135c94176601p-2, 0x1.e6288ec48e112p-1},
    {-0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1},
    {-0x1.111d262b1f677p-2, 0x1.ed740e7684963p-1},
    {-0x1.f19f97b215f1bp-3, 0x1.f0a7efb9230d7p-1},
    {-0x1.c0b826a7e4f63p-3, 0x1.f38f3ac64e589p-1},
    {-0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1},
    {-0x1.5e214448b3fc6p-3, 0x1.f8764fa714ba9p-1},
    {-0x1.2c8106e8e613ap-3, 0x1.fa7557f08a517p-1},
    {-0x1.f564e56a9730ep-4, 0x1.fc26470e19fd3p-1},
    {-0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1},
    {-0x1.2d52092ce19f6p-4, 0x1.fe9cdad01883ap-1},
    {-0x1.91f65f10dd814p-5, 0x1.ff621e3796d7ep-1},
    {-0x1.92155f7a3667ep-6, 0x1.ffd886084cd0dp-1},
};
__device__ __constant__ const double2 kRngLogInvHi[256] = {
    {0x1.fe00000000000p+0, -0x1.60e32f44788d9p-1},
    {0x1.fa00000000000p+0, -0x1.5cdb1dc6c1765p-1},
    {0x1.f640000000000p+0, -0x1.590c1d93dd73cp-1},
    {0x1.f240000000000p+0, -0x1.54f40ed7bcea8p-1},
    {0x1.ee80000000000p+0, -0x1.5115d58ce769cp-1},
    {0x1.eb00000000000p+0, -0x1.4d72d3a39fd00p-1},
    {0x1.e740000000000p+0, -0x1.4985ece016ba9p-1},
    {0x1.e3c0000000000p+0, -0x1.45d503d1c937dp-1},
    {0x1.e000000000000p+0, -0x1.41d8fe84672aep-1},
    {0x1.dcc0000000000p+0, -0x1.3e5e826c588a4p-1},
    {0x1.d940000000000p+0, -0x1.3a98b61f150b9p-1},
    {0x1.d5c0000000000p+0, -0x1.36cbbe7ab0764p-1},
    {0x1.d280000000000p+0, -0x1.333dc2e01e776p-1},
    {0x1.cf40000000000p+0, -0x1.2fa96aa2e62c1p-1},
    {0x1.cc00000000000p+0, -0x1.2c0e9ed448e8cp-1},
    {0x1.c8c0000000000p+0, -0x1.286d4808a75fcp-1},
    {0x1.c580000000000p+0, -0x1.24c54e53f0793p-1},
    {0x1.c280000000000p+0, -0x1.215f5b1a6e729p-1},
    {0x1.bf40000000000p+0, -0x1.1daa591d7b9f3p-1},
    {0x1.bc40000000000p+0, -0x1.1a38333834393p-1},
    {0x1.b940000000000p+0, -0x1.16c013206ab71p-1},
    {0x1.b640000000000p+0, -0x1.1341e3f53e439p-1},
    {0x1.b380000000000p+0, -0x1.1008d3f3ab146p-1},
    {0x1.b080000000000p+0, -0x1.0c7ecbf32e533p-1},
    {0x1.adc0000000000p+0, -0x1.093abae514ea2p-1},
    {0x1.ab00000000000p+0, -0x1.05f14bd26459cp-1},
    {0x1.a840000000000p+0, -0x1.02a26cf9b55edp-1},
    {0x1.a580000000000p+0, -0x1.fe9c1881e5cffp-2},
    {0x1.a2c0000000000p+0, -0x1.f7e82e660f5c1p-2},
    {0x1.a000000000000p+0, -0x1.f128f5faf06edp-2},
    {0x1.9d80000000000p+0, -0x1.eafcd2cea9d71p-2},
    {0x1.9b00000000000p+0, -0x1.e4c71a8687704p-2},
    {0x1.9840000000000p+0, -0x1.dde73454e855fp-2},
    {0x1.95c0000000000p+0, -0x1.d79cfa6d1dc32p-2},
    {0x1.9340000000000p+0, -0x1.d148cccde9dfbp-2},
    {0x1.90c0000000000p+0, -0x1.caea8bc716ed8p-2},
    {0x1.8e80000000000p+0, -0x1.c52699316cf6bp-2},
    {0x1.8c00000000000p+0, -0x1.beb4d9da71b7cp-2},
    {0x1.8980000000000p+0, -0x1.b838a7cb5c1f0p-2},
    {0x1.8740000000000p+0, -0x1.b2596fb0c4ad3p-2},
    {0x1.8500000000000p+0, -0x1.ac718c258b0e4p-2},
    {0x1.82c0000000000p+0, -0x1.a680e369d4104p-2},
    {0x1.8080000000000p+0, -0x1.a0875b4a61d17p-2},
    {0x1.7e40000000000p+0, -0x1.9a84d91dde4d2p-2},
    {0x1.7c00000000000p+0, -0x1.947941c2116fbp-2},
    {0x1.79c0000000000p+0, -0x1.8e64799901f7cp-2},
    {0x1.7780000000000p+0, -0x1.8846648600624p-2},
    {0x1.7580000000000p+0, -0x1.82ce6bdfe4d9dp-2},
    {0x1.7340000000000p+0, -0x1.7c9e7703f8cfap-2},
    {0x1.7140000000000p+0, -0x1.77166c744025ap-2},
    {0x1.6f40000000000p+0, -0x1.7186b11381193p-2},
    {0x1.6d00000000000p+0, -0x1.6b3bb2235943ep-2},
    {0x1.6b00000000000p+0, -0x1.659b57303e1f3p-2},
    {0x1.6900000000000p+0, -0x1.5ff3070a793d4p-2},
    {0x1.6700000000000p+0, -0x1.5a42ab0f4cfe2p-2},
    {0x1.6540000000000p+0, -0x1.5541aec91bfa0p-2},
    {0x1.6340000000000p+0, -0x1.4f81fe4763d00p-2},
    {0x1.6140000000000p+0, -0x1.49b9feb7c176bp-2},
    {0x1.5f80000000000p+0, -0x1.44a41b463c47cp-2},
    {0x1.5d80000000000p+0, -0x1.3ecc460ef5f50p-2},
    {0x1.5bc0000000000p+0, -0x1.39a8619f4518fp-2},
    {0x1.59c0000000000p+0, -0x1.33c05f128dda9p-2},
    {0x1.5800000000000p+0, -0x1.2e8e2bae11d31p-2},
    {0x1.5640000000000p+0, -0x1.29552f81ff523p-2},
    {0x1.5480000000000p+0, -0x1.241558bfd1404p-2},
    {0x1.52c0000000000p+0, -0x1.1ece95528ae7bp-2},
    {0x1.5100000000000p+0, -0x1.1980d2dd4236fp-2},
    {0x1.4f40000000000p+0, -0x1.142bfeb9a0474p-2},
    {0x1.4d80000000000p+0, -0x1.0ed005f657da4p-2},
    {0x1.4bc0000000000p+0, -0x1.096cd555917e6p-2},
    {0x1.4a40000000000p+0, -0x1.04c8de1841e02p-2},
    {0x1.4880000000000p+0, -0x1.feb0233e607ccp-3},
    {0x1.46c0000000000p+0, -0x1.f3bfa934d6768p-3},
    {0x1.4540000000000p+0, -0x1.ea5349e23ac0ep-3},
    {0x1.43c0000000000p+0, -0x1.e0dbc3d92aac9p-3},
    {0x1.4200000000000p+0, -0x1.d5c216b4fbb91p-3},
    {0x1.4080000000000p+0, -0x1.cc320c0176502p-3},
    {0x1.3f00000000000p+0, -0x1.c2968558c18c1p-3},
    {0x1.3d40000000000p+0, -0x1.b7526a22e4703p-3},
    {0x1.3bc0000000000p+0, -0x1.ad9da1f8273bfp-3},
    {0x1.3a40000000000p+0, -0x1.a3dd04b93865fp-3},
    {0x1.38c0000000000p+0, -0x1.9a10756988593p-3},
    {0x1.3740000000000p+0, -0x1.9037d6a1804c3p-3},
    {0x1.35c0000000000p+0, -0x1.86530a8c70cc6p-3},
    {0x1.3480000000000p+0, -0x1.7e0afd630c274p-3},
    {0x1.3300000000000p+0, -0x1.740f8f54037a5p-3},
    {0x1.3180000000000p+0, -0x1.6a079d0f7aad2p-3},
    {0x1.3000000000000p+0, -0x1.5ff3070a793d4p-3},
    {0x1.2ec0000000000p+0, -0x1.5782cb309162ep-3},
    {0x1.2d40000000000p+0, -0x1.4d56b5798ec03p-3},
    {0x1.2c00000000000p+0, -0x1.44d2b6ccb7d1ep-3},
    {0x1.2a80000000000p+0, -0x1.3a8eb2d31a376p-3},
    {0x1.2940000000000p+0, -0x1.31f693eb19966p-3},
    {0x1.27c0000000000p+0, -0x1.279a300ab4f7ap-3},
    {0x1.2680000000000p+0, -0x1.1eed90e2dc2c3p-3},
    {0x1.2540000000000p+0, -0x1.16377fb124192p-3},
    {0x1.2400000000000p+0, -0x1.0d77e7cd08e59p-3},
    {0x1.22c0000000000p+0, -0x1.04aeb449f66bfp-3},
    {0x1.2140000000000p+0, -0x1.f42dba3a22cedp-4},
    {0x1.2000000000000p+0, -0x1.e27076e2af2e6p-4},
    {0x1.1ec0000000000p+0, -0x1.d09f72b4c4824p-4},
    {0x1.1d80000000000p+0, -0x1.beba818146765p-4},
    {0x1.1c40000000000p+0, -0x1.acc17684332acp-4},
    {0x1.1b00000000000p+0, -0x1.9ab42462033adp-4},
    {0x1.1a00000000000p+0, -0x1.8c345d6319b21p-4},
    {0x1.18c0000000000p+0, -0x1.7a0216f649e12p-4},
    {0x1.1780000000000p+0, -0x1.67bb0726ec0fcp-4},
    {0x1.1640000000000p+0, -0x1.555efe40b50b5p-4},
    {0x1.1500000000000p+0, -0x1.42edcbea646f0p-4},
    {0x1.1400000000000p+0, -0x1.341d7961bd1d1p-4},
    {0x1.12c0000000000p+0, -0x1.2185b3b75a1cep-4},
    {0x1.11c0000000000p+0, -0x1.129644402e2acp-4},
    {0x1.1080000000000p+0, -0x1.ffae9119b9303p-5},
    {0x1.0f40000000000p+0, -0x1.da0478be39253p-5},
    {0x1.0e40000000000p+0, -0x1.bbc2bfc44f417p-5},
    {0x1.0d40000000000p+0, -0x1.9d644fdffa279p-5},
    {0x1.0c00000000000p+0, -0x1.77458f632dcfcp-5},
    {0x1.0b00000000000p+0, -0x1.58a5bafc8e4d5p-5},
    {0x1.09c0000000000p+0, -0x1.32348c7001697p-5},
    {0x1.08c0000000000p+0, -0x1.13523785971f3p-5},
    {0x1.07c0000000000p+0, -0x1.e8a3ee30cdcacp-6},
    {0x1.06c0000000000p+0, -0x1.aa6721ee835aap-6},
    {0x1.0580000000000p+0, -0x1.5c45a51b8d389p-6},
    {0x1.0480000000000p+0, -0x1.1d7f7eb9eebe7p-6},
    {0x1.0380000000000p+0, -0x1.bcf712c74384cp-7},
    {0x1.0280000000000p+0, -0x1.3e7295d25a7d9p-7},
    {0x1.0180000000000p+0, -0x1.7ee11ebd82e94p-8},
    {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.fa00000000000p-1, 0x1.82448a388a2aap-7},
    {0x1.f600000000000p-1, 0x1.432a925980cc1p-6},
    {0x1.f280000000000p-1, 0x1.b5cc258b718e6p-6},
    {0x1.ee80000000000p-1, 0x1.1ce5a62bc353ap-5},
    {0x1.eb00000000000p-1, 0x1.5715c4c03ceefp-5},
    {0x1.e780000000000p-1, 0x1.91b073efd7314p-5},
    {0x1.e380000000000p-1, 0x1.d52ed6405d86fp-5},
    {0x1.e000000000000p-1, 0x1.08598b59e3a07p-4},
    {0x1.dc80000000000p-1, 0x1.26536c3d8c369p-4},
    {0x1.d900000000000p-1, 0x1.4485e03dbdfadp-4},
    {0x1.d600000000000p-1, 0x1.5e95a4d9791cbp-4},
    {0x1.d280000000000p-1, 0x1.7d33687c293c9p-4},
    {0x1.cf00000000000p-1, 0x1.9c0c32d4d2548p-4},
    {0x1.cc00000000000p-1, 0x1.b6ac88dad5b1cp-4},
    {0x1.c880000000000p-1, 0x1.d5f55659210e2p-4},
    {0x1.c580000000000p-1, 0x1.f0f70cdd992e3p-4},
    {0x1.c280000000000p-1, 0x1.06135354d4b18p-3},
    {0x1.bf80000000000p-1, 0x1.13c2605c398c3p-3},
    {0x1.bc80000000000p-1, 0x1.2188fd9807263p-3},
    {0x1.b980000000000p-1, 0x1.2f677cbbc0a96p-3},
    {0x1.b680000000000p-1, 0x1.3d5e3126bc27fp-3},
    {0x1.b380000000000p-1, 0x1.4b6d6fefe22a4p-3},
    {0x1.b080000000000p-1, 0x1.59958ff1d52f1p-3},
    {0x1.ad80000000000p-1, 0x1.67d6e9d785771p-3},
    {0x1.ab00000000000p-1, 0x1.73cb9074fd14dp-3},
    {0x1.a800000000000p-1, 0x1.823c16551a3c2p-3},
    {0x1.a580000000000p-1, 0x1.8e588ebac2dbfp-3},
    {0x1.a300000000000p-1, 0x1.9a8778debaa38p-3},
    {0x1.a000000000000p-1, 0x1.a93ed3c8ad9e3p-3},
    {0x1.9d80000000000p-1, 0x1.b5971a213acdbp-3},
    {0x1.9b00000000000p-1, 0x1.c2028ab17f9b4p-3},
    {0x1.9880000000000p-1, 0x1.ce816157f1988p-3},
    {0x1.9600000000000p-1, 0x1.db13db0d48940p-3},
    {0x1.9380000000000p-1, 0x1.e7ba35eb77e2ap-3},
    {0x1.9100000000000p-1, 0x1.f474b134df229p-3},
    {0x1.8e80000000000p-1, 0x1.00a1c6adda473p-2},
    {0x1.8c00000000000p-1, 0x1.07138604d5862p-2},
    {0x1.8980000000000p-1, 0x1.0d8fb813eb1efp-2},
    {0x1.8780000000000p-1, 0x1.12c77cd00713bp-2},
    {0x1.8500000000000p-1, 0x1.1956d3b9bc2fap-2},
    {0x1.8280000000000p-1, 0x1.1ff0fe7cf47a7p-2},
    {0x1.8080000000000p-1, 0x1.25410494e56c7p-2},
    {0x1.7e00000000000p-1, 0x1.2bef07cdc9354p-2},
    {0x1.7c00000000000p-1, 0x1.314f1e1d35ce4p-2},
    {0x1.7980000000000p-1, 0x1.3811728564cb2p-2},
    {0x1.7780000000000p-1, 0x1.3d81fb5946dbap-2},
    {0x1.7580000000000p-1, 0x1.42f9f3ff62642p-2},
    {0x1.7380000000000p-1, 0x1.487970e958770p-2},
    {0x1.7100000000000p-1, 0x1.4f637ebba9810p-2},
    {0x1.6f00000000000p-1, 0x1.54f431b7be1a9p-2},
    {0x1.6d00000000000p-1, 0x1.5a8cadbbedfa1p-2},
    {0x1.6b00000000000p-1, 0x1.602d08af091ecp-2},
    {0x1.6900000000000p-1, 0x1.65d558d4ce00bp-2},
    {0x1.6700000000000p-1, 0x1.6b85b4cffa3fdp-2},
    {0x1.6500000000000p-1, 0x1.713e33a46a17cp-2},
    {0x1.6300000000000p-1, 0x1.76feecb947175p-2},
    {0x1.6180000000000p-1, 0x1.7b54ec1077a47p-2},
    {0x1.5f80000000000p-1, 0x1.812444990af63p-2},
    {0x1.5d80000000000p-1, 0x1.86fc19d05148ep-2},
    {0x1.5b80000000000p-1, 0x1.8cdc84a65a0bep-2},
    {0x1.5a00000000000p-1, 0x1.914a8635bf68ap-2},
    {0x1.5800000000000p-1, 0x1.973a3431356aep-2},
    {0x1.5600000000000p-1, 0x1.9d32bea15ed3bp-2},
    {0x1.5480000000000p-1, 0x1.a1b3071f75fdap-2},
    {0x1.5280000000000p-1, 0x1.a7bb53abd5d20p-2},
    {0x1.5100000000000p-1, 0x1.ac478d020506fp-2},
    {0x1.4f00000000000p-1, 0x1.b25fefb60cb2ep-2},
    {0x1.4d80000000000p-1, 0x1.b6f859e8ef63ap-2},
    {0x1.4c00000000000p-1, 0x1.bb9611b80e2fbp-2},
    {0x1.4a00000000000p-1, 0x1.c1c60693fa39ep-2},
    {0x1.4880000000000p-1, 0x1.c6704e4016ff8p-2},
    {0x1.4700000000000p-1, 0x1.cb200d2ceb643p-2},
    {0x1.4500000000000p-1, 0x1.d1684d49f46aep-2},
    {0x1.4380000000000p-1, 0x1.d624ff7bb5d47p-2},
    {0x1.4200000000000p-1, 0x1.dae75484c9616p-2},
    {0x1.4080000000000p-1, 0x1.dfaf59de8c15dp-2},
    {0x1.3f00000000000p-1, 0x1.e47d1d32e677ep-2},
    {0x1.3d80000000000p-1, 0x1.e950ac5d36dc1p-2},
    {0x1.3c00000000000p-1, 0x1.ee2a156b413e5p-2},
    {0x1.3a80000000000p-1, 0x1.f309669e24cf8p-2},
    {0x1.3900000000000p-1, 0x1.f7eeae6b5761dp-2},
    {0x1.3780000000000p-1, 0x1.fcd9fb7da6defp-2},
    {0x1.3600000000000p-1, 0x1.00e5ae5b207abp-1},
    {0x1.3480000000000p-1, 0x1.03617096e0952p-1},
    {0x1.3300000000000p-1, 0x1.05e04c1aa2c06p-1},
    {0x1.3180000000000p-1, 0x1.086248abc4f3bp-1},
    {0x1.3000000000000p-1, 0x1.0ae76e2d054fap-1},
    {0x1.2e80000000000p-1, 0x1.0d6fc49f16e94p-1},
    {0x1.2d80000000000p-1, 0x1.0f21c81d1adc3p-1},
    {0x1.2c00000000000p-1, 0x1.11af823c75aa8p-1},
    {0x1.2a80000000000p-1, 0x1.1440833add112p-1},
    {0x1.2900000000000p-1, 0x1.16d4d38c119fap-1},
    {0x1.2800000000000p-1, 0x1.188ee40f23ca6p-1},
    {0x1.2680000000000p-1, 0x1.1b28cbb6ec93fp-1},
    {0x1.2500000000000p-1, 0x1.1dc619de06944p-1},
    {0x1.2400000000000p-1, 0x1.1f8635fc61659p-1},
    {0x1.2280000000000p-1, 0x1.222942e4a6a9cp-1},
    {0x1.2180000000000p-1, 0x1.23ed3bf21ca33p-1},
    {0x1.2000000000000p-1, 0x1.269621134db92p-1},
    {0x1.1f00000000000p-1, 0x1.285e0842ca384p-1},
    {0x1.1d80000000000p-1, 0x1.2b0cdfbf7ad03p-1},
    {0x1.1c80000000000p-1, 0x1.2cd8c6b7c716fp-1},
    {0x1.1b00000000000p-1, 0x1.2f8dab636337ap-1},
    {0x1.1a00000000000p-1, 0x1.315da4434068bp-1},
    {0x1.1880000000000p-1, 0x1.3418b1a85622dp-1},
    {0x1.1780000000000p-1, 0x1.35eccf0ac61d0p-1},
    {0x1.1680000000000p-1, 0x1.37c299f3c366ap-1},
    {0x1.1500000000000p-1, 0x1.3a86767257111p-1},
    {0x1.1400000000000p-1, 0x1.3c6080c36bfb5p-1},
    {0x1.1300000000000p-1, 0x1.3e3c43918f76cp-1},
    {0x1.1180000000000p-1, 0x1.410928b8f950fp-1},
    {0x1.1080000000000p-1, 0x1.42e946de080bfp-1},
    {0x1.0f80000000000p-1, 0x1.44cb28e37c3eep-1},
    {0x1.0e80000000000p-1, 0x1.46aed21f117fcp-1},
    {0x1.0d00000000000p-1, 0x1.4987ace0dabb0p-1},
    {0x1.0c00000000000p-1, 0x1.4b6fd6f970c1fp-1},
    {0x1.0b00000000000p-1, 0x1.4d59d43fdaba2p-1},
    {0x1.0a00000000000p-1, 0x1.4f45a835a4e19p-1},
    {0x1.0900000000000p-1, 0x1.513356667fc57p-1},
    {0x1.0780000000000p-1, 0x1.541b5cb979809p-1},
    {0x1.0680000000000p-1, 0x1.560dbc45153c7p-1},
    {0x1.0580000000000p-1, 0x1.580202c6c7353p-1},
    {0x1.0480000000000p-1, 0x1.59f833f9d4290p-1},
    {0x1.0380000000000p-1, 0x1.5bf053a48690ep-1},
    {0x1.0280000000000p-1, 0x1.5dea65985a350p-1},
    {0x1.0180000000000p-1, 0x1.5fe66db228992p-1},
    {0x1.0080000000000p-1, 0x1.61e46fda56467p-1},
};
__device__ __constant__ const double kRngLogLo[256] = {
    0x1.ac1bb52fa589bp-56,
    0x1.cc2470e8a3df4p-55,
    0x1.64b378f7d53bcp-57,
    0x1.ee438d52d09fep-55,
    0x1.8de1d5230047fp-55,
    -0x1.1cd4d414e008dp-55,
    -0x1.6122cbf70330cp-55,
    -0x1.d974ae53ee0f4p-55,
    -0x1.9192f30bd1806p-55,
    0x1.384627475439ap-55,
    0x1.2a5f2939df863p-56,
    0x1.82a26ba886ba7p-55,
    -0x1.1f8b734c91c5dp-56,
    -0x1.8feee4c8899f3p-55,
    0x1.1a158f3917586p-55,
    0x1.a9a012e8d760ap-57,
    0x1.73a2437885c68p-56,
    -0x1.65a1afa4aeb59p-56,
    -0x1.13b181e903212p-55,
    0x1.f804c80abfff2p-59,
    0x1.77b269d1a5bf7p-56,
    0x1.d57f617ac6361p-55,
    -0x1.e119102a87320p-57,
    0x1.4e9eb28262d05p-56,
    -0x1.188f43b1000b1p-56,
    -0x1.535b8ee4f9efep-58,
    -0x1.b7c4b07224e0fp-56,
    -0x1.3c7ada895ff22p-58,
    -0x1.a763b39986482p-57,
    0x1.328df13bb38c3p-56,
    -0x1.3a8c72437300dp-57,
    -0x1.667923e1f5a8ep-57,
    -0x1.d895037a878a6p-56,
    0x1.ced86a647ee26p-56,
    0x1.a025573934564p-58,
    0x1.79806026ca7dep-56,
    -0x1.e615815805b57p-60,
    0x1.0f3c590a887cap-59,
    0x1.0cafe295ea7d7p-57,
    0x1.fc0536ca18103p-56,
    -0x1.8163d6f46f714p-59,
    0x1.be36a306f4fc5p-56,
    -0x1.8847a1dd2d8acp-59,
    -0x1.5d557b4737216p-56,
    0x1.16cc8bae0bbe4p-56,
    0x1.735f3a17be3a7p-56,
    0x1.620cdb09632dcp-60,
    0x1.308b32ff78826p-57,
    -0x1.55747742b9ed3p-56,
    -0x1.99f82a5539353p-56,
    -0x1.3899df49cac22p-56,
    0x1.da856ccd987b3p-56,
    0x1.f893d41c411f1p-56,
    0x1.bc60efafc6f6ep-57,
    0x1.8ebcb7dee9a3dp-56,
    0x1.6aadc72eeb980p-56,
    -0x1.84de5807b96b5p-56,
    -0x1.c58ab60d731b6p-60,
    0x1.d70c8309edcfcp-56,
    0x1.4313e09807affp-58,
    0x1.ae6c8cab0b631p-58,
    0x1.06380e1a7d303p-57,
    0x1.8f4cdb95ebdf9p-56,
    -0x1.301771c407dbfp-56,
    0x1.9bae06a5c872dp-65,
    -0x1.84f64b5c47f86p-58,
    -0x1.9d3d1b0e4d147p-56,
    0x1.9e7a4a75619eep-56,
    -0x1.c56bd2abfe82ap-56,
    -0x1.8d20550a30eeep-56,
    0x1.ae944b3ae19cfp-56,
    -0x1.6e32d5e8c707fp-57,
    0x1.aad908df8942ep-58,
    0x1.b2ce30cd2d061p-58,
    -0x1.9f8294df883d6p-59,
    -0x1.6e443597e4d40p-57,
    -0x1.039a653793a85p-57,
    0x1.73dee38a3fb6bp-57,
    -0x1.bf2e78548fd89p-57,
    0x1.6f9007e0a0d70p-57,
    -0x1.a1366e2c5a7aap-57,
    0x1.59dbd32f67a3ap-57,
    -0x1.ea57c1c8d979fp-57,
    0x1.3cd2c57073be9p-58,
    0x1.83e270efcc373p-58,
    0x1.b264062a84cdbp-58,
    0x1.eedcbac2a7f18p-62,
    0x1.bc60efafc6f6ep-58,
    0x1.8d45e51106d5ep-58,
    0x1.ffa95a6aaa4edp-58,
    -0x1.9f4f6543e1f88p-57,
    0x1.220a8abf098f4p-60,
    -0x1.b234b8d209720p-58,
    -0x1.95991a883feffp-59,
    0x1.4e47b44db8540p-57,
    0x1.e540be89c1eaap-59,
    -0x1.9a5dc5e9030acp-57,
    0x1.6f9a332ca3851p-57,
    -0x1.2334824fcc6ebp-58,
    0x1.61578001e0162p-60,
    -0x1.80006a9c6606cp-58,
    0x1.e2db7c7d5a130p-58,
    -0x1.f17d2016d0e25p-59,
    0x1.2099e1c184e8ep-59,
    0x1.4a697ab3424a9p-61,
    -0x1.32861063fdf57p-58,
    0x1.b692c214ddbecp-58,
    0x1.a1cde5c772a1ap-58,
    -0x1.ddd4f935996c9p-59,
    0x1.b599f227becbbp-58,
    -0x1.d81c3373f1357p-58,
    -0x1.122b956232089p-58,
    -0x1.ba13162a9c446p-60,
    0x1.c270480fd528ep-60,
    -0x1.e5bafa0943c21p-60,
    -0x1.0539a473b598bp-60,
    -0x1.18d3ca87b9296p-59,
    0x1.ce55c2b4e2b72p-59,
    0x1.237a70db06b41p-60,
    0x1.876e3f4b360c5p-59,
    -0x1.7086b1c00b395p-63,
    0x1.4a3a50b6c5621p-61,
    0x1.b10b6c3ec21b4p-60,
    0x1.d41fe63d2dbf9p-61,
    0x1.f6842688f499ap-62,
    0x1.ff29a11443a06p-65,
    0x1.61e96e2fc5d90p-62,
    0x0.0p+0,
    0x0.0p+0,
    0x1.04b16137f09a0p-62,
    -0x1.8cdaf39004192p-60,
    0x1.1b8afbfe81965p-62,
    -0x1.c39390333b61cp-59,
    -0x1.bbf88ec501b56p-61,
    0x1.d60449ab527bfp-61,
    0x1.16aeb2214c8c0p-59,
    -0x1.dd7009902bf32p-58,
    0x1.d604be2dd16f0p-58,
    0x1.1ba349aadbc6ep-58,
    0x1.f38745c5c450ap-58,
    -0x1.cf063e63e7075p-58,
    0x1.fb0be3ccc1532p-59,
    -0x1.0057eed1ca59fp-59,
    0x1.ce60c2a34a8fbp-59,
    0x1.f6c272c1dca71p-60,
    0x1.18a0d03ba5397p-58,
    -0x1.fdd94f6508b88p-57,
    -0x1.e7f50c701268fp-60,
    -0x1.9fbd3e17e5527p-57,
    0x1.97c284b6258aap-57,
    0x1.767ab73ca8d5ep-57,
    0x1.f4d12c6bf5a87p-57,
    -0x1.10614e0da5fb8p-57,
    -0x1.521a000b4cf01p-57,
    -0x1.1232ce70be781p-57,
    -0x1.46a9a5dd7ff12p-57,
    0x1.f47dfd871f87fp-57,
    0x1.bcafa9de97203p-57,
    -0x1.e2f8aadc42f8fp-57,
    0x1.f11aa3853a5f1p-57,
    -0x1.5744132a297b0p-58,
    0x1.aa11d49f96cb9p-58,
    0x1.11dc86c9b7564p-59,
    -0x1.27c77ded76aadp-58,
    0x1.8d688b9e17a8ap-56,
    0x1.cdb16ed4e9138p-56,
    -0x1.cdde2b0172bd5p-56,
    0x1.4a4508fbcba26p-57,
    0x1.7b9d68d50a15dp-56,
    0x1.5b513ff0c1450p-56,
    0x1.7ac0ef77f252ap-56,
    -0x1.82dad7fd86088p-56,
    -0x1.3d69909e5c3dcp-56,
    -0x1.e493a0702b236p-57,
    0x1.c1eab1642e36dp-56,
    -0x1.bbf082ccabbaep-56,
    0x1.b8465cf25f4c6p-56,
    -0x1.58cb3124b9245p-56,
    -0x1.aacfdbbdab914p-56,
    -0x1.e6c2bdfb3e037p-58,
    -0x1.6e8920c09b73fp-58,
    -0x1.7605a4748480ap-56,
    -0x1.8af2c8dafcb08p-57,
    -0x1.9367a05ae38d3p-56,
    -0x1.118d9eb4ea362p-56,
    -0x1.f4a28f81eb9c0p-60,
    -0x1.f4a66509e8b12p-58,
    0x1.fc8edbd999effp-56,
    -0x1.15a95af2b82b1p-56,
    -0x1.ad4bb98c1f2c5p-56,
    -0x1.89d2816cf838fp-57,
    0x1.87bcbcfd3e187p-59,
    0x1.ac97bab6eae83p-56,
    0x1.724065bdf021dp-57,
    0x1.d19914a95df12p-61,
    0x1.831dd125d6faap-59,
    -0x1.9a1eef8667ea6p-60,
    0x1.6fd02999b21e1p-59,
    -0x1.bfc00b8f3feaap-56,
    0x1.e960f17e68fffp-57,
    -0x1.89974d2ba308ap-58,
    0x1.d98a582717953p-56,
    -0x1.adcda7b942268p-57,
    -0x1.0b5837185a661p-56,
    0x1.29fcb117ce2fdp-56,
    0x1.96e555e2df7d3p-58,
    0x1.e25f30aadfe0dp-58,
    -0x1.74b71fb5e57e3p-62,
    -0x1.d0039e7235f9bp-60,
    -0x1.ffca6a88d3d8ep-57,
    0x1.410c04b4523dfp-56,
    0x1.1713a36138e19p-57,
    0x1.06613ff7c588ep-55,
    0x1.862e53e393760p-60,
    -0x1.263d54b0aeae2p-55,
    0x1.0d710fcfc4e0dp-55,
    -0x1.f489e14a27ed9p-55,
    -0x1.309d8ecea08ffp-55,
    -0x1.91eee7772c7c2p-55,
    -0x1.210ab9d03bb19p-55,
    0x1.d7508e57620b2p-55,
    0x1.89df1568ca0b0p-55,
    -0x1.d6892112c5e91p-55,
    0x1.b50bb38388177p-57,
    -0x1.2164ff40e9817p-56,
    0x1.f5308ddb9794cp-55,
    0x1.6e637b589c198p-55,
    0x1.e0efadd9db02bp-55,
    -0x1.d93cc9506f200p-55,
    -0x1.6dbf9e9688bbap-55,
    0x1.b3236255261cdp-55,
    -0x1.9811700a1baf8p-55,
    0x1.6c3a5f12642c9p-57,
    -0x1.9832c00a1160dp-56,
    -0x1.e6916bc7308c6p-56,
    0x1.5c72c107ee28bp-56,
    0x1.700f448ce4d66p-56,
    0x1.1930603d87b6ep-56,
    0x1.59673d064b8bap-55,
    0x1.d01b962fa5df6p-55,
    0x1.028b250ee3fadp-60,
    -0x1.3103eafd25009p-56,
    0x1.a2be41f8e9f3dp-55,
    0x1.f68ae35979f60p-55,
    0x1.c457b531506f6p-55,
    -0x1.34d6c7eb974a5p-57,
    0x1.d749362382a77p-56,
    0x1.ca64cc3d52c87p-56,
    0x1.662e3a6b95f54p-57,
    -0x1.b3bb5c3530094p-55,
    -0x1.e4959621ef696p-58,
    -0x1.6547469fa3842p-62,
    0x1.9d1fa26ddeb2dp-59,
    -0x1.7336877bddda4p-56,
    0x1.c54625b15c6d6p-58,
    -0x1.ee18ba867d3a5p-56,
};

struct RngTabs {
    const double2* sc;     // [256] (sin, cos)(2 pi j / 256)
    const double2* li;     // [256] (invc, -log(invc) hi)
    const double* ll;      // [256] -log(invc) lo
};

// The block's copy of the tables (every lane of the block calls it, then the
// caller's barrier); 10 KB of LDS.
struct RngTabsLds {
    double2 sc[256];
    double2 li[256];
    double ll[256];
};
__device__ __forceinline__ RngTabs rng_tabs_stage(RngTabsLds* t, const int tid, const int nthreads) {
    for (int k = tid; k < 256; k += nthreads) {
        t->sc[k] = kRngSinCos256[k];
        t->li[k] = kRngLogInvHi[k];
        t->ll[k] = kRngLogLo[k];
    }
    return RngTabs{t->sc, t->li, t->ll};
}

// sin(2 pi u), cos(2 pi u), u = (b + 1) 2^-32 (B = 2^32 wraps to the same
// angle 0): the top 8 bits of B pick 2 pi j / 256 from the table, the low 24
// give r = rem 2 pi 2^-32 in [0, 2 pi / 256), whose sin / cos come from their
// Taylor polynomials in z = r^2 (truncation below 4e-18), then the angle
// addition (two roundings per component).
__device__ __forceinline__ void rng_sincos2pi_tab(const uint32_t b, const RngTabs& T, double* sp,
                                                  double* cp) {
    const uint32_t B = b + 1u;
    const double2 t = T.sc[B >> 24];
    const double r = (double)(B & 0xFFFFFFu) * 0x1.921fb54442d18p-30;   // rem x 2 pi / 2^32
    const double z = r * r;
    const double ps = fma_k(z, fma_k(z, fma_kk(z, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0),
                            -1.0 / 6.0);
    const double sr = fma(r * z, ps, r);
    const double pc = fma_k(z, fma_k(z, fma_kk(z, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5);
    const double cr = fma(z, pc, 1.0);
    *sp = fma(t.x, cr, t.y * sr);
    *cp = fma(t.y, cr, -(t.x * sr));
}

// sin / cos of a wrapped heading |x| <= pi + 0.1 (every particle heading of the
// velocity model's predict, motion_model.py:50-56) from the same LDS table of
// (sin, cos)(2 pi j / 256) the device RNG stages: j = rint(x 128 / pi), the
// remainder r = x - j pi/128 (|r| <= pi/256: the first fma is exact -- j pi1
// has <= 53 bits and lies within a factor 2 of x -- the second one rounds
// once), sin r and cos r by their Taylor polynomials to r^7 / r^6 (truncation
// below 3e-21 relative), then the angle addition: within ~1.5 ulp (the
// fdlibm-kernel fast_sincos: < 1 ulp) at half its issue cost.  Anything
// larger goes to fast_sincos.
__device__ __forceinline__ void heading_sincos_tab(const double x, const RngTabs& T, double* sp,
                                                   double* cp) {
    constexpr double k128Pi = 40.74366543152521;              // 128 / pi
    constexpr double kPi128Hi = 0x1.921fb54442dp-6;           // pi / 128, 45 significant bits
    constexpr double kPi128Lo = 0x1.8469898cc5170p-54;        // pi / 128 - kPi128Hi
    if (!(fabs(x) <= 3.2415926535897931)) {
        fast_sincos(x, sp, cp);
        return;
    }
    const double j = rint(x * k128Pi);
    const double r = fma(-j, kPi128Lo, fma(-j, kPi128Hi, x));
    const double2 t = T.sc[(int)j & 255];
    const double z = r * r;
    const double sr = fma(r * z, fma_k(z, fma_kk(z, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), r);
    const double cr = fma(z, fma_k(z, fma_kk(z, -1.0 / 720.0, 1.0 / 24.0), -0.5), 1.0);
    *sp = fma(t.x, cr, t.y * sr);
    *cp = fma(t.y, cr, -(t.x * sr));
}

// log((a + 1) 2^-32), a a 32-bit word: m in [sqrt(1/2), sqrt(2)) as in
// fdlibm, r = m invc - 1 (one rounding, |r| <= 2^-7), log1p(r) by its degree-8
// Taylor polynomial (truncation < 2e-18 relative), plus e ln2 and -log(invc)
// (within 1.3 ulp; no reciprocal).
__device__ __forceinline__ double rng_log_tab(const uint32_t a, const RngTabs& T) {
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double d = (double)a + 1.0;                      // exact, in [1, 2^32]
    int e = __builtin_amdgcn_frexp_exp(d) - 32;            // d 2^-32 = m 2^e, m in [0.5, 1)
    double m = __builtin_amdgcn_frexp_mant(d);
    if (m < 0.70710678118654752440) {
        m = m + m;
        e -= 1;
    }
    const uint32_t hi = (uint32_t)(__double_as_longlong(m) >> 32);
    const uint32_t j = ((hi >> 13) & 0x7Fu) | (((hi >> 20) & 1u) << 7);
    const double2 t = T.li[j];
    const double r = fma(m, t.x, -1.0);
    const double z = r * r;
    double q = fma_kk(r, -1.0 / 8.0, 1.0 / 7.0);
    q = fma_k(r, q, -1.0 / 6.0);
    q = fma_k(r, q, 1.0 / 5.0);
    q = fma_k(r, q, -1.0 / 4.0);
    q = fma_k(r, q, 1.0 / 3.0);
    q = fma(r, q, -0.5);
    const double de = (double)e;
    return fma(de, ln2_hi, t.y) + (r + (fma(de, ln2_lo, T.ll[j]) + z * q));
}

}  // namespace slam
