// common.hpp -- shared host/device helpers for libslam_hip.so (gfx950 only).
//
// Numerics contract: every translation unit is compiled with
// -ffp-contract=off, so an a*b+c in this code is two roundings exactly like
// NumPy; a fused multiply-add is written as fma() where the reference's BLAS
// kernel fuses (mylib/transform.py:33 via OpenBLAS dgemm).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/slam_hip.h"
#include "fastmath.hpp"

namespace slam {

// ------------------------------------------------------------------ errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define SLAM_HIP_TRY(expr)                                                        \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess)                                                     \
            return ::slam::fail(SLAM_ERR_HIP, std::string(#expr) + ": " +         \
                                                  hipGetErrorString(e_));         \
    } while (0)

#define SLAM_ARG_CHECK(cond, msg)                                                 \
    do {                                                                          \
        if (!(cond)) return ::slam::fail(SLAM_ERR_ARG, msg);                      \
    } while (0)

// --------------------------------------------------------------- constants
constexpr double kPi = 3.141592653589793;        // np.pi
constexpr double kTwoPi = 6.283185307179586;     // np.pi * 2  (mylib/limit.py:23)
constexpr double kHalfPi = 1.5707963267948966;   // np.pi / 2.0 (mylib/transform.py:12)

// --------------------------------------------------------- device helpers
// mylib/limit.py:11-26: repeated subtraction of 2*pi from |a|, sign restored.
// The iteration cap only matters for |a| > 6.6e6 rad (and +-inf, which loops
// forever in the reference): such inputs come back unreduced.
__device__ __forceinline__ double wrap_angle(double a) {
    double r = fabs(a);
    int guard = 0;
    while (r > kPi && guard < (1 << 20)) {
        r -= kTwoPi;
        ++guard;
    }
    return (a < 0.0) ? -r : r;
}

// ---------------------------------------------------------- Philox-4x32-10
struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// 53-bit uniform in (0, 1].
__device__ __forceinline__ double u01_open0(uint32_t a, uint32_t b) {
    const uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return ((double)m + 1.0) * 0x1p-53;
}

// Two standard normals (Box-Muller) from one Philox block.
__device__ __forceinline__ void normal2(u32x4 r, double& n0, double& n1) {
    const double u1 = u01_open0(r.x, r.y);
    const double u2 = u01_open0(r.z, r.w);
    const double rad = sqrt(-2.0 * log(u1));
    double s, c;
    sincospi(2.0 * u2, &s, &c);
    n0 = rad * c;
    n1 = rad * s;
}

// Three standard normals from ONE Philox block: two Box-Muller pairs on 32-bit
// uniforms in (0, 1] (radius resolution 2^-32: |g| <= 6.66, a tail mass of
// 3e-11 per draw); the fourth normal of the block is not formed.  Half the
// Philox work of 53-bit uniforms; the per-step motion noise needs three
// normals per particle.  log and sin/cos from fastmath.hpp (< 2 ulp).
__device__ __forceinline__ void normal3(u32x4 r, double& n0, double& n1, double& n2) {
    const double d1 = (double)r.x + 1.0;                 // u = d 2^-32, exact
    const double u2 = ((double)r.y + 1.0) * 0x1p-32;
    const double d3 = (double)r.z + 1.0;
    const double u4 = ((double)r.w + 1.0) * 0x1p-32;
    const double ra = sqrt(-2.0 * rng_log_scaled(d1, -32));
    const double rb = sqrt(-2.0 * rng_log_scaled(d3, -32));
    double s, c;
    rng_sincos2pi(u2, &s, &c);
    n0 = ra * c;
    n1 = ra * s;
    rng_sincos2pi(u4, &s, &c);
    n2 = rb * c;
}

// RNG stream ids (counter word z)
enum : uint32_t { kStreamPredict = 1, kStreamResample = 2 };

// --------------------------------------------------- exact-cumsum binades
// Binade of a non-negative running sum: E such that s in [2^E, 2^(E+1));
// every s below 2^-1021 (zero and subnormals included) shares the uniform
// grid 2^-1074 and is binade -1022.
__device__ __forceinline__ int sum_binade(double s) {
    return (s < 0x1p-1021) ? -1022 : ilogb(s);
}

}  // namespace slam
