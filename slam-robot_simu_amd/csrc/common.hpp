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
        // one 32 x 32 -> 64 product per word (v_mad_u64_u32) for both halves
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
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

// Philox-2x32-10 (Random123): one 64-bit counter, one 32-bit key.
__device__ __forceinline__ void philox2x32(uint32_t& c0, uint32_t& c1, uint32_t k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p = (uint64_t)0xD256D193u * c0;
        const uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
        c0 = hi ^ k ^ c1;
        c1 = lo;
        k += 0x9E3779B9u;
    }
}

// One Box-Muller pair from two 32-bit words: uniforms (a + 1) 2^-32 and
// (b + 1) 2^-32 in (0, 1] (radius resolution 2^-32: |g| <= 6.66, a tail mass of
// 3e-11 per draw); log and sin/cos from the LDS tables of fastmath.hpp
// (rng_log_tab, rng_sincos2pi_tab: < 1.5 ulp), sqrt_pos.
__device__ __forceinline__ void bm_pair(uint32_t a, uint32_t b, const RngTabs& T, double& gc,
                                        double& gs) {
#ifdef SLAM_RNG_NO_TABLES                                   // A/B diagnostic: the round-2 forms
    (void)T;
    const double rad = sqrt_pos(-2.0 * rng_log_scaled((double)a + 1.0, -32));
    double s, c;
    rng_sincos2pi(((double)b + 1.0) * 0x1p-32, &s, &c);
#else
    const double rad = sqrt_pos(-2.0 * rng_log_tab(a, T));
    double s, c;
    rng_sincos2pi_tab(b, T, &s, &c);
#endif
    gc = rad * c;
    gs = rad * s;
}

// RNG stream ids (counter word z / Philox-2x32 key salt)
enum : uint32_t { kStreamPredict = 1, kStreamResample = 2, kStreamPredict2 = 3 };

// The six standard normals of particle pair p (particles 2p and 2p+1) at RNG
// step `rstep`: a Philox-4x32-10 block (counter p, kStreamPredict, rstep) feeds
// Box-Muller pairs A and B, a Philox-2x32-10 block (counter (p, rstep), key
// seed ^ kStreamPredict2 salt) pair C.  Particle 2p draws (A.c, A.s, B.c),
// particle 2p+1 (B.s, C.c, C.s): three pairs per two particles, no normal
// formed and dropped.
__device__ __forceinline__ void pair_normals(const uint64_t p, const uint32_t rstep,
                                             const uint64_t seed, const RngTabs& T, double g[6]) {
    const u32x4 r = philox4x32(u32x4{(uint32_t)p, (uint32_t)(p >> 32), kStreamPredict, rstep},
                               (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t c0 = (uint32_t)p, c1 = rstep;
    philox2x32(c0, c1, ((uint32_t)seed ^ (uint32_t)(seed >> 32) * 0x85EBCA6Bu) ^ (kStreamPredict2 * 0x27D4EB2Fu));
    bm_pair(r.x, r.y, T, g[0], g[1]);
    bm_pair(r.z, r.w, T, g[2], g[3]);
    bm_pair(c0, c1, T, g[4], g[5]);
}


// --------------------------------------------------- exact-cumsum binades
// Binade of a non-negative running sum: E such that s in [2^E, 2^(E+1));
// every s below 2^-1021 (zero and subnormals included) shares the uniform
// grid 2^-1074 and is binade -1022.
__device__ __forceinline__ int sum_binade(double s) {
    return (s < 0x1p-1021) ? -1022 : ilogb(s);
}

}  // namespace slam
