// pf_kernels.hpp -- particle-filter kernel interfaces (device side).
#pragma once
#include "common.hpp"

namespace slam {

constexpr int kMotionNone = 2;     // internal: likelihood-only pass

// Per-step closed-form words of the iso log-sum likelihood (StepIO.zc, one
// slot of kZcWords doubles per step), formed on the device at the start of
// every step (closed_prep_*):
//  * kZcSum + 2k, k < 8: S_ll, S_lx, S_ly, S_zz, S_zx, S_zy, D, E as
//    double-double (hi, lo) pairs -- the sums of landmarks / observations of
//    the step (the double-double form of likelihood_lanes);
//  * the expansion about the step's reference pose (p^, c^, s^): F^ = the
//    exact sum of squared residuals at it, A, B (gradient in the rotation)
//    and L2 (landmark second moment about p^) as double-doubles (hi, lo),
//    S_r (residual sum) and L1 (landmark sum about p^) rounded.
enum : int {
    kZcSum = 0,
    kZcPx = 16, kZcPy, kZcC, kZcS,
    kZcFh, kZcFl, kZcA, kZcAl, kZcB, kZcBl, kZcL2, kZcL2l,
    kZcSrx, kZcSry, kZcL1x, kZcL1y,
    kZcWords = 40,
};
constexpr int kClosedWords = kZcWords;
constexpr int kSumChunk = 8192;     // np.sum buffer size (particle_filter.py:234 order)
constexpr int kScanBlock = 2048;    // elements per block of the exact-cumsum passes
constexpr int kScanThreads = 256;
constexpr int kScanPer = kScanBlock / kScanThreads;  // 8
constexpr int kNormThreads = 256;
constexpr int kNormEPT = 4;                          // particles per lane in normalize
constexpr int kNormPer = kNormThreads * kNormEPT;    // particles per normalize block
#ifndef SLAM_DEFER_PPT
#define SLAM_DEFER_PPT 2
#endif
constexpr int kDeferPPT = SLAM_DEFER_PPT;            // particles per lane, deferred fused kernel
constexpr int kPartPer = 256 * kDeferPPT;            // particles per fused block (deferred path)

// Deferred normalisation (single-GPU handles): the fused kernel leaves, per
// kPartPer-particle block, its max unnormalised weight M_b with the first index,
// sums scaled by 1/M_b (sum u, sum u^2, sum u d, sum u d d^T with u = w_un/M_b
// and d = particle - refp; scaling keeps squares of tiny likelihoods out of
// the subnormal range) and its np.sum subtree (the pairwise sum of its four
// 128-element leaves).
// Per block also: the largest w_un before the first max (-1 if none), so
// the step end knows without a rescan whether a smaller weight can round to
// the same normalised maximum, and the particle at the first max (x_est).
struct DeferParts {
    double* pmax;
    int64_t* pidx;
    double* ppre;           // max w_un at indices before pidx (-1: none)
    double* pxe[3];         // particle (x, y, th) at pidx
    double* ps[11];         // sw, sw2, m1[3], m2[6]
    double* leaf;           // [blocks] the block's np.sum subtree (its kPartPer / 128 leaves, pairwise)
    int64_t* mark;          // [npad] resample-run starts: (RNG step << 32) | source (expand pass)
    int32_t* carry;         // [blocks] source of each fused block's first position
    // the resample gather reads source v at (x - goff)[v]: 0 on single-GPU
    // handles; npad on a sharded handle, whose particle arrays carry npad
    // staging slots on either side (particles received from lower ranks at
    // v = p, its own at npad + j, from higher ranks at 2 npad + p, so the
    // running max over a block's marks stays monotone)
    int64_t goff;
    int64_t glim;           // sources >= glim: the reference's IndexError (n; 3 npad when sharded)
};

// particle_filter.py:179-181 + the mlab.bivariate_normal constants
struct LikConst {
    double sx2, sy2;        // sigmax**2, sigmay**2 (as numpy squares the sqrt)
    double rsx2, rsy2;      // RN(1/sx2), RN(1/sy2) for the FMA-refined quotients
    double rho2;            // 2*rho
    double sxsy;            // sigmax*sigmay
    double d2;              // 2*(1-rho**2)
    double den, rden;       // 2*pi*sx*sy*sqrt(1-rho**2) and RN(1/den)
    double neg_nl_ln_den;   // -NL*log(den) (log-sum form)
    double rsxsy, rd2;      // RN(1/(sx*sy)), RN(1/d2) (log-sum form)
    double fast_min_l;      // log-sum form: L >= this -> exp(L); below, logsum_slow
                            // (every partial product provably stays normal above it)
    double normal_min_l;    // ln(DBL_MIN) + 1: a log prefix above it is a normal partial product
    double neg_ln_den;      // -log(den): log-prefix increment per landmark
    double expand_vmax;     // closed form: the expansion about the step's reference
                            // pose is taken when the particle's bound V <= this
                            // (|dL| <= 1e-14); beyond it the double-double form
    int32_t has_rho;
    int32_t iso;            // sx2 == sy2 and rho == 0 (log-sum shortcut)
    int32_t nl;
    int32_t closed;         // iso log-sum from the per-step landmark/observation sums (StepIO.zc)
};

struct PredictConst {
    double dt;
    double alphas[6];       // motion_model.py:20-29 a1..a6
    double q[9];            // device-RNG noise map for the linear model
    double np_recip;        // 1/NP (particle_filter.py:32), NP = global particle count
    double rstep;           // arange step 1/NP (particle_filter.py:213)
    int64_t n_global;       // global particle count (RNG counter space)
    int64_t gbase;          // global index of local particle 0
};

// Device-resident per-step inputs/outputs of a loaded batch.  Kernels read the
// step index from ctr[0] (advanced by the last block of normalize_kernel), so
// one captured step graph replays unchanged for every step.
struct StepIO {
    const double* ctl;      // [cap][2] control (v, omega)
    const double* z;        // [cap][2*NL] robot-frame observations
    double* zc;             // [cap][kZcWords] closed-form words (formed on the device per step)
    const double* ofs;      // [cap] host resample offset (NaN: device RNG)
    slam_pf_result* res;    // [cap] result records
    slam_pf_result* res_host;   // [cap] coherent pinned copy (device address): the last step of
                                // a device-resident batch stores the batch's records there
    int32_t* ctr;           // [0] step within the batch, [1] global RNG step, [2] / [3] the
                            // batch's first / last step (slam_pf_run's setup)
    int32_t cap;            // steps the arrays hold (the step end prepares step ctr[0] + 1 < cap)
    int32_t motion;         // the handle's motion model (reference pose of the expansion)
    double ess_band;        // result.ess_near: |ess - ESS_TH| <= ess_band * ESS_TH
};

struct BlockPartial {
    double maxv;
    int64_t maxi;
    double sw, sw2;
    double m1[3];
    double m2[6];
};

struct SpecialIn {
    int64_t idx;            // global element index
    uint64_t P;             // inclusive prefix of the integer increments
    double w;
    int32_t E;              // binade of the run that follows
    int32_t pad;
};

struct SpecialOut {
    double cs;              // exact cumsum at the special element
    uint64_t P;
    int32_t E;
    int32_t pad;
};

// device flag words
enum : int {
    kFlagResample = 0,      // resample at the start of the next step (ESS < ESS_TH)
    kFlagStatus = 1,        // bit0 clamp (reference IndexError), bit1 scan fallback
    kFlagNSpecial = 2,
    kFlagFallback = 3,
    kFlagMarkGen = 4,       // tag of the resample-run marks, advanced by every step end
    kFlagScanToken = 5,     // release token of the merged exact-cumsum launch
    kFlagDistDead = 6,      // sharded step: a peer wait expired once (sticky: later waits are skipped)
    kFlagDDWaves = 7,       // closed form: wavefronts of this step that took the double-double form
    kFlagWords = 8,
};

// Closed-form log-sum sums of one step (likelihood_lanes, iso): S_ll = sum |l|^2,
// S_l = sum l, S_zz = sum |z|^2, S_z = sum z, D = sum z.l, E = sum (z_y l_x - z_x l_y),
// each a double-double (hi, lo) -- exact products, compensated sums.  The same
// operations on the host (observations loaded from the caller) and on the
// device (observations simulated there).
struct DDSum {
    double h = 0.0, l = 0.0;
    __host__ __device__ void add(const double bh, const double bl = 0.0) {
        const double t = h + bh;
        const double bb = t - h;
        const double e = ((h - (t - bb)) + (bh - bb)) + (l + bl);
        h = t + e;
        l = e - (h - t);
    }
    __host__ __device__ void add_prod(const double a, const double b) {
        const double p = a * b;
        add(p, fma(a, b, -p));
    }
};

// DDSum of two double-double partials (the second added as (h, l))
__host__ __device__ inline DDSum dd_join(DDSum a, const DDSum& b) {
    a.add(b.h, b.l);
    return a;
}

// component k (0 S_ll, 1 S_lx, 2 S_ly, 3 S_zz, 4 S_zx, 5 S_zy, 6 D, 7 E) of
// landmark j's terms, added to S
__host__ __device__ inline void closed_term(DDSum& S, const int k, const double lx, const double ly,
                                            const double zx, const double zy) {
    switch (k) {
        case 0: S.add_prod(lx, lx); S.add_prod(ly, ly); break;
        case 1: S.add(lx); break;
        case 2: S.add(ly); break;
        case 3: S.add_prod(zx, zx); S.add_prod(zy, zy); break;
        case 4: S.add(zx); break;
        case 5: S.add(zy); break;
        case 6: S.add_prod(zx, lx); S.add_prod(zy, ly); break;
        default: S.add_prod(zy, lx); S.add_prod(-zx, ly); break;
    }
}

// The fixed summation order, shared by host and device: 64 lane partials
// (lane t takes landmarks t, t + 64, ... in order), then a butterfly over the
// lanes (offset 1, 2, ..., 32; the lower lane's partial on the left).
constexpr int kClosedLanes = 64;

__host__ __device__ inline DDSum closed_lane_partial(const int k, const int lane, const double* lm,
                                                     const double* z, const int32_t nl) {
    DDSum S;
    for (int32_t j = lane; j < nl; j += kClosedLanes)
        closed_term(S, k, lm[2 * j], lm[2 * j + 1], z[2 * j], z[2 * j + 1]);
    return S;
}

}  // namespace slam
