// ekf_kernels.inl -- EKF localisation (batched) and EKF-SLAM kernels (gfx950).
//
// Batched EKF: one lane owns one filter for a whole run; its state (3 + 9
// doubles) stays in registers across steps, only the observations stream in
// and the estimates stream out (16 B + 24 B per filter-step: HBM-bound).
//
// EKF-SLAM: the n x n covariance lives in HBM as a row-major matrix of which
// only the lower triangle (i >= j) is kept current.  The update is
//   PHt = P H^T   (n x m, m = 3k; H has 6 non-zeros per row)
//   S   = H PHt + R,  Sinv = S^-1   (one workgroup, in LDS)
//   K   = PHt Sinv,   mu += K e
//   P  -= K PHt^T    (lower triangle only; fp64 MFMA 16x16x4 tiles)
// The last line reads and writes the lower half of P once: 8 n^2 B per
// update, the HBM bound of the whole step.
#pragma once

#include "common.hpp"

namespace slam {

struct EKFConst {
    double dt, vel, omega;
    double q[9];
    double r[4];
    int32_t motion;          // SLAM_MOTION_LINEAR (the reference's __f) or _VELOCITY (motion_model.py)
    double alphas[6];        // motion_model.py:20-29 a1..a6 (velocity model)
};

// The prediction of an EKF driven by motion_model.py (north_star; oracle
// ekf_oracle.velocity_predict, same operation order):
//   f = moveWithoutNoise (motion_model.py:64-86): a = v / w, b = limit(w dt),
//       t1 = limit(t + b), x' = x + a (-sin t + sin t1), y' = y + a (cos t - cos t1);
//   G = d f / d(x, y, t): column 2 = (a (-cos t + cos t1), a (-sin t + sin t1), 1);
//   V = d f / d(v, w) (Thrun eq. 7.11), M = diag(sv^4, sw^4): moveWithNoise
//       hands sigma**2 to np.random.normal as the standard deviation (:46-47);
//   the yaw noise of gamma-hat (std sg^2, entering as gamma dt, :48, :56).
// Q = V M V^T + diag(0, 0, (sg^2 dt)^2) replaces the linear model's Q.
struct VelPredict {
    double xm, ym, tm, g02, g12;
    double q[9];
};

__device__ __forceinline__ VelPredict velocity_predict(const double x, const double y,
                                                       const double t, const double v,
                                                       const double om, const double dt,
                                                       const double* al) {
    VelPredict r;
    const double a = v / om;
    const double b = wrap_angle(om * dt);
    const double t1 = wrap_angle(t + b);
    double s0, c0, s1, c1;
    sincos(t, &s0, &c0);
    sincos(t1, &s1, &c1);
    r.xm = x + a * (-s0 + s1);
    r.ym = y + a * (c0 - c1);
    r.tm = t1;
    r.g02 = a * (-c0 + c1);
    r.g12 = a * (-s0 + s1);
    const double v00 = (-s0 + s1) / om, v10 = (c0 - c1) / om;
    const double v01 = (v * (s0 - s1)) / (om * om) + ((v * c1) * dt) / om;
    const double v11 = (-(v * (c0 - c1))) / (om * om) + ((v * s1) * dt) / om;
    const double v2 = v * v, w2 = om * om;
    const double sv = (al[0] * v2) + (al[1] * w2);
    const double sw = (al[2] * v2) + (al[3] * w2);
    const double sg = (al[4] * v2) + (al[5] * w2);
    const double mv = (sv * sv) * (sv * sv), mw = (sw * sw) * (sw * sw);
    const double gd = (sg * sg) * dt;
    const double mg = gd * gd;
    r.q[0] = ((v00 * v00) * mv) + ((v01 * v01) * mw);
    r.q[1] = ((v00 * v10) * mv) + ((v01 * v11) * mw);
    r.q[2] = (v01 * dt) * mw;
    r.q[4] = ((v10 * v10) * mv) + ((v11 * v11) * mw);
    r.q[5] = (v11 * dt) * mw;
    r.q[8] = ((dt * dt) * mw) + mg;
    r.q[3] = r.q[1];
    r.q[6] = r.q[2];
    r.q[7] = r.q[5];
    return r;
}

// One step of extended_kalman_filter.py:108-128 on a register-resident filter.
// Products with the structural 0/1 entries of A, B, C, jacobF are exact in the
// reference's BLAS calls; the remaining two-term sums follow OpenBLAS dgemm's
// accumulation (fma into a running sum, k ascending).  With c.motion =
// VELOCITY the prediction is velocity_predict's (G in place of jacobF, its Q).
__device__ __forceinline__ void ekf_filter_step(double& x, double& y, double& t, double* P,
                                                const double zx, const double zy, const double v,
                                                const double om, const EKFConst& c, double* xm_out) {
    double xm, ym, tm, f02, f12, q[9];
    if (c.motion == SLAM_MOTION_VELOCITY) {
        const VelPredict vp = velocity_predict(x, y, t, v, om, c.dt, c.alphas);
        xm = vp.xm;
        ym = vp.ym;
        tm = vp.tm;
        f02 = vp.g02;
        f12 = vp.g12;
#pragma unroll
        for (int k = 0; k < 9; ++k) q[k] = vp.q[k];
    } else {
        double sy, cy;
        sincos(t, &sy, &cy);
        // __f (:160-178): a = DT cos(yaw), b = DT sin(yaw); x' = A x + B u
        const double a = c.dt * cy, b = c.dt * sy;
        xm = x + v * a;
        ym = y + v * b;
        tm = wrap_angle(t + om * c.dt);
        // jacobF (:180-194) at the previous estimate
        f02 = (-c.dt) * v * sy;
        f12 = c.dt * v * cy;
#pragma unroll
        for (int k = 0; k < 9; ++k) q[k] = c.q[k];
    }
    // P_m = F P F^T + Q  (:117-118)
    double FP[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        FP[j] = fma(f02, P[6 + j], P[j]);
        FP[3 + j] = fma(f12, P[6 + j], P[3 + j]);
        FP[6 + j] = P[6 + j];
    }
    double Pm[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        Pm[3 * i + 0] = fma(FP[3 * i + 2], f02, FP[3 * i + 0]) + q[3 * i + 0];
        Pm[3 * i + 1] = fma(FP[3 * i + 2], f12, FP[3 * i + 1]) + q[3 * i + 1];
        Pm[3 * i + 2] = FP[3 * i + 2] + q[3 * i + 2];
    }
    // S = C P_m C^T + R; G = P_m C^T S^-1  (:149-158)
    const double s00 = Pm[0] + c.r[0], s01 = Pm[1] + c.r[1];
    const double s10 = Pm[3] + c.r[2], s11 = Pm[4] + c.r[3];
    // S^-1 by the adjugate with one correctly rounded reciprocal of det (the
    // reference's np.linalg.inv takes the LU route: neither form is its
    // rounding; four divisions cost 26 more fp64 VALU per filter-step)
    const double det = s00 * s11 - s01 * s10;
    const double rdet = 1.0 / det;
    const double i00 = s11 * rdet, i01 = -s01 * rdet, i10 = -s10 * rdet, i11 = s00 * rdet;
    double G[6];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        G[2 * i + 0] = fma(Pm[3 * i + 1], i10, Pm[3 * i + 0] * i00);
        G[2 * i + 1] = fma(Pm[3 * i + 1], i11, Pm[3 * i + 0] * i01);
    }
    // x_hat = x_m + G (z - C x_m), yaw wrapped  (:121-126)
    const double e0 = zx - xm, e1 = zy - ym;
    x = xm + fma(G[1], e1, G[0] * e0);
    y = ym + fma(G[3], e1, G[2] * e0);
    t = wrap_angle(tm + fma(G[5], e1, G[4] * e0));
    // P = (I - G C) P_m  (:128-129); the structural zeros of I - G C (third
    // column 0, 0, 1) contribute exact +0 / x terms: dropped / added directly
    const double M[6] = {1.0 - G[0], -G[1], -G[2], 1.0 - G[3], -G[4], -G[5]};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        P[j] = fma(M[1], Pm[3 + j], M[0] * Pm[j]);
        P[3 + j] = fma(M[3], Pm[3 + j], M[2] * Pm[j]);
        P[6 + j] = fma(M[5], Pm[3 + j], M[4] * Pm[j]) + Pm[6 + j];
    }
    if (xm_out) {
        xm_out[0] = xm;
        xm_out[1] = ym;
        xm_out[2] = tm;
    }
}

// n_steps steps for every filter in one launch.  SoA state: xs[3][B], Ps[9][B];
// z_all: [step][B][2]; xh_all: [step][B][3] (optional); xm_last: [B][3] x_hat_m
// of the last step (optional).
__global__ __launch_bounds__(256) void ekf_run_kernel(
    const int64_t B, const int32_t n_steps, const EKFConst c, const double v, const double om,
    double* __restrict__ xs, double* __restrict__ Ps, const double* __restrict__ z_all,
    double* __restrict__ xh_all, double* __restrict__ xm_last) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double x = xs[b], y = xs[B + b], t = xs[2 * B + b];
    double P[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) P[q] = Ps[q * B + b];
    double xm[3];
    for (int s = 0; s < n_steps; ++s) {
        const double2 z = reinterpret_cast<const double2*>(z_all)[(int64_t)s * B + b];
        ekf_filter_step(x, y, t, P, z.x, z.y, v, om, c, xm);
        if (xh_all) {
            double* o = xh_all + ((int64_t)s * B + b) * 3;
            o[0] = x;
            o[1] = y;
            o[2] = t;
        }
    }
    xs[b] = x;
    xs[B + b] = y;
    xs[2 * B + b] = t;
#pragma unroll
    for (int q = 0; q < 9; ++q) Ps[q * B + b] = P[q];
    if (xm_last && n_steps > 0) {
        xm_last[3 * b] = xm[0];
        xm_last[3 * b + 1] = xm[1];
        xm_last[3 * b + 2] = xm[2];
    }
}

// ====================================================================
// EKF-SLAM
// ====================================================================
constexpr int kEksTile = 128;        // rank-update tile (rows and columns)
constexpr int kEksThreads = 512;     // 8 waves: 4 (rows of 32) x 2 (columns of 64)
constexpr int kEksMaxM = 120;        // 3k <= 120 (S and S^-1 in LDS)
constexpr int kEksKC = 32;           // k-chunk staged in LDS per pass
constexpr int kEksKS = kEksKC + 1;   // odd LDS row stride: conflict-free fragment reads

struct EksConst {
    double dt;
    double q[9];
    double r_dist, r_dir, r_orient;
    int32_t motion;          // SLAM_MOTION_LINEAR / _VELOCITY (velocity_predict)
    double alphas[6];
};

// symmetric read from the lower-triangle storage
__device__ __forceinline__ double psym(const double* P, const int64_t ld, const int64_t i,
                                       const int64_t j) {
    return (i >= j) ? P[i * ld + j] : P[j * ld + i];
}

// Robot rows/columns of F P F^T (landmark part): P[i][0:3] <- P[i][0:3] F^T, i >= 3.
__global__ __launch_bounds__(256) void eks_predict_rows_kernel(double* __restrict__ P,
                                                               const int64_t n, const int64_t ld,
                                                               const double* __restrict__ mu,
                                                               const EksConst c, const double v,
                                                               const double om) {
    const int64_t i = 3 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double f02, f12;
    if (c.motion == SLAM_MOTION_VELOCITY) {
        const VelPredict vp = velocity_predict(mu[0], mu[1], mu[2], v, om, c.dt, c.alphas);
        f02 = vp.g02;
        f12 = vp.g12;
    } else {
        double sy, cy;
        sincos(mu[2], &sy, &cy);
        f02 = (-c.dt) * v * sy;
        f12 = c.dt * v * cy;
    }
    double* r = P + i * ld;
    const double p2 = r[2];
    r[0] = fma(p2, f02, r[0]);
    r[1] = fma(p2, f12, r[1]);
}

// Robot block and pose (after eks_predict_rows_kernel has read the old yaw).
__global__ void eks_predict_pose_kernel(double* __restrict__ P, const int64_t ld,
                                        double* __restrict__ mu, const EksConst c, const double v,
                                        const double om) {
    if (threadIdx.x != 0) return;
    const double x = mu[0], y = mu[1], t = mu[2];
    const bool vel = c.motion == SLAM_MOTION_VELOCITY;
    VelPredict vp{};
    double sy = 0.0, cy = 0.0, f02, f12;
    const double* q = c.q;
    if (vel) {
        vp = velocity_predict(x, y, t, v, om, c.dt, c.alphas);
        f02 = vp.g02;
        f12 = vp.g12;
        q = vp.q;
    } else {
        sincos(t, &sy, &cy);
        f02 = (-c.dt) * v * sy;
        f12 = c.dt * v * cy;
    }
    double p[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) p[3 * i + j] = psym(P, ld, i, j);
    double FP[9];
    for (int j = 0; j < 3; ++j) {
        FP[j] = fma(f02, p[6 + j], p[j]);
        FP[3 + j] = fma(f12, p[6 + j], p[3 + j]);
        FP[6 + j] = p[6 + j];
    }
    for (int i = 0; i < 3; ++i) {
        P[i * ld + 0] = fma(FP[3 * i + 2], f02, FP[3 * i + 0]) + q[3 * i + 0];
        P[i * ld + 1] = fma(FP[3 * i + 2], f12, FP[3 * i + 1]) + q[3 * i + 1];
        P[i * ld + 2] = FP[3 * i + 2] + q[3 * i + 2];
    }
    if (vel) {
        mu[0] = vp.xm;
        mu[1] = vp.ym;
        mu[2] = vp.tm;
        return;
    }
    const double a = c.dt * cy, b = c.dt * sy;
    mu[0] = x + v * a;
    mu[1] = y + v * b;
    mu[2] = wrap_angle(t + om * c.dt);
}

// Per observation t (landmark j = ids[t]): predicted ScanSensor measurement,
// its Jacobians (robot Hr, landmark Hl, 3x3 each), the wrapped innovation and
// the measurement variance diag(scan_cov(range)).  hs: [k][18]; e, rd: [M].
// The observed ids and measurements travel in the kernel arguments (1.3 KB,
// no host-to-device copies per update); the ids are stored for the later kernels.
struct EksObs {
    int64_t ids[kEksMaxM / 3];
    double obs[kEksMaxM];
};

__global__ void eks_build_kernel(const double* __restrict__ mu, const EksObs ob,
                                 int64_t* __restrict__ ids_out, const int32_t k, const int32_t M,
                                 const EksConst c, double* __restrict__ hs, double* __restrict__ e,
                                 double* __restrict__ rd) {
    const int t = threadIdx.x;
    for (int u = 3 * k + t; u < M; u += blockDim.x) {
        e[u] = 0.0;
        rd[u] = 1.0;
    }
    if (t >= k) return;
    const int64_t j = ob.ids[t];
    ids_out[t] = j;
    const double o[3] = {ob.obs[3 * t], ob.obs[3 * t + 1], ob.obs[3 * t + 2]};
    const double xr = mu[0], yr = mu[1], th = mu[2];
    const double lx = mu[3 + 3 * j], ly = mu[4 + 3 * j], lp = mu[5 + 3 * j];
    const double psi = kHalfPi - th;
    double s, co;
    sincos(psi, &s, &co);
    const double dx = lx - xr, dy = ly - yr;
    const double rx = co * dx - s * dy;
    const double ry = s * dx + co * dy;
    const double rng = hypot(rx, ry);
    const double brg = atan2(ry, rx);
    const double ori = wrap_angle(psi + lp);
    const double q = dx * dx + dy * dy;
    const double r = sqrt(q);
    double* H = hs + 18 * t;
    // Hr (d/d robot x, y, yaw)
    H[0] = -dx / r; H[1] = -dy / r; H[2] = 0.0;
    H[3] = dy / q;  H[4] = -dx / q; H[5] = -1.0;
    H[6] = 0.0;     H[7] = 0.0;     H[8] = -1.0;
    // Hl (d/d landmark x, y, phi)
    H[9] = dx / r;  H[10] = dy / r; H[11] = 0.0;
    H[12] = -dy / q; H[13] = dx / q; H[14] = 0.0;
    H[15] = 0.0;    H[16] = 0.0;    H[17] = 1.0;
    e[3 * t] = o[0] - rng;
    e[3 * t + 1] = wrap_angle(o[1] - brg);
    e[3 * t + 2] = wrap_angle(o[2] - ori);
    // graph_based_slam.py:187-192
    const double d = o[0] * c.r_dist;
    const double sd = o[0] * sin(c.r_dir);
    rd[3 * t] = d * d;
    rd[3 * t + 1] = sd * sd;
    rd[3 * t + 2] = c.r_dir * c.r_dir + c.r_orient * c.r_orient;
}

// PHt[i][u] = sum over the six non-zero columns of H row u of P[i][col] H[u][col]
// (one lane per row i; rows >= n and columns >= 3k are zero).
__global__ __launch_bounds__(256) void eks_pht_kernel(const double* __restrict__ P,
                                                      const int64_t n, const int64_t ld,
                                                      const int64_t n_pad,
                                                      const int64_t* __restrict__ ids,
                                                      const double* __restrict__ hs,
                                                      const int32_t k, const int32_t M,
                                                      double* __restrict__ pht) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    double* out = pht + i * M;
    if (i >= n) {
        for (int u = 0; u < M; ++u) out[u] = 0.0;
        return;
    }
    const double p0 = psym(P, ld, i, 0), p1 = psym(P, ld, i, 1), p2 = psym(P, ld, i, 2);
    // landmarks in groups of 8: the 24 P entries of a group are requested
    // together (one memory round trip per group, not per landmark)
    constexpr int kG = 8;
    for (int t0 = 0; t0 < k; t0 += kG) {
        double l[kG][3];
#pragma unroll
        for (int g = 0; g < kG; ++g) {
            if (t0 + g < k) {
                const int64_t c0 = 3 + 3 * ids[t0 + g];
#pragma unroll
                for (int j = 0; j < 3; ++j) l[g][j] = psym(P, ld, i, c0 + j);
            }
        }
#pragma unroll
        for (int g = 0; g < kG; ++g) {
            const int t = t0 + g;
            if (t < k) {
                const double* H = hs + 18 * t;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double acc = p0 * H[3 * a];
                    acc = fma(p1, H[3 * a + 1], acc);
                    acc = fma(p2, H[3 * a + 2], acc);
                    acc = fma(l[g][0], H[9 + 3 * a], acc);
                    acc = fma(l[g][1], H[9 + 3 * a + 1], acc);
                    acc = fma(l[g][2], H[9 + 3 * a + 2], acc);
                    out[3 * t + a] = acc;
                }
            }
        }
    }
    for (int u = 3 * k; u < M; ++u) out[u] = 0.0;
}

// S = H PHt + R (padded to M with the identity), inverted in place in LDS by
// Gauss-Jordan elimination (S is symmetric positive definite: no pivoting).
__global__ __launch_bounds__(1024) void eks_gain_kernel(const double* __restrict__ pht,
                                                        const int64_t* __restrict__ ids,
                                                        const double* __restrict__ hs,
                                                        const double* __restrict__ rd,
                                                        const int32_t k, const int32_t M,
                                                        double* __restrict__ sinv_out) {
    extern __shared__ double S[];           // M * M
    __shared__ double colp[kEksMaxM], rowp[kEksMaxM];
    const int m = 3 * k;
    for (int idx = threadIdx.x; idx < M * M; idx += blockDim.x) {
        const int a = idx / M, u = idx % M;
        double v;
        if (a < m && u < m) {
            const int t = a / 3, al = a % 3;
            const double* H = hs + 18 * t;
            const int64_t c0 = 3 + 3 * ids[t];
            double acc = H[3 * al] * pht[0 * M + u];
            acc = fma(H[3 * al + 1], pht[1 * M + u], acc);
            acc = fma(H[3 * al + 2], pht[2 * M + u], acc);
            acc = fma(H[9 + 3 * al], pht[c0 * M + u], acc);
            acc = fma(H[9 + 3 * al + 1], pht[(c0 + 1) * M + u], acc);
            acc = fma(H[9 + 3 * al + 2], pht[(c0 + 2) * M + u], acc);
            v = acc + ((a == u) ? rd[a] : 0.0);
        } else {
            v = (a == u) ? 1.0 : 0.0;
        }
        S[idx] = v;
    }
    __syncthreads();
    // Gauss-Jordan without pivoting (S is SPD), two barriers per pivot: the
    // pivot column and the scaled pivot row are captured from the old values,
    // then every entry is updated once.  Thread (r, j) of the 16 x 64 grid owns
    // columns j, j + 64 of rows r, r + 16, ... (no integer division).
    const int jl = threadIdx.x & 63, rl = threadIdx.x >> 6;
    for (int p = 0; p < M; ++p) {
        const double inv_p = 1.0 / S[p * M + p];
        for (int i = threadIdx.x; i < M; i += blockDim.x) {
            colp[i] = S[i * M + p];
            rowp[i] = (i == p) ? inv_p : S[p * M + i] * inv_p;
        }
        __syncthreads();
        for (int i = rl; i < M; i += 16)
            for (int j = jl; j < M; j += 64) {
                double v;
                if (i == p) v = rowp[j];
                else if (j == p) v = -colp[i] * inv_p;
                else v = S[i * M + j] - colp[i] * rowp[j];
                S[i * M + j] = v;
            }
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < M * M; idx += blockDim.x) sinv_out[idx] = S[idx];
}

// K = PHt S^-1 (rows of n_pad), mu += K e, yaw wrapped.
// K = PHt Sinv and mu += K e: one wave per row (rows strided over a resident
// grid), lane j forms K[i][j] and K[i][j + 64]; the PHt row is loaded once,
// coalesced, and its entries broadcast through SGPRs (v_readlane), Sinv is
// read from LDS along its rows.  Both sums run in the order of the one-lane-
// per-row form (v ascending from 0 with fma; dmu over u ascending).
constexpr int kEksApplyThreads = 1024;

__device__ __forceinline__ double readlane_d(const double x, const int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ __launch_bounds__(kEksApplyThreads) void eks_apply_kernel(
    const double* __restrict__ pht, const double* __restrict__ sinv, const double* __restrict__ e,
    const int64_t n, const int64_t n_pad, const int32_t M, double* __restrict__ kg,
    double* __restrict__ mu) {
    extern __shared__ double Si[];          // M * M
    __shared__ double es[kEksMaxM];
    for (int idx = threadIdx.x; idx < M * M; idx += blockDim.x) Si[idx] = sinv[idx];
    if (threadIdx.x < M) es[threadIdx.x] = e[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // lanes past M work on a clamped column (in-bounds, never stored): no
    // divergent branches in the loops
    const int j0 = min(lane, M - 1), j1 = min(lane + 64, M - 1);
    const bool c0 = lane < M, c1 = lane + 64 < M;
    const int64_t waves = (int64_t)gridDim.x * (kEksApplyThreads / 64);
    for (int64_t i = (int64_t)blockIdx.x * (kEksApplyThreads / 64) + (threadIdx.x >> 6);
         i < n_pad; i += waves) {
        const double* prow = pht + i * M;
        const double p0 = prow[j0], p1 = prow[j1];
        // M and 64 are multiples of 4: four broadcasts and eight LDS reads are
        // issued per group, the fma chains keep v ascending
        double k0 = 0.0, k1 = 0.0;
        for (int v = 0; v < M; v += 4) {
            const double src = (v < 64) ? p0 : p1;
            const int l = v & 63;
            double pv[4], s0[4], s1[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                pv[t] = readlane_d(src, l + t);
                s0[t] = Si[(v + t) * M + j0];
                s1[t] = Si[(v + t) * M + j1];
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                k0 = fma(pv[t], s0[t], k0);
                k1 = fma(pv[t], s1[t], k1);
            }
        }
        double* krow = kg + i * M;
        if (c0) krow[lane] = k0;
        if (c1) krow[lane + 64] = k1;
        if (i < n) {
            double dmu = 0.0;
            for (int u = 0; u < M; u += 4) {
                const double src = (u < 64) ? k0 : k1;
                const int l = u & 63;
                double kv[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) kv[t] = readlane_d(src, l + t);
#pragma unroll
                for (int t = 0; t < 4; ++t) dmu = fma(kv[t], es[u + t], dmu);
            }
            if (lane == 0) {
                double m = mu[i] + dmu;
                if (i == 2) m = wrap_angle(m);
                mu[i] = m;
            }
        }
    }
}

// Two workgroups per CU (4 waves per SIMD, <= 128 VGPRs): measured 2.33 ms per
// C4 update against 2.79 ms at the compiler's default of one workgroup per CU
// (144 VGPRs) -- the small spill of the bound costs less than the lost overlap.
#ifndef SLAM_EKS_WPE
#define SLAM_EKS_WPE 4
#endif
#define SLAM_EKS_ATTR __attribute__((amdgpu_waves_per_eu(SLAM_EKS_WPE)))
// P[i][j] -= sum_u K[i][u] PHt[j][u] for i >= j, one 128 x 128 lower tile per
// workgroup.  fp64 MFMA 16x16x4: A = K rows (lane l: row l&15, k l>>4),
// B = PHt^T (lane l: k l>>4, column l&15), D: column l&15, row (l>>4) + 4 r.
// Tiles are numbered so that each XCD (blockIdx % 8) takes a contiguous range
// of tile rows and reuses its K rows through its own L2.
__global__ __launch_bounds__(kEksThreads) SLAM_EKS_ATTR void eks_rank_update_kernel(
    double* __restrict__ P, const int64_t n, const int64_t ld, const double* __restrict__ kg,
    const double* __restrict__ pht, const int32_t M, const int64_t n_tiles) {
    __shared__ double Ks[kEksTile * kEksKS];    // K rows of the tile, one k-chunk
    __shared__ double Hs[kEksTile * kEksKS];    // PHt rows of the tile's columns
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t L = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (L >= n_tiles) return;
    int64_t ti = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > L) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
    const int64_t tj = L - ti * (ti + 1) / 2;
    const int64_t r0 = ti * kEksTile, c0 = tj * kEksTile;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = (wave >> 1) * 32;        // wave's 32 rows
    const int wc = (wave & 1) * 64;         // wave's 64 columns
    const int lr = lane & 15, lk = lane >> 4;
    typedef double double4v __attribute__((ext_vector_type(4)));
    // the P tile is the accumulators' starting value (loaded first, so its HBM
    // latency runs under the K / PH^T staging and the MFMAs); K is staged
    // negated, so the MFMAs leave P - K (PH^T)^T in place
    const bool diag = (ti == tj);
    double4v acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gi = r0 + wr + 16 * a + lk + 4 * r;
                const int64_t gj = c0 + wc + 16 * b + lr;
#ifdef EKS_PROBE_NOMEM
                acc[a][b][r] = (double)(gi ^ gj);
#else
                acc[a][b][r] = (gi < n && gj < n && (!diag || gj <= gi)) ? P[gi * ld + gj] : 0.0;
#endif
            }
    const double* ksrc = kg + r0 * M;
    const double* hsrc = pht + c0 * M;
#ifdef EKS_PROBE_NOMFMA
    for (int kc = 0; kc < 0; kc += kEksKC) {
#else
    for (int kc = 0; kc < M; kc += kEksKC) {
#endif
        const int kw = min(kEksKC, M - kc);             // multiple of 4
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kEksTile * kEksKC / kEksThreads; ++s) {
            const int idx = tid + s * kEksThreads;
            const int r = idx / kEksKC, q = idx % kEksKC;
            const bool ok = q < kw;
            Ks[r * kEksKS + q] = ok ? -ksrc[(int64_t)r * M + kc + q] : 0.0;
            Hs[r * kEksKS + q] = ok ? hsrc[(int64_t)r * M + kc + q] : 0.0;
        }
        __syncthreads();
        for (int k0 = 0; k0 < kw; k0 += 4) {
            double fa[2], fb[4];
#pragma unroll
            for (int a = 0; a < 2; ++a) fa[a] = Ks[(wr + 16 * a + lr) * kEksKS + k0 + lk];
#pragma unroll
            for (int b = 0; b < 4; ++b) fb[b] = Hs[(wc + 16 * b + lr) * kEksKS + k0 + lk];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gi = r0 + wr + 16 * a + lk + 4 * r;
                const int64_t gj = c0 + wc + 16 * b + lr;
#ifdef EKS_PROBE_NOMEM
                if (acc[a][b][r] == 1.2345) P[gi * ld + gj] = acc[a][b][r];
#else
                if (gi < n && gj < n && (!diag || gj <= gi)) P[gi * ld + gj] = acc[a][b][r];
#endif
            }
}

// Full symmetric copy-out of rows [i0, i0 + gridDim.y): dst[i - i0][j] = P_sym[i][j].
__global__ __launch_bounds__(256) void eks_symmetrize_kernel(const double* __restrict__ P,
                                                             const int64_t n, const int64_t ld,
                                                             const int64_t i0,
                                                             double* __restrict__ dst) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = i0 + blockIdx.y;
    if (j >= n || i >= n) return;
    dst[(int64_t)blockIdx.y * n + j] = psym(P, ld, i, j);
}

// rows[blockIdx.y] of the symmetric P (row i: the stored lower row, then
// column i of the lower triangle past the diagonal)
__global__ __launch_bounds__(256) void eks_gather_rows_kernel(const double* __restrict__ P,
                                                              const int64_t n, const int64_t ld,
                                                              const int64_t* __restrict__ rows,
                                                              double* __restrict__ dst) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = rows[blockIdx.y];
    if (j >= n) return;
    dst[(int64_t)blockIdx.y * n + j] = psym(P, ld, i, j);
}

__global__ __launch_bounds__(256) void eks_diag_kernel(double* __restrict__ P, const int64_t n,
                                                       const int64_t ld,
                                                       const double* __restrict__ dg) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) P[i * ld + i] = dg[i];
}


// ---------------------------------------------------------------------------
// Persistent, software-pipelined form of the same update for m <= 64 (the C4
// case): a workgroup walks the tiles of its XCD's band with a fixed stride and
// stages the whole k-range of K / PH^T in LDS at once (133 KB: one workgroup
// per CU, 2 waves per SIMD, up to 256 registers per lane).  While the MFMAs of
// tile t run, the P tile and the K / PH^T rows of tile t+1 are already in
// flight into a second register set.  The MFMA sequence per tile (k ascending
// in steps of 4) is the one of eks_rank_update_kernel: identical results.
constexpr int kEksPipeK = 64;
constexpr int kEksPipeKS = kEksPipeK + 1;
#ifndef SLAM_EKS_PIPE_WC
#define SLAM_EKS_PIPE_WC 2
#endif
// waves: 4 along the rows (32 each) x kEksPipeWC along the columns.  4 x 4
// (1024 threads, 4 waves per SIMD, 128 VGPRs with a small spill) measured
// 2.29 ms per C4 rank update against 2.06 ms for 4 x 2.
constexpr int kEksPipeWC = SLAM_EKS_PIPE_WC;
constexpr int kEksPipeThreads = 256 * kEksPipeWC;
constexpr int kEksPipeBB = 8 / kEksPipeWC;          // 16-column MFMA blocks per wave
constexpr int kEksPipeWPE = kEksPipeWC;             // waves per SIMD of the one workgroup per CU
typedef double eks_d4 __attribute__((ext_vector_type(4)));

// K = PH^T S^-1 and mu += K e for M <= 64 on the fp64 MFMA (the product is a
// GEMM, n_pad x M x M): one wave per 16-row strip, four 16-column blocks,
// v_mfma_f64_16x16x4 over the k-quads (entries past M read as 0), then each
// row's K e from its K entries (a 16-lane butterfly) and the mu update.
// 62 -> 26 us per C4 update against eks_apply_kernel (which stays for M > 64;
// SLAM_EKS_APPLY=lds selects it for comparison).
__global__ __launch_bounds__(256) void eks_apply_mfma_kernel(
    const double* __restrict__ pht, const double* __restrict__ sinv, const double* __restrict__ e,
    const int64_t n, const int64_t n_pad, const int32_t M, double* __restrict__ kg,
    double* __restrict__ mu) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    if (row0 >= n_pad) return;                       // wave-uniform
    eks_d4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = eks_d4{0.0, 0.0, 0.0, 0.0};
    const int nq = (M + 3) / 4;
    for (int q = 0; q < nq; ++q) {
        const int v = 4 * q + lk;
        const double a = (v < M) ? pht[(row0 + lr) * M + v] : 0.0;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const int u = 16 * cb + lr;
            const double b = (v < M && u < M) ? sinv[v * M + u] : 0.0;
            acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[cb], 0, 0, 0);
        }
    }
    double dm[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        const int u = 16 * cb + lr;
        const double eu = (u < M) ? e[u] : 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (u < M) kg[(row0 + lk + 4 * r) * M + u] = acc[cb][r];
            dm[r] = fma(acc[cb][r], eu, dm[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) dm[r] += __shfl_xor(dm[r], d, 64);
    if (lr == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = row0 + lk + 4 * r;
            if (i < n) {
                double m = mu[i] + dm[r];
                if (i == 2) m = wrap_angle(m);
                mu[i] = m;
            }
        }
    }
}

__device__ __forceinline__ void eks_tile_rc(const int64_t L, int64_t& ti, int64_t& tj) {
    ti = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > L) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
    tj = L - ti * (ti + 1) / 2;
}

__device__ __forceinline__ void eks_tile_load(eks_d4 (&t)[2][kEksPipeBB], const double* __restrict__ P,
                                              const int64_t n, const int64_t ld, const int64_t r0,
                                              const int64_t c0, const bool diag, const int wr,
                                              const int wc, const int lr, const int lk) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < kEksPipeBB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gi = r0 + wr + 16 * a + lk + 4 * r;
                const int64_t gj = c0 + wc + 16 * b + lr;
                t[a][b][r] = (gi < n && gj < n && (!diag || gj <= gi)) ? P[gi * ld + gj] : 0.0;
            }
}

constexpr int kEksPipePer = kEksTile * kEksPipeK / kEksPipeThreads;  // per lane and operand

__device__ __forceinline__ void eks_stage_load(double (&kv)[kEksPipePer], double (&hv)[kEksPipePer],
                                               const double* __restrict__ kg,
                                               const double* __restrict__ pht, const int32_t M,
                                               const int64_t r0, const int64_t c0) {
#pragma unroll
    for (int s = 0; s < kEksPipePer; ++s) {
        const int idx = threadIdx.x + s * kEksPipeThreads;
        const int r = idx / kEksPipeK, q = idx % kEksPipeK;
        const bool ok = q < M;
        kv[s] = ok ? -kg[(r0 + r) * M + q] : 0.0;       // K staged negated
        hv[s] = ok ? pht[(c0 + r) * M + q] : 0.0;
    }
}

__device__ __forceinline__ void eks_stage_store(const double (&kv)[kEksPipePer],
                                                const double (&hv)[kEksPipePer], double* Ks,
                                                double* Hs) {
#pragma unroll
    for (int s = 0; s < kEksPipePer; ++s) {
        const int idx = threadIdx.x + s * kEksPipeThreads;
        const int r = idx / kEksPipeK, q = idx % kEksPipeK;
        Ks[r * kEksPipeKS + q] = kv[s];
        Hs[r * kEksPipeKS + q] = hv[s];
    }
}

__device__ __forceinline__ void eks_frag_load(double (&fa)[2], double (&fb)[kEksPipeBB], const double* Ks,
                                              const double* Hs, const int k0, const int wr,
                                              const int wc, const int lr, const int lk) {
#pragma unroll
    for (int a = 0; a < 2; ++a) fa[a] = Ks[(wr + 16 * a + lr) * kEksPipeKS + k0 + lk];
#pragma unroll
    for (int b = 0; b < kEksPipeBB; ++b) fb[b] = Hs[(wc + 16 * b + lr) * kEksPipeKS + k0 + lk];
}

__device__ __forceinline__ void eks_frag_mfma(eks_d4 (&acc)[2][kEksPipeBB], const double (&fa)[2],
                                              const double (&fb)[kEksPipeBB]) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < kEksPipeBB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
}

__global__ __launch_bounds__(kEksPipeThreads) __attribute__((amdgpu_waves_per_eu(kEksPipeWPE)))
void eks_rank_update_pipelined_kernel(double* __restrict__ P, const int64_t n, const int64_t ld,
                                      const double* __restrict__ kg,
                                      const double* __restrict__ pht, const int32_t M,
                                      const int64_t n_tiles) {
    __shared__ double Ks[kEksTile * kEksPipeKS];
    __shared__ double Hs[kEksTile * kEksPipeKS];
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t xcd = blockIdx.x % 8, stride = gridDim.x / 8;
    const int64_t Lend = min(n_tiles, (xcd + 1) * per_xcd);
    int64_t L = xcd * per_xcd + blockIdx.x / 8;
    if (L >= Lend) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = (wave / kEksPipeWC) * 32, wc = (wave % kEksPipeWC) * (16 * kEksPipeBB);
    const int lr = lane & 15, lk = lane >> 4;
    int64_t ti, tj;
    eks_tile_rc(L, ti, tj);
    eks_d4 acc[2][kEksPipeBB], pre[2][kEksPipeBB];
    double kv[kEksPipePer], hv[kEksPipePer];
    eks_stage_load(kv, hv, kg, pht, M, ti * kEksTile, tj * kEksTile);
    eks_tile_load(acc, P, n, ld, ti * kEksTile, tj * kEksTile, ti == tj, wr, wc, lr, lk);
    eks_stage_store(kv, hv, Ks, Hs);
    __syncthreads();
    for (;;) {
        const int64_t r0 = ti * kEksTile, c0 = tj * kEksTile;
        const bool diag = (ti == tj);
        const int64_t Ln = L + stride;
        const bool more = Ln < Lend;
        int64_t tin = 0, tjn = 0;
        if (more) {
            eks_tile_rc(Ln, tin, tjn);
            eks_stage_load(kv, hv, kg, pht, M, tin * kEksTile, tjn * kEksTile);
#ifndef EKS_PROBE_NOMEM
            eks_tile_load(pre, P, n, ld, tin * kEksTile, tjn * kEksTile, tin == tjn, wr, wc, lr,
                          lk);
#endif
        }
        // k ascending in steps of 4; the fragments of step k+4 are read from
        // LDS while the MFMAs of step k run (two register sets)
        double fa0[2], fb0[kEksPipeBB], fa1[2], fb1[kEksPipeBB];
#ifdef EKS_PROBE_NOMFMA
        const int32_t Mk = 0;
#else
        const int32_t Mk = M;
#endif
        eks_frag_load(fa0, fb0, Ks, Hs, 0, wr, wc, lr, lk);
        int k0 = 0;
        for (; k0 + 4 < Mk; k0 += 8) {
            eks_frag_load(fa1, fb1, Ks, Hs, k0 + 4, wr, wc, lr, lk);
            eks_frag_mfma(acc, fa0, fb0);
            if (k0 + 8 < Mk) eks_frag_load(fa0, fb0, Ks, Hs, k0 + 8, wr, wc, lr, lk);
            eks_frag_mfma(acc, fa1, fb1);
        }
        if (k0 < Mk) eks_frag_mfma(acc, fa0, fb0);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < kEksPipeBB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gi = r0 + wr + 16 * a + lk + 4 * r;
                    const int64_t gj = c0 + wc + 16 * b + lr;
#ifdef EKS_PROBE_NOMEM
                    if (acc[a][b][r] == 1.2345) P[gi * ld + gj] = acc[a][b][r];
#else
                    if (gi < n && gj < n && (!diag || gj <= gi)) P[gi * ld + gj] = acc[a][b][r];
#endif
                }
        if (!more) break;
        __syncthreads();                // every wave is done reading this tile's K / PH^T
        eks_stage_store(kv, hv, Ks, Hs);
        __syncthreads();
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < kEksPipeBB; ++b) {
#ifdef EKS_PROBE_NOMEM
                acc[a][b] += 1.0;
#else
                acc[a][b] = pre[a][b];
#endif
            }
        L = Ln;
        ti = tin;
        tj = tjn;
    }
}

// ---- Fragment-streaming rank update (m <= 64): no LDS, no barriers.
//
// K (negated) and PH^T are first rewritten quad-major (eks_frag_layout_kernel):
// Kf[((q * n_pad) + row) * 4 + j] = -K[row][4 q + j], so the 16 x 4 MFMA
// operand of any 16 rows and k-quad q is one contiguous 512-byte run -- a
// wave loads it straight from L2 into registers.  Each wave then owns a
// 32 x 64 block of the 128 x 128 lower tile and walks the tiles on its own:
// while the MFMAs of the tile's last quads run, the next tile's P block and
// first operand quads are already in flight, and the waves of a SIMD drift out
// of phase, so HBM traffic and MFMA overlap without workgroup barriers (the
// LDS-staged kernels align every wave on two barriers per tile).
// Wave block (16 WM) x (16 WN); the 128 x 128 tile holds (8 / WM) x (8 / WN)
// waves.  2 x 4: 8 waves, 2 per SIMD (254 VGPRs); 2 x 2: 16 waves, 4 per SIMD.
template <int WM, int WN>
struct EksFragShape {
    static constexpr int kWaves = (8 / WM) * (8 / WN);
    static constexpr int kThreads = 64 * kWaves;
    static constexpr int kWavesPerSimd = kWaves / 4;
};

__global__ void eks_frag_layout_kernel(const double* __restrict__ kg, const double* __restrict__ pht,
                                       const int64_t n_pad, const int32_t M,
                                       double* __restrict__ Kf, double* __restrict__ Hf) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_pad * M) return;
    const int64_t i = idx / M;
    const int u = (int)(idx - i * M);
    const int64_t o = (((int64_t)(u >> 2) * n_pad) + i) * 4 + (u & 3);
    Kf[o] = -kg[idx];
    Hf[o] = pht[idx];
}

template <int Q, int WM, int WN, int PFQ = -1>
__global__ __launch_bounds__(64 * (8 / WM) * (8 / WN))
__attribute__((amdgpu_waves_per_eu((8 / WM) * (8 / WN) / 4)))
void eks_rank_update_frag_kernel(double* __restrict__ P, const int64_t n, const int64_t ld,
                                 const double* __restrict__ Kf, const double* __restrict__ Hf,
                                 const int64_t n_pad, const int64_t n_tiles) {
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t xcd = blockIdx.x % 8, stride = gridDim.x / 8;
    const int64_t Lend = min(n_tiles, (xcd + 1) * per_xcd);
    int64_t L = xcd * per_xcd + blockIdx.x / 8;
    if (L >= Lend) return;
    constexpr int WPR = 8 / WN;                              // waves along a tile row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave / WPR) * (16 * WM), wc = (wave % WPR) * (16 * WN);
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t qstride = n_pad * 4;                      // doubles per quad
    int64_t ti, tj;
    eks_tile_rc(L, ti, tj);
    eks_d4 acc[WM][WN], pre[WM][WN];
    double fa[3][WM], fb[3][WN];
    auto load_quad = [&](double (&a)[WM], double (&b)[WN], const int64_t r0, const int64_t c0,
                         const int q) {
        const double* kq = Kf + q * qstride + lk;
        const double* hq = Hf + q * qstride + lk;
#pragma unroll
        for (int x = 0; x < WM; ++x) a[x] = kq[(r0 + wr + 16 * x + lr) * 4];
#pragma unroll
        for (int y = 0; y < WN; ++y) b[y] = hq[(c0 + wc + 16 * y + lr) * 4];
    };
    auto load_p = [&](eks_d4 (&t)[WM][WN], const int64_t r0, const int64_t c0, const bool diag) {
#ifdef EKS_PROBE_NOMEM
#pragma unroll
        for (int x = 0; x < WM; ++x)
#pragma unroll
            for (int y = 0; y < WN; ++y) t[x][y] = eks_d4{(double)r0, (double)c0, 0.0, (double)diag};
        return;
#endif
#pragma unroll
        for (int x = 0; x < WM; ++x)
#pragma unroll
            for (int y = 0; y < WN; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gi = r0 + wr + 16 * x + lk + 4 * r;
                    const int64_t gj = c0 + wc + 16 * y + lr;
                    // P streams through once per update: non-temporal loads keep
                    // it from evicting the K / PH^T operand quads from L2
                    // (1.91 -> 1.81 ms per C4 update; non-temporal stores too:
                    // 1.84 ms)
                    t[x][y][r] = (gi < n && gj < n && (!diag || gj <= gi))
                                     ? __builtin_nontemporal_load(&P[gi * ld + gj])
                                     : 0.0;
                }
    };
    load_p(acc, ti * kEksTile, tj * kEksTile, ti == tj);
    load_quad(fa[0], fb[0], ti * kEksTile, tj * kEksTile, 0);
    if (Q > 1) load_quad(fa[1], fb[1], ti * kEksTile, tj * kEksTile, 1);
    for (;;) {
        const int64_t r0 = ti * kEksTile, c0 = tj * kEksTile;
        const bool diag = (ti == tj);
        const int64_t Ln = L + stride;
        const bool more = Ln < Lend;
        int64_t tin = 0, tjn = 0;
        if (more) eks_tile_rc(Ln, tin, tjn);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (q + 2 < Q) load_quad(fa[(q + 2) % 3], fb[(q + 2) % 3], r0, c0, q + 2);
            // the next tile's P block is requested at the top of the tile
            // (HBM latency is the long pole; measured 1.76 ms per C4 update
            // against 1.88 ms with the request after the last operand quad)
            constexpr int kPf = PFQ >= 0 ? (PFQ < Q ? PFQ : Q - 1) : 0;
            if (more && q == kPf) load_p(pre, tin * kEksTile, tjn * kEksTile, tin == tjn);
            const int s = q % 3;
#pragma unroll
            for (int x = 0; x < WM; ++x)
#pragma unroll
                for (int y = 0; y < WN; ++y)
#ifdef EKS_PROBE_NOMFMA
                    acc[x][y][0] += fa[s][x] * fb[s][y];
#else
                    acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s][x], fb[s][y], acc[x][y], 0, 0, 0);
#endif
        }
        if (more) {                                          // the next tile's first quads
            load_quad(fa[0], fb[0], tin * kEksTile, tjn * kEksTile, 0);
            if (Q > 1) load_quad(fa[1], fb[1], tin * kEksTile, tjn * kEksTile, 1);
        }
#pragma unroll
        for (int x = 0; x < WM; ++x)
#pragma unroll
            for (int y = 0; y < WN; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gi = r0 + wr + 16 * x + lk + 4 * r;
                    const int64_t gj = c0 + wc + 16 * y + lr;
#ifdef EKS_PROBE_NOMEM
                    if (acc[x][y][r] == 1.2345) P[gi * ld + gj] = acc[x][y][r];
#else
                    if (gi < n && gj < n && (!diag || gj <= gi)) P[gi * ld + gj] = acc[x][y][r];
#endif
                }
        if (!more) break;
#pragma unroll
        for (int x = 0; x < WM; ++x)
#pragma unroll
            for (int y = 0; y < WN; ++y) acc[x][y] = pre[x][y];
        L = Ln;
        ti = tin;
        tj = tjn;
    }
}

}  // namespace slam
