// graph_kernels.inl -- graph-based SLAM linearise / assemble / solve (gfx950).
//
// graph_based_slam.py: TrajectoryEstimator.setPairObs (:362-439) becomes one
// lane per edge writing its six blocks (42 doubles, structure-of-arrays);
// updateEstPose (:452-514) becomes a deterministic block assembly -- every
// 3x3 block of H and every 3-vector of b is summed in the reference's edge
// order by one lane per entry, from a plan built once per edge set -- and one
// of two solvers:
//   * dense (n <= kGraphDenseMax): LU with partial pivoting (det as numpy
//     computes it: sign * exp(sum log|u_kk|)), the 2-norm condition number
//     from a full Lanczos tridiagonalisation of sym(H) with full
//     re-orthogonalisation, the reference's gate (0.1 < det, cond < 1e15),
//     and delta = -H^-1 b by the LU factors;
//   * PCG on the 3x3 block-sparse H with a block-Jacobi preconditioner (large
//     trajectories, BASELINE config 5): det and cond are not formed.
#pragma once

#include "common.hpp"

namespace slam {

constexpr int kGraphDenseMax = 2048;    // unknowns handled by the dense path
constexpr int kGraphThreads = 1024;     // single-workgroup dense kernels

struct GraphConst {
    double r_dist, r_dir, r_orient;
};

// ------------------------------------------------------------- linearise
__device__ __forceinline__ void mat3_mul(const double* A, const double* B, double* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = A[3 * i] * B[j];
            acc = fma(A[3 * i + 1], B[3 + j], acc);
            C[3 * i + j] = fma(A[3 * i + 2], B[6 + j], acc);
        }
}

__device__ __forceinline__ void mat3_tmul(const double* A, const double* B, double* C) {
    // C = A^T B
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = A[i] * B[j];
            acc = fma(A[3 + i], B[3 + j], acc);
            C[3 * i + j] = fma(A[6 + i], B[6 + j], acc);
        }
}

// ScanSensor.getLandMarkCovMatrixOnMeasurementSys + tfMeasurement2World
// (graph_based_slam.py:175-215): R(ang) diag(v) R(ang)^T, ang = dir + yaw - pi/2.
__device__ __forceinline__ void meas_cov_world(const double dist, const double dir,
                                               const double yaw, const GraphConst& g,
                                               double* C) {
    const double dd = dist * g.r_dist;
    const double sd = dist * sin(g.r_dir);
    const double v0 = dd * dd, v1 = sd * sd, v2 = g.r_dir * g.r_dir + g.r_orient * g.r_orient;
    const double ang = dir + yaw - kHalfPi;
    double s, c;
    sincos(ang, &s, &c);
    // (R D) R^T with the structural zeros of R and D dropped (they add exact zeros)
    const double rd00 = c * v0, rd01 = -s * v1, rd10 = s * v0, rd11 = c * v1;
    C[0] = fma(rd01, -s, rd00 * c);
    C[1] = fma(rd01, c, rd00 * s);
    C[2] = 0.0;
    C[3] = fma(rd11, -s, rd10 * c);
    C[4] = fma(rd11, c, rd10 * s);
    C[5] = 0.0;
    C[6] = 0.0;
    C[7] = 0.0;
    C[8] = v2;
}

// 3x3 inverse by LU with partial pivoting (the LAPACK getrf/getrs route numpy's inv takes).
__device__ __forceinline__ void inv3_lu(const double* S, double* X) {
    double a[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) a[q] = S[q];
    int perm[3] = {0, 1, 2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int p = k;
        for (int i = k + 1; i < 3; ++i)
            if (fabs(a[3 * i + k]) > fabs(a[3 * p + k])) p = i;
        if (p != k) {
            for (int j = 0; j < 3; ++j) {
                const double t = a[3 * k + j];
                a[3 * k + j] = a[3 * p + j];
                a[3 * p + j] = t;
            }
            const int t = perm[k];
            perm[k] = perm[p];
            perm[p] = t;
        }
        const double r = 1.0 / a[4 * k];
        for (int i = k + 1; i < 3; ++i) {
            a[3 * i + k] *= r;
            for (int j = k + 1; j < 3; ++j) a[3 * i + j] -= a[3 * i + k] * a[3 * k + j];
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double x[3];
        for (int i = 0; i < 3; ++i) x[i] = (perm[i] == j) ? 1.0 : 0.0;
        for (int k = 0; k < 3; ++k)
            for (int i = k + 1; i < 3; ++i) x[i] -= x[k] * a[3 * i + k];
        for (int k = 2; k >= 0; --k) {
            x[k] /= a[4 * k];
            for (int i = 0; i < k; ++i) x[i] -= x[k] * a[3 * i + k];
        }
        for (int i = 0; i < 3; ++i) X[3 * i + j] = x[i];
    }
}

// One lane per edge: setPairObs (:362-439).  blocks: SoA [42][E] = BB, BA, AB,
// AA (row-major 3x3), b_B, b_A.
__global__ __launch_bounds__(256) void graph_linearize_kernel(const int64_t E,
                                                              const slam_graph_edge* __restrict__ edges,
                                                              const double* __restrict__ poses,
                                                              const GraphConst g,
                                                              double* __restrict__ blocks) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const slam_graph_edge ed = edges[e];
    const double* xb = poses + 3 * ed.pose_bfr;
    const double* xa = poses + 3 * ed.pose_aft;
    const double db = ed.obs_bfr[0], ab = ed.obs_bfr[1], ob = ed.obs_bfr[2];
    const double da = ed.obs_aft[0], aa = ed.obs_aft[1], oa = ed.obs_aft[2];
    // relative pose from the estimates (:517-537)
    const double rx = xa[0] - xb[0], ry = xa[1] - xb[1];
    const double rt = wrap_angle(xa[2] - xb[2]);
    // relative pose from the observations (:539-581)
    const double la1 = wrap_angle(kPi + aa - oa), la2 = wrap_angle(kHalfPi - oa);
    const double lb1 = wrap_angle(kPi + ab - ob), lb2 = wrap_angle(kHalfPi - ob);
    double sa, ca, sb, cb;
    sincos(la1, &sa, &ca);
    sincos(lb1, &sb, &cb);
    const double px = da * ca - db * cb;
    const double py = da * sa - db * sb;
    const double pt = wrap_angle(la2 - lb2);
    const double err[3] = {rx - px, ry - py, wrap_angle(rt - pt)};
    // information matrix (:410-417)
    double Ca[9], Cb[9], S[9], W[9];
    meas_cov_world(da, aa, xa[2], g, Ca);
    meas_cov_world(db, ab, xb[2], g, Cb);
#pragma unroll
    for (int q = 0; q < 9; ++q) S[q] = Ca[q] + Cb[q];
    inv3_lu(S, W);
    // Jacobians (:420-427)
    double st, ct;
    sincos(wrap_angle(xb[2] + ab), &st, &ct);
    const double Jb[9] = {-1.0, 0.0, db * st, 0.0, -1.0, -db * ct, 0.0, 0.0, -1.0};
    sincos(wrap_angle(xa[2] + aa), &st, &ct);
    const double Ja[9] = {1.0, 0.0, -da * st, 0.0, 1.0, da * ct, 0.0, 0.0, 1.0};
    double JbW[9], JaW[9], out[9];
    mat3_tmul(Jb, W, JbW);
    mat3_tmul(Ja, W, JaW);
    mat3_mul(JbW, Jb, out);
#pragma unroll
    for (int q = 0; q < 9; ++q) blocks[(int64_t)q * E + e] = out[q];
    mat3_mul(JbW, Ja, out);
#pragma unroll
    for (int q = 0; q < 9; ++q) blocks[(int64_t)(9 + q) * E + e] = out[q];
    mat3_mul(JaW, Jb, out);
#pragma unroll
    for (int q = 0; q < 9; ++q) blocks[(int64_t)(18 + q) * E + e] = out[q];
    mat3_mul(JaW, Ja, out);
#pragma unroll
    for (int q = 0; q < 9; ++q) blocks[(int64_t)(27 + q) * E + e] = out[q];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double acc = JbW[3 * i] * err[0];
        acc = fma(JbW[3 * i + 1], err[1], acc);
        blocks[(int64_t)(36 + i) * E + e] = fma(JbW[3 * i + 2], err[2], acc);
        acc = JaW[3 * i] * err[0];
        acc = fma(JaW[3 * i + 1], err[1], acc);
        blocks[(int64_t)(39 + i) * E + e] = fma(JaW[3 * i + 2], err[2], acc);
    }
}

// --------------------------------------------------------------- pairing
// estimateOpticalTrajectory :697-703, one lane per output edge e: its landmark
// l (last pair offset <= e), its rank k among l's pairs, and the combination
// (i, j), i < j, of itertools.combinations order: row i holds the m - 1 - i
// pairs (i, i+1 .. m-1), C(i) = i (2m - i - 1) / 2 pairs precede it.
__device__ __forceinline__ int64_t comb_before(const int64_t i, const int64_t m) {
    return i * (2 * m - i - 1) / 2;
}

__global__ __launch_bounds__(256) void graph_pair_kernel(
    const int64_t E, const int64_t n_lm, const int64_t* __restrict__ pair_off,
    const int64_t* __restrict__ lm_start, const slam_graph_half* __restrict__ grouped,
    slam_graph_edge* __restrict__ edges) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int64_t lo = 0, hi = n_lm;                  // pair_off[lo] <= e < pair_off[hi]
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (pair_off[mid] <= e) lo = mid;
        else hi = mid;
    }
    const int64_t m = lm_start[lo + 1] - lm_start[lo];
    const int64_t k = e - pair_off[lo];
    const double b = (double)(2 * m - 1);
    int64_t i = (int64_t)((b - sqrt(fmax(b * b - 8.0 * (double)k, 0.0))) * 0.5);
    if (i < 0) i = 0;
    if (i > m - 2) i = m - 2;
    while (i > 0 && comb_before(i, m) > k) --i;
    while (i < m - 2 && comb_before(i + 1, m) <= k) ++i;
    const int64_t j = k - comb_before(i, m) + i + 1;
    const slam_graph_half* ha = grouped + lm_start[lo] + i;
    const slam_graph_half* hb = grouped + lm_start[lo] + j;
    if (ha->time > hb->time) {                  // setPairObs :371-384
        const slam_graph_half* t = ha;
        ha = hb;
        hb = t;
    }
    slam_graph_edge out;
    out.time_bfr = ha->time;
    out.pose_bfr = ha->pose;
    out.time_aft = hb->time;
    out.pose_aft = hb->pose;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        out.obs_bfr[q] = ha->obs[q];
        out.obs_aft[q] = hb->obs[q];
    }
    edges[e] = out;
}

// -------------------------------------------------------------- assemble
// One lane per (block slot, entry): the slot's contributions in edge order
// (code = 4 e + part), starting from the anchor on slot 0 (:475).
__global__ __launch_bounds__(256) void graph_assemble_h_kernel(
    const int64_t n_slots, const int64_t E, const int64_t* __restrict__ cptr,
    const int64_t* __restrict__ clist, const double* __restrict__ blocks, const double anchor,
    double* __restrict__ val) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_slots * 9) return;
    const int64_t s = t / 9;
    const int q = (int)(t - s * 9);
    double acc = (s == 0 && (q == 0 || q == 4 || q == 8)) ? anchor : 0.0;
    // groups of 8 contributions: the codes, then the block entries, are loaded
    // together (a diagonal slot collects ~8 edges); the adds stay in edge order
    const int64_t c1 = cptr[s + 1];
    for (int64_t c0 = cptr[s]; c0 < c1; c0 += 8) {
        int64_t code[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) code[u] = (c0 + u < c1) ? clist[c0 + u] : -1;
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = (code[u] >= 0) ? blocks[(int64_t)((int)(code[u] & 3) * 9 + q) * E + (code[u] >> 2)]
                                  : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (code[u] >= 0) acc = acc + v[u];
    }
    val[t] = acc;
}

// b: one lane per (block row, entry); code = 2 e + side (0: bfr, 1: aft).
__global__ __launch_bounds__(256) void graph_assemble_b_kernel(
    const int64_t n_rows, const int64_t E, const int64_t* __restrict__ bptr,
    const int64_t* __restrict__ blist, const double* __restrict__ blocks, double* __restrict__ b) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rows * 3) return;
    const int64_t r = t / 3;
    const int a = (int)(t - r * 3);
    double acc = 0.0;
    const int64_t c1 = bptr[r + 1];
    for (int64_t c0 = bptr[r]; c0 < c1; c0 += 8) {
        int64_t code[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) code[u] = (c0 + u < c1) ? blist[c0 + u] : -1;
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = (code[u] >= 0) ? blocks[(int64_t)(36 + 3 * (code[u] & 1) + a) * E + (code[u] >> 1)]
                                  : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (code[u] >= 0) acc = acc + v[u];
    }
    b[t] = acc;
}

// BSR -> dense (n x n, zeroed beforehand)
__global__ __launch_bounds__(256) void graph_dense_scatter_kernel(
    const int64_t n_slots, const int64_t* __restrict__ srow, const int64_t* __restrict__ scol,
    const double* __restrict__ val, const int64_t n, double* __restrict__ A) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_slots * 9) return;
    const int64_t s = t / 9;
    const int q = (int)(t - s * 9);
    A[(3 * srow[s] + q / 3) * n + 3 * scol[s] + q % 3] = val[t];
}

// ----------------------------------------------------- block reductions
template <int NT>
__device__ __forceinline__ double block_sum_fixed(double v, double* sh) {
    // fixed-shape tree: xor butterfly inside the wave, waves in order
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
    for (int w = 0; w < NT / 64; ++w) r += sh[w];
    __syncthreads();
    return r;
}

template <int NT>
__device__ __forceinline__ void block_sum2_fixed(double& a, double& b, double* sh) {
    // two sums through one LDS round; sh holds 2 * NT / 64 doubles
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        a += __shfl_xor(a, d, 64);
        b += __shfl_xor(b, d, 64);
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        sh[threadIdx.x >> 6] = a;
        sh[NT / 64 + (threadIdx.x >> 6)] = b;
    }
    __syncthreads();
    a = 0.0;
    b = 0.0;
    for (int w = 0; w < NT / 64; ++w) {
        a += sh[w];
        b += sh[NT / 64 + w];
    }
    __syncthreads();
}

// --------------------------------------------------- dense LU (getrf)
// One workgroup.  A (n x n row-major) is overwritten by L\U, piv[k] = row
// swapped with k.  out: [0] = sign, [1] = sum log|u_kk|, [2] = 1 if a zero pivot.
__global__ __launch_bounds__(kGraphThreads) void graph_lu_kernel(double* __restrict__ A,
                                                                 const int n,
                                                                 int32_t* __restrict__ piv,
                                                                 double* __restrict__ out) {
    __shared__ double shv[kGraphThreads / 64];
    __shared__ int shi[kGraphThreads / 64];
    __shared__ int s_p;
    __shared__ double s_sign;
    __shared__ int s_zero;
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_sign = 1.0;
        s_zero = 0;
    }
    for (int k = 0; k < n; ++k) {
        // pivot: first row of max |A[i][k]|, i >= k (idamax)
        double bv = -1.0;
        int bi = n;
        for (int i = k + tid; i < n; i += kGraphThreads) {
            const double v = fabs(A[(int64_t)i * n + k]);
            if (v > bv) {
                bv = v;
                bi = i;
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const double ov = __shfl_xor(bv, d, 64);
            const int oi = __shfl_xor(bi, d, 64);
            if (ov > bv || (ov == bv && oi < bi)) {
                bv = ov;
                bi = oi;
            }
        }
        if ((tid & 63) == 0) {
            shv[tid >> 6] = bv;
            shi[tid >> 6] = bi;
        }
        __syncthreads();
        if (tid == 0) {
            double v = shv[0];
            int p = shi[0];
            for (int w = 1; w < kGraphThreads / 64; ++w)
                if (shv[w] > v || (shv[w] == v && shi[w] < p)) {
                    v = shv[w];
                    p = shi[w];
                }
            if (p >= n) p = k;
            s_p = p;
            piv[k] = p;
            if (p != k) s_sign = -s_sign;
        }
        __syncthreads();
        const int p = s_p;
        if (p != k)
            for (int j = tid; j < n; j += kGraphThreads) {
                const double t = A[(int64_t)k * n + j];
                A[(int64_t)k * n + j] = A[(int64_t)p * n + j];
                A[(int64_t)p * n + j] = t;
            }
        __syncthreads();
        const double ukk = A[(int64_t)k * n + k];
        if (ukk == 0.0) {
            if (tid == 0) s_zero = 1;
            __syncthreads();
            continue;
        }
        const double r = 1.0 / ukk;
        for (int i = k + 1 + tid; i < n; i += kGraphThreads) A[(int64_t)i * n + k] *= r;
        __syncthreads();
        // rank-1 update of the trailing block: one wave per row, lanes along j
        const int lane = tid & 63;
        for (int i = k + 1 + (tid >> 6); i < n; i += kGraphThreads / 64) {
            double* ai = A + (int64_t)i * n;
            const double lik = ai[k];
            const double* ak = A + (int64_t)k * n;
            for (int j = k + 1 + lane; j < n; j += 64) ai[j] -= lik * ak[j];
        }
        __syncthreads();
    }
    if (tid == 0) {
        double lg = 0.0, sg = s_sign;
        for (int k = 0; k < n; ++k) {
            const double u = A[(int64_t)k * n + k];
            if (u < 0.0) sg = -sg;
            lg += log(fabs(u));
        }
        out[0] = sg;
        out[1] = lg;
        out[2] = (double)s_zero;
    }
}

// x = -(LU)^-1 b (getrs with the pivots), one workgroup.  x may alias nothing.
__global__ __launch_bounds__(kGraphThreads) void graph_lu_solve_kernel(
    const double* __restrict__ LU, const int n, const int32_t* __restrict__ piv,
    const double* __restrict__ b, double* __restrict__ x) {
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += kGraphThreads) x[i] = b[i];
    __syncthreads();
    if (tid == 0)
        for (int k = 0; k < n; ++k)
            if (piv[k] != k) {
                const double t = x[k];
                x[k] = x[piv[k]];
                x[piv[k]] = t;
            }
    __syncthreads();
    for (int k = 0; k < n; ++k) {          // unit lower
        const double xk = x[k];
        for (int i = k + 1 + tid; i < n; i += kGraphThreads) x[i] -= xk * LU[(int64_t)i * n + k];
        __syncthreads();
    }
    for (int k = n - 1; k >= 0; --k) {     // upper
        if (tid == 0) x[k] /= LU[(int64_t)k * n + k];
        __syncthreads();
        const double xk = x[k];
        for (int i = tid; i < k; i += kGraphThreads) x[i] -= xk * LU[(int64_t)i * n + k];
        __syncthreads();
    }
    for (int i = tid; i < n; i += kGraphThreads) x[i] = -x[i];
}

// S = (A + A^T) / 2
__global__ __launch_bounds__(256) void graph_symmetrize_kernel(const double* __restrict__ A,
                                                               const int64_t n,
                                                               double* __restrict__ S) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * n) return;
    const int64_t i = t / n, j = t % n;
    S[t] = 0.5 * (A[i * n + j] + A[j * n + i]);
}

// Lanczos with full re-orthogonalisation on the symmetric S (n x n), m = n
// steps (restarting on breakdown), one workgroup; V: n x (n + 1) scratch,
// ab: alpha[n], beta[n].  Then the extreme |eigenvalues| of the tridiagonal
// by Sturm bisection: out[0] = max |lambda|, out[1] = min |lambda|.
__device__ int sturm_count(const double* al, const double* be, const int m, const double x) {
    // number of eigenvalues < x
    int c = 0;
    double q = al[0] - x;
    if (q < 0.0) ++c;
    for (int i = 1; i < m; ++i) {
        if (q == 0.0) q = 1e-300;
        q = (al[i] - x) - be[i - 1] * be[i - 1] / q;
        if (q < 0.0) ++c;
    }
    return c;
}

__device__ double kth_eig(const double* al, const double* be, const int m, const int k,
                          double lo, double hi) {
    // k-th smallest (0-based) eigenvalue by bisection to full precision
    for (int it = 0; it < 2100; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        if (sturm_count(al, be, m, mid) > k) hi = mid;
        else lo = mid;
    }
    return 0.5 * (lo + hi);
}

__global__ __launch_bounds__(kGraphThreads) void graph_lanczos_kernel(
    const double* __restrict__ S, const int n, double* __restrict__ V, double* __restrict__ al,
    double* __restrict__ be, double* __restrict__ h, double* __restrict__ out, const uint64_t seed) {
    __shared__ double sh[kGraphThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NW = kGraphThreads / 64;
    // start vector: Philox uniforms (deterministic, not orthogonal to anything)
    auto fill_random = [&](double* v, uint32_t salt) {
        for (int i = tid; i < n; i += kGraphThreads) {
            const u32x4 r = philox4x32(u32x4{(uint32_t)i, salt, 7u, 0u}, (uint32_t)seed,
                                       (uint32_t)(seed >> 32));
            v[i] = u01_open0(r.x, r.y) - 0.5;
        }
    };
    auto norm_of = [&](const double* v) {
        double s = 0.0;
        for (int i = tid; i < n; i += kGraphThreads) s = fma(v[i], v[i], s);
        return sqrt(block_sum_fixed<kGraphThreads>(s, sh));
    };
    // full re-orthogonalisation of w (= V column j+1 slot) against V[0..cnt)
    auto reorth = [&](double* w, int cnt) {
        for (int pass = 0; pass < 2; ++pass) {
            for (int c = wave; c < cnt; c += NW) {
                const double* vc = V + (int64_t)c * n;
                double s = 0.0;
                for (int i = lane; i < n; i += 64) s = fma(vc[i], w[i], s);
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
                if (lane == 0) h[c] = s;
            }
            __syncthreads();
            for (int i = tid; i < n; i += kGraphThreads) {
                double acc = w[i];
                for (int c = 0; c < cnt; ++c) acc = fma(-h[c], V[(int64_t)c * n + i], acc);
                w[i] = acc;
            }
            __syncthreads();
        }
    };
    double anorm = 0.0;
    {   // Frobenius norm scale for the breakdown test
        double s = 0.0;
        for (int64_t t = tid; t < (int64_t)n * n; t += kGraphThreads) s = fma(S[t], S[t], s);
        anorm = sqrt(block_sum_fixed<kGraphThreads>(s, sh));
    }
    fill_random(V, 0u);
    __syncthreads();
    {
        const double nv = norm_of(V);
        for (int i = tid; i < n; i += kGraphThreads) V[i] /= nv;
        __syncthreads();
    }
    for (int j = 0; j < n; ++j) {
        const double* vj = V + (int64_t)j * n;
        double* w = V + (int64_t)(j + 1) * n;
        // w = S v_j (one wave per row)
        for (int r = wave; r < n; r += NW) {
            const double* srow = S + (int64_t)r * n;
            double s = 0.0;
            for (int i = lane; i < n; i += 64) s = fma(srow[i], vj[i], s);
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
            if (lane == 0) w[r] = s;
        }
        __syncthreads();
        double a = 0.0;
        for (int i = tid; i < n; i += kGraphThreads) a = fma(w[i], vj[i], a);
        a = block_sum_fixed<kGraphThreads>(a, sh);
        if (tid == 0) al[j] = a;
        for (int i = tid; i < n; i += kGraphThreads) {
            double v = w[i] - a * vj[i];
            if (j > 0) v -= be[j - 1] * V[(int64_t)(j - 1) * n + i];
            w[i] = v;
        }
        __syncthreads();
        reorth(w, j + 1);
        double bn = norm_of(w);
        if (j + 1 < n && bn <= 1e-13 * anorm) {
            // invariant subspace: continue from a fresh direction (beta = 0)
            fill_random(w, (uint32_t)(j + 1));
            __syncthreads();
            reorth(w, j + 1);
            const double nv = norm_of(w);
            for (int i = tid; i < n; i += kGraphThreads) w[i] /= nv;
            bn = 0.0;
        } else if (j + 1 < n) {
            for (int i = tid; i < n; i += kGraphThreads) w[i] /= bn;
        }
        if (tid == 0) be[j] = bn;
        __syncthreads();
    }
    if (tid == 0) {
        // Gershgorin bounds
        double lo = al[0], hi = al[0];
        for (int i = 0; i < n; ++i) {
            const double r = (i > 0 ? fabs(be[i - 1]) : 0.0) + (i + 1 < n ? fabs(be[i]) : 0.0);
            lo = fmin(lo, al[i] - r);
            hi = fmax(hi, al[i] + r);
        }
        lo -= 1e-12 * fabs(lo) + 1e-300;
        hi += 1e-12 * fabs(hi) + 1e-300;
        const double lmin = kth_eig(al, be, n, 0, lo, hi);
        const double lmax = kth_eig(al, be, n, n - 1, lo, hi);
        const int neg = sturm_count(al, be, n, 0.0);
        double amin;
        if (neg == 0) amin = fabs(lmin);
        else if (neg == n) amin = fabs(lmax);
        else amin = fmin(fabs(kth_eig(al, be, n, neg - 1, lo, hi)), fabs(kth_eig(al, be, n, neg, lo, hi)));
        out[0] = fmax(fabs(lmin), fabs(lmax));
        out[1] = amin;
    }
}

// ------------------------------------------------------------------ PCG
// Two launches per CG iteration.  The scalar recurrences (alpha, beta, the
// convergence test) are folded redundantly by every workgroup from the
// previous launch's per-workgroup partials, in one fixed order, so all
// workgroups take identical decisions without a one-workgroup scalar launch
// between the vector passes.  A workgroup covers 64 whole poses (192 scalar
// rows), so the block-Jacobi preconditioner stays workgroup-local.
constexpr int kPcgThreads = 192;

struct PcgState {
    double rho[2];                  // rho_k = r_k . z_k in slot k & 1
    double rr0, rr;
    int32_t iter, done, status, pad;
};

// partial arrays: [0, nb) p.q ; [nb, 2nb) r.z ; [2nb, 3nb) r.r.  The strided
// sequential sum of each lane is read four loads at a time (missing terms
// add +0.0), the same order as the plain loop.
template <int NT>
__device__ __forceinline__ double pcg_fold_lane(const double* __restrict__ part, const int64_t nb) {
    double a = 0.0;
    for (int64_t k = threadIdx.x; k < nb; k += 4 * NT) {
        const double v0 = part[k];
        const double v1 = (k + NT < nb) ? part[k + NT] : 0.0;
        const double v2 = (k + 2 * NT < nb) ? part[k + 2 * NT] : 0.0;
        const double v3 = (k + 3 * NT < nb) ? part[k + 3 * NT] : 0.0;
        a += v0;
        a += v1;
        a += v2;
        a += v3;
    }
    return a;
}

__device__ __forceinline__ double pcg_fold(const double* __restrict__ part, const int64_t nb,
                                           double* sh) {
    return block_sum_fixed<kPcgThreads>(pcg_fold_lane<kPcgThreads>(part, nb), sh);
}

__device__ __forceinline__ bool pcg_lead() { return blockIdx.x == 0 && threadIdx.x == 0; }

// x = 0, r = -b, z = M^-1 r ; partials r.z, r.r
__global__ __launch_bounds__(kPcgThreads) void graph_pcg_start_kernel(
    const int64_t n, const double* __restrict__ minv, const double* __restrict__ b,
    double* __restrict__ x, double* __restrict__ r, double* __restrict__ z,
    double* __restrict__ part) {
    __shared__ double sh[2 * kPcgThreads / 64];
    __shared__ double rs[kPcgThreads];
    const int64_t nb = gridDim.x;
    const int64_t i = (int64_t)blockIdx.x * kPcgThreads + threadIdx.x;
    double ri = 0.0;
    if (i < n) {
        ri = -b[i];
        r[i] = ri;
        x[i] = 0.0;
    }
    rs[threadIdx.x] = ri;
    __syncthreads();
    double rz = 0.0, rr = 0.0;
    if (i < n) {
        const int a = (int)(i % 3);
        const double* m = minv + (i - a) * 3 + 3 * a;
        const double* rb = rs + threadIdx.x - a;
        double zi = m[0] * rb[0];
        zi = fma(m[1], rb[1], zi);
        zi = fma(m[2], rb[2], zi);
        z[i] = zi;
        rz = zi * ri;
        rr = ri * ri;
    }
    block_sum2_fixed<kPcgThreads>(rz, rr, sh);
    if (threadIdx.x == 0) {
        part[nb + blockIdx.x] = rz;
        part[2 * nb + blockIdx.x] = rr;
    }
}

// iteration k, first launch: rho_k and the convergence test from the r.z / r.r
// partials, then the direction and its image by the recurrences
//   p_k = z + beta p_{k-1},   q_k = H p_k = H z + beta q_{k-1}
// so the SpMV gathers z alone (p and q are updated in place on the own rows);
// partial p.q.  SpMV: a group of 8 lanes per block row, each lane one whole
// 3x3 block at a time (72 contiguous bytes, adjacent lanes adjacent blocks),
// the three row sums folded over the group by a fixed xor tree.
constexpr int kSpmvThreads = 512, kSpmvGroup = 8;    // 64 poses per workgroup
static_assert(kSpmvThreads / kSpmvGroup * 3 == kPcgThreads, "same workgroup count");

__device__ __forceinline__ void pcg_block_dot(const int64_t s, const int64_t* __restrict__ col,
                                              const double* __restrict__ val,
                                              const double* __restrict__ z, double& a0,
                                              double& a1, double& a2) {
    const double* v = val + s * 9;
    double b[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) b[j] = v[j];
    const int64_t c = 3 * col[s];
    const double z0 = z[c], z1 = z[c + 1], z2 = z[c + 2];
    a0 = fma(b[0], z0, a0);
    a0 = fma(b[1], z1, a0);
    a0 = fma(b[2], z2, a0);
    a1 = fma(b[3], z0, a1);
    a1 = fma(b[4], z1, a1);
    a1 = fma(b[5], z2, a1);
    a2 = fma(b[6], z0, a2);
    a2 = fma(b[7], z1, a2);
    a2 = fma(b[8], z2, a2);
}

__global__ __launch_bounds__(kSpmvThreads) void graph_pcg_dir_spmv_kernel(
    const int64_t nt, const int32_t k, const int64_t* __restrict__ rptr,
    const int64_t* __restrict__ col, const double* __restrict__ val,
    const double* __restrict__ z, double* __restrict__ p, double* __restrict__ q,
    double* __restrict__ part, PcgState* __restrict__ st, const double tol,
    const int32_t max_iter) {
    __shared__ double sh[2 * kSpmvThreads / 64];
    if (k > 0 && st->done) return;
    const int64_t nb = gridDim.x;
    double rz = pcg_fold_lane<kSpmvThreads>(part + nb, nb);
    double rr = pcg_fold_lane<kSpmvThreads>(part + 2 * nb, nb);
    block_sum2_fixed<kSpmvThreads>(rz, rr, sh);
    double beta = 0.0;
    int status = 0;
    if (k == 0) {
        if (rr == 0.0) status = 1;
    } else {
        if (rr <= tol * tol * st->rr0) status = 1;
        else if (k >= max_iter) status = 3;
        beta = rz / st->rho[(k - 1) & 1];
    }
    if (pcg_lead()) {
        st->rho[k & 1] = rz;
        st->rr = rr;
        st->iter = k;
        if (k == 0) st->rr0 = rr;
        st->status = status;
        st->done = status != 0;
    }
    if (status) return;
    const int g = threadIdx.x & (kSpmvGroup - 1);
    const int64_t rw = (int64_t)blockIdx.x * (kSpmvThreads / kSpmvGroup) + threadIdx.x / kSpmvGroup;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    if (rw < nt) {
        const int64_t s1 = rptr[rw + 1];
        for (int64_t s = rptr[rw] + g; s < s1; s += kSpmvGroup) pcg_block_dot(s, col, val, z, a0, a1, a2);
    }
#pragma unroll
    for (int d = 1; d < kSpmvGroup; d <<= 1) {
        a0 += __shfl_xor(a0, d, 64);
        a1 += __shfl_xor(a1, d, 64);
        a2 += __shfl_xor(a2, d, 64);
    }
    double pq = 0.0;
    if (rw < nt && g < 3) {
        const double hz = (g == 0) ? a0 : (g == 1) ? a1 : a2;
        const int64_t i = 3 * rw + g;
        const double pi = (k > 0) ? fma(beta, p[i], z[i]) : z[i];
        const double qi = (k > 0) ? fma(beta, q[i], hz) : hz;
        p[i] = pi;
        q[i] = qi;
        pq = qi * pi;
    }
    pq = block_sum_fixed<kSpmvThreads>(pq, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = pq;
}

// iteration k, second launch: alpha = rho_k / p.q (curvature gate), x += alpha p,
// r -= alpha q, z = M^-1 r ; partials r.z, r.r
__global__ __launch_bounds__(kPcgThreads) void graph_pcg_step_kernel(
    const int64_t n, const int32_t k, const double* __restrict__ minv,
    const double* __restrict__ p, const double* __restrict__ q, double* __restrict__ x,
    double* __restrict__ r, double* __restrict__ z, double* __restrict__ part,
    PcgState* __restrict__ st) {
    __shared__ double sh[2 * kPcgThreads / 64];
    __shared__ double rs[kPcgThreads];
    // own operands first: their loads run under the p.q fold
    const int64_t i = (int64_t)blockIdx.x * kPcgThreads + threadIdx.x;
    double xi = 0.0, ri = 0.0, pi = 0.0, qi = 0.0, m0 = 0.0, m1 = 0.0, m2 = 0.0;
    if (i < n) {
        xi = x[i];
        ri = r[i];
        pi = p[i];
        qi = q[i];
        const int a = (int)(i % 3);
        const double* m = minv + (i - a) * 3 + 3 * a;
        m0 = m[0];
        m1 = m[1];
        m2 = m[2];
    }
    if (st->done) return;
    const int64_t nb = gridDim.x;
    const double pq = pcg_fold(part, nb, sh);
    if (!(pq > 0.0)) {                  // not positive definite along p
        if (pcg_lead()) {
            st->done = 1;
            st->status = 2;
        }
        return;
    }
    const double alpha = st->rho[k & 1] / pq;
    if (i < n) {
        x[i] = fma(alpha, pi, xi);
        ri = fma(-alpha, qi, ri);
        r[i] = ri;
    }
    rs[threadIdx.x] = ri;
    __syncthreads();
    double rz = 0.0, rr = 0.0;
    if (i < n) {
        const double* rb = rs + threadIdx.x - (int)(i % 3);
        double zi = m0 * rb[0];
        zi = fma(m1, rb[1], zi);
        zi = fma(m2, rb[2], zi);
        z[i] = zi;
        rz = zi * ri;
        rr = ri * ri;
    }
    block_sum2_fixed<kPcgThreads>(rz, rr, sh);
    if (threadIdx.x == 0) {
        part[nb + blockIdx.x] = rz;
        part[2 * nb + blockIdx.x] = rr;
    }
}

// ------------------------------------------- condition number (PCG path)
// updateEstPose's gate (:494-498) needs cond(H) = lambda_max / lambda_min (H
// is symmetric positive definite up to rounding, so the 2-norm condition
// number numpy forms by SVD is the ratio of its extreme eigenvalues).  At
// config-5 size the dense route is out of reach (a 180 GB H); the extreme
// eigenvalues come from LOBPCG (block size 1) on the block-sparse H, run on
// a second stream beside the PCG solve:
//   side 0: lambda_min, preconditioned by the PCG's block-Jacobi inverses
//           (the preconditioner is what makes the smallest eigenvalue
//           converge in ~100-200 iterations; plain Lanczos needs thousands);
//   side 1: lambda_max, unpreconditioned.
// Per iteration, for each side still running: w = T (Hx - theta x) (T = the
// preconditioner or I); w' = w - (x.w) x, Hw' = H w - (x.w) Hx; Rayleigh-Ritz
// on span{x, w', p} from its 3x3 Gram and projected matrices (scaled to a
// unit diagonal, Cholesky, p dropped when it is nearly dependent, cyclic
// Jacobi); x <- the Ritz vector, p <- its (w', p) part.  Three launches:
// update (+ residual, preconditioner, x.w partials), SpMV of both sides'
// w (one read of every 3x3 block) + orthogonalisation + the 24 Gram
// partials, one-workgroup fold of the partials in a fixed order.  Every
// workgroup solves the small problems redundantly from the same folded
// totals, so the decisions are identical everywhere.  A side stops when
// theta moved less than tol * theta over kCondWin iterations; the estimate
// stops early when theta_max / theta_min >= cond_max already (Ritz values lie
// inside [lambda_min, lambda_max], so the true cond is at least that: the gate
// rejects for certain) or theta_min <= 0 (not positive definite).
constexpr int kCondHist = 64;
constexpr int kCondWin = 16;
constexpr int kCondGram = 12;   // per side: G00 G01 G02 G11 G12 G22, A00 A01 A02 A11 A12 A22

struct CondState {
    double theta[2][kCondHist];   // Ritz value of each side per iteration (ring)
    double tot[2 * kCondGram];    // the fold launch's totals
    double lam[2];                // the latest Ritz values (min side, max side)
    double coef[2][4];            // this iteration's update of each side: c0, c1, c2, 1 / |p'|
    int32_t iter, done, status, iters_side[2], conv[2], upd[2], win;   // win: the stall window
    // the gate's early decision (SLAM_GRAPH_COND_MARGIN; etol 0: off): both
    // sides moved less than etol (relative) over ewin iterations and
    // theta_max / theta_min * emargin < cond_max -> status 5
    double etol, emargin;
    int32_t ewin, econv[2];
    // merged mode: the SpMV launch's arrival tickets -- one 128-byte line per
    // residue class blockIdx % 8 (one XCD under round-robin dispatch), the
    // classes' last arrivers on line 0; each word re-zeroed by its last arriver
    alignas(128) uint32_t tk[9 * 32];
};

// last-arriver election over write-through partials (the particle filter's
// arrive_last_n): the storing waves drain, one lane takes an agent-scope
// ticket; no fence (an agent-scope fence writes back the XCD's L2)
__device__ __forceinline__ bool cond_arrive_n(uint32_t* counter, const uint32_t expected) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t == expected - 1) ? 1 : 0;
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last != 0;
}
__device__ __forceinline__ bool cond_arrive_last(uint32_t* tk) {
    const int G = gridDim.x < 8 ? (int)gridDim.x : 8, g = blockIdx.x % G;
    const uint32_t ng = (gridDim.x - g + G - 1) / G;
    if (!cond_arrive_n(tk + (1 + g) * 32, ng)) return false;
    return cond_arrive_n(tk, (uint32_t)G);
}

__device__ __forceinline__ uint64_t cond_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

template <int NT, int K>
__device__ __forceinline__ void block_sumK_fixed(double* v, double* sh) {
    // K sums through one LDS round; sh holds K * NT / 64 doubles
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v[j] += __shfl_xor(v[j], d, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int j = 0; j < K; ++j) sh[j * (NT / 64) + (threadIdx.x >> 6)] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double r = 0.0;
        for (int w = 0; w < NT / 64; ++w) r += sh[j * (NT / 64) + w];
        v[j] = r;
    }
    __syncthreads();
}

// One Jacobi rotation of the symmetric 3x3 C in the (P, Q) plane, eigenvectors
// accumulated in V; compile-time indices only (the arrays stay in registers).
template <int P, int Q>
__device__ __forceinline__ void jacobi_rot3(double (&C)[3][3], double (&V)[3][3]) {
    if (!(fabs(C[P][Q]) > 1e-19 * (fabs(C[P][P]) + fabs(C[Q][Q])))) return;   // settled (or NaN)
    const double tau = (C[Q][Q] - C[P][P]) / (2.0 * C[P][Q]);
    const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
    const double cs = 1.0 / sqrt(1.0 + t * t), sn = t * cs;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double ckp = C[k][P], ckq = C[k][Q];
        C[k][P] = cs * ckp - sn * ckq;
        C[k][Q] = sn * ckp + cs * ckq;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double cpk = C[P][k], cqk = C[Q][k];
        C[P][k] = cs * cpk - sn * cqk;
        C[Q][k] = sn * cpk + cs * cqk;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double vkp = V[k][P], vkq = V[k][Q];
        V[k][P] = cs * vkp - sn * vkq;
        V[k][Q] = sn * vkp + cs * vkq;
    }
}

// Rayleigh-Ritz on span{x, w, p} (p absent when g22 == 0): g / a the six
// distinct entries of the Gram and projected matrices.  Returns false when w
// adds no direction (the side has converged to rounding).  c: coefficients of
// the Ritz vector in (x, w, p), normalised so that |c0 x + c1 w + c2 p| = 1;
// pn: |c1 w + c2 p|.  The basis is scaled to a unit diagonal and its Gram
// factored by Cholesky; p is dropped when it is nearly dependent on x, w.
// Written with compile-time indices only (no scratch).
__device__ __forceinline__ bool cond_small(const double* g, const double* a, const bool want_max,
                                           double* c, double* theta, double* pn) {
    if (!(g[0] > 0.0) || !(g[3] > 0.0)) return false;
    const double s0 = 1.0 / sqrt(g[0]), s1 = 1.0 / sqrt(g[3]);
    const double g10 = g[1] * s1 * s0;
    const double l11q = 1.0 - g10 * g10;
    if (!(l11q > 1e-10)) return false;
    const double l11 = sqrt(l11q);
    // the p direction, when present and independent enough
    bool three = g[5] > 0.0;
    double s2 = 0.0, l20 = 0.0, l21 = 0.0, l22 = 1.0;
    if (three) {
        s2 = 1.0 / sqrt(g[5]);
        l20 = g[2] * s2 * s0;
        l21 = (g[4] * s2 * s1 - l20 * g10) / l11;
        const double l22q = 1.0 - l20 * l20 - l21 * l21;
        three = l22q > 1e-10;
        if (three) l22 = sqrt(l22q);
    }
    // Li = L^-1 (lower triangular; the third row / column is the identity's
    // when p is dropped, which decouples it)
    const double i11 = 1.0 / l11, i10 = -g10 * i11;
    double i22 = 1.0, i21 = 0.0, i20 = 0.0;
    if (three) {
        i22 = 1.0 / l22;
        i21 = -l21 * i11 * i22;
        i20 = -(l20 + l21 * i10) * i22;
    }
    const double Li[3][3] = {{1.0, 0.0, 0.0}, {i10, i11, 0.0}, {i20, i21, i22}};
    // As = s A s; a dropped p gets a diagonal entry no Ritz value of (x, w)
    // can lose to (so it is never selected)
    const double sc[3] = {s0, s1, three ? s2 : 0.0};
    double As[3][3] = {{a[0], a[1], a[2]}, {a[1], a[3], a[4]}, {a[2], a[4], a[5]}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) As[i][j] *= sc[i] * sc[j];
    if (!three) {
        As[0][2] = As[2][0] = As[1][2] = As[2][1] = 0.0;
        As[2][2] = want_max ? -__builtin_huge_val() : __builtin_huge_val();
    }
    // C = Li As Li^T
    double T[3][3], C[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k <= i; ++k) acc = fma(Li[i][k], As[k][j], acc);
            T[i][j] = acc;
        }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k <= j; ++k) acc = fma(T[i][k], Li[j][k], acc);
            C[i][j] = acc;
        }
    if (!three) {                      // keep the dummy entry exactly decoupled
        C[0][2] = C[2][0] = C[1][2] = C[2][1] = 0.0;
        C[2][2] = As[2][2];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) C[i][j] = C[j][i] = 0.5 * (C[i][j] + C[j][i]);
    double V[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    auto settled = [&](int p, int q) {
        return !(fabs(C[p][q]) > 1e-19 * (fabs(C[p][p]) + fabs(C[q][q])));
    };
    for (int sweep = 0; sweep < 12; ++sweep) {
        if (settled(0, 1) && settled(0, 2) && settled(1, 2)) break;
        jacobi_rot3<0, 1>(C, V);
        if (three) {
            jacobi_rot3<0, 2>(C, V);
            jacobi_rot3<1, 2>(C, V);
        }
    }
    // the wanted end (the dummy never wins)
    int e = 0;
    double best = C[0][0];
    if (want_max ? (C[1][1] > best) : (C[1][1] < best)) { e = 1; best = C[1][1]; }
    if (three && (want_max ? (C[2][2] > best) : (C[2][2] < best))) { e = 2; best = C[2][2]; }
    *theta = best;
    const double y0 = e == 0 ? V[0][0] : (e == 1 ? V[0][1] : V[0][2]);
    const double y1 = e == 0 ? V[1][0] : (e == 1 ? V[1][1] : V[1][2]);
    const double y2 = three ? (e == 0 ? V[2][0] : (e == 1 ? V[2][1] : V[2][2])) : 0.0;
    // c = s (Li^T y)
    c[0] = (Li[0][0] * y0 + Li[1][0] * y1 + Li[2][0] * y2) * s0;
    c[1] = (Li[1][1] * y1 + Li[2][1] * y2) * s1;
    c[2] = three ? (Li[2][2] * y2) * s2 : 0.0;
    const double pp = c[1] * c[1] * g[3] + 2.0 * c[1] * c[2] * g[4] + c[2] * c[2] * g[5];
    *pn = sqrt(fmax(pp, 0.0));
    return true;
}

// random start (cold) or the previous update's vectors (warm); p = Hp = 0
__global__ __launch_bounds__(256) void graph_cond_init_kernel(const int64_t n, const int cold,
                                                              const int win,
                                                              double* __restrict__ x,
                                                              double* __restrict__ p,
                                                              double* __restrict__ hp,
                                                              CondState* __restrict__ st,
                                                              const double etol = 0.0,
                                                              const int ewin = 0,
                                                              const double emargin = 0.0) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        st->iter = 0;
        st->done = 0;
        st->status = 0;
        st->conv[0] = st->conv[1] = 0;
        st->econv[0] = st->econv[1] = 0;
        st->iters_side[0] = st->iters_side[1] = 0;
        st->win = win;
        st->etol = etol;
        st->ewin = ewin;
        st->emargin = emargin;
    }
    for (int64_t t = i; t < 9 * 32; t += (int64_t)gridDim.x * 256) st->tk[t] = 0;
    if (i >= 2 * n) return;
    if (cold) x[i] = (double)(int64_t)(cond_mix64((uint64_t)i) >> 11) * 0x1.0p-52 - 1.0;
    p[i] = 0.0;
    hp[i] = 0.0;
}

__device__ __forceinline__ void cond_block_dot2(const int64_t s, const int64_t* __restrict__ col,
                                                const double* __restrict__ val,
                                                const double* __restrict__ v0,
                                                const double* __restrict__ v1, double* a) {
    const double* m = val + s * 9;
    double b[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) b[j] = m[j];
    const int64_t c = 3 * col[s];
    const double x0 = v0[c], x1 = v0[c + 1], x2 = v0[c + 2];
    const double y0 = v1[c], y1 = v1[c + 1], y2 = v1[c + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        a[r] = fma(b[3 * r], x0, a[r]);
        a[r] = fma(b[3 * r + 1], x1, a[r]);
        a[r] = fma(b[3 * r + 2], x2, a[r]);
        a[3 + r] = fma(b[3 * r], y0, a[3 + r]);
        a[3 + r] = fma(b[3 * r + 1], y1, a[3 + r]);
        a[3 + r] = fma(b[3 * r + 2], y2, a[3 + r]);
    }
}

// START = true: Hx of both sides' x, partials x.x and x.Hx (part rows 0, 6
// of each side's 12).  START = false: alpha = x.w (folded from the update
// launch's partials), Hw, w' = w - alpha x, Hw' = Hw - alpha Hx and the 24 Gram
// partials.  part: [24][nb] Gram, then [2][nb] x.w.  The 24 products of each
// of the workgroup's 192 rows go through LDS and are summed in a fixed order
// (three per wave: lanes take three rows each, then the xor butterfly).
template <int NT, bool WT>
__device__ __forceinline__ void cond_fold_body(const int64_t nb, const double* __restrict__ part,
                                               CondState* __restrict__ st, const int32_t k,
                                               const double tol, const int32_t max_iter,
                                               const double cond_max);

// FOLD (merged mode): the workgroup arriving last at the state's ticket also
// folds the launch's partials and decides iteration k (cond_fold_body), so an
// iteration is two launches instead of three.
constexpr int kCondRows = kSpmvThreads / kSpmvGroup * 3;   // 192 rows per workgroup
template <bool START, bool FOLD = false>
__global__ __launch_bounds__(kSpmvThreads) void graph_cond_spmv_kernel(
    const int64_t nt, const int64_t* __restrict__ rptr, const int64_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ x, double* __restrict__ hx,
    const double* __restrict__ w, double* __restrict__ w2, double* __restrict__ hw,
    const double* __restrict__ p, const double* __restrict__ hp, double* __restrict__ part,
    CondState* __restrict__ st, const int32_t k = 0, const double tol = 0.0,
    const int32_t max_iter = 0, const double cond_max = 0.0) {
    __shared__ double s_prod[2 * kCondGram][kCondRows];
    __shared__ double sh[2 * kSpmvThreads / 64];
    if (!START && st->done) return;
    const int64_t n = 3 * nt;
    const int64_t nb = gridDim.x;
    double alpha0 = 0.0, alpha1 = 0.0;
    bool run0 = true, run1 = true;
    if (!START) {
        double al0 = pcg_fold_lane<kSpmvThreads>(part + 2 * kCondGram * nb, nb);
        double al1 = pcg_fold_lane<kSpmvThreads>(part + (2 * kCondGram + 1) * nb, nb);
        block_sum2_fixed<kSpmvThreads>(al0, al1, sh);
        alpha0 = al0;
        alpha1 = al1;
        run0 = !st->conv[0];
        run1 = !st->conv[1];
    }
    const double* src = START ? x : w;
    const int g = threadIdx.x & (kSpmvGroup - 1);
    const int64_t rw = (int64_t)blockIdx.x * (kSpmvThreads / kSpmvGroup) + threadIdx.x / kSpmvGroup;
    double a[6] = {0, 0, 0, 0, 0, 0};
    if (rw < nt) {
        const int64_t s1 = rptr[rw + 1];
        for (int64_t s = rptr[rw] + g; s < s1; s += kSpmvGroup) cond_block_dot2(s, col, val, src, src + n, a);
    }
#pragma unroll
    for (int d = 1; d < kSpmvGroup; d <<= 1)
#pragma unroll
        for (int j = 0; j < 6; ++j) a[j] += __shfl_xor(a[j], d, 64);
    if (g < 3) {
        const int lr = (int)(threadIdx.x / kSpmvGroup) * 3 + g;      // row within the workgroup
        const int64_t i = 3 * rw + g;
        const bool ok = rw < nt;
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
            const double hv = (g == 0) ? a[3 * sd] : (g == 1) ? a[3 * sd + 1] : a[3 * sd + 2];
            const int64_t k = sd * n + i;
            const bool run = sd == 0 ? run0 : run1;
            const double al = sd == 0 ? alpha0 : alpha1;
            double o[kCondGram];
#pragma unroll
            for (int j = 0; j < kCondGram; ++j) o[j] = 0.0;
            if (START) {
                if (ok) {
                    hx[k] = hv;
                    const double xi = x[k];
                    o[0] = xi * xi;
                    o[6] = xi * hv;
                }
            } else if (ok && run) {
                const double xi = x[k], hxi = hx[k], pi = p[k], hpi = hp[k];
                const double wi = fma(-al, xi, w[k]);
                const double hwi = fma(-al, hxi, hv);
                w2[k] = wi;
                hw[k] = hwi;
                o[0] = xi * xi;
                o[1] = xi * wi;
                o[2] = xi * pi;
                o[3] = wi * wi;
                o[4] = wi * pi;
                o[5] = pi * pi;
                o[6] = xi * hxi;
                o[7] = 0.5 * (xi * hwi + wi * hxi);
                o[8] = 0.5 * (xi * hpi + pi * hxi);
                o[9] = wi * hwi;
                o[10] = 0.5 * (wi * hpi + pi * hwi);
                o[11] = pi * hpi;
            }
#pragma unroll
            for (int j = 0; j < kCondGram; ++j) s_prod[sd * kCondGram + j][lr] = o[j];
        }
    }
    __syncthreads();
    // wave v sums quantities 3v .. 3v + 2 over the 192 rows: lane l takes rows
    // l, l + 64, l + 128 in order, then the butterfly
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int j = 3 * wv + q;
        double v = s_prod[j][lane];
        v += s_prod[j][lane + 64];
        v += s_prod[j][lane + 128];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        if (lane == 0) {
            if constexpr (FOLD)                  // write-through: read by the last arriver
                __hip_atomic_store((uint64_t*)(part + j * nb + blockIdx.x),
                                   (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                part[j * nb + blockIdx.x] = v;
        }
    }
    if constexpr (FOLD) {
        if (!cond_arrive_last(st->tk)) return;
        cond_fold_body<kSpmvThreads, true>(nb, part, st, k, tol, max_iter, cond_max);
    }
}
static_assert(kSpmvThreads / 64 * 3 == 2 * kCondGram, "three Gram quantities per wave");

// One workgroup per iteration: the 24 Gram partial rows folded in a fixed
// order (one wave per row, lanes strided, then the xor butterfly), then the
// two small problems (one lane each, on different waves), the stopping tests
// and this iteration's update coefficients into the state; the update launch
// only applies them.  k = 0: x normalised, theta its Rayleigh quotient.
// The fold itself, by a workgroup of NT threads: row j by wave j % (NT / 64),
// each lane summing its strided entries four at a time (missing terms add
// +0.0: the order of the plain loop), the rows of a wave loaded together,
// then the xor butterfly -- the same totals whichever workgroup size folds.
// WT: the partials were stored by other workgroups of the same launch (the
// merged mode's last arriving workgroup): read them with agent-scope loads.
template <int NT, bool WT>
__device__ __forceinline__ void cond_fold_body(const int64_t nb, const double* __restrict__ part,
                                               CondState* __restrict__ st, const int32_t k,
                                               const double tol, const int32_t max_iter,
                                               const double cond_max) {
    constexpr int NW = NT / 64, RPW = (2 * kCondGram + NW - 1) / NW;
    __shared__ double s_tot[2 * kCondGram];
    __shared__ int s_conv[2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    auto ld = [&](const double* a) {
        if constexpr (WT)
            return __longlong_as_double((long long)__hip_atomic_load(
                (const uint64_t*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        else
            return *a;
    };
    double v[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) v[r] = 0.0;
    for (int64_t q = lane; q < nb; q += 4 * 64) {
        double a[RPW][4];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int j = wave + r * NW;
            const double* pj = part + (j < 2 * kCondGram ? j : 0) * nb;
            const bool ok = j < 2 * kCondGram;
            a[r][0] = ok ? ld(pj + q) : 0.0;
            a[r][1] = (ok && q + 64 < nb) ? ld(pj + q + 64) : 0.0;
            a[r][2] = (ok && q + 128 < nb) ? ld(pj + q + 128) : 0.0;
            a[r][3] = (ok && q + 192 < nb) ? ld(pj + q + 192) : 0.0;
        }
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            v[r] += a[r][0];
            v[r] += a[r][1];
            v[r] += a[r][2];
            v[r] += a[r][3];
        }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int j = wave + r * NW;
        double t = v[r];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, 64);
        if (lane == 0 && j < 2 * kCondGram) s_tot[j] = t;
    }
    __syncthreads();
    if (lane == 0 && wave < 2) {
        const int sd = wave;
        const double* t = s_tot + sd * kCondGram;
        double th = st->lam[sd], c0 = 1.0, c1 = 0.0, c2 = 0.0, pinv = 0.0;
        int upd = 0, conv = st->conv[sd];
        if (k == 0) {
            c0 = 1.0 / sqrt(t[0]);
            th = t[6] / t[0];
            upd = 1;
            conv = 0;
        } else if (!conv) {
            const double g[6] = {t[0], t[1], t[2], t[3], t[4], t[5]};
            const double a[6] = {t[6], t[7], t[8], t[9], t[10], t[11]};
            double c[3], theta, pn;
            if (!cond_small(g, a, sd == 1, c, &theta, &pn)) {
                conv = 1;                        // w' adds nothing: converged to rounding
            } else {
                th = theta;
                c0 = c[0];
                c1 = c[1];
                c2 = c[2];
                pinv = (pn > 0.0) ? 1.0 / pn : 0.0;
                upd = 1;
                const int win = st->win;
                const double old = st->theta[sd][(k - win) & (kCondHist - 1)];
                if (k >= win && fabs(old - theta) <= tol * fabs(theta)) conv = 1;
                const int ew = st->ewin;
                st->econv[sd] = st->etol > 0.0 && k >= ew &&
                                fabs(st->theta[sd][(k - ew) & (kCondHist - 1)] - theta) <=
                                    st->etol * fabs(theta);
                st->iters_side[sd] = k;
            }
        }
        st->theta[sd][k & (kCondHist - 1)] = th;
        st->lam[sd] = th;
        st->coef[sd][0] = c0;
        st->coef[sd][1] = c1;
        st->coef[sd][2] = c2;
        st->coef[sd][3] = pinv;
        st->upd[sd] = upd;
        st->conv[sd] = conv;
        s_conv[sd] = conv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t0 = st->lam[0], t1 = st->lam[1];
        int status = 0;
        if (!(t0 > 0.0)) status = 4;                                   // not positive definite
        else if (t1 >= cond_max * t0) status = 2;                      // cond >= cond_max for certain
        else if (s_conv[0] && s_conv[1]) status = 1;
        else if (st->etol > 0.0 && (s_conv[0] || st->econv[0]) && (s_conv[1] || st->econv[1]) &&
                 t1 * st->emargin < cond_max * t0)
            status = 5;                                                // decided with a margin
        else if (k >= max_iter) status = 3;
        st->iter = k;
        st->status = status;
        st->done = status != 0;
    }
}

constexpr int kCondFoldThreads = 1024;
__global__ __launch_bounds__(kCondFoldThreads) void graph_cond_fold_kernel(
    const int64_t nb, const double* __restrict__ part, CondState* __restrict__ st, const int32_t k,
    const double tol, const int32_t max_iter, const double cond_max) {
    if (st->done) return;
    cond_fold_body<kCondFoldThreads, false>(nb, part, st, k, tol, max_iter, cond_max);
}

// Applies the fold launch's coefficients to the own rows (x, Hx, p, Hp of each
// side it updated); unless the estimate is done, r = Hx - theta x, w = T r
// (side 0: the block-Jacobi inverse of the pose, the three rows of a pose in
// one workgroup; side 1: w = r) and the x.w partials.
__global__ __launch_bounds__(kPcgThreads) void graph_cond_update_kernel(
    const int64_t n, const int32_t k, const double* __restrict__ minv, double* __restrict__ x,
    double* __restrict__ hx, const double* __restrict__ w2, const double* __restrict__ hw,
    double* __restrict__ p, double* __restrict__ hp, double* __restrict__ w,
    double* __restrict__ part, const CondState* __restrict__ st) {
    __shared__ double sh[2 * kPcgThreads / 64];
    __shared__ double rs[kPcgThreads];
    const int32_t iter = st->iter;
    if (iter != k) return;                   // the fold launch stopped before this iteration
    const int64_t nb = gridDim.x;
    const int64_t i = (int64_t)blockIdx.x * kPcgThreads + threadIdx.x;
    const bool done = st->done;
    double xw0 = 0.0, xw1 = 0.0;
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
        const bool upd = st->upd[sd];
        const double c0 = st->coef[sd][0], c1 = st->coef[sd][1], c2 = st->coef[sd][2];
        const double pinv = st->coef[sd][3], th = st->lam[sd];
        const int64_t kk = sd * n + i;
        double xo = 0.0, hxo = 0.0;
        if (i < n && upd) {
            const double xi = x[kk], hxi = hx[kk];
            if (k == 0) {
                xo = xi * c0;
                hxo = hxi * c0;
            } else {
                const double wi = w2[kk], hwi = hw[kk], pi = p[kk], hpi = hp[kk];
                xo = fma(c2, pi, fma(c1, wi, c0 * xi));
                hxo = fma(c2, hpi, fma(c1, hwi, c0 * hxi));
                p[kk] = fma(c2, pi, c1 * wi) * pinv;
                hp[kk] = fma(c2, hpi, c1 * hwi) * pinv;
            }
            x[kk] = xo;
            hx[kk] = hxo;
        }
        if (done) continue;
        const bool act = upd && !st->conv[sd];
        const double ri = (i < n && act) ? fma(-th, xo, hxo) : 0.0;
        double wi = ri;
        if (sd == 0) {
            rs[threadIdx.x] = ri;
            __syncthreads();
            if (i < n) {
                const int a3 = (int)(i % 3);
                const double* m = minv + (i - a3) * 3 + 3 * a3;
                const double* rb = rs + threadIdx.x - a3;
                wi = m[0] * rb[0];
                wi = fma(m[1], rb[1], wi);
                wi = fma(m[2], rb[2], wi);
            }
        }
        if (i < n && act) {
            w[kk] = wi;
            if (sd == 0) xw0 = xo * wi;
            else xw1 = xo * wi;
        }
    }
    if (done) return;
    block_sum2_fixed<kPcgThreads>(xw0, xw1, sh);
    if (threadIdx.x == 0) {
        part[2 * kCondGram * nb + blockIdx.x] = xw0;
        part[(2 * kCondGram + 1) * nb + blockIdx.x] = xw1;
    }
}

// block-Jacobi preconditioner: inverses of the diagonal 3x3 blocks
__global__ __launch_bounds__(256) void graph_block_inv_kernel(const int64_t nb,
                                                              const int64_t* __restrict__ dslot,
                                                              const double* __restrict__ val,
                                                              double* __restrict__ minv) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    inv3_lu(val + dslot[b] * 9, minv + b * 9);
}

// ------------------------------------------------------- pose update
// updateEstPose :499-502 and the per-workgroup partials of Σδ² (:513), one lane per pose.
__global__ __launch_bounds__(256) void graph_pose_update_kernel(const int64_t nt,
                                                                const int64_t* __restrict__ times,
                                                                const double* __restrict__ delta,
                                                                double* __restrict__ poses,
                                                                double* __restrict__ part) {
    __shared__ double sh[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0.0;
    if (i < nt) {
        double* p = poses + 3 * times[i];
        const double d0 = delta[3 * i], d1 = delta[3 * i + 1], d2 = delta[3 * i + 2];
        p[0] = p[0] + d0;
        p[1] = p[1] + d1;
        p[2] = wrap_angle(p[2] + d2);
        s = fma(d0, d0, s);
        s = fma(d1, d1, s);
        s = fma(d2, d2, s);
    }
    s = block_sum_fixed<256>(s, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Σδ² from the pose-update partials, fixed order, one workgroup
__global__ __launch_bounds__(1024) void graph_dsum_kernel(const int64_t nparts,
                                                         const double* __restrict__ part,
                                                         double* __restrict__ dsum) {
    __shared__ double sh[16];
    double s = 0.0;
    for (int64_t k = threadIdx.x; k < nparts; k += 1024) s += part[k];
    s = block_sum_fixed<1024>(s, sh);
    if (threadIdx.x == 0) *dsum = s;
}

// ------------------------------------- the gate's certificate (PCG path)
// updateEstPose :494-496 solves only if 0.1 < det(H) and cond(H) < 1e15.  At
// config-5 size neither is formed; with M the block diagonal of H (the PCG's
// block-Jacobi preconditioner, M_i its 3x3 blocks) and P = M^-1/2 H M^-1/2
// (unit diagonal blocks, so tr P = n):
//   cond(H) <= cond(P) cond(M),   cond(M) <= max_i tr(M_i) * max_i tr(M_i^-1);
//   log det H = log det M + log det P,   log det P <= 0 (AM-GM with tr P = n),
//   log det P >= c(a) (tr(P^2) - n)  for any a <= lambda_min(P),
//                c(a) = (ln a - a + 1) / (a - 1)^2   (ln x >= (x - 1) + c(a)(x - 1)^2 on x >= a).
// These kernels form the four sums the bounds need -- sum_i log det M_i,
// tr(P^2) = sum over block slots (r, c) of tr(M_r^-1 H_rc M_c^-1 H_rc^T),
// max tr(M_i), max tr(M_i^-1) -- one lane per pose, one lane per block slot,
// per-workgroup partials folded by one workgroup in a fixed order.  With the
// LOBPCG estimate of lambda_min(H) (lambda_min(P) >= lambda_min(H) / max tr M_i)
// graph_api.hip turns them into the det decision.
struct CertState {
    double logdet_m, trp2, trm_max, trminv_max;
    int32_t bad, pad;              // diagonal blocks that are not positive definite
};
constexpr int kCertThreads = 256;

template <int NT>
__device__ __forceinline__ double block_max_fixed(double v, double* sh) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = fmax(v, __shfl_xor(v, d, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
    for (int w = 1; w < NT / 64; ++w) r = fmax(r, sh[w]);
    __syncthreads();
    return r;
}

// per pose i: log det of the symmetric part of M_i by its 3x3 Cholesky
// pivots (log d0 + log d1 + log d2), tr(M_i), tr(M_i^-1) (the block-Jacobi
// inverse).  part: [0, nb) log det, [nb, 2nb) bad, [2nb, 3nb) max tr M,
// [3nb, 4nb) max tr M^-1.
__global__ __launch_bounds__(kCertThreads) void graph_cert_pose_kernel(
    const int64_t nt, const int64_t* __restrict__ dslot, const double* __restrict__ val,
    const double* __restrict__ minv, double* __restrict__ part) {
    __shared__ double sh[2 * kCertThreads / 64];
    const int64_t nb = gridDim.x;
    const int64_t i = (int64_t)blockIdx.x * kCertThreads + threadIdx.x;
    double ld = 0.0, bad = 0.0, trm = 0.0, tri = 0.0;
    if (i < nt) {
        const double* a = val + dslot[i] * 9;
        const double s00 = a[0], s11 = a[4], s22 = a[8];
        const double s10 = 0.5 * (a[1] + a[3]), s20 = 0.5 * (a[2] + a[6]), s21 = 0.5 * (a[5] + a[7]);
        const double l10 = s10 / s00, l20 = s20 / s00;
        const double d1 = s11 - l10 * s10;
        const double l21 = (s21 - l20 * s10) / d1;
        const double d2 = (s22 - l20 * s20) - l21 * (s21 - l20 * s10);
        if (s00 > 0.0 && d1 > 0.0 && d2 > 0.0) ld = log(s00) + log(d1) + log(d2);
        else bad = 1.0;
        trm = s00 + s11 + s22;
        const double* m = minv + i * 9;
        tri = m[0] + m[4] + m[8];
    }
    block_sum2_fixed<kCertThreads>(ld, bad, sh);
    trm = block_max_fixed<kCertThreads>(trm, sh);
    tri = block_max_fixed<kCertThreads>(tri, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = ld;
        part[nb + blockIdx.x] = bad;
        part[2 * nb + blockIdx.x] = trm;
        part[3 * nb + blockIdx.x] = tri;
    }
}

// per block slot s = (r, c): tr(M_r^-1 H_rc M_c^-1 H_rc^T) = ||L_r^-1 H_rc L_c^-T||_F^2
// (the slot's share of tr(P^2)); part: one partial per workgroup
__global__ __launch_bounds__(kCertThreads) void graph_cert_slot_kernel(
    const int64_t n_slots, const int64_t* __restrict__ srow, const int64_t* __restrict__ scol,
    const double* __restrict__ val, const double* __restrict__ minv, double* __restrict__ part) {
    __shared__ double sh[kCertThreads / 64];
    const int64_t s = (int64_t)blockIdx.x * kCertThreads + threadIdx.x;
    double t = 0.0;
    if (s < n_slots) {
        const double* A = minv + srow[s] * 9;
        const double* B = val + s * 9;
        const double* C = minv + scol[s] * 9;
        double X[9], Y[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                X[3 * r + c] = fma(A[3 * r + 2], B[6 + c], fma(A[3 * r + 1], B[3 + c], A[3 * r] * B[c]));
                Y[3 * r + c] = fma(C[3 * r + 2], B[3 * c + 2], fma(C[3 * r + 1], B[3 * c + 1], C[3 * r] * B[3 * c]));
            }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) t = fma(X[3 * r + c], Y[3 * c + r], t);
    }
    t = block_sum_fixed<kCertThreads>(t, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// one workgroup: the partials of both kernels, fixed order -> CertState
__global__ __launch_bounds__(kCertThreads) void graph_cert_fold_kernel(
    const int64_t nb_pose, const double* __restrict__ ppart, const int64_t nb_slot,
    const double* __restrict__ spart, CertState* __restrict__ out) {
    __shared__ double sh[2 * kCertThreads / 64];
    double ld = 0.0, bad = 0.0, trm = 0.0, tri = 0.0, t2 = 0.0;
    for (int64_t k = threadIdx.x; k < nb_pose; k += kCertThreads) {
        ld += ppart[k];
        bad += ppart[nb_pose + k];
        trm = fmax(trm, ppart[2 * nb_pose + k]);
        tri = fmax(tri, ppart[3 * nb_pose + k]);
    }
    for (int64_t k = threadIdx.x; k < nb_slot; k += kCertThreads) t2 += spart[k];
    block_sum2_fixed<kCertThreads>(ld, bad, sh);
    t2 = block_sum_fixed<kCertThreads>(t2, sh);
    trm = block_max_fixed<kCertThreads>(trm, sh);
    tri = block_max_fixed<kCertThreads>(tri, sh);
    if (threadIdx.x == 0) {
        out->logdet_m = ld;
        out->trp2 = t2;
        out->trm_max = trm;
        out->trminv_max = tri;
        out->bad = (int32_t)bad;
    }
}

}  // namespace slam
