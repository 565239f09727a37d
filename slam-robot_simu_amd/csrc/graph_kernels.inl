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
    for (int64_t c = cptr[s]; c < cptr[s + 1]; ++c) {
        const int64_t code = clist[c];
        const int64_t e = code >> 2;
        const int part = (int)(code & 3);
        acc = acc + blocks[(int64_t)(part * 9 + q) * E + e];
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
    for (int64_t c = bptr[r]; c < bptr[r + 1]; ++c) {
        const int64_t code = blist[c];
        acc = acc + blocks[(int64_t)(36 + 3 * (code & 1) + a) * E + (code >> 1)];
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
// y = H x on the block-sparse matrix (one lane per scalar row).
__device__ __forceinline__ double bsr_row_dot(const int64_t r3, const int64_t* rptr,
                                              const int64_t* col, const double* val,
                                              const double* x) {
    const int64_t r = r3 / 3;
    const int a = (int)(r3 - 3 * r);
    double acc = 0.0;
    for (int64_t s = rptr[r]; s < rptr[r + 1]; ++s) {
        const double* v = val + s * 9 + 3 * a;
        const double* xc = x + 3 * col[s];
        acc = fma(v[0], xc[0], acc);
        acc = fma(v[1], xc[1], acc);
        acc = fma(v[2], xc[2], acc);
    }
    return acc;
}

// partial sums of 1024-element blocks (fixed order), finished by graph_pcg_scalar_kernel
template <int NT>
__device__ __forceinline__ void write_partial(double v, double* sh, double* part) {
    const double s = block_sum_fixed<NT>(v, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

struct PcgState {
    double rho, alpha, beta, rr0, rr;
    int32_t iter, done, status, pad;
};

// q = H p ; partial p.q
__global__ __launch_bounds__(256) void graph_pcg_spmv_kernel(
    const int64_t n, const int64_t* __restrict__ rptr, const int64_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ p, double* __restrict__ q,
    double* __restrict__ part, const PcgState* __restrict__ st) {
    __shared__ double sh[4];
    if (st->done) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double pq = 0.0;
    if (i < n) {
        const double v = bsr_row_dot(i, rptr, col, val, p);
        q[i] = v;
        pq = v * p[i];
    }
    write_partial<256>(pq, sh, part);
}

// z = M^-1 r (3x3 block inverses), partial r.z and r.r
__global__ __launch_bounds__(256) void graph_pcg_precond_kernel(
    const int64_t n, const double* __restrict__ minv, const double* __restrict__ r,
    double* __restrict__ z, double* __restrict__ part2, const PcgState* __restrict__ st,
    const int32_t first) {
    __shared__ double sh[4];
    if (!first && st->done) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double rz = 0.0, rr = 0.0;
    if (i < n) {
        const int64_t b = i / 3;
        const int a = (int)(i - 3 * b);
        const double* m = minv + b * 9 + 3 * a;
        const double* rb = r + 3 * b;
        double acc = m[0] * rb[0];
        acc = fma(m[1], rb[1], acc);
        acc = fma(m[2], rb[2], acc);
        z[i] = acc;
        rz = acc * r[i];
        rr = r[i] * r[i];
    }
    const double s1 = block_sum_fixed<256>(rz, sh);
    const double s2 = block_sum_fixed<256>(rr, sh);
    if (threadIdx.x == 0) {
        part2[2 * blockIdx.x] = s1;
        part2[2 * blockIdx.x + 1] = s2;
    }
}

// x += alpha p ; r -= alpha q
__global__ __launch_bounds__(256) void graph_pcg_axpy_kernel(const int64_t n,
                                                             double* __restrict__ x,
                                                             double* __restrict__ r,
                                                             const double* __restrict__ p,
                                                             const double* __restrict__ q,
                                                             const PcgState* __restrict__ st) {
    if (st->done) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double a = st->alpha;
    x[i] = fma(a, p[i], x[i]);
    r[i] = fma(-a, q[i], r[i]);
}

// p = z + beta p
__global__ __launch_bounds__(256) void graph_pcg_dir_kernel(const int64_t n,
                                                            double* __restrict__ p,
                                                            const double* __restrict__ z,
                                                            const PcgState* __restrict__ st,
                                                            const int32_t first) {
    if (!first && st->done) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    p[i] = first ? z[i] : fma(st->beta, p[i], z[i]);
}

// one workgroup: fold the partials in block order and update the scalars.
// mode 0: alpha = rho / p.q ; mode 1: rho' = r.z, beta, convergence ; mode 2: init.
__global__ __launch_bounds__(1024) void graph_pcg_scalar_kernel(const int64_t nparts,
                                                                const double* __restrict__ part,
                                                                PcgState* __restrict__ st,
                                                                const int32_t mode,
                                                                const double tol,
                                                                const int32_t max_iter) {
    __shared__ double sh[16];
    if (mode != 2 && st->done) return;
    const int stride = (mode == 0) ? 1 : 2;
    double a = 0.0, b = 0.0;
    for (int64_t k = threadIdx.x; k < nparts; k += blockDim.x) {
        a += part[stride * k];
        if (stride == 2) b += part[2 * k + 1];
    }
    a = block_sum_fixed<1024>(a, sh);
    b = block_sum_fixed<1024>(b, sh);
    if (threadIdx.x != 0) return;
    if (mode == 0) {
        if (!(a > 0.0)) {            // not positive definite along p
            st->done = 1;
            st->status = 2;
            return;
        }
        st->alpha = st->rho / a;
    } else if (mode == 1) {
        st->beta = a / st->rho;
        st->rho = a;
        st->rr = b;
        st->iter += 1;
        if (b <= tol * tol * st->rr0) {
            st->done = 1;
            st->status = 1;
        } else if (st->iter >= max_iter) {
            st->done = 1;
            st->status = 3;
        }
    } else {
        st->rho = a;
        st->rr0 = b;
        st->rr = b;
        st->iter = 0;
        st->status = 0;
        st->done = (b == 0.0) ? 1 : 0;
        if (b == 0.0) st->status = 1;
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
// updateEstPose :499-502 and Σδ² (:513, fixed-order), one workgroup.
__global__ __launch_bounds__(1024) void graph_pose_update_kernel(const int64_t nt,
                                                                 const int64_t* __restrict__ times,
                                                                 const double* __restrict__ delta,
                                                                 double* __restrict__ poses,
                                                                 double* __restrict__ dsum) {
    __shared__ double sh[16];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < nt; i += blockDim.x) {
        double* p = poses + 3 * times[i];
        const double d0 = delta[3 * i], d1 = delta[3 * i + 1], d2 = delta[3 * i + 2];
        p[0] = p[0] + d0;
        p[1] = p[1] + d1;
        p[2] = wrap_angle(p[2] + d2);
        s = fma(d0, d0, s);
        s = fma(d1, d1, s);
        s = fma(d2, d2, s);
    }
    s = block_sum_fixed<1024>(s, sh);
    if (threadIdx.x == 0) *dsum = s;
}

}  // namespace slam
