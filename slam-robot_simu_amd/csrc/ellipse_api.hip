// ellipse_api.hip -- ErrorEllipse.calc_error_ellipse (mylib/error_ellipse.py:39-55)
// over a batch of 2x2 covariances, one lane per matrix.
//
// np.linalg.eigh is LAPACK dsyevd (uplo L).  For n = 2 its steps reduce to:
// dsytrd leaves the matrix as it is (a length-1 reflector, tau = 0), dstedc
// hands the 2x2 tridiagonal (d = [a, c], e = [b]) to dsteqr, which zeroes e
// when |e| <= sqrt|a| sqrt|c| eps (or e^2 <= eps^2 |a| |c| + safmin, its
// iteration's test), otherwise takes the eigen-decomposition of
// the block from dlaev2 (rt1 of larger magnitude, eigenvector (cs1, sn1)) and
// applies the rotation to Z = I: Z = [[cs1, -sn1], [sn1, cs1]]; finally a
// selection sort puts the eigenvalues in increasing order (swap only on a
// strict decrease).  Those steps are restated here operation by operation
// (-ffp-contract=off), so eigenvalues and eigenvectors are LAPACK's doubles;
// the ellipse angle is the device atan2 (within an ulp of the C library's).
// Matrices whose norm needs dsyevd's / dsteqr's scaling (max |entry| outside
// ~[1e-122, 1e153]) are flagged (NaN outputs), not approximated.
#include <mutex>

#include "common.hpp"

namespace slam {

__device__ __forceinline__ void dlaev2_dev(const double a, const double b, const double c,
                                           double& rt1, double& rt2, double& cs1, double& sn1) {
    const double sm = a + c, df = a - c, adf = fabs(df), tb = b + b, ab = fabs(tb);
    double acmx, acmn;
    if (fabs(a) > fabs(c)) {
        acmx = a;
        acmn = c;
    } else {
        acmx = c;
        acmn = a;
    }
    double rt;
    if (adf > ab) {
        const double q = ab / adf;
        rt = adf * sqrt(1.0 + q * q);
    } else if (adf < ab) {
        const double q = adf / ab;
        rt = ab * sqrt(1.0 + q * q);
    } else {
        rt = ab * sqrt(2.0);
    }
    int sgn1;
    if (sm < 0.0) {
        rt1 = 0.5 * (sm - rt);
        sgn1 = -1;
        rt2 = (acmx / rt1) * acmn - (b / rt1) * b;
    } else if (sm > 0.0) {
        rt1 = 0.5 * (sm + rt);
        sgn1 = 1;
        rt2 = (acmx / rt1) * acmn - (b / rt1) * b;
    } else {
        rt1 = 0.5 * rt;
        rt2 = -0.5 * rt;
        sgn1 = 1;
    }
    int sgn2;
    double cs;
    if (df >= 0.0) {
        cs = df + rt;
        sgn2 = 1;
    } else {
        cs = df - rt;
        sgn2 = -1;
    }
    if (fabs(cs) > ab) {
        const double ct = -tb / cs;
        sn1 = 1.0 / sqrt(1.0 + ct * ct);
        cs1 = ct * sn1;
    } else if (ab == 0.0) {
        cs1 = 1.0;
        sn1 = 0.0;
    } else {
        const double tn = -cs / tb;
        cs1 = 1.0 / sqrt(1.0 + tn * tn);
        sn1 = tn * cs1;
    }
    if (sgn1 == sgn2) {
        const double tn = cs1;
        cs1 = -sn1;
        sn1 = tn;
    }
}

// out[k] = (major length, minor length, angle) of covariance k (row-major 2x2,
// the lower triangle is used as dsyevd uplo L does); column: the eigenvector
// column (column_vectors=True) instead of the reference's row quirk (:51)
__global__ __launch_bounds__(256) void error_ellipse_kernel(const int64_t n,
                                                            const double* __restrict__ cov,
                                                            const double chi, const int column,
                                                            double* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double a = cov[4 * k], b = cov[4 * k + 2], c = cov[4 * k + 3];   // A(1,1), A(2,1), A(2,2)
    const double anrm = fmax(fmax(fabs(a), fabs(b)), fabs(c));
    // dsyevd scales outside [sqrt(smlnum), sqrt(bignum)]; dsteqr outside [ssfmin, ssfmax]
    const bool scaled = anrm != 0.0 && (anrm < 0x1p-405 || anrm > 0x1p+508 || isnan(anrm));
    double w0 = a, w1 = c, z00 = 1.0, z01 = 0.0, z10 = 0.0, z11 = 1.0;
    const double eps = 0x1p-53, eps2 = 0x1p-106, safmin = 0x1p-1022;   // dlamch('E'), eps^2, ('S')
    const double tst = fabs(b);
    // the splitting test (dsteqr label 10), then the QL / QR iteration's own
    // (QR when |d(2)| < |d(1)|: the products in the other order)
    bool rotate = tst != 0.0 && !(tst <= (sqrt(fabs(a)) * sqrt(fabs(c))) * eps);
    if (rotate) {
        const double t2 = tst * tst;
        const double lim = (fabs(c) < fabs(a)) ? (eps2 * fabs(c)) * fabs(a) + safmin
                                               : (eps2 * fabs(a)) * fabs(c) + safmin;
        rotate = !(t2 <= lim);
    }
    if (rotate) {
        double rt1, rt2, cs1, sn1;
        dlaev2_dev(a, b, c, rt1, rt2, cs1, sn1);
        w0 = rt1;
        w1 = rt2;
        z00 = cs1;                                           // dlasr('R', 'V', ...) on Z = I
        z10 = sn1;
        z01 = -sn1;
        z11 = cs1;
    }
    if (w1 < w0) {                                           // dsteqr's selection sort
        double t = w0;
        w0 = w1;
        w1 = t;
        t = z00;
        z00 = z01;
        z01 = t;
        t = z10;
        z10 = z11;
        z11 = t;
    }
    // argmax / argmin of (w0, w1): first occurrence
    const int imax = (w1 > w0) ? 1 : 0;
    const int imin = (w1 < w0) ? 1 : 0;
    double v0, v1;
    if (column) {
        v0 = imax ? z01 : z00;
        v1 = imax ? z11 : z10;
    } else {                                                 // vec[idxmax]: a row
        v0 = imax ? z10 : z00;
        v1 = imax ? z11 : z01;
    }
    const double wmax = imax ? w1 : w0, wmin = imin ? w1 : w0;
    double l = sqrt(wmax * chi) * 2.0, s = sqrt(wmin * chi) * 2.0, ang = atan2(v1, v0);
    if (scaled) l = s = ang = NAN;
    out[3 * k] = l;
    out[3 * k + 1] = s;
    out[3 * k + 2] = ang;
}

namespace {
struct EllipseScratch {
    std::mutex mu;
    size_t cap = 0;
    double* buf = nullptr;
    hipStream_t stream = nullptr;
};
EllipseScratch& ellipse_scratch(int device) {
    static EllipseScratch s[64];
    return s[device & 63];
}
}  // namespace
}  // namespace slam

using namespace slam;

extern "C" int slam_error_ellipse(int64_t n, const double* covs, double chi, int32_t column_vectors,
                                  double* out, int device) {
    SLAM_ARG_CHECK(n >= 0 && (covs && out || n == 0), "slam_error_ellipse: bad arguments");
    if (n == 0) return SLAM_OK;
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev && device < 64, "slam_error_ellipse: no such HIP device");
    EllipseScratch& sc = ellipse_scratch(device);
    std::lock_guard<std::mutex> lock(sc.mu);
    SLAM_HIP_TRY(hipSetDevice(device));
    if (!sc.stream) SLAM_HIP_TRY(hipStreamCreateWithFlags(&sc.stream, hipStreamNonBlocking));
    if ((size_t)n > sc.cap) {
        if (sc.buf) (void)hipFree(sc.buf);
        sc.buf = nullptr;
        sc.cap = 0;
        SLAM_HIP_TRY(hipMalloc(&sc.buf, sizeof(double) * 7 * (size_t)n));
        sc.cap = (size_t)n;
    }
    double* d_cov = sc.buf;
    double* d_out = sc.buf + 4 * sc.cap;
    SLAM_HIP_TRY(hipMemcpyAsync(d_cov, covs, 32 * n, hipMemcpyHostToDevice, sc.stream));
    error_ellipse_kernel<<<(unsigned)((n + 255) / 256), 256, 0, sc.stream>>>(n, d_cov, chi,
                                                                            column_vectors ? 1 : 0, d_out);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(out, d_out, 24 * n, hipMemcpyDeviceToHost, sc.stream));
    SLAM_HIP_TRY(hipStreamSynchronize(sc.stream));
    return SLAM_OK;
}
