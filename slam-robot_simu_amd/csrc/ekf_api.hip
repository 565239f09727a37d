// ekf_api.hip -- C-ABI of the EKF localisation filter (batched) and of
// EKF-SLAM (include/slam_hip.h).
//
// ExtendedKalmanFilter (extended_kalman_filter.py:17-205) -> slam_ekf_*;
// EKF-SLAM (BASELINE config 4) -> slam_ekfslam_*.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ekf_kernels.inl"

using namespace slam;

struct slam_ekf {
    slam_ekf_config cfg;
    int device = 0;
    int64_t batch = 0;
    hipStream_t stream = nullptr;
    double* xs = nullptr;          // [3][B]
    double* Ps = nullptr;          // [9][B]
    double* z = nullptr;           // staging [steps][B][2]
    double* xh = nullptr;          // staging [steps][B][3]
    double* xm = nullptr;          // [B][3]
    int32_t cap_steps = 0;
};

struct slam_ekfslam {
    slam_ekfslam_config cfg;
    int device = 0;
    int64_t n_lm = 0, n = 0, ld = 0, n_pad = 0;
    int64_t pipe_grid = 0;         // persistent rank-update grid (resident workgroups, x8)
    int64_t frag_grid = 0;         // resident grid of the fragment-streaming rank update
    int32_t kernel_sel = 0;        // 0: fragment-streaming (m <= 64), 1: LDS-staged
    int32_t frag_shape = 0;        // 0: 8 waves of 32 x 64, 1: 16 waves of 32 x 32
    int32_t frag_pf = 0;           // experiment: where the next P block is requested
    int32_t apply_lds = 0;         // SLAM_EKS_APPLY=lds: the one-wave-per-row K = PH^T S^-1
    hipStream_t stream = nullptr;
    double* P = nullptr;           // n x ld, lower triangle current
    double* mu = nullptr;          // n
    double* pht = nullptr;         // n_pad x M
    double* kg = nullptr;          // n_pad x M
    double* kf = nullptr;          // -K quad-major: [M/4][n_pad][4]
    double* hf = nullptr;          // PH^T quad-major
    double* hs = nullptr;          // kEksMaxM/3 x 18
    double* e = nullptr;           // M
    double* rd = nullptr;          // M
    double* sinv = nullptr;        // M x M
    int64_t* ids = nullptr;        // k
    double* diag = nullptr;        // n (init_diag staging)
    hipEvent_t ev[6] = {};
    double last_ms[5] = {0, 0, 0, 0, 0};
};

namespace {

EKFConst ekf_const(const slam_ekf_config& c) {
    EKFConst k;
    k.dt = c.dt;
    k.vel = c.vel;
    k.omega = c.omega;
    for (int i = 0; i < 9; ++i) k.q[i] = c.q[i];
    for (int i = 0; i < 4; ++i) k.r[i] = c.r[i];
    k.motion = c.motion;
    for (int i = 0; i < 6; ++i) k.alphas[i] = c.alphas[i];
    return k;
}

int ekf_reserve(slam_ekf* h, int32_t steps) {
    if (steps <= h->cap_steps) return SLAM_OK;
    if (h->z) SLAM_HIP_TRY(hipFree(h->z));
    if (h->xh) SLAM_HIP_TRY(hipFree(h->xh));
    h->z = h->xh = nullptr;
    SLAM_HIP_TRY(hipMalloc(&h->z, (size_t)steps * h->batch * 2 * sizeof(double)));
    SLAM_HIP_TRY(hipMalloc(&h->xh, (size_t)steps * h->batch * 3 * sizeof(double)));
    h->cap_steps = steps;
    return SLAM_OK;
}

// host AoS [B][k] <-> device SoA [k][B]
int ekf_upload_soa(slam_ekf* h, double* dst, const double* src, int k) {
    std::vector<double> t((size_t)k * h->batch);
    for (int64_t b = 0; b < h->batch; ++b)
        for (int q = 0; q < k; ++q) t[(size_t)q * h->batch + b] = src[b * k + q];
    SLAM_HIP_TRY(hipMemcpyAsync(dst, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice,
                                h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int ekf_download_soa(slam_ekf* h, double* dst, const double* src, int k) {
    std::vector<double> t((size_t)k * h->batch);
    SLAM_HIP_TRY(hipMemcpyAsync(t.data(), src, t.size() * sizeof(double), hipMemcpyDeviceToHost,
                                h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    for (int64_t b = 0; b < h->batch; ++b)
        for (int q = 0; q < k; ++q) dst[b * k + q] = t[(size_t)q * h->batch + b];
    return SLAM_OK;
}

int ekf_launch(slam_ekf* h, int32_t steps, const double* control, double* xm_last,
               double* xh_all) {
    const double v = control ? control[0] : h->cfg.vel;
    const double om = control ? control[1] : h->cfg.omega;
    const int64_t blocks = (h->batch + 255) / 256;
    hipLaunchKernelGGL(ekf_run_kernel, dim3((unsigned)blocks), dim3(256), 0, h->stream, h->batch,
                       steps, ekf_const(h->cfg), v, om, h->xs, h->Ps, h->z, xh_all, xm_last);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// ---------------------------------------------------------------- EKF-SLAM
EksConst eks_const(const slam_ekfslam_config& c) {
    EksConst k;
    k.dt = c.dt;
    for (int i = 0; i < 9; ++i) k.q[i] = c.q_robot[i];
    k.r_dist = c.r_dist;
    k.r_dir = c.r_dir;
    k.r_orient = c.r_orient;
    k.motion = c.motion;
    for (int i = 0; i < 6; ++i) k.alphas[i] = c.alphas[i];
    return k;
}

int eks_predict(slam_ekfslam* h, const double* control) {
    const double v = control[0], om = control[1];
    const int64_t rows = h->n - 3;
    if (rows > 0)
        hipLaunchKernelGGL(eks_predict_rows_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256),
                           0, h->stream, h->P, h->n, h->ld, h->mu, eks_const(h->cfg), v, om);
    hipLaunchKernelGGL(eks_predict_pose_kernel, dim3(1), dim3(64), 0, h->stream, h->P, h->ld,
                       h->mu, eks_const(h->cfg), v, om);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int eks_update(slam_ekfslam* h, int32_t k, const int64_t* ids, const double* obs) {
    SLAM_ARG_CHECK(k >= 1 && 3 * k <= kEksMaxM, "slam_ekfslam_update: need 1 <= k <= 40");
    for (int32_t t = 0; t < k; ++t)
        SLAM_ARG_CHECK(ids[t] >= 0 && ids[t] < h->n_lm, "slam_ekfslam_update: landmark id out of range");
    const int32_t m = 3 * k;
    const int32_t M = (m + 3) / 4 * 4;
    EksObs ob{};
    for (int32_t t = 0; t < k; ++t) ob.ids[t] = ids[t];
    for (int32_t u = 0; u < 3 * k; ++u) ob.obs[u] = obs[u];
    const EksConst c = eks_const(h->cfg);
    SLAM_HIP_TRY(hipEventRecord(h->ev[0], h->stream));
    hipLaunchKernelGGL(eks_build_kernel, dim3(1), dim3(128), 0, h->stream, h->mu, ob, h->ids, k,
                       M, c, h->hs, h->e, h->rd);
    hipLaunchKernelGGL(eks_pht_kernel, dim3((unsigned)((h->n_pad + 255) / 256)), dim3(256), 0,
                       h->stream, h->P, h->n, h->ld, h->n_pad, h->ids, h->hs, k, M, h->pht);
    SLAM_HIP_TRY(hipEventRecord(h->ev[1], h->stream));
    const size_t sbytes = (size_t)M * M * sizeof(double);
    hipLaunchKernelGGL(eks_gain_kernel, dim3(1), dim3(1024), sbytes, h->stream, h->pht, h->ids,
                       h->hs, h->rd, k, M, h->sinv);
    SLAM_HIP_TRY(hipEventRecord(h->ev[2], h->stream));
    const int64_t apply_grid = std::min<int64_t>(512, (h->n_pad + 15) / 16);
    if (M <= 64 && !h->apply_lds) {
        hipLaunchKernelGGL(eks_apply_mfma_kernel, dim3((unsigned)((h->n_pad / 16 + 3) / 4)), dim3(256),
                           0, h->stream, h->pht, h->sinv, h->e, h->n, h->n_pad, M, h->kg, h->mu);
    } else {
        hipLaunchKernelGGL(eks_apply_kernel, dim3((unsigned)apply_grid), dim3(kEksApplyThreads),
                           sbytes, h->stream, h->pht, h->sinv, h->e, h->n, h->n_pad, M, h->kg, h->mu);
    }
    SLAM_HIP_TRY(hipEventRecord(h->ev[3], h->stream));
    const int64_t nt = h->n_pad / kEksTile;
    const int64_t tiles = nt * (nt + 1) / 2;
#ifndef SLAM_EKS_PIPE
#define SLAM_EKS_PIPE 1
#endif
    if (h->frag_grid > 0 && M <= kEksPipeK && h->kernel_sel == 0) {
        const int64_t tot = h->n_pad * M;
        hipLaunchKernelGGL(eks_frag_layout_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                           h->stream, h->kg, h->pht, h->n_pad, M, h->kf, h->hf);
#define SLAM_EKS_FRAG_S(QQ, WM, WN)                                                               \
    hipLaunchKernelGGL((eks_rank_update_frag_kernel<QQ, WM, WN>), dim3((unsigned)h->frag_grid),   \
                       dim3(EksFragShape<WM, WN>::kThreads), 0, h->stream, h->P, h->n, h->ld,      \
                       h->kf, h->hf, h->n_pad, tiles)
#define SLAM_EKS_FRAG(QQ)                                                                         \
    case QQ:                                                                                      \
        if (h->frag_shape == 1) SLAM_EKS_FRAG_S(QQ, 2, 2); else SLAM_EKS_FRAG_S(QQ, 2, 4);          \
        break
#define SLAM_EKS_FRAG_P(QQ, PF)                                                                   \
    hipLaunchKernelGGL((eks_rank_update_frag_kernel<QQ, 2, 4, PF>), dim3((unsigned)h->frag_grid), \
                       dim3(EksFragShape<2, 4>::kThreads), 0, h->stream, h->P, h->n, h->ld,        \
                       h->kf, h->hf, h->n_pad, tiles)
        if (M / 4 == 15 && h->frag_pf == 1) SLAM_EKS_FRAG_P(15, 7);
        else if (M / 4 == 15 && h->frag_pf == 2) SLAM_EKS_FRAG_P(15, 0);
        else switch (M / 4) {
            SLAM_EKS_FRAG(1); SLAM_EKS_FRAG(2); SLAM_EKS_FRAG(3); SLAM_EKS_FRAG(4);
            SLAM_EKS_FRAG(5); SLAM_EKS_FRAG(6); SLAM_EKS_FRAG(7); SLAM_EKS_FRAG(8);
            SLAM_EKS_FRAG(9); SLAM_EKS_FRAG(10); SLAM_EKS_FRAG(11); SLAM_EKS_FRAG(12);
            SLAM_EKS_FRAG(13); SLAM_EKS_FRAG(14); SLAM_EKS_FRAG(15); SLAM_EKS_FRAG(16);
            default: return fail(SLAM_ERR_ARG, "slam_ekfslam_update: bad operand width");
        }
#undef SLAM_EKS_FRAG_S
#undef SLAM_EKS_FRAG_P
#undef SLAM_EKS_FRAG
    } else if (SLAM_EKS_PIPE && h->pipe_grid > 0 && M <= kEksPipeK) {
        hipLaunchKernelGGL(eks_rank_update_pipelined_kernel, dim3((unsigned)h->pipe_grid),
                           dim3(kEksPipeThreads), 0, h->stream, h->P, h->n, h->ld, h->kg, h->pht, M,
                           tiles);
    } else {
        const int64_t grid = (tiles + 7) / 8 * 8;
        hipLaunchKernelGGL(eks_rank_update_kernel, dim3((unsigned)grid), dim3(kEksThreads), 0,
                           h->stream, h->P, h->n, h->ld, h->kg, h->pht, M, tiles);
    }
    SLAM_HIP_TRY(hipEventRecord(h->ev[4], h->stream));
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int eks_collect_timing(slam_ekfslam* h) {
    SLAM_HIP_TRY(hipEventSynchronize(h->ev[4]));
    float ms;
    for (int q = 0; q < 4; ++q) {
        SLAM_HIP_TRY(hipEventElapsedTime(&ms, h->ev[q], h->ev[q + 1]));
        h->last_ms[q] = ms;
    }
    return SLAM_OK;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ EKF
int slam_ekf_create(const slam_ekf_config* cfg, int64_t batch, int device, slam_ekf** out) {
    SLAM_ARG_CHECK(cfg && out && batch >= 1, "slam_ekf_create: bad arguments");
    SLAM_ARG_CHECK(cfg->motion == SLAM_MOTION_LINEAR || cfg->motion == SLAM_MOTION_VELOCITY,
                   "slam_ekf_create: bad motion model");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(SLAM_ERR_ARG, "slam_ekf_create: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    slam_ekf* h = new slam_ekf();
    h->cfg = *cfg;
    h->device = device;
    h->batch = batch;
    auto bail = [&](int rc) {
        slam_ekf_destroy(h);
        return rc;
    };
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&h->xs, 3 * batch * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->Ps, 9 * batch * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->xm, 3 * batch * sizeof(double)) != hipSuccess)
        return bail(fail(SLAM_ERR_HIP, "slam_ekf_create: allocation failed"));
    std::vector<double> x0((size_t)batch * 3), p0((size_t)batch * 9);
    for (int64_t b = 0; b < batch; ++b) {
        std::memcpy(&x0[b * 3], cfg->x0, 3 * sizeof(double));
        std::memcpy(&p0[b * 9], cfg->p0, 9 * sizeof(double));
    }
    int rc = slam_ekf_set_state(h, x0.data(), p0.data());
    if (rc != SLAM_OK) return bail(rc);
    *out = h;
    return SLAM_OK;
}

int slam_ekf_destroy(slam_ekf* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    for (double* p : {h->xs, h->Ps, h->z, h->xh, h->xm})
        if (p) (void)hipFree(p);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_ekf_set_state(slam_ekf* h, const double* x, const double* P) {
    SLAM_ARG_CHECK(h, "slam_ekf_set_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (x) {
        int rc = ekf_upload_soa(h, h->xs, x, 3);
        if (rc) return rc;
    }
    if (P) {
        int rc = ekf_upload_soa(h, h->Ps, P, 9);
        if (rc) return rc;
    }
    return SLAM_OK;
}

int slam_ekf_get_state(slam_ekf* h, double* x, double* P) {
    SLAM_ARG_CHECK(h, "slam_ekf_get_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (x) {
        int rc = ekf_download_soa(h, x, h->xs, 3);
        if (rc) return rc;
    }
    if (P) {
        int rc = ekf_download_soa(h, P, h->Ps, 9);
        if (rc) return rc;
    }
    return SLAM_OK;
}

int slam_ekf_step(slam_ekf* h, const double* control, const double* z, double* x_hat_m,
                  double* x_hat, double* P) {
    SLAM_ARG_CHECK(h && z, "slam_ekf_step: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = ekf_reserve(h, 1);
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemcpyAsync(h->z, z, h->batch * 2 * sizeof(double), hipMemcpyHostToDevice,
                                h->stream));
    rc = ekf_launch(h, 1, control, h->xm, nullptr);
    if (rc) return rc;
    if (x_hat_m) {
        SLAM_HIP_TRY(hipMemcpyAsync(x_hat_m, h->xm, h->batch * 3 * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return slam_ekf_get_state(h, x_hat, P);
}

int slam_ekf_run(slam_ekf* h, int32_t n_steps, const double* control, const double* z_all,
                 double* x_hat_all) {
    SLAM_ARG_CHECK(h && z_all && n_steps >= 1, "slam_ekf_run: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = ekf_reserve(h, n_steps);
    if (rc) return rc;
    const size_t zb = (size_t)n_steps * h->batch * 2 * sizeof(double);
    SLAM_HIP_TRY(hipMemcpyAsync(h->z, z_all, zb, hipMemcpyHostToDevice, h->stream));
    rc = ekf_launch(h, n_steps, control, h->xm, x_hat_all ? h->xh : nullptr);
    if (rc) return rc;
    if (x_hat_all)
        SLAM_HIP_TRY(hipMemcpyAsync(x_hat_all, h->xh, (size_t)n_steps * h->batch * 3 * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

// Device-resident variant for the bench: observations already on the device
// (z_dev: n_steps x B x 2), estimates to x_hat_dev (or NULL).  Asynchronous.
int slam_ekf_run_device(slam_ekf* h, int32_t n_steps, const double* control, const double* z_dev,
                        double* x_hat_dev) {
    SLAM_ARG_CHECK(h && z_dev && n_steps >= 1, "slam_ekf_run_device: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const double v = control ? control[0] : h->cfg.vel;
    const double om = control ? control[1] : h->cfg.omega;
    const int64_t blocks = (h->batch + 255) / 256;
    hipLaunchKernelGGL(ekf_run_kernel, dim3((unsigned)blocks), dim3(256), 0, h->stream, h->batch,
                       n_steps, ekf_const(h->cfg), v, om, h->xs, h->Ps, z_dev, x_hat_dev, h->xm);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int slam_ekf_load_observations(slam_ekf* h, int32_t n_steps, const double* z_all) {
    SLAM_ARG_CHECK(h && z_all && n_steps >= 1, "slam_ekf_load_observations: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = ekf_reserve(h, n_steps);
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemcpyAsync(h->z, z_all, (size_t)n_steps * h->batch * 2 * sizeof(double),
                                hipMemcpyHostToDevice, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekf_run_loaded(slam_ekf* h, int32_t n_steps, const double* control, int32_t keep_history) {
    SLAM_ARG_CHECK(h && n_steps >= 1 && n_steps <= h->cap_steps,
                   "slam_ekf_run_loaded: load at least n_steps observations first");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    return ekf_launch(h, n_steps, control, h->xm, keep_history ? h->xh : nullptr);
}

int slam_ekf_synchronize(slam_ekf* h) {
    SLAM_ARG_CHECK(h, "slam_ekf_synchronize: NULL handle");
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

// ------------------------------------------------------------- EKF-SLAM
int slam_ekfslam_create(const slam_ekfslam_config* cfg, int64_t n_landmarks, int device,
                        slam_ekfslam** out) {
    SLAM_ARG_CHECK(cfg && out && n_landmarks >= 1, "slam_ekfslam_create: bad arguments");
    SLAM_ARG_CHECK(cfg->motion == SLAM_MOTION_LINEAR || cfg->motion == SLAM_MOTION_VELOCITY,
                   "slam_ekfslam_create: bad motion model");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(SLAM_ERR_ARG, "slam_ekfslam_create: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    slam_ekfslam* h = new slam_ekfslam();
    h->cfg = *cfg;
    h->device = device;
    h->n_lm = n_landmarks;
    h->n = 3 + 3 * n_landmarks;
    // rows start on 128-byte lines: a tile row segment (16 lanes x 8 B) is one line
#ifndef SLAM_EKS_LD_ALIGN
#define SLAM_EKS_LD_ALIGN 16
#endif
#ifndef SLAM_EKS_LD_SKEW
#define SLAM_EKS_LD_SKEW 0
#endif
    h->ld = (h->n + SLAM_EKS_LD_ALIGN - 1) / SLAM_EKS_LD_ALIGN * SLAM_EKS_LD_ALIGN + SLAM_EKS_LD_SKEW;
    h->n_pad = (h->n + kEksTile - 1) / kEksTile * kEksTile;
    auto bail = [&](int rc) {
        slam_ekfslam_destroy(h);
        return rc;
    };
    {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, eks_rank_update_pipelined_kernel,
                                                         kEksPipeThreads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
                hipSuccess)
            h->pipe_grid = (int64_t)per_cu * cus / 8 * 8;
        // SLAM_EKS_KERNEL=pipe selects the LDS-staged kernel, =frag16 the
        // 16-wave fragment shape (comparison runs); default: 8 waves of 32 x 64
        const char* ks = std::getenv("SLAM_EKS_KERNEL");
        const std::string sel = ks ? ks : "";
        h->kernel_sel = sel == "pipe" ? 1 : 0;
        h->frag_shape = (sel == "frag16") ? 1 : 0;
        h->frag_pf = sel == "pfmid" ? 1 : sel == "pf0" ? 2 : 0;
        const char* ap = std::getenv("SLAM_EKS_APPLY");
        h->apply_lds = (ap && std::string(ap) == "lds") ? 1 : 0;
        const hipError_t oe =
            h->frag_shape == 1
                ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                      &per_cu, eks_rank_update_frag_kernel<15, 2, 2>, EksFragShape<2, 2>::kThreads, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                      &per_cu, eks_rank_update_frag_kernel<15, 2, 4>, EksFragShape<2, 4>::kThreads, 0);
        if (oe == hipSuccess && cus > 0) h->frag_grid = (int64_t)std::max(per_cu, 1) * cus / 8 * 8;
    }
    const size_t pbytes = (size_t)h->n * h->ld * sizeof(double);
    const size_t rows = (size_t)h->n_pad * kEksMaxM;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&h->P, pbytes) != hipSuccess ||
        hipMalloc(&h->mu, h->n * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->pht, rows * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->kg, rows * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->kf, (size_t)h->n_pad * kEksPipeK * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->hf, (size_t)h->n_pad * kEksPipeK * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->hs, (kEksMaxM / 3) * 18 * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->e, kEksMaxM * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->rd, kEksMaxM * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->sinv, kEksMaxM * kEksMaxM * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->ids, (kEksMaxM / 3) * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&h->diag, h->n * sizeof(double)) != hipSuccess)
        return bail(fail(SLAM_ERR_HIP, "slam_ekfslam_create: allocation failed (P is n^2 fp64)"));
    for (auto& e : h->ev)
        if (hipEventCreate(&e) != hipSuccess)
            return bail(fail(SLAM_ERR_HIP, "slam_ekfslam_create: event creation failed"));
    if (hipMemsetAsync(h->P, 0, pbytes, h->stream) != hipSuccess ||
        hipMemsetAsync(h->mu, 0, h->n * sizeof(double), h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess)
        return bail(fail(SLAM_ERR_HIP, "slam_ekfslam_create: initialisation failed"));
    const size_t big = (size_t)kEksMaxM * kEksMaxM * sizeof(double);
    if (hipFuncSetAttribute((const void*)eks_gain_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)big) != hipSuccess ||
        hipFuncSetAttribute((const void*)eks_apply_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)big) != hipSuccess)
        return bail(fail(SLAM_ERR_HIP, "slam_ekfslam_create: LDS attribute failed"));
    *out = h;
    return SLAM_OK;
}

int slam_ekfslam_destroy(slam_ekfslam* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    for (void* p : {(void*)h->P, (void*)h->mu, (void*)h->pht, (void*)h->kg, (void*)h->kf, (void*)h->hf,
                    (void*)h->hs,
                    (void*)h->e, (void*)h->rd, (void*)h->sinv, (void*)h->ids, (void*)h->diag})
        if (p) (void)hipFree(p);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_ekfslam_set_state(slam_ekfslam* h, const double* mu, const double* P) {
    SLAM_ARG_CHECK(h, "slam_ekfslam_set_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (mu)
        SLAM_HIP_TRY(hipMemcpyAsync(h->mu, mu, h->n * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    if (P)
        SLAM_HIP_TRY(hipMemcpy2DAsync(h->P, h->ld * sizeof(double), P, h->n * sizeof(double),
                                      h->n * sizeof(double), h->n, hipMemcpyHostToDevice,
                                      h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_init_diag(slam_ekfslam* h, const double* mu, const double* p_diag) {
    SLAM_ARG_CHECK(h && p_diag, "slam_ekfslam_init_diag: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (mu)
        SLAM_HIP_TRY(hipMemcpyAsync(h->mu, mu, h->n * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    SLAM_HIP_TRY(hipMemsetAsync(h->P, 0, (size_t)h->n * h->ld * sizeof(double), h->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(h->diag, p_diag, h->n * sizeof(double), hipMemcpyHostToDevice,
                                h->stream));
    hipLaunchKernelGGL(eks_diag_kernel, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0,
                       h->stream, h->P, h->n, h->ld, h->diag);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_get_state(slam_ekfslam* h, double* mu, double* P) {
    SLAM_ARG_CHECK(h, "slam_ekfslam_get_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (mu)
        SLAM_HIP_TRY(hipMemcpyAsync(mu, h->mu, h->n * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    if (P) {
        // symmetrise row blocks through the K scratch (n_pad x kEksMaxM doubles)
        const int64_t chunk = std::max<int64_t>(1, (h->n_pad * kEksMaxM) / h->n);
        for (int64_t i0 = 0; i0 < h->n; i0 += chunk) {
            const int64_t rows = std::min<int64_t>(chunk, h->n - i0);
            hipLaunchKernelGGL(eks_symmetrize_kernel, dim3((unsigned)((h->n + 255) / 256),
                               (unsigned)rows), dim3(256), 0, h->stream, h->P, h->n, h->ld, i0,
                               h->kg);
            SLAM_HIP_TRY(hipGetLastError());
            SLAM_HIP_TRY(hipMemcpyAsync(P + i0 * h->n, h->kg, rows * h->n * sizeof(double),
                                        hipMemcpyDeviceToHost, h->stream));
            SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
        }
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_get_rows(slam_ekfslam* h, int64_t k, const int64_t* rows, double* out) {
    SLAM_ARG_CHECK(h && (k == 0 || (rows && out)) && k >= 0, "slam_ekfslam_get_rows: bad argument");
    for (int64_t r = 0; r < k; ++r)
        SLAM_ARG_CHECK(rows[r] >= 0 && rows[r] < h->n, "slam_ekfslam_get_rows: row out of range");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    // batches of rows through the K scratch (n_pad x kEksMaxM doubles) and the
    // id scratch (kEksMaxM / 3 int64)
    const int64_t chunk = std::min<int64_t>(kEksMaxM / 3,
                                            std::max<int64_t>(1, (h->n_pad * kEksMaxM) / h->n));
    for (int64_t r0 = 0; r0 < k; r0 += chunk) {
        const int64_t cnt = std::min<int64_t>(chunk, k - r0);
        SLAM_HIP_TRY(hipMemcpyAsync(h->ids, rows + r0, cnt * sizeof(int64_t), hipMemcpyHostToDevice,
                                    h->stream));
        hipLaunchKernelGGL(eks_gather_rows_kernel, dim3((unsigned)((h->n + 255) / 256), (unsigned)cnt),
                           dim3(256), 0, h->stream, h->P, h->n, h->ld, h->ids, h->kg);
        SLAM_HIP_TRY(hipGetLastError());
        SLAM_HIP_TRY(hipMemcpyAsync(out + r0 * h->n, h->kg, cnt * h->n * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
        SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return SLAM_OK;
}

int slam_ekfslam_predict(slam_ekfslam* h, const double* control) {
    SLAM_ARG_CHECK(h && control, "slam_ekfslam_predict: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = eks_predict(h, control);
    if (rc) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_update(slam_ekfslam* h, int32_t k, const int64_t* ids, const double* obs) {
    SLAM_ARG_CHECK(h && ids && obs, "slam_ekfslam_update: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = eks_update(h, k, ids, obs);
    if (rc) return rc;
    rc = eks_collect_timing(h);
    if (rc) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_step(slam_ekfslam* h, const double* control, int32_t k, const int64_t* ids,
                      const double* obs) {
    SLAM_ARG_CHECK(h && control && ids && obs, "slam_ekfslam_step: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = eks_predict(h, control);
    if (rc) return rc;
    rc = eks_update(h, k, ids, obs);
    if (rc) return rc;
    rc = eks_collect_timing(h);
    if (rc) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_ekfslam_timing(slam_ekfslam* h, double* out) {
    SLAM_ARG_CHECK(h && out, "slam_ekfslam_timing: NULL argument");
    for (int q = 0; q < 5; ++q) out[q] = h->last_ms[q];
    return SLAM_OK;
}

}  // extern "C"
