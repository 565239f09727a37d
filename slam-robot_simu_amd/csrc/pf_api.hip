// pf_api.hip -- C-ABI of the particle filter (include/slam_hip.h).
//
// Replaces ParticleFilter (particle_filter.py:18-237).  One handle = one GPU,
// one HIP stream, SoA particle state resident in HBM.
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "pf_kernels.hpp"

#include "pf_kernels.inl"

namespace slam {

// numpy pairwise split of a tail buffer (< 8192 elements): leaves + post-order program
static void build_tail(int lo, int n, std::vector<int32_t>& leaves, std::vector<int32_t>& ops) {
    if (n <= 128) {
        ops.push_back((int32_t)(leaves.size() / 2));
        leaves.push_back(lo);
        leaves.push_back(n);
        return;
    }
    int h = n / 2;
    h -= h % 8;
    build_tail(lo, h, leaves, ops);
    build_tail(lo + h, n - h, leaves, ops);
    ops.push_back(-1);
}

struct Timer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[4];
    size_t used[4] = {0, 0, 0, 0};
};

}  // namespace slam

using namespace slam;

struct slam_pf {
    slam_pf_config cfg;
    int device = 0;
    int64_t n = 0;
    int32_t nl = 0;
    hipStream_t stream = nullptr;
    // state (ping-pong)
    double* x[2] = {nullptr, nullptr};
    double* y[2] = {nullptr, nullptr};
    double* th[2] = {nullptr, nullptr};
    int cur = 0;
    double *w = nullptr, *w_un = nullptr;
    // resample scratch
    double* c = nullptr;
    uint64_t* kincl = nullptr;
    int32_t* fexcl = nullptr;
    int32_t* idx = nullptr;
    int32_t nb_scan = 0;
    double *bsum = nullptr, *boff = nullptr;
    uint64_t *bk = nullptr, *boffk = nullptr, *ktot = nullptr;
    int32_t *bf = nullptr, *bofff = nullptr, *nspec = nullptr;
    SpecialIn* spec_in = nullptr;
    SpecialOut* spec_out = nullptr;
    // reductions
    int32_t nchunks = 0;
    double* part = nullptr;
    int32_t* tail_leaves = nullptr;
    int32_t* tail_ops = nullptr;
    int32_t n_tail_leaves = 0, n_tail_ops = 0;
    int32_t nb_norm = 0;
    BlockPartial* bp = nullptr;
    double* wsum = nullptr;
    double* refp = nullptr;
    int32_t* flags = nullptr;
    unsigned* counters = nullptr;   // last-arriver tickets (zeroed by the last block)
    // inputs
    double* lm = nullptr;
    double* z = nullptr;
    double* noise = nullptr;
    double* z_all = nullptr;
    int32_t z_steps = 0;
    slam_pf_result* res_dev = nullptr;
    int32_t res_cap = 0;
    slam_pf_result* res_host = nullptr;   // pinned
    LikConst lc;
    uint32_t stepno = 0;
    int32_t resample_next = 0;            // host mirror of the device flag
    bool timing = false;
    Timer tm;
};

namespace {

template <typename T>
int dalloc(T** p, size_t count) {
    if (count == 0) count = 1;
    SLAM_HIP_TRY(hipMalloc((void**)p, count * sizeof(T)));
    return SLAM_OK;
}

int make_lik_const(slam_pf* h) {
    // particle_filter.py:179-181 and the bivariate_normal constants, in numpy's order
    const double* R = h->cfg.r_cov;
    LikConst& lc = h->lc;
    const double sx = std::sqrt(R[0]), sy = std::sqrt(R[3]), sxy = std::sqrt(R[1]);
    if (!(sx > 0) || !(sy > 0) || std::isnan(sxy))
        return fail(SLAM_ERR_ARG, "r_cov: need R00 > 0, R11 > 0, R01 >= 0");
    const double rho = sxy / (sx * sy);
    lc.sx2 = sx * sx;
    lc.sy2 = sy * sy;
    lc.rsx2 = 1.0 / lc.sx2;
    lc.rsy2 = 1.0 / lc.sy2;
    lc.rho2 = 2 * rho;
    lc.sxsy = sx * sy;
    lc.d2 = 2 * (1 - rho * rho);
    lc.den = 2 * kPi * sx * sy * std::sqrt(1 - rho * rho);
    lc.rden = 1.0 / lc.den;
    lc.nl = h->nl;
    lc.neg_nl_ln_den = -(double)h->nl * std::log(lc.den);
    lc.has_rho = (rho != 0.0) ? 1 : 0;
    lc.rsxsy = 1.0 / lc.sxsy;
    lc.rd2 = 1.0 / lc.d2;
    lc.iso = (lc.sx2 == lc.sy2 && !lc.has_rho) ? 1 : 0;
    lc.pad = 0;
    return SLAM_OK;
}

PredictConst make_predict_const(slam_pf* h, const double* control) {
    PredictConst pc;
    const slam_pf_config& c = h->cfg;
    pc.dt = c.dt;
    pc.v = control[0];
    pc.om = control[1];
    pc.vdt_om = control[1] * c.dt;
    // motion_model.py:40-45 (the std passed to normal() is the squared "sigma")
    const double v2 = pc.v * pc.v, w2 = pc.om * pc.om;
    const double sv = (c.alphas[0] * v2) + (c.alphas[1] * w2);
    const double sw = (c.alphas[2] * v2) + (c.alphas[3] * w2);
    const double sg = (c.alphas[4] * v2) + (c.alphas[5] * w2);
    pc.sv = sv * sv;
    pc.sw = sw * sw;
    pc.sg = sg * sg;
    for (int k = 0; k < 9; ++k) pc.q[k] = c.q_factor[k];
    pc.np_recip = 1.0 / (double)h->n;
    pc.n_global = h->n;
    pc.gbase = 0;
    return pc;
}

void tic(slam_pf* h, int k) {
    if (!h->timing) return;
    Timer& t = h->tm;
    if (t.used[k] == t.ev[k].size()) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        t.ev[k].push_back({a, b});
    }
    (void)hipEventRecord(t.ev[k][t.used[k]].first, h->stream);
}

void toc(slam_pf* h, int k) {
    if (!h->timing) return;
    Timer& t = h->tm;
    (void)hipEventRecord(t.ev[k][t.used[k]].second, h->stream);
    t.used[k]++;
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// Launch the exact-cumsum + search passes.  force=1: run regardless of the
// device resample flag (stage/test entry points).
int launch_resample(slam_pf* h, double u, int32_t force) {
    const int64_t n = h->n;
    const int nb = h->nb_scan;
    hipStream_t s = h->stream;
    const double delta = 4.0 * (double)n * 0x1p-53 + 0x1p-45;
    tic(h, 2);
    scan_bsum_kernel<<<nb, kScanThreads, 0, s>>>(h->w, n, h->bsum, h->boff, 0.0, h->counters + 2,
                                                 h->flags, force);
    scan_classify_kernel<<<nb, kScanThreads, 0, s>>>(h->w, n, h->boff, h->c, h->kincl, h->fexcl,
                                                     h->bk, h->bf, h->boffk, h->bofff, h->ktot,
                                                     h->nspec, delta, 0, h->counters + 2, h->flags,
                                                     force);
    scan_emit_kernel<<<nb, kScanThreads, 0, s>>>(h->w, n, h->c, h->kincl, h->fexcl, h->boffk,
                                                 h->bofff, h->spec_in, 0, h->spec_out, h->nspec,
                                                 h->ktot, 1, h->c, h->counters + 2, h->flags,
                                                 force);
    scan_expand_kernel<<<nb, kScanThreads, 0, s>>>(n, h->kincl, h->fexcl, h->boffk, h->bofff,
                                                   h->spec_out, h->c, h->flags, force);
    const double step = 1.0 / (double)n;                      // particle_filter.py:213
    const double ofs = std::isnan(u) ? u : u * (1.0 / (double)n);   // :214
    resample_search_kernel<<<grid_for(n, 256), 256, 0, s>>>(n, h->c, h->idx, step, ofs,
                                                           1.0 / (double)n, h->cfg.seed,
                                                           h->stepno, h->flags, force);
    toc(h, 2);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int launch_fused(slam_pf* h, const PredictConst& pc, const double* z_dev, bool host_noise) {
    const int64_t n = h->n;
    const int src = h->cur, dst = 1 - h->cur;
    hipStream_t s = h->stream;
    const unsigned g = grid_for(n, 256);
    const int mot = h->cfg.motion, lik = h->cfg.likelihood;
    tic(h, 0);
#define SLAM_FUSED(M, L, HN)                                                                     \
    pf_fused_kernel<M, L, HN><<<g, 256, 0, s>>>(n, h->x[src], h->y[src], h->th[src], h->x[dst], \
                                                h->y[dst], h->th[dst], h->w, h->w_un, h->idx,    \
                                                h->flags, h->noise, h->lm, z_dev, pc, h->lc,     \
                                                h->cfg.seed, h->stepno)
    if (mot == kMotionNone) {
        if (lik == SLAM_LIK_PRODUCT) SLAM_FUSED(2, 0, false); else SLAM_FUSED(2, 1, false);
    } else if (mot == SLAM_MOTION_LINEAR) {
        if (lik == SLAM_LIK_PRODUCT) {
            if (host_noise) SLAM_FUSED(0, 0, true); else SLAM_FUSED(0, 0, false);
        } else {
            if (host_noise) SLAM_FUSED(0, 1, true); else SLAM_FUSED(0, 1, false);
        }
    } else {
        if (lik == SLAM_LIK_PRODUCT) {
            if (host_noise) SLAM_FUSED(1, 0, true); else SLAM_FUSED(1, 0, false);
        } else {
            if (host_noise) SLAM_FUSED(1, 1, true); else SLAM_FUSED(1, 1, false);
        }
    }
#undef SLAM_FUSED
    toc(h, 0);
    h->cur = dst;
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// numpy-order sum + normalise + reductions + result into res_dev[slot]
int launch_reduce(slam_pf* h, const double* w_src, int slot, int32_t resampled_known) {
    const int64_t n = h->n;
    hipStream_t s = h->stream;
    const int c = h->cur;
    tic(h, 1);
    chunk_sum_kernel<<<h->nchunks, 512, 0, s>>>(w_src, n, h->part, h->tail_leaves, h->tail_ops,
                                                 h->n_tail_leaves, h->n_tail_ops, h->counters,
                                                 h->wsum);
    normalize_kernel<<<h->nb_norm, kNormThreads, 0, s>>>(
        n, w_src, h->w, h->wsum, 1.0 / (double)n, h->x[c], h->y[c], h->th[c], h->refp, h->bp,
        h->counters + 1, h->flags, h->cfg.ess_threshold, h->res_dev + slot, resampled_known, 0);
    toc(h, 1);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int ensure_results(slam_pf* h, int32_t cap) {
    if (cap <= h->res_cap) return SLAM_OK;
    if (h->res_dev) (void)hipFree(h->res_dev);
    if (h->res_host) (void)hipHostFree(h->res_host);
    h->res_dev = nullptr;
    h->res_host = nullptr;
    SLAM_HIP_TRY(hipMalloc((void**)&h->res_dev, sizeof(slam_pf_result) * cap));
    SLAM_HIP_TRY(hipHostMalloc((void**)&h->res_host, sizeof(slam_pf_result) * cap));
    h->res_cap = cap;
    return SLAM_OK;
}

int sync_and_status(slam_pf* h, int32_t count, slam_pf_result* out) {
    SLAM_HIP_TRY(hipMemcpyAsync(h->res_host, h->res_dev, sizeof(slam_pf_result) * count,
                                hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    int rc = SLAM_OK;
    for (int i = 0; i < count; ++i) {
        if (out) out[i] = h->res_host[i];
        if (h->res_host[i].status & 1)
            rc = fail(SLAM_ERR_INDEX, "resample position beyond the last cumulative weight "
                                      "(IndexError in particle_filter.py:219); clamped to NP-1");
    }
    h->resample_next = h->res_host[count - 1].resample_next;
    return rc;
}

int set_flag(slam_pf* h, int word, int32_t v) {
    SLAM_HIP_TRY(hipMemcpyAsync(h->flags + word, &v, sizeof(int32_t), hipMemcpyHostToDevice,
                                h->stream));
    return SLAM_OK;
}

}  // namespace

extern "C" {

int slam_pf_create(const slam_pf_config* cfg, int64_t n_particles, int32_t n_landmarks,
                   const double* landmarks, int device, slam_pf** out) {
    SLAM_ARG_CHECK(cfg && out, "slam_pf_create: NULL argument");
    SLAM_ARG_CHECK(n_particles > 0 && n_particles < (int64_t(1) << 31),
                   "slam_pf_create: n_particles must be in [1, 2^31)");
    SLAM_ARG_CHECK(n_landmarks >= 0, "slam_pf_create: n_landmarks < 0");
    SLAM_ARG_CHECK(n_landmarks == 0 || landmarks, "slam_pf_create: landmarks is NULL");
    SLAM_ARG_CHECK(cfg->motion == SLAM_MOTION_LINEAR || cfg->motion == SLAM_MOTION_VELOCITY,
                   "slam_pf_create: bad motion model");
    SLAM_ARG_CHECK(cfg->likelihood == SLAM_LIK_PRODUCT || cfg->likelihood == SLAM_LIK_LOGSUM,
                   "slam_pf_create: bad likelihood mode");
    *out = nullptr;
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev, "slam_pf_create: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    slam_pf* h = new slam_pf();
    h->cfg = *cfg;
    h->device = device;
    h->n = n_particles;
    h->nl = n_landmarks;
    int rc = make_lik_const(h);
    if (rc) {
        delete h;
        return rc;
    }
    const int64_t n = n_particles;
    h->nb_scan = (int32_t)((n + kScanBlock - 1) / kScanBlock);
    h->nchunks = (int32_t)((n + kSumChunk - 1) / kSumChunk);
    h->nb_norm = (int32_t)std::min<int64_t>(kNormBlocksMax, (n + 2 * kNormThreads - 1) / (2 * kNormThreads));
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return fail(SLAM_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
#define A(p, cnt)                                   \
    if ((rc = dalloc(&(p), (size_t)(cnt))) != 0) { \
        slam_pf_destroy(h);                         \
        return rc;                                  \
    }
    for (int k = 0; k < 2; ++k) {
        A(h->x[k], n);
        A(h->y[k], n);
        A(h->th[k], n);
    }
    A(h->w, n);
    A(h->w_un, n);
    A(h->c, n);
    A(h->kincl, n);
    A(h->fexcl, n);
    A(h->idx, n);
    A(h->bsum, h->nb_scan);
    A(h->boff, h->nb_scan);
    A(h->bk, h->nb_scan);
    A(h->boffk, h->nb_scan);
    A(h->bf, h->nb_scan);
    A(h->bofff, h->nb_scan);
    A(h->ktot, 1);
    A(h->nspec, 1);
    A(h->spec_in, n);
    A(h->spec_out, n);
    A(h->part, h->nchunks);
    A(h->bp, h->nb_norm);
    A(h->wsum, 1);
    A(h->refp, 4);
    A(h->flags, kFlagWords);
    A(h->counters, 4);
    A(h->lm, 2 * std::max<int32_t>(n_landmarks, 1));
    A(h->z, 2 * std::max<int32_t>(n_landmarks, 1));
    A(h->noise, 3 * n);
#undef A
    // tail program for the last np.sum buffer
    std::vector<int32_t> leaves, ops;
    const int tail = (int)(n % kSumChunk);
    if (tail) build_tail(0, tail, leaves, ops);
    h->n_tail_leaves = (int32_t)(leaves.size() / 2);
    h->n_tail_ops = (int32_t)ops.size();
    if ((rc = dalloc(&h->tail_leaves, leaves.size() + 2)) || (rc = dalloc(&h->tail_ops, ops.size() + 1))) {
        slam_pf_destroy(h);
        return rc;
    }
    if (tail) {
        SLAM_HIP_TRY(hipMemcpy(h->tail_leaves, leaves.data(), leaves.size() * 4, hipMemcpyHostToDevice));
        SLAM_HIP_TRY(hipMemcpy(h->tail_ops, ops.data(), ops.size() * 4, hipMemcpyHostToDevice));
    }
    if ((rc = ensure_results(h, 1))) {
        slam_pf_destroy(h);
        return rc;
    }
    // initial state: particle_filter.py:81-84
    std::vector<double> tmp((size_t)n);
    for (int k = 0; k < 3; ++k) {
        std::fill(tmp.begin(), tmp.end(), cfg->x0[k]);
        double* d = (k == 0) ? h->x[0] : (k == 1) ? h->y[0] : h->th[0];
        SLAM_HIP_TRY(hipMemcpy(d, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice));
    }
    std::fill(tmp.begin(), tmp.end(), 1.0 / (double)n);
    SLAM_HIP_TRY(hipMemcpy(h->w, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice));
    SLAM_HIP_TRY(hipMemcpy(h->refp, cfg->x0, 3 * sizeof(double), hipMemcpyHostToDevice));
    SLAM_HIP_TRY(hipMemset(h->flags, 0, kFlagWords * sizeof(int32_t)));
    SLAM_HIP_TRY(hipMemset(h->counters, 0, 4 * sizeof(unsigned)));
    if (n_landmarks > 0)
        SLAM_HIP_TRY(hipMemcpy(h->lm, landmarks, 2 * n_landmarks * sizeof(double), hipMemcpyHostToDevice));
    *out = h;
    return SLAM_OK;
}

int slam_pf_destroy(slam_pf* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    void* ptrs[] = {h->x[0], h->x[1], h->y[0], h->y[1], h->th[0], h->th[1], h->w, h->w_un,
                    h->c, h->kincl, h->fexcl, h->idx, h->bsum, h->boff, h->bk, h->boffk,
                    h->bf, h->bofff, h->ktot, h->nspec, h->spec_in, h->spec_out, h->part,
                    h->tail_leaves, h->tail_ops, h->bp, h->wsum, h->refp, h->flags, h->counters, h->lm,
                    h->z, h->noise, h->z_all, h->res_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (h->res_host) (void)hipHostFree(h->res_host);
    for (int k = 0; k < 4; ++k)
        for (auto& pr : h->tm.ev[k]) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_pf_set_landmarks(slam_pf* h, const double* landmarks) {
    SLAM_ARG_CHECK(h && (landmarks || h->nl == 0), "slam_pf_set_landmarks: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (h->nl)
        SLAM_HIP_TRY(hipMemcpyAsync(h->lm, landmarks, 2 * h->nl * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_set_state(slam_pf* h, const double* x, const double* y, const double* th,
                      const double* w) {
    SLAM_ARG_CHECK(h, "slam_pf_set_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const size_t b = h->n * sizeof(double);
    const int c = h->cur;
    if (x) SLAM_HIP_TRY(hipMemcpyAsync(h->x[c], x, b, hipMemcpyHostToDevice, h->stream));
    if (y) SLAM_HIP_TRY(hipMemcpyAsync(h->y[c], y, b, hipMemcpyHostToDevice, h->stream));
    if (th) SLAM_HIP_TRY(hipMemcpyAsync(h->th[c], th, b, hipMemcpyHostToDevice, h->stream));
    if (w) {
        SLAM_HIP_TRY(hipMemcpyAsync(h->w, w, b, hipMemcpyHostToDevice, h->stream));
        // particle_filter.py:210-211: recompute the resample decision from these weights
        double s2 = 0.0;
        for (int64_t i = 0; i < h->n; ++i) s2 += w[i] * w[i];
        h->resample_next = (1.0 / s2 < h->cfg.ess_threshold) ? 1 : 0;
        int rc = set_flag(h, kFlagResample, h->resample_next);
        if (rc) return rc;
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_get_state(slam_pf* h, double* x, double* y, double* th, double* w) {
    SLAM_ARG_CHECK(h, "slam_pf_get_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const size_t b = h->n * sizeof(double);
    const int c = h->cur;
    if (x) SLAM_HIP_TRY(hipMemcpyAsync(x, h->x[c], b, hipMemcpyDeviceToHost, h->stream));
    if (y) SLAM_HIP_TRY(hipMemcpyAsync(y, h->y[c], b, hipMemcpyDeviceToHost, h->stream));
    if (th) SLAM_HIP_TRY(hipMemcpyAsync(th, h->th[c], b, hipMemcpyDeviceToHost, h->stream));
    if (w) SLAM_HIP_TRY(hipMemcpyAsync(w, h->w, b, hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_step(slam_pf* h, const double* control, const double* z, const double* noise,
                 double u_resample, slam_pf_result* res) {
    SLAM_ARG_CHECK(h && control && (z || h->nl == 0), "slam_pf_step: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = ensure_results(h, 1))) return rc;
    tic(h, 3);
    if (h->nl)
        SLAM_HIP_TRY(hipMemcpyAsync(h->z, z, 2 * h->nl * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    if (noise)
        SLAM_HIP_TRY(hipMemcpyAsync(h->noise, noise, 3 * h->n * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    const int32_t resampling = h->resample_next;
    if (resampling && (rc = launch_resample(h, u_resample, 0))) return rc;
    PredictConst pc = make_predict_const(h, control);
    if ((rc = launch_fused(h, pc, h->z, noise != nullptr))) return rc;
    if ((rc = launch_reduce(h, h->w_un, 0, resampling))) return rc;
    toc(h, 3);
    h->stepno++;
    return sync_and_status(h, 1, res);
}

int slam_pf_resample(slam_pf* h, double u_resample, int32_t force, int32_t* resampled) {
    SLAM_ARG_CHECK(h, "slam_pf_resample: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const int32_t go = force ? 1 : h->resample_next;
    if (resampled) *resampled = go;
    if (!go) return SLAM_OK;
    int rc = launch_resample(h, u_resample, 1);
    if (rc) return rc;
    const int src = h->cur, dst = 1 - h->cur;
    gather_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(
        h->n, h->idx, h->x[src], h->y[src], h->th[src], h->x[dst], h->y[dst], h->th[dst], h->w,
        1.0 / (double)h->n);
    SLAM_HIP_TRY(hipGetLastError());
    h->cur = dst;
    int32_t st = 0;
    SLAM_HIP_TRY(hipMemcpyAsync(&st, h->flags + kFlagStatus, 4, hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    h->resample_next = 0;
    if ((rc = set_flag(h, kFlagResample, 0)) || (rc = set_flag(h, kFlagStatus, 0))) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    if (st & 1)
        return fail(SLAM_ERR_INDEX, "resample position beyond the last cumulative weight "
                                    "(IndexError in particle_filter.py:219)");
    return SLAM_OK;
}

int slam_pf_resample_indices(slam_pf* h, double u_resample, int64_t* idx_out, int32_t* n_special) {
    SLAM_ARG_CHECK(h && idx_out, "slam_pf_resample_indices: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = launch_resample(h, u_resample, 1);
    if (rc) return rc;
    std::vector<int32_t> idx((size_t)h->n);
    int32_t fl[kFlagWords];
    SLAM_HIP_TRY(hipMemcpyAsync(idx.data(), h->idx, h->n * 4, hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(fl, h->flags, sizeof(fl), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->n; ++i) idx_out[i] = idx[i];
    if (n_special) *n_special = fl[kFlagNSpecial];
    if ((rc = set_flag(h, kFlagStatus, 0))) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    if (fl[kFlagStatus] & 1)
        return fail(SLAM_ERR_INDEX, "resample position beyond the last cumulative weight "
                                    "(IndexError in particle_filter.py:219)");
    return SLAM_OK;
}

int slam_pf_predict(slam_pf* h, const double* control, const double* noise) {
    SLAM_ARG_CHECK(h && control, "slam_pf_predict: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    // predict-only = fused kernel with zero landmarks and no resample gather;
    // weights are carried through unchanged (w_un = w * 1).
    if (noise)
        SLAM_HIP_TRY(hipMemcpyAsync(h->noise, noise, 3 * h->n * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    int rc = set_flag(h, kFlagResample, 0);
    if (rc) return rc;
    const int32_t nl = h->lc.nl;
    h->lc.nl = 0;
    PredictConst pc = make_predict_const(h, control);
    rc = launch_fused(h, pc, h->z, noise != nullptr);
    h->lc.nl = nl;
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemcpyAsync(h->w, h->w_un, h->n * 8, hipMemcpyDeviceToDevice, h->stream));
    if ((rc = set_flag(h, kFlagResample, h->resample_next))) return rc;
    h->stepno++;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_update(slam_pf* h, const double* z, slam_pf_result* res) {
    // __likelihood + estimate on the current particles (no motion, no resample)
    SLAM_ARG_CHECK(h && (z || h->nl == 0), "slam_pf_update: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = ensure_results(h, 1))) return rc;
    if (h->nl)
        SLAM_HIP_TRY(hipMemcpyAsync(h->z, z, 2 * h->nl * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    if ((rc = set_flag(h, kFlagResample, 0))) return rc;
    const int32_t saved = h->cfg.motion;
    h->cfg.motion = kMotionNone;
    const double ctl[2] = {0.0, 0.0};
    PredictConst pc = make_predict_const(h, ctl);
    rc = launch_fused(h, pc, h->z, false);
    h->cfg.motion = saved;
    if (rc) return rc;
    if ((rc = launch_reduce(h, h->w_un, 0, 0))) return rc;
    return sync_and_status(h, 1, res);
}

int slam_pf_weight_sum(slam_pf* h, double* sum_out) {
    SLAM_ARG_CHECK(h && sum_out, "slam_pf_weight_sum: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    chunk_sum_kernel<<<h->nchunks, 512, 0, h->stream>>>(h->w, h->n, h->part, h->tail_leaves,
                                                         h->tail_ops, h->n_tail_leaves,
                                                         h->n_tail_ops, h->counters, nullptr);
    SLAM_HIP_TRY(hipGetLastError());
    std::vector<double> p((size_t)h->nchunks);
    SLAM_HIP_TRY(hipMemcpyAsync(p.data(), h->part, h->nchunks * 8, hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    double s = 0.0;
    for (double v : p) s = s + v;
    *sum_out = s;
    return SLAM_OK;
}

int slam_pf_load_observations(slam_pf* h, int32_t n_steps, const double* z_all) {
    SLAM_ARG_CHECK(h && n_steps > 0 && (z_all || h->nl == 0), "slam_pf_load_observations: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (h->z_all) (void)hipFree(h->z_all);
    h->z_all = nullptr;
    const size_t cnt = (size_t)n_steps * 2 * std::max<int32_t>(h->nl, 1);
    SLAM_HIP_TRY(hipMalloc((void**)&h->z_all, cnt * sizeof(double)));
    if (h->nl)
        SLAM_HIP_TRY(hipMemcpy(h->z_all, z_all, (size_t)n_steps * 2 * h->nl * sizeof(double),
                               hipMemcpyHostToDevice));
    h->z_steps = n_steps;
    return SLAM_OK;
}

int slam_pf_run(slam_pf* h, int32_t first_step, int32_t n_steps, const double* controls,
                slam_pf_result* results) {
    SLAM_ARG_CHECK(h && controls && n_steps > 0, "slam_pf_run: bad argument");
    SLAM_ARG_CHECK(first_step >= 0 && first_step + n_steps <= h->z_steps,
                   "slam_pf_run: steps outside the loaded observations");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = ensure_results(h, n_steps))) return rc;
    // device-decided resampling: every pass is launched and gates on the flag
    if ((rc = set_flag(h, kFlagResample, h->resample_next))) return rc;
    for (int32_t k = 0; k < n_steps; ++k) {
        tic(h, 3);
        if ((rc = launch_resample(h, std::numeric_limits<double>::quiet_NaN(), 0))) return rc;
        PredictConst pc = make_predict_const(h, controls + 2 * k);
        const double* zk = h->z_all + (size_t)(first_step + k) * 2 * std::max<int32_t>(h->nl, 1);
        if ((rc = launch_fused(h, pc, zk, false))) return rc;
        if ((rc = launch_reduce(h, h->w_un, k, -1))) return rc;
        toc(h, 3);
        h->stepno++;
    }
    return sync_and_status(h, n_steps, results);
}

int slam_pf_enable_timing(slam_pf* h, int32_t on) {
    SLAM_ARG_CHECK(h, "slam_pf_enable_timing: NULL handle");
    h->timing = on != 0;
    for (int k = 0; k < 4; ++k) h->tm.used[k] = 0;
    return SLAM_OK;
}

int slam_pf_timing(slam_pf* h, int32_t kernel, double* total_ms, int64_t* launches) {
    SLAM_ARG_CHECK(h && kernel >= 0 && kernel < 4 && total_ms && launches, "slam_pf_timing: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    double tot = 0.0;
    for (size_t i = 0; i < h->tm.used[kernel]; ++i) {
        float ms = 0.f;
        SLAM_HIP_TRY(hipEventElapsedTime(&ms, h->tm.ev[kernel][i].first, h->tm.ev[kernel][i].second));
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int64_t)h->tm.used[kernel];
    return SLAM_OK;
}

}  // extern "C"
