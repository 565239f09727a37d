// pf_api.hip -- C-ABI of the particle filter (include/slam_hip.h).
//
// Replaces ParticleFilter (particle_filter.py:18-237).  One handle = one GPU
// (or one shard of a multi-GPU filter), one HIP stream, SoA particle state
// resident in HBM.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "comm.hpp"
#include "mt_stream.hpp"
#include "pf_kernels.inl"
#include "pf_dist.inl"

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

constexpr int kGraphLevels = 4;    // captured step graphs of 1, 2, 4 and 8 steps
constexpr int kGraphSteps = 1 << (kGraphLevels - 1);
constexpr int32_t kSetupCopyMax = 4096;   // batch controls the setup kernel copies itself

struct Timer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[4];
    size_t used[4] = {0, 0, 0, 0};
};

}  // namespace slam

using namespace slam;

struct slam_pf {
    slam_pf_config cfg;
    int device = 0;
    int64_t n = 0;            // local particles
    int64_t n_global = 0;     // particles of the whole filter
    int64_t gbase = 0;        // global index of local particle 0
    int32_t nl = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    std::vector<void*> allocs;
    // state (ping-pong)
    double* x[2] = {nullptr, nullptr};
    double* y[2] = {nullptr, nullptr};
    double* th[2] = {nullptr, nullptr};
    int cur = 0;
    double *w = nullptr, *w_un = nullptr;
    // exact cumsum scratch
    double* c = nullptr;
    uint64_t* kincl = nullptr;
    int32_t* fexcl = nullptr;
    int32_t* idx = nullptr;
    int32_t nb_scan = 0;
    double *bsum = nullptr, *boff = nullptr;
    uint64_t *bk = nullptr, *boffk = nullptr, *ktot = nullptr;
    int32_t *bf = nullptr, *bofff = nullptr, *nspec = nullptr;
    SpecialIn* spec_in = nullptr;
    SpecialIn* stage = nullptr;     // lean exact cumsum: per-tile staged specials
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
    unsigned* tk = nullptr;         // ticket blocks: +0 np.sum, +1 normalize, +2 scans (x kTicketWords)
    // inputs / step context
    double* lm = nullptr;
    double* noise = nullptr;
    int32_t cap = 0;                // steps the StepIO arrays hold
    double* ctl = nullptr;
    double* z_all = nullptr;
    double* zc = nullptr;                 // [cap][kZcWords] closed-form words (device-formed per step)
    double* ofs = nullptr;
    slam_pf_result* res_dev = nullptr;
    slam_pf_result* res_host = nullptr;   // pinned, coherent: the export kernel stores into it
    double* ctl_pin = nullptr;            // pinned, coherent staging of a batch's controls
    slam_pf_result* res_host_dev = nullptr;   // the two pinned buffers' device addresses
    double* ctl_pin_dev = nullptr;
    int32_t* ctr = nullptr;               // [0] step in batch, [1] RNG step
    int32_t z_steps = 0;
    LikConst lc;
    PredictConst pc;
    uint32_t stepno = 0;                  // host mirror of ctr[1]
    int32_t resample_next = 0;            // host mirror of the device flag
    bool timing = false;
    bool use_graph = true;
    hipGraphExec_t graph[kGraphLevels][2] = {};   // [log2 steps][ping-pong parity]
    Timer tm;
    double ofs_host = 0.0;          // pinned-free staging of one step's resample offset
    // deferred normalisation (single-GPU handles): current weights = w_un / s_cur
    bool deferred = false;
    bool scan_merged = false;   // exact cumsum in one launch (co-resident grid)
    bool scan_merged_ok = false;  // the merged launch is allowed for this handle
    double* s_cur = nullptr;
    DeferParts dp{};
    FinSlices fsl{};                      // NP > 2^20: the finalize's slice pre-pass (pf_finalize.inl)
    int32_t nb_part = 0;
    // NumPy's RandomState stream on the device (slam_pf_set_rng_mt19937)
    bool mt = false;
    MtBuffers mtb;
    double mr[4] = {0, 0, 0, 0};         // svd factor of R (mvn of the observation noise)
    double* truth = nullptr;             // [cap][4] true pose (x, y, cos, sin) per step
    int32_t truth_steps = 0;
    const double* noise_src = nullptr;   // fused kernel's host-noise input (default h->noise)
    double ess_band = 1e-9;              // result.ess_near band (relative to ESS_TH)
    // the closed-form words of step prep_step were formed by the previous
    // batch's last step end for the control prep_ctl (the setup kernel wrote
    // it as the guess for the next batch's first step); -1: none.  Any call
    // that can change the observations, landmarks or controls clears it.
    int32_t prep_step = -1;
    double prep_ctl[2] = {0.0, 0.0};
};

namespace {

int halloc(slam_pf* h, void** p, size_t bytes) {
    if (bytes == 0) bytes = 8;
    SLAM_HIP_TRY(hipMalloc(p, bytes));
    h->allocs.push_back(*p);
    return SLAM_OK;
}

template <typename T>
int dalloc(slam_pf* h, T** p, size_t count) {
    return halloc(h, (void**)p, count * sizeof(T));
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
    // closed-form log-sum (iso, NL > 0); SLAM_PF_CLOSED=0 keeps the landmark loop (diagnostic)
    const char* ce = std::getenv("SLAM_PF_CLOSED");
    lc.closed = (lc.iso && h->nl > 0 && !(ce && ce[0] == '0')) ? 1 : 0;
    // Log-sum fast-path bound.  A factor is at most 1/den (q >= 0), so the log of
    // the reference's partial product after landmark k is at least
    // L - (NL - k) max(0, -ln den).  L >= ln(DBL_MIN) + NL max(0, -ln den) + 1
    // keeps every partial product of particle_filter.py:192 in the normal range
    // (the 1-nat margin covers the rounding of both sums); below it the kernel
    // takes the reference's sequential product.  Past NL max(0, -ln den) = 700
    // the products may overflow: always the sequential product.
    const double climb = (double)h->nl * std::max(0.0, -std::log(lc.den));
    lc.normal_min_l = std::log(std::numeric_limits<double>::min()) + 1.0;
    lc.neg_ln_den = -std::log(lc.den);
    lc.fast_min_l = climb > 700.0 ? std::numeric_limits<double>::infinity()
                                  : lc.normal_min_l + climb;
    // closed form: the fp64 expansion while its rounding bound 11 u V stays
    // within |dL| <= 3e-13 (dL = dF / (2 sx2), under a third of the 1e-12
    // parity bar): V rsx2 <= 480; SLAM_PF_EXPAND_VMAX=<factor>
    // scales the bound (0: double-double only)
    const char* ve = std::getenv("SLAM_PF_EXPAND_VMAX");
    const double vf = ve ? std::atof(ve) : 1.0;
    lc.expand_vmax = vf * 480.0 * lc.sx2;
    return SLAM_OK;
}

void make_predict_const(slam_pf* h) {
    PredictConst& pc = h->pc;
    const slam_pf_config& c = h->cfg;
    pc.dt = c.dt;
    for (int k = 0; k < 6; ++k) pc.alphas[k] = c.alphas[k];
    for (int k = 0; k < 9; ++k) pc.q[k] = c.q_factor[k];
    pc.np_recip = 1.0 / (double)h->n_global;             // particle_filter.py:32
    pc.rstep = 1.0 / (double)h->n_global;                // :213 arange step (= NP_RECIP)
    pc.n_global = h->n_global;
    pc.gbase = h->gbase;
}

StepIO step_io(slam_pf* h) {
    StepIO io;
    io.ctl = h->ctl;
    io.z = h->z_all;
    io.zc = h->zc;
    io.ofs = h->ofs;
    io.res = h->res_dev;
    io.res_host = h->res_host_dev;
    io.ctr = h->ctr;
    io.cap = h->cap;
    io.motion = h->cfg.motion;
    io.ess_band = h->ess_band;
    return io;
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

void drop_graphs(slam_pf* h) {
    for (auto& gs : h->graph)
        for (auto& g : gs)
            if (g) {
                (void)hipGraphExecDestroy(g);
                g = nullptr;
            }
}

int launch_step(slam_pf* h, bool host_noise);

// One captured hipGraph of `steps` device-resident steps (slam_pf_run) for the
// handle's current ping-pong parity; the step context lives in device memory,
// so a replay needs no host input.  There is one graph per parity for each of
// 1, 2, 4 and 8 steps: a batch replays its binary decomposition, largest first
// (the even ones bring the parity back).
int capture_steps(slam_pf* h, hipGraphExec_t& ge, int steps) {
    const int cur0 = h->cur;
    // no timing events inside a graph: launch_step's tic / toc
    // would record events that never run on the stream
    const bool timing0 = h->timing;
    h->timing = false;
    hipGraph_t g;
    SLAM_HIP_TRY(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    int rc = SLAM_OK;
    for (int k = 0; k < steps && rc == SLAM_OK; ++k) rc = launch_step(h, false);
    const hipError_t e = hipStreamEndCapture(h->stream, &g);
    h->cur = cur0;
    h->timing = timing0;
    if (rc) return rc;
    if (e != hipSuccess) return fail(SLAM_ERR_HIP, "hipStreamEndCapture failed");
    SLAM_HIP_TRY(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    SLAM_HIP_TRY(hipGraphUpload(ge, h->stream));     // the first replay pays no upload
    return SLAM_OK;
}

void release(slam_pf* h, void* p) {
    if (!p) return;
    (void)hipFree(p);
    h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), p), h->allocs.end());
}

// (Re)allocate the StepIO arrays for `steps` steps.
int ensure_steps(slam_pf* h, int32_t steps) {
    if (steps <= h->cap) return SLAM_OK;
    drop_graphs(h);
    release(h, h->ctl);
    release(h, h->z_all);
    release(h, h->zc);
    release(h, h->ofs);
    release(h, h->truth);
    release(h, h->res_dev);
    if (h->res_host) (void)hipHostFree(h->res_host);
    h->res_host = nullptr;
    if (h->ctl_pin) (void)hipHostFree(h->ctl_pin);
    h->ctl_pin = nullptr;
    int rc;
    const size_t nlz = 2 * (size_t)std::max<int32_t>(h->nl, 1);
    if ((rc = dalloc(h, &h->ctl, 2 * (size_t)steps)) || (rc = dalloc(h, &h->z_all, nlz * steps)) ||
        (rc = dalloc(h, &h->zc, (size_t)kClosedWords * steps)) ||
        (rc = dalloc(h, &h->ofs, (size_t)steps)) || (rc = dalloc(h, &h->truth, 4 * (size_t)steps)) ||
        (rc = dalloc(h, &h->res_dev, (size_t)steps)))
        return rc;
    // fine-grained host memory: the setup kernel reads the controls and the
    // export kernel stores the results over the host link, uncached
    SLAM_HIP_TRY(hipHostMalloc((void**)&h->res_host, sizeof(slam_pf_result) * steps,
                               hipHostMallocMapped | hipHostMallocCoherent));
    SLAM_HIP_TRY(hipHostMalloc((void**)&h->ctl_pin, 2 * sizeof(double) * steps,
                               hipHostMallocMapped | hipHostMallocCoherent));
    SLAM_HIP_TRY(hipHostGetDevicePointer((void**)&h->res_host_dev, h->res_host, 0));
    SLAM_HIP_TRY(hipHostGetDevicePointer((void**)&h->ctl_pin_dev, h->ctl_pin, 0));
    h->cap = steps;
    h->z_steps = 0;
    h->truth_steps = 0;
    return SLAM_OK;
}

// Device words set by memset nodes (the value travels in the call; no host
// buffer, so the host does not wait as for a pageable copy)
int set_ctr(slam_pf* h, int32_t step) {
    SLAM_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)h->ctr, step, 1, h->stream));
    SLAM_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(h->ctr + 1), (int)h->stepno, 1, h->stream));
    // no batch bounds: the step end's export of a batch's records (ctr[2..3],
    // written by slam_pf_run's setup) must not fire for this step
    SLAM_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(h->ctr + 2), -1, 2, h->stream));
    return SLAM_OK;
}

int set_flag(slam_pf* h, int word, int32_t v) {
    SLAM_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(h->flags + word), v, 1, h->stream));
    return SLAM_OK;
}

// S1 stand-alone: 256-block totals of w and their prefix (normalize_kernel
// leaves the same arrays behind whenever the next step resamples).
int launch_bsum(slam_pf* h) {
    if (h->deferred)
        scan_bsum256_kernel<<<h->nb_part, kPartPer, 0, h->stream>>>(
            h->w_un, h->s_cur, h->pc.np_recip, h->n, h->bsum, h->boff, h->tk + 2 * kTicketWords);
    else
        scan_bsum_kernel<<<h->nb_norm, kNormThreads, 0, h->stream>>>(h->w, h->n, h->bsum, h->boff,
                                                                      h->tk + 2 * kTicketWords);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// Exact-cumsum passes S3..S7 (S1 with with_s1).  force=0: they gate on the
// device resample flag.
int launch_scans(slam_pf* h, int32_t force, bool with_s1) {
    const int64_t n = h->n;
    const int nb = h->nb_scan;
    hipStream_t s = h->stream;
    const double delta = 4.0 * (double)h->n_global * 0x1p-53 + 0x1p-45;
    if (with_s1) {
        const int rc = launch_bsum(h);
        if (rc) return rc;
    }
    if (h->deferred && h->scan_merged) {
        unsigned* tk = h->tk + 2 * kTicketWords;
        scan_lean_merged_kernel<<<nb, kScanThreads, 0, s>>>(
            h->w_un, h->s_cur, h->pc.np_recip, n, h->boff, delta, h->stage, h->bk, h->bf, h->boffk,
            h->bofff, h->ktot, h->nspec, tk, h->flags, force, h->spec_out, h->c, step_io(h), h->pc,
            h->cfg.seed, h->dp.mark, h->dp.carry, h->flags + kFlagScanToken, h->nb_part);
        SLAM_HIP_TRY(hipGetLastError());
        return SLAM_OK;
    }
    if (h->deferred) {
        unsigned* tk = h->tk + 2 * kTicketWords;
        scan_lean_classify_kernel<<<nb, kScanThreads, 0, s>>>(
            h->w_un, h->s_cur, h->pc.np_recip, n, h->boff, delta, h->stage, h->bk, h->bf, h->boffk,
            h->bofff, h->ktot, h->nspec, tk, h->flags, force, h->spec_out, h->c, h->nb_part);
        scan_lean_expand_kernel<<<nb, kScanThreads, 0, s>>>(
            h->w_un, h->s_cur, h->pc.np_recip, n, h->boff, delta, h->boffk, h->bofff, h->spec_out,
            h->c, h->flags, force, step_io(h), h->pc, h->cfg.seed, h->dp.mark,
            h->dp.carry, h->nb_part);
        SLAM_HIP_TRY(hipGetLastError());
        return SLAM_OK;
    }
    const double* w = h->deferred ? h->w_un : h->w;
    const double* sd = h->deferred ? h->s_cur : nullptr;
    const int32_t gran = h->deferred ? kPartPer : kNormPer;
    scan_classify_kernel<<<nb, kScanThreads, 0, s>>>(
        w, n, h->boff, nullptr, h->c, h->kincl, h->fexcl, h->bk, h->bf, h->boffk, h->bofff,
        h->ktot, h->nspec, delta, 0, h->tk + 2 * kTicketWords, h->flags, force, sd,
        h->pc.np_recip, gran);
    scan_emit_kernel<<<nb, kScanThreads, 0, s>>>(w, n, h->c, h->kincl, h->fexcl, h->boffk,
                                                 h->bofff, h->spec_in, 0, h->spec_out, h->nspec,
                                                 h->ktot, 1, h->c, h->tk + 2 * kTicketWords, h->flags,
                                                 force, sd, h->pc.np_recip);
    scan_expand_kernel<<<nb, kScanThreads, 0, s>>>(n, h->kincl, h->fexcl, h->boffk, h->bofff,
                                                   h->spec_out, h->c, h->flags, nullptr,
                                                   nullptr, force);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int launch_fused(slam_pf* h, int motion, bool host_noise) {
    const int64_t n = h->n;
    const int src = h->cur, dst = 1 - h->cur;
    hipStream_t s = h->stream;
    const unsigned g = h->deferred ? (unsigned)h->nb_part : grid_for(n, 256);
    const int lik = h->cfg.likelihood;
    const StepIO io = step_io(h);
    tic(h, 0);
    const double* w_in = h->deferred ? nullptr : h->w;     // deferred: read from w_un
    const double* nsrc = h->noise_src ? h->noise_src : h->noise;
#define SLAM_FUSED_D(M, L, HN, D)                                                                \
    pf_fused_kernel<M, L, HN, D><<<g, 256, 0, s>>>(n, h->x[src], h->y[src], h->th[src],         \
                                                   h->x[dst], h->y[dst], h->th[dst], w_in,      \
                                                   h->w_un, h->c, h->flags, nsrc, h->lm, io,     \
                                                   h->pc, h->lc, h->cfg.seed, h->s_cur, h->refp, \
                                                   h->dp)
#define SLAM_FUSED(M, L, HN) SLAM_FUSED_D(M, L, HN, true)     /* every handle is deferred */
    if (motion == kMotionNone) {
        if (lik == SLAM_LIK_PRODUCT) SLAM_FUSED(2, 0, false); else SLAM_FUSED(2, 1, false);
    } else if (motion == SLAM_MOTION_LINEAR) {
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
#undef SLAM_FUSED_D
    toc(h, 0);
    h->cur = dst;
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// numpy-order sum + normalise + reductions + result record res[ctr[0]]
int launch_reduce(slam_pf* h, int32_t resampled_known) {
    const int64_t n = h->n;
    hipStream_t s = h->stream;
    const int c = h->cur;
    tic(h, 1);
    if (h->deferred) {
        const bool sliced = h->fsl.nsl > 1;
        if (!sliced || (h->fsl.nsl <= kFinFastSlices && n / kSumChunk <= 2048)) {
            if (sliced)
                finalize_slices_kernel<<<h->fsl.nsl - 1, kFinThreads, 0, s>>>(n, h->dp, h->fsl);
            auto kern = sliced ? finalize_fast_kernel<true> : finalize_fast_kernel<false>;
            kern<<<1, kFinThreads, 0, s>>>(
                n, h->dp, h->w_un, h->s_cur, h->tail_leaves, h->tail_ops, h->n_tail_leaves,
                h->n_tail_ops, h->x[c], h->y[c], h->th[c], h->refp, h->flags, h->cfg.ess_threshold,
                step_io(h), resampled_known, h->pc.np_recip, h->boff, h->fsl);
            toc(h, 1);
            SLAM_HIP_TRY(hipGetLastError());
            return SLAM_OK;
        }
        if (h->fsl.nsl > 1)
            finalize_slices_kernel<<<h->fsl.nsl - 1, kFinThreads, 0, s>>>(n, h->dp, h->fsl);
        finalize_deferred_kernel<<<1, kFinThreads, 0, s>>>(
            n, h->dp, h->w_un, h->s_cur, h->tail_leaves, h->tail_ops, h->n_tail_leaves,
            h->n_tail_ops, h->x[c], h->y[c], h->th[c], h->refp, h->flags, h->cfg.ess_threshold,
            step_io(h), resampled_known, h->pc.np_recip, h->boff, h->fsl);
        toc(h, 1);
        SLAM_HIP_TRY(hipGetLastError());
        return SLAM_OK;
    }
    chunk_sum_kernel<<<h->nchunks, 512, 0, s>>>(h->w_un, n, h->part, h->tail_leaves, h->tail_ops,
                                                 h->n_tail_leaves, h->n_tail_ops, h->tk,
                                                 h->wsum);
    normalize_kernel<<<h->nb_norm, kNormThreads, 0, s>>>(n, h->w_un, h->w, h->wsum,
                                                          h->pc.np_recip, h->x[c], h->y[c],
                                                          h->th[c], h->refp, h->bp, h->bsum, 0);
    finalize_kernel<<<1, 1024, 0, s>>>(h->bp, h->nb_norm, h->bsum, h->boff, h->x[c], h->y[c],
                                        h->th[c], h->refp, h->wsum, h->flags,
                                        h->cfg.ess_threshold, step_io(h), resampled_known, 0);
    toc(h, 1);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// ---- NumPy's stream on the device (slam_pf_set_rng_mt19937)
//
// __observation (particle_filter.py:144-154) of step ctr[0] from the true pose:
// world2robot (mylib/transform.py:31-35: the 2x2 rotation through OpenBLAS's
// fused dgemm) plus the mvn(0, R) noise of normals [n3, n3 + 2 NL) (x @ M,
// dgemm order); then the step's closed-form words (iso handles).
__global__ __launch_bounds__(512) void pf_mt_observe_kernel(
    const double* __restrict__ normals, const int64_t n3, const double* __restrict__ lm,
    const int32_t nl, const double* __restrict__ truth, const int32_t* __restrict__ ctr,
    const double r0, const double r1, const double r2, const double r3, double* __restrict__ z_all,
    double* __restrict__ zc, const int32_t closed, const double* __restrict__ refp,
    const double* __restrict__ ctl, const double dt, const int32_t motion) {
    extern __shared__ double s_z[];
    const int32_t st = ctr[0];
    const double* t = truth + 4 * (size_t)st;
    const double tx = t[0], ty = t[1], c = t[2], s = t[3];
    double* z = z_all + (size_t)st * 2 * nl;
    for (int32_t l = threadIdx.x; l < nl; l += blockDim.x) {
        const double n0 = normals[n3 + 2 * l], n1 = normals[n3 + 2 * l + 1];
        const double w0 = fma(n1, r2, n0 * r0), w1 = fma(n1, r3, n0 * r1);
        const double dx = lm[2 * l] - tx, dy = lm[2 * l + 1] - ty;
        const double zx = fma(-s, dy, c * dx) + w0;
        const double zy = fma(c, dy, s * dx) + w1;
        z[2 * l] = zx;
        z[2 * l + 1] = zy;
        s_z[2 * l] = zx;
        s_z[2 * l + 1] = zy;
        s_z[2 * (nl + l)] = lm[2 * l];          // the sums read both from LDS
        s_z[2 * (nl + l) + 1] = lm[2 * l + 1];
    }
    __syncthreads();
    if (closed)
        closed_prep_block(s_z + 2 * nl, s_z, nl, refp, ctl[2 * st], ctl[2 * st + 1], dt, motion,
                          zc + (size_t)st * kZcWords);
}

// The step ctr[0]'s closed-form words from its loaded observations (sync-mode
// steps and the first step of a device-resident batch; later steps of a batch
// are prepared by the previous step's end).
__global__ __launch_bounds__(512) void pf_prestep_kernel(const double* __restrict__ lm,
                                                         const double* __restrict__ z_all,
                                                         const int32_t nl,
                                                         const int32_t* __restrict__ ctr,
                                                         const double* __restrict__ refp,
                                                         const double* __restrict__ ctl,
                                                         const double dt, const int32_t motion,
                                                         double* __restrict__ zc) {
    const int32_t st = ctr[0];
    closed_prep_block(lm, z_all + (size_t)st * 2 * nl, nl, refp, ctl[2 * st], ctl[2 * st + 1], dt,
                      motion, zc + (size_t)st * kZcWords);
}

int launch_prestep(slam_pf* h) {
    if (!h->lc.closed) return SLAM_OK;
    pf_prestep_kernel<<<1, 512, 0, h->stream>>>(h->lm, h->z_all, h->nl, h->ctr, h->refp, h->ctl,
                                                h->pc.dt, h->cfg.motion, h->zc);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// A device-resident batch's setup in one launch (slam_pf_run): the batch's
// controls read from the coherent pinned staging over the host link (ncopy of
// them; 0 when a copy already moved them), the step counters and the resample
// flag (rflag < 0: left as it is), then -- unless the device observes (NumPy stream) -- the first step's
// closed-form words as pf_prestep_kernel forms them.  One stream operation in
// place of a host-to-device copy, three memsets and the prestep.
__global__ __launch_bounds__(512) void pf_run_setup_kernel(
    const double* __restrict__ ctl_host, const int32_t nsteps, const int32_t ncopy, const int32_t first,
    const int32_t stepno, const int32_t rflag, double* __restrict__ ctl, int32_t* __restrict__ ctr,
    int32_t* __restrict__ flags, double* __restrict__ ctl_next, const int32_t prep,
    const double* __restrict__ lm,
    const double* __restrict__ z_all, const int32_t nl, const double* __restrict__ refp,
    const double dt, const int32_t motion, double* __restrict__ zc) {
    for (int k = (int)threadIdx.x; k < 2 * ncopy; k += (int)blockDim.x)
        ctl[2 * (size_t)first + k] = ctl_host[k];
    // the guess for the next batch's first control (this batch's last): the
    // last step end forms that step's closed-form words with it, and the next
    // setup skips its own forming when the guess was right
    if (ctl_next && threadIdx.x < 2) ctl_next[threadIdx.x] = ctl_host[2 * (nsteps - 1) + threadIdx.x];
    if (threadIdx.x == 0) {
        ctr[0] = first;
        ctr[1] = stepno;
        ctr[2] = first;
        ctr[3] = first + nsteps - 1;
        if (rflag >= 0) flags[kFlagResample] = rflag;
    }
    if (prep)
        closed_prep_block(lm, z_all + (size_t)first * 2 * nl, nl, refp, ctl_host[0], ctl_host[1], dt,
                          motion, zc + (size_t)first * kZcWords);
}

int launch_run_setup(slam_pf* h, int32_t first_step, int32_t n_steps, const double* controls,
                     int32_t rflag, int32_t* prep_next = nullptr) {
    std::memcpy(h->ctl_pin, controls, 2 * (size_t)n_steps * sizeof(double));
    // the first step's words: already formed by the previous batch's last
    // step end when it continued this one with the same control
    const bool formed = h->prep_step == first_step && h->prep_ctl[0] == controls[0] &&
                        h->prep_ctl[1] == controls[1];
    const int32_t next = first_step + n_steps;
    const bool guess = prep_next && h->deferred && !h->mt && h->lc.closed && next < h->cap;
    h->prep_step = -1;                      // (re)armed by the caller once the batch succeeded
    if (prep_next) *prep_next = guess ? next : -1;
    int32_t ncopy = n_steps;
    if (n_steps > kSetupCopyMax) {                 // long batches: one DMA copy instead
        SLAM_HIP_TRY(hipMemcpyAsync(h->ctl + 2 * first_step, h->ctl_pin,
                                    2 * (size_t)n_steps * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
        ncopy = 0;
    }
    pf_run_setup_kernel<<<1, 512, 0, h->stream>>>(
        h->ctl_pin_dev, n_steps, ncopy, first_step, (int32_t)h->stepno, rflag, h->ctl, h->ctr,
        h->flags, guess ? h->ctl + 2 * (size_t)next : nullptr,
        (!h->mt && h->lc.closed && !formed) ? 1 : 0, h->lm, h->z_all, h->nl, h->refp, h->pc.dt,
        h->cfg.motion, h->zc);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// The batch's result records into the coherent pinned buffer (stores over the
// host link; visible to the host once the stream has synchronised)
__global__ __launch_bounds__(256) void pf_export_kernel(const uint64_t* __restrict__ src,
                                                        const int64_t words,
                                                        uint64_t* __restrict__ dst) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < words; k += 256 * (int64_t)gridDim.x)
        dst[k] = src[k];
}

// mvn(0, Q, NP) (particle_filter.py:165): noise = normals @ M, OpenBLAS's order
__global__ __launch_bounds__(256) void pf_mt_noise_kernel(const int64_t n,
                                                          const double* __restrict__ g,
                                                          const PredictConst pc,
                                                          double* __restrict__ noise) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double n0 = g[3 * i], n1 = g[3 * i + 1], n2 = g[3 * i + 2];
#pragma unroll
    for (int j = 0; j < 3; ++j)
        noise[3 * i + j] = fma(n2, pc.q[6 + j], fma(n1, pc.q[3 + j], n0 * pc.q[j]));
}

// the step's draws: [rand() if resampling] -> mvn(Q, NP) -> mvn(R, NL)
int launch_mt(slam_pf* h) {
    const int64_t n3 = 3 * h->n;
    int rc = mt_enqueue(h->mtb, 0, h->flags + kFlagResample, h->pc.np_recip, h->ofs, h->ctr,
                        n3 + 2 * (int64_t)h->nl, h->flags + kFlagStatus, h->stream);
    if (rc) return rc;
    if (h->nl > 0)
        pf_mt_observe_kernel<<<1, 512, 32 * (size_t)h->nl, h->stream>>>(
            h->mtb.normals, n3, h->lm, h->nl, h->truth, h->ctr, h->mr[0], h->mr[1], h->mr[2],
            h->mr[3], h->z_all, h->zc, h->lc.closed, h->refp, h->ctl, h->pc.dt, h->cfg.motion);
    if (h->cfg.motion == SLAM_MOTION_LINEAR)
        pf_mt_noise_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(h->n, h->mtb.normals, h->pc,
                                                                     h->noise);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// The device-RNG normals of particle pairs [p0, p0 + count) (slam_debug_pair_normals)
__global__ __launch_bounds__(256) void debug_pair_normals_kernel(const uint64_t p0, const int64_t count,
                                                                const uint32_t rstep, const uint64_t seed,
                                                                double* __restrict__ out) {
    __shared__ RngTabsLds s_rng;
    const RngTabs T = rng_tabs_stage(&s_rng, (int)threadIdx.x, 256);
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    double g[6];
    pair_normals(p0 + (uint64_t)i, rstep, seed, T, g);
#pragma unroll
    for (int j = 0; j < 6; ++j) out[6 * i + j] = g[j];
}

// One whole device-decided step (scans gate on the flag; no host decision).
int launch_step(slam_pf* h, bool host_noise) {
    int rc;
    if (h->mt) {
        if ((rc = launch_mt(h))) return rc;
        host_noise = true;
    }
    tic(h, 2);
#ifndef SLAM_NO_SCAN_LAUNCH       // A/B diagnostic only: wrong on resample steps
    if ((rc = launch_scans(h, 0, false))) return rc;
#endif
    toc(h, 2);
    if ((rc = launch_fused(h, h->cfg.motion, host_noise))) return rc;
    return launch_reduce(h, -1);
}

// The records of steps [first, first + count) from the coherent host buffer:
// stored there by the batch's last step end (exported: slam_pf_run on a
// deferred handle) or by one export launch here.
int sync_results(slam_pf* h, int32_t first, int32_t count, slam_pf_result* out, bool exported = false) {
    static_assert(sizeof(slam_pf_result) % 8 == 0, "result records move as 8-byte words");
    if (!exported) {
        const int64_t words = (int64_t)count * (int64_t)(sizeof(slam_pf_result) / 8);
        pf_export_kernel<<<std::min<unsigned>(grid_for(words, 256), 64u), 256, 0, h->stream>>>(
            reinterpret_cast<const uint64_t*>(h->res_dev + first), words,
            reinterpret_cast<uint64_t*>(h->res_host_dev + first));
        SLAM_HIP_TRY(hipGetLastError());
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    const slam_pf_result* r = h->res_host + first;
    int rc = SLAM_OK;
    for (int i = 0; i < count; ++i) {
        if (out) out[i] = r[i];
        // every condition named in one message (status word and step), the
        // IndexError taking precedence as the reference's own error
        const int32_t st = r[i].status;
        if (st & (1 | 8 | 256)) {
            std::string msg;
            if (st & 1) msg += "resample position beyond the last cumulative weight "
                               "(IndexError in particle_filter.py:219); clamped to NP-1; ";
            if (st & 8) msg += "exact-cumsum launch: release token timed out; ";
            if (st & 256) msg += "mt19937 draw: candidate bound exhausted; ";
            char tail[96];
            std::snprintf(tail, sizeof tail, "record %d of the batch, status 0x%x, n_special %d", (int)(first + i),
                          (unsigned)st, (int)r[i].n_special);
            rc = fail((st & 1) ? SLAM_ERR_INDEX : SLAM_ERR_HIP, msg + tail);
        }
    }
    h->resample_next = r[count - 1].resample_next;
    return rc;
}

int create_impl(const slam_pf_config* cfg, int64_t n_local, int64_t n_global, int64_t gbase,
                int32_t n_landmarks, const double* landmarks, int device, slam_pf** out,
                bool deferred, bool dist_shard) {
    SLAM_ARG_CHECK(cfg && out, "slam_pf_create: NULL argument");
    SLAM_ARG_CHECK(n_local > 0 && n_global < (int64_t(1) << 31) && gbase >= 0 &&
                       gbase + n_local <= n_global,
                   "slam_pf_create: need 0 < n_local, gbase + n_local <= n_global < 2^31");
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
    h->n = n_local;
    h->n_global = n_global;
    h->gbase = gbase;
    h->nl = n_landmarks;
    int rc = make_lik_const(h);
    if (rc) {
        delete h;
        return rc;
    }
    make_predict_const(h);
    const int64_t n = n_local;
    h->nb_scan = (int32_t)((n + kScanBlock - 1) / kScanBlock);
    h->nchunks = (int32_t)((n + kSumChunk - 1) / kSumChunk);
    h->nb_norm = (int32_t)((n + kNormPer - 1) / kNormPer);
    h->nb_part = (int32_t)((n + kPartPer - 1) / kPartPer);
    h->deferred = deferred;
    {
        // merged exact-cumsum launch only when its whole grid is co-resident
        // (its blocks wait for the last one); otherwise two launches
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, scan_lean_merged_kernel,
                                                         kScanThreads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
                hipSuccess)
            h->scan_merged_ok = deferred && (int64_t)h->nb_scan <= (int64_t)per_cu * cus / 2;
        h->scan_merged = h->scan_merged_ok;
    }
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return fail(SLAM_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
#define A(p, cnt)                                         \
    if ((rc = dalloc(h, &(p), (size_t)(cnt))) != 0) {     \
        slam_pf_destroy(h);                               \
        return rc;                                        \
    }
    // deferred handles: particle and weight arrays padded to whole fused blocks
    // (the fused kernel moves particle pairs with 16-byte loads and stores)
    // (a sharded handle: npad staging slots on either side of each particle
    // array for the particles a resample receives from other ranks, DeferParts.goff)
    const int64_t npad = deferred ? (int64_t)h->nb_part * kPartPer : n;
    const int64_t side = dist_shard ? npad : 0;
    for (int k = 0; k < 2; ++k) {
        A(h->x[k], npad + 2 * side);
        A(h->y[k], npad + 2 * side);
        A(h->th[k], npad + 2 * side);
        if (npad > n || side) {
            SLAM_HIP_TRY(hipMemsetAsync(h->x[k], 0, sizeof(double) * (npad + 2 * side), h->stream));
            SLAM_HIP_TRY(hipMemsetAsync(h->y[k], 0, sizeof(double) * (npad + 2 * side), h->stream));
            SLAM_HIP_TRY(hipMemsetAsync(h->th[k], 0, sizeof(double) * (npad + 2 * side), h->stream));
        }
        h->x[k] += side;
        h->y[k] += side;
        h->th[k] += side;
    }
    h->dp.goff = side;
    h->dp.glim = dist_shard ? 3 * npad : n;
    A(h->w, n);
    A(h->w_un, npad);
    if (npad > n) SLAM_HIP_TRY(hipMemsetAsync(h->w_un, 0, sizeof(double) * npad, h->stream));
    A(h->c, npad);
    A(h->kincl, n);
    A(h->fexcl, n);
    A(h->idx, n);
    A(h->bsum, std::max(h->nb_norm, h->nb_part));
    A(h->boff, std::max(h->nb_norm, h->nb_part) + 1);
    A(h->s_cur, 1);
    A(h->dp.pmax, h->nb_part + 1);                        // + 1: the finalize's pair loads
    A(h->dp.pidx, h->nb_part);
    A(h->dp.ppre, h->nb_part);
    for (int q = 0; q < 3; ++q) A(h->dp.pxe[q], h->nb_part);
    for (int q = 0; q < 11; ++q) A(h->dp.ps[q], h->nb_part + 1);
    A(h->dp.leaf, (size_t)(kPartPer / 128) * h->nb_part);
    A(h->dp.mark, npad);
    A(h->dp.carry, h->nb_part + 1);
    if (deferred && h->nb_part > kFinThreads * kFinRegBlocks) {
        const int32_t per = kFinThreads * kFinRegBlocks;
        h->fsl.nsl = (h->nb_part + per - 1) / per;
        A(h->fsl.m, h->fsl.nsl);
        A(h->fsl.q, 11 * (size_t)h->fsl.nsl);
        A(h->fsl.buf, std::max<int64_t>(n / kSumChunk, 1));
        A(h->fsl.cblk, kSliceCand * (size_t)h->fsl.nsl);
        A(h->fsl.cpm, kSliceCand * (size_t)h->fsl.nsl);
        A(h->fsl.ncand, h->fsl.nsl);
        A(h->fsl.pre, h->nb_part + 1);
        A(h->fsl.u, h->fsl.nsl);
    }
    SLAM_HIP_TRY(hipMemsetAsync(h->dp.mark, 0xff, sizeof(int64_t) * npad, h->stream));
    SLAM_HIP_TRY(hipMemsetAsync(h->dp.carry, 0, sizeof(int32_t) * (h->nb_part + 1), h->stream));
    // tile totals: 2048-element tiles (shards) or 512-element wave tiles (deferred)
    const int32_t ntile_max = std::max(h->nb_scan, h->nb_part);
    A(h->bk, ntile_max);
    A(h->boffk, ntile_max);
    A(h->bf, ntile_max);
    A(h->bofff, ntile_max);
    A(h->ktot, 1);
    A(h->nspec, 1);
    A(h->spec_in, n);
    if (deferred) A(h->stage, n);
    A(h->spec_out, n);
    A(h->part, h->nchunks);
    A(h->bp, h->nb_norm);
    A(h->wsum, 1);
    // [0..2] last estimate, [4..6] the one before, [7] moves of the first
    // expansion reference (closed_prep_reference)
    A(h->refp, 8);
    A(h->flags, kFlagWords);
    A(h->tk, 4 * kTicketWords);
    A(h->lm, 2 * std::max<int32_t>(n_landmarks, 1));
    A(h->noise, 3 * n);
    A(h->ctr, 4);
#undef A
    std::vector<int32_t> leaves, ops;
    const int tail = (int)(n % kSumChunk);
    if (tail) build_tail(0, tail, leaves, ops);
    h->n_tail_leaves = (int32_t)(leaves.size() / 2);
    h->n_tail_ops = (int32_t)ops.size();
    if ((rc = dalloc(h, &h->tail_leaves, leaves.size() + 2)) ||
        (rc = dalloc(h, &h->tail_ops, ops.size() + 1)) || (rc = ensure_steps(h, 1))) {
        slam_pf_destroy(h);
        return rc;
    }
    if (tail) {
        SLAM_HIP_TRY(hipMemcpy(h->tail_leaves, leaves.data(), leaves.size() * 4, hipMemcpyHostToDevice));
        SLAM_HIP_TRY(hipMemcpy(h->tail_ops, ops.data(), ops.size() * 4, hipMemcpyHostToDevice));
    }
    // initial state: particle_filter.py:81-84
    std::vector<double> tmp((size_t)n);
    for (int k = 0; k < 3; ++k) {
        std::fill(tmp.begin(), tmp.end(), cfg->x0[k]);
        double* d = (k == 0) ? h->x[0] : (k == 1) ? h->y[0] : h->th[0];
        SLAM_HIP_TRY(hipMemcpy(d, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice));
    }
    std::fill(tmp.begin(), tmp.end(), 1.0 / (double)n_global);
    SLAM_HIP_TRY(hipMemcpy(h->w, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice));
    SLAM_HIP_TRY(hipMemcpy(h->w_un, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice));
    const double one = 1.0;
    SLAM_HIP_TRY(hipMemcpy(h->s_cur, &one, sizeof(double), hipMemcpyHostToDevice));
    {
        const double rp[8] = {cfg->x0[0], cfg->x0[1], cfg->x0[2], 0.0,
                               cfg->x0[0], cfg->x0[1], cfg->x0[2], 1.0};
        SLAM_HIP_TRY(hipMemcpy(h->refp, rp, sizeof(rp), hipMemcpyHostToDevice));
    }
    SLAM_HIP_TRY(hipMemset(h->flags, 0, kFlagWords * sizeof(int32_t)));
    SLAM_HIP_TRY(hipMemset(h->tk, 0, 4 * kTicketWords * sizeof(unsigned)));
    SLAM_HIP_TRY(hipMemset(h->ctr, 0, 2 * sizeof(int32_t)));
    SLAM_HIP_TRY(hipMemsetD32((hipDeviceptr_t)(h->ctr + 2), -1, 2));   // no batch bounds yet
    if (n_landmarks > 0)
        SLAM_HIP_TRY(hipMemcpy(h->lm, landmarks, 2 * n_landmarks * sizeof(double), hipMemcpyHostToDevice));
    *out = h;
    return SLAM_OK;
}

// deferred path: h->w <- w_un / s_cur (the current normalised weights)
int materialize_w(slam_pf* h) {
    if (!h->deferred) return SLAM_OK;
    normalize_only_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(h->n, h->w_un, h->s_cur,
                                                                       h->pc.np_recip, h->w);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int set_s_one(slam_pf* h) {
    static const double one = 1.0;
    if (h->deferred)
        SLAM_HIP_TRY(hipMemcpyAsync(h->s_cur, &one, sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    return SLAM_OK;
}

// stage one sync-mode step's inputs into StepIO slot 0
int stage_inputs(slam_pf* h, const double* control, const double* z, const double* noise,
                 double u) {
    if (h->nl && z)
        SLAM_HIP_TRY(hipMemcpyAsync(h->z_all, z, 2 * h->nl * sizeof(double), hipMemcpyHostToDevice,
                                    h->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(h->ctl, control, 2 * sizeof(double), hipMemcpyHostToDevice, h->stream));
    h->ofs_host = std::isnan(u) ? u : u * h->pc.np_recip;           // particle_filter.py:214
    SLAM_HIP_TRY(hipMemcpyAsync(h->ofs, &h->ofs_host, sizeof(double), hipMemcpyHostToDevice, h->stream));
    if (noise)
        SLAM_HIP_TRY(hipMemcpyAsync(h->noise, noise, 3 * h->n * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    h->z_steps = 0;   // slot 0 now holds a single staged step
    const int rc = set_ctr(h, 0);
    if (rc || !z) return rc;
    return launch_prestep(h);
}

}  // namespace

#include "pf_dist_api.inl"

#ifdef SLAM_PROBE_COUNT_SLOW
extern "C" int slam_probe_slow_count(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe_slow), 16) != hipSuccess) return -1;
    unsigned long long z[2] = {0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_probe_slow), z, 16) == hipSuccess ? 0 : -1;
}
#endif

#ifdef SLAM_FIN_PROBE
extern "C" int slam_fin_probe_read(long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fin_probe), sizeof(long long) * 32) == hipSuccess ? 0 : -1;
}
#endif

#ifdef SLAM_PROBE_FUSED
extern "C" int slam_fprobe_read(unsigned long long* out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprobe), sizeof(unsigned long long) * count) == hipSuccess
               ? 0 : -1;
}
#endif

#ifdef SLAM_PROBE
extern "C" int slam_probe_read(unsigned long long* out, int count) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe), sizeof(unsigned long long) * count) != hipSuccess) return -1;
    unsigned long long z[32] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" {

int slam_pf_create(const slam_pf_config* cfg, int64_t n_particles, int32_t n_landmarks,
                   const double* landmarks, int device, slam_pf** out) {
    return create_impl(cfg, n_particles, n_particles, 0, n_landmarks, landmarks, device, out, true,
                       false);
}

int slam_pf_destroy(slam_pf* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    drop_graphs(h);
    mt_free(h->mtb);
    for (void* p : h->allocs) (void)hipFree(p);
    if (h->res_host) (void)hipHostFree(h->res_host);
    if (h->ctl_pin) (void)hipHostFree(h->ctl_pin);
    for (int k = 0; k < 4; ++k)
        for (auto& pr : h->tm.ev[k]) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    if (h->stream && h->own_stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_pf_set_stream(slam_pf* h, void* stream, int32_t external) {
    SLAM_ARG_CHECK(h, "slam_pf_set_stream: NULL handle");
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    drop_graphs(h);
    if (h->own_stream) (void)hipStreamDestroy(h->stream);
    if (external) {              // the caller's stream (NULL = the default stream)
        h->stream = (hipStream_t)stream;
        h->own_stream = false;
    } else {
        SLAM_HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    return SLAM_OK;
}

int slam_pf_set_landmarks(slam_pf* h, const double* landmarks) {
    SLAM_ARG_CHECK(h && (landmarks || h->nl == 0), "slam_pf_set_landmarks: NULL argument");
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (h->nl) {
        SLAM_HIP_TRY(hipMemcpyAsync(h->lm, landmarks, 2 * h->nl * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_set_state(slam_pf* h, const double* x, const double* y, const double* th,
                      const double* w) {
    SLAM_ARG_CHECK(h, "slam_pf_set_state: NULL handle");
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const size_t b = h->n * sizeof(double);
    const int c = h->cur;
    if (x) SLAM_HIP_TRY(hipMemcpyAsync(h->x[c], x, b, hipMemcpyHostToDevice, h->stream));
    if (y) SLAM_HIP_TRY(hipMemcpyAsync(h->y[c], y, b, hipMemcpyHostToDevice, h->stream));
    if (th) SLAM_HIP_TRY(hipMemcpyAsync(h->th[c], th, b, hipMemcpyHostToDevice, h->stream));
    if (w) {
        if (h->deferred) {
            static const double one = 1.0;
            SLAM_HIP_TRY(hipMemcpyAsync(h->w_un, w, b, hipMemcpyHostToDevice, h->stream));
            SLAM_HIP_TRY(hipMemcpyAsync(h->s_cur, &one, sizeof(double), hipMemcpyHostToDevice,
                                        h->stream));
        } else {
            SLAM_HIP_TRY(hipMemcpyAsync(h->w, w, b, hipMemcpyHostToDevice, h->stream));
        }
        // particle_filter.py:210-211: the resample decision from these weights
        // (single GPU; a shard's caller decides from the global ESS)
        if (h->n == h->n_global) {
            double s2 = 0.0;
            for (int64_t i = 0; i < h->n; ++i) s2 += w[i] * w[i];
            h->resample_next = (1.0 / s2 < h->cfg.ess_threshold) ? 1 : 0;
            int rc = set_flag(h, kFlagResample, h->resample_next);
            if (rc) return rc;
        }
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
    if (w) {
        int rc = materialize_w(h);
        if (rc) return rc;
        SLAM_HIP_TRY(hipMemcpyAsync(w, h->w, b, hipMemcpyDeviceToHost, h->stream));
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_get_weights_raw(slam_pf* h, double* w_un, double* s) {
    SLAM_ARG_CHECK(h, "slam_pf_get_weights_raw: NULL handle");
    SLAM_ARG_CHECK(h->deferred, "slam_pf_get_weights_raw: not a deferred (single-GPU) handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (w_un)
        SLAM_HIP_TRY(hipMemcpyAsync(w_un, h->w_un, h->n * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    if (s) SLAM_HIP_TRY(hipMemcpyAsync(s, h->s_cur, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_step(slam_pf* h, const double* control, const double* z, const double* noise,
                 double u_resample, slam_pf_result* res) {
    SLAM_ARG_CHECK(h && control && (z || h->nl == 0), "slam_pf_step: NULL argument");
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_step: sharded handle (use the shard entry points)");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = stage_inputs(h, control, z, noise, u_resample))) return rc;
    tic(h, 3);
    const int32_t resampling = h->resample_next;
    if (resampling) {
        tic(h, 2);
        if ((rc = launch_scans(h, 1, true))) return rc;
        toc(h, 2);
    }
    if ((rc = launch_fused(h, h->cfg.motion, noise != nullptr))) return rc;
    if ((rc = launch_reduce(h, resampling))) return rc;
    toc(h, 3);
    h->stepno++;
    return sync_results(h, 0, 1, res);
}

// Stand-alone exact cumsum (slam_pf_resample, slam_pf_resample_indices): its
// expand pass writes run marks with the offset of StepIO slot ctr[0], so the
// caller's offset goes into slot 0 and ctr[0] back to 0 first -- the previous
// step end had advanced ctr[0] past the staged slot (an out-of-bounds or stale
// offset: round 6, test_gpu_zz_order) -- and afterwards the mark generation
// moves on, so that these marks (not meant for a gather) never win the next
// step's running max.
static int stage_scan_offset(slam_pf* h, double u) {
    h->ofs_host = std::isnan(u) ? u : u * h->pc.np_recip;           // particle_filter.py:214
    SLAM_HIP_TRY(hipMemcpyAsync(h->ofs, &h->ofs_host, sizeof(double), hipMemcpyHostToDevice, h->stream));
    return set_ctr(h, 0);
}
static int retire_scan_marks(slam_pf* h) {
    mark_gen_bump_kernel<<<1, 1, 0, h->stream>>>(h->flags);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int slam_pf_resample(slam_pf* h, double u_resample, int32_t force, int32_t* resampled) {
    SLAM_ARG_CHECK(h, "slam_pf_resample: NULL handle");
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_resample: sharded handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const int32_t go = force ? 1 : h->resample_next;
    if (resampled) *resampled = go;
    if (!go) return SLAM_OK;
    int rc = stage_scan_offset(h, u_resample);
    if (rc || (rc = launch_scans(h, 1, true)) || (rc = retire_scan_marks(h))) return rc;
    const double ofs = std::isnan(u_resample) ? u_resample : u_resample * h->pc.np_recip;
    resample_search_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(
        h->n, h->c, h->idx, h->pc.rstep, ofs, h->pc.np_recip, h->cfg.seed, h->stepno, h->flags);
    const int src = h->cur, dst = 1 - h->cur;
    gather_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(
        h->n, h->idx, h->x[src], h->y[src], h->th[src], h->x[dst], h->y[dst], h->th[dst],
        h->deferred ? h->w_un : h->w, h->pc.np_recip);
    SLAM_HIP_TRY(hipGetLastError());
    if ((rc = set_s_one(h))) return rc;
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
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_resample_indices: sharded handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = stage_scan_offset(h, u_resample);
    if (rc || (rc = launch_scans(h, 1, true)) || (rc = retire_scan_marks(h))) return rc;
    const double ofs = std::isnan(u_resample) ? u_resample : u_resample * h->pc.np_recip;
    resample_search_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(
        h->n, h->c, h->idx, h->pc.rstep, ofs, h->pc.np_recip, h->cfg.seed, h->stepno, h->flags);
    SLAM_HIP_TRY(hipGetLastError());
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
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    // predict only: fused kernel with zero landmarks and no resample gather;
    // the weights pass through unchanged (w_un = w * 1).
    int rc;
    if ((rc = stage_inputs(h, control, nullptr, noise, std::nan("")))) return rc;
    if ((rc = set_flag(h, kFlagResample, 0))) return rc;
    const int32_t nl = h->lc.nl;
    const double lnd = h->lc.neg_nl_ln_den;
    h->lc.nl = 0;
    h->lc.neg_nl_ln_den = 0.0;          // zero landmarks: likelihood factor exactly 1
    rc = launch_fused(h, h->cfg.motion, noise != nullptr);
    h->lc.nl = nl;
    h->lc.neg_nl_ln_den = lnd;
    if (rc) return rc;
    if (h->deferred) {
        if ((rc = set_s_one(h))) return rc;   // w_un now holds the normalised weights
    } else {
        SLAM_HIP_TRY(hipMemcpyAsync(h->w, h->w_un, h->n * 8, hipMemcpyDeviceToDevice, h->stream));
    }
    if ((rc = set_flag(h, kFlagResample, h->resample_next))) return rc;
    h->stepno++;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_update(slam_pf* h, const double* z, slam_pf_result* res) {
    // __likelihood + estimate on the current particles (no motion, no resample)
    SLAM_ARG_CHECK(h && (z || h->nl == 0), "slam_pf_update: NULL argument");
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_update: sharded handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    const double ctl[2] = {0.0, 0.0};
    if ((rc = stage_inputs(h, ctl, z, nullptr, std::nan("")))) return rc;
    if ((rc = set_flag(h, kFlagResample, 0))) return rc;
    if ((rc = launch_fused(h, kMotionNone, false))) return rc;
    if ((rc = launch_reduce(h, 0))) return rc;
    return sync_results(h, 0, 1, res);
}

int slam_debug_pair_normals(int device, uint64_t p0, int64_t count, uint32_t rstep, uint64_t seed,
                            double* out) {
    SLAM_ARG_CHECK(out && count >= 0 && count <= (int64_t(1) << 26),
                   "slam_debug_pair_normals: bad arguments");
    if (count == 0) return SLAM_OK;
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev, "slam_debug_pair_normals: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    double* d = nullptr;
    SLAM_HIP_TRY(hipMalloc(&d, 6 * count * sizeof(double)));
    debug_pair_normals_kernel<<<grid_for(count, 256), 256>>>(p0, count, rstep, seed, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, d, 6 * count * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SLAM_ERR_HIP, std::string("slam_debug_pair_normals: ") + hipGetErrorString(e));
    return SLAM_OK;
}

int slam_pf_weight_sum(slam_pf* h, double* sum_out) {
    SLAM_ARG_CHECK(h && sum_out, "slam_pf_weight_sum: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = materialize_w(h);
    if (rc) return rc;
    chunk_sum_kernel<<<h->nchunks, 512, 0, h->stream>>>(h->w, h->n, h->part, h->tail_leaves,
                                                         h->tail_ops, h->n_tail_leaves,
                                                         h->n_tail_ops, h->tk, h->wsum);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(sum_out, h->wsum, 8, hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_load_observations(slam_pf* h, int32_t n_steps, const double* z_all) {
    SLAM_ARG_CHECK(h && n_steps > 0 && (z_all || h->nl == 0), "slam_pf_load_observations: bad argument");
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = ensure_steps(h, n_steps);
    if (rc) return rc;
    if (h->nl) {
        SLAM_HIP_TRY(hipMemcpyAsync(h->z_all, z_all, (size_t)n_steps * 2 * h->nl * sizeof(double),
                                    hipMemcpyHostToDevice, h->stream));
    }
    std::vector<double> nan((size_t)n_steps, std::nan(""));
    SLAM_HIP_TRY(hipMemcpyAsync(h->ofs, nan.data(), n_steps * sizeof(double), hipMemcpyHostToDevice,
                                h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    h->z_steps = n_steps;
    return SLAM_OK;
}

int slam_pf_run(slam_pf* h, int32_t first_step, int32_t n_steps, const double* controls,
                slam_pf_result* results) {
    SLAM_ARG_CHECK(h && controls && n_steps > 0, "slam_pf_run: bad argument");
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_run: sharded handle");
    SLAM_ARG_CHECK(first_step >= 0 && first_step + n_steps <= (h->mt ? h->truth_steps : h->z_steps),
                   h->mt ? "slam_pf_run: steps outside the loaded true poses (slam_pf_load_truth)"
                         : "slam_pf_run: steps outside the loaded observations");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    int32_t prep_next = -1;
    // a batch continuing the previous one with nothing changed in between
    // (prep_step, cleared by every call that could): the previous step end
    // left the block-total prefix for a resampling first step already
    const bool continues = (h->prep_step == first_step);
    if ((rc = launch_run_setup(h, first_step, n_steps, controls, h->resample_next, &prep_next)))
        return rc;
    if (h->resample_next && !continues && (rc = launch_bsum(h))) return rc;   // the first step's scan prefix
    const bool graphs = h->use_graph && !h->timing;
    int32_t k = 0;
    while (k < n_steps) {
        if (graphs) {
            int lv = kGraphLevels - 1;
            while ((1 << lv) > n_steps - k) --lv;
            hipGraphExec_t& ge = h->graph[lv][h->cur];
            if (!ge && (rc = capture_steps(h, ge, 1 << lv))) return rc;
            SLAM_HIP_TRY(hipGraphLaunch(ge, h->stream));
            const int done = 1 << lv;
            if (done & 1) h->cur = 1 - h->cur;
            k += done;
            h->stepno += done;
        } else {
            tic(h, 3);
            if ((rc = launch_step(h, false))) return rc;
            toc(h, 3);
            ++k;
            h->stepno++;
        }
    }
    rc = sync_results(h, first_step, n_steps, results, h->deferred);
    if (rc == SLAM_OK && prep_next >= 0) {
        h->prep_step = prep_next;
        h->prep_ctl[0] = controls[2 * (n_steps - 1)];
        h->prep_ctl[1] = controls[2 * (n_steps - 1) + 1];
    }
    return rc;
}

int slam_pf_prepare_graphs(slam_pf* h, double* capture_ms) {
    SLAM_ARG_CHECK(h, "slam_pf_prepare_graphs: NULL handle");
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_prepare_graphs: sharded handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const auto t0 = std::chrono::steady_clock::now();
    int rc = SLAM_OK;
    if (h->use_graph) {
        const int cur0 = h->cur;
        for (int par = 0; par < 2 && rc == SLAM_OK; ++par) {
            h->cur = par;
            for (int lv = 0; lv < kGraphLevels && rc == SLAM_OK; ++lv)
                if (!h->graph[lv][par]) rc = capture_steps(h, h->graph[lv][par], 1 << lv);
        }
        h->cur = cur0;
    }
    if (capture_ms)
        *capture_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int slam_pf_set_rng_mt19937(slam_pf* h, const uint32_t* key, int32_t pos, int32_t has_gauss,
                            double gauss, const double* r_factor) {
    SLAM_ARG_CHECK(h && key && r_factor, "slam_pf_set_rng_mt19937: NULL argument");
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_set_rng_mt19937: sharded handle");
    SLAM_ARG_CHECK(h->nl <= 2048, "slam_pf_set_rng_mt19937: at most 2048 landmarks");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    int rc = mt_reserve(h->mtb, 3 * h->n + 2 * (int64_t)h->nl, 1, h->device);
    if (rc) return rc;
    if ((rc = mt_set_state(h->mtb, key, pos, has_gauss, gauss, h->stream))) return rc;
    for (int k = 0; k < 4; ++k) h->mr[k] = r_factor[k];
    if (!h->mt) drop_graphs(h);              // captured steps without the draws
    h->mt = true;
    h->noise_src = h->cfg.motion == SLAM_MOTION_LINEAR ? h->noise : h->mtb.normals;
    return SLAM_OK;
}

int slam_pf_get_rng_mt19937(slam_pf* h, uint32_t* key, int32_t* pos, int32_t* has_gauss,
                            double* gauss) {
    SLAM_ARG_CHECK(h, "slam_pf_get_rng_mt19937: NULL handle");
    SLAM_ARG_CHECK(h->mt, "slam_pf_get_rng_mt19937: the device stream is not enabled");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    return mt_get_state(h->mtb, key, pos, has_gauss, gauss, h->stream);
}

int slam_pf_rng_mt19937_info(slam_pf* h, int64_t* out) {
    SLAM_ARG_CHECK(h && out, "slam_pf_rng_mt19937_info: NULL argument");
    SLAM_ARG_CHECK(h->mt, "slam_pf_rng_mt19937_info: the device stream is not enabled");
    const MtBuffers& b = h->mtb;
    out[0] = b.cap * (int64_t)sizeof(uint32_t);
    out[1] = b.R;
    out[2] = b.S;
    out[3] = b.need > 0 ? (int64_t)b.R * b.S / b.need : 0;
    return SLAM_OK;
}

int slam_pf_step_truth(slam_pf* h, const double* control, const double* truth, double* z_out,
                       slam_pf_result* res) {
    SLAM_ARG_CHECK(h && control && truth, "slam_pf_step_truth: NULL argument");
    h->prep_step = -1;
    SLAM_ARG_CHECK(h->mt, "slam_pf_step_truth: enable the device stream first (slam_pf_set_rng_mt19937)");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    SLAM_HIP_TRY(hipMemcpyAsync(h->ctl, control, 2 * sizeof(double), hipMemcpyHostToDevice, h->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(h->truth, truth, 4 * sizeof(double), hipMemcpyHostToDevice, h->stream));
    h->z_steps = 0;
    h->truth_steps = 0;
    const int32_t resampling = h->resample_next;
    if ((rc = set_ctr(h, 0)) || (rc = set_flag(h, kFlagResample, resampling))) return rc;
    tic(h, 3);
    if ((rc = launch_mt(h))) return rc;
    if (resampling) {
        tic(h, 2);
        if ((rc = launch_scans(h, 1, true))) return rc;
        toc(h, 2);
    }
    if ((rc = launch_fused(h, h->cfg.motion, true))) return rc;
    if ((rc = launch_reduce(h, resampling))) return rc;
    toc(h, 3);
    h->stepno++;
    if (z_out && h->nl)
        SLAM_HIP_TRY(hipMemcpyAsync(z_out, h->z_all, 2 * h->nl * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    return sync_results(h, 0, 1, res);
}

int slam_pf_load_truth(slam_pf* h, int32_t n_steps, const double* truth) {
    SLAM_ARG_CHECK(h && n_steps > 0 && truth, "slam_pf_load_truth: bad argument");
    h->prep_step = -1;
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = ensure_steps(h, n_steps);
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemcpyAsync(h->truth, truth, (size_t)n_steps * 4 * sizeof(double),
                                hipMemcpyHostToDevice, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    h->truth_steps = n_steps;
    return SLAM_OK;
}

int slam_pf_enable_timing(slam_pf* h, int32_t on) {
    SLAM_ARG_CHECK(h, "slam_pf_enable_timing: NULL handle");
    h->timing = on != 0;
    for (int k = 0; k < 4; ++k) h->tm.used[k] = 0;
    return SLAM_OK;
}

int slam_pf_set_graphs(slam_pf* h, int32_t on) {
    SLAM_ARG_CHECK(h, "slam_pf_set_graphs: NULL handle");
    h->use_graph = on != 0;
    return SLAM_OK;
}

int slam_pf_set_scan_merged(slam_pf* h, int32_t on) {
    SLAM_ARG_CHECK(h, "slam_pf_set_scan_merged: NULL handle");
    SLAM_ARG_CHECK(!on || h->scan_merged_ok,
                   "slam_pf_set_scan_merged: the merged launch needs a single-GPU handle whose "
                   "scan grid is co-resident");
    h->scan_merged = on != 0;
    drop_graphs(h);
    return SLAM_OK;
}

int slam_pf_set_resample_next(slam_pf* h, int32_t on) {
    SLAM_ARG_CHECK(h, "slam_pf_set_resample_next: NULL handle");
    SLAM_ARG_CHECK(h->n == h->n_global, "slam_pf_set_resample_next: sharded handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    h->prep_step = -1;                       // the next run forms its scan prefix itself
    h->resample_next = on ? 1 : 0;
    int rc = set_flag(h, kFlagResample, h->resample_next);
    if (rc) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_pf_set_ess_band(slam_pf* h, double band) {
    SLAM_ARG_CHECK(h && band >= 0.0, "slam_pf_set_ess_band: bad argument");
    h->ess_band = band;
    drop_graphs(h);                  // captured step kernels carry the band
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
