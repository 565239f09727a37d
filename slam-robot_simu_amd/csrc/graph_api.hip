// graph_api.hip -- C-ABI of graph-based SLAM (include/slam_hip.h).
//
// TrajectoryEstimator (graph_based_slam.py:330-581) -> slam_graph_*.  The
// block structure of H and the per-block accumulation plan (which edge parts
// land in which 3x3 block, in the reference's edge order) are built on the
// device once per edge set (graph_build.inl: radix sorts, uniques, binary
// searches; SLAM_GRAPH_HOST_BUILD=1 builds the same arrays on the host, for
// the tests); every Gauss-Newton iteration then runs entirely on the device:
// linearise -> assemble -> solve -> pose update.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "graph_kernels.inl"
#include "graph_build.inl"

using namespace slam;

constexpr int kGateInfo = 14;     // slam_graph_gate_info words

struct slam_graph {
    slam_graph_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<void*> allocs;     // dense-path buffers (per edge set, small systems only)
    void* arena = nullptr;         // structure + solver buffers of the edge set (grow-only)
    size_t arena_bytes = 0;
    int64_t dense_n = 0;           // unknowns the dense buffers were sized for
    // poses
    int64_t T = 0;
    double* poses = nullptr;
    // edges and structure
    int64_t E = 0, nt = 0, n_slots = 0;
    std::vector<int64_t> times_h;
    slam_graph_edge* edges = nullptr;
    double* blocks = nullptr;      // [42][E]
    int64_t *times = nullptr, *srow = nullptr, *scol = nullptr, *rptr = nullptr;
    int64_t *cptr = nullptr, *clist = nullptr, *bptr = nullptr, *blist = nullptr;
    int64_t* dslot = nullptr;
    double *val = nullptr, *b = nullptr, *delta = nullptr, *dsum = nullptr;
    // dense path
    double *A = nullptr, *LU = nullptr, *S = nullptr, *V = nullptr, *lan = nullptr;
    int32_t* piv = nullptr;
    double* luout = nullptr;       // [0..2] LU, [3..4] Lanczos
    // PCG
    double *minv = nullptr, *r = nullptr, *z = nullptr, *p = nullptr;
    double* q = nullptr;
    double* part = nullptr;
    PcgState* st = nullptr;
    // condition-number estimate of the PCG path (second stream)
    hipStream_t cstream = nullptr;
    hipEvent_t cev[3] = {};        // [0] operands ready (main stream), [1]/[2] estimate start/end
    double *cx = nullptr, *chx = nullptr, *cp = nullptr, *chp = nullptr;
    double *cw = nullptr, *cw2 = nullptr, *chw = nullptr, *cpart = nullptr;
    CondState* cst = nullptr;
    int64_t* cnt_host = nullptr;   // pinned: the structure build's two counts, then its times
    int64_t cnt_cap = 0;           // (a pageable read-back stalled the host ~7 ms now and then)
    PcgState* pcg_host = nullptr;  // pinned copies of the device states: the polls of the
    CondState* cond_host = nullptr;  // two streams must not block the host (pageable copies do)
    bool cond_warm = false;        // cx holds the previous update's vectors of this edge set
    int32_t cond_last_iters = 0;
    double cond_info[7] = {0, 0, 0, 0, 0, 0, 0};
    // the gate's log-det sums (cond_mode SLAM_GRAPH_COND_MARGIN)
    double* cert_part = nullptr;   // per-workgroup partials of the certificate kernels
    CertState* cert = nullptr;
    CertState* cert_host = nullptr;  // pinned
    double gate_info[kGateInfo] = {};
    hipEvent_t ev[5] = {};
    double last[5] = {0, 0, 0, 0, 0};
    int32_t pcg_last_iters = 0;    // iteration count of the previous PCG solve
    bool pcg_failed = false;       // the last update's PCG solve did not converge
};

namespace {

void free_list(std::vector<void*>& l) {
    for (void* p : l) (void)hipFree(p);
    l.clear();
}

template <typename T>
int galloc(slam_graph* h, T** p, size_t count) {
    void* q = nullptr;
    SLAM_HIP_TRY(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
    h->allocs.push_back(q);
    *p = (T*)q;
    return SLAM_OK;
}

#define GTRY(x)               \
    do {                      \
        int rc_ = (x);        \
        if (rc_) return rc_;  \
    } while (0)

template <typename T>
int upload(slam_graph* h, T* dst, const std::vector<T>& src) {
    if (src.empty()) return SLAM_OK;
    SLAM_HIP_TRY(hipMemcpyAsync(dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice,
                                h->stream));
    return SLAM_OK;
}

unsigned nblk(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// carve 256-byte aligned arrays out of one allocation
struct Carver {
    char* base;
    size_t off = 0;
    template <typename T>
    T* take(int64_t count) {
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += ((size_t)std::max<int64_t>(count, 1) * sizeof(T) + 255) / 256 * 256;
        return p;
    }
};

// the edge set's device arrays, sized by the upper bounds nt <= min(2E, T) and
// slots <= 2E + nt (carve twice: sizes, then pointers); one allocation reused
// while it is large enough
struct BuildScratch {
    int64_t *tl, *tl_s, *keys, *keys_s, *ukeys, *rb, *ra, *sl, *sl_s, *cval, *bkey, *bkey_s, *bval;
    int64_t* cnt;                  // [0] nt, [1] slots
    void* tmp;
    size_t tmp_bytes;
};

int carve_edge_set(slam_graph* h, int64_t E, int64_t nt_ub, size_t tmp_bytes, BuildScratch* bs) {
    const int64_t K = 2 * E + nt_ub;
    const int64_t n = 3 * nt_ub;
    for (int pass = 0; pass < 2; ++pass) {
        Carver c{pass ? (char*)h->arena : nullptr};
        h->edges = c.take<slam_graph_edge>(E);
        h->blocks = c.take<double>(42 * E);
        h->times = c.take<int64_t>(nt_ub);
        h->srow = c.take<int64_t>(K);
        h->scol = c.take<int64_t>(K);
        h->rptr = c.take<int64_t>(nt_ub + 1);
        h->cptr = c.take<int64_t>(K + 1);
        h->clist = c.take<int64_t>(4 * E);
        h->bptr = c.take<int64_t>(nt_ub + 1);
        h->blist = c.take<int64_t>(2 * E);
        h->dslot = c.take<int64_t>(nt_ub);
        h->val = c.take<double>(9 * K);
        h->b = c.take<double>(n);
        h->delta = c.take<double>(n);
        h->dsum = c.take<double>(1);
        h->minv = c.take<double>(9 * nt_ub);
        h->r = c.take<double>(n);
        h->z = c.take<double>(n);
        h->p = c.take<double>(n);
        h->q = c.take<double>(n);
        h->part = c.take<double>(3 * (int64_t)nblk(n, kPcgThreads) + 3);
        h->st = c.take<PcgState>(1);
        h->cx = c.take<double>(2 * n);
        h->chx = c.take<double>(2 * n);
        h->cp = c.take<double>(2 * n);
        h->chp = c.take<double>(2 * n);
        h->cw = c.take<double>(2 * n);
        h->cw2 = c.take<double>(2 * n);
        h->chw = c.take<double>(2 * n);
        h->cpart = c.take<double>((2 * kCondGram + 2) * (int64_t)nblk(n, kPcgThreads) + 8);
        h->cst = c.take<CondState>(1);
        h->cert_part = c.take<double>(4 * (int64_t)nblk(nt_ub, kCertThreads) +
                                      (int64_t)nblk(K, kCertThreads) + 8);
        h->cert = c.take<CertState>(1);
        h->luout = c.take<double>(8);
        if (bs) {
            bs->tl = c.take<int64_t>(2 * E);
            bs->tl_s = c.take<int64_t>(2 * E);
            bs->keys = c.take<int64_t>(K);
            bs->keys_s = c.take<int64_t>(K);
            bs->ukeys = c.take<int64_t>(K);
            bs->rb = c.take<int64_t>(E);
            bs->ra = c.take<int64_t>(E);
            bs->sl = c.take<int64_t>(4 * E);
            bs->sl_s = c.take<int64_t>(4 * E);
            bs->cval = c.take<int64_t>(4 * E);
            bs->bkey = c.take<int64_t>(2 * E);
            bs->bkey_s = c.take<int64_t>(2 * E);
            bs->bval = c.take<int64_t>(2 * E);
            bs->cnt = c.take<int64_t>(2);
            bs->tmp = c.take<char>((int64_t)tmp_bytes);
            bs->tmp_bytes = tmp_bytes;
        }
        if (pass == 0 && c.off > h->arena_bytes) {
            if (h->arena) SLAM_HIP_TRY(hipFree(h->arena));
            h->arena = nullptr;
            h->arena_bytes = 0;
            SLAM_HIP_TRY(hipMalloc(&h->arena, c.off + c.off / 4));
            h->arena_bytes = c.off + c.off / 4;
        }
    }
    return SLAM_OK;
}

// dense-path buffers (n = 3 nt <= kGraphDenseMax), grow-only
int dense_buffers(slam_graph* h, int64_t n) {
    if (n > kGraphDenseMax) return SLAM_OK;
    if (n <= h->dense_n && h->A) return SLAM_OK;
    free_list(h->allocs);
    GTRY(galloc(h, &h->A, n * n));
    GTRY(galloc(h, &h->LU, n * n));
    GTRY(galloc(h, &h->S, n * n));
    GTRY(galloc(h, &h->V, n * (n + 1)));
    GTRY(galloc(h, &h->lan, 3 * n + 8));
    GTRY(galloc(h, &h->piv, n));
    h->dense_n = n;
    return SLAM_OK;
}

int finish_structure(slam_graph* h, int64_t E, int64_t nt, int64_t ns) {
    h->E = E;
    h->pcg_last_iters = 0;
    h->cond_warm = false;
    h->cond_last_iters = 0;
    h->nt = nt;
    h->n_slots = ns;
    const int64_t n = 3 * nt;
    if (n <= kGraphDenseMax) {
        GTRY(dense_buffers(h, n));
    } else {
        free_list(h->allocs);
        h->A = h->LU = h->S = h->V = h->lan = nullptr;
        h->piv = nullptr;
        h->dense_n = 0;
    }
    return SLAM_OK;
}

// the structure on the device (graph_build.inl)
int build_structure_device(slam_graph* h, int64_t E, const slam_graph_edge* ed) {
    const int64_t nt_ub = std::min<int64_t>(2 * E, h->T);
    const int64_t K = 2 * E + nt_ub;
    const int tbits = bits_for((uint64_t)h->T);
    const int sbits = bits_for((uint64_t)K);
    hipStream_t s = h->stream;
    // temporary storage of the largest rocPRIM call
    size_t tb = 0, t1 = 0;
    int64_t* np = nullptr;
    auto q = [&](hipError_t e) { return e == hipSuccess; };
    if (!q(rocprim::radix_sort_keys(nullptr, t1, np, np, (size_t)(2 * E), 0, tbits, s))) goto qfail;
    tb = std::max(tb, t1);
    if (!q(rocprim::unique(nullptr, t1, np, np, np, (size_t)(2 * E), rocprim::equal_to<int64_t>(), s)))
        goto qfail;
    tb = std::max(tb, t1);
    if (!q(rocprim::radix_sort_keys(nullptr, t1, np, np, (size_t)K, 0, 64, s))) goto qfail;
    tb = std::max(tb, t1);
    if (!q(rocprim::unique(nullptr, t1, np, np, np, (size_t)K, rocprim::equal_to<int64_t>(), s))) goto qfail;
    tb = std::max(tb, t1);
    if (!q(rocprim::radix_sort_pairs(nullptr, t1, np, np, np, np, (size_t)(4 * E), 0, sbits, s)))
        goto qfail;
    tb = std::max(tb, t1);
    if (!q(rocprim::radix_sort_pairs(nullptr, t1, np, np, np, np, (size_t)(2 * E), 0, tbits, s)))
        goto qfail;
    tb = std::max(tb, t1);
    {
        BuildScratch bs{};
        GTRY(carve_edge_set(h, E, nt_ub, tb, &bs));
        SLAM_HIP_TRY(hipMemcpyAsync(h->edges, ed, E * sizeof(slam_graph_edge), hipMemcpyHostToDevice, s));
        // distinct times (:457-467 order)
        hipLaunchKernelGGL(gb_times_kernel, dim3(nblk(E)), dim3(256), 0, s, E, h->edges, bs.tl);
        size_t t = bs.tmp_bytes;
        if (!q(rocprim::radix_sort_keys(bs.tmp, t, bs.tl, bs.tl_s, (size_t)(2 * E), 0, tbits, s))) goto rfail;
        t = bs.tmp_bytes;
        if (!q(rocprim::unique(bs.tmp, t, bs.tl_s, h->times, bs.cnt, (size_t)(2 * E),
                               rocprim::equal_to<int64_t>(), s)))
            goto rfail;
        // slots of H: unique sorted keys r nt + c
        hipLaunchKernelGGL(gb_keys_kernel, dim3(nblk(std::max(E, nt_ub))), dim3(256), 0, s, E, h->edges,
                           h->times, bs.cnt, nt_ub, bs.rb, bs.ra, bs.keys, bs.bkey, bs.bval);
        t = bs.tmp_bytes;
        if (!q(rocprim::radix_sort_keys(bs.tmp, t, bs.keys, bs.keys_s, (size_t)K, 0, 64, s))) goto rfail;
        t = bs.tmp_bytes;
        if (!q(rocprim::unique(bs.tmp, t, bs.keys_s, bs.ukeys, bs.cnt + 1, (size_t)K,
                               rocprim::equal_to<int64_t>(), s)))
            goto rfail;
        hipLaunchKernelGGL(gb_count_kernel, dim3(1), dim3(1), 0, s, bs.ukeys, bs.cnt + 1);
        hipLaunchKernelGGL(gb_slots_kernel, dim3(nblk(std::max(K, nt_ub + 1))), dim3(256), 0, s, bs.ukeys,
                           bs.cnt + 1, bs.cnt, nt_ub + 1, h->srow, h->scol, h->dslot, h->rptr);
        // H plan: edge parts grouped by slot, edge order kept (stable sort)
        hipLaunchKernelGGL(gb_parts_kernel, dim3(nblk(4 * E)), dim3(256), 0, s, E, bs.rb, bs.ra, bs.cnt,
                           bs.ukeys, bs.cnt + 1, bs.sl, bs.cval);
        t = bs.tmp_bytes;
        if (!q(rocprim::radix_sort_pairs(bs.tmp, t, bs.sl, bs.sl_s, bs.cval, h->clist, (size_t)(4 * E), 0,
                                         sbits, s)))
            goto rfail;
        hipLaunchKernelGGL(gb_offsets_kernel, dim3(nblk(K + 1)), dim3(256), 0, s, bs.sl_s, 4 * E,
                           bs.cnt + 1, K + 1, h->cptr);
        // b plan: (edge, side) grouped by row, edge order kept
        t = bs.tmp_bytes;
        if (!q(rocprim::radix_sort_pairs(bs.tmp, t, bs.bkey, bs.bkey_s, bs.bval, h->blist, (size_t)(2 * E),
                                         0, tbits, s)))
            goto rfail;
        hipLaunchKernelGGL(gb_offsets_kernel, dim3(nblk(nt_ub + 1)), dim3(256), 0, s, bs.bkey_s, 2 * E,
                           bs.cnt, nt_ub + 1, h->bptr);
        SLAM_HIP_TRY(hipGetLastError());
        // read back through pinned memory: the counts, then the distinct times
        const int64_t need = std::max<int64_t>(2, nt_ub);
        if (h->cnt_cap < need) {
            if (h->cnt_host) SLAM_HIP_TRY(hipHostFree(h->cnt_host));
            h->cnt_host = nullptr;
            h->cnt_cap = 0;
            SLAM_HIP_TRY(hipHostMalloc(&h->cnt_host, (size_t)need * sizeof(int64_t)));
            h->cnt_cap = need;
        }
        SLAM_HIP_TRY(hipMemcpyAsync(h->cnt_host, bs.cnt, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
        const int64_t cnt[2] = {h->cnt_host[0], h->cnt_host[1]};
        SLAM_HIP_TRY(hipMemcpyAsync(h->cnt_host, h->times, cnt[0] * sizeof(int64_t),
                                    hipMemcpyDeviceToHost, s));
        GTRY(finish_structure(h, E, cnt[0], cnt[1]));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
        h->times_h.assign(h->cnt_host, h->cnt_host + cnt[0]);
        return SLAM_OK;
    }
rfail:
    return fail(SLAM_ERR_HIP, "graph structure build: rocPRIM call failed");
qfail:
    return fail(SLAM_ERR_HIP, "graph structure build: rocPRIM size query failed");
}

// the same arrays from a host pass (SLAM_GRAPH_HOST_BUILD=1; the tests compare the two)
int build_structure_host(slam_graph* h, int64_t E, const slam_graph_edge* ed) {
    std::vector<int64_t> tl;
    tl.reserve(2 * E);
    for (int64_t e = 0; e < E; ++e) {
        tl.push_back(ed[e].time_bfr);
        tl.push_back(ed[e].time_aft);
    }
    std::sort(tl.begin(), tl.end());
    tl.erase(std::unique(tl.begin(), tl.end()), tl.end());
    const int64_t nt = (int64_t)tl.size();
    auto rank = [&](int64_t t) { return (int64_t)(std::lower_bound(tl.begin(), tl.end(), t) - tl.begin()); };
    std::vector<int64_t> rb(E), ra(E);
    std::vector<int64_t> keys;
    keys.reserve(4 * E + nt);
    for (int64_t i = 0; i < nt; ++i) keys.push_back(i * nt + i);
    for (int64_t e = 0; e < E; ++e) {
        rb[e] = rank(ed[e].time_bfr);
        ra[e] = rank(ed[e].time_aft);
        keys.push_back(rb[e] * nt + ra[e]);
        keys.push_back(ra[e] * nt + rb[e]);
    }
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const int64_t ns = (int64_t)keys.size();
    auto slot = [&](int64_t r, int64_t c) {
        return (int64_t)(std::lower_bound(keys.begin(), keys.end(), r * nt + c) - keys.begin());
    };
    std::vector<int64_t> srow(ns), scol(ns), rptr(nt + 1, 0), dslot(nt);
    for (int64_t s = 0; s < ns; ++s) {
        srow[s] = keys[s] / nt;
        scol[s] = keys[s] % nt;
        rptr[srow[s] + 1]++;
        if (srow[s] == scol[s]) dslot[srow[s]] = s;
    }
    for (int64_t i = 0; i < nt; ++i) rptr[i + 1] += rptr[i];
    // accumulation plan, stable in edge order (updateEstPose :484-492)
    std::vector<int64_t> cnt(ns + 1, 0), sl(4 * E);
    for (int64_t e = 0; e < E; ++e) {
        sl[4 * e + 0] = slot(rb[e], rb[e]);
        sl[4 * e + 1] = slot(rb[e], ra[e]);
        sl[4 * e + 2] = slot(ra[e], rb[e]);
        sl[4 * e + 3] = slot(ra[e], ra[e]);
        for (int k = 0; k < 4; ++k) cnt[sl[4 * e + k] + 1]++;
    }
    for (int64_t s = 0; s < ns; ++s) cnt[s + 1] += cnt[s];
    std::vector<int64_t> cptr = cnt, clist(4 * E);
    for (int64_t c = 0; c < 4 * E; ++c) clist[cnt[sl[c]]++] = c;     // c = 4 e + part
    std::vector<int64_t> bc(nt + 1, 0), blist(2 * E);
    for (int64_t e = 0; e < E; ++e) {
        bc[rb[e] + 1]++;
        bc[ra[e] + 1]++;
    }
    for (int64_t i = 0; i < nt; ++i) bc[i + 1] += bc[i];
    std::vector<int64_t> bptr = bc;
    for (int64_t e = 0; e < E; ++e) {
        blist[bc[rb[e]]++] = 2 * e;
        blist[bc[ra[e]]++] = 2 * e + 1;
    }
    // device buffers (the same carve as the device build)
    GTRY(carve_edge_set(h, E, std::min<int64_t>(2 * E, h->T), 0, nullptr));
    h->times_h = tl;
    GTRY(finish_structure(h, E, nt, ns));
    SLAM_HIP_TRY(hipMemcpyAsync(h->edges, ed, E * sizeof(slam_graph_edge), hipMemcpyHostToDevice,
                                h->stream));
    GTRY(upload(h, h->times, tl));
    GTRY(upload(h, h->srow, srow));
    GTRY(upload(h, h->scol, scol));
    GTRY(upload(h, h->rptr, rptr));
    GTRY(upload(h, h->cptr, cptr));
    GTRY(upload(h, h->clist, clist));
    GTRY(upload(h, h->bptr, bptr));
    GTRY(upload(h, h->blist, blist));
    GTRY(upload(h, h->dslot, dslot));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int build_structure(slam_graph* h, int64_t E, const slam_graph_edge* ed) {
    const char* hb = std::getenv("SLAM_GRAPH_HOST_BUILD");
    if (hb && hb[0] == '1') return build_structure_host(h, E, ed);
    return build_structure_device(h, E, ed);
}

GraphConst gconst(const slam_graph_config& c) { return GraphConst{c.r_dist, c.r_dir, c.r_orient}; }

int linearize_assemble(slam_graph* h) {
    SLAM_HIP_TRY(hipEventRecord(h->ev[0], h->stream));
    hipLaunchKernelGGL(graph_linearize_kernel, dim3(nblk(h->E)), dim3(256), 0, h->stream, h->E,
                       h->edges, h->poses, gconst(h->cfg), h->blocks);
    SLAM_HIP_TRY(hipEventRecord(h->ev[1], h->stream));
    hipLaunchKernelGGL(graph_assemble_h_kernel, dim3(nblk(9 * h->n_slots)), dim3(256), 0,
                       h->stream, h->n_slots, h->E, h->cptr, h->clist, h->blocks, h->cfg.anchor,
                       h->val);
    hipLaunchKernelGGL(graph_assemble_b_kernel, dim3(nblk(3 * h->nt)), dim3(256), 0, h->stream,
                       h->nt, h->E, h->bptr, h->blist, h->blocks, h->b);
    SLAM_HIP_TRY(hipEventRecord(h->ev[2], h->stream));
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int dense_matrix(slam_graph* h) {
    const int64_t n = 3 * h->nt;
    SLAM_HIP_TRY(hipMemsetAsync(h->A, 0, n * n * sizeof(double), h->stream));
    hipLaunchKernelGGL(graph_dense_scatter_kernel, dim3(nblk(9 * h->n_slots)), dim3(256), 0,
                       h->stream, h->n_slots, h->srow, h->scol, h->val, n, h->A);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// dense path: det, cond, gate, delta (updateEstPose :494-502)
int solve_dense(slam_graph* h, double* stats, bool* solved) {
    const int64_t n = 3 * h->nt;
    GTRY(dense_matrix(h));
    SLAM_HIP_TRY(hipMemcpyAsync(h->LU, h->A, n * n * sizeof(double), hipMemcpyDeviceToDevice,
                                h->stream));
    hipLaunchKernelGGL(graph_symmetrize_kernel, dim3(nblk(n * n)), dim3(256), 0, h->stream, h->A, n,
                       h->S);
    hipLaunchKernelGGL(graph_lu_kernel, dim3(1), dim3(kGraphThreads), 0, h->stream, h->LU, (int)n,
                       h->piv, h->luout);
    hipLaunchKernelGGL(graph_lanczos_kernel, dim3(1), dim3(kGraphThreads), 0, h->stream, h->S,
                       (int)n, h->V, h->lan, h->lan + n, h->lan + 2 * n, h->luout + 3,
                       (uint64_t)0x5EEDULL);
    SLAM_HIP_TRY(hipGetLastError());
    double lo[5];
    SLAM_HIP_TRY(hipMemcpyAsync(lo, h->luout, 5 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    // numpy det: sign * exp(logdet); a zero pivot gives 0 (getrf info > 0)
    const double det = (lo[2] != 0.0) ? 0.0 : lo[0] * std::exp(lo[1]);
    const double cond = (lo[4] > 0.0) ? lo[3] / lo[4] : std::numeric_limits<double>::infinity();
    stats[2] = det;
    stats[3] = cond;
    *solved = (h->cfg.det_min < det) && (cond < h->cfg.cond_max);
    if (*solved)
        hipLaunchKernelGGL(graph_lu_solve_kernel, dim3(1), dim3(kGraphThreads), 0, h->stream,
                           h->LU, (int)n, h->piv, h->b, h->delta);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// the estimate's stall window (kCondWin; SLAM_GRAPH_COND_WIN 2..32 for A/B)
static int cond_win() {
    static const int w = [] {
        const char* e = std::getenv("SLAM_GRAPH_COND_WIN");
        const int v = e ? std::atoi(e) : 0;
        return (v >= 2 && v <= 32) ? v : kCondWin;
    }();
    return w;
}

// condition-number estimate (graph_kernels.inl: LOBPCG for the extreme
// eigenvalues) on h->cstream, enqueued in batches of `count` iterations
// starting at iteration k0 (k0 = 0: the start sequence first).
// The certificate mode's early decision of the estimate (CondState.etol): both
// sides moved less than 1e-3 (relative) over 8 iterations and the estimate
// clears cond_max by a factor 100 (status 5).  A Ritz ratio under-estimates
// cond, so the factor is the margin the VERDICT r4 asked for; with the
// tight test (1e-5 over 16, status 1) the gate keeps a factor 10.
constexpr double kCertEarlyTol = 1e-3, kCertEarlyMargin = 100.0, kCertConvMargin = 10.0;
constexpr int kCertEarlyWin = 8;

int cond_enqueue(slam_graph* h, int32_t k0, int32_t count) {
    const int64_t n = 3 * h->nt;
    const bool early = h->cfg.cond_mode == SLAM_GRAPH_COND_MARGIN;
    const unsigned nb = nblk(n, kPcgThreads);
    hipStream_t s = h->cstream;
    const double tol = h->cfg.cond_tol > 0.0 ? h->cfg.cond_tol : 1e-5;
    const int32_t mx = h->cfg.cond_max_iter > 0 ? h->cfg.cond_max_iter : 3000;
    int32_t k = k0;
    // merged (default): the SpMV launch's last workgroup folds and decides
    // the iteration (two launches per iteration); SLAM_GRAPH_COND_MERGED=0
    // keeps the separate one-workgroup fold launch (same totals, A/B)
    static const bool merged = [] {
        const char* e = std::getenv("SLAM_GRAPH_COND_MERGED");
        return !(e && e[0] == '0');
    }();
    if (merged) {
        if (k0 == 0) {
            hipLaunchKernelGGL(graph_cond_init_kernel, dim3(nblk(2 * n)), dim3(256), 0, s, n,
                               h->cond_warm ? 0 : 1, cond_win(), h->cx, h->cp, h->chp, h->cst,
                               early ? kCertEarlyTol : 0.0, kCertEarlyWin, kCertEarlyMargin);
            hipLaunchKernelGGL((graph_cond_spmv_kernel<true, true>), dim3(nb), dim3(kSpmvThreads), 0, s,
                               h->nt, h->rptr, h->scol, h->val, h->cx, h->chx, h->cw, h->cw2, h->chw,
                               h->cp, h->chp, h->cpart, h->cst, 0, tol, mx, h->cfg.cond_max);
            hipLaunchKernelGGL(graph_cond_update_kernel, dim3(nb), dim3(kPcgThreads), 0, s, n, 0,
                               h->minv, h->cx, h->chx, h->cw2, h->chw, h->cp, h->chp, h->cw,
                               h->cpart, h->cst);
            k = 1;
        }
        for (; k < k0 + count; ++k) {
            hipLaunchKernelGGL((graph_cond_spmv_kernel<false, true>), dim3(nb), dim3(kSpmvThreads), 0,
                               s, h->nt, h->rptr, h->scol, h->val, h->cx, h->chx, h->cw, h->cw2,
                               h->chw, h->cp, h->chp, h->cpart, h->cst, k, tol, mx, h->cfg.cond_max);
            hipLaunchKernelGGL(graph_cond_update_kernel, dim3(nb), dim3(kPcgThreads), 0, s, n, k,
                               h->minv, h->cx, h->chx, h->cw2, h->chw, h->cp, h->chp, h->cw,
                               h->cpart, h->cst);
        }
        SLAM_HIP_TRY(hipGetLastError());
        return SLAM_OK;
    }
    if (k0 == 0) {
        hipLaunchKernelGGL(graph_cond_init_kernel, dim3(nblk(2 * n)), dim3(256), 0, s, n,
                           h->cond_warm ? 0 : 1, cond_win(), h->cx, h->cp, h->chp, h->cst,
                           early ? kCertEarlyTol : 0.0, kCertEarlyWin, kCertEarlyMargin);
        hipLaunchKernelGGL(graph_cond_spmv_kernel<true>, dim3(nb), dim3(kSpmvThreads), 0, s, h->nt,
                           h->rptr, h->scol, h->val, h->cx, h->chx, h->cw, h->cw2, h->chw, h->cp,
                           h->chp, h->cpart, h->cst);
        hipLaunchKernelGGL(graph_cond_fold_kernel, dim3(1), dim3(kCondFoldThreads), 0, s,
                           (int64_t)nb, h->cpart, h->cst, 0, tol, mx, h->cfg.cond_max);
        hipLaunchKernelGGL(graph_cond_update_kernel, dim3(nb), dim3(kPcgThreads), 0, s, n, 0,
                           h->minv, h->cx, h->chx, h->cw2, h->chw, h->cp, h->chp, h->cw, h->cpart,
                           h->cst);
        k = 1;
    }
    for (; k < k0 + count; ++k) {
        hipLaunchKernelGGL(graph_cond_spmv_kernel<false>, dim3(nb), dim3(kSpmvThreads), 0, s, h->nt,
                           h->rptr, h->scol, h->val, h->cx, h->chx, h->cw, h->cw2, h->chw, h->cp,
                           h->chp, h->cpart, h->cst);
        hipLaunchKernelGGL(graph_cond_fold_kernel, dim3(1), dim3(kCondFoldThreads), 0, s,
                           (int64_t)nb, h->cpart, h->cst, k, tol, mx, h->cfg.cond_max);
        hipLaunchKernelGGL(graph_cond_update_kernel, dim3(nb), dim3(kPcgThreads), 0, s, n, k,
                           h->minv, h->cx, h->chx, h->cw2, h->chw, h->cp, h->chp, h->cw, h->cpart,
                           h->cst);
    }
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// ---- the gate's certificate (SLAM_GRAPH_COND_MARGIN; graph_kernels.inl)
// The certificate's sums on the second stream beside the PCG (after the
// block-Jacobi inverses): one lane per pose, one per block slot, one fold.
int cert_enqueue(slam_graph* h) {
    hipStream_t s = h->cstream;
    const unsigned nbp = nblk(h->nt, kCertThreads), nbs = nblk(h->n_slots, kCertThreads);
    hipLaunchKernelGGL(graph_cert_pose_kernel, dim3(nbp), dim3(kCertThreads), 0, s, h->nt, h->dslot,
                       h->val, h->minv, h->cert_part);
    hipLaunchKernelGGL(graph_cert_slot_kernel, dim3(nbs), dim3(kCertThreads), 0, s, h->n_slots,
                       h->srow, h->scol, h->val, h->minv, h->cert_part + 4 * (int64_t)nbp);
    hipLaunchKernelGGL(graph_cert_fold_kernel, dim3(1), dim3(kCertThreads), 0, s, (int64_t)nbp,
                       h->cert_part, (int64_t)nbs, h->cert_part + 4 * (int64_t)nbp, h->cert);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(h->cert_host, h->cert, sizeof(CertState), hipMemcpyDeviceToHost, s));
    return SLAM_OK;
}

// det(H) from the dense LU (n <= kGraphDenseMax): the certificate's fallback
int dense_det(slam_graph* h, double* det) {
    const int64_t n = 3 * h->nt;
    GTRY(dense_matrix(h));
    SLAM_HIP_TRY(hipMemcpyAsync(h->LU, h->A, n * n * sizeof(double), hipMemcpyDeviceToDevice,
                                h->stream));
    hipLaunchKernelGGL(graph_lu_kernel, dim3(1), dim3(kGraphThreads), 0, h->stream, h->LU, (int)n,
                       h->piv, h->luout);
    SLAM_HIP_TRY(hipGetLastError());
    double lo[3];
    SLAM_HIP_TRY(hipMemcpyAsync(lo, h->luout, 3 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    *det = (lo[2] != 0.0) ? 0.0 : lo[0] * std::exp(lo[1]);
    return SLAM_OK;
}

// cond(H) by the dense path's Lanczos (n <= kGraphDenseMax): the certificate's fallback
int dense_cond(slam_graph* h, double* cond) {
    const int64_t n = 3 * h->nt;
    GTRY(dense_matrix(h));
    hipLaunchKernelGGL(graph_symmetrize_kernel, dim3(nblk(n * n)), dim3(256), 0, h->stream, h->A, n,
                       h->S);
    hipLaunchKernelGGL(graph_lanczos_kernel, dim3(1), dim3(kGraphThreads), 0, h->stream, h->S,
                       (int)n, h->V, h->lan, h->lan + n, h->lan + 2 * n, h->luout + 3,
                       (uint64_t)0x5EEDULL);
    SLAM_HIP_TRY(hipGetLastError());
    double lo[2];
    SLAM_HIP_TRY(hipMemcpyAsync(lo, h->luout + 3, 2 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    *cond = (lo[1] > 0.0) ? lo[0] / lo[1] : std::numeric_limits<double>::infinity();
    return SLAM_OK;
}

// The gate (:494-496) in the estimate-with-margin mode (SLAM_GRAPH_COND_MARGIN,
// formerly named CERTIFY), from the LOBPCG estimate (cs, run beside the PCG
// with the early decision) and the log-det sums (ct).  Not a certificate: the
// estimate's Ritz value over-estimates lambda_min(H), so each half passes
// only with a margin against that error (VERDICT / ADVICE r5):
//  * cond: the Ritz ratio under-estimates cond; status 5 (the early stop)
//    passes with cond x 100 < cond_max, status 1 (tightly converged) with cond
//    x 10 < cond_max, and a converged estimate inside that band is decided by
//    the estimate itself (decision 5, as SLAM_GRAPH_COND_ESTIMATE does: the
//    reference applies such updates); status 2 / 4 rejects (cond >= cond_max,
//    or not positive definite, for certain); anything else is undecided;
//  * det: log det H in [log det M + c(a) (tr(P^2) - n), log det M] (Fischer
//    above; the quadratic bound of ln below, valid for any a <= lambda_min(P),
//    graph_kernels.inl), with a = lambda~min(H) / (F max tr M_i), F =
//    kGateDetMargin = 1000: the lower end stays a bound unless the Ritz value
//    over-estimates lambda_min(H) by more than F (lambda_min(P) >= lambda_min(H)
//    / lambda_max(M) >= lambda_min(H) / max tr M_i).  gate_info reports the
//    largest factor the decision tolerates (det_margin).  Passes above ln
//    det_min, rejects below the upper end (rigorous), undecided inside;
// an undecided half takes the dense path's own det / Lanczos cond when n <=
// kGraphDenseMax, otherwise the update is not solved and gate_info says
// "undecided" (a possible parity gap, not a rejection).
// SLAM_GRAPH_GATE_RITZ_SCALE=<f> (diagnostic, tests): the gate uses f x the
// estimate's lambda_min, emulating an estimate that over-estimates it by f.
constexpr double kGateDetMargin = 1000.0;

double gate_ritz_scale() {
    const char* e = std::getenv("SLAM_GRAPH_GATE_RITZ_SCALE");
    const double f = e ? std::atof(e) : 1.0;
    return f > 0.0 ? f : 1.0;
}

// the log-det lower end for lambda_min(P) >= a
double logdet_lower(const CertState& ct, const double a, const int64_t n) {
    const double c = (std::log(a) - a + 1.0) / ((a - 1.0) * (a - 1.0));
    return ct.logdet_m + c * std::max(0.0, ct.trp2 - (double)n);
}

int cert_gate(slam_graph* h, const CondState& cs, double* stats, bool* gate) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t n = 3 * h->nt;
    SLAM_HIP_TRY(hipStreamSynchronize(h->cstream));
    const CertState ct = *h->cert_host;
    const double lam0 = cs.lam[0] * gate_ritz_scale();
    double* g = h->gate_info;
    g[0] = 1.0;
    g[6] = lam0;
    g[7] = cs.lam[1];
    g[8] = ct.trp2;
    g[9] = (double)n;
    g[10] = cs.iter;
    // ---- cond (:495)
    const double inf = std::numeric_limits<double>::infinity();
    double cond = (cs.status == 4 || !(lam0 > 0.0)) ? inf : cs.lam[1] / lam0;
    int cond_dec;
    if ((cs.status == 5 && kCertEarlyMargin * cond < h->cfg.cond_max) ||
        (cs.status == 1 && kCertConvMargin * cond < h->cfg.cond_max))
        cond_dec = 1;
    else if (cs.status == 1 && cond < h->cfg.cond_max) cond_dec = 5;    // converged, inside the band
    else if (cs.status == 2 || cs.status == 4) cond_dec = 0;
    else cond_dec = -1;
    if (cond_dec < 0 && n <= kGraphDenseMax) {
        GTRY(dense_cond(h, &cond));
        cond_dec = cond < h->cfg.cond_max ? 3 : 2;
    }
    g[2] = cond_dec;
    g[5] = cond;
    g[13] = (cond > 0.0) ? h->cfg.cond_max / cond : inf;
    // ---- det (:494)
    const double ln_min = h->cfg.det_min > 0.0 ? std::log(h->cfg.det_min) : -inf;
    const double hi = ct.logdet_m;                 // Fischer: det H <= prod det M_i
    const bool have = ct.bad == 0 && lam0 > 0.0 && ct.trm_max > 0.0 && cs.status != 4;
    const double a1 = have ? lam0 / ct.trm_max : 0.0;     // a at margin 1
    double lo = -inf;
    if (have) lo = logdet_lower(ct, a1 / kGateDetMargin, n);
    // the largest margin F with the lower end still above ln det_min (lo falls as a does)
    double fmax = 0.0;
    if (have && logdet_lower(ct, a1, n) > ln_min) {
        double l = 0.0, u = 700.0;                 // ln F
        if (logdet_lower(ct, a1 * std::exp(-u), n) > ln_min) l = u;
        for (int it = 0; it < 60 && u - l > 1e-3; ++it) {
            const double m = 0.5 * (l + u);
            if (logdet_lower(ct, a1 * std::exp(-m), n) > ln_min) l = m;
            else u = m;
        }
        fmax = std::exp(l);
    }
    g[3] = lo;
    g[4] = hi;
    g[12] = fmax;
    int det_dec;
    double det;
    if (ct.bad == 0 && lo > ln_min) {
        det_dec = 1;                               // passed with the margin
        det = std::exp(lo);                        // det >= this unless the margin failed (inf past the double range, as numpy)
    } else if (ct.bad == 0 && hi < ln_min) {
        det_dec = 0;                               // rejected by the upper bound
        det = std::exp(hi);                        // det <= this
    } else if (n <= kGraphDenseMax) {
        GTRY(dense_det(h, &det));                  // the reference's own det (numpy's LU)
        det_dec = (h->cfg.det_min < det) ? 3 : 2;
    } else {
        det_dec = -1;
        det = std::numeric_limits<double>::quiet_NaN();
    }
    g[1] = det_dec;
    g[0] = (det_dec >= 2 || (cond_dec >= 2 && cond_dec <= 3)) ? 2.0 : 1.0;   // 2: a half took the dense path's value
    stats[2] = det;
    stats[3] = cond;
    *gate = (det_dec == 1 || det_dec == 3) && (cond_dec == 1 || cond_dec == 3 || cond_dec == 5);
    g[11] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return SLAM_OK;
}

// PCG on H delta = -b with block-Jacobi (large trajectories): two launches per
// iteration, enqueued in chunks between host polls of the device state.  The
// gate's condition number (:495) is estimated on a second stream at the same
// time (cond_mode SLAM_GRAPH_COND_ESTIMATE); the solve is applied only if the
// gate passes, as the reference inverts H only then (:496-497).
int solve_pcg(slam_graph* h, double* stats, bool* solved, int32_t* iters) {
    const int64_t n = 3 * h->nt;
    const unsigned nb = nblk(n, kPcgThreads);
    const bool cert = (h->cfg.cond_mode == SLAM_GRAPH_COND_MARGIN);
    const bool est = (h->cfg.cond_mode == SLAM_GRAPH_COND_ESTIMATE) || cert;   // the estimate runs
    hipLaunchKernelGGL(graph_block_inv_kernel, dim3(nblk(h->nt)), dim3(256), 0, h->stream, h->nt,
                       h->dslot, h->val, h->minv);
    if (est) {
        SLAM_HIP_TRY(hipEventRecord(h->cev[0], h->stream));
        SLAM_HIP_TRY(hipStreamWaitEvent(h->cstream, h->cev[0], 0));
        SLAM_HIP_TRY(hipEventRecord(h->cev[1], h->cstream));
    }
    if (cert) GTRY(cert_enqueue(h));
    hipLaunchKernelGGL(graph_pcg_start_kernel, dim3(nb), dim3(kPcgThreads), 0, h->stream, n,
                       h->minv, h->b, h->delta, h->r, h->z, h->part);
    SLAM_HIP_TRY(hipGetLastError());
    PcgState& s = *h->pcg_host;
    CondState& cs = *h->cond_host;
    s = PcgState{};
    cs = CondState{};
    // The first batch runs through the previous solve's iteration count (the
    // Gauss-Newton steps of one edge set converge in similar counts), so a
    // repeated solve usually needs a single host poll; then batches of 8.
    int32_t k_end = std::max<int32_t>(16, std::min<int32_t>(h->pcg_last_iters + 1, 1024));
    int32_t c_end = std::max<int32_t>(cond_win() + 1, std::min<int32_t>(h->cond_last_iters + 1, 1024));
    bool pcg_done = false, cond_done = !est, abandoned = false;
    int32_t k0 = 0, c0 = 0;
    while (!pcg_done || !cond_done) {
        // the two streams' launches interleaved in proportion to their batch
        // lengths, so the estimate starts with the solve instead of after the
        // host has enqueued the whole PCG batch (~1 ms of launch calls)
        const int32_t np = pcg_done ? 0 : k_end - k0;
        const int32_t nc = cond_done ? 0 : c_end - c0;
        for (int32_t ip = 0, ic = 0; ip < np || ic < nc;) {
            if (ic < nc && (ip >= np || (int64_t)ic * np <= (int64_t)ip * nc)) {
                GTRY(cond_enqueue(h, c0 + ic, 1));
                ++ic;
            } else {
                const int32_t k = k0 + ip;
                hipLaunchKernelGGL(graph_pcg_dir_spmv_kernel, dim3(nb), dim3(kSpmvThreads), 0,
                                   h->stream, h->nt, k, h->rptr, h->scol, h->val, h->z, h->p, h->q,
                                   h->part, h->st, h->cfg.pcg_tol, h->cfg.pcg_max_iter);
                hipLaunchKernelGGL(graph_pcg_step_kernel, dim3(nb), dim3(kPcgThreads), 0, h->stream,
                                   n, k, h->minv, h->p, h->q, h->delta, h->r, h->z, h->part, h->st);
                ++ip;
            }
        }
        SLAM_HIP_TRY(hipGetLastError());
        if (!pcg_done)
            SLAM_HIP_TRY(hipMemcpyAsync(h->pcg_host, h->st, sizeof(PcgState), hipMemcpyDeviceToHost,
                                        h->stream));
        if (!cond_done)
            SLAM_HIP_TRY(hipMemcpyAsync(h->cond_host, h->cst, sizeof(CondState), hipMemcpyDeviceToHost,
                                        h->cstream));
        if (!pcg_done) {
            SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
            pcg_done = s.done;
            k0 = k_end;
            k_end += 8;
        }
        if (!cond_done) {
            SLAM_HIP_TRY(hipStreamSynchronize(h->cstream));
            cond_done = cs.done;
            c0 = c_end;
            c_end += 16;
            // the gate rejects H for certain (cond >= cond_max, or not positive
            // definite): the reference does not solve (:496), neither do we
            if (cs.done && (cs.status == 2 || cs.status == 4) && !pcg_done) {
                pcg_done = true;
                abandoned = true;
            }
        }
    }
    *iters = s.iter;
    h->pcg_last_iters = (s.status == 1) ? s.iter : 0;
    const bool pcg_ok = (s.status == 1);
    stats[2] = std::numeric_limits<double>::quiet_NaN();     // det: not formed at this size
    stats[3] = std::numeric_limits<double>::quiet_NaN();
    bool gate = true;
    for (double& v : h->cond_info) v = 0.0;
    for (double& v : h->gate_info) v = 0.0;
    if (est) {
        SLAM_HIP_TRY(hipEventRecord(h->cev[2], h->cstream));
        SLAM_HIP_TRY(hipEventSynchronize(h->cev[2]));
        float ms = 0.f;
        SLAM_HIP_TRY(hipEventElapsedTime(&ms, h->cev[1], h->cev[2]));
        const double cond = (cs.status == 4 || !(cs.lam[0] > 0.0))
                                ? std::numeric_limits<double>::infinity()
                                : cs.lam[1] / cs.lam[0];
        stats[3] = cond;
        // :496 -- only a converged estimate certifies cond < cond_max: Ritz
        // values lie inside [lambda_min, lambda_max], so an estimate stopped
        // at cond_max_iter (status 3) only bounds cond from below and cannot
        // pass the gate; status 2 / 4 reject for certain
        gate = (cs.status == 1) && cond < h->cfg.cond_max;
        h->cond_warm = (cs.status == 1 || cs.status == 3 || cs.status == 5);
        h->cond_last_iters = (cs.status == 1 || cs.status == 5) ? cs.iter : 0;
        h->cond_info[0] = cs.iter;
        h->cond_info[1] = cs.status;
        h->cond_info[2] = cs.lam[0];
        h->cond_info[3] = cs.lam[1];
        h->cond_info[4] = cs.iters_side[0];
        h->cond_info[5] = cs.iters_side[1];
        h->cond_info[6] = ms;
        if (cert && pcg_ok && !abandoned) GTRY(cert_gate(h, cs, stats, &gate));
    }
    *solved = pcg_ok && gate && !abandoned;
    h->pcg_failed = !pcg_ok && !abandoned;
    if (abandoned) {
        *iters = -1;
        h->pcg_last_iters = 0;
    }
    return SLAM_OK;
}

int do_update(slam_graph* h, double* stats) {
    stats[0] = stats[1] = stats[2] = stats[3] = 0.0;
    for (double& x : h->last) x = 0.0;
    h->pcg_failed = false;
    if (h->E == 0 || 3 * h->nt <= 3) return SLAM_OK;        // :469 (leng > 3)
    GTRY(linearize_assemble(h));
    const int64_t n = 3 * h->nt;
    const bool dense = (h->cfg.solver == SLAM_GRAPH_DENSE) ||
                       (h->cfg.solver == SLAM_GRAPH_AUTO && n <= kGraphDenseMax);
    if (dense && n > kGraphDenseMax)
        return fail(SLAM_ERR_ARG, "slam_graph_update: dense solver limited to 2048 unknowns");
    bool solved = false;
    int32_t iters = 0;
    if (dense) GTRY(solve_dense(h, stats, &solved));
    else GTRY(solve_pcg(h, stats, &solved, &iters));
    SLAM_HIP_TRY(hipEventRecord(h->ev[3], h->stream));
    if (solved) {
        hipLaunchKernelGGL(graph_pose_update_kernel, dim3(nblk(h->nt)), dim3(256), 0, h->stream,
                           h->nt, h->times, h->delta, h->poses, h->part);
        hipLaunchKernelGGL(graph_dsum_kernel, dim3(1), dim3(1024), 0, h->stream,
                           (int64_t)nblk(h->nt), h->part, h->dsum);
        SLAM_HIP_TRY(hipGetLastError());
        SLAM_HIP_TRY(hipMemcpyAsync(&stats[1], h->dsum, sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
        stats[0] = 1.0;
    }
    SLAM_HIP_TRY(hipEventRecord(h->ev[4], h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    float ms;
    for (int k = 0; k < 4; ++k) {
        SLAM_HIP_TRY(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1]));
        h->last[k] = ms;
    }
    h->last[4] = iters;
    return SLAM_OK;
}

}  // namespace

extern "C" {

int slam_graph_create(const slam_graph_config* cfg, int device, slam_graph** out) {
    SLAM_ARG_CHECK(cfg && out, "slam_graph_create: NULL argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(SLAM_ERR_ARG, "slam_graph_create: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    slam_graph* h = new slam_graph();
    h->cfg = *cfg;
    if (h->cfg.pcg_max_iter <= 0) h->cfg.pcg_max_iter = 10000;
    if (!(h->cfg.cond_tol > 0.0)) h->cfg.cond_tol = 1e-5;
    if (h->cfg.cond_max_iter <= 0) h->cfg.cond_max_iter = 3000;
    if (!(h->cfg.pcg_tol > 0.0)) h->cfg.pcg_tol = 1e-10;
    h->device = device;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking) != hipSuccess) {
        slam_graph_destroy(h);
        return fail(SLAM_ERR_HIP, "slam_graph_create: stream creation failed");
    }
    for (auto& e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) {
            slam_graph_destroy(h);
            return fail(SLAM_ERR_HIP, "slam_graph_create: event creation failed");
        }
    for (auto& e : h->cev)
        if (hipEventCreate(&e) != hipSuccess) {
            slam_graph_destroy(h);
            return fail(SLAM_ERR_HIP, "slam_graph_create: event creation failed");
        }
    if (hipHostMalloc(&h->pcg_host, sizeof(PcgState)) != hipSuccess ||
        hipHostMalloc(&h->cond_host, sizeof(CondState)) != hipSuccess ||
        hipHostMalloc(&h->cert_host, sizeof(CertState)) != hipSuccess) {
        slam_graph_destroy(h);
        return fail(SLAM_ERR_HIP, "slam_graph_create: pinned state buffers");
    }
    *out = h;
    return SLAM_OK;
}

int slam_graph_destroy(slam_graph* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    free_list(h->allocs);
    if (h->arena) (void)hipFree(h->arena);
    if (h->poses) (void)hipFree(h->poses);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : h->cev)
        if (e) (void)hipEventDestroy(e);
    if (h->pcg_host) (void)hipHostFree(h->pcg_host);
    if (h->cnt_host) (void)hipHostFree(h->cnt_host);
    if (h->cond_host) (void)hipHostFree(h->cond_host);
    if (h->cert_host) (void)hipHostFree(h->cert_host);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_graph_set_poses(slam_graph* h, int64_t n_poses, const double* poses) {
    SLAM_ARG_CHECK(h && poses && n_poses >= 1, "slam_graph_set_poses: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (n_poses != h->T) {
        if (h->poses) SLAM_HIP_TRY(hipFree(h->poses));
        h->poses = nullptr;
        SLAM_HIP_TRY(hipMalloc(&h->poses, 3 * n_poses * sizeof(double)));
        h->T = n_poses;
    }
    SLAM_HIP_TRY(hipMemcpyAsync(h->poses, poses, 3 * n_poses * sizeof(double),
                                hipMemcpyHostToDevice, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_graph_get_poses(slam_graph* h, double* poses) {
    SLAM_ARG_CHECK(h && poses && h->poses, "slam_graph_get_poses: no poses");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    SLAM_HIP_TRY(hipMemcpyAsync(poses, h->poses, 3 * h->T * sizeof(double), hipMemcpyDeviceToHost,
                                h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_graph_set_edges(slam_graph* h, int64_t n_edges, const slam_graph_edge* edges) {
    SLAM_ARG_CHECK(h && n_edges >= 0 && (edges || n_edges == 0), "slam_graph_set_edges: bad arguments");
    SLAM_ARG_CHECK(h->poses, "slam_graph_set_edges: set the poses first");
    for (int64_t e = 0; e < n_edges; ++e) {
        const slam_graph_edge& d = edges[e];
        SLAM_ARG_CHECK(d.pose_bfr >= 0 && d.pose_bfr < h->T && d.pose_aft >= 0 && d.pose_aft < h->T &&
                           d.time_bfr >= 0 && d.time_bfr < h->T && d.time_aft >= 0 &&
                           d.time_aft < h->T,
                       "slam_graph_set_edges: pose / time index out of range");
    }
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (n_edges == 0) {
        h->E = h->nt = h->n_slots = 0;
        h->times_h.clear();
        return SLAM_OK;
    }
    return build_structure(h, n_edges, edges);
}

int slam_graph_update(slam_graph* h, double* stats) {
    SLAM_ARG_CHECK(h && stats && h->poses, "slam_graph_update: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    return do_update(h, stats);
}

int slam_graph_optimize(slam_graph* h, double delta_sum_th, int32_t max_iter, double* stats,
                        int32_t* n_iter) {
    SLAM_ARG_CHECK(h && h->poses && max_iter >= 1, "slam_graph_optimize: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int32_t it = 0;
    double s[4] = {0, 0, 0, 0};
    double dsum = delta_sum_th;
    while (delta_sum_th <= dsum && it < max_iter) {            // :692
        GTRY(do_update(h, s));
        if (stats) std::memcpy(stats + 4 * it, s, sizeof(s));
        dsum = s[1];
        ++it;
        // is_calc = 0 ends the loop as in the reference (:706-709: sum delta^2 = 0);
        // on the PCG path that is a solver failure, not a converged trajectory
        if (h->pcg_failed) {
            if (n_iter) *n_iter = it;
            return fail(SLAM_ERR_SOLVE, "slam_graph_optimize: PCG did not converge within "
                                        "pcg_max_iter iterations; poses left at the last "
                                        "converged Gauss-Newton step");
        }
    }
    if (n_iter) *n_iter = it;
    return SLAM_OK;
}

int slam_graph_get_system(slam_graph* h, int64_t* n_times, int64_t* times, double* H, double* b,
                          double* blocks) {
    SLAM_ARG_CHECK(h && n_times, "slam_graph_get_system: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    *n_times = h->nt;
    if (times) std::memcpy(times, h->times_h.data(), h->nt * sizeof(int64_t));
    const int64_t n = 3 * h->nt;
    if (H) {
        SLAM_ARG_CHECK(h->A, "slam_graph_get_system: dense H only up to 2048 unknowns");
        GTRY(dense_matrix(h));
        SLAM_HIP_TRY(hipMemcpyAsync(H, h->A, n * n * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    }
    if (b)
        SLAM_HIP_TRY(hipMemcpyAsync(b, h->b, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (blocks && h->E) {
        std::vector<double> t(42 * h->E);
        SLAM_HIP_TRY(hipMemcpyAsync(t.data(), h->blocks, t.size() * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
        SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
        for (int64_t e = 0; e < h->E; ++e)
            for (int q = 0; q < 42; ++q) blocks[42 * e + q] = t[q * h->E + e];
    }
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_graph_get_bsr(slam_graph* h, int64_t* n_slots, int64_t* rows, int64_t* cols,
                       double* vals) {
    SLAM_ARG_CHECK(h && n_slots, "slam_graph_get_bsr: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    *n_slots = h->n_slots;
    if (rows)
        SLAM_HIP_TRY(hipMemcpyAsync(rows, h->srow, h->n_slots * sizeof(int64_t),
                                    hipMemcpyDeviceToHost, h->stream));
    if (cols)
        SLAM_HIP_TRY(hipMemcpyAsync(cols, h->scol, h->n_slots * sizeof(int64_t),
                                    hipMemcpyDeviceToHost, h->stream));
    if (vals)
        SLAM_HIP_TRY(hipMemcpyAsync(vals, h->val, 9 * h->n_slots * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_graph_get_delta(slam_graph* h, double* delta) {
    SLAM_ARG_CHECK(h && delta, "slam_graph_get_delta: bad arguments");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (h->nt)
        SLAM_HIP_TRY(hipMemcpyAsync(delta, h->delta, 3 * h->nt * sizeof(double),
                                    hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    return SLAM_OK;
}

int slam_graph_timing(slam_graph* h, double* out) {
    SLAM_ARG_CHECK(h && out, "slam_graph_timing: NULL argument");
    for (int k = 0; k < 5; ++k) out[k] = h->last[k];
    return SLAM_OK;
}

int slam_graph_cond_info(slam_graph* h, double* out) {
    SLAM_ARG_CHECK(h && out, "slam_graph_cond_info: NULL argument");
    for (int k = 0; k < 7; ++k) out[k] = h->cond_info[k];
    return SLAM_OK;
}

int slam_graph_gate_info(slam_graph* h, double* out) {
    SLAM_ARG_CHECK(h && out, "slam_graph_gate_info: NULL argument");
    for (int k = 0; k < kGateInfo; ++k) out[k] = h->gate_info[k];
    return SLAM_OK;
}

int slam_graph_pair_halves(int64_t n_halves, const slam_graph_half* halves, int64_t n_landmarks,
                           int device, int64_t* n_edges, slam_graph_edge* edges) {
    SLAM_ARG_CHECK(n_edges && n_halves >= 0 && n_landmarks >= 0 && (halves || n_halves == 0),
                   "slam_graph_pair_halves: bad arguments");
    // stable grouping by landmark id (counting sort), pair offsets per landmark
    std::vector<int64_t> lm_start(n_landmarks + 1, 0);
    for (int64_t q = 0; q < n_halves; ++q) {
        const int64_t l = halves[q].landmark;
        if (l >= 0 && l < n_landmarks) lm_start[l + 1]++;
    }
    std::vector<int64_t> pair_off(n_landmarks + 1, 0);
    for (int64_t l = 0; l < n_landmarks; ++l) {
        const int64_t m = lm_start[l + 1];
        pair_off[l + 1] = pair_off[l] + m * (m - 1) / 2;
        lm_start[l + 1] += lm_start[l];
    }
    const int64_t E = pair_off[n_landmarks];
    *n_edges = E;
    if (!edges || E == 0) return SLAM_OK;
    std::vector<slam_graph_half> grouped(lm_start[n_landmarks]);
    {
        std::vector<int64_t> fill(lm_start.begin(), lm_start.end() - 1);
        for (int64_t q = 0; q < n_halves; ++q) {
            const int64_t l = halves[q].landmark;
            if (l >= 0 && l < n_landmarks) grouped[fill[l]++] = halves[q];
        }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(SLAM_ERR_ARG, "slam_graph_pair_halves: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    int64_t *d_off = nullptr, *d_start = nullptr;
    slam_graph_half* d_half = nullptr;
    slam_graph_edge* d_edges = nullptr;
    int rc = SLAM_OK;
    if (hipMalloc(&d_off, pair_off.size() * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&d_start, lm_start.size() * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&d_half, grouped.size() * sizeof(slam_graph_half)) != hipSuccess ||
        hipMalloc(&d_edges, (size_t)E * sizeof(slam_graph_edge)) != hipSuccess) {
        rc = fail(SLAM_ERR_HIP, "slam_graph_pair_halves: device allocation failed");
    } else if (hipMemcpy(d_off, pair_off.data(), pair_off.size() * sizeof(int64_t),
                         hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(d_start, lm_start.data(), lm_start.size() * sizeof(int64_t),
                         hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(d_half, grouped.data(), grouped.size() * sizeof(slam_graph_half),
                         hipMemcpyHostToDevice) != hipSuccess) {
        rc = fail(SLAM_ERR_HIP, "slam_graph_pair_halves: upload failed");
    } else {
        hipLaunchKernelGGL(graph_pair_kernel, dim3(nblk(E)), dim3(256), 0, nullptr, E,
                           n_landmarks, d_off, d_start, d_half, d_edges);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpy(edges, d_edges, (size_t)E * sizeof(slam_graph_edge),
                      hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(SLAM_ERR_HIP, "slam_graph_pair_halves: kernel or download failed");
    }
    (void)hipFree(d_off);
    (void)hipFree(d_start);
    (void)hipFree(d_half);
    (void)hipFree(d_edges);
    return rc;
}

int slam_graph_linearize_solve(const slam_graph_config* cfg, const slam_graph_edge* edges,
                               int64_t n_edges, double* poses, int64_t n_poses, double* stats,
                               int device) {
    SLAM_ARG_CHECK(poses && stats, "slam_graph_linearize_solve: NULL argument");
    slam_graph* h = nullptr;
    int rc = slam_graph_create(cfg, device, &h);
    if (rc) return rc;
    rc = slam_graph_set_poses(h, n_poses, poses);
    if (!rc) rc = slam_graph_set_edges(h, n_edges, edges);
    if (!rc) rc = slam_graph_update(h, stats);
    if (!rc) rc = slam_graph_get_poses(h, poses);
    slam_graph_destroy(h);
    return rc;
}

}  // extern "C"
