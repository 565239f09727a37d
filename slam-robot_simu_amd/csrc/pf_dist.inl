// pf_dist.inl -- the sharded particle filter's device-resident step
// (BASELINE config 3: 8 x 1,048,576 particles, one shard per GPU).
//
// Each rank holds a contiguous shard of one filter in the single-GPU layout
// (deferred normalisation: w = w_un / s, fused predict + likelihood with block
// partials).  The exchanges are peer-memory pushes over xGMI into a
// per-rank exchange region that every peer has mapped (IPC): a rank stores its
// data into its slot of every peer's region, then publishes the step number in
// that peer's flag word (system-scope release); a reader spins on its own flag
// words (system-scope acquire, bounded).  Every kernel is enqueued every step
// and gates on the device resample flag, so a step needs no host decision and
// K steps replay as one hipGraph.  Per step:
//
//   resample steps only (particle_filter.py:200-224, exact cumsum :212):
//     classify -> emit + push specials -> fold (wait) -> expand + hi + counts
//     -> pack + push items -> unpack (wait)
//   every step:
//     fused predict + likelihood (the single-GPU kernel) -> record + push
//     -> global finalize (wait): np.sum in the reference's global order
//     (:234), max / first argmax (:115-117), ESS (:210), covariance, result
//
// Every rank folds the gathered data in rank order, so all ranks hold the same
// result, bit-identical to one GPU holding all particles (the exact cumsum and
// the numpy-order sum do not depend on how the particles are split, as long as
// every shard but the last holds whole 8192-element np.sum buffers).
#pragma once
#include "pf_kernels.hpp"

namespace slam {

constexpr int kDistMaxWorld = 16;
constexpr int kDistWin = 4;                // argmax tie window entries per record
enum : int { kXG1 = 0, kXSpec = 1, kXItem = 2 };

// status bits of a distributed step (result.status)
enum : int {
    kDistStWait = 1 << 4,       // a peer did not publish in time (bounded wait expired)
    kDistStTie = 1 << 5,        // first argmax not resolved by the tie window (estimate provisional)
    kDistStDegenerate = 1 << 6, // every weight NaN -> 1/NP: covariance not formed
    kDistStItems = 1 << 7,      // resample exchange inconsistent
};

struct DistWin {
    int64_t idx;                // global index
    double v;                   // w_un
    double x[3];
};

// per-rank reduction record (the G1 exchange), followed by the np.sum buffer partials
struct DistRec {
    int64_t nchunk;             // buffer partials that follow
    int64_t idx;                // global index of the first occurrence of M
    double M;                   // max w_un of the shard (-1: empty)
    double xc[3];               // particle at idx
    double q[11];               // sw, sw2, m1[3], m2[6] scaled by 1/M (sw2 by 1/M^2)
    double T;                   // sum of w_un (approximate: exact-cumsum base offsets)
    double x0[3];               // particle at local 0 (degenerate-case estimate)
    int64_t nwin;               // entries of win (elements within 2^-48 of M, index order)
    DistWin win[kDistWin];
};

struct DistLayout {
    int64_t flags = 0;          // uint64 [3][kDistMaxWorld]
    int64_t g1 = 0;             // [2 parities][world] records of rec_stride bytes
    int64_t spec_hdr = 0;       // [world] {nspec, ktot}
    int64_t spec = 0;           // [world][cap_spec] SpecialIn
    int64_t item_hdr = 0;       // [world] {count, pad}
    int64_t item = 0;           // [world][cap_item] ShardItem
    int64_t total = 0;
    int64_t rec_stride = 0, cap_spec = 0, cap_item = 0;
};

struct DistPeers {
    char* base[kDistMaxWorld];  // every rank's exchange region as mapped in this process
    int64_t gb[kDistMaxWorld + 1];
    DistLayout L;
    int32_t world, rank;
};

// device scratch of one rank (regular memory)
struct DistScratch {
    int32_t spec_base;          // specials of the lower ranks
    int32_t nspec_g;            // all specials
    uint64_t k_base;            // increment prefix of the lower ranks
    uint64_t ktot_g;
    double base_off;            // approximate cumsum before local element 0
    double c_left;              // exact cumsum just before local element 0 (-inf on rank 0)
    int64_t lo0;                // positions <= c_left
    int64_t pad;
    int64_t dbase[kDistMaxWorld];   // per destination: selected sources before its range
    int64_t dcnt[kDistMaxWorld];    // per destination: items sent
};

__device__ __forceinline__ uint64_t* dist_flags(const DistPeers& P, const int q) {
    return reinterpret_cast<uint64_t*>(P.base[q] + P.L.flags);
}

// publish `epoch` in flag word [kind][my rank] of every peer (after the data)
__device__ __forceinline__ void dist_signal(const DistPeers& P, const int kind, const uint64_t epoch) {
    __threadfence_system();
    if ((int)threadIdx.x < P.world)
        __hip_atomic_store(dist_flags(P, threadIdx.x) + kind * kDistMaxWorld + P.rank, epoch,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait until every peer published `epoch` in my flag words [kind][q]
// (bounded: ~2^24 polls, ~20 s, then status bit kDistStWait and proceed)
__device__ __forceinline__ void dist_wait(const DistPeers& P, const int kind, const uint64_t epoch,
                                          int32_t* flags) {
    if ((int)threadIdx.x < P.world) {
        const uint64_t* f = dist_flags(P, P.rank) + kind * kDistMaxWorld + threadIdx.x;
        int64_t polls = 0;
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
            if (++polls > (int64_t(1) << 24)) {
                atomicOr(&flags[kFlagStatus], kDistStWait);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

__device__ __forceinline__ uint64_t ld_sys(const void* p) {
    return __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys_d(const double* p) {
    return __longlong_as_double((long long)ld_sys(p));
}
template <typename S>
__device__ __forceinline__ S ld_sys_struct(const S* p) {
    S v;
    uint64_t* d = reinterpret_cast<uint64_t*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(S) / 8); ++k) d[k] = ld_sys(reinterpret_cast<const uint64_t*>(p) + k);
    return v;
}

__device__ __forceinline__ uint64_t dist_epoch(const StepIO& io) { return (uint64_t)io.ctr[1] + 1; }

__device__ __forceinline__ bool dist_resampling(const int32_t* flags) {
    return flags[kFlagResample] == 1;
}

// owner rank of global position / particle g
__device__ __forceinline__ int dist_owner(const DistPeers& P, const int64_t g) {
    int d = 0;
    while (d + 1 < P.world && P.gb[d + 1] <= g) ++d;
    return d;
}

// ---------------------------------------------------------------- resample
// emit the local specials (write-through) and, in the last block, push the
// list with (nspec, ktot) into every peer's slot, then signal kXSpec
__global__ __launch_bounds__(kScanThreads) void dist_emit_push_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_div, const double np_recip,
    const int64_t n, const double* __restrict__ approx, const uint64_t* __restrict__ kincl,
    const int32_t* __restrict__ fexcl, const uint64_t* __restrict__ boffk,
    const int32_t* __restrict__ bofff, SpecialIn* __restrict__ spec, const int64_t gbase,
    const int32_t* __restrict__ nspec_p, const uint64_t* __restrict__ ktot_p,
    unsigned* __restrict__ counter, int32_t* __restrict__ flags, const DistPeers P, StepIO io) {
    if (!dist_resampling(flags)) return;
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        const int32_t f = fexcl[i];
        if (f & 1) {
            SpecialIn e;
            e.idx = gbase + i;
            e.P = boffk[blockIdx.x] + kincl[i];
            e.w = norm_w(w_un[i], *s_div, np_recip);
            e.E = sum_binade(approx[i]);
            e.pad = 0;
            st_wt_struct(&spec[bofff[blockIdx.x] + (f >> 1)], e);
        }
    }
    if (!arrive_last(counter)) return;
    const int32_t ns = *nspec_p;
    const uint64_t kt = *ktot_p;
    for (int q = 0; q < P.world; ++q) {
        char* rb = P.base[q];
        SpecialIn* dst = reinterpret_cast<SpecialIn*>(rb + P.L.spec) + (int64_t)P.rank * P.L.cap_spec;
        for (int32_t m = threadIdx.x; m < ns; m += blockDim.x) dst[m] = ld_wt_struct(&spec[m]);
        if (threadIdx.x == 0) {
            int64_t* hdr = reinterpret_cast<int64_t*>(rb + P.L.spec_hdr) + 2 * P.rank;
            hdr[0] = ns;
            hdr[1] = (int64_t)kt;
        }
    }
    __syncthreads();
    dist_signal(P, kXSpec, dist_epoch(io));
}

// wait for every rank's specials, concatenate them in rank order with global
// increment prefixes, fold them sequentially (the exact cumsum's specials),
// and derive this rank's offsets and the cumsum just before its first element
__global__ __launch_bounds__(256) void dist_fold_kernel(
    SpecialIn* __restrict__ spec_g, SpecialOut* __restrict__ spec_go, const int64_t n_global,
    int32_t* __restrict__ flags, DistScratch* __restrict__ scr, const DistPeers P, StepIO io,
    const double step, const double np_recip, const uint64_t seed) {
    if (!dist_resampling(flags)) return;
    dist_wait(P, kXSpec, dist_epoch(io), flags);
    __shared__ int64_t s_ns[kDistMaxWorld], s_off[kDistMaxWorld + 1];
    __shared__ uint64_t s_kt[kDistMaxWorld], s_koff[kDistMaxWorld + 1];
    const char* mine = P.base[P.rank];
    if (threadIdx.x == 0) {
        int64_t no = 0;
        uint64_t ko = 0;
        for (int q = 0; q < P.world; ++q) {
            const int64_t* hdr = reinterpret_cast<const int64_t*>(mine + P.L.spec_hdr) + 2 * q;
            s_ns[q] = (int64_t)ld_sys(hdr);
            s_kt[q] = ld_sys(hdr + 1);
            s_off[q] = no;
            s_koff[q] = ko;
            no += s_ns[q];
            ko += s_kt[q];
        }
        s_off[P.world] = no;
        s_koff[P.world] = ko;
        for (int d = 0; d < kDistMaxWorld; ++d) {
            scr->dbase[d] = 0;
            scr->dcnt[d] = 0;
        }
        scr->spec_base = (int32_t)s_off[P.rank];
        scr->k_base = s_koff[P.rank];
        scr->nspec_g = (int32_t)no;
        scr->ktot_g = ko;
    }
    __syncthreads();
    for (int q = 0; q < P.world; ++q) {
        const SpecialIn* src = reinterpret_cast<const SpecialIn*>(mine + P.L.spec) + (int64_t)q * P.L.cap_spec;
        for (int64_t m = threadIdx.x; m < s_ns[q]; m += blockDim.x) {
            SpecialIn e = ld_sys_struct(&src[m]);
            e.P += s_koff[q];
            spec_g[s_off[q] + m] = e;
        }
    }
    __syncthreads();
    serial_fold(spec_g, spec_go, (int32_t)s_off[P.world], s_koff[P.world], n_global, flags, nullptr,
                nullptr, 0, false, nullptr, np_recip);
    __syncthreads();
    if (threadIdx.x == 0) {
        double cl = -INFINITY;
        int64_t lo0 = 0;
        if (P.rank > 0 && s_off[P.rank] > 0) {
            const SpecialOut p = spec_go[s_off[P.rank] - 1];
            cl = p.cs + (double)(s_koff[P.rank] - p.P) * ldexp(1.0, p.E - 52);
            const double ofs = resample_offset(io.ofs[io.ctr[0]], np_recip, seed, (uint32_t)io.ctr[1]);
            lo0 = count_positions(cl, n_global, step, ofs);
        }
        scr->c_left = cl;
        scr->lo0 = lo0;
    }
}

// exact cumsum of local element i from the folded specials (scan_expand's rule)
__device__ __forceinline__ double dist_expand_c(const int64_t i, const uint64_t* __restrict__ kincl,
                                                const int32_t* __restrict__ fexcl,
                                                const uint64_t* __restrict__ boffk,
                                                const int32_t* __restrict__ bofff,
                                                const SpecialOut* __restrict__ so,
                                                const int32_t spec_base, const uint64_t k_base) {
    const int64_t b = i / kScanBlock;
    const int32_t f = fexcl[i];
    const int32_t m = bofff[b] + spec_base + (f >> 1);
    if (f & 1) return so[m].cs;
    const SpecialOut& p = so[m - 1];
    const uint64_t K = boffk[b] + k_base + kincl[i] - p.P;
    return p.cs + (double)K * ldexp(1.0, p.E - 52);
}

// expand the local exact cumsum, hi_j = #positions <= c_j; count the selected
// sources (hi_j > lo_j) per block (the last block scans the counts) and, per
// destination rank d, the selected sources before its positions (dbase) and
// overlapping them (dcnt) -- block-reduced in LDS, one global atomic per block
// (both zeroed by dist_fold_kernel)
__global__ __launch_bounds__(kScanThreads) void dist_expand_hi_kernel(
    const int64_t n, const uint64_t* __restrict__ kincl, const int32_t* __restrict__ fexcl,
    const uint64_t* __restrict__ boffk, const int32_t* __restrict__ bofff,
    const SpecialOut* __restrict__ so, double* __restrict__ c, int64_t* __restrict__ hi,
    int32_t* __restrict__ bsel, int32_t* __restrict__ bsel_off, unsigned* __restrict__ counter,
    int32_t* __restrict__ flags, DistScratch* __restrict__ scr, const DistPeers P, StepIO io,
    const int64_t n_global, const double step, const double np_recip, const uint64_t seed) {
    if (!dist_resampling(flags) || flags[kFlagFallback]) return;
    __shared__ int32_t shs[kScanThreads / 64 + 1];
    __shared__ int32_t s_cb[kDistMaxWorld], s_cc[kDistMaxWorld];
    if ((int)threadIdx.x < kDistMaxWorld) {
        s_cb[threadIdx.x] = 0;
        s_cc[threadIdx.x] = 0;
    }
    const int32_t sb = scr->spec_base;
    const uint64_t kb = scr->k_base;
    const double ofs = resample_offset(io.ofs[io.ctr[0]], np_recip, seed, (uint32_t)io.ctr[1]);
    const int64_t gbase = P.gb[P.rank];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    int64_t prev;
    if (base == 0) prev = scr->lo0;
    else if (base < n) prev = count_positions(dist_expand_c(base - 1, kincl, fexcl, boffk, bofff, so, sb, kb),
                                              n_global, step, ofs);
    else prev = 0;
    __syncthreads();
    int32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        const double ci = dist_expand_c(i, kincl, fexcl, boffk, bofff, so, sb, kb);
        c[i] = ci;
        int64_t h = count_positions(ci, n_global, step, ofs);
        if (gbase + i == n_global - 1) {
            if (h < n_global) atomicOr(&flags[kFlagStatus], 1);   // IndexError in the reference
            h = n_global;
        }
        hi[i] = h;
        if (h > prev) {
            ++cnt;
            for (int d = 0; d < P.world; ++d) {
                if (h <= P.gb[d]) atomicAdd(&s_cb[d], 1);
                else if (prev < P.gb[d + 1]) atomicAdd(&s_cc[d], 1);
            }
        }
        prev = h;
    }
    int32_t tot;
    block_excl_scan<int32_t, kScanThreads>(cnt, shs, tot);   // (its barriers publish s_cb / s_cc)
    if ((int)threadIdx.x < P.world) {
        const int d = threadIdx.x;
        if (s_cb[d]) atomicAdd((unsigned long long*)&scr->dbase[d], (unsigned long long)s_cb[d]);
        if (s_cc[d]) atomicAdd((unsigned long long*)&scr->dcnt[d], (unsigned long long)s_cc[d]);
    }
    if (threadIdx.x == 0) st_wt_i(&bsel[blockIdx.x], tot);
    if (!arrive_last(counter)) return;
    block_scan_array<int32_t, kScanThreads>(bsel, bsel_off, gridDim.x, nullptr, shs, true);
}

// items to every destination: each selected source overlapping a destination's
// positions, with its clipped position range, stored into the destination's
// slot for this rank; the last block writes the counts and signals kXItem
__global__ __launch_bounds__(kScanThreads) void dist_pack_push_kernel(
    const int64_t n, const double* __restrict__ xs, const double* __restrict__ ys,
    const double* __restrict__ ts, const int64_t* __restrict__ hi,
    const int32_t* __restrict__ bsel_off, unsigned* __restrict__ counter,
    int32_t* __restrict__ flags, const DistScratch* __restrict__ scr, const DistPeers P,
    StepIO io) {
    if (!dist_resampling(flags) || flags[kFlagFallback]) return;
    __shared__ int32_t shs[kScanThreads / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    int64_t hv[kScanPer];
    bool sel[kScanPer];
    int64_t prev = (base == 0) ? scr->lo0 : (base < n ? hi[base - 1] : 0);
    int32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        hv[k] = (i < n) ? hi[i] : prev;
        sel[k] = (i < n) && hv[k] > prev;
        cnt += sel[k] ? 1 : 0;
        if (i < n) prev = hv[k];
    }
    int32_t tot;
    int64_t ps = (int64_t)bsel_off[blockIdx.x] + block_excl_scan<int32_t, kScanThreads>(cnt, shs, tot);
    prev = (base == 0) ? scr->lo0 : (base < n ? hi[base - 1] : 0);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        if (sel[k]) {
            const int64_t lo = prev, h = hv[k];
            ShardItem it;
            it.x = xs[i];
            it.y = ys[i];
            it.th = ts[i];
            for (int d = dist_owner(P, lo); d < P.world && P.gb[d] < h; ++d) {
                const int64_t slot = ps - scr->dbase[d];
                it.lo = lo > P.gb[d] ? lo : P.gb[d];
                it.hi = h < P.gb[d + 1] ? h : P.gb[d + 1];
                ShardItem* dst = reinterpret_cast<ShardItem*>(P.base[d] + P.L.item) +
                                 (int64_t)P.rank * P.L.cap_item;
                if (slot >= 0 && slot < P.L.cap_item) dst[slot] = it;
                else atomicOr(&flags[kFlagStatus], kDistStItems);
            }
            ++ps;
        }
        prev = hv[k];
    }
    if (!arrive_last(counter)) return;
    if ((int)threadIdx.x < P.world) {
        int64_t* hdr = reinterpret_cast<int64_t*>(P.base[threadIdx.x] + P.L.item_hdr) + 2 * P.rank;
        hdr[0] = scr->dcnt[threadIdx.x];
    }
    __syncthreads();
    dist_signal(P, kXItem, dist_epoch(io));
}

// wait for every rank's items; every local position takes the item whose range
// covers it (items of rank q cover a contiguous stretch of positions, ranks in
// order); the last block marks the resample done (flag 2: w = 1/NP)
__global__ __launch_bounds__(256) void dist_unpack_kernel(
    const int64_t n, double* __restrict__ xs, double* __restrict__ ys, double* __restrict__ ts,
    unsigned* __restrict__ counter, int32_t* __restrict__ flags, const DistPeers P, StepIO io) {
    if (!dist_resampling(flags) || flags[kFlagFallback]) return;
    dist_wait(P, kXItem, dist_epoch(io), flags);
    __shared__ int64_t s_cnt[kDistMaxWorld], s_first[kDistMaxWorld];
    const char* mine = P.base[P.rank];
    const ShardItem* items = reinterpret_cast<const ShardItem*>(mine + P.L.item);
    if ((int)threadIdx.x < P.world) {
        const int q = threadIdx.x;
        const int64_t cq = (int64_t)ld_sys(reinterpret_cast<const int64_t*>(mine + P.L.item_hdr) + 2 * q);
        s_cnt[q] = cq;
        s_first[q] = cq > 0 ? (int64_t)ld_sys(&items[(int64_t)q * P.L.cap_item].lo) : INT64_MAX;
    }
    __syncthreads();
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        const int64_t g = P.gb[P.rank] + p;
        int q = -1;
        for (int r = 0; r < P.world; ++r)
            if (s_cnt[r] > 0 && s_first[r] <= g) q = r;
        bool ok = q >= 0;
        if (ok) {
            const ShardItem* L = items + (int64_t)q * P.L.cap_item;
            int64_t a = 0, b = s_cnt[q];                    // first item with hi > g
            while (a < b) {
                const int64_t m = (a + b) >> 1;
                if ((int64_t)ld_sys(&L[m].hi) > g) b = m;
                else a = m + 1;
            }
            ok = a < s_cnt[q] && (int64_t)ld_sys(&L[a].lo) <= g;
            if (ok) {
                xs[p] = ld_sys_d(&L[a].x);
                ys[p] = ld_sys_d(&L[a].y);
                ts[p] = ld_sys_d(&L[a].th);
            }
        }
        if (!ok) atomicOr(&flags[kFlagStatus], kDistStItems);
    }
    if (!arrive_last(counter)) return;
    if (threadIdx.x == 0) flags[kFlagResample] = 2;        // gathered: the fused kernel uses w = 1/NP
}

// ---------------------------------------------------------------- record
// The shard's reduction record from the fused kernel's block partials,
// pushed into every peer's G1 slot (parity = epoch & 1), then kXG1.
// One workgroup of kFinThreads lanes.
__global__ __launch_bounds__(kFinThreads) void dist_record_push_kernel(
    const int64_t n, const DeferParts dp, const double* __restrict__ w_un,
    const int32_t* __restrict__ tail_leaves, const int32_t* __restrict__ tail_ops,
    const int32_t n_tail_leaves, const int32_t n_tail_ops, const double* __restrict__ xs,
    const double* __restrict__ ys, const double* __restrict__ ts, const DistPeers P, StepIO io) {
    __shared__ double sh[2048];
    __shared__ double s_q[11][kFinThreads];
    __shared__ double s_wm[kFinWaves];
    __shared__ unsigned long long s_min;
    __shared__ DistRec rec;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
    const int64_t gbase = P.gb[P.rank];
    double* chunks = sh;                                    // reused below (nch <= 2048)
    // ---- np.sum buffer partials: 64 leaves per 8192-element buffer, perfect tree
    for (int64_t c = tid; c < nfull; c += kFinThreads) {
        const double* Lp = dp.leaf + 64 * c;
        double a[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) a[j] = Lp[2 * j] + Lp[2 * j + 1];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = a[2 * j] + a[2 * j + 1];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[2 * j] + a[2 * j + 1];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = a[2 * j] + a[2 * j + 1];
        chunks[c] = (a[0] + a[1]) + (a[2] + a[3]);
    }
    __syncthreads();
    if (nch > nfull) {
        __shared__ double tl[1024];
        const double t = tail_chunk_sum(w_un + nfull * kSumChunk, tail_leaves, tail_ops, n_tail_leaves,
                                        n_tail_ops, tl);
        if (tid == 0) chunks[nfull] = t;
    }
    // ---- block maxima: M, the first block holding it
    double m = -1.0;
    for (int64_t b = tid; b < nb; b += kFinThreads) m = fmax(m, dp.pmax[b]);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) m = fmax(m, __shfl_xor(m, d, 64));
    if (lane == 0) s_wm[wave] = m;
    if (tid == 0) s_min = ~0ull;
    __syncthreads();
    double M = s_wm[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) M = fmax(M, s_wm[w]);
    const double thr = M * (1.0 - 0x1p-48);                // tie window (2^-48 relative)
    // ---- scaled sums over the blocks (lane-strided, then a fixed tree)
    double acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = 0.0;
    double T = 0.0;
    unsigned long long first = ~0ull;
    for (int64_t b = tid; b < nb; b += kFinThreads) {
        const double pm = dp.pmax[b];
        if (M > 0.0) {
            const double r = pm / M;
            acc[0] += r * dp.ps[0][b];
            acc[1] += (r * r) * dp.ps[1][b];
#pragma unroll
            for (int j = 2; j < 11; ++j) acc[j] += r * dp.ps[j][b];
        }
        T += pm * dp.ps[0][b];
        if (pm >= thr && first == ~0ull) first = (unsigned long long)b;
    }
    if (first != ~0ull) atomicMin(&s_min, first);
#pragma unroll
    for (int j = 0; j < 11; ++j) s_q[j][tid] = acc[j];
    __syncthreads();
    if (tid < 11) {
        double r = 0.0;
        for (int k = 0; k < kFinThreads; ++k) r = r + s_q[tid][k];
        rec.q[tid] = r;
    }
    __syncthreads();
    // T: the same fixed tree through s_q[0]
    s_q[0][tid] = T;
    __syncthreads();
    if (tid == 0) {
        double r = 0.0;
        for (int k = 0; k < kFinThreads; ++k) r = r + s_q[0][k];
        rec.T = r;
        rec.M = M;
        rec.nchunk = nch;
        rec.x0[0] = xs[0];
        rec.x0[1] = ys[0];
        rec.x0[2] = ts[0];
        rec.nwin = 0;
    }
    __syncthreads();
    // ---- tie window: the first kDistWin elements (index order) with w_un >= thr,
    // scanning the blocks from the first candidate on (usually one element: M)
    if (M > 0.0 && wave == 0) {
        int64_t cnt = 0;
        for (int64_t b = (int64_t)s_min; b < nb && cnt < kDistWin; ++b) {
            if (dp.pmax[b] < thr) continue;
            for (int e0 = 0; e0 < kPartPer && cnt < kDistWin; e0 += 64) {
                const int64_t i = b * kPartPer + e0 + lane;
                const double v = (i < n) ? w_un[i] : -1.0;
                unsigned long long hit = __ballot(v >= thr);
                while (hit && cnt < kDistWin) {
                    const int l = __ffsll((long long)hit) - 1;
                    hit &= hit - 1;
                    if (lane == l) {
                        DistWin& wv = rec.win[cnt];
                        wv.idx = gbase + i;
                        wv.v = v;
                        wv.x[0] = xs[i];
                        wv.x[1] = ys[i];
                        wv.x[2] = ts[i];
                    }
                    ++cnt;
                }
            }
        }
        if (lane == 0) rec.nwin = cnt;
    }
    __syncthreads();
    if (tid == 0) {
        // the first occurrence of M: a window entry, else the first block holding M
        rec.idx = -1;
        for (int k = 0; k < (int)rec.nwin; ++k)
            if (rec.win[k].v == M) {
                rec.idx = rec.win[k].idx;
                for (int j = 0; j < 3; ++j) rec.xc[j] = rec.win[k].x[j];
                break;
            }
        for (int64_t b = 0; rec.idx < 0 && b < nb; ++b)
            if (dp.pmax[b] == M) {
                rec.idx = gbase + dp.pidx[b];
                for (int j = 0; j < 3; ++j) rec.xc[j] = dp.pxe[j][b];
            }
    }
    __syncthreads();
    // ---- push into every peer's slot (parity = epoch & 1)
    const uint64_t epoch = dist_epoch(io);
    const int64_t words = (int64_t)sizeof(DistRec) / 8;
    for (int q = 0; q < P.world; ++q) {
        char* slot = P.base[q] + P.L.g1 + ((int64_t)(epoch & 1) * P.world + P.rank) * P.L.rec_stride;
        uint64_t* dst = reinterpret_cast<uint64_t*>(slot);
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&rec);
        for (int64_t k = tid; k < words; k += kFinThreads) dst[k] = src[k];
        double* dch = reinterpret_cast<double*>(slot + sizeof(DistRec));
        for (int64_t c = tid; c < nch; c += kFinThreads) dch[c] = chunks[c];
    }
    __syncthreads();
    dist_signal(P, kXG1, epoch);
}

// ---------------------------------------------------------------- finalize
// Wait for every rank's record and form the step's global result -- the same
// on every rank: s = np.sum in the reference's order (buffer partials, ranks in
// order), the exact max and first argmax of w = w_un / s, ESS and covariance
// from the scaled sums, the result record, the next step's resample flag and,
// when it resamples, this rank's exact-cumsum base offsets.
__global__ __launch_bounds__(kFinThreads) void dist_finalize_kernel(
    const int64_t n, const DeferParts dp, double* __restrict__ s_cur, double* __restrict__ refp,
    int32_t* __restrict__ flags, const double ess_th, StepIO io, const double np_recip,
    double* __restrict__ boff, DistScratch* __restrict__ scr, const DistPeers P) {
    __shared__ double s_rq[kDistMaxWorld][11];
    __shared__ double s_M[kDistMaxWorld], s_T[kDistMaxWorld];
    __shared__ double s_s;
    __shared__ int32_t s_do_off;
    const int tid = threadIdx.x;
    const uint64_t epoch = dist_epoch(io);
    dist_wait(P, kXG1, epoch, flags);
    const char* g1 = P.base[P.rank] + P.L.g1 + (int64_t)(epoch & 1) * P.world * P.L.rec_stride;
    auto rec_of = [&](int q) { return reinterpret_cast<const DistRec*>(g1 + (int64_t)q * P.L.rec_stride); };
    if (tid < P.world) {
        const DistRec* r = rec_of(tid);
        s_M[tid] = ld_sys_d(&r->M);
        s_T[tid] = ld_sys_d(&r->T);
        for (int j = 0; j < 11; ++j) s_rq[tid][j] = ld_sys_d(&r->q[j]);
    }
    __syncthreads();
    if (tid == 0) {
        // np.sum (particle_filter.py:234): buffer partials left to right, ranks in order
        double s = 0.0;
        for (int q = 0; q < P.world; ++q) {
            const DistRec* r = rec_of(q);
            const int64_t nc = (int64_t)ld_sys(&r->nchunk);
            const double* ch = reinterpret_cast<const double*>(reinterpret_cast<const char*>(r) + sizeof(DistRec));
            for (int64_t c = 0; c < nc; ++c) s = s + ld_sys_d(&ch[c]);
        }
        s_s = s;
        double M = -1.0;
        for (int q = 0; q < P.world; ++q) M = fmax(M, s_M[q]);
        const bool ok = (s > 0.0) && !isinf(s) && (M > 0.0);
        BlockPartial tot;
        bp_zero(tot);
        double xe[3] = {0.0, 0.0, 0.0};
        int32_t st = 0;
        if (ok) {
            const double mval = M / s;
            // first rank whose max rounds to the maximum, then its first element that does
            int win = 0;
            while (win < P.world && !(s_M[win] > 0.0 && s_M[win] / s == mval)) ++win;
            const DistRec* r = rec_of(win);
            const int nw = (int)ld_sys(&r->nwin);
            int k = 0;
            while (k < nw && !(ld_sys_d(&r->win[k].v) / s == mval)) ++k;
            if (k < nw) {
                tot.maxi = (int64_t)ld_sys(&r->win[k].idx);
                for (int j = 0; j < 3; ++j) xe[j] = ld_sys_d(&r->win[k].x[j]);
            } else {                                        // window exhausted: M's own element
                tot.maxi = (int64_t)ld_sys(&r->idx);
                for (int j = 0; j < 3; ++j) xe[j] = ld_sys_d(&r->xc[j]);
                st |= kDistStTie;
            }
            tot.maxv = mval;
            // scaled sums: ranks in order, each rescaled from its max to the global max
            double a[11];
            for (int j = 0; j < 11; ++j) a[j] = 0.0;
            for (int q = 0; q < P.world; ++q) {
                if (!(s_M[q] > 0.0)) continue;
                const double rr = s_M[q] / M;
                a[0] += rr * s_rq[q][0];
                a[1] += (rr * rr) * s_rq[q][1];
                for (int j = 2; j < 11; ++j) a[j] += rr * s_rq[q][j];
            }
            const double f = M / s;
            tot.sw = a[0] * f;
            tot.sw2 = a[1] * (f * f);
            for (int j = 0; j < 3; ++j) tot.m1[j] = a[2 + j] * f;
            for (int j = 0; j < 6; ++j) tot.m2[j] = a[5 + j] * f;
        } else {
            // every weight NaN -> 1/NP (particle_filter.py:236): argmax 0
            const DistRec* r0 = rec_of(0);
            tot.maxv = np_recip;
            tot.maxi = 0;
            for (int j = 0; j < 3; ++j) xe[j] = ld_sys_d(&r0->x0[j]);
            tot.sw = 1.0;
            tot.sw2 = np_recip;                             // ESS = NP
            for (int j = 0; j < 3; ++j) tot.m1[j] = NAN;
            for (int j = 0; j < 6; ++j) tot.m2[j] = NAN;
            st |= kDistStDegenerate;
        }
        flags[kFlagStatus] |= st;
        const int32_t stp = io.ctr[0];
        write_result_xe(tot, xe, refp, s, flags, ess_th, io.res + stp, -1);
        io.ctr[0] = stp + 1;
        io.ctr[1] = io.ctr[1] + 1;
        *s_cur = s;
        s_do_off = flags[kFlagResample];
        if (s_do_off) {
            double bo = 0.0;
            for (int q = 0; q < P.rank; ++q) bo = bo + s_T[q];
            scr->base_off = bo / s;
        }
    }
    __syncthreads();
    if (s_do_off) {
        // this rank's fused-block prefix of w for the next step's exact cumsum
        const double s = s_s;
        const int64_t nb = (n + kPartPer - 1) / kPartPer;
        const int per = (int)((nb + kFinThreads - 1) / kFinThreads);
        const int64_t b0 = (int64_t)tid * per;
        auto btot = [&](int64_t b) { return (dp.pmax[b] / s) * dp.ps[0][b]; };
        double loc = 0.0;
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) loc += btot(b0 + k);
        __shared__ double shx[kFinThreads / 64 + 1];
        double total;
        double ex = block_excl_scan<double, kFinThreads>(loc, shx, total);
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) {
                boff[b0 + k] = ex;
                ex = ex + btot(b0 + k);
            }
        if (tid == 0) boff[nb] = total;
    }
}

}  // namespace slam
