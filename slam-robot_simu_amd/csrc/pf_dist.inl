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
    int64_t item = 0;           // [world][cap_item] DistItem (own slot unused: self_items)
    int64_t pitem = 0;          // [cap_item] DistRun at its first local position (merged exchange)
    int64_t pcarry = 0;         // [cap_item / kPartPer + 1] (epoch << 32) | run start of each fused block
    int64_t total = 0;
    int64_t rec_stride = 0, cap_spec = 0, cap_item = 0;
};

// a resampled particle with its destination positions [lo, hi) (global), 48 B
struct alignas(16) DistItem {
    double x, y, th;
    int64_t lo, hi, pad;
};

// a resampled particle received from a peer, at the first position of its run
// in this rank's shard (the merged exchange; no count exchange needed)
struct alignas(16) DistRun {
    double x, y, th;
    uint64_t tag;               // (epoch << 32) | run length
};

struct DistPeers {
    char* base[kDistMaxWorld];  // every rank's exchange region as mapped in this process
                                // (collective mode: only this rank's own)
    DistItem* self_items;       // items this rank sends itself (regular memory, cap_item)
    // collective mode (slam_dist_set_collective): every push stays in this
    // rank's own region / send area and the host moves it with RCCL
    // collectives (or device copies between held shards) between the launches
    DistItem* item_out;         // [world][cap_item] items per destination rank
    int64_t* cnt_out;           // [world] item counts per destination rank
    int32_t coll;
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
    int64_t lo0;                // positions <= c_left (the first one this rank's sources serve)
    int64_t hi0;                // positions served by this rank and the lower ones (merged exchange)
    int64_t covered;            // positions covered by the received items (unpack; reset by its last block)
    int32_t rel[4];             // dist_resample_merged_kernel: release tokens of phases A / D
    int64_t dbase[kDistMaxWorld];   // per destination: selected sources before its range
    int64_t dcnt[kDistMaxWorld];    // per destination: items sent
};

__device__ __forceinline__ uint64_t* dist_flags(const DistPeers& P, const int q) {
    return reinterpret_cast<uint64_t*>(P.base[q] + P.L.flags);
}

// the ranks a push reaches: every peer's region, or (collective mode) only
// this rank's own slot, which the collective then carries to the peers
__device__ __forceinline__ int dist_push_lo(const DistPeers& P) { return P.coll ? P.rank : 0; }
__device__ __forceinline__ int dist_push_hi(const DistPeers& P) { return P.coll ? P.rank + 1 : P.world; }

// publish `epoch` in flag word [kind][my rank] of every peer (after the data).
// One system-scope release per block: on gfx950 it writes back the L2, so
// every lane's stores complete first (barrier), then lane 0 fences once and
// stores the flags.  Data that other blocks stored earlier in the launch was
// written with system-scope stores (dist_store_item) and had completed before
// their tickets.
// One rank (world 1): no peer to publish to -- every wait on the flags is the
// same block's (or a later launch's, behind the kernel boundary), and every
// read of the published data is a system-scope load, so the block's drained
// stores and a barrier are enough (SLAM_DIST_W1_FLAGS keeps the flags, A/B).
__device__ __forceinline__ bool dist_single_rank(const DistPeers& P) {
#ifdef SLAM_DIST_W1_FLAGS
    (void)P;
    return false;
#else
    return P.world == 1;
#endif
}

__device__ __forceinline__ void dist_signal(const DistPeers& P, const int kind, const uint64_t epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (dist_single_rank(P)) return;
    if (threadIdx.x == 0) {
        __threadfence_system();
        for (int q = dist_push_lo(P); q < dist_push_hi(P); ++q)
            __hip_atomic_store(dist_flags(P, q) + kind * kDistMaxWorld + P.rank, epoch,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// #{i in [0, N): fl(fl(i*step) + ofs) <= x}  (resample positions are monotone)
__device__ __forceinline__ int64_t count_positions(const double x, const int64_t N,
                                                   const double step, const double ofs) {
    int64_t lo = 0, hi = N;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const double pos = (double)mid * step + ofs;
        if (pos <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// A wait that expired marks the shard dead (flags[kFlagDistDead], never reset
// on this handle): every later wait reports kDistStWait at once instead of
// polling again, so a dead peer costs one bounded wait per handle, not one per
// wait of every replayed step.
__device__ __forceinline__ bool dist_dead(int32_t* flags) {
    return __hip_atomic_load(&flags[kFlagDistDead], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void dist_mark_dead(int32_t* flags) {
    atomicOr(&flags[kFlagStatus], kDistStWait);
    __hip_atomic_store(&flags[kFlagDistDead], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait until every peer published `epoch` in my flag words [kind][q]
// (bounded: ~2^24 polls, ~20 s, then status bit kDistStWait and proceed)
__device__ __forceinline__ void dist_wait(const DistPeers& P, const int kind, const uint64_t epoch,
                                          int32_t* flags) {
    if ((int)threadIdx.x < P.world && !dist_single_rank(P)) {
        const uint64_t* f = dist_flags(P, P.rank) + kind * kDistMaxWorld + threadIdx.x;
        if (dist_dead(flags)) {
            atomicOr(&flags[kFlagStatus], kDistStWait);
        } else {
            int64_t polls = 0;
            while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
                if (++polls > (int64_t(1) << 24)) {
                    dist_mark_dead(flags);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
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


// own items: write-through stores to regular memory; a peer's: system-scope
// stores into its exchange region, so
// they have completed at system scope once the storing block's vmcnt drains
// (before its ticket) -- no per-block L2 writeback
__device__ __forceinline__ void dist_store_item(const DistPeers& P, const int d, const int64_t slot,
                                                const double x, const double y, const double th,
                                                const int64_t lo, const int64_t hi) {
    if (d == P.rank) {
        // write-through (agent scope): the one-launch exchange unpacks them on other
        // XCDs, whose L2s do not see this one's dirty lines
        uint64_t* p = reinterpret_cast<uint64_t*>(P.self_items + slot);
        st_wt(p + 0, (uint64_t)__double_as_longlong(x));
        st_wt(p + 1, (uint64_t)__double_as_longlong(y));
        st_wt(p + 2, (uint64_t)__double_as_longlong(th));
        st_wt(p + 3, (uint64_t)lo);
        st_wt(p + 4, (uint64_t)hi);
        return;
    }
    if (P.coll) {                       // the send area for rank d (a collective moves it)
        DistItem* it = P.item_out + (int64_t)d * P.L.cap_item + slot;
        it->x = x;
        it->y = y;
        it->th = th;
        it->lo = lo;
        it->hi = hi;
        return;
    }
    uint64_t* p = reinterpret_cast<uint64_t*>(reinterpret_cast<DistItem*>(P.base[d] + P.L.item) +
                                              (int64_t)P.rank * P.L.cap_item + slot);
    const uint64_t v[5] = {(uint64_t)__double_as_longlong(x), (uint64_t)__double_as_longlong(y),
                           (uint64_t)__double_as_longlong(th), (uint64_t)lo, (uint64_t)hi};
#pragma unroll
    for (int k = 0; k < 5; ++k) __hip_atomic_store(p + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
    for (int q = dist_push_lo(P); q < dist_push_hi(P); ++q) {
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
            const double x = xs[i], y = ys[i], th = ts[i];
            for (int d = dist_owner(P, lo); d < P.world && P.gb[d] < h; ++d) {
                const int64_t slot = ps - scr->dbase[d];
                if (slot >= 0 && slot < P.L.cap_item)
                    dist_store_item(P, d, slot, x, y, th, lo > P.gb[d] ? lo : P.gb[d],
                                    h < P.gb[d + 1] ? h : P.gb[d + 1]);
                else atomicOr(&flags[kFlagStatus], kDistStItems);
            }
            ++ps;
        }
        prev = hv[k];
    }
    if (!arrive_last(counter)) return;                      // (drains this block's item stores)
    if ((int)threadIdx.x < P.world) {
        if (!P.coll || (int)threadIdx.x == P.rank) {
            int64_t* hdr = reinterpret_cast<int64_t*>(P.base[threadIdx.x] + P.L.item_hdr) + 2 * P.rank;
            hdr[0] = scr->dcnt[threadIdx.x];
        }
        if (P.coll) P.cnt_out[threadIdx.x] = scr->dcnt[threadIdx.x];
    }
    __syncthreads();
    dist_signal(P, kXItem, dist_epoch(io));
}

// collective mode: the peers' data of `kind` has arrived (the collective ran
// before this launch on the stream): publish it in this rank's flag words, so
// that the waits of the following kernels pass
__global__ void dist_publish_kernel(const DistPeers P, const int kind, const StepIO io) {
    if ((int)threadIdx.x < P.world)
        __hip_atomic_store(dist_flags(P, P.rank) + kind * kDistMaxWorld + threadIdx.x, dist_epoch(io),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait for every rank's items and hand them to the fused kernel's resample
// gather (the single-GPU expand pass's inverse map): item k (ranks in order,
// each rank's items in position order) is stored at local index k of the
// particle arrays -- the pre-resample particles were packed already -- with a
// run mark (mark generation | npad + k: DeferParts.goff) at its first local position and the carry of
// every fused block whose first position it covers.  Items never outnumber the
// positions (disjoint, non-empty ranges), so k < n.  The last block checks that
// the ranges tile the shard (status kDistStItems otherwise).  The resample flag
// stays 1: the fused kernel gathers through the marks, at weight 1/NP.
// the item offsets of every source rank in this rank's region (thread 0)
__device__ __forceinline__ void dist_item_offsets(const DistPeers& P, int64_t* s_off) {
    const char* mine = P.base[P.rank];
    int64_t o = 0;
    for (int q = 0; q < P.world; ++q) {
        s_off[q] = o;
        // a count outside [0, cap] (a peer that never published) reads no slot past the region
        const int64_t c = (int64_t)ld_sys(reinterpret_cast<const int64_t*>(mine + P.L.item_hdr) + 2 * q);
        o += c < 0 ? 0 : (c > P.L.cap_item ? P.L.cap_item : c);
    }
    s_off[P.world] = o;
}

// grid-stride over the received items (s_off: offsets per source rank, in LDS)
__device__ void dist_unpack_items(const int64_t n, double* __restrict__ xs, double* __restrict__ ys,
                                  double* __restrict__ ts, int64_t* __restrict__ mark,
                                  int32_t* __restrict__ carry, unsigned* __restrict__ counter,
                                  int32_t* __restrict__ flags, DistScratch* __restrict__ scr,
                                  const DistPeers& P, const int64_t* s_off) {
    __shared__ unsigned long long s_cov;
    if (threadIdx.x == 0) s_cov = 0;
    __syncthreads();
    const DistItem* items = reinterpret_cast<const DistItem*>(P.base[P.rank] + P.L.item);
    const int64_t ntot = s_off[P.world] < n ? s_off[P.world] : n;
    const int64_t gb = P.gb[P.rank];
    const int64_t gen = (int64_t)(uint32_t)flags[kFlagMarkGen] << 32;
    const int64_t goff = (n + kPartPer - 1) / kPartPer * kPartPer;   // npad
    uint64_t cov = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ntot;
         k += (int64_t)gridDim.x * blockDim.x) {
        int q = 0;
        while (q + 1 < P.world && s_off[q + 1] <= k) ++q;
        int64_t lo, hi;
        double x, y, th;
        if (q == P.rank) {                                  // own items: regular memory
            const uint64_t* it = reinterpret_cast<const uint64_t*>(P.self_items + (k - s_off[q]));
            x = __longlong_as_double((long long)ld_wt(it + 0));
            y = __longlong_as_double((long long)ld_wt(it + 1));
            th = __longlong_as_double((long long)ld_wt(it + 2));
            lo = (int64_t)ld_wt(it + 3) - gb;
            hi = (int64_t)ld_wt(it + 4) - gb;
        } else {
            const DistItem* it = items + (int64_t)q * P.L.cap_item + (k - s_off[q]);
            lo = (int64_t)ld_sys(&it->lo) - gb;
            hi = (int64_t)ld_sys(&it->hi) - gb;
            x = ld_sys_d(&it->x);
            y = ld_sys_d(&it->y);
            th = ld_sys_d(&it->th);
        }
        if (!(lo >= 0 && lo < hi && hi <= n)) {
            atomicOr(&flags[kFlagStatus], kDistStItems);
            continue;
        }
        xs[k] = x;
        ys[k] = y;
        ts[k] = th;
        mark[lo] = gen | (goff + k);                        // gather source goff + k (DeferParts.goff)
        for (int64_t b = (lo + kPartPer - 1) / kPartPer; b * kPartPer < hi; ++b)
            carry[b] = (int32_t)(goff + k);
        cov += (uint64_t)(hi - lo);
    }
    cov = wave_sum_u64(cov);
    if ((threadIdx.x & 63) == 0 && cov) atomicAdd(&s_cov, (unsigned long long)cov);
    __syncthreads();
    if (threadIdx.x == 0 && s_cov) atomicAdd((unsigned long long*)&scr->covered, s_cov);
    if (!arrive_last(counter)) return;
    if (threadIdx.x == 0) {
        const unsigned long long c = atomicExch((unsigned long long*)&scr->covered, 0ull);
        if ((int64_t)c != n || s_off[P.world] > n) atomicOr(&flags[kFlagStatus], kDistStItems);
    }
}

// wait for every rank's items and hand them to the fused kernel's resample
// gather (the single-GPU expand pass's inverse map): item k (ranks in order,
// each rank's items in position order) is stored at local index k of the
// particle arrays -- the pre-resample particles were packed already -- with a
// run mark (mark generation | npad + k: DeferParts.goff) at its first local position and the carry of
// every fused block whose first position it covers.  Items never outnumber the
// positions (disjoint, non-empty ranges), so k < n.  The last block checks that
// the ranges tile the shard (status kDistStItems otherwise).  The resample flag
// stays 1: the fused kernel gathers through the marks, at weight 1/NP.
__global__ __launch_bounds__(256) void dist_unpack_kernel(
    const int64_t n, double* __restrict__ xs, double* __restrict__ ys, double* __restrict__ ts,
    int64_t* __restrict__ mark, int32_t* __restrict__ carry, unsigned* __restrict__ counter,
    int32_t* __restrict__ flags, DistScratch* __restrict__ scr, const DistPeers P, StepIO io) {
    if (!dist_resampling(flags) || flags[kFlagFallback]) return;
    dist_wait(P, kXItem, dist_epoch(io), flags);
    __shared__ int64_t s_off[kDistMaxWorld + 1];
    if (threadIdx.x == 0) dist_item_offsets(P, s_off);
    __syncthreads();
    dist_unpack_items(n, xs, ys, ts, mark, carry, counter, flags, scr, P, s_off);
}

// ---------------------------------------------------------------- resample, one launch
// The whole exchange side of a resample step in ONE launch (one shard per
// process; the grid must be co-resident -- checked on the host -- because its
// blocks wait for one another):
//   A  every wave classifies its 512-element tile of w = w_un / s with the
//      global approximate prefix (the lean exact cumsum's pass A) and stages its
//      special elements; the last block scans the tile totals, pushes this
//      rank's specials (global index, rank-local increment prefix) into every
//      peer's slot, waits for every rank's, folds the global list in rank
//      order (one wave, 63 specials per round), derives the first positions
//      this rank's and the next rank's sources serve (lo0, hi0) and releases
//      the grid;
//   B  every wave expands its tile's exact cumsum from the classification it
//      kept in registers, counts the systematic positions at or below each
//      c_j (a run [s_j, e_j) per selected source) and places every run where
//      its positions are (dist_place_runs): this rank's part as the fused
//      kernel's run marks and carries, a peer's part at its first local
//      position in that peer's region.  World 1 ends here;
//   D  the last block publishes kXItem, waits for every rank's and releases
//      the grid; every block takes the positions other ranks serve
//      ([0, lo0) and [hi0, n) locally) from its region (dist_take_runs).
// The five-launch form (grids that are not co-resident) packs the items
// instead and dist_unpack_kernel hands them to the fused kernel.
constexpr int kDistTokenWait = 1 << 22;
constexpr int kDistBfLds = 2048;            // block offsets staged in LDS (nb_scan <= 2048: n <= 2^22)

// bounded wait of thread 0 for `token` in a write-through word; the block's
// threads then all see the released data (agent-scope acquire)
__device__ __forceinline__ bool dist_token_wait(const int32_t* word, const int32_t token,
                                                int32_t* flags) {
    __shared__ int s_go;
    if (threadIdx.x == 0) {
        int go = 0;
        const int bound = dist_dead(flags) ? 1 : kDistTokenWait;   // dead: one look, no poll
        for (int it = 0; it < bound; ++it) {
            if (ld_wt_i(word) == token) {
                go = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!go) dist_mark_dead(flags);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_go = go;
    }
    __syncthreads();
    return s_go != 0;
}

__device__ __forceinline__ void dist_token_release(int32_t* word, const int32_t token) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        st_wt_i(word, token);
    }
}

// Merged exchange, phase B: the runs of this lane's selected sources (global
// positions [lv, hv), local source j0 + k) that fall in destination d's shard.
// This rank's own positions get the fused kernel's inverse map directly -- a
// run mark (mark generation | npad + j) at the run's first position and the
// carry of every fused block whose first position lies in the run, as the
// single-GPU expand pass writes them; a peer's get the particle stored at the
// run's first local position of its region, tagged with the epoch and the
// run length, and the carries in its region (system-scope stores: complete
// when the storing block takes its ticket).
__device__ __forceinline__ void dist_store_run(DistRun* r, const double x, const double y, const double th,
                                               const uint64_t tag) {
    uint64_t* q = reinterpret_cast<uint64_t*>(r);
    __hip_atomic_store(q + 0, (uint64_t)__double_as_longlong(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, (uint64_t)__double_as_longlong(y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 2, (uint64_t)__double_as_longlong(th), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 3, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void dist_place_runs(const DistPeers& P, const int d,
                                                const int64_t (&lv)[kScanPer],
                                                const int64_t (&hv)[kScanPer], const int64_t j0,
                                                const int64_t npad, const int64_t gen,
                                                const uint64_t epoch, const double* __restrict__ xs,
                                                const double* __restrict__ ys,
                                                const double* __restrict__ ts,
                                                int64_t* __restrict__ mark,
                                                int32_t* __restrict__ carry) {
    const int lane = threadIdx.x & 63;
    const int64_t g0 = P.gb[d], g1 = P.gb[d + 1];
    const bool own = d == P.rank;
    DistRun* runs = reinterpret_cast<DistRun*>(P.base[d] + P.L.pitem);
    uint64_t* pcar = reinterpret_cast<uint64_t*>(P.base[d] + P.L.pcarry);
    const uint64_t etag = epoch << 32;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t lo = lv[k] > g0 ? lv[k] : g0, hi = hv[k] < g1 ? hv[k] : g1;
        const int64_t p0 = lo - g0, p1 = hi - g0, j = j0 + k;
        int64_t flo = 0, fhi = 0;
        if (hv[k] > lv[k] && lo < hi) {
            if (own) mark[p0] = gen | (npad + j);
            else dist_store_run(runs + p0, xs[j], ys[j], ts[j], etag | (uint64_t)(p1 - p0));
            flo = (p0 + kPartPer - 1) / kPartPer;
            fhi = (p1 + kPartPer - 1) / kPartPer;
        }
        // carries, written by the whole wave (a heavy source may own many)
        uint64_t act = __ballot(fhi > flo);
        while (act) {
            const int l = __ffsll((unsigned long long)act) - 1;
            act &= act - 1;
            const int64_t L = __shfl(flo, l, 64), H = __shfl(fhi, l, 64);
            if (own) {
                const int32_t v = (int32_t)(npad + __shfl(j, l, 64));
                for (int64_t f = L + lane; f < H; f += 64) carry[f] = v;
            } else {
                const uint64_t v = etag | (uint64_t)__shfl(p0, l, 64);
                for (int64_t f = L + lane; f < H; f += 64)
                    __hip_atomic_store(pcar + f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// Merged exchange, phase D (after every rank's kXItem): the positions of this
// shard that other ranks' sources serve -- [0, a) from the lower ranks, [b, n)
// from the higher ones, a / b from the global fold (lo0, hi0) -- take the
// runs the peers stored: the particle into the staging slot of gather index v
// (v = p below a, 2 npad + p from b: x[v - npad]), a run mark at p, and the
// carry of every fused block starting there.  The run lengths must tile both
// ranges (status kDistStItems otherwise; the last block checks).
__device__ void dist_take_runs(const DistPeers& P, const int64_t n, const int64_t npad,
                               const int64_t lo0, const int64_t hi0, const int64_t gen,
                               const uint64_t epoch, double* __restrict__ xs,
                               double* __restrict__ ys, double* __restrict__ ts,
                               int64_t* __restrict__ mark, int32_t* __restrict__ carry,
                               unsigned* __restrict__ counter, int32_t* __restrict__ flags,
                               DistScratch* __restrict__ scr) {
    __shared__ unsigned long long s_cov;
    __shared__ int s_bad;
    if (threadIdx.x == 0) {
        s_cov = 0;
        s_bad = 0;
    }
    __syncthreads();
    const int64_t gb = P.gb[P.rank];
    auto local = [&](int64_t v) {
        v -= gb;
        return v < 0 ? (int64_t)0 : (v > n ? n : v);
    };
    const int64_t a = local(lo0), b = local(hi0) > a ? local(hi0) : a;
    const int64_t m = a + (n - b);
    const DistRun* runs = reinterpret_cast<const DistRun*>(P.base[P.rank] + P.L.pitem);
    const uint64_t* pcar = reinterpret_cast<const uint64_t*>(P.base[P.rank] + P.L.pcarry);
    const uint32_t e32 = (uint32_t)epoch;
    uint64_t cov = 0;
    bool bad = false;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = t < a ? t : b + (t - a);
        const uint64_t tag = ld_sys(&runs[p].tag);
        if ((uint32_t)(tag >> 32) == e32) {
            const int64_t v = p < a ? p : 2 * npad + p;
            xs[v - npad] = ld_sys_d(&runs[p].x);
            ys[v - npad] = ld_sys_d(&runs[p].y);
            ts[v - npad] = ld_sys_d(&runs[p].th);
            mark[p] = gen | v;
            cov += tag & 0xFFFFFFFFu;
        }
        if (p % kPartPer == 0) {                            // a fused block starts here
            const uint64_t c = ld_sys(pcar + p / kPartPer);
            const int64_t p0 = (int64_t)(uint32_t)c;
            if ((uint32_t)(c >> 32) == e32 && p0 <= p)
                carry[p / kPartPer] = (int32_t)(p < a ? p0 : 2 * npad + p0);
            else
                bad = true;
        }
    }
    cov = wave_sum_u64(cov);
    if ((threadIdx.x & 63) == 0 && cov) atomicAdd(&s_cov, (unsigned long long)cov);
    if (bad) s_bad = 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_cov) atomicAdd((unsigned long long*)&scr->covered, s_cov);
        if (s_bad) atomicOr(&flags[kFlagStatus], kDistStItems);
    }
    if (!arrive_last(counter)) return;
    if (threadIdx.x == 0) {
        const unsigned long long c = atomicExch((unsigned long long*)&scr->covered, 0ull);
        if ((int64_t)c != m) atomicOr(&flags[kFlagStatus], kDistStItems);
    }
}

// the global fold over every rank's specials (in this rank's exchange region),
// by wave 0 of the calling block: lean_place_fold's 63-per-round walk.  Writes
// every global SpecialOut; sets the fallback flag when a run check fails.
__device__ void dist_fold_global(const DistPeers& P, const int64_t* s_off, const uint64_t* s_koff,
                                 const int64_t M, const uint64_t ktot, const int64_t n_global,
                                 SpecialOut* __restrict__ out, int32_t* __restrict__ flags) {
    __shared__ int s_bad;
    if (threadIdx.x == 0) {
        s_bad = 0;
        flags[kFlagNSpecial] = (int32_t)M;
    }
    __syncthreads();
    const char* mine = P.base[P.rank];
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        auto load_special = [&](const int64_t m, SpecialIn& e) {
            int q = 0;
            while (q + 1 < P.world && s_off[q + 1] <= m) ++q;
            const SpecialIn* src = reinterpret_cast<const SpecialIn*>(mine + P.L.spec) + (int64_t)q * P.L.cap_spec;
            e = ld_sys_struct(&src[m - s_off[q]]);
            e.P += s_koff[q];
        };
        double s = 0.0;
        bool bad = false;
        for (int64_t t0 = 0; t0 < M; t0 += 63) {
            const int64_t m = t0 + lane;
            SpecialIn e{};
            if (m < M) load_special(m, e);
            int64_t nidx = __shfl_down((long long)e.idx, 1, 64);
            uint64_t nP = (uint64_t)__shfl_down((long long)e.P, 1, 64);
            if (m + 1 >= M) {
                nidx = n_global;
                nP = ktot;
            }
            const bool mine_l = (lane < 63) && (m < M);
            const bool run = mine_l && (nidx - e.idx > 1);
            const uint64_t K = nP - e.P;
            const int E = e.E;
            double lo = -__builtin_inf(), hi = __builtin_inf(), ku = 0.0;
            if (run) {
                lo = (E == -1022) ? 0.0 : ldexp(1.0, E);
                hi = (E == -1022) ? 0x1p-1021 : ldexp(1.0, E + 1);
                ku = (double)K * ldexp(1.0, E - 52);
                if ((double)K >= 0x1p53) bad = true;
            }
            const double w = mine_l ? e.w : 0.0;
            // the chain: two dependent adds per special, the operands read into
            // scalars (fully unrolled: the reads do not wait on the chain); each
            // lane keeps the sums at its own special and checks its binade after
            double cs = 0.0, cr = 0.0;
            const int lim = (M - t0 < 63) ? (int)(M - t0) : 63;
#pragma unroll
            for (int l = 0; l < 63; ++l) {
                if (l < lim) {                            // wave-uniform
                    s = s + readlane_d(w, l);             // the special element's own add
                    if (lane == l) cs = s;
                    s = s + readlane_d(ku, l);            // the run: K ulps, exact
                    if (lane == l) cr = s;
                }
            }
            if (lane < lim && (!(cs >= lo) || !(cs < hi) || !(cr < hi))) bad = true;   // its run keeps the binade
            if (mine_l) {
                SpecialOut o;
                o.cs = cs;
                o.P = e.P;
                o.E = e.E;
                o.pad = 0;
                st_wt_struct(&out[m], o);
            }
        }
        if (__any(bad) && lane == 0) s_bad = 1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_bad) flags[kFlagStatus] |= 2;
        st_wt_i(&flags[kFlagFallback], s_bad ? 1 : 0);
    }
}

__global__ __launch_bounds__(kScanThreads) void dist_resample_merged_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_in, const double np_recip,
    const int64_t n, const double* __restrict__ boff, const double delta,
    SpecialIn* __restrict__ stage, uint64_t* __restrict__ bk, int32_t* __restrict__ bf,
    uint64_t* __restrict__ boffk, int32_t* __restrict__ bofff, uint64_t* __restrict__ ktot_p,
    int32_t* __restrict__ nspec_p, unsigned* __restrict__ tk, int32_t* __restrict__ flags,
    SpecialOut* __restrict__ spec_go, DistScratch* __restrict__ scr,
    double* __restrict__ xs, double* __restrict__ ys, double* __restrict__ ts,
    int64_t* __restrict__ mark, int32_t* __restrict__ carry, const DistPeers P, StepIO io,
    const PredictConst pc, const uint64_t seed, const int ntiles) {
    if (!dist_resampling(flags)) return;
    __shared__ int64_t s_off[kDistMaxWorld + 1];
    __shared__ uint64_t s_koff[kDistMaxWorld + 1];
    const uint64_t epoch = dist_epoch(io);
    const int32_t tokA = ld_wt_i(&scr->rel[0]) + 1;        // read before this block arrives
    const int32_t tokB = ld_wt_i(&scr->rel[1]) + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * kTilesPerBlock + wave;
    const bool active = tile < ntiles;
    const int64_t gbase = P.gb[P.rank], n_global = P.gb[P.world];
    if (blockIdx.x == 0) PROBE_AT(16);
    // ---- A: classify + stage
    TileScan tsc;
    uint64_t ktile = 0, kofs, kblk;
    int32_t ftile = 0, fofs, fblk;
    if (active)
        wave_tile_classify(w_un, *s_in, np_recip, n, tile, boff[tile] + scr->base_off, delta, tsc,
                           ktile, ftile);
    block_tile_offsets(ktile, ftile, kofs, fofs, kblk, fblk);
    if (active) wave_tile_stage(blockIdx.x, tile, tsc, kofs, fofs, kblk, fblk, stage, bk, bf);
    else if (threadIdx.x == 0) {
        st_wt(&bk[blockIdx.x], kblk);
        st_wt_i(&bf[blockIdx.x], fblk);
    }
    if (arrive_last(tk)) {
        PROBE_AT(17);
        __shared__ uint64_t shk[kScanThreads / 64 + 1];
        __shared__ int32_t shf[kScanThreads / 64 + 1];
        block_scan_array<uint64_t, kScanThreads>(bk, boffk, gridDim.x, ktot_p, shk, true);
        __syncthreads();
        block_scan_array<int32_t, kScanThreads>(bf, bofff, gridDim.x, nspec_p, shf, true);
        __syncthreads();
        const int32_t ns = ld_wt_i(nspec_p);
        const uint64_t kt = ld_wt(ktot_p);
        PROBE_AT(18);
        // this rank's specials in order -> every peer's slot (tile by a search of
        // the block offsets, staged in LDS)
        __shared__ int32_t s_bf[kDistBfLds];
        const bool bf_lds = (int)gridDim.x <= kDistBfLds;
        if (bf_lds)
            for (int k = threadIdx.x; k < (int)gridDim.x; k += blockDim.x) s_bf[k] = ld_wt_i(&bofff[k]);
        __syncthreads();
        auto bf_at = [&](const int k) { return bf_lds ? s_bf[k] : ld_wt_i(&bofff[k]); };
        for (int32_t m = threadIdx.x; m < ns; m += blockDim.x) {
            int lo = 0, hi = (int)gridDim.x - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (bf_at(mid) <= m) lo = mid;
                else hi = mid - 1;
            }
            SpecialIn e = ld_wt_struct(&stage[(int64_t)lo * kScanBlock + (m - bf_at(lo))]);
            e.P += ld_wt(&boffk[lo]);
            e.idx += gbase;
            if (m < P.L.cap_spec)
                for (int q = 0; q < P.world; ++q)
                    reinterpret_cast<SpecialIn*>(P.base[q] + P.L.spec)[(int64_t)P.rank * P.L.cap_spec + m] = e;
        }
        if ((int)threadIdx.x < P.world) {
            int64_t* hdr = reinterpret_cast<int64_t*>(P.base[threadIdx.x] + P.L.spec_hdr) + 2 * P.rank;
            hdr[0] = ns < P.L.cap_spec ? ns : P.L.cap_spec;
            hdr[1] = (int64_t)kt;
        }
        if (ns > P.L.cap_spec && threadIdx.x == 0) atomicOr(&flags[kFlagStatus], kDistStItems);
        __syncthreads();
        dist_signal(P, kXSpec, epoch);
        PROBE_AT(19);
        dist_wait(P, kXSpec, epoch, flags);
        PROBE_AT(20);
        if (threadIdx.x == 0) {
            const char* mine = P.base[P.rank];
            int64_t no = 0;
            uint64_t ko = 0;
            for (int q = 0; q < P.world; ++q) {
                const int64_t* hdr = reinterpret_cast<const int64_t*>(mine + P.L.spec_hdr) + 2 * q;
                s_off[q] = no;
                s_koff[q] = ko;
                no += (int64_t)ld_sys(hdr);
                ko += ld_sys(hdr + 1);
            }
            s_off[P.world] = no;
            s_koff[P.world] = ko;
        }
        __syncthreads();
        dist_fold_global(P, s_off, s_koff, s_off[P.world], s_koff[P.world], n_global, spec_go, flags);
        PROBE_AT(21);
        if (threadIdx.x == 0) {
            const int64_t sb = s_off[P.rank];
            double cl = -INFINITY;
            int64_t lo0 = 0;
            if (P.rank > 0 && sb > 0) {
                const SpecialOut p = ld_wt_struct(&spec_go[sb - 1]);
                cl = p.cs + (double)(s_koff[P.rank] - p.P) * ldexp(1.0, p.E - 52);
                const double ofs = resample_offset(io.ofs[io.ctr[0]], np_recip, seed, (uint32_t)io.ctr[1]);
                lo0 = positions_upto(cl, n_global, pc.rstep, ofs);
            }
            scr->spec_base = (int32_t)sb;
            scr->k_base = s_koff[P.rank];
            scr->nspec_g = (int32_t)s_off[P.world];
            scr->ktot_g = s_koff[P.world];
            // the first position the next rank's sources serve: everything
            // from there on (and before lo0) arrives from the peers
            int64_t hi0 = n_global;
            if (P.rank + 1 < P.world) {
                const int64_t sb1 = s_off[P.rank + 1];
                double c1 = -INFINITY;
                if (sb1 > 0) {
                    const SpecialOut p1 = ld_wt_struct(&spec_go[sb1 - 1]);
                    c1 = p1.cs + (double)(s_koff[P.rank + 1] - p1.P) * ldexp(1.0, p1.E - 52);
                }
                const double ofs = resample_offset(io.ofs[io.ctr[0]], np_recip, seed, (uint32_t)io.ctr[1]);
                hi0 = positions_upto(c1, n_global, pc.rstep, ofs);
            }
            scr->c_left = cl;
            scr->lo0 = lo0;
            scr->hi0 = hi0;
        }
        dist_token_release(&scr->rel[0], tokA);
        PROBE_AT(22);
    } else {
        dist_token_wait(&scr->rel[0], tokA, flags);
    }
    __syncthreads();
    if (ld_wt_i(&flags[kFlagFallback])) return;             // block-uniform
    // ---- B: expand, positions; every run placed where its positions are
    const double ofs = resample_offset(io.ofs[io.ctr[0]], np_recip, seed, (uint32_t)io.ctr[1]);
    const int32_t sb = ld_wt_i(&scr->spec_base);
    const int64_t npad = (int64_t)ntiles * kPartPer;        // the gather offset (DeferParts.goff)
    const int64_t gen = (int64_t)(uint32_t)flags[kFlagMarkGen] << 32;
    if (active) {
        const uint64_t kb = ld_wt(&scr->k_base);
        const int64_t b = blockIdx.x;
        const uint64_t bk0 = ld_wt(&boffk[b]) + kofs + kb;
        const int32_t bf0 = ld_wt_i(&bofff[b]) + fofs + sb;
        uint64_t kin = bk0 + tsc.kex;
        int32_t m = bf0 + tsc.fex;
        double out[kScanPer];
        SpecialOut p = ld_wt_struct(&spec_go[m > 0 ? m - 1 : 0]);
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            kin += tsc.kk[k];
            if (tsc.ff[k]) {
                p = ld_wt_struct(&spec_go[m]);
                out[k] = p.cs;
                ++m;
            } else {
                out[k] = p.cs + (double)(kin - p.P) * ldexp(1.0, p.E - 52);
            }
        }
        double cprev = __shfl_up(out[kScanPer - 1], 1, 64);
        if (lane == 0) {
            if (tile == 0) {
                cprev = ld_wt_d(&scr->c_left);
            } else {
                const SpecialOut q = ld_wt_struct(&spec_go[bf0 - 1]);
                cprev = q.cs + (double)(bk0 - q.P) * ldexp(1.0, q.E - 52);
            }
        }
        int64_t sj = positions_upto(cprev, n_global, pc.rstep, ofs);
        const int64_t j0 = tile * kWaveTile + 8 * lane;
        int64_t lv[kScanPer], hv[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int64_t j = j0 + k;
            int64_t ej = sj;
            if (j < n) {
                ej = positions_upto(out[k], n_global, pc.rstep, ofs);
                if (gbase + j == n_global - 1) {
                    if (ej < n_global) atomicOr(&flags[kFlagStatus], 1);   // IndexError in the reference
                    ej = n_global;
                }
            }
            lv[k] = sj;
            hv[k] = ej;
            sj = ej;
        }
        // the destinations this wave's runs reach (positions are monotone
        // over the lanes): usually this rank alone
        const int64_t wlo = __shfl(lv[0], 0, 64), whi = __shfl(hv[kScanPer - 1], 63, 64);
        if (whi > wlo) {
            const int dlo = dist_owner(P, wlo), dhi = dist_owner(P, whi - 1);
            for (int d = dlo; d <= dhi; ++d)
                dist_place_runs(P, d, lv, hv, j0, npad, gen, epoch, xs, ys, ts, mark, carry);
        }
    }
    PROBE_MAX(23);
    if (P.world == 1) return;                               // every run is this rank's own
    // ---- D: publish, wait for every rank's runs, take the received ones
    if (arrive_last(tk + kTicketWords)) {                   // (drains this block's run stores)
        dist_signal(P, kXItem, epoch);
        PROBE_AT(26);
        dist_wait(P, kXItem, epoch, flags);
        dist_token_release(&scr->rel[1], tokB);
    } else {
        dist_token_wait(&scr->rel[1], tokB, flags);
    }
    __syncthreads();
    dist_take_runs(P, n, npad, (int64_t)ld_wt(&scr->lo0), (int64_t)ld_wt(&scr->hi0), gen, epoch, xs,
                   ys, ts, mark, carry, tk + 3 * kTicketWords, flags, scr);
}

// ---------------------------------------------------------------- record
// The shard's reduction record from the fused kernel's block partials,
// pushed into every peer's G1 slot (parity = epoch & 1), then kXG1.  One
// workgroup of kFinThreads lanes, laid out like finalize_deferred_kernel:
// every lane issues the loads of its blocks and leaves first; the sums are
// wave butterflies (a fixed order); the tie-window candidates are the first
// kDistWin blocks whose max is within 2^-48 of M, found in parallel (the
// window then reads only those blocks).
__device__ __forceinline__ void dist_record(const int64_t n, const DeferParts& dp,
                                            const double* __restrict__ w_un,
                                            const int32_t* __restrict__ tail_leaves,
                                            const int32_t* __restrict__ tail_ops,
                                            const int32_t n_tail_leaves, const int32_t n_tail_ops,
                                            const double* __restrict__ xs,
                                            const double* __restrict__ ys,
                                            const double* __restrict__ ts, const DistPeers& P,
                                            const uint64_t epoch, double* sh) {
    __shared__ double s_q[12][kFinThreads];             // lane sums (transposed reduction)
    __shared__ double s_wm[kFinWaves];
    __shared__ unsigned long long s_cand[kDistWin], s_mblk;
    __shared__ DistRec rec;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
    const int64_t gbase = P.gb[P.rank];
    if (tid < kDistWin) s_cand[tid] = ~0ull;
    if (tid == 0) s_mblk = ~0ull;
    // ---- loads up front: this lane's blocks tid + kFinThreads k and its leaves
    double pm[kFinRegBlocks], q[kFinRegBlocks][11];
    bool has[kFinRegBlocks];
#pragma unroll
    for (int kp = 0; kp < kFinRegBlocks / 2; ++kp) {     // neighbour pairs (finalize_deferred_kernel)
        const int64_t b = fin_blk(tid, 2 * kp);
        has[2 * kp] = b < nb;
        has[2 * kp + 1] = b + 1 < nb;
        const int64_t bb = has[2 * kp] ? b : 0;
        const double2 t = *reinterpret_cast<const double2*>(dp.pmax + bb);
        pm[2 * kp] = t.x;
        pm[2 * kp + 1] = t.y;
#pragma unroll
        for (int j = 0; j < 11; ++j) {
            const double2 u = *reinterpret_cast<const double2*>(dp.ps[j] + bb);
            q[2 * kp][j] = u.x;
            q[2 * kp + 1][j] = u.y;
        }
    }
    const int part = tid & (kFinLeafLanes - 1);
    double L[4];                                   // fused-block subtree sums
    {
        const int64_t c = tid / kFinLeafLanes;
        const double* Lp = dp.leaf + 16 * (c < nfull ? c : 0) + 4 * part;
#pragma unroll
        for (int j = 0; j < 4; ++j) L[j] = Lp[j];
    }
    const int64_t bx0 = tid + (int64_t)kFinThreads * kFinRegBlocks;   // NP > 2^20 only
    double mlane = -1.0;
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k)
        if (has[k]) mlane = fmax(mlane, pm[k]);
    for (int64_t b = bx0; b < nb; b += kFinThreads) mlane = fmax(mlane, dp.pmax[b]);
    // lane sums scaled by the lane's max; T = sum of w_un (unscaled)
    double acc[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = 0.0;
    {
        const double rm = mlane > 0.0 ? 1.0 / mlane : 0.0;
        auto add = [&](const double p, const double* qq) {
            if (mlane > 0.0) {
                const double r = p * rm;
                acc[0] += r * qq[0];
                acc[1] += (r * r) * qq[1];
#pragma unroll
                for (int j = 2; j < 11; ++j) acc[j] += r * qq[j];
            }
            acc[11] += p * qq[0];
        };
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k)
            if (has[k]) add(pm[k], q[k]);
        for (int64_t b = bx0; b < nb; b += kFinThreads) {
            double qq[11];
#pragma unroll
            for (int j = 0; j < 11; ++j) qq[j] = dp.ps[j][b];
            add(dp.pmax[b], qq);
        }
    }
    const double mx = wave_max_f64(mlane);
    if (lane == 0) s_wm[wave] = mx;
    // ---- np.sum buffer partials: 4 lanes per 8192-element buffer, pairwise tree
    for (int64_t c0 = 0; c0 < nfull; c0 += kFinBufPerRound) {
        const int64_t c = c0 + tid / kFinLeafLanes;
        double v = 0.0;
        if (c < nfull) {
            if (c0 > 0) {
                const double* Lp = dp.leaf + 16 * c + 4 * part;
#pragma unroll
                for (int j = 0; j < 4; ++j) L[j] = Lp[j];
            }
            v = (L[0] + L[1]) + (L[2] + L[3]);
        }
        static_assert(kFinLeafLanes == 4, "two quad swaps");
        {
            const double o = dpp_f64<kDppXor1>(v);
            v = (part & 1) ? (o + v) : (v + o);              // left operand = lower lane
        }
        {
            const double o = dpp_f64<kDppXor2>(v);
            v = (part & 2) ? (o + v) : (v + o);
        }
        if (part == 0 && c < nfull) sh[c] = v;
    }
    __syncthreads();
    PROBE_AT(0);
    double M = s_wm[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) M = fmax(M, s_wm[w]);
    const double thr = M * (1.0 - 0x1p-48);                 // tie window (2^-48 relative)
    {
        const double rl = (mlane > 0.0 && M > 0.0) ? mlane / M : 0.0;
        acc[0] *= rl;
        acc[1] *= rl * rl;
#pragma unroll
        for (int j = 2; j < 11; ++j) acc[j] *= rl;
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) s_q[j][tid] = acc[j];
    // first block holding M, and the first kDistWin candidate blocks (index order)
    if (M > 0.0) {
        unsigned long long mb = ~0ull;
#pragma unroll
        for (int k = kFinRegBlocks - 1; k >= 0; --k)
            if (has[k] && pm[k] == M) mb = (unsigned long long)fin_blk(tid, k);
        for (int64_t b = bx0; b < nb && mb == ~0ull; b += kFinThreads)
            if (dp.pmax[b] == M) mb = (unsigned long long)b;
        if (mb != ~0ull) atomicMin(&s_mblk, mb);
    }
    PROBE_AT(1);
    unsigned long long prev = 0;                            // candidates must be >= prev
    for (int r = 0; r < kDistWin; ++r) {
        unsigned long long cb = ~0ull;
        if (M > 0.0) {
#pragma unroll
            for (int k = kFinRegBlocks - 1; k >= 0; --k) {
                const unsigned long long b = (unsigned long long)fin_blk(tid, k);
                if (has[k] && pm[k] >= thr && b >= prev) cb = b;
            }
            for (int64_t b = bx0; b < nb && cb == ~0ull; b += kFinThreads)
                if ((unsigned long long)b >= prev && dp.pmax[b] >= thr) cb = (unsigned long long)b;
        }
        if (cb != ~0ull) atomicMin(&s_cand[r], cb);
        __syncthreads();
        const unsigned long long got = s_cand[r];
        if (got == ~0ull) break;                            // block-uniform
        prev = got + 1;
    }
    __syncthreads();
    PROBE_AT(2);
    // the 12 sums (written to s_q before the candidate rounds' barriers): wave w
    // reduces quantities w and w + 8 -- lane-strided reads, then one butterfly
    // with the lower lane on the left (a fixed order; twelve butterflies per
    // wave were a 3.7 us dependent chain of lane permutes)
    for (int j = wave; j < 12; j += kFinWaves) {
        double r = s_q[j][lane];
#pragma unroll
        for (int m = 1; m < kFinThreads / 64; ++m) r = r + s_q[j][lane + 64 * m];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double o = xor_f64(r, d);
            r = (lane & d) ? (o + r) : (r + o);
        }
        if (lane == 0) {
            if (j < 11) rec.q[j] = r;
            else rec.T = r;
        }
    }
    if (nch > nfull) {
        __shared__ double tl[1024];
        const double t = tail_chunk_sum(w_un + nfull * kSumChunk, tail_leaves, tail_ops, n_tail_leaves,
                                        n_tail_ops, tl);
        if (tid == 0) sh[nfull] = t;
    }
    if (tid == 0) {
        rec.M = M;
        rec.nchunk = nch;
        rec.x0[0] = xs[0];
        rec.x0[1] = ys[0];
        rec.x0[2] = ts[0];
        rec.nwin = 0;
    }
    __syncthreads();
    // ---- tie window: the first kDistWin elements (index order) with w_un >= thr,
    // from the candidate blocks (usually one element: M) -- one element per lane,
    // a candidate block per round (block-uniform loop)
    PROBE_AT(3);
#ifndef SLAM_FIN_AB                                   // finalize-width A/B builds skip the sharded path's check
    static_assert(kFinThreads == kPartPer, "one lane per element of a fused block");
#endif
    {
        __shared__ int s_wh[kFinWaves];
        int cnt = 0;
        for (int r = 0; r < kDistWin && cnt < kDistWin && M > 0.0; ++r) {
            const unsigned long long cb = s_cand[r];
            if (cb == ~0ull) break;
            const int64_t i = (int64_t)cb * kPartPer + tid;
            const double v = (i < n) ? w_un[i] : -1.0;
            const bool hit = v >= thr;
            const unsigned long long bal = __ballot(hit);
            if (lane == 0) s_wh[wave] = __popcll(bal);
            __syncthreads();
            int before = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < kFinWaves; ++w) {
                before += (w < wave) ? s_wh[w] : 0;
                tot += s_wh[w];
            }
            const int rank = cnt + before + __popcll(bal & ((1ull << lane) - 1ull));
            if (hit && rank < kDistWin) {
                DistWin& wv = rec.win[rank];
                wv.idx = gbase + i;
                wv.v = v;
                wv.x[0] = xs[i];
                wv.x[1] = ys[i];
                wv.x[2] = ts[i];
            }
            cnt += tot;
            __syncthreads();                                // s_wh reused
        }
        if (tid == 0) rec.nwin = cnt < kDistWin ? cnt : kDistWin;
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
        if (rec.idx < 0 && s_mblk != ~0ull) {
            const int64_t b = (int64_t)s_mblk;
            rec.idx = gbase + dp.pidx[b];
            for (int j = 0; j < 3; ++j) rec.xc[j] = dp.pxe[j][b];
        }
    }
    __syncthreads();
    // ---- push into every peer's slot (parity = epoch & 1)
    PROBE_AT(28);
    const int64_t words = (int64_t)sizeof(DistRec) / 8;
    for (int qq = dist_push_lo(P); qq < dist_push_hi(P); ++qq) {
        char* slot = P.base[qq] + P.L.g1 + ((int64_t)(epoch & 1) * P.world + P.rank) * P.L.rec_stride;
        uint64_t* dst = reinterpret_cast<uint64_t*>(slot);
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&rec);
        for (int64_t k = tid; k < words; k += kFinThreads) dst[k] = src[k];
        double* dch = reinterpret_cast<double*>(slot + sizeof(DistRec));
        for (int64_t c = tid; c < nch; c += kFinThreads) dch[c] = sh[c];
    }
    __syncthreads();
    dist_signal(P, kXG1, epoch);
    PROBE_AT(29);
}

// ---------------------------------------------------------------- finalize
// Wait for every rank's record and form the step's global result -- the same
// on every rank: s = np.sum in the reference's order (buffer partials, ranks in
// order: staged through LDS, then one left-to-right chain), the exact max and
// first argmax of w = w_un / s, ESS and covariance from the scaled sums, the
// result record, the next step's resample flag and, when it resamples, this
// rank's exact-cumsum base offsets.
__device__ __forceinline__ void dist_finalize(const int64_t n, const DeferParts& dp,
                                              double* __restrict__ s_cur, double* __restrict__ refp,
                                              int32_t* __restrict__ flags, const double ess_th,
                                              const StepIO& io, const double np_recip,
                                              double* __restrict__ boff,
                                              DistScratch* __restrict__ scr, const DistPeers& P,
                                              const uint64_t epoch, double* sh) {
    constexpr int kStage = 2048;                            // LDS doubles per staged round
    __shared__ double s_rq[kDistMaxWorld][11];
    __shared__ double s_M[kDistMaxWorld], s_T[kDistMaxWorld];
    __shared__ int64_t s_nc[kDistMaxWorld + 1];
    __shared__ double s_s;
    __shared__ int32_t s_do_off;
    const int tid = threadIdx.x;
    __shared__ DistRec s_rec[kDistMaxWorld];
    dist_wait(P, kXG1, epoch, flags);
    PROBE_AT(30);
    const char* g1 = P.base[P.rank] + P.L.g1 + (int64_t)(epoch & 1) * P.world * P.L.rec_stride;
    auto rec_of = [&](int q) { return reinterpret_cast<const DistRec*>(g1 + (int64_t)q * P.L.rec_stride); };
    {   // every rank's record into LDS (one parallel round of system-scope loads)
        constexpr int kW = (int)(sizeof(DistRec) / 8);
        for (int e = tid; e < P.world * kW; e += kFinThreads) {
            const int q = e / kW, k = e - q * kW;
            reinterpret_cast<uint64_t*>(&s_rec[q])[k] = ld_sys(reinterpret_cast<const uint64_t*>(rec_of(q)) + k);
        }
    }
    __syncthreads();
    if (tid < P.world) {
        const DistRec& r = s_rec[tid];
        s_M[tid] = r.M;
        s_T[tid] = r.T;
        s_nc[tid] = r.nchunk;
        for (int j = 0; j < 11; ++j) s_rq[tid][j] = r.q[j];
    }
    __syncthreads();
    if (tid == 0) {                                         // s_nc -> exclusive prefix
        int64_t o = 0;
        for (int q = 0; q < P.world; ++q) {
            const int64_t c = s_nc[q];
            s_nc[q] = o;
            o += c;
        }
        s_nc[P.world] = o;
    }
    __syncthreads();
    // np.sum (particle_filter.py:234): buffer partials left to right, ranks in order
    const int64_t ntot = s_nc[P.world];
    double s = 0.0;
    for (int64_t g0 = 0; g0 < ntot; g0 += kStage) {
        const int64_t cnt = ntot - g0 < kStage ? ntot - g0 : kStage;
        for (int64_t e = tid; e < cnt; e += kFinThreads) {
            const int64_t g = g0 + e;
            int q = 0;
            while (q + 1 < P.world && s_nc[q + 1] <= g) ++q;
            const double* ch = reinterpret_cast<const double*>(reinterpret_cast<const char*>(rec_of(q)) +
                                                               sizeof(DistRec));
            sh[e] = ld_sys_d(&ch[g - s_nc[q]]);
        }
        __syncthreads();
        if (tid == 0) s = lds_chain_sum(s, sh, (int)cnt);     // same adds, next 16 words in flight
        __syncthreads();
    }
    if (tid == 0) {
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
            const DistRec& r = s_rec[win];
            const int nw = (int)r.nwin;
            int k = 0;
            while (k < nw && !(r.win[k].v / s == mval)) ++k;
            if (k < nw) {
                tot.maxi = r.win[k].idx;
                for (int j = 0; j < 3; ++j) xe[j] = r.win[k].x[j];
            } else {                                        // window exhausted: M's own element
                tot.maxi = r.idx;
                for (int j = 0; j < 3; ++j) xe[j] = r.xc[j];
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
            tot.maxv = np_recip;
            tot.maxi = 0;
            for (int j = 0; j < 3; ++j) xe[j] = s_rec[0].x0[j];
            tot.sw = 1.0;
            tot.sw2 = np_recip;                             // ESS = NP
            for (int j = 0; j < 3; ++j) tot.m1[j] = NAN;
            for (int j = 0; j < 6; ++j) tot.m2[j] = NAN;
            st |= kDistStDegenerate;
        }
        flags[kFlagStatus] |= st;
        const int32_t stp = io.ctr[0];
        write_result_xe(tot, xe, refp, s, flags, ess_th, io.ess_band, io.res + stp, -1);
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

// RECORD / FINALIZE: one workgroup.  A process holding one shard runs both in
// one launch (push, then wait for the peers); a process holding several
// (LOCAL mode, one stream) launches every shard's record before any finalize.
template <bool RECORD, bool FINALIZE>
__global__ __launch_bounds__(kFinThreads) void dist_reduce_kernel(
    const int64_t n, const DeferParts dp, const double* __restrict__ w_un,
    const int32_t* __restrict__ tail_leaves, const int32_t* __restrict__ tail_ops,
    const int32_t n_tail_leaves, const int32_t n_tail_ops, const double* __restrict__ xs,
    const double* __restrict__ ys, const double* __restrict__ ts, double* __restrict__ s_cur,
    double* __restrict__ refp, int32_t* __restrict__ flags, const double ess_th, StepIO io,
    const double np_recip, double* __restrict__ boff, DistScratch* __restrict__ scr,
    const DistPeers P) {
    __shared__ double sh[2048];                             // buffer partials (nch <= 2048)
    const uint64_t epoch = dist_epoch(io);
    PROBE_AT(27);
    if (RECORD)
        dist_record(n, dp, w_un, tail_leaves, tail_ops, n_tail_leaves, n_tail_ops, xs, ys, ts, P,
                    epoch, sh);
    if (FINALIZE) {
        if (RECORD) __syncthreads();
        dist_finalize(n, dp, s_cur, refp, flags, ess_th, io, np_recip, boff, scr, P, epoch, sh);
        PROBE_AT(31);
    }
}

}  // namespace slam
