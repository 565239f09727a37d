// pf_shard.inl -- kernels of the multi-GPU (sharded) particle filter.
//
// The particles of one filter are split into contiguous shards, one per GPU.
// Exchange points (done by the caller, e.g. torch.distributed over RCCL):
//   A  all-gather of the shards' approximate weight totals (exact-cumsum classification)
//   B  all-gather of the shards' special-element lists (global sequential fold)
//   C  all-to-all of the resampled particles (global systematic resampling)
//   D  all-gather of the np.sum buffer partials (global normalisation, numpy order)
//   E  all-gather of the shards' reduction records (argmax, ESS, moments)
// Every rank folds the gathered data in rank order, so all ranks hold the
// same bit-identical global result -- and the same result as one GPU running
// all particles.
#pragma once
#include "pf_kernels.hpp"

namespace slam {

struct ShardRecord {
    BlockPartial bp;
    double x_cand[3];       // state of the shard's argmax particle
    double pad;
};

struct ShardItem {          // resampled particle with its global destination range
    double x, y, th;
    int64_t lo, hi;
};

struct ShardScratch {
    double ofs_host = 0.0;          // staging word for async copies
    bool host_noise = false;        // this step's noise came from the host
    int64_t* meta_dev = nullptr;    // [world*2] nspec, ktot per rank (device copy)
    int64_t* gb_dev = nullptr;      // [world+1] shard bases
    int64_t* cnt_dev = nullptr;     // [2*world] start/end per destination
    int64_t* off_dev = nullptr;     // [world+1] send offsets
    SpecialIn* spec_g = nullptr;    // global special list
    SpecialOut* spec_go = nullptr;  // its fold
    int64_t spec_cap = 0;
    int32_t* spec_base = nullptr;   // [1]
    uint64_t* k_base = nullptr;     // [1]
    int32_t* nspec_g = nullptr;     // [1]
    uint64_t* ktot_g = nullptr;     // [1]
    double* base_off = nullptr;     // [1]
    double* c_left = nullptr;       // [1]
    int64_t* hi = nullptr;          // [n_local] positions count(c_j)
    int64_t lo0_host = 0;
    int32_t world = 0;
    std::vector<int64_t> gb, start, end, off;
    int64_t n_send = 0;
};

// base_off = sum of the lower ranks' approximate totals (rank order)
__global__ void shard_prefix_kernel(const double* __restrict__ totals, const int32_t rank,
                                    double* __restrict__ out) {
    if (threadIdx.x || blockIdx.x) return;
    double s = 0.0;
    for (int r = 0; r < rank; ++r) s = s + totals[r];
    *out = s;
}

__global__ void shard_meta_kernel(const int32_t* __restrict__ nspec, const uint64_t* __restrict__ ktot,
                                  int64_t* __restrict__ meta) {
    if (threadIdx.x || blockIdx.x) return;
    meta[0] = *nspec;
    meta[1] = (int64_t)*ktot;
}

// concatenate the gathered lists into one global list with global increment prefixes
__global__ void shard_concat_kernel(const SpecialIn* __restrict__ lists, const int64_t cap,
                                    const int64_t* __restrict__ meta, const int32_t world,
                                    SpecialIn* __restrict__ out) {
    const int32_t r = blockIdx.y;
    int64_t nbefore = 0;
    uint64_t kbefore = 0;
    for (int q = 0; q < r; ++q) {
        nbefore += meta[2 * q];
        kbefore += (uint64_t)meta[2 * q + 1];
    }
    const int64_t cnt = meta[2 * r];
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cnt;
         k += (int64_t)gridDim.x * blockDim.x) {
        SpecialIn e = lists[r * cap + k];
        e.P += kbefore;
        out[nbefore + k] = e;
    }
}

// exact cumsum just before this shard (c_left), from the global fold
__global__ void shard_left_kernel(const SpecialOut* __restrict__ so, const int32_t* __restrict__ spec_base,
                                  const uint64_t* __restrict__ k_base, const int64_t gbase,
                                  double* __restrict__ c_left) {
    if (threadIdx.x || blockIdx.x) return;
    if (gbase == 0) {
        *c_left = -INFINITY;
        return;
    }
    const SpecialOut p = so[*spec_base - 1];
    *c_left = p.cs + (double)(*k_base - p.P) * ldexp(1.0, p.E - 52);
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

// hi_j = #positions <= c_j for every local j (the last global particle takes the rest)
__global__ __launch_bounds__(256) void shard_hi_kernel(const double* __restrict__ c, const int64_t n,
                                                       const int64_t gbase, const int64_t N,
                                                       const double step, const double* __restrict__ ofs_p,
                                                       const double np_recip, const uint64_t seed,
                                                       const int32_t* __restrict__ ctr,
                                                       int64_t* __restrict__ hi,
                                                       int32_t* __restrict__ flags) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const double ofs = resample_offset(ofs_p[ctr[0]], np_recip, seed, (uint32_t)ctr[1]);
    int64_t h = count_positions(c[j], N, step, ofs);
    if (gbase + j == N - 1) {
        if (h < N) atomicOr(&flags[kFlagStatus], 1);      // IndexError in the reference
        h = N;
    }
    hi[j] = h;
}

__device__ __forceinline__ int64_t lo_of(const int64_t* hi, const int64_t j, const int64_t lo0) {
    return j == 0 ? lo0 : hi[j - 1];
}

// per destination d: item range [start_d, end_d) of local j's overlapping [gb_d, gb_{d+1})
__global__ void shard_dest_kernel(const int64_t* __restrict__ hi, const int64_t n,
                                  const double* __restrict__ c_left, const int64_t N,
                                  const double step, const double* __restrict__ ofs_p,
                                  const double np_recip, const uint64_t seed,
                                  const int32_t* __restrict__ ctr, const int64_t* __restrict__ gb,
                                  const int32_t world, int64_t* __restrict__ se,
                                  int64_t* __restrict__ lo0_out) {
    if (threadIdx.x || blockIdx.x) return;
    const double ofs = resample_offset(ofs_p[ctr[0]], np_recip, seed, (uint32_t)ctr[1]);
    const int64_t lo0 = isinf(*c_left) ? 0 : count_positions(*c_left, N, step, ofs);
    *lo0_out = lo0;
    for (int d = 0; d < world; ++d) {
        // start: first j with hi_j > gb_d
        int64_t a = 0, b = n;
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            if (hi[m] > gb[d]) b = m;
            else a = m + 1;
        }
        const int64_t s = a;
        // end: first j with lo_j >= gb_{d+1}
        a = 0;
        b = n;
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            if (lo_of(hi, m, lo0) >= gb[d + 1]) b = m;
            else a = m + 1;
        }
        se[2 * d] = s;
        se[2 * d + 1] = a > s ? a : s;
    }
}

__global__ __launch_bounds__(256) void shard_pack_kernel(
    const double* __restrict__ xs, const double* __restrict__ ys, const double* __restrict__ ts,
    const int64_t* __restrict__ hi, const int64_t lo0, const int64_t* __restrict__ se,
    const int64_t* __restrict__ off, const int64_t* __restrict__ gb, const int32_t world,
    const int64_t total, ShardItem* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= total) return;
    int d = 0;
    while (d + 1 < world && off[d + 1] <= k) ++d;
    const int64_t j = se[2 * d] + (k - off[d]);
    ShardItem it;
    it.x = xs[j];
    it.y = ys[j];
    it.th = ts[j];
    const int64_t lo = lo_of(hi, j, lo0);
    it.lo = lo > gb[d] ? lo : gb[d];
    it.hi = hi[j] < gb[d + 1] ? hi[j] : gb[d + 1];
    out[k] = it;
}

// expand received items into this shard's positions
__global__ __launch_bounds__(256) void shard_unpack_kernel(const ShardItem* __restrict__ items,
                                                           const int64_t m, const int64_t n,
                                                           const int64_t gbase, double* __restrict__ xs,
                                                           double* __restrict__ ys,
                                                           double* __restrict__ ts,
                                                           double* __restrict__ w, const double np_recip,
                                                           int32_t* __restrict__ flags) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int64_t P = gbase + p;
    int64_t a = 0, b = m;                                // first item with hi > P
    while (a < b) {
        const int64_t mid = (a + b) >> 1;
        if (items[mid].hi > P) b = mid;
        else a = mid + 1;
    }
    if (a >= m || items[a].lo > P) {
        atomicOr(&flags[kFlagStatus], 4);                // exchange inconsistency
        a = (a < m) ? a : m - 1;
    }
    const ShardItem it = items[a];
    xs[p] = it.x;
    ys[p] = it.y;
    ts[p] = it.th;
    w[p] = np_recip;
}

// numpy-order fold of the gathered buffer partials (global order)
__global__ void shard_fold_sum_kernel(const double* __restrict__ parts, const int64_t nparts,
                                      double* __restrict__ s_out) {
    __shared__ double sh[1024];
    double s = 0.0;
    for (int64_t c0 = 0; c0 < nparts; c0 += 1024) {
        const int cnt = (int)((nparts - c0) < 1024 ? (nparts - c0) : 1024);
        __syncthreads();
        for (int k = threadIdx.x; k < cnt; k += blockDim.x) sh[k] = parts[c0 + k];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 0; k < cnt; ++k) s = s + sh[k];
    }
    if (threadIdx.x == 0) *s_out = s;
}

// the shard's reduction record: block partials in block order + argmax state
__global__ __launch_bounds__(kNormThreads) void shard_record_kernel(
    const BlockPartial* __restrict__ bp, const int32_t nb, const double* __restrict__ xs,
    const double* __restrict__ ys, const double* __restrict__ ts, const int64_t gbase,
    ShardRecord* __restrict__ out) {
    __shared__ BlockPartial shp[kNormThreads / 64];
    BlockPartial c;
    bp_zero(c);
    for (int k = threadIdx.x; k < nb; k += blockDim.x) bp_merge(c, bp[k]);
    const BlockPartial tot = bp_block_reduce(c, shp);
    if (threadIdx.x == 0) {
        ShardRecord r;
        r.bp = tot;
        const int64_t li = tot.maxi - gbase;
        r.x_cand[0] = xs[li];
        r.x_cand[1] = ys[li];
        r.x_cand[2] = ts[li];
        r.pad = 0.0;
        *out = r;
    }
}

// combine the gathered records in rank order -> result (identical on every rank)
__global__ void shard_finish_kernel(const ShardRecord* __restrict__ recs, const int32_t world,
                                    double* __restrict__ refp, const double* __restrict__ s_in,
                                    int32_t* __restrict__ flags, const double ess_th,
                                    slam_pf_result* __restrict__ res, const int32_t resampled) {
    if (threadIdx.x || blockIdx.x) return;
    BlockPartial r = recs[0].bp;
    int win = 0;
    for (int k = 1; k < world; ++k) {
        const BlockPartial& o = recs[k].bp;
        if (o.maxv > r.maxv || (o.maxv == r.maxv && o.maxi < r.maxi)) win = k;
        bp_merge(r, o);
    }
    slam_pf_result o;
    o.max_idx = r.maxi;
    o.max_val = r.maxv;
    for (int q = 0; q < 3; ++q) o.x_est[q] = recs[win].x_cand[q];
    const double inv = 1.0 / r.sw;
    const double mu[3] = {r.m1[0] * inv, r.m1[1] * inv, r.m1[2] * inv};
    const double m2[9] = {r.m2[0], r.m2[1], r.m2[2], r.m2[1], r.m2[3], r.m2[4], r.m2[2], r.m2[4], r.m2[5]};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) o.cov[3 * a + b] = m2[3 * a + b] * inv - mu[a] * mu[b];
    o.ess = 1.0 / r.sw2;
    o.weight_sum = *s_in;
    o.resampled = resampled;
    o.resample_next = (o.ess < ess_th) ? 1 : 0;
    o.status = flags[kFlagStatus];
    o.n_special = flags[kFlagNSpecial];
    flags[kFlagResample] = 0;
    flags[kFlagStatus] = 0;
    for (int q = 0; q < 3; ++q) refp[q] = o.x_est[q];
    *res = o;
}

}  // namespace slam
