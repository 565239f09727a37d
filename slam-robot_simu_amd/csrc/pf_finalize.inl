// pf_finalize.inl -- end of a deferred-normalisation PF step (included by
// pf_kernels.inl).  One workgroup of 512 lanes (8 waves, two per SIMD: the
// serial parts of the step end -- np.sum's left-to-right buffer chain, the
// result record -- run on a wave that shares its SIMD with one other wave
// only).
//
// Work: np.sum of the unnormalised weights from the fused blocks' leaf sums
// (particle_filter.py:234), the block partials rescaled to the global max and
// combined in a fixed order (ESS :210 and the weighted covariance), the exact
// max / first argmax of w = w_un / s (:115-117), the result record, the step
// context, s for the next step, and -- when the next step resamples -- the
// prefix of the fused-block weight totals for its exact cumsum (:212).
//
// Latency plan: every lane issues the loads of its four fused blocks and its
// sixteen leaves first (NP <= 2^20: one memory round trip); the argmax
// records of the few candidate blocks are fetched while lane 0 runs the
// serial buffer chain.  Argmax: fl(w_un / s) is monotone in w_un, so the
// first block b with fl(M_b / s) == fl(M / s) holds it; inside b the first
// index of M_b is the answer unless a smaller weight before it rounds to the
// same value (fl(pre_b / s) == fl(M / s)), which is then checked element by
// element.  A non-positive or non-finite s (all weights NaN -> 1/NP, :236)
// takes a slow whole-array pass.

#ifdef SLAM_FIN_PROBE
__device__ long long g_fin_probe[32];
#define FIN_STAMP(k) do { if (threadIdx.x == 0) g_fin_probe[k] = wall_clock64(); } while (0)
#define FIN_STAMP_IF(c, k) do { if (c) g_fin_probe[k] = wall_clock64(); } while (0)
#else
#define FIN_STAMP(k) do { } while (0)
#define FIN_STAMP_IF(c, k) do { } while (0)
#endif

#ifndef SLAM_FIN_THREADS
#define SLAM_FIN_THREADS 512
#endif
constexpr int kFinThreads = SLAM_FIN_THREADS;
constexpr int kFinWaves = kFinThreads / 64;
constexpr int kFinRegBlocks = 2048 / kFinThreads;   // fused blocks held in registers per lane (2048)
constexpr int kFinLeafLanes = 4;            // lanes per 8192-element buffer (16 leaves each)
constexpr int kFinBufPerRound = kFinThreads / kFinLeafLanes;   // 128 buffers per round
constexpr int kFinCand = 8;                 // argmax candidate records staged in LDS
constexpr int kFinBatch = 8;                // loads in flight per lane beyond the registers (NP > 2^20)
constexpr int kFinSumBatch = 2;             // blocks (12 loads each) in flight in the sums pass
constexpr int kFinPrefixRounds = 32;        // the next step's block prefix in registers (NP <= 2^23)

struct FinRecord {
    double pre, xe[3];
    int64_t pi;
};

__device__ __forceinline__ void fin_load_record(const DeferParts& dp, const int64_t b, FinRecord& f) {
    f.pre = dp.ppre[b];
    f.pi = dp.pidx[b];
#pragma unroll
    for (int j = 0; j < 3; ++j) f.xe[j] = dp.pxe[j][b];
}

// A lane of the np.sum pass takes 4 consecutive fused blocks of a buffer: each
// block left the pairwise sum of its four 128-element leaves (a perfect
// subtree of the buffer's tree), so (b0 + b1) + (b2 + b3) is the lane's
// 16-leaf subtree.
static_assert(kSumChunk == 16 * kPartPer, "a buffer is 16 fused blocks, 4 per np.sum lane");

// s + a[0] + a[1] + ... + a[cnt - 1], left to right (np.sum's buffer chain),
// with the next 16 LDS words in flight while the current 16 are added
__device__ __forceinline__ double lds_chain_sum(double s, const double* a, const int cnt) {
    constexpr int B = 16;
    int k = 0;
    if (cnt >= 2 * B) {
        // two register batches alternating (no copy between them): batch A
        // holds [k, k + B), B the next B; each is refilled while the other
        // is added
        double ra[B], rb[B];
#pragma unroll
        for (int j = 0; j < B; ++j) ra[j] = a[j];
        for (; k + 2 * B <= cnt; k += 2 * B) {
#pragma unroll
            for (int j = 0; j < B; ++j) rb[j] = a[k + B + j];
            __asm__ volatile("" ::: "memory");          // (the reads before the adds)
            __asm__ volatile("" : "+v"(s));
#pragma unroll
            for (int j = 0; j < B; ++j) s = s + ra[j];
            const int nk = (k + 3 * B <= cnt) ? k + 2 * B : k;   // past the end: a harmless re-read
#pragma unroll
            for (int j = 0; j < B; ++j) ra[j] = a[nk + j];
            __asm__ volatile("" ::: "memory");
            __asm__ volatile("" : "+v"(s));
#pragma unroll
            for (int j = 0; j < B; ++j) s = s + rb[j];
        }
    }
    for (; k < cnt; ++k) s = s + a[k];
    return s;
}

// register block k of lane t (k < kFinRegBlocks): neighbour pairs, increasing in k
__device__ __forceinline__ int64_t fin_blk(const int t, const int k) {
    static_assert(kFinRegBlocks % 2 == 0, "pairs of blocks");
    return 2 * (int64_t)t + (k & 1) + 2 * (int64_t)kFinThreads * (k >> 1);
}

// NP > 2^20 (round 5): slices of 2048 fused blocks beyond the first, one
// workgroup each, laid out like the finalize's register blocks: the slice's
// max M_g, its 11 partial sums scaled to M_g (lane sums over the lane's four
// blocks, rescaled to M_g, then the finalize's transposed reduction), and the
// np.sum value of each of its 128 buffers (pairwise over the buffer's 16
// block subtrees).  The finalize then rescales the slices to the global max
// and continues np.sum's left-to-right chain over the buffer values, instead
// of pulling every block through one CU (a 2^23-particle finalize: 1.7 MB).
// slice g's buffers are g * kFinBufPerRound ...: a slice of 2048 fused blocks
// must be exactly one round of buffers (16 blocks each), i.e. 512 lanes
static_assert(kFinThreads * kFinRegBlocks == 16 * kFinBufPerRound,
              "a finalize slice (2048 fused blocks) must span kFinBufPerRound buffers");
constexpr int kSliceCand = 4;               // argmax candidate blocks a slice lists
struct FinSlices {
    double* m;          // [nsl] slice max (slice 0: the finalize's own)
    double* q;          // [nsl][11] slice sums scaled to the slice max
    double* buf;        // [nfull] np.sum value of each full 8192-element buffer
    int64_t* cblk;      // [nsl][kSliceCand] blocks with M_b within 2^-48 of the slice max
    double* cpm;        // [nsl][kSliceCand] their maxima
    int32_t* ncand;     // [nsl] how many there were (> kSliceCand: the slice is scanned)
    double* pre;        // [nb] the next step's block prefix inside each slice, w_un units
    double* u;          // [nsl] the slice's total of w_un (pre's units)
    int32_t nsl;        // slices of 2048 fused blocks; <= 1: no pre-pass
};

__global__ __launch_bounds__(kFinThreads) void finalize_slices_kernel(const int64_t n,
                                                                      const DeferParts dp,
                                                                      const FinSlices sl) {
    __shared__ double s_q[11][kFinThreads];
    __shared__ double s_wmax[kFinWaves];
    __shared__ int s_nc;
    __shared__ int64_t s_cb[kSliceCand];
    __shared__ double s_cp[kSliceCand];
    __shared__ double s_pw[2][kFinWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = 1 + (int)blockIdx.x;
    if (tid == 0) s_nc = 0;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t b_base = (int64_t)g * kFinThreads * kFinRegBlocks;
    double pm[kFinRegBlocks], q[kFinRegBlocks][11];
    bool has[kFinRegBlocks];
#pragma unroll
    for (int kp = 0; kp < kFinRegBlocks / 2; ++kp) {
        const int64_t b = b_base + fin_blk(tid, 2 * kp);
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
    // the slice's buffers: 4 lanes per buffer, pairwise
    {
        const int part = tid & (kFinLeafLanes - 1);
        const int64_t c = (int64_t)g * kFinBufPerRound + tid / kFinLeafLanes;
        double v = 0.0;
        if (c < nfull) {
            const double* Lp = dp.leaf + 16 * c + 4 * part;
            v = (Lp[0] + Lp[1]) + (Lp[2] + Lp[3]);
        }
        {
            const double o = dpp_f64<kDppXor1>(v);
            v = (part & 1) ? (o + v) : (v + o);
        }
        {
            const double o = dpp_f64<kDppXor2>(v);
            v = (part & 2) ? (o + v) : (v + o);
        }
        if (part == 0 && c < nfull) sl.buf[c] = v;
    }
    double mlane = -1.0;
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k)
        if (has[k]) mlane = fmax(mlane, pm[k]);
    double acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = 0.0;
    if (mlane > 0.0) {
        const double rm = 1.0 / mlane;
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k) {
            if (has[k]) {
                const double r = pm[k] * rm;
                acc[0] += r * q[k][0];
                acc[1] += (r * r) * q[k][1];
#pragma unroll
                for (int j = 2; j < 11; ++j) acc[j] += r * q[k][j];
            }
        }
    }
    const double mx = wave_max_f64(mlane);
    if (lane == 0) s_wmax[wave] = mx;
    __syncthreads();
    double M = s_wmax[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) M = fmax(M, s_wmax[w]);
    {
        const double rl = (mlane > 0.0 && M > 0.0) ? mlane / M : 0.0;
        acc[0] *= rl;
        acc[1] *= rl * rl;
#pragma unroll
        for (int j = 2; j < 11; ++j) acc[j] *= rl;
#pragma unroll
        for (int j = 0; j < 11; ++j) s_q[j][tid] = acc[j];
    }
    // the slice's argmax candidates (a global candidate in this slice is one:
    // the global max is >= M); the finalize checks them instead of the slice
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k) {
        if (has[k] && pm[k] >= M * (1.0 - 0x1p-48)) {
            const int slot = atomicAdd(&s_nc, 1);
            if (slot < kSliceCand) {
                s_cb[slot] = b_base + fin_blk(tid, k);
                s_cp[slot] = pm[k];
            }
        }
    }
    // the next step's block prefix (S1) inside the slice in w_un units (M_b
    // times the block's sum of w_un / M_b): the finalize scales it by 1 / s
    // and offsets it by the slices before, when the next step resamples
    double u0[2], u1[2], pex[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        u0[hf] = has[2 * hf] ? pm[2 * hf] * q[2 * hf][0] : 0.0;
        u1[hf] = has[2 * hf + 1] ? pm[2 * hf + 1] * q[2 * hf + 1][0] : 0.0;
        double wt;
        pex[hf] = wave_excl_scan_rows(u0[hf] + u1[hf], wt);
        if (lane == 63) s_pw[hf][wave] = wt;
    }
    __syncthreads();
    {
        double tot[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            double base = 0.0, all = 0.0;
#pragma unroll
            for (int w = 0; w < kFinWaves; ++w) {
                if (w < wave) base = base + s_pw[hf][w];
                all = all + s_pw[hf][w];
            }
            pex[hf] = base + pex[hf];
            tot[hf] = all;
        }
        pex[1] = tot[0] + pex[1];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int64_t b = b_base + fin_blk(tid, 2 * hf);
            if (b + 1 < nb) *reinterpret_cast<double2*>(sl.pre + b) = double2{pex[hf], pex[hf] + u0[hf]};
            else if (b < nb) sl.pre[b] = pex[hf];
        }
        if (tid == 0) sl.u[g] = tot[0] + tot[1];
    }
    for (int j = wave; j < 11; j += kFinWaves) {
        double r = s_q[j][lane];
#pragma unroll
        for (int m = 1; m < kFinThreads / 64; ++m) r = r + s_q[j][lane + 64 * m];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double o = xor_f64(r, d);
            r = (lane & d) ? (o + r) : (r + o);
        }
        if (lane == 0) sl.q[(int64_t)g * 11 + j] = r;
    }
    if (tid < kSliceCand) {
        const bool in = tid < s_nc;
        sl.cblk[g * kSliceCand + tid] = in ? s_cb[tid] : -1;
        sl.cpm[g * kSliceCand + tid] = in ? s_cp[tid] : -1.0;
    }
    if (tid == 0) {
        sl.m[g] = M;
        sl.ncand[g] = s_nc;
    }
}

// The next step's fused-block totals of w = w_un / s for its exact cumsum
// (S1): boff[b] = the exclusive prefix, boff[nb] = the total.  Called by the
// whole workgroup when the step just finalised resamples next.  pm / q0 /
// has: the lane's register blocks fin_blk(tid, k) (block max, sum of w_un /
// M_b); sh: 2048 doubles of LDS; scr: kFinThreads doubles of LDS.
__device__ void fin_next_prefix(const int64_t n, const int64_t nb, const bool ok, const double s,
                                const double np_recip, const double (&pm)[kFinRegBlocks],
                                const double (&q0)[kFinRegBlocks], const bool (&has)[kFinRegBlocks],
                                const double* __restrict__ w_un, const DeferParts& dp,
                                double* __restrict__ boff, double* sh, double* scr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (ok && nb <= (int64_t)kFinThreads * kFinRegBlocks) {
        // fused-block totals of w for the next step's exact cumsum (S1) from the
        // registers (round 6): lane t holds blocks 2t, 2t + 1 of each half of
        // 2 kFinThreads blocks; both halves' pair sums scanned over the lanes at
        // once (wave scans, one barrier).  An approximate prefix: the exact
        // cumsum classifies against it with a margin, any fixed
        // order serves.
        static_assert(kFinRegBlocks == 4, "two halves of lane pairs");
        double t0[2], t1[2], p[2], tot[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            t0[hf] = has[2 * hf] ? (pm[2 * hf] / s) * q0[2 * hf] : 0.0;
            t1[hf] = has[2 * hf + 1] ? (pm[2 * hf + 1] / s) * q0[2 * hf + 1] : 0.0;
            p[hf] = t0[hf] + t1[hf];
        }
        double wt[2], ex[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            ex[hf] = wave_excl_scan_rows(p[hf], wt[hf]);
            if (lane == 63) scr[hf * kFinWaves + wave] = wt[hf];
        }
        __syncthreads();
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            double base = 0.0, all = 0.0;
#pragma unroll
            for (int w = 0; w < kFinWaves; ++w) {
                if (w < wave) base = base + scr[hf * kFinWaves + w];
                all = all + scr[hf * kFinWaves + w];
            }
            ex[hf] = base + ex[hf];
            tot[hf] = all;
        }
        ex[1] = tot[0] + ex[1];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int64_t b = fin_blk(tid, 2 * hf);
            if (b + 1 < nb) {
                *reinterpret_cast<double2*>(boff + b) = double2{ex[hf], ex[hf] + t0[hf]};
            } else if (b < nb) {
                boff[b] = ex[hf];
            }
        }
        if (tid == 0) boff[nb] = tot[0] + tot[1];
    } else if (ok && (nb + kFinWaves * 64 - 1) / (kFinWaves * 64) <= kFinPrefixRounds) {
        // NP <= 2^23 (round 6: the batched form below took 39 us at 2^23): wave
        // w takes the contiguous blocks [w R 64, (w+1) R 64) in R rounds of 64
        // (lane l: block w R 64 + 64 r + l, coalesced), every load issued
        // first; inclusive wave scans carry the running total over the rounds,
        // then the waves' totals in order
        const int R = (int)((nb + kFinWaves * 64 - 1) / (kFinWaves * 64));
        const int64_t wb0 = (int64_t)wave * R * 64;
        double pv[kFinPrefixRounds], qv[kFinPrefixRounds];
#pragma unroll
        for (int r = 0; r < kFinPrefixRounds; ++r) {
            if (r < R) {
                const int64_t b = wb0 + 64 * r + lane;
                const int64_t bb = b < nb ? b : 0;
                pv[r] = dp.pmax[bb];
                qv[r] = dp.ps[0][bb];
            }
        }
        // the rounds' scans are independent (interleaved by the scheduler); the
        // running total over the rounds is added after
        double ex[kFinPrefixRounds], rt[kFinPrefixRounds];
#pragma unroll
        for (int r = 0; r < kFinPrefixRounds; ++r) {
            if (r < R) {
                const int64_t b = wb0 + 64 * r + lane;
                const double t = b < nb ? (pv[r] / s) * qv[r] : 0.0;
                ex[r] = wave_excl_scan_rows(t, rt[r]);
            }
        }
        double run = 0.0;
#pragma unroll
        for (int r = 0; r < kFinPrefixRounds; ++r) {
            if (r < R) {
                ex[r] = run + ex[r];
                run = run + rt[r];
            }
        }
        if (lane == 0) scr[wave] = run;
        __syncthreads();
        double base = 0.0, all = 0.0;
#pragma unroll
        for (int w = 0; w < kFinWaves; ++w) {
            if (w < wave) base = base + scr[w];
            all = all + scr[w];
        }
#pragma unroll
        for (int r = 0; r < kFinPrefixRounds; ++r) {
            if (r < R) {
                const int64_t b = wb0 + 64 * r + lane;
                if (b < nb) boff[b] = base + ex[r];
            }
        }
        if (tid == 0) boff[nb] = all;
    } else {
        // fused-block totals of w for the next step's exact cumsum (S1), moved
        // through LDS so that lane t owns the contiguous blocks [t per, (t+1) per)
        auto btot_slow = [&](int64_t b) {
            double v = 0.0;
            const int64_t e = (b + 1) * kPartPer < n ? (b + 1) * kPartPer : n;
            for (int64_t i = b * kPartPer; i < e; ++i) v += norm_w(w_un[i], s, np_recip);
            return v;
        };
        const bool in_lds = ok && nb <= 2048;
        if (in_lds) {
#pragma unroll
            for (int k = 0; k < kFinRegBlocks; ++k)
                if (has[k]) sh[fin_blk(tid, k)] = (pm[k] / s) * q0[k];
        }
        __syncthreads();
        auto btot = [&](int64_t b) {
            if (in_lds) return sh[b];
            if (ok) return (dp.pmax[b] / s) * dp.ps[0][b];
            return btot_slow(b);
        };
        const int per = (int)((nb + kFinThreads - 1) / kFinThreads);
        const int64_t b0 = (int64_t)tid * per;
        // batches of kFinBatch totals (their loads together), then the adds in order
        auto btot_batch = [&](const int k0, double (&t)[kFinBatch]) {
#pragma unroll
            for (int u = 0; u < kFinBatch; ++u) {
                const int64_t b = b0 + k0 + u;
                t[u] = (k0 + u < per && b < nb) ? btot(b) : 0.0;
            }
        };
        double loc = 0.0;
        for (int k0 = 0; k0 < per; k0 += kFinBatch) {
            double t[kFinBatch];
            btot_batch(k0, t);
#pragma unroll
            for (int u = 0; u < kFinBatch; ++u)
                if (k0 + u < per && b0 + k0 + u < nb) loc += t[u];
        }
        double total;
        double ex = block_excl_scan<double, kFinThreads>(loc, scr, total);
        for (int k0 = 0; k0 < per; k0 += kFinBatch) {
            double t[kFinBatch];
            btot_batch(k0, t);
#pragma unroll
            for (int u = 0; u < kFinBatch; ++u)
                if (k0 + u < per && b0 + k0 + u < nb) {
                    boff[b0 + k0 + u] = ex;
                    ex = ex + t[u];
                }
        }
        if (tid == 0) boff[nb] = total;
    }
}

__global__ __launch_bounds__(kFinThreads) void finalize_deferred_kernel(
    const int64_t n, const DeferParts dp, const double* __restrict__ w_un,
    double* __restrict__ s_cur, const int32_t* __restrict__ tail_leaves,
    const int32_t* __restrict__ tail_ops, const int32_t n_tail_leaves, const int32_t n_tail_ops,
    const double* __restrict__ xs, const double* __restrict__ ys, const double* __restrict__ ts,
    double* __restrict__ refp, int32_t* __restrict__ flags, const double ess_th, StepIO io,
    const int32_t resampled_known, const double np_recip, double* __restrict__ boff,
    const FinSlices sl) {
    __shared__ double sh[2048];                      // buffer sums / tail leaves / block totals
    __shared__ double s_q[11][kFinThreads];
    __shared__ BlockPartial shp[kFinWaves];
    __shared__ double s_wmax[kFinWaves];
    __shared__ double s_tot[11];
    __shared__ double s_s;
    __shared__ unsigned long long s_min;
    __shared__ int32_t s_flag;
    __shared__ int64_t s_mi;
    __shared__ double s_xe[3];
    __shared__ int s_ncand;
    __shared__ int64_t s_cblk[kFinCand];
    __shared__ FinRecord s_crec[kFinCand];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
    FIN_STAMP(0);
    // the step, and the batch's bounds (the last step exports the batch's records)
    const int32_t st_now = io.ctr[0], b_first = io.ctr[2], b_last = io.ctr[3];
    const bool exp = io.res_host != nullptr && st_now == b_last && b_first <= b_last;
    if (tid == 0) {
        s_ncand = 0;
        s_min = ~0ull;
        s_flag = 0;
    }
    // ---- loads, issued up front: this lane's blocks fin_blk(tid, k) (pairs of
    // neighbours, one 16-byte load per array: the partial arrays hold nb + 1
    // entries) and its leaves
    double pm[kFinRegBlocks], q[kFinRegBlocks][11];
    bool has[kFinRegBlocks];
#pragma unroll
    for (int kp = 0; kp < kFinRegBlocks / 2; ++kp) {
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
    // ---- lane partial sums scaled to the lane's max (rescaled to the global
    // max once that is known); q dies here except the totals q[k][0]
    double mlane = -1.0;
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k)
        if (has[k]) mlane = fmax(mlane, pm[k]);
    // NP > 2^20: blocks beyond the registers (two passes: max, then sums)
    // (round 5: every loop over the blocks beyond the registers issues a batch
    // of loads before it uses them -- one memory round trip per iteration made
    // the 2^23-particle finalize 50-110 us; the adds keep their order)
    const int64_t bx0 = tid + (int64_t)kFinThreads * kFinRegBlocks;
    const bool sliced = sl.nsl > 1;                  // blocks beyond the registers pre-reduced
    const int64_t bxs = sliced ? nb : bx0;           // (the loops below then do nothing)
    for (int64_t b0 = bxs; b0 < nb; b0 += kFinBatch * (int64_t)kFinThreads) {
        double v[kFinBatch];
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u) {
            const int64_t b = b0 + (int64_t)u * kFinThreads;
            v[u] = (b < nb) ? dp.pmax[b] : -1.0;
        }
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u) mlane = fmax(mlane, v[u]);
    }
    double acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = 0.0;
    if (mlane > 0.0) {
        const double rm = 1.0 / mlane;
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k) {
            if (has[k]) {
                const double r = pm[k] * rm;
                acc[0] += r * q[k][0];
                acc[1] += (r * r) * q[k][1];
#pragma unroll
                for (int j = 2; j < 11; ++j) acc[j] += r * q[k][j];
            }
        }
        for (int64_t b0 = bxs; b0 < nb; b0 += kFinSumBatch * (int64_t)kFinThreads) {
            double pv[kFinSumBatch], qv[kFinSumBatch][11];
#pragma unroll
            for (int u = 0; u < kFinSumBatch; ++u) {
                const int64_t b = b0 + (int64_t)u * kFinThreads;
                const int64_t bb = (b < nb) ? b : b0;
                pv[u] = dp.pmax[bb];
#pragma unroll
                for (int j = 0; j < 11; ++j) qv[u][j] = dp.ps[j][bb];
            }
#pragma unroll
            for (int u = 0; u < kFinSumBatch; ++u) {
                if (b0 + (int64_t)u * kFinThreads < nb) {
                    const double r = pv[u] * rm;
                    acc[0] += r * qv[u][0];
                    acc[1] += (r * r) * qv[u][1];
#pragma unroll
                    for (int j = 2; j < 11; ++j) acc[j] += r * qv[u][j];
                }
            }
        }
    }
    const double mx = wave_max_f64(mlane);
    if (lane == 0) s_wmax[wave] = mx;
    // ---- np.sum: 8192-element buffers, 128 per round, pairwise inside
    // (sliced: only the first slice's round here, the slices' buffer values after)
    double s = 0.0;
    const int64_t nleaf = sliced ? (nfull < kFinBufPerRound ? nfull : kFinBufPerRound) : nfull;
    for (int64_t c0 = 0; c0 < nleaf; c0 += kFinBufPerRound) {
        const int64_t cnt = (nfull - c0 < kFinBufPerRound) ? nfull - c0 : kFinBufPerRound;
        const int64_t c = c0 + tid / kFinLeafLanes;
        double v = 0.0;
        if (tid / kFinLeafLanes < cnt) {
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
            v = (part & 1) ? (o + v) : (v + o);          // left operand = lower lane
        }
        {
            const double o = dpp_f64<kDppXor2>(v);
            v = (part & 2) ? (o + v) : (v + o);
        }
        if (c0 > 0) __syncthreads();                     // lane 0 is done with the previous round
        if (part == 0 && tid / kFinLeafLanes < cnt) sh[tid / kFinLeafLanes] = v;
        __syncthreads();
        if (c0 + kFinBufPerRound < nfull && tid == 0) {  // not the last round: fold it now
            s = lds_chain_sum(s, sh, (int)cnt);
        }
    }
    if (nfull == 0) __syncthreads();                     // s_wmax visible
    int64_t last_cnt = nfull - ((nfull - 1) / kFinBufPerRound) * kFinBufPerRound;
    if (sliced && nfull > kFinBufPerRound) {
        // the slices' buffer values, staged 2048 at a time behind the chain so far
        for (int64_t c0 = kFinBufPerRound; c0 < nfull; c0 += 2048) {
            const int64_t cnt = (nfull - c0 < 2048) ? nfull - c0 : 2048;
            __syncthreads();                                  // lane 0 is done with sh
            for (int64_t k = tid; k < cnt; k += kFinThreads) sh[k] = sl.buf[c0 + k];
            __syncthreads();
            if (c0 + 2048 < nfull && tid == 0) s = lds_chain_sum(s, sh, (int)cnt);
            last_cnt = cnt;
        }
    }
    double M = s_wmax[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) M = fmax(M, s_wmax[w]);
    if (sliced) {                                        // the slices' maxima (every wave alike)
        double msl = -1.0;
        for (int g = 1 + lane; g < sl.nsl; g += 64) msl = fmax(msl, sl.m[g]);
        M = fmax(M, wave_max_f64(msl));
    }
    FIN_STAMP(1);
    if (tid == 0) {
        // the last round's buffers left to right (the other waves meanwhile
        // rescale their partials and fetch the argmax candidates)
        __builtin_amdgcn_s_setprio(3);
        if (nfull > 0)
            s = lds_chain_sum(s, sh, (int)last_cnt);
        __builtin_amdgcn_s_setprio(0);
    }
    {
        const double rl = (mlane > 0.0 && M > 0.0) ? mlane / M : 0.0;
        acc[0] *= rl;
        acc[1] *= rl * rl;
#pragma unroll
        for (int j = 2; j < 11; ++j) acc[j] *= rl;
#pragma unroll
        for (int j = 0; j < 11; ++j) s_q[j][tid] = acc[j];
    }
    // argmax records of the candidate blocks (fl(M_b / s) == fl(M / s) needs
    // M_b within 2 ulp of M), staged in LDS
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k) {
        if (has[k] && pm[k] >= M * (1.0 - 0x1p-48)) {
            const int slot = atomicAdd(&s_ncand, 1);
            if (slot < kFinCand) {
                const int64_t b = fin_blk(tid, k);
                FinRecord f;
                fin_load_record(dp, b, f);
                s_cblk[slot] = b;
                s_crec[slot] = f;
            }
        }
    }
    if (nch > nfull) {
        __syncthreads();                                  // sh reused by the tail
        const double tsum = tail_chunk_sum(w_un + nfull * kSumChunk, tail_leaves, tail_ops,
                                           n_tail_leaves, n_tail_ops, sh);
        if (tid == 0) s = s + tsum;
    }
    if (tid == 0) s_s = s;
    __syncthreads();
    s = s_s;
    FIN_STAMP(2);
    const bool ok = (s > 0.0) && !isinf(s) && (M > 0.0);
    BlockPartial tot;
    bp_zero(tot);
    if (ok) {
        // ---- the 11 sums: wave w reduces quantities w and w + 8 (lane-strided
        // reads, then a butterfly with the lower lane on the left)
        for (int j = wave; j < 11; j += kFinWaves) {
            double r = s_q[j][lane];
#pragma unroll
            for (int m = 1; m < kFinThreads / 64; ++m) r = r + s_q[j][lane + 64 * m];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const double o = xor_f64(r, d);
                r = (lane & d) ? (o + r) : (r + o);
            }
            if (lane == 0) s_tot[j] = r;
        }
        if (sliced) {                                    // + the slices, rescaled to M, in order
            __syncthreads();
            if (tid < 11) {
                double r = s_tot[tid];
                for (int g = 1; g < sl.nsl; ++g) {
                    const double mg = sl.m[g];
                    if (mg > 0.0) {
                        const double f = mg / M;
                        r = r + sl.q[(int64_t)g * 11 + tid] * (tid == 1 ? f * f : f);
                    }
                }
                s_tot[tid] = r;
            }
        }
        // ---- argmax: the first block whose max rounds to fl(M / s)
        const double mval = M / s;
        unsigned long long cb = ~0ull;
#pragma unroll
        for (int k = kFinRegBlocks - 1; k >= 0; --k)
            if (has[k] && pm[k] >= M * (1.0 - 0x1p-48) && pm[k] / s == mval)
                cb = (unsigned long long)fin_blk(tid, k);
        for (int64_t b0 = bx0; b0 < nb && cb == ~0ull; b0 += kFinBatch * (int64_t)kFinThreads) {
            double v[kFinBatch];
#pragma unroll
            for (int u = 0; u < kFinBatch; ++u) {
                const int64_t b = b0 + (int64_t)u * kFinThreads;
                v[u] = (b < nb) ? dp.pmax[b] : -1.0;
            }
#pragma unroll
            for (int u = 0; u < kFinBatch; ++u) {
                const int64_t b = b0 + (int64_t)u * kFinThreads;
                if (cb == ~0ull && b < nb && v[u] / s == mval) cb = (unsigned long long)b;
            }
        }
        if (cb != ~0ull) atomicMin(&s_min, cb);
        __syncthreads();
        const int64_t bc = (int64_t)s_min;
        if (tid == 0) {
            // block bc's record: staged, or loaded if bc was not a staged candidate
            int slot = -1;
            const int nc = min(s_ncand, kFinCand);
            for (int j = 0; j < nc; ++j)
                if (s_cblk[j] == bc) slot = j;
            FinRecord f;
            if (slot >= 0) f = s_crec[slot];
            else fin_load_record(dp, bc, f);
            s_mi = f.pi;
            s_xe[0] = f.xe[0];
            s_xe[1] = f.xe[1];
            s_xe[2] = f.xe[2];
            s_flag = (f.pre / s == mval) ? 1 : 0;
            if (s_flag) s_min = ~0ull;
        }
        __syncthreads();
        if (s_flag) {
            // a smaller weight ahead of the block max rounds to the same maximum:
            // the first index of the block whose w equals mval
            for (int e = tid; e < kPartPer; e += kFinThreads) {
                const int64_t i = bc * kPartPer + e;
                if (i < n && norm_w(w_un[i], s, np_recip) == mval)
                    atomicMin(&s_min, (unsigned long long)i);
            }
            __syncthreads();
            if (tid == 0) {
                const int64_t i = (int64_t)s_min;
                s_mi = i;
                s_xe[0] = xs[i];
                s_xe[1] = ys[i];
                s_xe[2] = ts[i];
            }
        }
        if (tid == 0) {
            const double f = M / s;                      // back from max-relative to w_un / s
            tot.maxv = mval;
            tot.maxi = s_mi;
            tot.sw = s_tot[0] * f;
            tot.sw2 = s_tot[1] * (f * f);
            for (int j = 0; j < 3; ++j) tot.m1[j] = s_tot[2 + j] * f;
            for (int j = 0; j < 6; ++j) tot.m2[j] = s_tot[5 + j] * f;
        }
    } else {
        // ---- every weight through the reference's division (slow, degenerate case)
        BlockPartial a;
        bp_zero(a);
        const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
        for (int64_t i = tid; i < n; i += kFinThreads) {
            const double v = norm_w(w_un[i], s, np_recip);
            BlockPartial o;
            o.maxv = v;
            o.maxi = i;
            o.sw = v;
            o.sw2 = v * v;
            const double d0 = xs[i] - r0, d1 = ys[i] - r1, d2 = ts[i] - r2;
            const double v0 = v * d0, v1 = v * d1, v2 = v * d2;
            o.m1[0] = v0; o.m1[1] = v1; o.m1[2] = v2;
            o.m2[0] = v0 * d0; o.m2[1] = v0 * d1; o.m2[2] = v0 * d2;
            o.m2[3] = v1 * d1; o.m2[4] = v1 * d2; o.m2[5] = v2 * d2;
            bp_merge(a, o);
        }
        tot = bp_block_reduce(a, shp);
        if (tid == 0) {
            s_xe[0] = xs[tot.maxi];
            s_xe[1] = ys[tot.maxi];
            s_xe[2] = ts[tot.maxi];
        }
    }
    FIN_STAMP(3);
    if (tid == 0) {
        const int32_t st = io.ctr[0];
        s_flag = write_result_xe(tot, s_xe, refp, s, flags, ess_th, io.ess_band, io.res + st,
                                 resampled_known, exp ? io.res_host + st : nullptr);
        io.ctr[0] = st + 1;
        io.ctr[1] = io.ctr[1] + 1;
        *s_cur = s;
    }
    __syncthreads();
    FIN_STAMP(4);
    if (exp && tid >= 1 && tid < 64) {
        // the batch's earlier records (stored by earlier launches) to the host
        // buffer; this step's record went there from write_result_xe
        for (int32_t k = b_first + tid - 1; k < st_now; k += 63) io.res_host[k] = io.res[k];
    }
    if (s_flag) {
        double q0[kFinRegBlocks];
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k) q0[k] = q[k][0];
        fin_next_prefix(n, nb, ok, s, np_recip, pm, q0, has, w_un, dp, boff, sh, &s_q[0][0]);
    }
    FIN_STAMP(5);
}

// ---------------------------------------------------------------------------
// NP <= 2^24 (round 6): the same work as
// finalize_deferred_kernel in an order built around its latencies (phase
// probe).  The leaves are requested first, so np.sum's buffer chain
// starts on lane 0 after one round trip and runs while the block partials are
// still arriving; each wave requests the argmax records of its own candidate
// blocks (within 2^-48 of the wave's max -- a superset of the global
// candidates) as soon as the block maxima arrive; the step context and the
// flag words the record reads are fetched with the partials.  SLICED (NP >
// 2^20, finalize_slices_kernel ran first): the slices' buffer values, maxima,
// sums and argmax candidate lists are fetched in the same first round trip,
// so the chain runs over every buffer from LDS and the argmax checks the
// listed candidates instead of walking the blocks beyond the registers.
constexpr int kFinFastSlices = 16;          // SLICED: NP <= 2^24
constexpr int kFinSlBuf = 4;                // SLICED: slice buffer values per lane (nfull <= 2048)
template <bool SLICED>
__global__ __launch_bounds__(kFinThreads) void finalize_fast_kernel(
    const int64_t n, const DeferParts dp, const double* __restrict__ w_un,
    double* __restrict__ s_cur, const int32_t* __restrict__ tail_leaves,
    const int32_t* __restrict__ tail_ops, const int32_t n_tail_leaves, const int32_t n_tail_ops,
    const double* __restrict__ xs, const double* __restrict__ ys, const double* __restrict__ ts,
    double* __restrict__ refp, int32_t* __restrict__ flags, const double ess_th, StepIO io,
    const int32_t resampled_known, const double np_recip, double* __restrict__ boff,
    const FinSlices sl) {
    static_assert(kFinThreads == 512 && kFinRegBlocks == 4, "the register layout of fin_blk");
    static_assert(kFinSlBuf * kFinThreads + kFinBufPerRound >= 2048, "every buffer of sh");
    static_assert((kFinFastSlices - 1) * 11 <= kFinThreads, "one slice sum per lane");
    __shared__ double s_slm[kFinFastSlices];
    __shared__ double s_slq[kFinFastSlices][11];
    __shared__ int32_t s_slnc[kFinFastSlices];
    __shared__ double s_slu[kFinFastSlices];
    __shared__ double sh[2048];                      // buffer values / tail leaves / block totals
    __shared__ double s_q[11][kFinThreads];
    __shared__ BlockPartial shp[kFinWaves];
    __shared__ double s_wmax[kFinWaves];
    __shared__ double s_tot[11];
    __shared__ double s_s;
    __shared__ unsigned long long s_min;
    __shared__ int32_t s_flag;
    __shared__ int64_t s_mi;
    __shared__ double s_xe[3];
    __shared__ int s_ncand;
    __shared__ int64_t s_cblk[kFinCand];
    __shared__ FinRecord s_crec[kFinCand];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
    FIN_STAMP(0);
    // the step, the batch's bounds and the flag words the record reads: lane 0,
    // first in its load queue (used at the end; the wait counts only them)
    int32_t st_now = 0, b_first = 0, b_last = -1, rstep = 0;
    FlagWords fw{};
    double rp[3] = {0.0, 0.0, 0.0};
    if (tid == 0) {
        st_now = io.ctr[0];
        rstep = io.ctr[1];
        b_first = io.ctr[2];
        b_last = io.ctr[3];
        fw = load_flag_words(flags);
        rp[0] = refp[0];
        rp[1] = refp[1];
        rp[2] = refp[2];
        s_ncand = 0;
        s_min = ~0ull;
        s_flag = 0;
    }
    // ---- loads: the leaves, then the partials of the lane's blocks
    // fin_blk(tid, k) (pairs of neighbours, one 16-byte load per array: the
    // partial arrays hold nb + 1 entries), the step context, the flag words
    // SLICED: the slices' buffer values first (the chain reads them right after
    // the first round's), then the leaves
    const int nsl = SLICED ? sl.nsl : 1;
    double bufv[kFinSlBuf] = {};
    if constexpr (SLICED) {
#pragma unroll
        for (int k = 0; k < kFinSlBuf; ++k) {
            const int64_t c = kFinBufPerRound + tid + (int64_t)kFinThreads * k;
            if (c < nfull) bufv[k] = sl.buf[c];
        }
        __asm__ volatile("" ::: "memory");
    }
    const int part = tid & (kFinLeafLanes - 1);
    double L[4];
    {
        const int64_t c = tid / kFinLeafLanes;
        const double* Lp = dp.leaf + 16 * (c < nfull ? c : 0) + 4 * part;
#pragma unroll
        for (int j = 0; j < 4; ++j) L[j] = Lp[j];
        __asm__ volatile("" ::: "memory");              // the leaves' loads issue first
    }
    double pm[kFinRegBlocks], q[kFinRegBlocks][11];
    bool has[kFinRegBlocks];
#pragma unroll
    for (int kp = 0; kp < kFinRegBlocks / 2; ++kp) {
        const int64_t b = fin_blk(tid, 2 * kp);
        has[2 * kp] = b < nb;
        has[2 * kp + 1] = b + 1 < nb;
        const int64_t bb = has[2 * kp] ? b : 0;
        const double2 t = *reinterpret_cast<const double2*>(dp.pmax + bb);
        pm[2 * kp] = t.x;
        pm[2 * kp + 1] = t.y;
    }
    __asm__ volatile("" ::: "memory");                  // then the partial sums
#pragma unroll
    for (int kp = 0; kp < kFinRegBlocks / 2; ++kp) {
        const int64_t b = fin_blk(tid, 2 * kp);
        const int64_t bb = b < nb ? b : 0;
#pragma unroll
        for (int j = 0; j < 11; ++j) {
            const double2 u = *reinterpret_cast<const double2*>(dp.ps[j] + bb);
            q[2 * kp][j] = u.x;
            q[2 * kp + 1][j] = u.y;
        }
    }
    // SLICED: the slices' maxima, candidate lists and sums
    double slm = -1.0, slq = 0.0, ccp = -1.0, slu = 0.0;
    int64_t ccb = -1;
    int32_t sncv = 0;
    if constexpr (SLICED) {
        if (tid >= 1 && tid < nsl) {
            slm = sl.m[tid];
            sncv = sl.ncand[tid];
            slu = sl.u[tid];
        }
        if (tid < (nsl - 1) * kSliceCand) {
            const int g = 1 + tid / kSliceCand;
            ccb = sl.cblk[g * kSliceCand + tid % kSliceCand];
            ccp = sl.cpm[g * kSliceCand + tid % kSliceCand];     // unlisted: -1
        }
        if (tid < (nsl - 1) * 11) slq = sl.q[11 + tid];
    }
    // every load above is issued before the first use of a leaf (the scheduler
    // would otherwise wait for the leaves between them)
    __asm__ volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) __asm__ volatile("" : "+v"(L[j]));
#pragma unroll
    for (int k = 0; k < kFinSlBuf; ++k) __asm__ volatile("" : "+v"(bufv[k]));
    // ---- np.sum's buffer values (one round of <= 128 buffers, pairwise inside)
    {
        const int64_t c = tid / kFinLeafLanes;
        double v = (c < nfull) ? (L[0] + L[1]) + (L[2] + L[3]) : 0.0;
        {
            const double o = dpp_f64<kDppXor1>(v);
            v = (part & 1) ? (o + v) : (v + o);          // left operand = lower lane
        }
        {
            const double o = dpp_f64<kDppXor2>(v);
            v = (part & 2) ? (o + v) : (v + o);
        }
        if (part == 0 && c < nfull) sh[c] = v;
    }
    if constexpr (SLICED) {
#pragma unroll
        for (int k = 0; k < kFinSlBuf; ++k) {
            const int64_t c = kFinBufPerRound + tid + (int64_t)kFinThreads * k;
            if (c < nfull) sh[c] = bufv[k];
        }
    }
    __syncthreads();                                     // sh
    FIN_STAMP(1);
    double s = 0.0;
    if (tid == 0 && nfull > 0) {
        // the buffers left to right while the other waves take their partials
        // (a whole wave walking the lanes by readlane measured slower: 14.9
        // against 8.8 us for the 1,024 buffers of 2^23)
        __builtin_amdgcn_s_setprio(3);
        s = lds_chain_sum(s, sh, (int)nfull);
        __builtin_amdgcn_s_setprio(0);
    }
    // ---- block maxima; each wave's argmax candidates (into registers: the
    // lane's first block within 2^-48 of the wave's max)
    double mlane = -1.0;
#pragma unroll
    for (int k = 0; k < kFinRegBlocks; ++k)
        if (has[k]) mlane = fmax(mlane, pm[k]);
    const double wm = wave_max_f64(SLICED ? fmax(mlane, slm) : mlane);   // + the slices' maxima
    if (lane == 0) s_wmax[wave] = wm;
    if constexpr (SLICED) {
        if (tid < nsl) {
            s_slm[tid] = slm;
            s_slnc[tid] = sncv;
            s_slu[tid] = slu;
        }
        if (tid < (nsl - 1) * 11) s_slq[1 + tid / 11][tid % 11] = slq;
    }
    double cpm = -1.0;
    int64_t cblk = -1;
#pragma unroll
    for (int k = kFinRegBlocks - 1; k >= 0; --k) {
        if (has[k] && pm[k] >= wm * (1.0 - 0x1p-48)) {
            cpm = pm[k];
            cblk = fin_blk(tid, k);
        }
    }
    FinRecord cr{};
    if (cblk >= 0) fin_load_record(dp, cblk, cr);
    __asm__ volatile("" ::: "memory");                  // requested before the sums wait
    // ---- lane partial sums scaled to the lane's max
    double acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = 0.0;
    if (mlane > 0.0) {
        const double rm = 1.0 / mlane;
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k) {
            if (has[k]) {
                const double r = pm[k] * rm;
                acc[0] += r * q[k][0];
                acc[1] += (r * r) * q[k][1];
#pragma unroll
                for (int j = 2; j < 11; ++j) acc[j] += r * q[k][j];
            }
        }
    }
    __syncthreads();                                     // s_wmax
    double M = s_wmax[0];
#pragma unroll
    for (int w = 1; w < kFinWaves; ++w) M = fmax(M, s_wmax[w]);
    {
        const double rl = (mlane > 0.0 && M > 0.0) ? mlane / M : 0.0;
        acc[0] *= rl;
        acc[1] *= rl * rl;
#pragma unroll
        for (int j = 2; j < 11; ++j) acc[j] *= rl;
#pragma unroll
        for (int j = 0; j < 11; ++j) s_q[j][tid] = acc[j];
    }
    if (cblk >= 0 && cpm >= M * (1.0 - 0x1p-48)) {
        const int slot = atomicAdd(&s_ncand, 1);
        if (slot < kFinCand) {
            s_cblk[slot] = cblk;
            s_crec[slot] = cr;
        }
    }
    // SLICED: the listed candidates of the slices, records staged the same way
    const bool slc = SLICED && ccb >= 0 && ccp >= M * (1.0 - 0x1p-48);
    if (slc) {
        FinRecord f;
        fin_load_record(dp, ccb, f);
        const int slot = atomicAdd(&s_ncand, 1);
        if (slot < kFinCand) {
            s_cblk[slot] = ccb;
            s_crec[slot] = f;
        }
    }
    if (nch > nfull) {
        __syncthreads();                                 // sh reused by the tail
        const double tsum = tail_chunk_sum(w_un + nfull * kSumChunk, tail_leaves, tail_ops,
                                           n_tail_leaves, n_tail_ops, sh);
        if (tid == 0) s = s + tsum;
    }
    if (tid == 0) s_s = s;
    __syncthreads();
    s = s_s;
    FIN_STAMP(2);
    const bool ok = (s > 0.0) && !isinf(s) && (M > 0.0);
    BlockPartial tot;
    bp_zero(tot);
    if (ok) {
        // ---- the 11 sums: wave w reduces quantities w and w + 8 (lane-strided
        // reads, then the wave's rows by DPP: a fixed order, no LDS permutes)
        for (int j = wave; j < 11; j += kFinWaves) {
            double r = s_q[j][lane];
#pragma unroll
            for (int m = 1; m < kFinThreads / 64; ++m) r = r + s_q[j][lane + 64 * m];
            r = wave_sum_rows(r);
            if (lane == 0) s_tot[j] = r;
        }
        if constexpr (SLICED) {                         // + the slices, rescaled to M, in order
            __syncthreads();
            if (tid < 11) {
                double r = s_tot[tid];
                for (int g = 1; g < nsl; ++g) {
                    const double mg = s_slm[g];
                    if (mg > 0.0) {
                        const double f = mg / M;
                        r = r + s_slq[g][tid] * (tid == 1 ? f * f : f);
                    }
                }
                s_tot[tid] = r;
            }
        }
        // ---- argmax: the first block whose max rounds to fl(M / s)
        const double mval = M / s;
        unsigned long long cb = ~0ull;
#pragma unroll
        for (int k = kFinRegBlocks - 1; k >= 0; --k)
            if (has[k] && pm[k] >= M * (1.0 - 0x1p-48) && pm[k] / s == mval)
                cb = (unsigned long long)fin_blk(tid, k);
        if constexpr (SLICED) {
            if (slc && ccp / s == mval) cb = min(cb, (unsigned long long)ccb);
            // a slice with more candidates than it listed: all of its blocks
            for (int g = 1; g < nsl; ++g) {
                if (s_slnc[g] > kSliceCand && s_slm[g] >= M * (1.0 - 0x1p-48)) {
                    double v[kFinRegBlocks];
#pragma unroll
                    for (int k = 0; k < kFinRegBlocks; ++k) {
                        const int64_t b = (int64_t)g * kFinThreads * kFinRegBlocks + fin_blk(tid, k);
                        v[k] = b < nb ? dp.pmax[b] : -1.0;
                    }
#pragma unroll
                    for (int k = kFinRegBlocks - 1; k >= 0; --k) {
                        const int64_t b = (int64_t)g * kFinThreads * kFinRegBlocks + fin_blk(tid, k);
                        if (b < nb && v[k] / s == mval) cb = min(cb, (unsigned long long)b);
                    }
                }
            }
        }
        if (cb != ~0ull) atomicMin(&s_min, cb);
        __syncthreads();
        const int64_t bc = (int64_t)s_min;
        if (tid == 0) {
            // block bc's record: staged, or loaded if it was not a staged candidate
            int slot = -1;
            const int nc = min(s_ncand, kFinCand);
            for (int j = 0; j < nc; ++j)
                if (s_cblk[j] == bc) slot = j;
            FinRecord f;
            if (slot >= 0) f = s_crec[slot];
            else fin_load_record(dp, bc, f);
            s_mi = f.pi;
            s_xe[0] = f.xe[0];
            s_xe[1] = f.xe[1];
            s_xe[2] = f.xe[2];
            s_flag = (f.pre / s == mval) ? 1 : 0;
            if (s_flag) s_min = ~0ull;
        }
        __syncthreads();
        if (s_flag) {
            // a smaller weight ahead of the block max rounds to the same maximum:
            // the first index of the block whose w equals mval
            for (int e = tid; e < kPartPer; e += kFinThreads) {
                const int64_t i = bc * kPartPer + e;
                if (i < n && norm_w(w_un[i], s, np_recip) == mval)
                    atomicMin(&s_min, (unsigned long long)i);
            }
            __syncthreads();
            if (tid == 0) {
                const int64_t i = (int64_t)s_min;
                s_mi = i;
                s_xe[0] = xs[i];
                s_xe[1] = ys[i];
                s_xe[2] = ts[i];
            }
        }
        if (tid == 0) {
            const double f = M / s;                      // back from max-relative to w_un / s
            tot.maxv = mval;
            tot.maxi = s_mi;
            tot.sw = s_tot[0] * f;
            tot.sw2 = s_tot[1] * (f * f);
            for (int j = 0; j < 3; ++j) tot.m1[j] = s_tot[2 + j] * f;
            for (int j = 0; j < 6; ++j) tot.m2[j] = s_tot[5 + j] * f;
        }
    } else {
        // ---- every weight through the reference's division (slow, degenerate case)
        BlockPartial a;
        bp_zero(a);
        const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
        for (int64_t i = tid; i < n; i += kFinThreads) {
            const double v = norm_w(w_un[i], s, np_recip);
            BlockPartial o;
            o.maxv = v;
            o.maxi = i;
            o.sw = v;
            o.sw2 = v * v;
            const double d0 = xs[i] - r0, d1 = ys[i] - r1, d2 = ts[i] - r2;
            const double v0 = v * d0, v1 = v * d1, v2 = v * d2;
            o.m1[0] = v0; o.m1[1] = v1; o.m1[2] = v2;
            o.m2[0] = v0 * d0; o.m2[1] = v0 * d1; o.m2[2] = v0 * d2;
            o.m2[3] = v1 * d1; o.m2[4] = v1 * d2; o.m2[5] = v2 * d2;
            bp_merge(a, o);
        }
        tot = bp_block_reduce(a, shp);
        if (tid == 0) {
            s_xe[0] = xs[tot.maxi];
            s_xe[1] = ys[tot.maxi];
            s_xe[2] = ts[tot.maxi];
        }
    }
    FIN_STAMP(3);
    __shared__ int32_t s_exp[3];
    if (tid == 0) {
        const bool exp = io.res_host != nullptr && st_now == b_last && b_first <= b_last;
        s_exp[0] = exp ? 1 : 0;
        s_exp[1] = b_first;
        s_exp[2] = st_now;
        s_flag = write_result_fw(tot, s_xe, refp, rp, s, flags, fw, ess_th, io.ess_band,
                                 io.res + st_now, resampled_known, exp ? io.res_host + st_now : nullptr);
        io.ctr[0] = st_now + 1;
        io.ctr[1] = rstep + 1;
        *s_cur = s;
    }
    __syncthreads();
    FIN_STAMP(4);
    if (s_exp[0] && tid >= 1 && tid < 64) {
        // the batch's earlier records (stored by earlier launches) to the host
        // buffer; this step's record went there from write_result_fw
        for (int32_t k = s_exp[1] + tid - 1; k < s_exp[2]; k += 63) io.res_host[k] = io.res[k];
    }
    if (s_flag) {
        double q0[kFinRegBlocks];
#pragma unroll
        for (int k = 0; k < kFinRegBlocks; ++k) q0[k] = q[k][0];
        if (SLICED && ok) {
            // the slices' own prefixes (finalize_slices_kernel), w_un units:
            // slice 0 from the registers the same way, then every block's
            // (U_0 + ... + U_{g-1} + pre_b) / s
            double u0[2], u1[2], pex[2], tot[2];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                u0[hf] = has[2 * hf] ? pm[2 * hf] * q0[2 * hf] : 0.0;
                u1[hf] = has[2 * hf + 1] ? pm[2 * hf + 1] * q0[2 * hf + 1] : 0.0;
                double wt;
                pex[hf] = wave_excl_scan_rows(u0[hf] + u1[hf], wt);
                if (lane == 63) s_q[hf][wave] = wt;
            }
            // slices g >= 1: block 2048 + tid + 512 i (slice 1 + i / 4, coalesced),
            // the first batch of 32 requested before the barrier
            const int nrest = (nsl - 1) * kFinRegBlocks;
            constexpr int kB = 32;
            auto pre_batch = [&](const int i0, double (&pv)[kB]) {
#pragma unroll
                for (int i = 0; i < kB; ++i) {
                    const int64_t b = (int64_t)kFinThreads * kFinRegBlocks + tid + (int64_t)kFinThreads * (i0 + i);
                    pv[i] = (i0 + i < nrest && b < nb) ? sl.pre[b] : 0.0;
                }
            };
            double pv[kB];
            pre_batch(0, pv);
            __syncthreads();
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                double base = 0.0, all = 0.0;
#pragma unroll
                for (int w = 0; w < kFinWaves; ++w) {
                    if (w < wave) base = base + s_q[hf][w];
                    all = all + s_q[hf][w];
                }
                pex[hf] = base + pex[hf];
                tot[hf] = all;
            }
            pex[1] = tot[0] + pex[1];
            const double rs = 1.0 / s;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int64_t b = fin_blk(tid, 2 * hf);
                if (b + 1 < nb)
                    *reinterpret_cast<double2*>(boff + b) = double2{pex[hf] * rs, (pex[hf] + u0[hf]) * rs};
                else if (b < nb)
                    boff[b] = pex[hf] * rs;
            }
            // U_0 + ... + U_{g-1} for every slice (every lane, in slice order)
            double ubs[kFinFastSlices];
            ubs[0] = 0.0;
            ubs[1] = tot[0] + tot[1];
#pragma unroll
            for (int g = 2; g < kFinFastSlices; ++g) ubs[g] = (g - 1 < nsl) ? ubs[g - 1] + s_slu[g - 1] : ubs[g - 1];
            double utot = ubs[1];
#pragma unroll
            for (int g = 1; g < kFinFastSlices; ++g)
                if (g < nsl) utot = utot + s_slu[g];
#pragma unroll
            for (int i0 = 0; i0 < (kFinFastSlices - 1) * kFinRegBlocks; i0 += kB) {
                if (i0 < nrest) {
                    if (i0 > 0) pre_batch(i0, pv);
#pragma unroll
                    for (int i = 0; i < kB; ++i) {
                        const int64_t b = (int64_t)kFinThreads * kFinRegBlocks + tid + (int64_t)kFinThreads * (i0 + i);
                        if (i0 + i < nrest && b < nb) boff[b] = (ubs[1 + (i0 + i) / kFinRegBlocks] + pv[i]) * rs;
                    }
                }
            }
            if (tid == 0) boff[nb] = utot * rs;
        } else {
            fin_next_prefix(n, nb, ok, s, np_recip, pm, q0, has, w_un, dp, boff, sh, &s_q[0][0]);
        }
    }
    FIN_STAMP(5);
}
