// pf_stepend.inl -- the end of a deferred-normalisation PF step (included by
// pf_kernels.inl ahead of the fused kernel).
//
// Work (particle_filter.py:113-117, :210-237): np.sum of the unnormalised
// weights in NumPy's order (:234), the block partials rescaled to the global
// max and combined in a fixed order (ESS :210, the weighted covariance), the
// exact max / first argmax of w = w_un / s (:115-117), the result record, the
// step context, s for the next step and -- when the next step resamples -- the
// prefix of the fused-block weight totals for its exact cumsum (:212).
//
// One canonical order, two executions (bit-identical results):
//  * folded into the fused kernel (round 4; single-GPU handles with NP a
//    multiple of 8192): the 16th fused block of an np.sum buffer to finish
//    (a ticket per buffer) folds its buffer's 16 block partials into a group
//    record; the last group to finish (a second ticket) runs the step end --
//    no step-end launch and no kernel boundary;
//  * stepend_kernel, one 256-lane workgroup after the fused kernel (sync-mode
//    steps of any NP, the likelihood-only update): the same group records,
//    one wave per group, then the same step end.
// Group record of buffer g (fused blocks 16g .. 16g+15, lanes j of one wave):
// gm = max M_j; q_k = the blocks' sums scaled by r_j = M_j / gm (r_j^2 for
// sum u^2) summed as a perfect pairwise tree over the 16 lanes; buf = the
// buffer's np.sum, the same tree over the blocks' subtree sums.  Step end:
// M = max gm; lane t sums the records g = t, t + 256, ... scaled by gm / M,
// then a 64-lane butterfly per wave and ((w0 + w1) + (w2 + w3)); s = the
// buffers' sums left to right (np.sum's buffer chain).
//
// Hand-offs inside the fused launch (MI355X_MICROARCH "Valid forms", row 1):
// every byte another workgroup reads -- the block partials, the group records
// and, for the rare element passes, the particles and weights -- is stored
// write-through (sc1: agent-scope relaxed atomic stores, 16-byte buffer
// stores with cache bits sc1) and loaded with sc1 loads; every storing wave
// drains (s_waitcnt vmcnt(0)) before the workgroup barrier and one lane takes
// the ticket (arrive_last_n).

constexpr int kGroupBlocks = kSumChunk / kPartPer;   // fused blocks per np.sum buffer (16)
constexpr int kEndThreads = 256;
static_assert(kGroupBlocks == 16, "a group is one 16-lane row of a wave");

struct alignas(16) GroupRec {
    double gm;          // max unnormalised weight of the group's blocks
    double q[11];       // sw, sw2, m1[3], m2[6] scaled to gm
    double buf;         // np.sum of the buffer (full groups)
    double pad[3];
};
static_assert(sizeof(GroupRec) == 128, "one 128-byte line per group record");

__device__ void write_result_xe(const BlockPartial& r, const double* xe, double* refp,
                                const double s, int32_t* flags, const double ess_th,
                                const double ess_band, slam_pf_result* res,
                                const int32_t resampled_known);

// s + a[0] + a[1] + ... + a[cnt - 1], left to right (np.sum's buffer chain),
// with the next 16 LDS words in flight while the current 16 are added
__device__ __forceinline__ double lds_chain_sum(double s, const double* a, const int cnt) {
    constexpr int B = 16;
    int k = 0;
    if (cnt >= B) {
        double cur[B];
#pragma unroll
        for (int j = 0; j < B; ++j) cur[j] = a[j];
        for (; k + 2 * B <= cnt; k += B) {
            double nxt[B];
#pragma unroll
            for (int j = 0; j < B; ++j) nxt[j] = a[k + B + j];
#pragma unroll
            for (int j = 0; j < B; ++j) s = s + cur[j];
#pragma unroll
            for (int j = 0; j < B; ++j) cur[j] = nxt[j];
        }
#pragma unroll
        for (int j = 0; j < B; ++j) s = s + cur[j];
        k += B;
    }
    for (; k < cnt; ++k) s = s + a[k];
    return s;
}

// pairwise sum over the 16 lanes of a row (lower lane on the left): a perfect
// binary tree, np.sum's within a buffer
__device__ __forceinline__ double row16_tree(double v) {
    const int lane = (int)__lane_id();
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
        const double o = xor_f64(v, d);
        v = (lane & d) ? (o + v) : (v + o);
    }
    return v;
}

// Group records by the 16-lane rows of one wave: row r folds buffer g_r
// (g_r < 0: none); the row's first lane stores the record write-through.
__device__ void group_fold_rows(const DeferParts& dp, const int64_t g_r, const int64_t nb,
                                GroupRec* __restrict__ grec) {
    const int lane = (int)__lane_id();
    const int64_t b = g_r * kGroupBlocks + (lane & 15);
    const bool has = g_r >= 0 && b < nb;
    // every load issued first (one round trip)
    double m = 0.0, L = 0.0, q[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) q[k] = 0.0;
    if (has) {
        m = ld_wt_d(dp.pmax + b);
        L = ld_wt_d(dp.leaf + b);
#pragma unroll
        for (int k = 0; k < 11; ++k) q[k] = ld_wt_d(dp.ps[k] + b);
    }
    double gm = m;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) gm = fmax(gm, xor_f64(gm, d));
    const double r = (m > 0.0 && gm > 0.0) ? m / gm : 0.0;
    double v[11];
    v[0] = row16_tree(r * q[0]);
    v[1] = row16_tree((r * r) * q[1]);
#pragma unroll
    for (int k = 2; k < 11; ++k) v[k] = row16_tree(r * q[k]);
    const double buf = row16_tree(L);
    if ((lane & 15) == 0 && g_r >= 0) {
        GroupRec* out = grec + g_r;
        st_wt_d(&out->gm, gm);
#pragma unroll
        for (int k = 0; k < 11; ++k) st_wt_d(&out->q[k], v[k]);
        st_wt_d(&out->buf, buf);
    }
}

// The step end proper, by one 256-lane workgroup once every group record of
// the step is published.  xs/ys/ts/w_un: this step's particles and weights
// (read only by the rare element passes, sc1 loads).  nfull: buffers whose
// np.sum is their record's buf; tail_sum: np.sum of a last partial buffer.
__device__ void step_end_final(const DeferParts& dp, const int64_t G, const int64_t nfull,
                               const double tail_sum, const int64_t nb, const int64_t n,
                               const double* w_un, const double* xs, const double* ys,
                               const double* ts, double* s_out, double* refp, int32_t* flags,
                               const StepIO& io, const double np_recip) {
    __shared__ double e_buf[kEndThreads];
    __shared__ double e_red[11][kEndThreads / 64];
    __shared__ double e_m[kEndThreads / 64];
    __shared__ double e_s, e_xe[3];
    __shared__ unsigned long long e_min;
    __shared__ int64_t e_mi;
    __shared__ int e_flag, e_resample;
    __shared__ BlockPartial e_shp[kEndThreads / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const GroupRec* __restrict__ rec = dp.grec;
    if (t == 0) {
        e_min = ~0ull;
        e_flag = 0;
    }
    // ---- M = max gm
    double ml = -1.0;
    for (int64_t g = t; g < G; g += kEndThreads) ml = fmax(ml, ld_wt_d(&rec[g].gm));
    ml = wave_max_f64(ml);
    if (lane == 0) e_m[wave] = ml;
    __syncthreads();
    const double M = fmax(fmax(e_m[0], e_m[1]), fmax(e_m[2], e_m[3]));
    // ---- the scaled sums (lane t: records t, t + 256, ...) and np.sum's
    //      buffer chain (lane 0, 256 buffers per round through LDS)
    double acc[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) acc[k] = 0.0;
    double s = 0.0;
    for (int64_t g0 = 0; g0 < G; g0 += kEndThreads) {
        const int64_t g = g0 + t;
        if (g < G) {
            const double gm = ld_wt_d(&rec[g].gm);
            double q[11];
#pragma unroll
            for (int k = 0; k < 11; ++k) q[k] = ld_wt_d(&rec[g].q[k]);
            const double bf = ld_wt_d(&rec[g].buf);
            const double r = (gm > 0.0 && M > 0.0) ? gm / M : 0.0;
            acc[0] += r * q[0];
            acc[1] += (r * r) * q[1];
#pragma unroll
            for (int k = 2; k < 11; ++k) acc[k] += r * q[k];
            e_buf[t] = bf;
        }
        __syncthreads();
        if (t == 0) {
            const int64_t cnt = (nfull - g0 < kEndThreads) ? nfull - g0 : kEndThreads;
            if (cnt > 0) s = lds_chain_sum(s, e_buf, (int)cnt);
        }
        __syncthreads();
    }
    if (t == 0) {
        if (nfull < G) s = s + tail_sum;
        e_s = s;
    }
#pragma unroll
    for (int k = 0; k < 11; ++k) {
        double v = acc[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double o = xor_f64(v, d);
            v = (lane & d) ? (o + v) : (v + o);
        }
        if (lane == 0) e_red[k][wave] = v;
    }
    __syncthreads();
    s = e_s;
    const bool ok = (s > 0.0) && !isinf(s) && (M > 0.0);
    BlockPartial tot;
    bp_zero(tot);
    if (ok) {
        // ---- argmax: the first group whose fl(gm / s) == fl(M / s) holds the
        // first block whose fl(M_b / s) does (fl(./s) is monotone), and that
        // block's first maximum is the answer unless a smaller weight before
        // it rounds to the same value (its ppre), checked element by element
        const double mval = M / s;
        unsigned long long cg = ~0ull;
        for (int64_t g = t; g < G; g += kEndThreads) {
            const double gm = ld_wt_d(&rec[g].gm);
            if (gm >= M * (1.0 - 0x1p-48) && gm / s == mval) {
                cg = (unsigned long long)g;
                break;
            }
        }
        if (cg != ~0ull) atomicMin(&e_min, cg);
        __syncthreads();
        if (wave == 0) {
            const int64_t g = (int64_t)e_min;
            const int64_t b = g * kGroupBlocks + (lane & 15);
            const bool hit = lane < 16 && b < nb && ld_wt_d(dp.pmax + b) / s == mval;
            const uint64_t bal = __ballot(hit);
            const int64_t bc = g * kGroupBlocks + (__ffsll((unsigned long long)bal) - 1);
            if (lane == 0) {
                e_mi = (int64_t)ld_wt(dp.pidx + bc);
                for (int j = 0; j < 3; ++j) e_xe[j] = ld_wt_d(dp.pxe[j] + bc);
                const double pre = ld_wt_d(dp.ppre + bc);
                e_flag = (pre / s == mval) ? 1 : 0;
                e_min = (unsigned long long)bc;
            }
        }
        __syncthreads();
        if (e_flag) {
            const int64_t bc = (int64_t)e_min;
            __syncthreads();
            if (t == 0) e_min = ~0ull;
            __syncthreads();
            for (int e = t; e < kPartPer; e += kEndThreads) {
                const int64_t i = bc * kPartPer + e;
                if (i < n && norm_w(ld_wt_d(w_un + i), s, np_recip) == mval)
                    atomicMin(&e_min, (unsigned long long)i);
            }
            __syncthreads();
            if (t == 0) {
                const int64_t i = (int64_t)e_min;
                e_mi = i;
                e_xe[0] = ld_wt_d(xs + i);
                e_xe[1] = ld_wt_d(ys + i);
                e_xe[2] = ld_wt_d(ts + i);
            }
        }
        if (t == 0) {
            const double f = M / s;                  // from max-relative to w_un / s
            double red[11];
            for (int k = 0; k < 11; ++k)
                red[k] = (e_red[k][0] + e_red[k][1]) + (e_red[k][2] + e_red[k][3]);
            tot.maxv = mval;
            tot.maxi = e_mi;
            tot.sw = red[0] * f;
            tot.sw2 = red[1] * (f * f);
            for (int j = 0; j < 3; ++j) tot.m1[j] = red[2 + j] * f;
            for (int j = 0; j < 6; ++j) tot.m2[j] = red[5 + j] * f;
        }
    } else {
        // ---- every weight through the reference's division (s not positive
        // and finite: all weights NaN -> 1/NP, :236; slow, degenerate case)
        BlockPartial a;
        bp_zero(a);
        const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
        for (int64_t i = t; i < n; i += kEndThreads) {
            const double v = norm_w(ld_wt_d(w_un + i), s, np_recip);
            const double x = ld_wt_d(xs + i), y = ld_wt_d(ys + i), th = ld_wt_d(ts + i);
            BlockPartial o;
            o.maxv = v;
            o.maxi = i;
            o.sw = v;
            o.sw2 = v * v;
            const double d0 = x - r0, d1 = y - r1, d2 = th - r2;
            const double v0 = v * d0, v1 = v * d1, v2 = v * d2;
            o.m1[0] = v0; o.m1[1] = v1; o.m1[2] = v2;
            o.m2[0] = v0 * d0; o.m2[1] = v0 * d1; o.m2[2] = v0 * d2;
            o.m2[3] = v1 * d1; o.m2[4] = v1 * d2; o.m2[5] = v2 * d2;
            bp_merge(a, o);
        }
        tot = bp_block_reduce(a, e_shp);
        if (t == 0) {
            e_xe[0] = ld_wt_d(xs + tot.maxi);
            e_xe[1] = ld_wt_d(ys + tot.maxi);
            e_xe[2] = ld_wt_d(ts + tot.maxi);
        }
    }
    if (t == 0) {
        const int32_t st = io.ctr[0];
        write_result_xe(tot, e_xe, refp, s, flags, dp.ess_th, io.ess_band, io.res + st,
                        dp.resampled_known);
        e_resample = flags[kFlagResample];
        io.ctr[0] = st + 1;
        io.ctr[1] = io.ctr[1] + 1;
        *s_out = s;
    }
    __syncthreads();
    if (e_resample) {
        // fused-block totals of w for the next step's exact cumsum (S1): lane t
        // owns the contiguous blocks [t per, (t + 1) per)
        auto btot = [&](int64_t b) {
            if (ok) return (ld_wt_d(dp.pmax + b) / s) * ld_wt_d(dp.ps[0] + b);
            double v = 0.0;
            const int64_t e = (b + 1) * kPartPer < n ? (b + 1) * kPartPer : n;
            for (int64_t i = b * kPartPer; i < e; ++i) v += norm_w(ld_wt_d(w_un + i), s, np_recip);
            return v;
        };
        const int per = (int)((nb + kEndThreads - 1) / kEndThreads);
        const int64_t b0 = (int64_t)t * per;
        double loc = 0.0;
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) loc += btot(b0 + k);
        double total;
        double ex = block_excl_scan<double, kEndThreads>(loc, e_buf, total);
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) {
                dp.boff[b0 + k] = ex;
                ex = ex + btot(b0 + k);
            }
        if (t == 0) dp.boff[nb] = total;
    }
}
