// pf_fused4.inl -- the fused step kernel in ONE round of blocks (included by
// pf_kernels.inl after pf_fused_kernel).
//
// pf_fused_kernel holds two particles per lane: 2048 blocks of 512 particles
// at 2^20, of which 1,024 fit on the chip at once (4 waves per SIMD at <= 128
// VGPRs), so the launch runs two staggered rounds whose ramp and tail cost ~8
// us of its ~30 (the same kernel at 2^23 spends 21-22.5 us per
// 2^20).  Here a lane holds FOUR consecutive particles and a block 1,024: at
// 2^20 the 1,024 blocks are all resident from the start.  The lane works its
// particles as two pairs, one after the other (a scheduling barrier between
// them keeps the second pair's work from being hoisted into the first's, so
// the register peak stays the pair kernel's); each pair is exactly the pair
// kernel's arithmetic (same RNG pair index, predict, likelihood), so the
// particles and weights are bit-identical to pf_fused_kernel's.
//
// The block partials keep the 512-particle granularity (DeferParts, one
// "tile" per half block: waves 0-1 and 2-3), summed in the pair kernel's
// order -- lane t of the pair kernel held particles 2t, 2t+1 and its even /
// odd lane pairs were added as (q(2l) + q(2l+1)); a lane here holds 4l .. 4l+3
// and adds (q01 + q23) -- so the finalize, the exact cumsum's run marks and
// carries, and the sharded record are unchanged.
//
// particle_filter.py:156-198 (predict, likelihood), :216-222 (gather),
// :226-237 (the normalisation's np.sum leaves); motion_model.py:31-62.
// (Included inside namespace slam.)

constexpr int kF4PPT = 4;                        // particles per lane
constexpr int kF4Block = 256 * kF4PPT;           // particles per block: two partial tiles
static_assert(kDeferPPT == 2 && kF4Block == 2 * kPartPer, "two pair-kernel tiles per block");

// LDS of one block: the epilogue's lane-pair sums alias the RNG tables (the
// tables are dead once every wave has passed the epilogue's first barrier)
struct F4Lds {
    union {
        RngTabsLds rng;
        double q[2][11 * 128];
    } u;
    double w[2][kPartPer];
    double seg[2][11 * 16];
    double acc[2][8 * (kPartPer / 128)];
    double mv[4], pre[4];
    int64_t mi[4];
    int32_t wmax[4];
};

// Epilogue of one block = two 512-particle tiles; the same values and the
// same summation order per tile as defer_epilogue.  Three barriers.  The
// caller has staged the lane's weights in L.w (invalid particles as 0).
__device__ __forceinline__ void defer_epilogue4(const int64_t base, const int64_t n,
                                                const double* wv, const double* xv,
                                                const double* yv, const double* tv,
                                                const double* __restrict__ refp,
                                                const DeferParts& dp, F4Lds& L, const int wave,
                                                const int32_t nb_part) {
    constexpr int kQ = 11;
    const int lane = (int)__lane_id();
    const int T = wave >> 1;                          // tile of this wave
    const int tl = ((wave & 1) << 6) | lane;          // lane within the tile
    const int64_t tbase = base + (int64_t)T * kPartPer;
    const int64_t tile = base / kPartPer + T;
    double m = -1.0;
    int64_t mi = INT64_MAX;
#pragma unroll
    for (int k = 0; k < kF4PPT; ++k) {
        const int64_t i = tbase + kF4PPT * tl + k;
        const bool ok = i < n;
        if (ok && wv[k] > m) {
            m = wv[k];
            mi = i;
        }
    }
    const double mv = wave_max_f64(m);
    if (lane == 0) L.mv[wave] = mv;
    __syncthreads();                                                    // (1)
    const double M = fmax(L.mv[2 * T], L.mv[2 * T + 1]);
    const int64_t cand = wave_min_i64((m == M) ? mi : INT64_MAX);
    if (lane == 0) L.mi[wave] = cand;
    const double rs = (M > 0.0) ? 1.0 / M : 0.0;
    const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
    double q[kQ];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        double p[kQ];
#pragma unroll
        for (int k = 2 * h; k < 2 * h + 2; ++k) {
            const bool ok = tbase + kF4PPT * tl + k < n;
            const double u = ok ? wv[k] * rs : 0.0;
            const double d0 = xv[k] - r0, d1 = yv[k] - r1, d2 = tv[k] - r2;
            const double ud0 = u * d0, ud1 = u * d1, ud2 = u * d2;
            const double f[kQ] = {u,        u * u,    ud0,      ud1,      ud2,     ud0 * d0,
                                  ud0 * d1, ud0 * d2, ud1 * d1, ud1 * d2, ud2 * d2};
#pragma unroll
            for (int j = 0; j < kQ; ++j) p[j] = (k == 2 * h) ? 0.0 + f[j] : p[j] + f[j];
        }
#pragma unroll
        for (int j = 0; j < kQ; ++j) q[j] = h ? q[j] + p[j] : p[j];     // (2l) + (2l+1)
    }
#pragma unroll
    for (int j = 0; j < kQ; ++j) L.u.q[T][j * 128 + tl] = q[j];
    __syncthreads();                                                    // (2)
    const int64_t bi = L.mi[2 * T] < L.mi[2 * T + 1] ? L.mi[2 * T] : L.mi[2 * T + 1];
    double pre = -1.0;
#pragma unroll
    for (int k = 0; k < kF4PPT; ++k) {
        const int64_t i = tbase + kF4PPT * tl + k;
        if (i < bi) pre = fmax(pre, wv[k]);
        if (i == bi && tile < nb_part) {
            dp.pxe[0][tile] = xv[k];
            dp.pxe[1][tile] = yv[k];
            dp.pxe[2][tile] = tv[k];
        }
    }
    pre = wave_max_f64(pre);
    if (lane == 0) L.pre[wave] = pre;
    // quantity it / 16, segment it % 16: pairs seg, seg + 16, ..., seg + 112;
    // then leaf (it - 176) >> 3, accumulator it & 7: elements k, k + 8, ...
    for (int it = tl; it < kQ * 16 + 8 * (kPartPer / 128); it += 128) {
        if (it < kQ * 16) {
            const double* a = L.u.q[T] + (it >> 4) * 128 + (it & 15);
            double acc = a[0];
#pragma unroll
            for (int mm = 1; mm < 8; ++mm) acc = acc + a[16 * mm];
            L.seg[T][it] = acc;
        } else {
            const int li = it - kQ * 16;
            const double* a = L.w[T] + (li >> 3) * 128 + (li & 7);
            double acc = a[0];
#pragma unroll
            for (int mm = 1; mm < 16; ++mm) acc = acc + a[8 * mm];
            L.acc[T][li] = acc;
        }
    }
    __syncthreads();                                                    // (3)
    if (tile >= nb_part) return;
    if (!(wave & 1)) {
        if (lane < kQ) {
            double acc = L.seg[T][16 * lane];
            for (int mm = 1; mm < 16; ++mm) acc = acc + L.seg[T][16 * lane + mm];
            dp.ps[lane][tile] = acc;
        }
    } else if (lane < 4) {
        // the tile's np.sum subtree: its four leaves, then their pair sums
        const double* r = L.acc[T] + 8 * lane;
        double v = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int d = 1; d < 4; d <<= 1) {
            const double o = xor_f64(v, d);
            v = (lane & d) ? (o + v) : (v + o);
        }
        if (lane == 0) dp.leaf[tile] = v;
    } else if (lane == 32) {
        dp.pmax[tile] = M;
        dp.pidx[tile] = bi;
        dp.ppre[tile] = fmax(L.pre[2 * T], L.pre[2 * T + 1]);
    }
}

template <int MOTION, int LIK, bool HOSTNOISE>
__global__ __launch_bounds__(256) SLAM_FUSED_ATTR void pf_fused4_kernel(
    const int64_t n, const double* __restrict__ xs, const double* __restrict__ ys,
    const double* __restrict__ ts, double* __restrict__ xo, double* __restrict__ yo,
    double* __restrict__ to, double* __restrict__ w_un, const double* __restrict__ c,
    int32_t* __restrict__ flags, const double* __restrict__ noise, const double* __restrict__ lm,
    StepIO io, PredictConst pc, LikConst lc, uint64_t seed, const double* __restrict__ s_in,
    const double* __restrict__ refp, DeferParts dp, const int32_t nb_part) {
    __shared__ F4Lds L;
    const int32_t st = io.ctr[0];
    const uint32_t rstep = (uint32_t)io.ctr[1];
    const int32_t rflag = flags[kFlagResample];
    const double* __restrict__ zs = io.z + (size_t)st * 2 * (size_t)(lc.nl > 0 ? lc.nl : 1);
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = (int)__lane_id();
    const int t = (wave << 6) | lane;
    const int64_t base = (int64_t)blockIdx.x * kF4Block;
    const int64_t i0 = base + kF4PPT * (int64_t)t;
    RngTabs rtab{};
    if constexpr (MOTION != kMotionNone && !HOSTNOISE) {
        rtab = rng_tabs_stage(&L.u.rng, (int)threadIdx.x, 256);
        __syncthreads();
    }

    // ---- resample gather (particle_filter.py:216-221): the source of each of
    //      the lane's four positions from the expand pass's run marks and the
    //      tile's carry (a running max), or -- after a scan fallback -- by a
    //      search of the exact cumsum
    const bool gather = rflag == 1;
    int32_t src[kF4PPT];
    if (gather) {
        if (!flags[kFlagFallback]) {
            const uint32_t mgen = (uint32_t)flags[kFlagMarkGen];
            int32_t r[kF4PPT];
#pragma unroll
            for (int k = 0; k < kF4PPT; ++k) {
                const int64_t mk = i0 + k < n ? dp.mark[i0 + k] : -1;
                r[k] = ((uint64_t)mk >> 32) == mgen ? (int32_t)mk : -1;
                if (k > 0) r[k] = r[k] > r[k - 1] ? r[k] : r[k - 1];
            }
            int32_t before;
            const int32_t v = wave_max_scan_i32(r[kF4PPT - 1], before);
            if (lane == 63) L.wmax[wave] = v;
            __syncthreads();
            int32_t run = dp.carry[base / kPartPer + (wave >> 1)];
            if (wave & 1) run = L.wmax[wave - 1] > run ? L.wmax[wave - 1] : run;
            run = before > run ? before : run;
#pragma unroll
            for (int k = 0; k < kF4PPT; ++k) src[k] = r[k] > run ? r[k] : run;
        } else {
            const double ofs = resample_offset(io.ofs[st], pc.np_recip, seed, rstep);
#pragma unroll
            for (int k = 0; k < kF4PPT; ++k) {
                const int64_t ik = i0 + k < n ? i0 + k : n - 1;
                src[k] = (int32_t)search_c(c, 0, n, (double)ik * pc.rstep + ofs);
            }
        }
#pragma unroll
        for (int k = 0; k < kF4PPT; ++k) {
            if (src[k] >= n) {
                src[k] = (int32_t)(n - 1);                        // IndexError in the reference
                if (i0 + k < n) atomicOr(&flags[kFlagStatus], 1);
            }
            src[k] = src[k] < 0 ? 0 : src[k];
        }
    }

    const double v_in = io.ctl[2 * st], om_in = io.ctl[2 * st + 1];
    const double s_prev = *s_in;
    const double* __restrict__ zc = io.zc + (size_t)st * kZcWords;
    double wv[kF4PPT], xv[kF4PPT], yv[kF4PPT], tv[kF4PPT];
    int dd_waves = 0;                       // halves (128-particle waves of the pair kernel)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int64_t ih = i0 + 2 * h;
        // the step's control laundered per pair: the values derived from it on
        // the VALU (noise scales, turn terms) are formed again for the second
        // pair instead of being held in VGPRs across the first
        double v = v_in, om = om_in;
        asm volatile("" : "+s"(v), "+s"(om));
        // loads of the pair first (previous weights, particles, host normals),
        // so that their latency runs under the device RNG
        const double2 wu = *reinterpret_cast<const double2*>(w_un + ih);
        double x[2], y[2], th[2];
        if (!gather) {
            const double2 a = *reinterpret_cast<const double2*>(xs + ih);
            const double2 b = *reinterpret_cast<const double2*>(ys + ih);
            const double2 c2 = *reinterpret_cast<const double2*>(ts + ih);
            x[0] = a.x;
            x[1] = a.y;
            y[0] = b.x;
            y[1] = b.y;
            th[0] = c2.x;
            th[1] = c2.y;
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                x[k] = xs[src[2 * h + k]];
                y[k] = ys[src[2 * h + k]];
                th[k] = ts[src[2 * h + k]];
            }
        }
        double g[2][3];
        if constexpr (MOTION == kMotionNone) {
#pragma unroll
            for (int k = 0; k < 2; ++k) g[k][0] = g[k][1] = g[k][2] = 0.0;
        } else if constexpr (HOSTNOISE) {
            if (ih + 2 <= n) {
                const double2* q2 = reinterpret_cast<const double2*>(noise + 3 * ih);
                const double2 a = q2[0], b = q2[1], c3 = q2[2];
                g[0][0] = a.x;
                g[0][1] = a.y;
                g[0][2] = b.x;
                g[1][0] = b.y;
                g[1][1] = c3.x;
                g[1][2] = c3.y;
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int64_t ik = ih + k < n ? ih + k : n - 1;
#pragma unroll
                    for (int j = 0; j < 3; ++j) g[k][j] = noise[3 * ik + j];
                }
            }
        } else {
            double hh[6];
            pair_normals((uint64_t)(pc.gbase + ih) >> 1, rstep, seed, rtab, hh);
#pragma unroll
            for (int j = 0; j < 6; ++j) g[j / 3][j % 3] = hh[j];
            if (MOTION == SLAM_MOTION_LINEAR) {                   // noise_j = sum_k g_k q[k][j]
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const double h0 = g[k][0], h1 = g[k][1], h2 = g[k][2];
                    g[k][0] = h0 * pc.q[0] + h1 * pc.q[3] + h2 * pc.q[6];
                    g[k][1] = h0 * pc.q[1] + h1 * pc.q[4] + h2 * pc.q[7];
                    g[k][2] = h0 * pc.q[2] + h1 * pc.q[5] + h2 * pc.q[8];
                }
            }
        }
        double px[2], py[2], pt[2], sp[2], cp[2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
            predict_particle<MOTION>(x[k], y[k], th[k], v, om, g[k][0], g[k][1], g[k][2], pc,
                                     px[k], py[k], pt[k], sp[k], cp[k]);
        *reinterpret_cast<double2*>(xo + ih) = double2{px[0], px[1]};
        *reinterpret_cast<double2*>(yo + ih) = double2{py[0], py[1]};
        *reinterpret_cast<double2*>(to + ih) = double2{pt[0], pt[1]};
        double bn[2];
        const int lane_dd = likelihood_lanes<LIK, 2>(px, py, sp, cp, lm, zs, zc, lc, bn, wave);
        dd_waves += __ballot(lane_dd) != 0 ? 1 : 0;
        // previous weights: particle_filter.py:222 (a resampled step starts from
        // 1/NP) / :235-236 (w_un / s, NaN -> 1/NP); particle_filter.py:194
        const double wp[2] = {wu.x, wu.y};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const double pw = rflag ? pc.np_recip : norm_w(wp[k], s_prev, pc.np_recip);
            wv[2 * h + k] = ih + k < n ? pw * bn[k] : 0.0;
            xv[2 * h + k] = px[k];
            yv[2 * h + k] = py[k];
            tv[2 * h + k] = pt[k];
        }
        *reinterpret_cast<double2*>(w_un + ih) = double2{wv[2 * h], wv[2 * h + 1]};
        *reinterpret_cast<double2*>(&L.w[wave >> 1][kF4PPT * (t & 127) + 2 * h]) =
            double2{wv[2 * h], wv[2 * h + 1]};
        __builtin_amdgcn_sched_barrier(0);        // the second pair after the first
    }
    {
        // the first pair's outputs back from where they were stored (L2 / LDS)
        // rather than held in 16 VGPRs across the second pair (which spilled):
        // the index passes through an empty asm, so the loads are not folded
        // into the stored values
        int64_t ir = i0;
        int32_t lr = kF4PPT * (t & 127);
        asm volatile("" : "+v"(ir), "+v"(lr));
        const double2 a = *reinterpret_cast<const double2*>(xo + ir);
        const double2 b = *reinterpret_cast<const double2*>(yo + ir);
        const double2 c2 = *reinterpret_cast<const double2*>(to + ir);
        const double2 d = *reinterpret_cast<const double2*>(&L.w[wave >> 1][lr]);
        xv[0] = a.x;
        xv[1] = a.y;
        yv[0] = b.x;
        yv[1] = b.y;
        tv[0] = c2.x;
        tv[1] = c2.y;
        wv[0] = d.x;
        wv[1] = d.y;
    }
    if (dd_waves && lane == 0) atomicAdd(&flags[kFlagDDWaves], dd_waves);
    defer_epilogue4(base, n, wv, xv, yv, tv, refp, dp, L, wave, nb_part);
    // block 0, after its own particles: the NEXT step's closed-form words
    // (as pf_fused_kernel)
    if (MOTION != kMotionNone && lc.closed && blockIdx.x == 0 && st + 1 < io.cap) {
        __shared__ double s_prep[16];
        const int32_t sn = st + 1;
        closed_prep_sums(lm, io.z + (size_t)sn * 2 * lc.nl, lc.nl, wave, 4, s_prep);
        __syncthreads();
        if (threadIdx.x == 0) {
            double px, py, pth;
            closed_prep_reference(refp, 2, io.ctl[2 * sn], io.ctl[2 * sn + 1], pc.dt, io.motion, px,
                                  py, pth);
            closed_prep_constants(s_prep, lc.nl, px, py, pth, io.zc + (size_t)sn * kZcWords);
        }
    }
}

