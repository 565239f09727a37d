// pf_finscan.inl -- the end of PF step t and, when step t + 1 resamples, its
// exact cumsum, in ONE launch (included by pf_api.hip after pf_kernels.inl).
//
// finalize_deferred_kernel runs on one CU that pulls all 2048 fused-block
// partials (262 KB), and the next step's scan_lean_merged_kernel is a launch
// of its own that exits at once on the two steps in three that do not
// resample.  Here the scan grid does both:
//
//  F1  every block: the register work of the finalize lanes (lane L owns the
//      fused blocks L + 512 k, as in finalize_deferred_kernel) -- one wave
//      per lane, the 48 partials, the 64 leaves of np.sum buffer L and the 4
//      argmax records loaded one per lane in a single round trip; the lane's
//      max, its sums scaled to that max and buffer L's pairwise sum are
//      staged write-through.
//  F2  the last arriving block: finalize_deferred_kernel's remaining steps,
//      the same operations in the same order (bit-identical), reading 512
//      staged lanes (~50 KB) instead of the block partials; the result record,
//      the step context, s, and -- when the next step resamples -- the
//      prefix of the fused-block totals for its scan.  Then it releases the
//      grid (a write-through token).
//  S   when the next step resamples: scan_lean_merged_kernel's body, with the
//      values F2 wrote in this launch (s, boff, ctr, the mark tag) read
//      write-through.
//
// particle_filter.py:115-117 (max / argmax), :210 (ESS), :212 (cumsum),
// :234-236 (np.sum and the division), as finalize_deferred_kernel.
namespace slam {

constexpr int kFsLanes = kFinThreads;          // 512 finalize lanes
constexpr int kFsA = 12;                       // staged per lane: mlane, acc[11]
constexpr int kFsMaxTailLeaves = 128;
constexpr int kFlagFinToken = 6;               // flag word: release token of F2
static_assert(kFlagFinToken < kFlagWords, "flag words");

// staging area of one handle (device memory, one allocation)
struct FinStage {
    double* a;          // [kFsLanes][kFsA]
    double* pm;         // [kFsLanes][4] block maxima of the lane's blocks
    double* buf;        // [128] np.sum buffer sums (full buffers)
};

// F1 for finalize lane L, one wave (wave-uniform control flow)
__device__ __forceinline__ void finscan_lane(const int L, const int64_t nb, const int64_t nfull,
                                             const DeferParts& dp, const FinStage& fs) {
    const int lane = threadIdx.x & 63;
    // lane j < 48: block L + 512 (j / 12), column j % 12 (0: pmax, 1..11: ps[c - 1])
    double v = 0.0;
    if (lane < 4 * kFsA) {
        const int k = lane / kFsA, col = lane % kFsA;
        const int64_t b = L + (int64_t)kFsLanes * k;
        // per-lane column: a select chain (an indexed read of the kernel
        // argument's pointer array would go through scratch)
        const double* p = dp.pmax;
#pragma unroll
        for (int cc = 1; cc < kFsA; ++cc)
            if (col == cc) p = dp.ps[cc - 1];
        if (b < nb) v = p[b];
    }
    double lf = 0.0;
    if (L < nfull) lf = dp.leaf[64 * (int64_t)L + lane];
    // every lane forms the lane's sums from the 48 values (uniform, in the order
    // of finalize_deferred_kernel: max over k, then k = 0..3 into acc)
    double pm[4];
    bool has[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        has[k] = L + (int64_t)kFsLanes * k < nb;
        pm[k] = __shfl(v, kFsA * k, 64);
    }
    double mlane = -1.0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (has[k]) mlane = fmax(mlane, pm[k]);
    double acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = 0.0;
    if (mlane > 0.0) {
        const double rm = 1.0 / mlane;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (has[k]) {
                const double r = pm[k] * rm;
                acc[0] += r * __shfl(v, kFsA * k + 1, 64);
                acc[1] += (r * r) * __shfl(v, kFsA * k + 2, 64);
#pragma unroll
                for (int j = 2; j < 11; ++j) acc[j] += r * __shfl(v, kFsA * k + 1 + j, 64);
            }
        }
    }
    // np.sum buffer L: the pairwise tree of its 64 leaves (16-leaf subtrees of
    // the four lanes of finalize_deferred_kernel, then their pair sums)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_xor(lf, d, 64);
        lf = (lane & d) ? (o + lf) : (lf + o);
    }
    // staged write-through: lane j < 12 one value of a[], lanes 12..15 the maxima
    double out = 0.0;
    if (lane == 0) out = mlane;
#pragma unroll
    for (int j = 0; j < 11; ++j)
        if (lane == 1 + j) out = acc[j];
    if (lane < kFsA) st_wt_d(&fs.a[(int64_t)L * kFsA + lane], out);
    if (lane >= kFsA && lane < kFsA + 4) {
        const int k = lane - kFsA;
        st_wt_d(&fs.pm[4 * L + k], has[k] ? pm[k] : -1.0);
    }
    if (lane == 16 && L < nfull) st_wt_d(&fs.buf[L], lf);
}

__global__ __launch_bounds__(kScanThreads) __attribute__((amdgpu_waves_per_eu(4))) void finscan_kernel(
    const int64_t n, const DeferParts dp, const FinStage fs, const double* __restrict__ w_un,
    double* __restrict__ s_cur, const int32_t* __restrict__ tail_leaves,
    const int32_t* __restrict__ tail_ops, const int32_t n_tail_leaves, const int32_t n_tail_ops,
    const double* __restrict__ xs, const double* __restrict__ ys, const double* __restrict__ ts,
    double* __restrict__ refp, int32_t* __restrict__ flags, const double ess_th, const StepIO io,
    const double np_recip, double* __restrict__ boff, unsigned* __restrict__ tk_fin,
    int32_t* __restrict__ fin_token_word,
    // the scan (scan_lean_merged_kernel's arguments)
    const double delta, SpecialIn* __restrict__ stage, uint64_t* __restrict__ bk,
    int32_t* __restrict__ bf, uint64_t* __restrict__ boffk, int32_t* __restrict__ bofff,
    uint64_t* __restrict__ ktot, int32_t* __restrict__ nspec, unsigned* __restrict__ tk_scan,
    SpecialOut* __restrict__ spec_out, double* __restrict__ c, const PredictConst pc,
    const uint64_t seed, int32_t* __restrict__ scan_token_word, const int ntiles) {
    __shared__ int s_go;
    __shared__ double s_s;
    __shared__ double s_tot[11];
    __shared__ unsigned long long s_min;
    __shared__ int32_t s_flag;
    __shared__ int64_t s_mi;
    __shared__ double s_xe[3];
    __shared__ int s_ncand;
    __shared__ int64_t s_cblk[kFinCand];
    __shared__ FinRecord s_crec[kFinCand];
    __shared__ double s_sh[kFsMaxTailLeaves];
    __shared__ double s_wt[8 + 1];
    __shared__ double s_buf[128];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = (int)gridDim.x;
    const int64_t nb = (n + kPartPer - 1) / kPartPer;
    const int64_t nfull = n / kSumChunk;
    const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
    // tokens read before this block arrives (the releasing block arrives last)
    const int32_t fin_token = ld_wt_i(fin_token_word) + 1;
    const int32_t scan_token = ld_wt_i(scan_token_word) + 1;

    // ---------------- F1
    for (int L = (int)blockIdx.x + G * wave; L < kFsLanes; L += 4 * G) finscan_lane(L, nb, nfull, dp, fs);
    if (arrive_last(tk_fin)) {
        // ---------------- F2 (finalize_deferred_kernel from the staged lanes)
        if (tid == 0) {
            s_ncand = 0;
            s_min = ~0ull;
            s_flag = 0;
        }
        // np.sum of the tail buffer (< 8192 elements) first: few registers live
        double tsum = 0.0;
        if (nch > nfull)
            tsum = tail_chunk_sum(w_un + nfull * kSumChunk, tail_leaves, tail_ops, n_tail_leaves,
                                  n_tail_ops, s_sh);
        // lane l of every wave: the 8 finalize lanes l + 64 m (every wave sees all 512)
        double ml[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) ml[m] = ld_wt_d(&fs.a[(int64_t)(lane + 64 * m) * kFsA]);
        // the sums this wave reduces: quantities wave, wave + 4, wave + 8
        double q[3][8];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int j = wave + 4 * r;
#pragma unroll
            for (int m = 0; m < 8; ++m)
                q[r][m] = (j < 11) ? ld_wt_d(&fs.a[(int64_t)(lane + 64 * m) * kFsA + 1 + j]) : 0.0;
        }
        // the block maxima of this thread's two lanes (m = 2 wave, 2 wave + 1)
        double pmv[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int k = 0; k < 4; ++k) pmv[h][k] = ld_wt_d(&fs.pm[4 * (lane + 64 * (2 * wave + h)) + k]);
        // the np.sum buffer sums into LDS (thread 0 chains them)
        if (tid < nfull) s_buf[tid] = ld_wt_d(&fs.buf[tid]);
        double M = -1.0;
#pragma unroll
        for (int m = 0; m < 8; ++m) M = fmax(M, ml[m]);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) M = fmax(M, __shfl_xor(M, d, 64));
        __syncthreads();                                  // s_ncand etc. initialised
        double s = 0.0;
        if (tid == 0) {
            // np.sum: the full buffers left to right (one round of <= 128)
            __builtin_amdgcn_s_setprio(3);
            for (int k = 0; k < nfull; ++k) s = s + s_buf[k];
            __builtin_amdgcn_s_setprio(0);
        } else {
            // argmax records of the candidate blocks, staged in LDS meanwhile
            // (fl(M_b / s) == fl(M / s) needs M_b within 2 ulp of M)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t b = (lane + 64 * (2 * wave + h)) + (int64_t)kFsLanes * k;
                    if (b < nb && pmv[h][k] >= M * (1.0 - 0x1p-48)) {
                        const int slot = atomicAdd(&s_ncand, 1);
                        if (slot < kFinCand) {
                            FinRecord f;
                            fin_load_record(dp, b, f);
                            s_cblk[slot] = b;
                            s_crec[slot] = f;
                        }
                    }
                }
        }
        if (tid == 0) {
            // thread 0's own two lanes (lanes 0 and 64)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t b = 64 * h + (int64_t)kFsLanes * k;
                    if (b < nb && pmv[h][k] >= M * (1.0 - 0x1p-48)) {
                        const int slot = atomicAdd(&s_ncand, 1);
                        if (slot < kFinCand) {
                            FinRecord f;
                            fin_load_record(dp, b, f);
                            s_cblk[slot] = b;
                            s_crec[slot] = f;
                        }
                    }
                }
        }
        if (nch > nfull) s = s + tsum;                 // thread 0: the tail buffer last
        if (tid == 0) s_s = s;
        __syncthreads();
        s = s_s;
        const bool ok = (s > 0.0) && !isinf(s) && (M > 0.0);
        BlockPartial tot;
        bp_zero(tot);
        if (ok) {
            // the 11 sums: lane-strided over the 8 lanes, then the butterfly
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int j = wave + 4 * r;
                if (j < 11) {
                    double acc = 0.0;
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        const double rl = (ml[m] > 0.0 && M > 0.0) ? ml[m] / M : 0.0;
                        const double val = (j == 1) ? q[r][m] * (rl * rl) : q[r][m] * rl;
                        acc = (m == 0) ? val : acc + val;
                    }
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const double o = __shfl_xor(acc, d, 64);
                        acc = (lane & d) ? (o + acc) : (acc + o);
                    }
                    if (lane == 0) s_tot[j] = acc;
                }
            }
            // argmax: the first block whose max rounds to fl(M / s)
            const double mval = M / s;
            unsigned long long cb = ~0ull;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t b = (lane + 64 * (2 * wave + h)) + (int64_t)kFsLanes * k;
                    if (b < nb && pmv[h][k] >= M * (1.0 - 0x1p-48) && pmv[h][k] / s == mval &&
                        (unsigned long long)b < cb)
                        cb = (unsigned long long)b;
                }
            if (cb != ~0ull) atomicMin(&s_min, cb);
            __syncthreads();
            const int64_t bc = (int64_t)s_min;
            if (tid == 0) {
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
                for (int e = tid; e < kPartPer; e += blockDim.x) {
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
                const double f = M / s;
                tot.maxv = mval;
                tot.maxi = s_mi;
                tot.sw = s_tot[0] * f;
                tot.sw2 = s_tot[1] * (f * f);
                for (int j = 0; j < 3; ++j) tot.m1[j] = s_tot[2 + j] * f;
                for (int j = 0; j < 6; ++j) tot.m2[j] = s_tot[5 + j] * f;
            }
        } else {
            // every weight through the reference's division (degenerate case),
            // with finalize_deferred_kernel's 512 lane partials and tree: this
            // thread plays lanes tid (wave w) and tid + 256 (wave w + 4)
            __shared__ BlockPartial shp[kFsLanes / 64];
            const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
#pragma unroll
            for (int hv = 0; hv < 2; ++hv) {
                BlockPartial a;
                bp_zero(a);
                for (int64_t i = tid + kScanThreads * hv; i < n; i += kFsLanes) {
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
                bp_wave_reduce(a);
                if (lane == 0) shp[wave + 4 * hv] = a;
            }
            __syncthreads();
            if (tid < 64) {
                if (tid < kFsLanes / 64) tot = shp[tid];
                else bp_zero(tot);
                bp_wave_reduce<8>(tot);
            }
            __syncthreads();
            if (tid == 0) {
                s_xe[0] = xs[tot.maxi];
                s_xe[1] = ys[tot.maxi];
                s_xe[2] = ts[tot.maxi];
            }
        }
        if (tid == 0) {
            const int32_t st = io.ctr[0];
            write_result_xe(tot, s_xe, refp, s, flags, ess_th, io.res + st, -1);
            s_flag = flags[kFlagResample];
            io.ctr[0] = st + 1;
            io.ctr[1] = io.ctr[1] + 1;
            st_wt_d(s_cur, s);
        }
        __syncthreads();
        if (s_flag) {
            // fused-block totals of w for the next step's exact cumsum: the 512
            // lanes of finalize_deferred_kernel (lane t owns the contiguous
            // blocks [t per, (t + 1) per)) as two virtual waves per wave
            const int per = (int)((nb + kFsLanes - 1) / kFsLanes);
            auto btot = [&](int64_t b) {
                if (ok) return (dp.pmax[b] / s) * dp.ps[0][b];
                double v = 0.0;
                const int64_t e = (b + 1) * kPartPer < n ? (b + 1) * kPartPer : n;
                for (int64_t i = b * kPartPer; i < e; ++i) v += norm_w(w_un[i], s, np_recip);
                return v;
            };
            double loc[2], inc[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t b0 = (int64_t)(64 * (wave + 4 * h) + lane) * per;
                loc[h] = 0.0;
                for (int k = 0; k < per; ++k)
                    if (b0 + k < nb) loc[h] += btot(b0 + k);
                inc[h] = wave_incl_scan(loc[h]);
                if (lane == 63) s_wt[wave + 4 * h] = inc[h];
            }
            __syncthreads();
            if (tid == 0) {
                double run = 0.0;
                for (int k = 0; k < 8; ++k) {
                    const double t = s_wt[k];
                    s_wt[k] = run;
                    run = run + t;
                }
                s_wt[8] = run;
            }
            __syncthreads();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                double ex = __shfl_up(inc[h], 1, 64);
                if (lane == 0) ex = 0.0;
                ex = s_wt[wave + 4 * h] + ex;
                const int64_t b0 = (int64_t)(64 * (wave + 4 * h) + lane) * per;
                for (int k = 0; k < per; ++k)
                    if (b0 + k < nb) {
                        st_wt_d(&boff[b0 + k], ex);
                        ex = ex + btot(b0 + k);
                    }
            }
            if (tid == 0) st_wt_d(&boff[nb], s_wt[8]);
        }
        // release the grid (every store of this block drained and written back first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st_wt_i(fin_token_word, fin_token);
            s_go = 1;
        }
    } else if (tid == 0) {
        int go = 0;
        for (int it = 0; it < (1 << 22); ++it) {
            if (ld_wt_i(fin_token_word) == fin_token) {
                go = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!go) atomicOr(&flags[kFlagStatus], 8);        // token never came: skip, do not hang
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_go = go;
    }
    __syncthreads();
    if (!s_go || ld_wt_i(&flags[kFlagResample]) != 1) return;

    // ---------------- S: scan_lean_merged_kernel's body for the next step
    __shared__ int s_go2;
    const double s = ld_wt_d(s_cur);
    const int32_t ctr0 = ld_wt_i(&io.ctr[0]), ctr1 = ld_wt_i(&io.ctr[1]);
    const double ofs = resample_offset(io.ofs[ctr0], pc.np_recip, seed, (uint32_t)ctr1);
    const int64_t gen = (int64_t)(uint32_t)ld_wt_i(&flags[kFlagMarkGen]) << 32;
    const int64_t tile = (int64_t)blockIdx.x * kTilesPerBlock + wave;
    const bool active = tile < ntiles;
    TileScan tsc;
    uint64_t ktile = 0, kofs, kblk;
    int32_t ftile = 0, fofs, fblk;
    if (active)
        wave_tile_classify(w_un, s, np_recip, n, tile, ld_wt_d(&boff[tile]), delta, tsc, ktile, ftile);
    block_tile_offsets(ktile, ftile, kofs, fofs, kblk, fblk);
    if (active) wave_tile_stage(tile, tsc, kofs, fofs, kblk, fblk, stage, bk, bf);
    else if (tid == 0) {
        st_wt(&bk[blockIdx.x], kblk);
        st_wt_i(&bf[blockIdx.x], fblk);
    }
    if (arrive_last(tk_scan)) {
        lean_last_block(bk, bf, boffk, bofff, ktot, nspec, G, stage, n, spec_out, flags, w_un, s_cur,
                        np_recip, c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st_wt_i(scan_token_word, scan_token);
            s_go2 = 1;
        }
    } else if (tid == 0) {
        int go = 0;
        for (int it = 0; it < (1 << 22); ++it) {
            if (ld_wt_i(scan_token_word) == scan_token) {
                go = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!go) atomicOr(&flags[kFlagStatus], 8);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_go2 = go;
    }
    __syncthreads();
    if (!active || !s_go2 || ld_wt_i(&flags[kFlagFallback])) return;
    wave_tile_expand(tile, tsc, n, boffk, bofff, kofs, fofs, spec_out, c, dp.mark, dp.carry, ofs, gen,
                     pc, true);
}

}  // namespace slam
