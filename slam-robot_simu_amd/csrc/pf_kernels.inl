// pf_kernels.inl -- gfx950 kernels of the particle-filter step (included by pf_api.hip).
//
// Step = fused [systematic-resample gather +] predict + likelihood ->
//        numpy-order chunk sums -> normalise + reductions + result record.
// The exact sequential cumsum that feeds the resample gather is computed by
// the scan_* passes (launched at the start of a step; they gate on the
// device resample flag, so a device-resident run needs no host decisions).
// Particles are SoA fp64 (x[], y[], th[]) in HBM, one particle per lane.
#include <type_traits>

#include "pf_kernels.hpp"

// Phase stamps of the resample passes (probe builds only: -DSLAM_PROBE,
// read back with slam_probe_read; never in the product library).  PROBE_MAX
// samples every 32nd block: one atomic word taking every block's stamp
// serialises them (~12 ns each) and would time itself.
#ifdef SLAM_PROBE
__device__ unsigned long long g_probe[32];
#define PROBE_AT(k) do { if (threadIdx.x == 0) g_probe[k] = wall_clock64(); } while (0)
#define PROBE_MAX(k) do { if (threadIdx.x == 0 && (blockIdx.x & 31) == 0) atomicMax(&g_probe[k], (unsigned long long)wall_clock64()); } while (0)
#else
#define PROBE_AT(k) do { } while (0)
#define PROBE_MAX(k) do { } while (0)
#endif

namespace slam {

// Fused-kernel phase stamps (probe builds only: -DSLAM_PROBE_FUSED): per block,
// wave 0's wall clock at entry, after the table staging, after the normals,
// after predict (its loads consumed), after the likelihood and at the end.
#ifdef SLAM_PROBE_FUSED
constexpr int kFProbeBlocks = 1 << 14;
__device__ unsigned long long g_fprobe[kFProbeBlocks * 8];
#define FPROBE(k, dep) do { asm volatile("" :: "v"(dep)); \
    if (threadIdx.x == 0 && blockIdx.x < kFProbeBlocks) g_fprobe[blockIdx.x * 8 + (k)] = wall_clock64(); } while (0)
#else
#define FPROBE(k, dep) do { } while (0)
#endif

#ifdef SLAM_PROBE_COUNT_SLOW
__device__ unsigned long long g_probe_slow[2];   // slow particles, blocks with any (probe builds)
#endif

// ====================================================================
// wave / block helpers (wave = 64 lanes)
// ====================================================================
// DPP row_shr:D of a 32- or 64-bit integer; lanes without a source read 0
template <int D, typename T>
__device__ __forceinline__ T dpp_row_shr0(const T v) {
    constexpr int kCtrl = 0x110 + D;
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, kCtrl, 0xF, 0xF, false);
        const uint32_t hi =
            (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), kCtrl, 0xF, 0xF, false);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
    }
}
template <typename T>
__device__ __forceinline__ T readlane_int(const T v, const int l) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__builtin_amdgcn_readlane((int)v, l);
    }
}

// inclusive wave scan.  Integers (exact in any order): Hillis-Steele inside
// each 16-lane row by DPP row shifts, then the lower rows' totals read into
// scalars; floating point keeps the lane-shuffle order.
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    if constexpr (std::is_integral<T>::value) {
        v += dpp_row_shr0<1>(v);
        v += dpp_row_shr0<2>(v);
        v += dpp_row_shr0<4>(v);
        v += dpp_row_shr0<8>(v);
        const T r0 = readlane_int(v, 15), r1 = readlane_int(v, 31), r2 = readlane_int(v, 47);
        const int row = (int)((threadIdx.x & 63) >> 4);
        v += (row >= 1 ? r0 : T(0)) + (row >= 2 ? r1 : T(0)) + (row >= 3 ? r2 : T(0));
        return v;
    } else {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            T o = __shfl_up(v, d, 64);
            if (lane >= d) v = v + o;
        }
        return v;
    }
}

// Exclusive wave scan of non-negative doubles in the integer scan's order (DPP
// row shifts, then the lower rows' totals: ~6x shorter in latency than the
// shuffle form; any fixed order serves an approximate prefix), formed
// without a subtraction (inc - v loses a small prefix ahead of a large
// element: its relative error is unbounded, which the exact cumsum's margins
// do not cover); `total` = the wave's sum (every lane).
__device__ __forceinline__ double wave_excl_scan_rows(double v, double& total) {
    auto sh = [](double x, auto d) {
        return __longlong_as_double((long long)dpp_row_shr0<decltype(d)::value>(
            (uint64_t)__double_as_longlong(x)));
    };
    v = v + sh(v, std::integral_constant<int, 1>{});
    v = v + sh(v, std::integral_constant<int, 2>{});
    v = v + sh(v, std::integral_constant<int, 4>{});
    v = v + sh(v, std::integral_constant<int, 8>{});
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const double r0 = __longlong_as_double((long long)readlane_int(b, 15));
    const double r1 = __longlong_as_double((long long)readlane_int(b, 31));
    const double r2 = __longlong_as_double((long long)readlane_int(b, 47));
    const double r3 = __longlong_as_double((long long)readlane_int(b, 63));
    const int row = (int)((threadIdx.x & 63) >> 4);
    double below = 0.0;
    if (row >= 1) below = r0;
    if (row >= 2) below = below + r1;
    if (row >= 3) below = below + r2;
    total = ((r0 + r1) + r2) + r3;
    const double prev = sh(v, std::integral_constant<int, 1>{});   // the row's inclusive, one lane down
    return (threadIdx.x & 15) ? below + prev : below;
}

// Sum over the wave in the same row order (every lane gets it): the rows'
// inclusive DPP scans, then ((row0 + row1) + row2) + row3.
__device__ __forceinline__ double wave_sum_rows(double v) {
    double total;
    (void)wave_excl_scan_rows(v, total);
    return total;
}

// Exclusive block scan over NT threads; sh needs NT/64+1 entries.  Returns the
// exclusive prefix of v, writes the block total to `total`.
template <typename T, int NT>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const T inc = wave_incl_scan(v);
    T ex;
    if constexpr (std::is_integral<T>::value) {
        ex = inc - v;
    } else {
        ex = __shfl_up(inc, 1, 64);
        if (lane == 0) ex = T(0);
    }
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = T(0);
        for (int k = 0; k < NT / 64; ++k) {
            const T t = sh[k];
            sh[k] = run;
            run = run + t;
        }
        sh[NT / 64] = run;
    }
    __syncthreads();
    const T r = sh[wid] + ex;
    total = sh[NT / 64];
    __syncthreads();
    return r;
}

// FMA-refined quotient x/d with rd = RN(1/d): q0 = RN(x*rd), r = x - d*q0
// (exact by FMA), q1 = RN(q0 + r*rd) -- the correctly rounded quotient for
// normal operands (Markstein); checked against IEEE division in the tests.
__device__ __forceinline__ double div_refined(double x, double d, double rd) {
    const double q0 = x * rd;
    const double r = fma(-q0, d, x);
    return fma(r, rd, q0);
}

// ---- write-through (sc1) hand-off words, MI355X_MICROARCH "Valid forms" row 1:
// the bytes one block hands to the last-arriving block are stored and loaded
// with agent-scope relaxed atomics (global_store/load ... sc1), the storing
// waves drain (vmcnt(0)) before the block barrier, one lane takes the ticket.
__device__ __forceinline__ void st_wt(void* p, uint64_t v) {
    __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_wt(const void* p) {
    return __hip_atomic_load((uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_d(double* p, double v) { st_wt(p, (uint64_t)__double_as_longlong(v)); }
__device__ __forceinline__ double ld_wt_d(const double* p) { return __longlong_as_double((long long)ld_wt(p)); }
__device__ __forceinline__ void st_wt_i(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_wt_i(const int32_t* p) {
    return __hip_atomic_load((int32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename S>
__device__ __forceinline__ void st_wt_struct(S* dst, const S& v) {
    static_assert(sizeof(S) % 8 == 0, "8-byte granules");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(S) / 8); ++k) st_wt(reinterpret_cast<uint64_t*>(dst) + k, src[k]);
}
template <typename S>
__device__ __forceinline__ S ld_wt_struct(const S* p) {
    S v;
    uint64_t* d = reinterpret_cast<uint64_t*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(S) / 8); ++k) d[k] = ld_wt(reinterpret_cast<const uint64_t*>(p) + k);
    return v;
}

// ---- last-arriver election (Guideline 16 / microarch "fanin" + "dequeue"):
// every block takes a ticket after publishing its write-through partials.
// One counter word serialises its arrivals (~12 ns each), so the tickets are
// two-level: blocks with equal blockIdx % 8 (one XCD under round-robin
// dispatch) share a counter on a 128-B line of its own, and the last of each
// residue class takes a ticket on the top word.  A ticket block is
// kTicketWords unsigned words; every word is re-zeroed by its last arriver.
constexpr int kTicketStride = 32;                       // 128 B
constexpr int kTicketWords = 9 * kTicketStride;

__device__ __forceinline__ bool arrive_last_n(unsigned* counter, const unsigned expected) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t =
            __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t == expected - 1) ? 1 : 0;
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last != 0;
}

__device__ __forceinline__ int ticket_groups() { return gridDim.x < 8 ? (int)gridDim.x : 8; }

// level 1 of the two-level ticket: true in the last block of this residue class
__device__ __forceinline__ bool arrive_group(unsigned* tk) {
    const int G = ticket_groups(), g = blockIdx.x % G;
    const unsigned ng = (gridDim.x - g + G - 1) / G;
    return arrive_last_n(tk + (1 + g) * kTicketStride, ng);
}

__device__ __forceinline__ bool arrive_last(unsigned* tk) {
    if (!arrive_group(tk)) return false;
    return arrive_last_n(tk, (unsigned)ticket_groups());
}

// ---- systematic resampling positions (particle_filter.py:213-215)
__device__ __forceinline__ double resample_offset(const double ofs_host, const double np_recip,
                                                  const uint64_t seed, const uint32_t stepno) {
    if (!isnan(ofs_host)) return ofs_host;
    const u32x4 ctr{0u, 0u, kStreamResample, stepno};
    const u32x4 r = philox4x32(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t m = ((uint64_t)(r.x >> 5) << 26) | (uint64_t)(r.y >> 6);
    return ((double)m * 0x1p-53) * np_recip;                 // rand() * NP_RECIP
}

// first j in [0, n) with c[j] >= pos (the while loop of :218-220); n if none
__device__ __forceinline__ int64_t lower_bound_c(const double* __restrict__ c, const int64_t n,
                                                 const double pos) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (c[mid] < pos) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ====================================================================
// fused [resample gather +] predict + likelihood
//      (particle_filter.py:156-198, :216-222; motion_model.py:31-62)
// ====================================================================
// weight of the current step from the deferred representation:
// particle_filter.py:235-236  w = w_un / s, NaN -> 1/NP
__device__ __forceinline__ double norm_w(const double wu, const double s, const double np_recip) {
    const double v = wu / s;
    return isnan(v) ? np_recip : v;
}

// (value, index) max with the first index on ties (np.argmax)
__device__ __forceinline__ void max_first(double& v, int64_t& i, const double ov, const int64_t oi) {
    if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}

// ---- wave reductions through DPP lane moves (VALU, no LDS round trip):
// quad_perm [1,0,3,2] is the lane-xor-1 partner (bit-identical to
// __shfl_xor(v, 1)); max / min over the wave by quad swaps, the half-row and
// row mirrors, then the four row results read into scalars.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(const uint64_t v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(const double v) {
    return __longlong_as_double((long long)dpp_u64<CTRL>((uint64_t)__double_as_longlong(v)));
}
__device__ __forceinline__ uint64_t readlane_u64(const uint64_t v, const int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// the lane-xor-d partner of a butterfly step (d a constant after unrolling):
// quad swaps by DPP for d = 1, 2, the LDS permute beyond
__device__ __forceinline__ double xor_f64(const double v, const int d) {
    if (d == 1) return dpp_f64<kDppXor1>(v);
    if (d == 2) return dpp_f64<kDppXor2>(v);
    return __shfl_xor(v, d, 64);
}
// inclusive max-scan of an int32 over the wave, and the exclusive value
// (lane 0: -1): row shifts by DPP (lanes without a source read -1), then the
// three lower rows' maxima read into scalars
__device__ __forceinline__ int32_t wave_max_scan_i32(int32_t v, int32_t& excl) {
    constexpr int kRowShr = 0x110;                                      // row_shr:d = 0x110 + d
    int32_t o;
    o = __builtin_amdgcn_update_dpp(-1, v, kRowShr + 1, 0xF, 0xF, false);
    v = o > v ? o : v;
    o = __builtin_amdgcn_update_dpp(-1, v, kRowShr + 2, 0xF, 0xF, false);
    v = o > v ? o : v;
    o = __builtin_amdgcn_update_dpp(-1, v, kRowShr + 4, 0xF, 0xF, false);
    v = o > v ? o : v;
    o = __builtin_amdgcn_update_dpp(-1, v, kRowShr + 8, 0xF, 0xF, false);
    v = o > v ? o : v;
    const int lane = (int)__lane_id(), row = lane >> 4;
    const int32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
    const int32_t r2 = __builtin_amdgcn_readlane(v, 47);
    const int32_t m01 = r0 > r1 ? r0 : r1, m012 = m01 > r2 ? m01 : r2;
    const int32_t below = row == 0 ? -1 : row == 1 ? r0 : row == 2 ? m01 : m012;
    v = below > v ? below : v;
    // lane l - 1's inclusive value: within the row by row_shr:1, the row's
    // first lane takes the rows below
    const int32_t prev = __builtin_amdgcn_update_dpp(-1, v, kRowShr + 1, 0xF, 0xF, false);
    excl = (lane & 15) ? prev : below;
    return v;
}

// integer sums over the wave (every lane gets them; any order is exact)
__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
    v += __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppMirror, 0xF, 0xF, false);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
           __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    v += dpp_u64<kDppXor1>(v);
    v += dpp_u64<kDppXor2>(v);
    v += dpp_u64<kDppHalfMirror>(v);
    v += dpp_u64<kDppMirror>(v);
    return readlane_u64(v, 0) + readlane_u64(v, 16) + readlane_u64(v, 32) + readlane_u64(v, 48);
}

// max over the wave (every lane gets it); fmax semantics as the butterfly's
__device__ __forceinline__ double wave_max_f64(double v) {
    v = fmax(v, dpp_f64<kDppXor1>(v));
    v = fmax(v, dpp_f64<kDppXor2>(v));
    v = fmax(v, dpp_f64<kDppHalfMirror>(v));
    v = fmax(v, dpp_f64<kDppMirror>(v));
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const double r0 = __longlong_as_double((long long)readlane_u64(b, 0));
    const double r1 = __longlong_as_double((long long)readlane_u64(b, 16));
    const double r2 = __longlong_as_double((long long)readlane_u64(b, 32));
    const double r3 = __longlong_as_double((long long)readlane_u64(b, 48));
    return fmax(fmax(r0, r1), fmax(r2, r3));
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
    int64_t o;
    o = (int64_t)dpp_u64<kDppXor1>((uint64_t)v);
    v = o < v ? o : v;
    o = (int64_t)dpp_u64<kDppXor2>((uint64_t)v);
    v = o < v ? o : v;
    o = (int64_t)dpp_u64<kDppHalfMirror>((uint64_t)v);
    v = o < v ? o : v;
    o = (int64_t)dpp_u64<kDppMirror>((uint64_t)v);
    v = o < v ? o : v;
    const int64_t r0 = (int64_t)readlane_u64((uint64_t)v, 0), r1 = (int64_t)readlane_u64((uint64_t)v, 16);
    const int64_t r2 = (int64_t)readlane_u64((uint64_t)v, 32), r3 = (int64_t)readlane_u64((uint64_t)v, 48);
    const int64_t a = r0 < r1 ? r0 : r1, b = r2 < r3 ? r2 : r3;
    return a < b ? a : b;
}

// Deferred-path epilogue of a 256-lane, kPartPer-particle fused block (see
// DeferParts).  Lane t holds particles kDeferPPT t + k (k < kDeferPPT); invalid
// ones carry w = 0.  Three barriers: (1) the wave maxima, (2) the lane-pair
// moment sums and the wave argmax candidates, (3) the segment sums and leaf
// accumulators.  Every sum has a fixed order: per lane over k, lane pairs
// (2l, 2l+1), 16 pair-strided segments of 8 (conflict-free LDS reads) left to
// right, then the 16 segments.
#ifndef SLAM_EPI_FMA
#define SLAM_EPI_FMA 0
#endif
__device__ void defer_epilogue(const int64_t base, const int64_t n, const double* wv,
                               const double* xv, const double* yv, const double* tv,
                               const double* __restrict__ refp, const DeferParts& dp,
                               const int wave_s, const int blk) {
    constexpr int kQ = 11;
    constexpr int kLeaves = kPartPer / 128;
    __shared__ double s_w[kPartPer];
    __shared__ double s_q[kQ * 128];
    __shared__ double s_seg[kQ * 16];
    __shared__ double s_acc[8 * kLeaves];
    __shared__ double s_mv[4], s_pre[4];
    __shared__ int64_t s_mi[4];
    // the thread index from the wave's SGPR index and the lane id (both
    // rematerialised: threadIdx.x itself would be held across the kernel)
    const int lane = (int)__lane_id(), wave = wave_s, t = (wave << 6) | lane;
    // lane max and its first particle, then the wave max
    double m = -1.0;
    int64_t mi = INT64_MAX;
#pragma unroll
    for (int k = 0; k < kDeferPPT; ++k) {
        const int64_t i = base + kDeferPPT * t + k;
        const bool ok = i < n;
        s_w[kDeferPPT * t + k] = ok ? wv[k] : 0.0;
        if (ok && wv[k] > m) {
            m = wv[k];
            mi = i;
        }
    }
    const double mv = wave_max_f64(m);
    if (lane == 0) s_mv[wave] = mv;
    __syncthreads();                                                    // (1)
    const double M = fmax(fmax(s_mv[0], s_mv[1]), fmax(s_mv[2], s_mv[3]));
    // first index holding M in this wave
    const int64_t cand = wave_min_i64((m == M) ? mi : INT64_MAX);
    if (lane == 0) s_mi[wave] = cand;
    // moments scaled by the block max, lane-pair sums into LDS
    const double rs = (M > 0.0) ? 1.0 / M : 0.0;
    const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
    double q[kQ];
#pragma unroll
    for (int j = 0; j < kQ; ++j) q[j] = 0.0;
#pragma unroll
    for (int k = 0; k < kDeferPPT; ++k) {
        const bool ok = base + kDeferPPT * t + k < n;
        const double u = ok ? wv[k] * rs : 0.0;
        const double d0 = xv[k] - r0, d1 = yv[k] - r1, d2 = tv[k] - r2;
        const double ud0 = u * d0, ud1 = u * d1, ud2 = u * d2;
        q[0] += u;
        q[2] += ud0;
        q[3] += ud1;
        q[4] += ud2;
#if SLAM_EPI_FMA
        // the second moments as fused multiply-adds (one rounding each; the
        // partials are the filter's own, not the reference's: cov 1e-6)
        q[1] = fma(u, u, q[1]);
        q[5] = fma(ud0, d0, q[5]);
        q[6] = fma(ud0, d1, q[6]);
        q[7] = fma(ud0, d2, q[7]);
        q[8] = fma(ud1, d1, q[8]);
        q[9] = fma(ud1, d2, q[9]);
        q[10] = fma(ud2, d2, q[10]);
#else
        q[1] += u * u;
        q[5] += ud0 * d0;
        q[6] += ud0 * d1;
        q[7] += ud0 * d2;
        q[8] += ud1 * d1;
        q[9] += ud1 * d2;
        q[10] += ud2 * d2;
#endif
    }
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
        const double o = dpp_f64<kDppXor1>(q[j]);
        q[j] = (lane & 1) ? o + q[j] : q[j] + o;                     // (2l) + (2l+1)
    }
    if (!(lane & 1)) {
#pragma unroll
        for (int j = 0; j < kQ; ++j) s_q[j * 128 + (t >> 1)] = q[j];
    }
    __syncthreads();                                                    // (2)
    // the block's first max index; the largest weight before it; x_est candidate
    int64_t bi = s_mi[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) bi = s_mi[w] < bi ? s_mi[w] : bi;
    double pre = -1.0;
#pragma unroll
    for (int k = 0; k < kDeferPPT; ++k) {
        const int64_t i = base + kDeferPPT * t + k;
        if (i < bi) pre = fmax(pre, wv[k]);
        if (i == bi) {
            dp.pxe[0][blk] = xv[k];
            dp.pxe[1][blk] = yv[k];
            dp.pxe[2][blk] = tv[k];
        }
    }
    pre = wave_max_f64(pre);
    if (lane == 0) s_pre[wave] = pre;
    if (t < kQ * 16) {
        // quantity t / 16, segment t % 16: pairs seg, seg + 16, ..., seg + 112
        const double* a = s_q + (t >> 4) * 128 + (t & 15);
        double acc = a[0];
#pragma unroll
        for (int mm = 1; mm < 8; ++mm) acc = acc + a[16 * mm];
        s_seg[t] = acc;
    } else if (t >= 192 && t < 192 + 8 * kLeaves) {
        // leaf (t-192)>>3, accumulator k = t & 7: elements k, k+8, ..., k+120
        const double* a = s_w + ((t - 192) >> 3) * 128 + (t & 7);
        double acc = a[0];
#pragma unroll
        for (int mm = 1; mm < 16; ++mm) acc = acc + a[8 * mm];
        s_acc[t - 192] = acc;
    }
    __syncthreads();                                                    // (3)
    if (t < kQ) {
        double acc = s_seg[16 * t];
        for (int mm = 1; mm < 16; ++mm) acc = acc + s_seg[16 * t + mm];
        dp.ps[t][blk] = acc;
    } else if (t >= 64 && t < 128) {
        // the block's np.sum subtree: its kLeaves leaves, then their pair sums
        // (wave 1; lane l < kLeaves holds leaf l)
        double v = 0.0;
        if (t - 64 < kLeaves) {
            const double* r = s_acc + 8 * (t - 64);
            v = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        }
#pragma unroll
        for (int d = 1; d < kLeaves; d <<= 1) {
            const double o = xor_f64(v, d);
            v = (lane & d) ? (o + v) : (v + o);
        }
        if (t == 64) dp.leaf[blk] = v;
    } else if (t == 128) {
        dp.pmax[blk] = M;
        dp.pidx[blk] = bi;
        dp.ppre[blk] = fmax(fmax(s_pre[0], s_pre[1]), fmax(s_pre[2], s_pre[3]));
    }
}

// first j in [lo, hi) with c[j] >= pos, hi if none: the while loop of
// particle_filter.py:218-220 over the exact cumsum, restricted to a bracket
// known to hold the answer
__device__ __forceinline__ int64_t search_c(const double* __restrict__ c, int64_t lo, int64_t hi,
                                            const double pos) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (c[mid] < pos) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Predict one particle (particle_filter.py:129-140, :165-166; motion_model.py:
// 40-56) from its state and standard normals g, and give the likelihood the
// rotation of mylib/transform.py:31-33 for the predicted heading:
// ls = sin(pi/2 - th'), lc = cos(pi/2 - th').
//  * linear model: ls, lc from fast_sincos(pi/2 - th') exactly as the
//    reference forms them (the C1 parity path);
//  * velocity model: sin/cos(th + w dt) and sin/cos(th') by angle addition
//    from sin/cos(th) and the small turn increments w dt and gamma dt (two
//    kernel-only sin/cos instead of two range-reduced ones; within 2 ulp of
//    the direct evaluation).
// SLAM_TAB_SINCOS (default 1): the velocity model's sin/cos(th) from the LDS
// table (heading_sincos_tab) instead of fast_sincos.
#ifndef SLAM_TAB_SINCOS
#define SLAM_TAB_SINCOS 1
#endif
template <int MOTION>
__device__ __forceinline__ void predict_particle(const double x, const double y, const double th,
                                                 const double v, const double om, const double g0,
                                                 const double g1, const double g2,
                                                 const PredictConst& pc, double& xn, double& yn,
                                                 double& tn, double& ls, double& lc,
                                                 const RngTabs& T) {
    if (MOTION == kMotionNone) {           // likelihood-only entry (particle_filter.py:170)
        xn = x;
        yn = y;
        tn = th;
        fast_sincos(kHalfPi - tn, &ls, &lc);
    } else if (MOTION == SLAM_MOTION_LINEAR) {
        // particle_filter.py:129-140 then + v (:166); A = I, B = diag(V, V, w)
        double sn, cs;
        fast_sincos(th, &sn, &cs);
        const double a = pc.dt * cs;
        const double b = pc.dt * sn;
        xn = (x + v * a) + g0;
        yn = (y + v * b) + g1;
        tn = wrap_angle(th + om * pc.dt) + g2;
        fast_sincos(kHalfPi - tn, &ls, &lc);
    } else {
        // motion_model.py:40-56 (the std handed to normal() is sigma**2)
        const double v2 = v * v, w2 = om * om;
        const double sv = (pc.alphas[0] * v2) + (pc.alphas[1] * w2);
        const double sw = (pc.alphas[2] * v2) + (pc.alphas[3] * w2);
        const double sg = (pc.alphas[4] * v2) + (pc.alphas[5] * w2);
        const double vh = v + (0.0 + (sv * sv) * g0);
        const double wh = om + (0.0 + (sw * sw) * g1);
        const double gh = 0.0 + (sg * sg) * g2;
        const double a = vh / wh;
        const double b = wh * pc.dt;
        double s0, c0, sb, cb, s1, c1, se, ce;
#if SLAM_TAB_SINCOS
        heading_sincos_tab(th, T, &s0, &c0);
#else
        (void)T;
        fast_sincos(th, &s0, &c0);
#endif
        small_sincos(b, &sb, &cb);
        rotate_sc(s0, c0, sb, cb, &s1, &c1);                 // (th + w dt)
        xn = (x - (a * s0)) + (a * s1);
        yn = (y + (a * c0)) - (a * c1);
        tn = wrap_angle(th + (wh + gh) * pc.dt);
        small_sincos(gh * pc.dt, &se, &ce);
        rotate_sc(s1, c1, se, ce, &lc, &ls);                 // th' = th + w dt + gamma dt
    }
}

// double-double values (closed-form log-sum): explicit fma, -ffp-contract=off
struct dd_t {
    double h, l;
};
__device__ __forceinline__ dd_t dd_two_prod(const double a, const double b) {
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__device__ __forceinline__ dd_t dd_renorm(const double p, const double e) {
    const double r = p + e;
    return {r, e - (r - p)};
}
__device__ __forceinline__ dd_t dd_add2(const dd_t a, const dd_t b) {
    const double t = a.h + b.h;
    const double bb = t - a.h;
    return dd_renorm(t, ((a.h - (t - bb)) + (b.h - bb)) + (a.l + b.l));
}
__device__ __forceinline__ dd_t dd_mul_d(const dd_t a, const double b) {
    const double p = a.h * b;
    return dd_renorm(p, fma(a.h, b, -p) + a.l * b);
}
__device__ __forceinline__ dd_t dd_mul(const dd_t a, const dd_t b) {
    const double p = a.h * b.h;
    return dd_renorm(p, fma(a.h, b.h, -p) + (a.h * b.l + a.l * b.h));
}
__device__ __forceinline__ dd_t dd_scale(const dd_t a, const double p2) {   // p2 = +-2^k: exact
    return {a.h * p2, a.l * p2};
}
__device__ __forceinline__ dd_t dd_neg(const dd_t a) { return {-a.h, -a.l}; }

// ====================================================================
// per-step closed-form words (StepIO.zc slot, pf_kernels.hpp kZc*)
// ====================================================================
// Part 1 (every wave of a block, one sum per wave): the eight landmark /
// observation sums of the step as double-doubles in the fixed order of
// closed_lane_partial (64 lane partials, then a butterfly with the lower lane
// on the left), into sdd[16] (LDS).  The caller barriers before part 2.
__device__ void closed_prep_sums(const double* __restrict__ lm, const double* __restrict__ z,
                                 const int32_t nl, const int wave, const int nwaves, double* sdd) {
    const int lane = (int)__lane_id();
    for (int k = wave; k < 8; k += nwaves) {
        DDSum S = closed_lane_partial(k, lane, lm, z, nl);
#pragma unroll
        for (int d = 1; d < kClosedLanes; d <<= 1) {
            DDSum o;
            o.h = __shfl_xor(S.h, d, 64);
            o.l = __shfl_xor(S.l, d, 64);
            if ((lane & d) == 0) S = dd_join(S, o);
            else S = dd_join(o, S);
        }
        if (lane == 0) {
            sdd[2 * k] = S.h;
            sdd[2 * k + 1] = S.l;
        }
    }
}

// The expansion's reference pose for a step: the estimate two steps back (rp:
// x, y, th; refp[4..6] at the step's start, refp[0..2] at the previous step's
// end) moved `moves` times by the step's control, noise free (motion_model.py
// :64-86 / particle_filter.py:129-140): twice, or once for the first step after
// the handle's creation (refp[7] = 1: the initial pose is the particles' state
// before that step's predict).  Any finite pose gives exact constants; a close
// one keeps every particle on the fp64 expansion.
__device__ void closed_prep_reference(const double* rp, const int moves, const double v,
                                      const double om, const double dt, const int motion,
                                      double& px, double& py, double& pth) {
    px = rp[0];
    py = rp[1];
    pth = rp[2];
    if (!(isfinite(px) && isfinite(py) && fabs(pth) < 1e6)) px = py = pth = 0.0;
    for (int k = 0; k < moves; ++k) {
        double s0, c0;
        fast_sincos(pth, &s0, &c0);
        const double t1 = wrap_angle(pth + om * dt);
        const double a = v / om;
        if (motion == SLAM_MOTION_VELOCITY && om != 0.0 && isfinite(a)) {
            double s1, c1;
            fast_sincos(t1, &s1, &c1);
            px = (px - a * s0) + a * s1;
            py = (py + a * c0) - a * c1;
        } else if (isfinite(v)) {
            px = px + v * (dt * c0);
            py = py + v * (dt * s0);
        }
        if (isfinite(t1)) pth = t1;
    }
}

// Part 2 (one lane): the constants of the expansion about (p^, c^, s^) from the
// eight sums, each formed in double-double from the exact identities
//   l^ = l - p^:  L1 = S_l - NL p^,  L2 = S_ll - 2 p^.S_l + NL |p^|^2,
//   D^ = D - p^.S_z,  E^ = E - (p^_x S_zy - p^_y S_zx),
//   A = c^ L2 - D^,  B = s^ L2 - E^,  S_r = R^ L1 - S_z,
//   F^ = (c^^2 + s^^2) L2 - 2 (c^ D^ + s^ E^) + S_zz
// (F^ = sum_j |R^(l_j - p^) - z_j|^2, A = sum r^.l^, B = sum r^ x l^), then
// rounded (F^, A, B, L2 kept as double-doubles).
__device__ void closed_prep_constants(const double* sdd, const int32_t nl, const double px,
                                      const double py, const double pth, double* __restrict__ zc) {
    double sh, ch;
    fast_sincos(kHalfPi - pth, &sh, &ch);                 // mylib/transform.py:31
    const dd_t Sll{sdd[0], sdd[1]}, Slx{sdd[2], sdd[3]}, Sly{sdd[4], sdd[5]}, Szz{sdd[6], sdd[7]};
    const dd_t Szx{sdd[8], sdd[9]}, Szy{sdd[10], sdd[11]}, Dd{sdd[12], sdd[13]}, Ed{sdd[14], sdd[15]};
    const double fnl = (double)nl;
    const dd_t L1x = dd_add2(Slx, dd_neg(dd_two_prod(fnl, px)));
    const dd_t L1y = dd_add2(Sly, dd_neg(dd_two_prod(fnl, py)));
    const dd_t r2 = dd_add2(dd_two_prod(px, px), dd_two_prod(py, py));
    const dd_t t1 = dd_add2(dd_mul_d(Slx, px), dd_mul_d(Sly, py));
    const dd_t L2 = dd_add2(dd_add2(Sll, dd_scale(t1, -2.0)), dd_mul_d(r2, fnl));
    const dd_t Dh = dd_add2(Dd, dd_neg(dd_add2(dd_mul_d(Szx, px), dd_mul_d(Szy, py))));
    const dd_t Eh = dd_add2(Ed, dd_neg(dd_add2(dd_mul_d(Szy, px), dd_mul_d(Szx, -py))));
    const dd_t A = dd_add2(dd_mul_d(L2, ch), dd_neg(Dh));
    const dd_t B = dd_add2(dd_mul_d(L2, sh), dd_neg(Eh));
    const dd_t Srx = dd_add2(dd_add2(dd_mul_d(L1x, ch), dd_neg(dd_mul_d(L1y, sh))), dd_neg(Szx));
    const dd_t Sry = dd_add2(dd_add2(dd_mul_d(L1x, sh), dd_mul_d(L1y, ch)), dd_neg(Szy));
    const dd_t kk = dd_add2(dd_two_prod(ch, ch), dd_two_prod(sh, sh));
    const dd_t rr = dd_add2(dd_mul_d(Dh, ch), dd_mul_d(Eh, sh));
    const dd_t F = dd_add2(dd_add2(dd_mul(kk, L2), dd_scale(rr, -2.0)), Szz);
    for (int k = 0; k < 16; ++k) zc[kZcSum + k] = sdd[k];
    zc[kZcPx] = px;
    zc[kZcPy] = py;
    zc[kZcC] = ch;
    zc[kZcS] = sh;
    zc[kZcFh] = F.h;
    zc[kZcFl] = F.l;
    zc[kZcA] = A.h;
    zc[kZcAl] = A.l;
    zc[kZcB] = B.h;
    zc[kZcBl] = B.l;
    zc[kZcSrx] = Srx.h;
    zc[kZcSry] = Sry.h;
    zc[kZcL2] = L2.h;
    zc[kZcL2l] = L2.l;
    zc[kZcL1x] = L1x.h;
    zc[kZcL1y] = L1y.h;
}

// Both parts by one block (prestep / observation kernels): refp[4..6] = the
// estimate two steps back, refp[7] the moves from it (2; 1 after creation),
// (v, om) the step's control.
__device__ void closed_prep_block(const double* __restrict__ lm, const double* __restrict__ z,
                                  const int32_t nl, const double* refp, const double v,
                                  const double om, const double dt, const int motion,
                                  double* __restrict__ zc) {
    __shared__ double sdd[16];
    closed_prep_sums(lm, z, nl, (int)(threadIdx.x >> 6), (int)(blockDim.x >> 6), sdd);
    __syncthreads();
    if (threadIdx.x == 0) {
        double px, py, pth;
        closed_prep_reference(refp + 4, refp[7] == 1.0 ? 1 : 2, v, om, dt, motion, px, py, pth);
        closed_prep_constants(sdd, nl, px, py, pth, zc);
    }
}

// One landmark factor in the reference's rounding order
// (particle_filter.py:187-191: mylib/transform.py:31-35 then mlab.bivariate_normal).
template <int RHO = -1>
__device__ __forceinline__ double ref_q(const double xn, const double yn, const double sp,
                                        const double cp, const double lx, const double ly,
                                        const double zx, const double zy, const LikConst& lc);

// TAB: exp from the LDS table htab (product mode; exp_nhalf: the bits of
// exp_tab(-y/2), the table's values halved) instead of exp_lean.  Without
// rho, q >= 0 (a sum of two rounded non-negative quotients), so the argument
// is never positive.
// RHO: 1 / 0 when the caller has hoisted the lc.has_rho test out of its loop.
template <bool TAB = false, int RHO = -1>
__device__ __forceinline__ double ref_factor(const double xn, const double yn, const double sp,
                                             const double cp, const double lx, const double ly,
                                             const double zx, const double zy, const LikConst& lc,
                                             const double2* htab = nullptr) {
    const bool rho = RHO < 0 ? lc.has_rho : RHO > 0;
    const double q = ref_q<RHO>(xn, yn, sp, cp, lx, ly, zx, zy, lc);
    double e;
    if (rho) {
        const double a = (-q) / lc.d2;
        e = TAB ? exp_nhalf<false>(-2.0 * a, htab) : exp_lean(a);   // -2a exact: a's bits
    } else {
        e = TAB ? exp_nhalf<true>(q, htab) : exp_lean((-q) * 0.5);   // d2 == 2 exactly
    }
    return div_refined(e, lc.den, lc.rden);
}

// Log-sum slow path for one particle whose total L may leave the normal range
// somewhere along the reference's sequential product (particle_filter.py:192).
// Walk the log prefix s_j = log(f_1 ... f_j) to the first landmark j0 where it
// drops below ln(DBL_MIN) + 1: up to j0 - 1 the reference's partial product is
// a normal number equal to exp(s_{j0-1}); from j0 on, the factors are formed
// and multiplied exactly as the reference does (ref_factor), so the subnormal
// roundings and the zero set are the reference's.  Once the product is 0 it
// stays 0 (early exit).  The prefix uses the reference's residuals and q
// (ref_factor's rounding order) summed in double-double, so exp(s) is within
// ~1e-13 of the reference's normal-range partial product even for particles
// metres off every landmark (|s| ~ 700, where a plain fp64 chain of 100 sums
// is off by ~5e-12).
template <int RHO>
__device__ __forceinline__ double ref_q(const double xn, const double yn, const double sp,
                                        const double cp, const double lx, const double ly,
                                        const double zx, const double zy, const LikConst& lc) {
    const double dxw = lx - xn;
    const double dyw = ly - yn;
    const double rx = fma(-sp, dyw, cp * dxw);
    const double ry = fma(cp, dyw, sp * dxw);
    const double dx = rx - zx;
    const double dy = ry - zy;
    double q = div_refined(dx * dx, lc.sx2, lc.rsx2) + div_refined(dy * dy, lc.sy2, lc.rsy2);
    if (RHO < 0 ? lc.has_rho : RHO > 0) q = q - ((lc.rho2 * dx) * dy) / lc.sxsy;
    return q;
}

// double from/to lane l (uniform result, SGPR-held)
__device__ __forceinline__ double readlane_d(const double v, const int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// double-double a + b (TwoSum of the high parts, low parts added, renormalised)
__device__ __forceinline__ void dd_add(double& ah, double& al, const double bh, const double bl) {
    const double t = ah + bh;
    const double bb = t - ah;
    const double e = ((ah - (t - bb)) + (bh - bb)) + (al + bl);
    ah = t + e;
    al = e - (ah - t);
}

// One slow particle per WAVE (every lane passes the same particle): the log
// prefix of 64 landmarks at a time -- one ref_q per lane, a double-double
// inclusive wave scan plus the carry of the previous chunks -- then the first
// landmark j0 whose prefix leaves the normal range by ballot, and the exact
// tail from j0 (uniform across the wave).  A lane-serial walk of 100 landmarks
// is a ~10 us dependency chain; this one is a few hundred issue slots.
// inlined: a call costs the fused kernel 176 B of scratch and ~10 us per launch
#ifdef SLAM_SLOW_NOINLINE
#define SLAM_SLOW_ATTR __noinline__
#else
#define SLAM_SLOW_ATTR __forceinline__
#endif
__device__ SLAM_SLOW_ATTR double logsum_slow(const double xn, const double yn, const double sp,
                                           const double cp, const double* __restrict__ lm,
                                           const double* __restrict__ z, const LikConst& lc) {
    const int nl = lc.nl;
    const int lane = (int)__lane_id();
    double ch = 0.0, cl = 0.0;               // sum of q over the landmarks before this chunk
    double s_prev = 0.0;                     // log prefix before j0 (0: empty product = 1)
    int j0 = nl;
    for (int base = 0; base < nl; base += 64) {
        const int j = base + lane;
        double h = (j < nl) ? ref_q(xn, yn, sp, cp, lm[2 * j], lm[2 * j + 1], z[2 * j],
                                     z[2 * j + 1], lc)
                            : 0.0;
        double l = 0.0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {   // inclusive scan, lower lanes on the left
            const double oh = __shfl_up(h, d, 64), ol = __shfl_up(l, d, 64);
            if (lane >= d) {
                double th = oh, tl = ol;
                dd_add(th, tl, h, l);
                h = th;
                l = tl;
            }
        }
        double th = ch, tl = cl;
        dd_add(th, tl, h, l);                // + the previous chunks
        const double sq = th + tl;
        const double sj = lc.has_rho ? fma(-sq, lc.rd2, (double)(j + 1) * lc.neg_ln_den)
                                     : fma(-0.5, sq, (double)(j + 1) * lc.neg_ln_den);
        const unsigned long long below = __ballot(j < nl && !(sj >= lc.normal_min_l));
        if (below) {
            const int f = __ffsll((long long)below) - 1;     // first lane below
            const double sp_lane = __shfl(sj, f > 0 ? f - 1 : 0, 64);
            j0 = base + f;
            if (f > 0) s_prev = sp_lane;                     // else the previous chunk's last
            break;
        }
        const int last = (nl - base < 64 ? nl - base : 64) - 1;
        s_prev = __shfl(sj, last, 64);
        ch = __shfl(th, 63, 64);
        cl = __shfl(tl, 63, 64);
    }
    // the exact tail: the factors of 64 landmarks at a time, one per lane,
    // then the reference's left-to-right product over them (round 5: the
    // factors used to be formed inside the serial loop, ~60 issue slots per
    // landmark for the whole wave -- several us per slow particle)
    double acc = exp_lean(s_prev);           // s_prev = 0 -> exactly 1 (j0 = 0)
#ifdef SLAM_SLOW_SERIAL_TAIL                                 // A/B diagnostic: the round-4 form
    for (int j = j0; j < nl; ++j) {
        acc = acc * ref_factor(xn, yn, sp, cp, lm[2 * j], lm[2 * j + 1], z[2 * j], z[2 * j + 1], lc);
        if (acc == 0.0) break;
    }
    return acc;
#endif
    for (int base = j0; base < nl && acc != 0.0; base += 64) {
        const int j = base + lane;
        const double f = (j < nl) ? ref_factor(xn, yn, sp, cp, lm[2 * j], lm[2 * j + 1], z[2 * j],
                                               z[2 * j + 1], lc)
                                  : 1.0;
        const int cnt = (nl - base < 64) ? nl - base : 64;
        for (int l = 0; l < cnt; ++l) {
            acc = acc * readlane_d(f, l);
            if (acc == 0.0) break;
        }
    }
    return acc;
}

// Likelihood of P particles of one lane (particle_filter.py:170-192 with
// mylib/transform.py:31-35 per landmark).  The landmark loop is shared: each
// landmark and observation is loaded once (scalar loads, uniform across the
// wave) and applied to the P particles, whose accumulators are independent
// dependency chains.  sp/cp: sin/cos(pi/2 - th) of each particle.
//
// LOGSUM: prod_j exp(-q_j/d2)/den = exp(L), L = -sum_j q_j/d2 - NL ln den, one
// exp per particle.  Two accumulators per particle (the x and y squares) keep
// the rounding of the sum within ~5e-13 relative of the weight on the fast path
// (a single chain reaches 8e-13 at L ~ -650 and 5e-12 at L ~ -700).  A particle whose L is
// below lc.fast_min_l -- where some partial product of the reference's
// sequential loop could have left the normal range (subnormal or zero) --
// takes logsum_slow instead, so the zero set and the subnormal roundings are
// the reference's (identical zero sets, <= 1e-12 relative).
// Returns 1 when one of the lane's particles took the closed form's
// double-double evaluation.
template <int LIK, int P>
__device__ __forceinline__ int likelihood_lanes(const double* xn, const double* yn,
                                                 const double* sp, const double* cp,
                                                 const double* __restrict__ lm,
                                                 const double* __restrict__ z,
                                                 const double* __restrict__ zc, const LikConst& lc,
                                                 double* bn, const int wave_s, const double* pw) {
    const int nl = lc.nl;
    if (LIK == SLAM_LIK_PRODUCT) {
        // the exp table in LDS, t.x halved for exp_nhalf (every lane of the
        // block reaches this barrier)
        __shared__ double2 s_etab[64];
        if (threadIdx.x < 64) {
            const double2 t = kExpTab64[threadIdx.x];
            s_etab[threadIdx.x] = make_double2(t.x * 0.5, t.y);
        }
        __syncthreads();
        double acc[P];
#pragma unroll
        for (int k = 0; k < P; ++k) acc[k] = 1.0;
        // the rho test hoisted: the P particles' chains interleave in one block
        auto walk = [&](auto rho) {
            for (int j = 0; j < nl; ++j) {
                const double lx = lm[2 * j], ly = lm[2 * j + 1], zx = z[2 * j], zy = z[2 * j + 1];
#pragma unroll
                for (int k = 0; k < P; ++k)
                    acc[k] = acc[k] * ref_factor<true, decltype(rho)::value>(xn[k], yn[k], sp[k], cp[k], lx,
                                                                            ly, zx, zy, lc, s_etab);
            }
        };
        if (lc.has_rho) walk(std::integral_constant<int, 1>{});
        else walk(std::integral_constant<int, 0>{});
#pragma unroll
        for (int k = 0; k < P; ++k) bn[k] = acc[k];
        return 0;
    }
    double L[P];
    int lane_dd = 0;
    if (lc.closed) {
        // sum_j |R(l_j - p) - z_j|^2 in closed form (iso: q_j = that / sx2).
        // Fast form: the expansion about the step's reference pose (p^, c^, s^),
        // exact as a polynomial identity for any particle (x, y, c, s):
        //   d = p - p^, dc = c - c^, ds = s - s^, (u, v) = R(c, s) d,
        //   F = F^ + 2 (dc A + ds B) + (dc^2 + ds^2) L2            [rotation terms]
        //          - 2 S_r.(u, v) - 2 (dR L1).(u, v) + NL (u^2 + v^2),  dR = [[dc, -ds], [ds, dc]]
        // (DESIGN 4.3).  The rotation terms, which carry the cloud's heading
        // spread (|dc A| and dc^2 L2 reach ~10 while F ~ NL sx2), are formed to
        // ~u^2 from double-double dc, ds (TwoSum) and A, B, L2 (exact products,
        // TwoSum) and summed with F^ in double-double; the translation terms
        // round in fp64 within 11 u V, V = 2 (|gx u| + |gy v| + |Srx u| +
        // |Sry v|) + t5 their magnitudes, so V <= expand_vmax keeps |dL| <=
        // 3e-13 (the worst case; the measured difference to the double-double
        // form is ~1e-14).  Beyond it (a particle far from the reference pose) the
        // double-double form of the same sum from the eight sums.  Either way
        // the exact value of the sum for the particle's rounded c, s up to that
        // bound and one final rounding: the difference to the reference is its
        // own rounding (~1e-14 relative of the weight).
        const double fnl = (double)nl;
        const double phx = zc[kZcPx], phy = zc[kZcPy], chh = zc[kZcC], shh = zc[kZcS];
        const double Fh = zc[kZcFh], Fl = zc[kZcFl];
        const double Ah = zc[kZcA], Al = zc[kZcAl], Bh = zc[kZcB], Bl = zc[kZcBl];
        const double L2h = zc[kZcL2], L2l = zc[kZcL2l];
        const double Srx = zc[kZcSrx], Sry = zc[kZcSry];
        const double L1x = zc[kZcL1x], L1y = zc[kZcL1y];
        bool dd[P];
        int any_dd = 0;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const double c = cp[k], sn = sp[k];
            const double dx = xn[k] - phx, dy = yn[k] - phy;
            const double dc = c - chh, ds = sn - shh;
            const double dcb = dc - c, dsb = ds - sn;                       // TwoSum errors of dc, ds
            const double dce = (c - (dc - dcb)) + (-chh - dcb);
            const double dse = (sn - (ds - dsb)) + (-shh - dsb);
            // rotation terms to ~u^2: 2 t1 = 2 (dc A + ds B), t3 = (dc^2 + ds^2) L2
            const double p1 = dc * Ah, e1 = fma(dc, Ah, -p1);
            const double p2 = ds * Bh, e2 = fma(ds, Bh, -p2);
            const double q1 = dc * dc, f1 = fma(dc, dc, -q1);
            const double q2 = ds * ds, f2 = fma(ds, ds, -q2);
            const double a2 = q1 + q2;
            const double a2b = a2 - q1;
            const double a2e = ((q1 - (a2 - a2b)) + (q2 - a2b)) + (f1 + f2);
            const double p3 = a2 * L2h;
            // + the low parts of dc, ds: 2 (dce dc + dse ds) in t3, (dce A + dse B) in t1
            const double a2x = a2e + 2.0 * fma(dce, dc, dse * ds);
            const double e3 = fma(a2, L2h, -p3) + fma(a2x, L2h, a2 * L2l);
            // translation terms in fp64: t2 = S_r . R d, t4 = dR L1 . R d, t5 = NL |R d|^2
            const double u = fma(c, dx, -(sn * dy));
            const double v = fma(sn, dx, c * dy);
            const double t2 = fma(Srx, u, Sry * v);
            const double gx = fma(dc, L1x, -(ds * L1y)), gy = fma(ds, L1x, dc * L1y);
            const double t4 = fma(gx, u, gy * v);
            const double t5 = fma(u, u, v * v) * fnl;
            // F^h + 2 p1 + 2 p2 + p3 by TwoSum, then every low part
            double h = Fh, lo;
            {
                const double b = 2.0 * p1, t = h + b, bb = t - h;
                lo = (h - (t - bb)) + (b - bb);
                h = t;
            }
            {
                const double b = 2.0 * p2, t = h + b, bb = t - h;
                lo += (h - (t - bb)) + (b - bb);
                h = t;
            }
            {
                const double t = h + p3, bb = t - h;
                lo += (h - (t - bb)) + (p3 - bb);
                h = t;
            }
            const double rot_lo =
                fma(2.0, (e1 + e2) + (fma(dc, Al, ds * Bl) + fma(dce, Ah, dse * Bh)), e3);
            lo = lo + ((Fl + rot_lo) + (fma(-2.0, t2 + t4, t5)));
            const double F = h + lo;
            const double V = fma(2.0, fma(fabs(u), fabs(gx) + fabs(Srx), fabs(v) * (fabs(gy) + fabs(Sry))), t5);
            dd[k] = !(V <= lc.expand_vmax);                                  // also NaN
            any_dd |= dd[k] ? 1 : 0;
            L[k] = nl ? fma(-0.5, F * lc.rsx2, lc.neg_nl_ln_den) : lc.neg_nl_ln_den;
        }
        lane_dd = any_dd;
        if (any_dd) {
            const dd_t Sll{zc[0], zc[1]}, Slx{zc[2], zc[3]}, Sly{zc[4], zc[5]}, Szz{zc[6], zc[7]};
            const dd_t Szx{zc[8], zc[9]}, Szy{zc[10], zc[11]}, Dd{zc[12], zc[13]}, Ed{zc[14], zc[15]};
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (!dd[k]) continue;
                const double x = xn[k], y = yn[k], c = cp[k], sn = sp[k];
                const dd_t r2 = dd_add2(dd_two_prod(x, x), dd_two_prod(y, y));          // |p|^2
                const dd_t t1 = dd_add2(dd_mul_d(Slx, x), dd_mul_d(Sly, y));            // p . S_l
                const dd_t p1 = dd_add2(dd_add2(Sll, dd_scale(t1, -2.0)), dd_mul_d(r2, fnl));
                const dd_t kk = dd_add2(dd_two_prod(c, c), dd_two_prod(sn, sn));
                const dd_t q1 = dd_add2(Dd, dd_scale(dd_add2(dd_mul_d(Szx, x), dd_mul_d(Szy, y)), -1.0));
                const dd_t q2 = dd_add2(Ed, dd_scale(dd_add2(dd_mul_d(Szy, x), dd_mul_d(Szx, -y)), -1.0));
                const dd_t rr = dd_add2(dd_mul_d(q1, c), dd_mul_d(q2, sn));
                const dd_t acc = dd_add2(dd_add2(dd_mul(kk, p1), dd_scale(rr, -2.0)), Szz);
                L[k] = nl ? fma(-0.5, acc.h * lc.rsx2, lc.neg_nl_ln_den) : lc.neg_nl_ln_den;
            }
        }
    } else if (lc.iso) {
        double a[P][2];
#pragma unroll
        for (int k = 0; k < P; ++k) a[k][0] = a[k][1] = 0.0;
#pragma unroll 4
        for (int j = 0; j < nl; ++j) {
            const double lx = lm[2 * j], ly = lm[2 * j + 1], zx = z[2 * j], zy = z[2 * j + 1];
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const double dxw = lx - xn[k];
                const double dyw = ly - yn[k];
                const double dx = fma(cp[k], dxw, fma(-sp[k], dyw, -zx));
                const double dy = fma(sp[k], dxw, fma(cp[k], dyw, -zy));
                a[k][0] = fma(dx, dx, a[k][0]);
                a[k][1] = fma(dy, dy, a[k][1]);
            }
        }
#pragma unroll
        for (int k = 0; k < P; ++k) L[k] = fma(-0.5, (a[k][0] + a[k][1]) * lc.rsx2, lc.neg_nl_ln_den);
    } else {
        double a[P][2];
#pragma unroll
        for (int k = 0; k < P; ++k) a[k][0] = a[k][1] = 0.0;
        for (int j = 0; j < nl; j += 2) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (j + h >= nl) break;
                const double lx = lm[2 * (j + h)], ly = lm[2 * (j + h) + 1];
                const double zx = z[2 * (j + h)], zy = z[2 * (j + h) + 1];
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    const double dxw = lx - xn[k];
                    const double dyw = ly - yn[k];
                    const double dx = fma(cp[k], dxw, fma(-sp[k], dyw, -zx));
                    const double dy = fma(sp[k], dxw, fma(cp[k], dyw, -zy));
                    double q = fma(dx * lc.rsx2, dx, (dy * lc.rsy2) * dy);
                    if (lc.has_rho) q = q - ((lc.rho2 * dx) * dy) * lc.rsxsy;
                    a[k][h] = a[k][h] + q;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const double s = a[k][0] + a[k][1];
            L[k] = lc.has_rho ? fma(-s, lc.rd2, lc.neg_nl_ln_den) : fma(-0.5, s, lc.neg_nl_ln_den);
        }
    }
    bool slow[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        bn[k] = exp_lean(L[k]);
        slow[k] = !(L[k] >= lc.fast_min_l);                 // also NaN
        // a zero previous weight makes the weight 0 for any finite likelihood,
        // and below fast_min_l the likelihood is finite (a NaN L still goes
        // the reference's way): the exact product is not needed
#ifndef SLAM_NO_ZERO_SKIP                                   // A/B diagnostic
        if (slow[k] && pw[k] == 0.0 && !isnan(L[k])) {
            slow[k] = false;
            bn[k] = 0.0;
        }
#endif
#ifdef SLAM_PROBE_NO_SLOW                                  // timing probe only: not exact
        slow[k] = false;
#endif
    }
    // The few slow particles (bench workload: ~1,500 of 2^20 on every third
    // step, ~100 on the step after) are taken by their own wave, one at a
    // time with all 64 lanes on it: no block barrier and no LDS staging, so a
    // wave without one pays two ballots.  Wave-uniform loops.
#pragma unroll
    for (int k = 0; k < P; ++k) {
        unsigned long long m = __ballot(slow[k]);
#ifdef SLAM_PROBE_COUNT_SLOW                               // probe builds only
        if (__lane_id() == 0 && m) {
            atomicAdd(&g_probe_slow[0], (unsigned long long)__popcll(m));
            atomicAdd(&g_probe_slow[1], 1ull);
        }
#endif
        while (m) {
            const int l = __ffsll((long long)m) - 1;
            m &= m - 1;
            const double r = logsum_slow(__shfl(xn[k], l, 64), __shfl(yn[k], l, 64),
                                         __shfl(sp[k], l, 64), __shfl(cp[k], l, 64), lm, z, lc);
            if ((int)__lane_id() == l) bn[k] = r;
        }
    }
    return lane_dd;
}

// The fused step kernel: [resample gather +] predict + likelihood + weight.
// DEFER = false (shards): one particle per lane, previous weights normalised
// in w_in.  DEFER = true (single GPU, gbase = 0, particle arrays padded to
// whole blocks): lane t of block b holds the consecutive particles
// b kPartPer + kDeferPPT t + k -- 16-byte loads and stores, one device-RNG
// pair per lane -- and the previous weights are w_un / s (read and rewritten
// in place), followed by the block epilogue that replaces the normalise pass.
// Four waves per SIMD (<= 128 VGPRs): the log-sum kernel's slow-path product
// would otherwise push it to 129 and three waves.
#ifndef SLAM_FUSED_WPE
#define SLAM_FUSED_WPE 4
#endif
#if SLAM_FUSED_WPE > 0
#define SLAM_FUSED_ATTR __attribute__((amdgpu_waves_per_eu(SLAM_FUSED_WPE)))
#else
#define SLAM_FUSED_ATTR
#endif
// One fused block's tile (blk: 256 lanes x P particles): the body of
// pf_fused_kernel (a persistent grid walking tiles measured slower: DESIGN 4.4).
template <int MOTION, int LIK, bool HOSTNOISE, bool DEFER>
__device__ __forceinline__ void pf_fused_tile(
    const int64_t blk, const int32_t st, const uint32_t rstep, const int32_t rflag,
    const double* __restrict__ zs, const int wave_s, const RngTabs& rtab,
    const int64_t n, const double* __restrict__ xs, const double* __restrict__ ys,
    const double* __restrict__ ts, double* __restrict__ xo, double* __restrict__ yo,
    double* __restrict__ to, const double* __restrict__ w_in, double* __restrict__ w_un,
    const double* __restrict__ c, int32_t* __restrict__ flags, const double* __restrict__ noise,
    const double* __restrict__ lm, const StepIO& io, const PredictConst& pc, const LikConst& lc,
    const uint64_t seed, const double* __restrict__ s_in, const double* __restrict__ refp,
    const DeferParts& dp) {
    constexpr int P = DEFER ? kDeferPPT : 1;
    const int64_t base = blk * (256 * P);
    const int64_t i0 = base + P * (int64_t)threadIdx.x;
    bool valid[P];
    int64_t idx[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        valid[k] = i0 + k < n;
        idx[k] = valid[k] ? i0 + k : n - 1;
    }

    // ---- every load of the lane first (the previous weights and, without a
    //      resample gather, the particle pair), so that their latency runs
    //      under the device RNG below; the weights are consumed at the end
    double wprev[P];
    double lx[P], ly[P], lt[P];
    if (DEFER) {
#pragma unroll
        for (int h = 0; h < P; h += 2) {
            const double2 wu = *reinterpret_cast<const double2*>(w_un + i0 + h);
            wprev[h] = wu.x;
            wprev[h + 1] = wu.y;
        }
        if (rflag != 1) {
#pragma unroll
            for (int h = 0; h < P; h += 2) {
                const double2 a = *reinterpret_cast<const double2*>(xs + i0 + h);
                const double2 b = *reinterpret_cast<const double2*>(ys + i0 + h);
                const double2 c2 = *reinterpret_cast<const double2*>(ts + i0 + h);
                lx[h] = a.x;
                lx[h + 1] = a.y;
                ly[h] = b.x;
                ly[h + 1] = b.y;
                lt[h] = c2.x;
                lt[h + 1] = c2.y;
            }
        }
    } else {
        wprev[0] = w_in[idx[0]];
    }
    // host / pre-drawn noise of the lane's particles (particle-major [n][3]):
    // three 16-byte loads per pair, issued with the others
    double gn[P][3];
    if (HOSTNOISE && MOTION != kMotionNone) {
        if (DEFER && i0 + P <= n) {
#pragma unroll
            for (int h = 0; h < P; h += 2) {
                const double2* q2 = reinterpret_cast<const double2*>(noise + 3 * (i0 + h));
                const double2 a = q2[0], b = q2[1], c3 = q2[2];
                gn[h][0] = a.x;
                gn[h][1] = a.y;
                gn[h][2] = b.x;
                gn[h + 1][0] = b.y;
                gn[h + 1][1] = c3.x;
                gn[h + 1][2] = c3.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k)
#pragma unroll
                for (int j = 0; j < 3; ++j) gn[k][j] = noise[3 * idx[k] + j];
        }
    }

    // ---- source particles: the resample gather (rflag 1: search the exact
    //      cumsum here; 2: already gathered) or the particles themselves
    double x[P], y[P], th[P];
    if (DEFER && rflag == 1 && !flags[kFlagFallback]) {
        // the expand pass's inverse map: run starts in mark[], the block's
        // first source in carry[]; a running max over the block's positions
        __shared__ int32_t s_wmax[4];
        const uint32_t mgen = (uint32_t)flags[kFlagMarkGen];
        int32_t r[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int64_t mk = valid[k] ? dp.mark[i0 + k] : -1;
            r[k] = ((uint64_t)mk >> 32) == mgen ? (int32_t)mk : -1;
            if (k > 0) r[k] = r[k] > r[k - 1] ? r[k] : r[k - 1];
        }
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        int32_t before;
        const int32_t v = wave_max_scan_i32(r[P - 1], before);
        if (lane == 63) s_wmax[wave] = v;
        __syncthreads();
        int32_t run = dp.carry[blk];
        for (int w = 0; w < wave; ++w) run = s_wmax[w] > run ? s_wmax[w] : run;
        run = before > run ? before : run;
        const double* gx = xs - dp.goff;                         // the gather base
        const double* gy = ys - dp.goff;
        const double* gt = ts - dp.goff;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            int64_t src = r[k] > run ? r[k] : run;
            if (src >= dp.glim) {
                src = dp.goff + n - 1;                           // IndexError in the reference
                if (valid[k]) atomicOr(&flags[kFlagStatus], 1);
            }
            src = src < 0 ? 0 : src;
            x[k] = gx[src];
            y[k] = gy[src];
            th[k] = gt[src];
        }
    } else if (rflag == 1) {
        // bracket: the sources of the block's first and last positions (two
        // lanes of different waves search the whole cumsum); every lane then
        // searches only between them (the index map is monotone), a few
        // probes when the weight is concentrated -- which it is whenever
        // ESS < NP/100 triggered the resample
        __shared__ int64_t s_br[2];
        const double ofs = resample_offset(io.ofs[st], pc.np_recip, seed, rstep);
        const int64_t ilast = (base + 256 * P < n ? base + 256 * P : n) - 1;
        if (threadIdx.x == 0) s_br[0] = search_c(c, 0, n, (double)base * pc.rstep + ofs);
        if (threadIdx.x == 64 || (blockDim.x <= 64 && threadIdx.x == 0))
            s_br[1] = search_c(c, 0, n, (double)ilast * pc.rstep + ofs);
        __syncthreads();
        int64_t lo = s_br[0];
        const int64_t hi = s_br[1] < n ? s_br[1] + 1 : n;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            int64_t src = search_c(c, lo, hi, (double)idx[k] * pc.rstep + ofs);   // arange value + ofs
            lo = src;
            if (src >= n) {
                src = n - 1;                                     // IndexError in the reference
                if (valid[k]) atomicOr(&flags[kFlagStatus], 1);
            }
            x[k] = xs[src];
            y[k] = ys[src];
            th[k] = ts[src];
        }
    } else if (DEFER) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            x[k] = lx[k];
            y[k] = ly[k];
            th[k] = lt[k];
        }
    } else {
        x[0] = xs[idx[0]];
        y[0] = ys[idx[0]];
        th[0] = ts[idx[0]];
    }

    // ---- standard normals of the motion noise
    double g[P][3];
    if (MOTION == kMotionNone) {
#pragma unroll
        for (int k = 0; k < P; ++k) g[k][0] = g[k][1] = g[k][2] = 0.0;
    } else if (HOSTNOISE) {
#pragma unroll
        for (int k = 0; k < P; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) g[k][j] = gn[k][j];
    } else {
        const uint64_t gi = (uint64_t)(pc.gbase + i0);
        double h[6];
        if (DEFER) {                                          // gi even: whole pairs
#pragma unroll
            for (int pr = 0; pr < P / 2; ++pr) {
#ifdef SLAM_PROBE_NO_RNG                                      // instruction-count probe only
                for (int j = 0; j < 6; ++j) h[j] = 0.0;
#else
                pair_normals((gi >> 1) + pr, rstep, seed, rtab, h);
#endif
#pragma unroll
                for (int j = 0; j < 6; ++j) g[2 * pr + j / 3][j % 3] = h[j];
            }
        } else {
            pair_normals(gi >> 1, rstep, seed, rtab, h);
            const bool odd = gi & 1;
#pragma unroll
            for (int j = 0; j < 3; ++j) g[0][j] = odd ? h[3 + j] : h[j];
        }
        if (MOTION == SLAM_MOTION_LINEAR) {                   // noise_j = sum_k g_k q[k][j]
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const double h0 = g[k][0], h1 = g[k][1], h2 = g[k][2];
                g[k][0] = h0 * pc.q[0] + h1 * pc.q[3] + h2 * pc.q[6];
                g[k][1] = h0 * pc.q[1] + h1 * pc.q[4] + h2 * pc.q[7];
                g[k][2] = h0 * pc.q[2] + h1 * pc.q[5] + h2 * pc.q[8];
            }
        }
    }

    FPROBE(2, g[P - 1][2]);
    // ---- predict (control of this step: particle_filter.py:46-58 / motion_model.py:40-45)
    const double v = io.ctl[2 * st], om = io.ctl[2 * st + 1];
    double xv[P], yv[P], tv[P], sp[P], cp[P];
#pragma unroll
    for (int k = 0; k < P; ++k)
        predict_particle<MOTION>(x[k], y[k], th[k], v, om, g[k][0], g[k][1], g[k][2], pc, xv[k],
                                 yv[k], tv[k], sp[k], cp[k], rtab);
    if (DEFER) {                       // padded arrays: the pair is stored whole
#pragma unroll
        for (int h = 0; h < P; h += 2) {
            *reinterpret_cast<double2*>(xo + i0 + h) = double2{xv[h], xv[h + 1]};
            *reinterpret_cast<double2*>(yo + i0 + h) = double2{yv[h], yv[h + 1]};
            *reinterpret_cast<double2*>(to + i0 + h) = double2{tv[h], tv[h + 1]};
        }
    } else if (valid[0]) {
        xo[i0] = xv[0];
        yo[i0] = yv[0];
        to[i0] = tv[0];
    }

    FPROBE(3, xv[P - 1] + sp[P - 1]);
    // previous weights: particle_filter.py:222 (a resampled step starts from
    // 1/NP) / :235-236 (deferred: w_un / s, NaN -> 1/NP)
    double pw[P];
    const double s_prev = DEFER ? *s_in : 1.0;
#pragma unroll
    for (int k = 0; k < P; ++k)
        pw[k] = rflag ? pc.np_recip : (DEFER ? norm_w(wprev[k], s_prev, pc.np_recip) : wprev[k]);
    // ---- likelihood and weight (particle_filter.py:170-198)
    double bn[P];
#ifdef SLAM_PROBE_NO_LIK                                   // timing probe only: not exact
#pragma unroll
    for (int k = 0; k < P; ++k) bn[k] = exp_lean(-1e-3 * (xv[k] + yv[k] + sp[k] + cp[k]));
    const int lane_dd = 0;
#else
    const int lane_dd = likelihood_lanes<LIK, P>(xv, yv, sp, cp, lm, zs,
                                                 io.zc + (size_t)st * kZcWords, lc, bn, wave_s, pw);
#endif
    FPROBE(4, bn[P - 1]);
    if (__ballot(lane_dd) != 0 && __lane_id() == 0) atomicAdd(&flags[kFlagDDWaves], 1);
    double wv[P];
#pragma unroll
    for (int k = 0; k < P; ++k) wv[k] = valid[k] ? pw[k] * bn[k] : 0.0;   // particle_filter.py:194
    if constexpr (DEFER) {
#pragma unroll
        for (int h = 0; h < P; h += 2)
            *reinterpret_cast<double2*>(w_un + i0 + h) = double2{wv[h], wv[h + 1]};
#ifndef SLAM_NO_EPILOGUE
        defer_epilogue(base, n, wv, xv, yv, tv, refp, dp, wave_s, (int)blk);
#endif
        FPROBE(5, wv[0]);
    } else if (valid[0]) {
        w_un[i0] = wv[0];
    }
}

// The step's first fused block, after its own particles: the NEXT step's
// closed-form words (StepIO.zc) -- its eight sums (two per wave)
// and its expansion about this step's refp (the estimate two steps before it)
// moved twice.  Off the step's critical path: the next launch reads them; a
// step staged by the host is prepared again by its prestep.
template <int MOTION>
__device__ __forceinline__ void pf_fused_prep_next(const int32_t st, const int wave_s,
                                                   const double* __restrict__ lm,
                                                   const StepIO& io, const PredictConst& pc,
                                                   const LikConst& lc,
                                                   const double* __restrict__ refp) {
    if (MOTION != kMotionNone && lc.closed && blockIdx.x == 0 && st + 1 < io.cap) {
        __shared__ double s_prep[16];
        const int32_t sn = st + 1;
        closed_prep_sums(lm, io.z + (size_t)sn * 2 * lc.nl, lc.nl, wave_s, 4, s_prep);
        __syncthreads();
        if (threadIdx.x == 0) {
            double px, py, pth;
            closed_prep_reference(refp, 2, io.ctl[2 * sn], io.ctl[2 * sn + 1], pc.dt, io.motion,
                                  px, py, pth);
            closed_prep_constants(s_prep, lc.nl, px, py, pth, io.zc + (size_t)sn * kZcWords);
        }
    }
}

#define SLAM_FUSED_PARAMS                                                                          \
    const int64_t n, const double* __restrict__ xs, const double* __restrict__ ys,                  \
        const double* __restrict__ ts, double* __restrict__ xo, double* __restrict__ yo,            \
        double* __restrict__ to, const double* __restrict__ w_in, double* __restrict__ w_un,        \
        const double* __restrict__ c, int32_t* __restrict__ flags,                                  \
        const double* __restrict__ noise, const double* __restrict__ lm, StepIO io,                 \
        PredictConst pc, LikConst lc, uint64_t seed, const double* __restrict__ s_in,               \
        const double* __restrict__ refp, DeferParts dp
#define SLAM_FUSED_ARGS n, xs, ys, ts, xo, yo, to, w_in, w_un, c, flags, noise, lm, io, pc, lc, \
                        seed, s_in, refp, dp

// The step's uniform inputs and the RNG tables (every lane reaches the barrier)
#define SLAM_FUSED_PROLOGUE                                                                      \
    const int32_t st = io.ctr[0];                                                                \
    const uint32_t rstep = (uint32_t)io.ctr[1];                                                  \
    const int32_t rflag = flags[kFlagResample];                                                  \
    const double* __restrict__ zs = io.z + (size_t)st * 2 * (size_t)(lc.nl > 0 ? lc.nl : 1);     \
    const int wave_s = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);                    \
    __shared__ RngTabsLds s_rng;                                                                 \
    RngTabs rtab{};                                                                              \
    if constexpr ((MOTION != kMotionNone && !HOSTNOISE) ||                                      \
                  (MOTION == SLAM_MOTION_VELOCITY && SLAM_TAB_SINCOS)) {                         \
        rtab = rng_tabs_stage(&s_rng, (int)threadIdx.x, 256);                                    \
        __syncthreads();                                                                         \
    }

template <int MOTION, int LIK, bool HOSTNOISE, bool DEFER>
__global__ __launch_bounds__(256) SLAM_FUSED_ATTR void pf_fused_kernel(SLAM_FUSED_PARAMS) {
    static_assert(!DEFER || kDeferPPT % 2 == 0, "the deferred path moves particle pairs");
    SLAM_FUSED_PROLOGUE
    pf_fused_tile<MOTION, LIK, HOSTNOISE, DEFER>(blockIdx.x, st, rstep, rflag, zs, wave_s, rtab,
                                                 SLAM_FUSED_ARGS);
    if constexpr (DEFER) pf_fused_prep_next<MOTION>(st, wave_s, lm, io, pc, lc, refp);
}

// ====================================================================
// numpy-order chunk sums (np.sum: 8192-element buffers, pairwise inside)
// ====================================================================
// Full chunk: 512 threads = 64 leaves x 8 accumulators; accumulator k of leaf
// L sums elements L*128 + k + 8m (m = 0..15) left to right; leaves combine as
// a perfect binary tree, which the xor-butterfly reproduces exactly.
// Tail chunk (< 8192): host-built leaf table + post-order combine program.
// With s_out != null the last block folds the partials left to right.
__global__ __launch_bounds__(512) void chunk_sum_kernel(
    const double* __restrict__ w, const int64_t n, double* __restrict__ part,
    const int32_t* __restrict__ tail_leaves, const int32_t* __restrict__ tail_ops,
    const int32_t n_tail_leaves, const int32_t n_tail_ops, unsigned* __restrict__ counter,
    double* __restrict__ s_out) {
    __shared__ double sh[1024];
    const int64_t base = (int64_t)blockIdx.x * kSumChunk;
    const int64_t len = (n - base < kSumChunk) ? (n - base) : kSumChunk;
    const int t = threadIdx.x;
    double blk = 0.0;
    if (len == kSumChunk) {
        const int leaf = t >> 3, k = t & 7;
        const double* p = w + base + leaf * 128 + k;
        double r = p[0];
#pragma unroll
        for (int m = 1; m < 16; ++m) r = r + p[8 * m];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) r = r + __shfl_xor(r, d, 64);
        if ((t & 63) == 0) sh[t >> 6] = r;
        __syncthreads();
        if (t == 0) blk = ((sh[0] + sh[1]) + (sh[2] + sh[3])) + ((sh[4] + sh[5]) + (sh[6] + sh[7]));
    } else {
        // tail: leaves of <= 128 elements, one per thread
        for (int L = t; L < n_tail_leaves; L += blockDim.x) {
            const int lo = tail_leaves[2 * L], cnt = tail_leaves[2 * L + 1];
            const double* a = w + base + lo;
            double res;
            if (cnt < 8) {
                res = 0.0;
                for (int i = 0; i < cnt; ++i) res = res + a[i];
            } else {
                double r[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) r[k] = a[k];
                int i = 8;
                const int stop = cnt - (cnt % 8);
                for (; i < stop; i += 8) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) r[k] = r[k] + a[i + k];
                }
                res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < cnt; ++i) res = res + a[i];
            }
            sh[L] = res;
        }
        __syncthreads();
        if (t == 0) {
            double stk[16];
            int sp = 0;
            for (int o = 0; o < n_tail_ops; ++o) {
                const int op = tail_ops[o];
                if (op >= 0) {
                    stk[sp++] = sh[op];
                } else {
                    const double b = stk[--sp];
                    const double a = stk[--sp];
                    stk[sp++] = a + b;
                }
            }
            blk = stk[0];
        }
    }
    if (t == 0) st_wt_d(&part[blockIdx.x], blk);
    if (!s_out) return;
    if (!arrive_last(counter)) return;
    double s = 0.0;                                   // buffer partials left to right
    const int nc = gridDim.x;
    for (int c0 = 0; c0 < nc; c0 += 1024) {
        const int cnt = min(1024, nc - c0);
        __syncthreads();
        for (int k = t; k < cnt; k += blockDim.x) sh[k] = ld_wt_d(&part[c0 + k]);
        __syncthreads();
        if (t == 0)
            for (int k = 0; k < cnt; ++k) s = s + sh[k];
    }
    if (t == 0) *s_out = s;
}

// exclusive scan of a small per-block array (write-through words) by one block
template <typename T, int NT>
__device__ void block_scan_array(const T* in, T* out, const int nb, T* total, T* sh,
                                 const bool wt = false) {
    const int per = (nb + NT - 1) / NT;
    const int b0 = threadIdx.x * per;
    auto ld = [](const T* p) -> T {
        if constexpr (sizeof(T) == 8) {
            const uint64_t u = ld_wt(p);
            T v;
            __builtin_memcpy(&v, &u, 8);
            return v;
        } else {
            return (T)ld_wt_i((const int32_t*)p);
        }
    };
    // up to kMaxPer words per thread stay in registers between the two passes
    // (one memory round trip instead of two)
    constexpr int kMaxPer = 8;
    const bool cached = per <= kMaxPer;
    T cv[kMaxPer];
    T loc = T(0);
    if (cached) {
#pragma unroll
        for (int k = 0; k < kMaxPer; ++k) {
            cv[k] = (k < per && b0 + k < nb) ? ld(in + b0 + k) : T(0);
            loc = loc + cv[k];
        }
    } else {
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) loc = loc + ld(in + b0 + k);
    }
    T tot;
    T ex = block_excl_scan<T, NT>(loc, sh, tot);
    auto st = [wt](T* p, const T v) {
        if (!wt) {
            *p = v;
        } else if constexpr (sizeof(T) == 8) {
            uint64_t u;
            __builtin_memcpy(&u, &v, 8);
            st_wt(p, u);
        } else {
            st_wt_i((int32_t*)p, (int32_t)v);
        }
    };
    if (cached) {
#pragma unroll
        for (int k = 0; k < kMaxPer; ++k)
            if (k < per && b0 + k < nb) {
                st(out + b0 + k, ex);
                ex = ex + cv[k];
            }
    } else {
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) {
                const T v = ld(in + b0 + k);
                st(out + b0 + k, ex);
                ex = ex + v;
            }
    }
    if (threadIdx.x == 0 && total) st(total, tot);
}

// The two tile-total scans of the exact cumsum (increments k: u64, special
// counts f: i32) with both arrays' loads issued together (one memory round
// trip for both); the same sums as two block_scan_array calls.
template <int NT, int kC = 8>
__device__ __forceinline__ void block_scan_pair(const uint64_t* kin, uint64_t* kout, uint64_t* ktotal,
                                const int32_t* fin, int32_t* fout, int32_t* ftotal, const int nb,
                                uint64_t* shk, int32_t* shf, int32_t* f_lds = nullptr) {
    // Up to two entries per thread: thread-contiguous, in registers, one
    // block scan per array.  Beyond, coalesced: wave w owns the contiguous
    // span [w*span, (w+1)*span) and walks it in rounds of 64 consecutive
    // entries (one per lane), kC rounds' loads in flight; each round is a DPP
    // wave scan.  (The thread-contiguous layout touches one cache line per
    // lane per access: 17-27 us for the 4,096 tile totals of NP = 2^23 in one
    // CU, against 7 us here.)
    constexpr int W = NT / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (nb <= 2 * NT) {
        const int b0 = 2 * threadIdx.x;
        uint64_t k2[2];
        int32_t f2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool ok = b0 + k < nb;
            k2[k] = ok ? ld_wt(kin + b0 + k) : 0;
            f2[k] = ok ? ld_wt_i(fin + b0 + k) : 0;
        }
        uint64_t ktot;
        int32_t ftot;
        uint64_t kex = block_excl_scan<uint64_t, NT>(k2[0] + k2[1], shk, ktot);
        int32_t fex = block_excl_scan<int32_t, NT>(f2[0] + f2[1], shf, ftot);
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (b0 + k < nb) {
                st_wt(kout + b0 + k, kex);
                st_wt_i(fout + b0 + k, fex);
                if (f_lds) f_lds[b0 + k] = fex;
                kex = kex + k2[k];
                fex = fex + f2[k];
            }
        if (threadIdx.x == 0) {
            st_wt(ktotal, ktot);
            st_wt_i(ftotal, ftot);
        }
        return;
    }
    const int span = ((nb + W * 64 - 1) / (W * 64)) * 64;
    const int R = span / 64;
    const int e0 = wid * span + lane;
    uint64_t kv[kC];
    int32_t fv[kC];
    uint64_t kloc = 0;
    int32_t floc = 0;
    for (int r0 = 0; r0 < R; r0 += kC) {
#pragma unroll
        for (int r = 0; r < kC; ++r) {
            const int e = e0 + (r0 + r) * 64;
            const bool ok = r0 + r < R && e < nb;
            kv[r] = ok ? ld_wt(kin + e) : 0;
            fv[r] = ok ? ld_wt_i(fin + e) : 0;
        }
#pragma unroll
        for (int r = 0; r < kC; ++r) {
            kloc = kloc + kv[r];
            floc = floc + fv[r];
        }
    }
    uint64_t ktot;
    int32_t ftot;
    // lane 0's exclusive prefix over the block = the sum of the lower waves
    uint64_t krun = readlane_int(block_excl_scan<uint64_t, NT>(kloc, shk, ktot), 0);
    int32_t frun = readlane_int(block_excl_scan<int32_t, NT>(floc, shf, ftot), 0);
    for (int r0 = 0; r0 < R; r0 += kC) {
        if (R > kC) {                              // (one chunk: still in registers)
#pragma unroll
            for (int r = 0; r < kC; ++r) {
                const int e = e0 + (r0 + r) * 64;
                const bool ok = r0 + r < R && e < nb;
                kv[r] = ok ? ld_wt(kin + e) : 0;
                fv[r] = ok ? ld_wt_i(fin + e) : 0;
            }
        }
#pragma unroll
        for (int r = 0; r < kC; ++r) {
            if (r0 + r < R) {                      // (wave-uniform)
                const uint64_t ki = wave_incl_scan(kv[r]);
                const int32_t fi = wave_incl_scan(fv[r]);
                const int e = e0 + (r0 + r) * 64;
                if (e < nb) {
                    const int32_t fex = frun + (fi - fv[r]);
                    st_wt(kout + e, krun + (ki - kv[r]));
                    st_wt_i(fout + e, fex);
                    if (f_lds) f_lds[e] = fex;
                }
                krun += readlane_int(ki, 63);
                frun += readlane_int(fi, 63);
            }
        }
    }
    if (threadIdx.x == 0) {
        st_wt(ktotal, ktot);
        st_wt_i(ftotal, ftot);
    }
}

// ====================================================================
// normalise (particle_filter.py:226-237) + reductions; the last block
// combines the block partials in block order and writes the step result.
// ====================================================================
__device__ __forceinline__ void bp_zero(BlockPartial& a) {
    a.maxv = -1.0;
    a.maxi = INT64_MAX;
    a.sw = a.sw2 = 0.0;
    for (int k = 0; k < 3; ++k) a.m1[k] = 0.0;
    for (int k = 0; k < 6; ++k) a.m2[k] = 0.0;
}

__device__ __forceinline__ void bp_merge(BlockPartial& r, const BlockPartial& o) {
    if (o.maxv > r.maxv || (o.maxv == r.maxv && o.maxi < r.maxi)) {
        r.maxv = o.maxv;
        r.maxi = o.maxi;
    }
    r.sw += o.sw;
    r.sw2 += o.sw2;
    for (int q = 0; q < 3; ++q) r.m1[q] += o.m1[q];
    for (int q = 0; q < 6; ++q) r.m2[q] += o.m2[q];
}

// xor-butterfly over the 64 lanes (lower lane always on the left: a fixed tree)
template <int W = 64>
__device__ __forceinline__ void bp_wave_reduce(BlockPartial& a) {
#pragma unroll
    for (int d = 1; d < W; d <<= 1) {
        BlockPartial o;
        o.maxv = __shfl_xor(a.maxv, d, 64);
        o.maxi = __shfl_xor(a.maxi, d, 64);
        o.sw = __shfl_xor(a.sw, d, 64);
        o.sw2 = __shfl_xor(a.sw2, d, 64);
#pragma unroll
        for (int k = 0; k < 3; ++k) o.m1[k] = __shfl_xor(a.m1[k], d, 64);
#pragma unroll
        for (int k = 0; k < 6; ++k) o.m2[k] = __shfl_xor(a.m2[k], d, 64);
        if (threadIdx.x & d) {
            bp_merge(o, a);
            a = o;
        } else {
            bp_merge(a, o);
        }
    }
}

// block-level fixed-order reduction of per-thread partials (result in thread 0):
// a butterfly inside every wave, then a butterfly over the wave partials in wave 0
__device__ __forceinline__ BlockPartial bp_block_reduce(BlockPartial a, BlockPartial* shp) {
    bp_wave_reduce(a);
    const int nw = (int)(blockDim.x >> 6);
    if ((threadIdx.x & 63) == 0) shp[threadIdx.x >> 6] = a;
    __syncthreads();
    BlockPartial r;
    if (threadIdx.x < 64) {
        if ((int)threadIdx.x < nw) r = shp[threadIdx.x];
        else bp_zero(r);
        if (nw > 8) bp_wave_reduce<16>(r);
        else if (nw > 4) bp_wave_reduce<8>(r);
        else bp_wave_reduce<4>(r);
    }
    __syncthreads();
    return r;
}

// result record from the combined partial (x_est = particle at the argmax)
__device__ void write_result(const BlockPartial& r, const double* xs, const double* ys,
                             const double* ts, const int64_t gbase, double* refp,
                             const double s, int32_t* flags, const double ess_th,
                             const double ess_band, slam_pf_result* res,
                             const int32_t resampled_known) {
    slam_pf_result o;
    const int64_t mi = r.maxi;
    o.max_idx = mi;
    o.max_val = r.maxv;
    o.x_est[0] = xs[mi - gbase];
    o.x_est[1] = ys[mi - gbase];
    o.x_est[2] = ts[mi - gbase];
    const double inv = 1.0 / r.sw;
    const double mu[3] = {r.m1[0] * inv, r.m1[1] * inv, r.m1[2] * inv};
    const double m2[9] = {r.m2[0], r.m2[1], r.m2[2], r.m2[1], r.m2[3], r.m2[4], r.m2[2], r.m2[4], r.m2[5]};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) o.cov[3 * a + b] = m2[3 * a + b] * inv - mu[a] * mu[b];
    o.ess = 1.0 / r.sw2;
    o.weight_sum = s;
    o.resampled = resampled_known >= 0 ? resampled_known : (flags[kFlagResample] != 0);
    o.resample_next = (o.ess < ess_th) ? 1 : 0;
    o.ess_near = (fabs(o.ess - ess_th) <= ess_band * ess_th) ? 1 : 0;
    o.status = flags[kFlagStatus];
    o.n_special = flags[kFlagNSpecial];
    o.dd_waves = flags[kFlagDDWaves];
    flags[kFlagDDWaves] = 0;
    flags[kFlagResample] = o.resample_next;
    flags[kFlagMarkGen] = flags[kFlagMarkGen] + 1;
    flags[kFlagStatus] = 0;
    // the estimate, kept two steps deep as the expansion's reference
    // (closed_prep_reference: the argmax particle is the same bits however
    // the filter is sharded, which a summed mean would not be)
    for (int k = 0; k < 3; ++k) {
        refp[4 + k] = refp[k];
        refp[k] = o.x_est[k];
    }
    refp[7] = 2.0;
    *res = o;
}

// result record with x_est given (deferred path: taken from the block partials)
// The flag words the step's record reads (fetched early by the finalize, whose
// record is on the step's critical path)
struct FlagWords {
    int32_t resample, status, n_special, dd_waves, mark_gen;
};
__device__ __forceinline__ FlagWords load_flag_words(const int32_t* flags) {
    return FlagWords{flags[kFlagResample], flags[kFlagStatus], flags[kFlagNSpecial],
                     flags[kFlagDDWaves], flags[kFlagMarkGen]};
}

__device__ int32_t write_result_fw(const BlockPartial& r, const double* xe, double* refp,
                                const double (&rp)[3], const double s, int32_t* flags,
                                const FlagWords fw, const double ess_th,
                                const double ess_band, slam_pf_result* res,
                                const int32_t resampled_known, slam_pf_result* res_host = nullptr) {
    slam_pf_result o;
    o.max_idx = r.maxi;
    o.max_val = r.maxv;
    o.x_est[0] = xe[0];
    o.x_est[1] = xe[1];
    o.x_est[2] = xe[2];
    const double inv = 1.0 / r.sw;
    const double mu[3] = {r.m1[0] * inv, r.m1[1] * inv, r.m1[2] * inv};
    const double m2[9] = {r.m2[0], r.m2[1], r.m2[2], r.m2[1], r.m2[3], r.m2[4], r.m2[2], r.m2[4], r.m2[5]};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) o.cov[3 * a + b] = m2[3 * a + b] * inv - mu[a] * mu[b];
    o.ess = 1.0 / r.sw2;
    o.weight_sum = s;
    o.resampled = resampled_known >= 0 ? resampled_known : (fw.resample != 0);
    o.resample_next = (o.ess < ess_th) ? 1 : 0;
    o.ess_near = (fabs(o.ess - ess_th) <= ess_band * ess_th) ? 1 : 0;
    o.status = fw.status;
    o.n_special = fw.n_special;
    o.dd_waves = fw.dd_waves;
    flags[kFlagDDWaves] = 0;
    flags[kFlagResample] = o.resample_next;
    flags[kFlagMarkGen] = fw.mark_gen + 1;
    flags[kFlagStatus] = 0;
    // the estimate, kept two steps deep as the expansion's reference
    // (closed_prep_reference: the argmax particle is the same bits however
    // the filter is sharded, which a summed mean would not be)
    for (int k = 0; k < 3; ++k) {
        refp[4 + k] = rp[k];
        refp[k] = o.x_est[k];
    }
    refp[7] = 2.0;
    *res = o;
    if (res_host) *res_host = o;
    return o.resample_next;
}

// returns resample_next (the flag it stored)
__device__ int32_t write_result_xe(const BlockPartial& r, const double* xe, double* refp,
                                const double s, int32_t* flags, const double ess_th,
                                const double ess_band, slam_pf_result* res,
                                const int32_t resampled_known, slam_pf_result* res_host = nullptr) {
    const double rp[3] = {refp[0], refp[1], refp[2]};
    return write_result_fw(r, xe, refp, rp, s, flags, load_flag_words(flags), ess_th, ess_band, res,
                           resampled_known, res_host);
}

// One normalise block = kNormPer particles (kNormThreads lanes x kNormEPT,
// coalesced per k); all loads of a lane are issued before any use.
__global__ __launch_bounds__(kNormThreads) void normalize_kernel(
    const int64_t n, const double* __restrict__ w_un, double* __restrict__ w,
    const double* __restrict__ s_in, const double np_recip, const double* __restrict__ xs,
    const double* __restrict__ ys, const double* __restrict__ ts, const double* __restrict__ refp,
    BlockPartial* __restrict__ bp, double* __restrict__ bsum, const int64_t gbase) {
    __shared__ BlockPartial shp[kNormThreads / 64];
    const double s = *s_in;
    const double r0 = refp[0], r1 = refp[1], r2 = refp[2];
    const int64_t base = (int64_t)blockIdx.x * kNormPer + threadIdx.x;
    double wu[kNormEPT], xv[kNormEPT], yv[kNormEPT], tv[kNormEPT];
    if (base + (kNormEPT - 1) * kNormThreads < n) {
#pragma unroll
        for (int k = 0; k < kNormEPT; ++k) {
            const int64_t i = base + k * kNormThreads;
            wu[k] = w_un[i];
            xv[k] = xs[i];
            yv[k] = ys[i];
            tv[k] = ts[i];
        }
    } else {
#pragma unroll
        for (int k = 0; k < kNormEPT; ++k) {
            const int64_t i = base + k * kNormThreads;
            const bool ok = i < n;
            wu[k] = ok ? w_un[i] : 0.0;
            xv[k] = ok ? xs[i] : r0;
            yv[k] = ok ? ys[i] : r1;
            tv[k] = ok ? ts[i] : r2;
        }
    }
    BlockPartial a;
    bp_zero(a);
#pragma unroll
    for (int k = 0; k < kNormEPT; ++k) {
        const int64_t i = base + k * kNormThreads;
        if (i < n) {
            double v = wu[k] / s;                        // particle_filter.py:235
            if (isnan(v)) v = np_recip;                  // :236
            w[i] = v;
            if (v > a.maxv) {
                a.maxv = v;
                a.maxi = gbase + i;
            }
            a.sw += v;
            a.sw2 += v * v;
            const double d0 = xv[k] - r0, d1 = yv[k] - r1, d2 = tv[k] - r2;
            const double v0 = v * d0, v1 = v * d1, v2 = v * d2;
            a.m1[0] += v0;
            a.m1[1] += v1;
            a.m1[2] += v2;
            a.m2[0] += v0 * d0;
            a.m2[1] += v0 * d1;
            a.m2[2] += v0 * d2;
            a.m2[3] += v1 * d1;
            a.m2[4] += v1 * d2;
            a.m2[5] += v2 * d2;
        }
    }
    const BlockPartial r = bp_block_reduce(a, shp);
    if (threadIdx.x == 0) {
        bp[blockIdx.x] = r;
        bsum[blockIdx.x] = r.sw;                         // approximate block total (S1)
    }
}

// Combine the normalise blocks' partials in block order (one block of up to
// 1024 lanes, one partial per lane, then a fixed tree), write the step's
// result record, advance the step context, and -- when the next step
// resamples -- scan the block totals for its exact cumsum.  A separate launch
// instead of a last-arriver tail: the kernel boundary costs less than the
// serial ticket/load chain of an in-kernel combine.
__global__ __launch_bounds__(1024) void finalize_kernel(
    const BlockPartial* __restrict__ bp, const int32_t nb, const double* __restrict__ bsum,
    double* __restrict__ boff, const double* __restrict__ xs, const double* __restrict__ ys,
    const double* __restrict__ ts, double* __restrict__ refp, const double* __restrict__ s_in,
    int32_t* __restrict__ flags, const double ess_th, StepIO io, const int32_t resampled_known,
    const int64_t gbase) {
    __shared__ BlockPartial shp[1024 / 64];
    __shared__ double shd[1024 / 64 + 1];
    __shared__ int32_t want_scan;
    BlockPartial c;
    bp_zero(c);
    for (int k = threadIdx.x; k < nb; k += blockDim.x) bp_merge(c, bp[k]);
    const BlockPartial tot = bp_block_reduce(c, shp);
    if (threadIdx.x == 0) {
        const int32_t st = io.ctr[0];
        write_result(tot, xs, ys, ts, gbase, refp, *s_in, flags, ess_th, io.ess_band, io.res + st,
                     resampled_known);
        want_scan = flags[kFlagResample];
        io.ctr[0] = st + 1;                              // advance the step context
        io.ctr[1] = io.ctr[1] + 1;
    }
    __syncthreads();
    if (want_scan) {
        // exclusive prefix of the block totals (plain loads: previous kernel's data)
        const int per = (nb + 1023) / 1024;
        const int b0 = threadIdx.x * per;
        double loc = 0.0;
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) loc += bsum[b0 + k];
        double total;
        double ex = block_excl_scan<double, 1024>(loc, shd, total);
        for (int k = 0; k < per; ++k)
            if (b0 + k < nb) {
                const double v = bsum[b0 + k];
                boff[b0 + k] = ex;
                ex = ex + v;
            }
        if (threadIdx.x == 0) boff[nb] = total;
    }
}

// np.sum of one full 8192-element buffer from its 64 leaf sums (perfect
// pairwise tree, left + right at every node).
__device__ __forceinline__ double chunk_tree64(const double* __restrict__ L) {
    double stk[7];
    for (int i = 0; i < 64; ++i) {
        double v = L[i];
        int b = 0;
        for (; (i >> b) & 1; ++b) v = stk[b] + v;
        stk[b] = v;
    }
    return stk[6];
}

// np.sum of a tail buffer (< 8192 elements) from raw weights: leaves by the
// block's lanes, the post-order program by lane 0 (as chunk_sum_kernel).
__device__ double tail_chunk_sum(const double* __restrict__ w, const int32_t* __restrict__ leaves,
                                 const int32_t* __restrict__ ops, const int32_t n_leaves,
                                 const int32_t n_ops, double* sh) {
    for (int L = threadIdx.x; L < n_leaves; L += blockDim.x) {
        const int lo = leaves[2 * L], cnt = leaves[2 * L + 1];
        const double* a = w + lo;
        double res;
        if (cnt < 8) {
            res = 0.0;
            for (int i = 0; i < cnt; ++i) res = res + a[i];
        } else {
            double r[8];
            for (int k = 0; k < 8; ++k) r[k] = a[k];
            int i = 8;
            const int stop = cnt - (cnt % 8);
            for (; i < stop; i += 8)
                for (int k = 0; k < 8; ++k) r[k] = r[k] + a[i + k];
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            for (; i < cnt; ++i) res = res + a[i];
        }
        sh[L] = res;
    }
    __syncthreads();
    double out = 0.0;
    if (threadIdx.x == 0) {
        double stk[16];
        int sp = 0;
        for (int o = 0; o < n_ops; ++o) {
            const int op = ops[o];
            if (op >= 0) {
                stk[sp++] = sh[op];
            } else {
                const double b = stk[--sp];
                const double a = stk[--sp];
                stk[sp++] = a + b;
            }
        }
        out = stk[0];
    }
    __syncthreads();
    return out;
}

#include "pf_finalize.inl"

// w = w_un / s (NaN -> 1/NP): materialise the current weights (get_state, np.sum)
__global__ __launch_bounds__(256) void normalize_only_kernel(const int64_t n,
                                                             const double* __restrict__ w_un,
                                                             const double* __restrict__ s,
                                                             const double np_recip,
                                                             double* __restrict__ w) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) w[i] = norm_w(w_un[i], *s, np_recip);
}

// S1 of the deferred path: 256-block totals of w = w_un / s and their prefix.
__global__ __launch_bounds__(kPartPer) void scan_bsum256_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_in, const double np_recip,
    const int64_t n, double* __restrict__ bsum, double* __restrict__ boff,
    unsigned* __restrict__ counter) {
    __shared__ double sh[kPartPer / 64 + 1];
    const int64_t i = (int64_t)blockIdx.x * kPartPer + threadIdx.x;
    const double v = (i < n) ? norm_w(w_un[i], *s_in, np_recip) : 0.0;
    double tot;
    block_excl_scan<double, kPartPer>(v, sh, tot);
    if (threadIdx.x == 0) st_wt_d(&bsum[blockIdx.x], tot);
    if (!arrive_last(counter)) return;
    block_scan_array<double, kPartPer>(bsum, boff, gridDim.x, boff + gridDim.x, sh);
}

// ====================================================================
// exact sequential cumsum (np.cumsum, particle_filter.py:212)
// ====================================================================
// S1: approximate totals of kNormPer-element blocks of w; the last block scans
// them into boff (boff[nb] = total).  normalize_kernel produces the same
// arrays as a by-product when the next step resamples.
__global__ __launch_bounds__(kNormThreads) void scan_bsum_kernel(
    const double* __restrict__ w, const int64_t n, double* __restrict__ bsum,
    double* __restrict__ boff, unsigned* __restrict__ counter) {
    __shared__ double sh[kNormThreads / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * kNormPer + threadIdx.x;
    double loc = 0.0;
#pragma unroll
    for (int k = 0; k < kNormEPT; ++k) {
        const int64_t i = base + k * kNormThreads;
        if (i < n) loc += w[i];
    }
    double tot;
    block_excl_scan<double, kNormThreads>(loc, sh, tot);
    if (threadIdx.x == 0) st_wt_d(&bsum[blockIdx.x], tot);
    if (!arrive_last(counter)) return;
    block_scan_array<double, kNormThreads>(bsum, boff, gridDim.x, boff + gridDim.x, sh);
}

// the weight an exact-cumsum pass reads: w itself, or w_un / s on the deferred path
__device__ __forceinline__ double scan_w(const double* __restrict__ w, const int64_t i,
                                         const double* __restrict__ s_div, const double np_recip) {
    return s_div ? norm_w(w[i], *s_div, np_recip) : w[i];
}

// S3: classify every element; k_i = increment on the run's ulp grid.  The last
// block scans the per-block special counts and increment sums.
// base_off: approximate cumsum before local element 0 (other ranks' weight).
__global__ __launch_bounds__(kScanThreads) void scan_classify_kernel(
    const double* __restrict__ w, const int64_t n, const double* __restrict__ boff,
    const double* __restrict__ base_off, double* __restrict__ approx,
    uint64_t* __restrict__ kincl, int32_t* __restrict__ fexcl, uint64_t* __restrict__ bk,
    int32_t* __restrict__ bf, uint64_t* __restrict__ boffk, int32_t* __restrict__ bofff,
    uint64_t* __restrict__ ktot, int32_t* __restrict__ nspec, const double delta,
    const int64_t gbase, unsigned* __restrict__ counter, const int32_t* __restrict__ flags,
    const int32_t force, const double* __restrict__ s_div, const double np_recip,
    const int32_t gran) {
    if (!force && flags[kFlagResample] != 1) return;
    __shared__ double shd[kScanThreads / 64 + 1];
    __shared__ uint64_t shk[kScanThreads / 64 + 1];
    __shared__ int32_t shf[kScanThreads / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    double v[kScanPer];
    double loc = 0.0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        v[k] = (base + k < n) ? scan_w(w, base + k, s_div, np_recip) : 0.0;
        loc += v[k];
    }
    double dtot;
    double run = block_excl_scan<double, kScanThreads>(loc, shd, dtot) +
                 boff[(int64_t)blockIdx.x * (kScanBlock / gran)] +
                 (base_off ? *base_off : 0.0);
    uint64_t kk[kScanPer];
    int32_t ff[kScanPer];
    uint64_t ksum = 0;
    int32_t fsum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const double prev = run;
        run = run + v[k];
        const int64_t gi = gbase + base + k;
        bool reg = (gi != 0) && (base + k < n);
        uint64_t inc = 0;
        if (reg) {
            const int E = sum_binade(run);
            reg = (sum_binade(prev) == E);
            if (reg && E != -1022) reg = prev >= ldexp(1.0, E) * (1.0 + delta);
            if (reg) reg = run <= ldexp(1.0, E + 1) * (1.0 - delta);
            if (reg) {
                const double t = ldexp(v[k], 52 - E);
                const double fl = floor(t);
                reg = (t - fl) != 0.5;
                inc = (uint64_t)rint(t);
            }
        }
        kk[k] = reg ? inc : 0;
        ff[k] = (reg || base + k >= n) ? 0 : 1;
        ksum += kk[k];
        fsum += ff[k];
        if (base + k < n) approx[base + k] = run;
    }
    uint64_t ktot_b;
    int32_t ftot_b;
    uint64_t kex = block_excl_scan<uint64_t, kScanThreads>(ksum, shk, ktot_b);
    int32_t fex = block_excl_scan<int32_t, kScanThreads>(fsum, shf, ftot_b);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (base + k < n) {
            kex += kk[k];
            kincl[base + k] = kex;
            fexcl[base + k] = (fex << 1) | ff[k];
            fex += ff[k];
        }
    }
    if (threadIdx.x == 0) {
        st_wt(&bk[blockIdx.x], ktot_b);
        st_wt_i(&bf[blockIdx.x], ftot_b);
    }
    if (!arrive_last(counter)) return;
    block_scan_array<uint64_t, kScanThreads>(bk, boffk, gridDim.x, ktot, shk);
    __syncthreads();
    block_scan_array<int32_t, kScanThreads>(bf, bofff, gridDim.x, nspec, shf);
}

// S6: sequential fold over the ordered special elements (one block; tiles in
// LDS).  Runs of regular elements are added as one exact integer multiple of
// their binade's ulp.  Falls back to the plain sequential recurrence if a
// run check fails (flags status bit 1).
__device__ void serial_fold(const SpecialIn* __restrict__ spec, SpecialOut* __restrict__ out,
                            const int32_t M, const uint64_t ktot, const int64_t n_total,
                            int32_t* __restrict__ flags, const double* __restrict__ w,
                            double* __restrict__ c, const int64_t n_local, const bool wt_loads,
                            const double* __restrict__ s_div, const double np_recip) {
    __shared__ SpecialIn tile[257];
    __shared__ int bad;
    double s = 0.0;
    if (threadIdx.x == 0) {
        bad = 0;
        flags[kFlagNSpecial] = M;
    }
    for (int32_t t0 = 0; t0 < M; t0 += 256) {
        __syncthreads();
        const int32_t cnt = min(257, M - t0);
        for (int k = threadIdx.x; k < cnt; k += blockDim.x)
            tile[k] = wt_loads ? ld_wt_struct(&spec[t0 + k]) : spec[t0 + k];
        __syncthreads();
        if (threadIdx.x == 0 && !bad) {
            const int lim = min(256, M - t0);
            for (int k = 0; k < lim; ++k) {
                const SpecialIn& e = tile[k];
                s = s + e.w;
                SpecialOut o;
                o.cs = s;
                o.P = e.P;
                o.E = e.E;
                o.pad = 0;
                const bool last = (t0 + k + 1 >= M);
                const int64_t nxt = last ? n_total : tile[k + 1].idx;
                if (nxt - e.idx > 1) {
                    const uint64_t K = (last ? ktot : tile[k + 1].P) - e.P;
                    const int E = e.E;
                    if (sum_binade(s) != E) { bad = 1; break; }
                    const double s2 = s + (double)K * ldexp(1.0, E - 52);
                    const double hi = (E == -1022) ? 0x1p-1021 : ldexp(1.0, E + 1);
                    if (!(s2 < hi) || (double)K >= 0x1p53) { bad = 1; break; }
                    s = s2;
                }
                out[t0 + k] = o;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && bad) {
        flags[kFlagStatus] |= 2;
        flags[kFlagFallback] = 1;
        double r = 0.0;
        for (int64_t i = 0; i < n_local; ++i) {
            r = r + scan_w(w, i, s_div, np_recip);
            c[i] = r;
        }
    } else if (threadIdx.x == 0) {
        flags[kFlagFallback] = 0;
    }
}

// S5: scatter the special elements into an ordered list (write-through); the
// last block folds them (single GPU).  Multi-GPU gathers the lists first and
// runs scan_fold_kernel on the concatenation.
__global__ __launch_bounds__(kScanThreads) void scan_emit_kernel(
    const double* __restrict__ w, const int64_t n, const double* __restrict__ approx,
    const uint64_t* __restrict__ kincl, const int32_t* __restrict__ fexcl,
    const uint64_t* __restrict__ boffk, const int32_t* __restrict__ bofff,
    SpecialIn* __restrict__ spec, const int64_t gbase, SpecialOut* __restrict__ spec_out,
    const int32_t* __restrict__ nspec_p, const uint64_t* __restrict__ ktot_p,
    const int32_t do_fold, double* __restrict__ c, unsigned* __restrict__ counter,
    int32_t* __restrict__ flags, const int32_t force, const double* __restrict__ s_div,
    const double np_recip) {
    if (!force && flags[kFlagResample] != 1) return;
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        const int32_t f = fexcl[i];
        if (f & 1) {
            const int32_t m = bofff[blockIdx.x] + (f >> 1);
            SpecialIn s;
            s.idx = gbase + i;
            s.P = boffk[blockIdx.x] + kincl[i];
            s.w = scan_w(w, i, s_div, np_recip);
            s.E = sum_binade(approx[i]);
            s.pad = 0;
            st_wt_struct(&spec[m], s);
        }
    }
    if (!do_fold) return;
    if (!arrive_last(counter)) return;
    serial_fold(spec, spec_out, *nspec_p, *ktot_p, n, flags, w, c, n, true, s_div, np_recip);
}

// S6 stand-alone (multi-GPU: over the gathered global list)
__global__ __launch_bounds__(256) void scan_fold_kernel(
    const SpecialIn* __restrict__ spec, SpecialOut* __restrict__ out, const int32_t* __restrict__ M,
    const uint64_t* __restrict__ ktot, const int64_t n_total, int32_t* __restrict__ flags,
    const double* __restrict__ w, double* __restrict__ c, const int64_t n_local) {
    serial_fold(spec, out, *M, *ktot, n_total, flags, w, c, n_local, false, nullptr, 0.0);
}

// S7: expand the exact cumsum from the specials.  spec_base / k_base: global
// special count and increment prefix before local element 0 (multi-GPU).
__global__ __launch_bounds__(kScanThreads) void scan_expand_kernel(
    const int64_t n, const uint64_t* __restrict__ kincl, const int32_t* __restrict__ fexcl,
    const uint64_t* __restrict__ boffk, const int32_t* __restrict__ bofff,
    const SpecialOut* __restrict__ so, double* __restrict__ c, const int32_t* __restrict__ flags,
    const int32_t* __restrict__ spec_base, const uint64_t* __restrict__ k_base,
    const int32_t force) {
    if (!force && flags[kFlagResample] != 1) return;
    if (flags[kFlagFallback]) return;
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    const uint64_t bko = boffk[blockIdx.x] + (k_base ? *k_base : 0);
    const int32_t bfo = bofff[blockIdx.x] + (spec_base ? *spec_base : 0);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        const int32_t f = fexcl[i];
        const int32_t m = bfo + (f >> 1);
        if (f & 1) {
            c[i] = so[m].cs;
        } else {
            const SpecialOut& p = so[m - 1];
            const uint64_t K = bko + kincl[i] - p.P;
            c[i] = p.cs + (double)K * ldexp(1.0, p.E - 52);
        }
    }
}

// ====================================================================
// Lean exact cumsum (single-GPU handles), one WAVE per 512-element tile (a
// fused block's particles): no per-element scratch and no block barrier in
// the per-tile work -- the tile's prefix sums are wave scans.  Pass A
// classifies each tile and stages its few special elements; its last block
// places them in global order and folds them; pass C expands c from the
// classification (kept in registers in the merged launch, recomputed in the
// two-launch form) and writes the inverse resample map.  Reads w once (twice
// in the two-launch form), writes c once.
// ====================================================================
constexpr int kWaveTile = 64 * kScanPer;                 // 512 elements
static_assert(kWaveTile == kPartPer, "a scan tile is a fused block (boff, carry indexing)");
constexpr int kTilesPerBlock = kScanThreads / 64;

struct TileScan {
    uint64_t kex;            // exclusive prefix of the tile-local increments (this lane)
    int32_t fex;             // exclusive prefix of the tile-local special count (this lane)
    uint64_t kk[kScanPer];   // increments of this lane's elements (0 for specials)
    int32_t ff[kScanPer];    // special flags
    double v[kScanPer];      // the weights
    int E[kScanPer];         // binade of the approximate prefix after the element
};

// exclusive wave scan; `total` = the wave's sum (every lane)
template <typename T>
__device__ __forceinline__ T wave_excl_scan(const T v, T& total) {
    const T inc = wave_incl_scan(v);
    if constexpr (std::is_integral<T>::value) {
        total = readlane_int(inc, 63);
        return inc - v;
    } else {
        T ex = __shfl_up(inc, 1, 64);
        if ((threadIdx.x & 63) == 0) ex = T(0);
        total = __shfl(inc, 63, 64);
        return ex;
    }
}

// Tile `tile` of the weights w = w_un / s, lane l owns elements 8l .. 8l+7
// (four 16-byte loads; w_un is padded to whole tiles).  off: the approximate
// prefix before the tile (the finalize pass's fused-block prefix).
__device__ __forceinline__ void wave_tile_classify(const double* __restrict__ w_un,
                                                   const double s, const double np_recip,
                                                   const int64_t n, const int64_t tile,
                                                   const double off, const double delta,
                                                   TileScan& ts, uint64_t& ktile,
                                                   int32_t& ftile) {
    const int lane = threadIdx.x & 63;
    const int64_t base = tile * kWaveTile + 8 * lane;
#pragma unroll
    for (int h = 0; h < kScanPer; h += 2) {
        const double2 w2 = *reinterpret_cast<const double2*>(w_un + base + h);
        ts.v[h] = (base + h < n) ? norm_w(w2.x, s, np_recip) : 0.0;
        ts.v[h + 1] = (base + h + 1 < n) ? norm_w(w2.y, s, np_recip) : 0.0;
    }
    double loc = 0.0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) loc += ts.v[k];
    // the approximate prefix (any fixed order: the classification's margins
    // cover its error, and pass C recomputes it with this same code)
    double wtot;
    double run = wave_excl_scan_rows(loc, wtot) + off;
    uint64_t ksum = 0;
    int32_t fsum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const double prev = run;
        run = run + ts.v[k];
        const int64_t gi = base + k;
        bool reg = (gi != 0) && (gi < n);
        uint64_t inc = 0;
        const int E = sum_binade(run);
        if (reg) {
            reg = (sum_binade(prev) == E);
            if (reg && E != -1022) reg = prev >= ldexp(1.0, E) * (1.0 + delta);
            if (reg) reg = run <= ldexp(1.0, E + 1) * (1.0 - delta);
            if (reg) {
                const double tt = ldexp(ts.v[k], 52 - E);
                const double fl = floor(tt);
                reg = (tt - fl) != 0.5;
                inc = (uint64_t)rint(tt);
            }
        }
        ts.kk[k] = reg ? inc : 0;
        ts.ff[k] = (reg || gi >= n) ? 0 : 1;
        ts.E[k] = E;
        ksum += ts.kk[k];
        fsum += ts.ff[k];
    }
    ts.kex = wave_excl_scan(ksum, ktile);
    ts.fex = wave_excl_scan(fsum, ftile);
}

// The four tiles of a block combine their totals (LDS, one barrier): the
// block's staging area, its (k, f) totals and the tiles' exclusive offsets
// inside the block.  The last arriver then scans one total per block.
__device__ __forceinline__ void block_tile_offsets(const uint64_t ktile, const int32_t ftile,
                                                   uint64_t& kofs, int32_t& fofs,
                                                   uint64_t& kblk, int32_t& fblk) {
    __shared__ uint64_t s_kt[kTilesPerBlock];
    __shared__ int32_t s_ft[kTilesPerBlock];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_kt[wave] = ktile;
        s_ft[wave] = ftile;
    }
    __syncthreads();
    kofs = 0;
    fofs = 0;
    kblk = 0;
    fblk = 0;
#pragma unroll
    for (int w = 0; w < kTilesPerBlock; ++w) {
        if (w < wave) {
            kofs += s_kt[w];
            fofs += s_ft[w];
        }
        kblk += s_kt[w];
        fblk += s_ft[w];
    }
}

// Stage a classified tile's specials in its block's area (block-local P,
// write-through); thread 0 publishes the block totals.
__device__ __forceinline__ void wave_tile_stage(const int64_t b, const int64_t tile,
                                                const TileScan& ts,
                                                const uint64_t kofs, const int32_t fofs,
                                                const uint64_t kblk, const int32_t fblk,
                                                SpecialIn* __restrict__ stage,
                                                uint64_t* __restrict__ bk,
                                                int32_t* __restrict__ bf) {
    const int lane = threadIdx.x & 63;
    uint64_t kex = kofs + ts.kex;
    int32_t fex = fofs + ts.fex;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        kex += ts.kk[k];
        if (ts.ff[k]) {
            SpecialIn r;
            r.idx = tile * kWaveTile + 8 * lane + k;
            r.P = kex;                                  // block-local inclusive prefix
            r.w = ts.v[k];
            r.E = ts.E[k];
            r.pad = 0;
            st_wt_struct(&stage[b * kScanBlock + fex], r);
            ++fex;
        }
    }
    if (threadIdx.x == 0) {
        st_wt(&bk[b], kblk);
        st_wt_i(&bf[b], fblk);
    }
}


// The lean path's place + fold (last block of pass A): the M specials, in
// global order, are located in the tiles' staging areas (tile offsets bofff in
// LDS, searched per lane), given their global P, and folded by wave 0 in
// chunks of 64: lane l precomputes everything that does not depend on the
// running sum (the exact run increment K u of the following regular run, the
// binade bounds the checks use), then the running sum walks the 64 lanes --
// two dependent adds per special, operands read from the lanes into SGPRs.
// Bit-identical to serial_fold; a failed run check takes the same fallback
// (the plain sequential recurrence, flagged).
constexpr int kFoldTilesLds = 4096;
__device__ __forceinline__ void lean_place_fold(const SpecialIn* __restrict__ stage,
                                const uint64_t* __restrict__ boffk,
                                const int32_t* __restrict__ bofff, const int ntiles,
                                const int32_t M, const uint64_t ktot, const int64_t n,
                                SpecialOut* __restrict__ out, int32_t* __restrict__ flags,
                                const double* __restrict__ w_un, const double* __restrict__ s_in,
                                const double np_recip, double* __restrict__ c,
                                int32_t* __restrict__ s_off) {
    // s_off: the tiles' special offsets in LDS (kFoldTilesLds words), already
    // filled by the scan that produced bofff when ntiles fits
    __shared__ int s_bad;
    const bool in_lds = ntiles <= kFoldTilesLds;
    if (threadIdx.x == 0) {
        s_bad = 0;
        flags[kFlagNSpecial] = M;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        // special m: its tile (last tile whose offset is <= m), then the staged record
        auto load_special = [&](const int64_t m, SpecialIn& e) {
            int lo = 0, hi = ntiles - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                const int32_t o = in_lds ? s_off[mid] : ld_wt_i(&bofff[mid]);
                if (o <= m) lo = mid;
                else hi = mid - 1;
            }
            const int32_t o = in_lds ? s_off[lo] : ld_wt_i(&bofff[lo]);
            e = ld_wt_struct(&stage[(int64_t)lo * kScanBlock + (m - o)]);
            e.P += ld_wt(&boffk[lo]);
        };
        double s = 0.0;
        bool bad = false;
        // chunks of 63 specials: lane 63 only supplies the next chunk's first
        for (int64_t t0 = 0; t0 < M; t0 += 63) {
            const int64_t m = t0 + lane;
            SpecialIn e{};
            if (m < M) load_special(m, e);
            // the following special's index and prefix (or the end of the array)
            int64_t nidx = __shfl_down((long long)e.idx, 1, 64);
            uint64_t nP = (uint64_t)__shfl_down((long long)e.P, 1, 64);
            if (m + 1 >= M) {
                nidx = n;
                nP = ktot;
            }
            const bool mine = (lane < 63) && (m < M);
            const bool run = mine && (nidx - e.idx > 1);
            const uint64_t K = nP - e.P;
            const int E = e.E;
            double lo = -__builtin_inf(), hi = __builtin_inf(), ku = 0.0;
            if (run) {
                lo = (E == -1022) ? 0.0 : ldexp(1.0, E);
                hi = (E == -1022) ? 0x1p-1021 : ldexp(1.0, E + 1);
                ku = (double)K * ldexp(1.0, E - 52);
                if ((double)K >= 0x1p53) bad = true;
            }
            const double w = mine ? e.w : 0.0;
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
            if (mine) {
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
        if (s_bad) {
            flags[kFlagStatus] |= 2;
            st_wt_i(&flags[kFlagFallback], 1);
            double r = 0.0;
            for (int64_t i = 0; i < n; ++i) {
                r = r + norm_w(w_un[i], *s_in, np_recip);
                c[i] = r;
            }
        } else {
            st_wt_i(&flags[kFlagFallback], 0);
        }
    }
}

// Number of systematic positions at or below v: #{i in [0, n) :
// fl(fl(i (1/NP)) + ofs) <= v} (particle_filter.py:213-215; the positions are
// monotone in i).  An estimate from the inverse, then exact steps.
// The count is carried as a double (exact: n < 2^31), so the position of index
// i is fl(fl(i (1/NP)) + ofs) without an int64 -> double conversion per probe.
__device__ __forceinline__ int64_t positions_upto(const double v, const int64_t n,
                                                  const double rstep, const double ofs) {
    if (!(v >= ofs)) return 0;
    const double dn = (double)n;
    double e = floor((v - ofs) * dn) + 1.0;
    e = e < 0.0 ? 0.0 : (e > dn ? dn : e);
    while (e > 0.0 && (e - 1.0) * rstep + ofs > v) e = e - 1.0;
    while (e < dn && e * rstep + ofs <= v) e = e + 1.0;
    return (int64_t)e;
}

// Pass C for one tile, once the specials are folded: every c_i from the
// tile's classification and the folded specials, then the inverse resample
// map.  Source j serves the positions i with c_{j-1} < pos_i <= c_j (the
// lower_bound of particle_filter.py:218-220), a run [s_j, e_j) with s_j =
// #positions <= c_{j-1}.  A selected element marks the start of its run
// (mark[s_j] = tagged j) and gives every fused block whose first position lies
// in the run its carry (carry[fb] = j); positions past the last cumulative
// weight (the reference's IndexError) are marked with j = n.  The fused block
// then reads its marks and carry and takes a running max -- no search.
// wt: the folded data were handed over inside the same launch.
__device__ void wave_tile_expand(const int64_t b, const int64_t tile, const TileScan& ts,
                                 const int64_t n,
                                 const uint64_t* __restrict__ boffk,
                                 const int32_t* __restrict__ bofff, const uint64_t kofs,
                                 const int32_t fofs, const SpecialOut* __restrict__ so,
                                 double* __restrict__ c, int64_t* __restrict__ mark,
                                 int32_t* __restrict__ carry, const double ofs, const int64_t gen,
                                 const PredictConst& pc, const bool wt, const bool store_c = true) {
    const int lane = threadIdx.x & 63;
    auto ld_so = [wt, so](const int32_t m) { return wt ? ld_wt_struct(&so[m]) : so[m]; };
    const uint64_t bk0 = (wt ? ld_wt(&boffk[b]) : boffk[b]) + kofs;   // the tile's global offsets
    const int32_t bf0 = (wt ? ld_wt_i(&bofff[b]) : bofff[b]) + fofs;
    uint64_t kin = bk0 + ts.kex;
    int32_t m = bf0 + ts.fex;
    double out[kScanPer];
    SpecialOut p = ld_so(m > 0 ? m - 1 : 0);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        kin += ts.kk[k];
        if (ts.ff[k]) {
            p = ld_so(m);
            out[k] = p.cs;
            ++m;
        } else {
            out[k] = p.cs + (double)(kin - p.P) * ldexp(1.0, p.E - 52);
        }
    }
    const int64_t j0 = tile * kWaveTile + 8 * lane;
    if (store_c) {                                 // (the device-decided step needs only the marks)
#pragma unroll
        for (int h = 0; h < kScanPer; h += 2)      // c is padded to whole tiles
            *reinterpret_cast<double2*>(c + j0 + h) = double2{out[h], out[h + 1]};
    }
    PROBE_MAX(6);
    if (!mark) return;
    // ---- inverse map: runs of this lane's elements
    double cprev = __shfl_up(out[kScanPer - 1], 1, 64);
    if (lane == 0) {
        if (tile == 0) {
            cprev = -__builtin_inf();
        } else {                             // element j0 - 1 from its run's special
            const SpecialOut q = ld_so(bf0 - 1);
            cprev = q.cs + (double)(bk0 - q.P) * ldexp(1.0, q.E - 52);
        }
    }
    int64_t sj = positions_upto(cprev, n, pc.rstep, ofs);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t j = j0 + k;
        const bool ok = j < n;
        const int64_t ej = ok ? positions_upto(out[k], n, pc.rstep, ofs) : sj;
        // the fused blocks whose first position lies in the run
        int64_t flo = 0, fhi = 0, val = j;
        if (ok && ej > sj) {
            mark[sj] = gen | j;
            flo = (sj + kPartPer - 1) / kPartPer;
            fhi = (ej + kPartPer - 1) / kPartPer;
        }
        if (ok && j == n - 1 && ej < n) mark[ej] = gen | n;
        // carries, written by the whole wave (a heavy element may own many)
        uint64_t act = __ballot(fhi > flo);
        while (act) {
            const int l = __ffsll((unsigned long long)act) - 1;
            act &= act - 1;
            const int64_t L = __shfl(flo, l, 64), H = __shfl(fhi, l, 64);
            const int32_t J = (int32_t)__shfl(val, l, 64);
            for (int64_t f = L + lane; f < H; f += 64) carry[f] = J;
        }
        const bool beyond = ok && j == n - 1 && ej < n;
        if (__any(beyond)) {
            const int l = __ffsll((unsigned long long)__ballot(beyond)) - 1;
            const int64_t e2 = __shfl(ej, l, 64);
            for (int64_t f = (e2 + kPartPer - 1) / kPartPer + lane; f * kPartPer < n; f += 64)
                carry[f] = (int32_t)n;
        }
        sj = ej;
    }
    PROBE_MAX(7);
}

// the last block of pass A: block-total scans, then place + fold
template <int kC>
__device__ __forceinline__ void lean_last_block(uint64_t* __restrict__ bk, int32_t* __restrict__ bf,
                                                uint64_t* __restrict__ boffk,
                                                int32_t* __restrict__ bofff,
                                                uint64_t* __restrict__ ktot,
                                                int32_t* __restrict__ nspec, const int nblocks,
                                                const SpecialIn* __restrict__ stage,
                                                const int64_t n, SpecialOut* __restrict__ spec_out,
                                                int32_t* __restrict__ flags,
                                                const double* __restrict__ w_un,
                                                const double* __restrict__ s_in,
                                                const double np_recip, double* __restrict__ c) {
    __shared__ uint64_t shk[kScanThreads / 64 + 1];
    __shared__ int32_t shf[kScanThreads / 64 + 1];
    __shared__ int32_t s_off[kFoldTilesLds];
    PROBE_AT(1);
    block_scan_pair<kScanThreads, kC>(bk, boffk, ktot, bf, bofff, nspec, nblocks, shk, shf,
                                  nblocks <= kFoldTilesLds ? s_off : nullptr);
    __syncthreads();
    PROBE_AT(2);
    lean_place_fold(stage, boffk, bofff, nblocks, ld_wt_i(nspec), ld_wt(ktot), n, spec_out, flags,
                    w_un, s_in, np_recip, c, s_off);
    PROBE_AT(4);
}

// A stand-alone exact cumsum's run marks retired (pf_api.hip retire_scan_marks)
__global__ void mark_gen_bump_kernel(int32_t* __restrict__ flags) {
    flags[kFlagMarkGen] = flags[kFlagMarkGen] + 1;
}

// Pass A (two-launch form): classify and stage every tile; the last block
// scans the tile totals, places and folds.  (A grid-stride form over the
// co-resident blocks measured slower: 50 + 57 against 45 + 45 us at 2^23 --
// the passes are VALU-bound and the loop raised their VGPRs, 5 waves/SIMD.)
__global__ __launch_bounds__(kScanThreads) void scan_lean_classify_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_in, const double np_recip,
    const int64_t n, const double* __restrict__ boff, const double delta,
    SpecialIn* __restrict__ stage, uint64_t* __restrict__ bk, int32_t* __restrict__ bf,
    uint64_t* __restrict__ boffk, int32_t* __restrict__ bofff, uint64_t* __restrict__ ktot,
    int32_t* __restrict__ nspec, unsigned* __restrict__ counter, int32_t* __restrict__ flags,
    const int32_t force, SpecialOut* __restrict__ spec_out, double* __restrict__ c,
    const int ntiles) {
    if (!force && flags[kFlagResample] != 1) return;
    if (blockIdx.x == 0) PROBE_AT(0);
    const int64_t tile = (int64_t)blockIdx.x * kTilesPerBlock + (threadIdx.x >> 6);
    TileScan ts;
    uint64_t ktile = 0, kofs, kblk;
    int32_t ftile = 0, fofs, fblk;
    if (tile < ntiles)
        wave_tile_classify(w_un, *s_in, np_recip, n, tile, boff[tile], delta, ts, ktile, ftile);
    block_tile_offsets(ktile, ftile, kofs, fofs, kblk, fblk);
    if (tile < ntiles) wave_tile_stage(blockIdx.x, tile, ts, kofs, fofs, kblk, fblk, stage, bk, bf);
    else if (threadIdx.x == 0) {
        st_wt(&bk[blockIdx.x], kblk);
        st_wt_i(&bf[blockIdx.x], fblk);
    }
    PROBE_MAX(12);
    if (!arrive_last(counter)) return;
    lean_last_block<8>(bk, bf, boffk, bofff, ktot, nspec, (int)gridDim.x, stage, n, spec_out,
                       flags, w_un, s_in, np_recip, c);
}

// Pass C (two-launch form): the identical classification, then the expansion.
__global__ __launch_bounds__(kScanThreads) void scan_lean_expand_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_in, const double np_recip,
    const int64_t n, const double* __restrict__ boff, const double delta,
    const uint64_t* __restrict__ boffk, const int32_t* __restrict__ bofff,
    const SpecialOut* __restrict__ so, double* __restrict__ c, const int32_t* __restrict__ flags,
    const int32_t force, const StepIO io, const PredictConst pc, const uint64_t seed,
    int64_t* __restrict__ mark, int32_t* __restrict__ carry, const int ntiles) {
    if (!force && flags[kFlagResample] != 1) return;
    if (flags[kFlagFallback]) return;
    if (blockIdx.x == 0) PROBE_AT(5);
    const int64_t tile = (int64_t)blockIdx.x * kTilesPerBlock + (threadIdx.x >> 6);
    const double ofs = mark ? resample_offset(io.ofs[io.ctr[0]], pc.np_recip, seed, (uint32_t)io.ctr[1]) : 0.0;
    const int64_t gen = (int64_t)(uint32_t)flags[kFlagMarkGen] << 32;
    TileScan ts;
    uint64_t ktile = 0, kofs, kblk;
    int32_t ftile = 0, fofs, fblk;
    if (tile < ntiles)
        wave_tile_classify(w_un, *s_in, np_recip, n, tile, boff[tile], delta, ts, ktile, ftile);
    block_tile_offsets(ktile, ftile, kofs, fofs, kblk, fblk);
    PROBE_MAX(9);
    if (tile < ntiles)
        wave_tile_expand(blockIdx.x, tile, ts, n, boffk, bofff, kofs, fofs, so, c, mark, carry,
                         ofs, gen, pc, false, force != 0 || !mark);   // (device-decided: marks only)
}

// Passes A and C in ONE launch (NP up to the co-resident grid, checked on the
// host): classify and stage; the last block scans, places and folds and then
// releases the others, which waited on a write-through token with their
// tiles' classification still in registers, and every wave expands its tile.
// The wait is bounded: a token that never arrives sets status bit 3 and the
// block skips its expansion instead of hanging the device.
__global__ __launch_bounds__(kScanThreads) void scan_lean_merged_kernel(
    const double* __restrict__ w_un, const double* __restrict__ s_in, const double np_recip,
    const int64_t n, const double* __restrict__ boff, const double delta,
    SpecialIn* __restrict__ stage, uint64_t* __restrict__ bk, int32_t* __restrict__ bf,
    uint64_t* __restrict__ boffk, int32_t* __restrict__ bofff, uint64_t* __restrict__ ktot,
    int32_t* __restrict__ nspec, unsigned* __restrict__ counter, int32_t* __restrict__ flags,
    const int32_t force, SpecialOut* __restrict__ spec_out, double* __restrict__ c,
    const StepIO io, const PredictConst pc, const uint64_t seed, int64_t* __restrict__ mark,
    int32_t* __restrict__ carry, int32_t* __restrict__ token_word, const int ntiles) {
    if (!force && flags[kFlagResample] != 1) return;
    __shared__ int s_go;
    if (blockIdx.x == 0) PROBE_AT(0);
    const int32_t token = ld_wt_i(token_word) + 1;     // read before this block arrives
    const double ofs = resample_offset(io.ofs[io.ctr[0]], pc.np_recip, seed, (uint32_t)io.ctr[1]);
    const int64_t gen = (int64_t)(uint32_t)flags[kFlagMarkGen] << 32;
    const int64_t tile = (int64_t)blockIdx.x * kTilesPerBlock + (threadIdx.x >> 6);
    const bool active = tile < ntiles;
    TileScan ts;
    uint64_t ktile = 0, kofs, kblk;
    int32_t ftile = 0, fofs, fblk;
    if (active)
        wave_tile_classify(w_un, *s_in, np_recip, n, tile, boff[tile], delta, ts, ktile, ftile);
    block_tile_offsets(ktile, ftile, kofs, fofs, kblk, fblk);
    if (active) wave_tile_stage(blockIdx.x, tile, ts, kofs, fofs, kblk, fblk, stage, bk, bf);
    else if (threadIdx.x == 0) {
        st_wt(&bk[blockIdx.x], kblk);
        st_wt_i(&bf[blockIdx.x], fblk);
    }
    PROBE_MAX(12);
    if (arrive_last(counter)) {
        lean_last_block<4>(bk, bf, boffk, bofff, ktot, nspec, (int)gridDim.x, stage, n, spec_out,
                        flags, w_un, s_in, np_recip, c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st_wt_i(token_word, token);
            s_go = 1;
        }
    } else if (threadIdx.x == 0) {
        int go = 0;
        for (int it = 0; it < (1 << 22); ++it) {
            if (ld_wt_i(token_word) == token) {
                go = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!go) atomicOr(&flags[kFlagStatus], 8);   // token never came: skip, do not hang
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_go = go;
    }
    __syncthreads();
    if (blockIdx.x == 0) PROBE_AT(5);
    if (!active || !s_go || ld_wt_i(&flags[kFlagFallback])) return;
    wave_tile_expand(blockIdx.x, tile, ts, n, boffk, bofff, kofs, fofs, spec_out, c, mark, carry,
                     ofs, gen, pc,
                     true, force != 0);
}

// gather for the stand-alone resampling stage (particle_filter.py:216-222)
__global__ __launch_bounds__(256) void gather_kernel(
    const int64_t n, const int32_t* __restrict__ idx, const double* __restrict__ xs,
    const double* __restrict__ ys, const double* __restrict__ ts, double* __restrict__ xo,
    double* __restrict__ yo, double* __restrict__ to, double* __restrict__ w, const double np_recip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t j = idx[i];
    xo[i] = xs[j];
    yo[i] = ys[j];
    to[i] = ts[j];
    w[i] = np_recip;
}

// stand-alone systematic positions + lower_bound (particle_filter.py:213-221)
__global__ __launch_bounds__(256) void resample_search_kernel(
    const int64_t n, const double* __restrict__ c, int32_t* __restrict__ idx, const double step,
    const double ofs_host, const double np_recip, const uint64_t seed, const uint32_t stepno,
    int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double ofs = resample_offset(ofs_host, np_recip, seed, stepno);
    const double pos = (double)i * step + ofs;
    int64_t lo = lower_bound_c(c, n, pos);
    if (lo >= n) {
        lo = n - 1;
        atomicOr(&flags[kFlagStatus], 1);
    }
    idx[i] = (int32_t)lo;
}

}  // namespace slam
