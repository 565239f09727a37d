// rng_api.hip -- NumPy's legacy RandomState stream on the device (mt19937.hpp).
//
// A request (mt_enqueue) is four launches, none of which needs the host:
//   mt_round_kernel   when fewer words than a request can read lie ahead: R
//                     workgroups each generate S words of the untempered
//                     MT19937 sequence (one 624-word block per barrier) from
//                     their segment's pre-window, then jump that pre-window
//                     R S words ahead (mt_stream.hpp);
//   mt_count_kernel   per candidate pair (4 words): the polar test
//                     0 < x1^2 + x2^2 < 1, accepted candidates per block;
//   mt_emit_kernel    the block's offset (the counts of the blocks before it,
//                     summed by the block itself: no scan launch), the rank of
//                     every accepted candidate; the first P give the
//                     normals f x2, f x1 (f = sqrt(-2 log(r2) / r2), glibc's
//                     log), the P-th ends the draw;
//   mt_finish_kernel  the pre-draw doubles, the cached normal in slot 0, the
//                     new key / pos / cache exactly as NumPy leaves them.
// The draw order is NumPy's: legacy_gauss (legacy-distributions.c) returns
// f x2 and caches f x1; random_sample takes two words per double.
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "mt_stream.hpp"

namespace slam {

constexpr int kMtGenThreads = 640;   // one lane per word of a block
constexpr int kMtCandPerThread = 4;
constexpr int kMtCountThreads = 256;
constexpr int kMtCandPerBlock = kMtCountThreads * kMtCandPerThread;
// emit blocks sum their predecessors' counts themselves up to this many blocks
// (O(nb^2) reads in all); beyond, one prefix launch
#ifndef SLAM_MT_EMIT_SUM_MAX
#define SLAM_MT_EMIT_SUM_MAX 4096
#endif
constexpr int kMtEmitSumMax = SLAM_MT_EMIT_SUM_MAX;
// requests one parallel round feeds: the jump (~160 us, LDS-bound) is paid
// once per round, the sequential generation grows with it; 4 -> 16 took the
// device stream from 0.229 to 0.201 ms per 2^20-particle step, 16 -> 32 from
// 0.150 to 0.145, 32 -> 64 (round 4) from 0.121 to 0.118 (the ring is 2 GB
// at that request size, the one-time priming ~300 ms).  Larger requests feed
// fewer (at least 4) so that the ring stays within kMtRingWordsMax.
constexpr int64_t kMtRoundsAhead = 64;
constexpr int64_t kMtRingWordsMax = int64_t(1) << 29;     // 2 GB of words

// ------------------------------------------------------------------ kernels

// word i of the block after A, from A alone: the words it needs from its own
// block (X[n + 397] for i >= 227) are expanded through the recurrence, so a
// block is one parallel phase (one barrier) instead of three dependent ones
__device__ __forceinline__ uint32_t mt_block_word(const uint32_t* A, const int i) {
    constexpr int D = kMtN - kMtM;   // 227
    if (i < D) return mt_next(A[i], A[i + 1], A[i + kMtM]);
    if (i < 2 * D) {
        const int j = i - D;
        return mt_next(A[i], A[i + 1], mt_next(A[j], A[j + 1], A[j + kMtM]));
    }
    if (i < kMtN - 1) {
        const int j = i - D, k = j - D;
        const uint32_t p1 = mt_next(A[k], A[k + 1], A[k + kMtM]);
        return mt_next(A[i], A[i + 1], mt_next(A[j], A[j + 1], p1));
    }
    // i = 623: X[n + 1] is the new block's word 0, X[n + 397] its word 396
    const uint32_t w0 = mt_next(A[0], A[1], A[kMtM]);
    const int k = kMtM - 1 - D;      // 169
    const uint32_t w396 = mt_next(A[kMtM - 1], A[kMtM], mt_next(A[k], A[k + 1], A[k + kMtM]));
    return mt_next(A[kMtN - 1], w0, w396);
}

// LDS-only barrier: __syncthreads() would also wait for the ring stores of the
// block (a full store round trip per 624 words)
__device__ __forceinline__ void mt_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One round: segment r (workgroup r) = stream words [g1 + r S, g1 + (r + 1) S),
// generated from its pre-window seg[r]; then seg[r] <- the pre-window one round
// later (R > 1: jump-ahead by R S; R = 1: the segment's last block).  Runs only
// when fewer than `need` words lie ahead of the position.
__global__ __launch_bounds__(kMtGenThreads) void mt_round_kernel(
    const MtDeviceState* __restrict__ st, uint32_t* __restrict__ X, const int64_t cap,
    uint32_t* __restrict__ seg, const uint32_t* __restrict__ q_idx, const int32_t n_idx,
    const int64_t S, const int32_t R, const int64_t need) {
    extern __shared__ uint32_t sm[];
    const int64_t p = st->p, g1 = st->g1;
    if (g1 - p >= need) return;
    uint32_t* Wl = sm + 2 * kMtN;                       // Y[0 .. kMtConvWords] (R > 1)
    const int t = threadIdx.x;
    const int64_t m = g1 + (int64_t)blockIdx.x * S;     // the segment's first word
    uint32_t* sg = seg + (size_t)blockIdx.x * kMtN;
    // Y[0..623] = the pre-window (stream words m - 1 ...); stream word m + k = Y[k + 1]
    if (t < kMtN) {
        const uint32_t v = sg[t];
        sm[t] = v;
        if (R > 1) {
            Wl[t] = v;
            Wl[kMtConvWords + 1 + t] = 0u;              // the padding offset's window
        }
        if (t >= 1) X[(m + t - 1) & (cap - 1)] = v;
    }
    __syncthreads();
    const int64_t K = S / kMtN;
    int a = 0;
    for (int64_t b = 1; b <= K; ++b) {
        if (t < kMtN) {
            const uint32_t v = mt_block_word(sm + a * kMtN, t);
            sm[(a ^ 1) * kMtN + t] = v;
            const int64_t y = b * kMtN + t;
            if (y <= S) X[(m + y - 1) & (cap - 1)] = v;
            if (R > 1 && y < kMtConvWords + 1) Wl[y] = v;
        }
        mt_lds_barrier();
        a ^= 1;
    }
    if (t >= kMtN) return;
    if (R == 1) {
        sg[t] = sm[a * kMtN + t];                       // Y[S .. S + 623]
        return;
    }
    // pre-window R S words on: word j = XOR over the set bits i of q of Y[i + j]
    // (q's set bits as a list of 16-bit offsets, padded with an offset that
    // lands in the zero tail of Wl; 16 LDS reads in flight per round)
    uint32_t acc = 0;
    for (int k = 0; k < n_idx; k += 16) {
        uint32_t v[16];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t pr = q_idx[k / 2 + u];
            v[2 * u] = Wl[(pr & 0xffffu) + t];
            v[2 * u + 1] = Wl[(pr >> 16) + t];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc ^= v[u];
    }
    sg[t] = acc;
}

// Set-state priming: stream words [0, 624 + R S + 624) from the key in one
// workgroup, so that every segment's first pre-window can be read off.
__global__ __launch_bounds__(kMtGenThreads) void mt_prime_kernel(const uint32_t* __restrict__ key,
                                                                 uint32_t* __restrict__ X,
                                                                 const int64_t cap,
                                                                 const int64_t nblk) {
    __shared__ uint32_t buf[2][kMtN];
    const int t = threadIdx.x;
    if (t < kMtN) {
        const uint32_t v = key[t];
        buf[0][t] = v;
        X[t] = v;
    }
    __syncthreads();
    int a = 0;
    for (int64_t b = 1; b <= nblk; ++b) {
        if (t < kMtN) {
            const uint32_t v = mt_block_word(buf[a], t);
            buf[a ^ 1][t] = v;
            X[(b * kMtN + t) & (cap - 1)] = v;
        }
        mt_lds_barrier();
        a ^= 1;
    }
}

// seg[r] <- stream words [623 + r S, 623 + r S + 624) (the first round's pre-windows)
__global__ void mt_seed_segments_kernel(const uint32_t* __restrict__ X, const int64_t cap,
                                        uint32_t* __restrict__ seg, const int64_t S) {
    const int r = blockIdx.x;
    for (int j = threadIdx.x; j < kMtN; j += blockDim.x)
        seg[(size_t)r * kMtN + j] = X[(kMtN - 1 + (int64_t)r * S + j) & (cap - 1)];
}

__device__ __forceinline__ int64_t mt_pre_words(const int32_t* pre_flag, const int64_t n_pre) {
    return pre_flag ? (*pre_flag ? 2 : 0) : 2 * n_pre;
}

__device__ __forceinline__ uint32_t mt_word(const uint32_t* __restrict__ X, const int64_t k,
                                            const int64_t cap) {
    return mt_temper(X[k & (cap - 1)]);
}

// The kMtCandPerThread candidates of a lane, stream words w .. w + 15: five
// 16-byte loads of the 4-word-aligned window (the ring holds a power of two of
// words, so no load straddles its wrap) shifted by w & 3 (uniform across the
// grid: w = w0 + 4 c), instead of sixteen 4-byte loads; same words: candidate c is
// words w0 + 4c .. + 3 (two legacy doubles, the polar test)
static_assert(kMtCandPerThread == 4, "four candidates = sixteen words per lane");
__device__ __forceinline__ void mt_lane_candidates(const uint32_t* __restrict__ X, const int64_t w,
                                                   const int64_t cap, double x1[4], double x2[4],
                                                   double r2[4], bool ok[4]) {
    const int64_t base = w & ~(int64_t)3;
    const int a = (int)(w & 3);
    uint32_t v[20];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint4 q = *reinterpret_cast<const uint4*>(X + ((base + 4 * i) & (cap - 1)));
        v[4 * i] = q.x;
        v[4 * i + 1] = q.y;
        v[4 * i + 2] = q.z;
        v[4 * i + 3] = q.w;
    }
    uint32_t u[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        u[i] = mt_temper(a == 0 ? v[i] : a == 1 ? v[i + 1] : a == 2 ? v[i + 2] : v[i + 3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x1[k] = 2.0 * mt_legacy_double(u[4 * k], u[4 * k + 1]) - 1.0;
        x2[k] = 2.0 * mt_legacy_double(u[4 * k + 2], u[4 * k + 3]) - 1.0;
        r2[k] = x1[k] * x1[k] + x2[k] * x2[k];
        ok[k] = !(r2[k] >= 1.0 || r2[k] == 0.0);
    }
}

__device__ __forceinline__ int64_t mt_pairs(const MtDeviceState* st, const int64_t g) {
    const int64_t m = g - (st->has_gauss ? 1 : 0);
    return m > 0 ? (m + 1) / 2 : 0;
}

// inclusive prefix over the block's threads (kMtCountThreads), total via *tot
__device__ __forceinline__ int mt_block_scan(int v, int* tot) {
    __shared__ int s_w[kMtCountThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    if (lane == 63) s_w[wave] = v;
    __syncthreads();
    int add = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kMtCountThreads / 64; ++w) {
        add += (w < wave) ? s_w[w] : 0;
        all += s_w[w];
    }
    *tot = all;
    return v + add;
}

__global__ __launch_bounds__(kMtCountThreads) void mt_count_kernel(
    MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X, const int64_t cap,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const int64_t ncand,
    unsigned* __restrict__ bcnt, const int64_t round_words, const int64_t need) {
    const int64_t p = st->p;
    const int64_t w0 = p + mt_pre_words(pre_flag, n_pre);
    const int64_t c0 = (int64_t)blockIdx.x * kMtCandPerBlock + threadIdx.x * kMtCandPerThread;
    int cnt = 0;
    double x1[kMtCandPerThread], x2[kMtCandPerThread], r2[kMtCandPerThread];
    bool ok[kMtCandPerThread];
    mt_lane_candidates(X, w0 + 4 * c0, cap, x1, x2, r2, ok);
#pragma unroll
    for (int k = 0; k < kMtCandPerThread; ++k) cnt += (c0 + k < ncand && ok[k]) ? 1 : 0;
    int tot;
    (void)mt_block_scan(cnt, &tot);
    if (threadIdx.x == 0) {
        bcnt[blockIdx.x] = (unsigned)tot;
        // the round launched before this pass generated R S words if it ran
        if (blockIdx.x == 0 && st->g1 - p < need) st->g1 += round_words;
    }
}

// exclusive prefix of the count blocks' accepted pairs (one workgroup)
__global__ __launch_bounds__(1024) void mt_bcnt_prefix_kernel(const unsigned* __restrict__ bcnt,
                                                              const int64_t nb,
                                                              unsigned* __restrict__ bpre) {
    __shared__ unsigned s_w[16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t per = (nb + 1023) / 1024, b0 = (int64_t)t * per;
    unsigned loc = 0;
    for (int64_t k = 0; k < per; ++k)
        if (b0 + k < nb) loc += bcnt[b0 + k];
    unsigned inc = loc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    unsigned base = 0;
    for (int w = 0; w < wave; ++w) base += s_w[w];
    unsigned ex = base + inc - loc;
    for (int64_t k = 0; k < per; ++k)
        if (b0 + k < nb) {
            bpre[b0 + k] = ex;
            ex += bcnt[b0 + k];
        }
    if (t == 1023) bpre[nb] = base + inc;
}

__global__ __launch_bounds__(kMtCountThreads) void mt_emit_kernel(
    MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X, const int64_t cap,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const int64_t ncand,
    const unsigned* __restrict__ bcnt, const unsigned* __restrict__ bpre, const int64_t nb,
    const int64_t g, const GlibcLogTable* __restrict__ tab, double* __restrict__ normals,
    int32_t* __restrict__ status) {
    const int64_t pw = mt_pre_words(pre_flag, n_pre);
    const int64_t w0 = st->p + pw;
    const int h = st->has_gauss ? 1 : 0;
    const int64_t P = mt_pairs(st, g);
    const int64_t c0 = (int64_t)blockIdx.x * kMtCandPerBlock + threadIdx.x * kMtCandPerThread;
    // the accepted pairs of the blocks before this one (integer sums: any order);
    // block 0 sums every block's count for the short-draw check.  Up to
    // kMtEmitSumMax blocks each block sums its predecessors' counts itself
    // (no scan launch); beyond, mt_bcnt_prefix_kernel's prefix (bpre) keeps
    // the reads linear in the block count
    const int64_t nsum = bpre ? 0 : (blockIdx.x == 0 ? nb : (int64_t)blockIdx.x);
    int64_t part = 0;
    if (bpre && threadIdx.x == 0) part = bpre[blockIdx.x == 0 ? nb : blockIdx.x];
    for (int64_t i = threadIdx.x; i < nsum; i += kMtCountThreads) part += bcnt[i];
    double x1[kMtCandPerThread], x2[kMtCandPerThread], r2[kMtCandPerThread];
    bool acc[kMtCandPerThread];
    int cnt = 0;
    mt_lane_candidates(X, w0 + 4 * c0, cap, x1, x2, r2, acc);
#pragma unroll
    for (int k = 0; k < kMtCandPerThread; ++k) {
        acc[k] = acc[k] && c0 + k < ncand;
        cnt += acc[k] ? 1 : 0;
    }
    __shared__ long long s_part[kMtCountThreads / 64];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) part += __shfl_xor(part, d, 64);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = part;
    int tot;
    const int incl = mt_block_scan(cnt, &tot);          // (its barrier publishes s_part)
    int64_t before = 0;
#pragma unroll
    for (int w = 0; w < kMtCountThreads / 64; ++w) before += s_part[w];
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            const bool shrt = before < P;
            st->short_draw = shrt ? 1 : 0;
            if (shrt && status) atomicOr(status, 256);
        }
        before = 0;
    }
    int64_t q = before + incl - cnt;
    if (q >= P) return;
#pragma unroll
    for (int k = 0; k < kMtCandPerThread; ++k) {
        if (!acc[k]) continue;
        if (q < P) {
            const double f = sqrt(-2.0 * glibc_log(r2[k], *tab) / r2[k]);
            const int64_t k1 = h + 2 * q;
            if (k1 < g) normals[k1] = f * x2[k];
            if (k1 + 1 < g) normals[k1 + 1] = f * x1[k];
            else st->new_gauss = f * x1[k];            // odd remainder: NumPy's cached normal
            if (q == P - 1) st->j_end = pw + 4 * (c0 + k + 1);
        }
        ++q;
    }
}

__global__ __launch_bounds__(kMtGenThreads) void mt_finish_kernel(
    MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X, const int64_t cap,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const double pre_scale,
    double* __restrict__ pre_out, const int32_t* __restrict__ pre_index, const int64_t g,
    double* __restrict__ normals) {
    const int64_t p = st->p;
    const int64_t pw = mt_pre_words(pre_flag, n_pre);
    const int h = st->has_gauss ? 1 : 0;
    const int64_t P = mt_pairs(st, g);
    // pre-draw doubles (random_sample): stream words p + 2k, p + 2k + 1
    if (pre_flag) {
        if (threadIdx.x == 0 && pre_out) {
            double* o = pre_out + (pre_index ? *pre_index : 0);
            *o = *pre_flag ? mt_legacy_double(mt_word(X, p, cap), mt_word(X, p + 1, cap)) * pre_scale
                           : (double)NAN;
        }
    } else if (pre_out) {
        for (int64_t k = threadIdx.x; k < n_pre; k += blockDim.x)
            pre_out[k] = mt_legacy_double(mt_word(X, p + 2 * k, cap), mt_word(X, p + 2 * k + 1, cap)) *
                         pre_scale;
    }
    __syncthreads();                                    // every lane has read st->p
    if (threadIdx.x == 0) {
        if (h && g > 0) normals[0] = st->gauss;
        st->p = p + (P > 0 ? st->j_end : pw);
        if (g > 0) {
            const int64_t m = g - h;
            const bool odd = m > 0 && (m & 1);
            st->has_gauss = odd ? 1 : 0;
            st->gauss = odd ? st->new_gauss : 0.0;
        }
    }
}

// ------------------------------------------------------------- host side

namespace {

// upper bound on the candidate pairs one request of g normals examines:
// the expected P / (pi/4) plus 12 standard deviations of the negative binomial
int64_t cand_bound(int64_t g) {
    const double P = (double)((g + 1) / 2);
    const double p = 0.7853981633974483;
    const double mean = P / p, sd = std::sqrt(P * (1.0 - p)) / p;
    return (int64_t)std::ceil(mean + 12.0 * sd) + 64;
}

// ---- MT19937's characteristic polynomial and jump polynomials (GF(2))
typedef std::vector<uint64_t> Bits;

inline int bit_of(const Bits& v, size_t i) { return (int)((v[i >> 6] >> (i & 63)) & 1u); }

// dst ^= src << sh (bit shift toward higher degree), dst/src of equal length
void xor_shifted(Bits& dst, const Bits& src, size_t sh) {
    const size_t q = sh >> 6, r = sh & 63, W = dst.size();
    for (size_t w = W; w-- > q;) {
        uint64_t v = src[w - q] << r;
        if (r && w >= q + 1) v |= src[w - q - 1] >> (64 - r);
        dst[w] ^= v;
    }
}

// Berlekamp-Massey over GF(2): the minimal polynomial of the bit sequence s
// as phi(x) = sum_i C_i x^(L - i) (bits 0 .. L), and its degree L.
Bits berlekamp_massey(const std::vector<uint8_t>& s, int& L_out) {
    const size_t n = s.size(), W = (n + 127) / 64 + 2;
    Bits R(W + 2, 0);                                    // reversed sequence
    for (size_t t = 0; t < n; ++t)
        if (s[n - 1 - t]) R[t >> 6] |= 1ull << (t & 63);
    auto window = [&](size_t off, size_t w) -> uint64_t {
        const size_t bit = off + 64 * w, qq = bit >> 6, rr = bit & 63;
        const uint64_t lo = qq < R.size() ? R[qq] : 0, hi = qq + 1 < R.size() ? R[qq + 1] : 0;
        return rr ? (lo >> rr) | (hi << (64 - rr)) : lo;
    };
    Bits C(W, 0), B(W, 0), T;
    C[0] = B[0] = 1;
    int L = 0;
    size_t m = 1;
    for (size_t k = 0; k < n; ++k) {
        uint64_t acc = 0;                                // s_k + sum_i C_i s_(k-i)
        for (size_t w = 0; w <= (size_t)L / 64; ++w) acc ^= C[w] & window(n - 1 - k, w);
        if (!__builtin_parityll(acc)) {
            ++m;
            continue;
        }
        if ((size_t)2 * L <= k) {
            T = C;
            xor_shifted(C, B, m);
            L = (int)(k + 1) - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, m);
            ++m;
        }
    }
    L_out = L;
    Bits phi((size_t)L / 64 + 2, 0);
    for (int i = 0; i <= L; ++i)
        if (bit_of(C, i)) phi[(size_t)(L - i) >> 6] |= 1ull << ((L - i) & 63);
    return phi;
}

struct Gf2Mod {
    int L = 0;
    size_t W = 0;                                        // words of a residue
    Bits phi;
    void reduce(Bits& r) const {                          // r: 2 W + 2 words, bits >= L cleared
        for (long bit = (long)(r.size() * 64) - 1; bit >= L; --bit) {
            if (!((r[(size_t)bit >> 6] >> (bit & 63)) & 1u)) continue;
            const size_t d = (size_t)bit - (size_t)L;
            // r ^= phi << d
            const size_t q = d >> 6, rr = d & 63;
            for (size_t w = 0; w < phi.size() && w + q < r.size(); ++w) {
                r[w + q] ^= phi[w] << rr;
                if (rr && w + q + 1 < r.size()) r[w + q + 1] ^= phi[w] >> (64 - rr);
            }
        }
    }
    Bits sqr(const Bits& a) const {
        Bits r(2 * W + 2, 0);
        for (size_t w = 0; w < W; ++w) {
            uint64_t lo = 0, hi = 0;
            for (int k = 0; k < 32; ++k) {
                lo |= ((a[w] >> k) & 1ull) << (2 * k);
                hi |= ((a[w] >> (32 + k)) & 1ull) << (2 * k);
            }
            r[2 * w] = lo;
            r[2 * w + 1] = hi;
        }
        reduce(r);
        r.resize(W);
        return r;
    }
    Bits mulx(const Bits& a) const {
        Bits r(2 * W + 2, 0);
        for (size_t w = 0; w < W; ++w) {
            r[w] |= a[w] << 1;
            r[w + 1] |= a[w] >> 63;
        }
        reduce(r);
        r.resize(W);
        return r;
    }
    Bits xpow(uint64_t E) const {                          // x^E mod phi
        Bits r(W, 0);
        r[0] = 1;
        for (int b = 63; b >= 0; --b) {
            r = sqr(r);
            if ((E >> b) & 1u) r = mulx(r);
        }
        return r;
    }
};

// phi from the most significant bit of the stream of NumPy's default seed
// (any non-zero state has the same minimal polynomial: phi is irreducible)
int mt_phi(Gf2Mod& out) {
    static std::mutex mu;
    static Gf2Mod G;
    static bool ok = false;
    std::lock_guard<std::mutex> lock(mu);
    if (!ok) {
        std::vector<uint32_t> X(kMtN);
        X[0] = 5489u;
        for (int i = 1; i < kMtN; ++i) X[i] = 1812433253u * (X[i - 1] ^ (X[i - 1] >> 30)) + (uint32_t)i;
        const size_t n = 2 * (size_t)kMtDeg + 256;
        X.resize(n);
        for (size_t k = kMtN; k < n; ++k) X[k] = mt_next(X[k - kMtN], X[k - kMtN + 1], X[k - kMtN + kMtM]);
        std::vector<uint8_t> s(n);
        for (size_t k = 0; k < n; ++k) s[k] = (uint8_t)(X[k] >> 31);
        int L = 0;
        Bits phi = berlekamp_massey(s, L);
        if (L != kMtDeg) return fail(SLAM_ERR_ARG, "mt19937: characteristic polynomial of wrong degree");
        G.L = L;
        G.W = (size_t)kMtQWords;
        G.phi = phi;
        ok = true;
    }
    out = G;
    return SLAM_OK;
}

int jump_poly(uint64_t J, Bits& q) {
    Gf2Mod G;
    const int rc = mt_phi(G);
    if (rc) return rc;
    q = G.xpow(J);
    return SLAM_OK;
}

typedef double (*log_fn)(double);

bool table_matches(const GlibcLogTable& T, log_fn lg) {
    // deterministic probes: both branches, every table entry, the polar range
    uint64_t s = 0x9E3779B97F4A7C15ULL;
    auto next = [&s]() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    };
    for (int k = 0; k < (1 << 16); ++k) {
        const uint64_t r = next();
        double x;
        switch (k & 3) {
            case 0: x = (double)(r >> 11) * 0x1p-53; break;                       // (0, 1)
            case 1: x = 1.0 - (double)(r >> 11) * 0x1p-57; break;                 // near 1 below
            case 2: x = 1.0 + (double)(r >> 11) * 0x1p-57; break;                 // near 1 above
            default: x = std::ldexp(0.5 + (double)(r >> 12) * 0x1p-53, (int)(r % 200) - 100);
        }
        if (!(x > 0.0)) continue;
        const double a = glibc_log(x, T), b = lg(x);
        if (mt_bits(a) != mt_bits(b)) return false;
    }
    return true;
}

int load_table(GlibcLogTable* out) {
    void* sym = dlsym(RTLD_DEFAULT, "log");
    if (!sym) return fail(SLAM_ERR_ARG, "glibc log table: log() not found in this process");
    Dl_info info;
    if (!dladdr(sym, &info) || !info.dli_fname)
        return fail(SLAM_ERR_ARG, "glibc log table: cannot locate the C library providing log()");
    FILE* f = std::fopen(info.dli_fname, "rb");
    if (!f) return fail(SLAM_ERR_ARG, std::string("glibc log table: cannot read ") + info.dli_fname);
    std::vector<unsigned char> img;
    unsigned char chunk[1 << 16];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) img.insert(img.end(), chunk, chunk + got);
    std::fclose(f);
    // struct log_data {ln2hi, ln2lo, poly[5], poly1[11], tab[128][2], tab2[128][2]}
    const uint64_t ln2hi = 0x3fe62e42fefa3800ULL, ln2lo = 0x3d2ef35793c76730ULL;
    const size_t need = sizeof(double) * (18 + 512);
    log_fn lg = reinterpret_cast<log_fn>(sym);
    for (size_t o = 0; o + need <= img.size(); o += 8) {
        uint64_t w0, w1;
        std::memcpy(&w0, &img[o], 8);
        if (w0 != ln2hi) continue;
        std::memcpy(&w1, &img[o + 8], 8);
        if (w1 != ln2lo) continue;
        double d[18 + 512];
        std::memcpy(d, &img[o], need);
        if (d[7] != -0.5 || !(std::fabs(d[2] + 0.5) < 1e-12)) continue;   // B[0] = -0.5, A[0] ~ -0.5
        GlibcLogTable T{};
        T.ln2hi = d[0];
        T.ln2lo = d[1];
        for (int k = 0; k < 5; ++k) T.poly[k] = d[2 + k];
        for (int k = 0; k < 11; ++k) T.poly1[k] = d[7 + k];
        for (int k = 0; k < 256; ++k) T.tab[k] = d[18 + k];
        for (int k = 0; k < 256; ++k) T.tab2[k] = d[18 + 256 + k];
        for (int fb = 1; fb >= 0; --fb) {
            T.fma_build = fb;
            if (table_matches(T, lg)) {
                *out = T;
                return SLAM_OK;
            }
        }
    }
    return fail(SLAM_ERR_ARG, std::string("glibc log table: no table in ") + info.dli_fname +
                                  " reproduces its log() bit for bit (not glibc 2.28+'s log?)");
}

}  // namespace

int glibc_log_table(GlibcLogTable* out) {
    static std::mutex mu;
    static bool ok = false;
    static GlibcLogTable T;
    std::lock_guard<std::mutex> lock(mu);
    if (!ok) {
        const int rc = load_table(&T);
        if (rc) return rc;
        ok = true;
    }
    *out = T;
    return SLAM_OK;
}

void mt_free(MtBuffers& b) {
    void* ps[] = {b.st, b.tab, b.X, b.seg, b.q, b.bcnt, b.bpre, b.normals, b.pre};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    b = MtBuffers{};
}

namespace {

size_t round_lds_bytes(int32_t R) {
    return sizeof(uint32_t) * (2 * (size_t)kMtN + (R > 1 ? (size_t)kMtConvWords + 1 + kMtN : 0));
}

// the first round's pre-windows from the key (one workgroup, R S + 1248 words)
int mt_prime(const MtBuffers& b, const uint32_t* key_dev, hipStream_t s) {
    const int64_t nblk = (b.R * b.S + 2 * kMtN) / kMtN + 1;
    mt_prime_kernel<<<1, kMtGenThreads, 0, s>>>(key_dev, b.X, b.cap, nblk);
    mt_seed_segments_kernel<<<b.R, 256, 0, s>>>(b.X, b.cap, b.seg, b.S);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

}  // namespace

int mt_reserve(MtBuffers& b, int64_t g_cap, int64_t pre_cap, int device) {
    if (b.st && g_cap <= b.g_cap && pre_cap <= b.pre_cap) return SLAM_OK;
    g_cap = std::max<int64_t>(g_cap, b.g_cap);
    pre_cap = std::max<int64_t>(pre_cap, b.pre_cap);
    SLAM_HIP_TRY(hipSetDevice(device));
    // a regrow keeps the stream where it is
    std::vector<uint32_t> key(kMtN, 0);
    int32_t pos = kMtN, hg = 0;
    double gs = 0.0;
    const bool had = b.st != nullptr;
    int rc = SLAM_OK;
    if (had && (rc = mt_get_state(b, key.data(), &pos, &hg, &gs, nullptr))) return rc;
    GlibcLogTable T;
    rc = glibc_log_table(&T);
    if (rc) return rc;
    mt_free(b);
    b.device = device;
    b.g_cap = g_cap;
    b.pre_cap = pre_cap;
    b.cand_cap = cand_bound(std::max<int64_t>(g_cap, 1));
    b.nb_count = (b.cand_cap + kMtCandPerBlock - 1) / kMtCandPerBlock;
    // a request reads at most 2 pre_cap + 4 cand_cap words past the position,
    // then the block it ends in (the state NumPy reports)
    b.need = 2 * pre_cap + 4 * b.cand_cap + 2 * kMtN;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    b.R = (int32_t)std::min<int64_t>(std::min<int64_t>(kMtMaxSegs, cus), b.need / kMtMinSeg);
    if (b.R < 1) b.R = 1;
    // R > 1: a round covers kMtRoundsAhead requests, so the jump (a fixed
    // cost per round) is paid once per that many requests
    // segment length and live words for a given number of requests per round:
    // the ring holds [p - 624, g1 + R S) while a round writes (it runs only
    // when g1 - p < need) and [p - 624, g1) with g1 - p < need + R S after it,
    // so need + R S + a few blocks (round 5; the round-4 bound counted R S twice)
    auto seg_len = [&](int64_t ahead) {
        const int64_t span = b.R > 1 ? ahead * b.need : b.need;
        int64_t S = (span + (int64_t)b.R * kMtN - 1) / ((int64_t)b.R * kMtN) * kMtN;
        if (b.R > 1 && S < kMtMinSeg) S = kMtMinSeg;
        return std::max<int64_t>(S, kMtN);
    };
    auto live_words = [&](int64_t S) {
        const int64_t RS = (int64_t)b.R * S;
        return std::max<int64_t>(b.need + RS + 4 * kMtN, RS + 3 * kMtN);
    };
    int64_t ahead = kMtRoundsAhead;
    while (ahead > 4 && live_words(seg_len(ahead)) > kMtRingWordsMax) ahead >>= 1;
    if (const char* e = std::getenv("SLAM_MT_ROUNDS_AHEAD")) {   // diagnostic A/B
        const long v = std::atol(e);
        if (v >= 1 && v <= 64) ahead = v;
    }
    b.S = seg_len(ahead);
    const int64_t RS = (int64_t)b.R * b.S;
    const int64_t live = live_words(b.S);
    b.cap = 1;
    while (b.cap < live) b.cap <<= 1;                    // a power of two: index & (cap - 1)
    SLAM_HIP_TRY(hipMalloc(&b.st, sizeof(MtDeviceState)));
    SLAM_HIP_TRY(hipMalloc(&b.tab, sizeof(GlibcLogTable)));
    SLAM_HIP_TRY(hipMalloc(&b.X, sizeof(uint32_t) * (size_t)b.cap));
    SLAM_HIP_TRY(hipMalloc(&b.seg, sizeof(uint32_t) * kMtN * (size_t)b.R));
    SLAM_HIP_TRY(hipMalloc(&b.q, sizeof(uint32_t) * (kMtDeg / 2 + 16)));
    SLAM_HIP_TRY(hipMalloc(&b.bcnt, sizeof(unsigned) * (size_t)std::max<int64_t>(b.nb_count, 1)));
    SLAM_HIP_TRY(hipMalloc(&b.bpre, sizeof(unsigned) * (size_t)(b.nb_count + 1)));
    SLAM_HIP_TRY(hipMalloc(&b.normals, sizeof(double) * (size_t)std::max<int64_t>(g_cap, 1)));
    SLAM_HIP_TRY(hipMalloc(&b.pre, sizeof(double) * (size_t)std::max<int64_t>(pre_cap, 1)));
    SLAM_HIP_TRY(hipMemcpy(b.tab, &T, sizeof(T), hipMemcpyHostToDevice));
    b.n_idx = 0;
    if (b.R > 1) {
        Bits q;
        if ((rc = jump_poly((uint64_t)RS, q))) return rc;
        std::vector<uint16_t> idx;
        for (int i = 0; i < kMtDeg; ++i)
            if (bit_of(q, (size_t)i)) idx.push_back((uint16_t)i);
        while (idx.size() % 16) idx.push_back((uint16_t)(kMtConvWords + 1));   // -> zero words
        b.n_idx = (int32_t)idx.size();
        SLAM_HIP_TRY(hipMemcpy(b.q, idx.data(), sizeof(uint16_t) * idx.size(), hipMemcpyHostToDevice));
    }
    const size_t lds = round_lds_bytes(b.R);
    if (lds > 64 * 1024)
        SLAM_HIP_TRY(hipFuncSetAttribute((const void*)mt_round_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return had ? mt_set_state(b, key.data(), pos, hg, gs, nullptr) : SLAM_OK;
}

int mt_set_state(MtBuffers& b, const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss,
                 hipStream_t s) {
    SLAM_ARG_CHECK(b.st && key, "mt19937 state: no buffers / key");
    SLAM_ARG_CHECK(pos >= 0 && pos <= kMtN, "mt19937 state: pos outside [0, 624]");
    SLAM_HIP_TRY(hipSetDevice(b.device));
    MtDeviceState h{};
    h.p = pos;
    h.g1 = kMtN;                                          // the key itself
    h.has_gauss = has_gauss ? 1 : 0;
    h.gauss = has_gauss ? gauss : 0.0;
    SLAM_HIP_TRY(hipMemcpyAsync(b.st, &h, sizeof(h), hipMemcpyHostToDevice, s));
    // the key is staged in seg[0] for the priming pass (which reads it first
    // and then the seeding pass overwrites seg)
    SLAM_HIP_TRY(hipMemcpyAsync(b.seg, key, sizeof(uint32_t) * kMtN, hipMemcpyHostToDevice, s));
    const int rc = mt_prime(b, b.seg, s);
    if (rc) return rc;
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    return SLAM_OK;
}

int mt_get_state(const MtBuffers& b, uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss,
                 hipStream_t s) {
    SLAM_ARG_CHECK(b.st, "mt19937 state: no buffers");
    SLAM_HIP_TRY(hipSetDevice(b.device));
    MtDeviceState h;
    SLAM_HIP_TRY(hipMemcpyAsync(&h, b.st, sizeof(h), hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    // NumPy's (key, pos): the block holding the next word; pos = 624 when the
    // last draw ended on a block boundary (it regenerates lazily)
    int64_t blk;
    int32_t ps;
    if (h.p > 0 && h.p % kMtN == 0) {
        blk = h.p / kMtN - 1;
        ps = kMtN;
    } else {
        blk = h.p / kMtN;
        ps = (int32_t)(h.p % kMtN);
    }
    if (key) {
        SLAM_ARG_CHECK((blk + 1) * kMtN <= h.g1, "mt19937 state: block not generated (internal)");
        const int64_t k0 = (blk * kMtN) & (b.cap - 1);
        const int64_t n0 = std::min<int64_t>(kMtN, b.cap - k0);   // the ring may wrap inside the block
        SLAM_HIP_TRY(hipMemcpyAsync(key, b.X + k0, sizeof(uint32_t) * n0, hipMemcpyDeviceToHost, s));
        if (n0 < kMtN)
            SLAM_HIP_TRY(hipMemcpyAsync(key + n0, b.X, sizeof(uint32_t) * (kMtN - n0),
                                        hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
    }
    if (pos) *pos = ps;
    if (has_gauss) *has_gauss = h.has_gauss;
    if (gauss) *gauss = h.gauss;
    return SLAM_OK;
}

int mt_enqueue(const MtBuffers& b, int64_t n_pre, const int32_t* pre_flag, double pre_scale,
               double* pre_out, const int32_t* pre_index, int64_t g, int32_t* status, hipStream_t s) {
    SLAM_ARG_CHECK(b.st, "mt19937 draw: no buffers");
    SLAM_ARG_CHECK(g >= 0 && g <= b.g_cap && n_pre >= 0 && n_pre <= b.pre_cap &&
                       (pre_flag == nullptr || b.pre_cap >= 1),
                   "mt19937 draw: request larger than the reserved buffers");
    const int64_t ncand = g > 0 ? cand_bound(g) : 0;
    SLAM_ARG_CHECK(ncand <= b.cand_cap, "mt19937 draw: candidate buffers too small");
    const int64_t RS = (int64_t)b.R * b.S;
    mt_round_kernel<<<b.R, kMtGenThreads, round_lds_bytes(b.R), s>>>(b.st, b.X, b.cap, b.seg, b.q,
                                                                   b.n_idx, b.S, b.R, b.need);
    SLAM_HIP_TRY(hipGetLastError());
    const unsigned nbc = (unsigned)((ncand + kMtCandPerBlock - 1) / kMtCandPerBlock);
    mt_count_kernel<<<std::max(nbc, 1u), kMtCountThreads, 0, s>>>(b.st, b.X, b.cap, pre_flag, n_pre,
                                                                   ncand, b.bcnt, RS, b.need);
    const bool pre_scan = nbc > (unsigned)kMtEmitSumMax;
    if (pre_scan) mt_bcnt_prefix_kernel<<<1, 1024, 0, s>>>(b.bcnt, (int64_t)nbc, b.bpre);
    if (nbc > 0)
        mt_emit_kernel<<<nbc, kMtCountThreads, 0, s>>>(b.st, b.X, b.cap, pre_flag, n_pre, ncand,
                                                       b.bcnt, pre_scan ? b.bpre : nullptr,
                                                       (int64_t)nbc, g, b.tab, b.normals, status);
    SLAM_HIP_TRY(hipGetLastError());
    mt_finish_kernel<<<1, kMtGenThreads, 0, s>>>(b.st, b.X, b.cap, pre_flag, n_pre, pre_scale, pre_out,
                                                 pre_index, g, b.normals);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int mt_jump_window_host(const uint32_t* win, uint64_t J, uint32_t* out) {
    Bits q;
    int rc = jump_poly(J, q);
    if (rc) return rc;
    std::vector<uint32_t> Y(win, win + kMtN);
    Y.resize(kMtConvWords + 1);
    for (size_t k = kMtN; k < Y.size(); ++k) Y[k] = mt_next(Y[k - kMtN], Y[k - kMtN + 1], Y[k - kMtN + kMtM]);
    for (int j = 0; j < kMtN; ++j) {
        uint32_t acc = 0;
        for (int i = 0; i < kMtDeg; ++i)
            if (bit_of(q, (size_t)i)) acc ^= Y[(size_t)i + j];
        out[j] = acc;
    }
    return SLAM_OK;
}

}  // namespace slam

using namespace slam;

// ------------------------------------------------------- standalone stream

struct slam_mt {
    int device = 0;
    hipStream_t stream = nullptr;
    MtBuffers b;
    int32_t* status = nullptr;
};

extern "C" {

int slam_glibc_log(int64_t n, const double* x, double* out) {
    SLAM_ARG_CHECK(n >= 0 && (n == 0 || (x && out)), "slam_glibc_log: bad arguments");
    GlibcLogTable T;
    const int rc = glibc_log_table(&T);
    if (rc) return rc;
    for (int64_t i = 0; i < n; ++i) out[i] = glibc_log(x[i], T);
    return SLAM_OK;
}

int slam_mt_jump_window(const uint32_t* window, uint64_t n_words, uint32_t* out) {
    SLAM_ARG_CHECK(window && out, "slam_mt_jump_window: NULL argument");
    return mt_jump_window_host(window, n_words, out);
}

int slam_mt_create(const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss, int device,
                   slam_mt** out) {
    SLAM_ARG_CHECK(key && out, "slam_mt_create: NULL argument");
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev, "slam_mt_create: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    slam_mt* h = new slam_mt;
    h->device = device;
    int rc;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&h->status, sizeof(int32_t)) != hipSuccess) {
        rc = fail(SLAM_ERR_HIP, "slam_mt_create: stream / status allocation failed");
    } else if ((rc = mt_reserve(h->b, 1, 1, device)) == SLAM_OK) {
        rc = mt_set_state(h->b, key, pos, has_gauss, gauss, h->stream);
    }
    if (rc) {
        mt_free(h->b);
        if (h->status) (void)hipFree(h->status);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return rc;
    }
    *out = h;
    return SLAM_OK;
}

int slam_mt_destroy(slam_mt* h) {
    if (!h) return SLAM_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    mt_free(h->b);
    if (h->status) (void)hipFree(h->status);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SLAM_OK;
}

int slam_mt_set_state(slam_mt* h, const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss) {
    SLAM_ARG_CHECK(h && key, "slam_mt_set_state: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    return mt_set_state(h->b, key, pos, has_gauss, gauss, h->stream);
}

int slam_mt_get_state(slam_mt* h, uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss) {
    SLAM_ARG_CHECK(h, "slam_mt_get_state: NULL handle");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    return mt_get_state(h->b, key, pos, has_gauss, gauss, h->stream);
}

static int mt_draw(slam_mt* h, int64_t n_pre, int64_t g, double* pre_host, double* g_host) {
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = mt_reserve(h->b, std::max<int64_t>(g, 1), std::max<int64_t>(n_pre, 1), h->device);
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemsetAsync(h->status, 0, sizeof(int32_t), h->stream));
    if ((rc = mt_enqueue(h->b, n_pre, nullptr, 1.0, h->b.pre, nullptr, g, h->status, h->stream)))
        return rc;
    int32_t st = 0;
    if (n_pre && pre_host)
        SLAM_HIP_TRY(hipMemcpyAsync(pre_host, h->b.pre, n_pre * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    if (g && g_host)
        SLAM_HIP_TRY(hipMemcpyAsync(g_host, h->b.normals, g * sizeof(double), hipMemcpyDeviceToHost,
                                    h->stream));
    SLAM_HIP_TRY(hipMemcpyAsync(&st, h->status, sizeof(st), hipMemcpyDeviceToHost, h->stream));
    SLAM_HIP_TRY(hipStreamSynchronize(h->stream));
    if (st & 256) return fail(SLAM_ERR_HIP, "mt19937 draw: candidate bound exhausted");
    return SLAM_OK;
}

int slam_mt_random_sample(slam_mt* h, int64_t n, double* out) {
    SLAM_ARG_CHECK(h && n >= 0 && (n == 0 || out), "slam_mt_random_sample: bad arguments");
    if (n == 0) return SLAM_OK;
    return mt_draw(h, n, 0, out, nullptr);
}

int slam_mt_standard_normal(slam_mt* h, int64_t n, double* out) {
    SLAM_ARG_CHECK(h && n >= 0 && (n == 0 || out), "slam_mt_standard_normal: bad arguments");
    if (n == 0) return SLAM_OK;
    return mt_draw(h, 0, n, nullptr, out);
}

}  // extern "C"
