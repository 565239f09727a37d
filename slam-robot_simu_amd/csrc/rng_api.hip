// rng_api.hip -- NumPy's legacy RandomState stream on the device (mt19937.hpp).
//
// A request (mt_enqueue) is five launches, none of which needs the host:
//   mt_gen_kernel     one workgroup: the untempered MT19937 sequence from the
//                     current key, one block of 624 words per barrier (every
//                     word expanded from the previous block alone);
//   mt_count_kernel   per candidate pair (4 words): the polar test
//                     0 < x1^2 + x2^2 < 1, accepted candidates per block;
//   mt_scan_kernel    exclusive prefix of the block counts;
//   mt_emit_kernel    rank of every accepted candidate; the first P give the
//                     normals f x2, f x1 (f = sqrt(-2 log(r2) / r2), glibc's
//                     log), the P-th ends the draw;
//   mt_finish_kernel  the pre-draw doubles, the cached normal in slot 0, the
//                     new key / pos / cache exactly as NumPy leaves them.
// The draw order is NumPy's: legacy_gauss (legacy-distributions.c) returns
// f x2 and caches f x1; random_sample takes two words per double.
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
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
constexpr int kMtScanThreads = 1024;

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

__global__ __launch_bounds__(kMtGenThreads) void mt_gen_kernel(const MtDeviceState* __restrict__ st,
                                                               uint32_t* __restrict__ X,
                                                               const int64_t nblk) {
    __shared__ uint32_t buf[2][kMtN];
    const int t = threadIdx.x;
    for (int i = t; i < kMtN; i += kMtGenThreads) {
        const uint32_t v = st->key[i];
        buf[0][i] = v;
        X[i] = v;
    }
    __syncthreads();
    int a = 0;
    for (int64_t b = 1; b <= nblk; ++b) {
        const uint32_t* A = buf[a];
        uint32_t* Bn = buf[a ^ 1];
        uint32_t* out = X + b * kMtN;
        if (t < kMtN) {
            const uint32_t v = mt_block_word(A, t);
            Bn[t] = v;
            out[t] = v;
        }
        // LDS-only barrier: __syncthreads() would also wait for the global
        // stores of the block (a full store round trip per block)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        a ^= 1;
    }
}

__device__ __forceinline__ int64_t mt_pre_words(const int32_t* pre_flag, const int64_t n_pre) {
    return pre_flag ? (*pre_flag ? 2 : 0) : 2 * n_pre;
}

// candidate c: words X[w], ..., X[w + 3] (two legacy doubles)
__device__ __forceinline__ bool mt_candidate(const uint32_t* __restrict__ X, const int64_t w,
                                             double& x1, double& x2, double& r2) {
    const uint32_t w0 = mt_temper(X[w]), w1 = mt_temper(X[w + 1]);
    const uint32_t w2 = mt_temper(X[w + 2]), w3 = mt_temper(X[w + 3]);
    x1 = 2.0 * mt_legacy_double(w0, w1) - 1.0;
    x2 = 2.0 * mt_legacy_double(w2, w3) - 1.0;
    r2 = x1 * x1 + x2 * x2;
    return !(r2 >= 1.0 || r2 == 0.0);
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
    const MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const int64_t ncand,
    unsigned* __restrict__ bcnt) {
    const int64_t w0 = st->pos + mt_pre_words(pre_flag, n_pre);
    const int64_t c0 = (int64_t)blockIdx.x * kMtCandPerBlock + threadIdx.x * kMtCandPerThread;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kMtCandPerThread; ++k) {
        const int64_t c = c0 + k;
        double x1, x2, r2;
        if (c < ncand && mt_candidate(X, w0 + 4 * c, x1, x2, r2)) ++cnt;
    }
    int tot;
    (void)mt_block_scan(cnt, &tot);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = (unsigned)tot;
}

__global__ __launch_bounds__(kMtScanThreads) void mt_scan_kernel(
    MtDeviceState* __restrict__ st, const unsigned* __restrict__ bcnt, const int64_t nb,
    int64_t* __restrict__ boff, const int64_t g, int32_t* __restrict__ status) {
    __shared__ int64_t s_w[kMtScanThreads / 64];
    __shared__ int64_t s_carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < nb; base += kMtScanThreads) {
        const int64_t i = base + threadIdx.x;
        int64_t v = i < nb ? (int64_t)bcnt[i] : 0;
        const int64_t own = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(v, d, 64);
            if (lane >= d) v += o;
        }
        if (lane == 63) s_w[wave] = v;
        __syncthreads();
        int64_t add = s_carry, all = 0;
        for (int w = 0; w < kMtScanThreads / 64; ++w) {
            add += (w < wave) ? s_w[w] : 0;
            all += s_w[w];
        }
        if (i < nb) boff[i] = add + v - own;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const bool shrt = s_carry < mt_pairs(st, g);
        st->short_draw = shrt ? 1 : 0;
        if (shrt && status) atomicOr(status, 256);
    }
}

__global__ __launch_bounds__(kMtCountThreads) void mt_emit_kernel(
    MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const int64_t ncand,
    const int64_t* __restrict__ boff, const int64_t g, const GlibcLogTable* __restrict__ tab,
    double* __restrict__ normals) {
    const int64_t pw = mt_pre_words(pre_flag, n_pre);
    const int64_t w0 = st->pos + pw;
    const int h = st->has_gauss ? 1 : 0;
    const int64_t P = mt_pairs(st, g);
    const int64_t c0 = (int64_t)blockIdx.x * kMtCandPerBlock + threadIdx.x * kMtCandPerThread;
    double x1[kMtCandPerThread], x2[kMtCandPerThread], r2[kMtCandPerThread];
    bool acc[kMtCandPerThread];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kMtCandPerThread; ++k) {
        const int64_t c = c0 + k;
        acc[k] = c < ncand && mt_candidate(X, w0 + 4 * c, x1[k], x2[k], r2[k]);
        cnt += acc[k] ? 1 : 0;
    }
    int tot;
    const int incl = mt_block_scan(cnt, &tot);
    int64_t q = boff[blockIdx.x] + incl - cnt;
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
    MtDeviceState* __restrict__ st, const uint32_t* __restrict__ X,
    const int32_t* __restrict__ pre_flag, const int64_t n_pre, const double pre_scale,
    double* __restrict__ pre_out, const int32_t* __restrict__ pre_index, const int64_t g,
    double* __restrict__ normals) {
    __shared__ int64_t s_blk;
    __shared__ int32_t s_pos;
    const int64_t p = st->pos;
    const int64_t pw = mt_pre_words(pre_flag, n_pre);
    const int h = st->has_gauss ? 1 : 0;
    const int64_t P = mt_pairs(st, g);
    // pre-draw doubles (random_sample): words X[p + 2k], X[p + 2k + 1]
    if (pre_flag) {
        if (threadIdx.x == 0 && pre_out) {
            double* o = pre_out + (pre_index ? *pre_index : 0);
            *o = *pre_flag ? mt_legacy_double(mt_temper(X[p]), mt_temper(X[p + 1])) * pre_scale
                           : (double)NAN;
        }
    } else if (pre_out) {
        for (int64_t k = threadIdx.x; k < n_pre; k += blockDim.x)
            pre_out[k] = mt_legacy_double(mt_temper(X[p + 2 * k]), mt_temper(X[p + 2 * k + 1])) *
                         pre_scale;
    }
    if (threadIdx.x == 0) {
        if (h && g > 0) normals[0] = st->gauss;
        const int64_t e = p + (P > 0 ? st->j_end : pw);
        if (e > 0 && e % kMtN == 0) {                        // NumPy regenerates lazily: pos 624
            s_blk = e / kMtN - 1;
            s_pos = kMtN;
        } else {
            s_blk = e / kMtN;
            s_pos = (int32_t)(e % kMtN);
        }
    }
    __syncthreads();
    const uint32_t* src = X + s_blk * kMtN;
    for (int i = threadIdx.x; i < kMtN; i += blockDim.x) st->key[i] = src[i];
    if (threadIdx.x == 0) {
        st->pos = s_pos;
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

int64_t blocks_for(int64_t pre_words, int64_t ncand) {
    // pos <= 624; the state after the draw needs the whole block it ends in
    return (kMtN + pre_words + 4 * ncand) / kMtN + 2;
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
    void* ps[] = {b.st, b.tab, b.X, b.bcnt, b.boff, b.normals, b.pre};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    b = MtBuffers{};
}

int mt_reserve(MtBuffers& b, int64_t g_cap, int64_t pre_cap, int device) {
    if (b.st && g_cap <= b.g_cap && pre_cap <= b.pre_cap) return SLAM_OK;
    g_cap = std::max<int64_t>(g_cap, b.g_cap);
    pre_cap = std::max<int64_t>(pre_cap, b.pre_cap);
    SLAM_HIP_TRY(hipSetDevice(device));
    // keep the state across a regrow
    MtDeviceState keep{};
    const bool had = b.st != nullptr;
    if (had) SLAM_HIP_TRY(hipMemcpy(&keep, b.st, sizeof(keep), hipMemcpyDeviceToHost));
    GlibcLogTable T;
    int rc = glibc_log_table(&T);
    if (rc) return rc;
    mt_free(b);
    b.device = device;
    b.g_cap = g_cap;
    b.pre_cap = pre_cap;
    b.cand_cap = cand_bound(std::max<int64_t>(g_cap, 1));
    b.nblk = blocks_for(2 * pre_cap, b.cand_cap);
    b.nb_count = (b.cand_cap + kMtCandPerBlock - 1) / kMtCandPerBlock;
    SLAM_HIP_TRY(hipMalloc(&b.st, sizeof(MtDeviceState)));
    SLAM_HIP_TRY(hipMalloc(&b.tab, sizeof(GlibcLogTable)));
    SLAM_HIP_TRY(hipMalloc(&b.X, sizeof(uint32_t) * kMtN * (size_t)(b.nblk + 1)));
    SLAM_HIP_TRY(hipMalloc(&b.bcnt, sizeof(unsigned) * (size_t)b.nb_count));
    SLAM_HIP_TRY(hipMalloc(&b.boff, sizeof(int64_t) * (size_t)b.nb_count));
    SLAM_HIP_TRY(hipMalloc(&b.normals, sizeof(double) * (size_t)std::max<int64_t>(g_cap, 1)));
    SLAM_HIP_TRY(hipMalloc(&b.pre, sizeof(double) * (size_t)std::max<int64_t>(pre_cap, 1)));
    SLAM_HIP_TRY(hipMemcpy(b.tab, &T, sizeof(T), hipMemcpyHostToDevice));
    SLAM_HIP_TRY(hipMemcpy(b.st, &keep, sizeof(keep), hipMemcpyHostToDevice));
    return SLAM_OK;
}

int mt_set_state(MtBuffers& b, const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss,
                 hipStream_t s) {
    SLAM_ARG_CHECK(b.st && key, "mt19937 state: no buffers / key");
    SLAM_ARG_CHECK(pos >= 0 && pos <= kMtN, "mt19937 state: pos outside [0, 624]");
    MtDeviceState h{};
    std::memcpy(h.key, key, sizeof(h.key));
    h.pos = pos;
    h.has_gauss = has_gauss ? 1 : 0;
    h.gauss = has_gauss ? gauss : 0.0;
    SLAM_HIP_TRY(hipMemcpyAsync(b.st, &h, sizeof(h), hipMemcpyHostToDevice, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    return SLAM_OK;
}

int mt_get_state(const MtBuffers& b, uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss,
                 hipStream_t s) {
    SLAM_ARG_CHECK(b.st, "mt19937 state: no buffers");
    MtDeviceState h;
    SLAM_HIP_TRY(hipMemcpyAsync(&h, b.st, sizeof(h), hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    if (key) std::memcpy(key, h.key, sizeof(h.key));
    if (pos) *pos = h.pos;
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
    const int64_t pre_words = pre_flag ? 2 : 2 * n_pre;
    const int64_t ncand = g > 0 ? cand_bound(g) : 0;
    const int64_t nblk = blocks_for(pre_words, ncand);
    SLAM_ARG_CHECK(nblk <= b.nblk, "mt19937 draw: stream buffer too small");
    mt_gen_kernel<<<1, kMtGenThreads, 0, s>>>(b.st, b.X, nblk);
    SLAM_HIP_TRY(hipGetLastError());
    const unsigned nbc = (unsigned)((ncand + kMtCandPerBlock - 1) / kMtCandPerBlock);
    if (nbc > 0) {
        mt_count_kernel<<<nbc, kMtCountThreads, 0, s>>>(b.st, b.X, pre_flag, n_pre, ncand, b.bcnt);
        mt_scan_kernel<<<1, kMtScanThreads, 0, s>>>(b.st, b.bcnt, nbc, b.boff, g, status);
        mt_emit_kernel<<<nbc, kMtCountThreads, 0, s>>>(b.st, b.X, pre_flag, n_pre, ncand, b.boff, g,
                                                       b.tab, b.normals);
        SLAM_HIP_TRY(hipGetLastError());
    }
    mt_finish_kernel<<<1, kMtGenThreads, 0, s>>>(b.st, b.X, pre_flag, n_pre, pre_scale, pre_out,
                                                 pre_index, g, b.normals);
    SLAM_HIP_TRY(hipGetLastError());
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
