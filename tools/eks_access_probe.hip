// EKF-SLAM rank-update access-pattern probe (development tool, round 6;
// VERDICT r5 item 5).  The C4 covariance (n = 30,003, row-major, lower
// triangle current, 128 x 128 tiles walked as eks_rank_update_frag_kernel
// walks them: XCD-contiguous ranges of the lower-triangle tile list, one
// workgroup of 8 waves per CU, a wave owning 32 x 64 of the tile, the next
// tile's block requested at the top of the current one) read and written back
// with no arithmetic, in three lane layouts:
//   frag  -- the MFMA accumulator layout the kernel uses: lane (lr, lk) holds
//            rows lk + 4r of column lr: 8-byte lanes, 4 rows x 128 B per load;
//   wide  -- 16-byte lanes, two adjacent columns: 2 rows x 512 B per load;
//   rows  -- whole 1 KB tile rows per wave instruction pair (dwordx4, 64 lanes).
// Prints the time and the bytes moved (algorithmic: 16 B per lower-triangle
// element, read + written) per layout; run under rocprofv3 --pmc FETCH_SIZE /
// WRITE_SIZE to calibrate the counters for these patterns.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

constexpr int kTile = 128;
typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void tile_rc(const long L, long& ti, long& tj) {
    ti = (long)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > L) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
    tj = L - ti * (ti + 1) / 2;
}

template <int MODE>
__global__ __launch_bounds__(512) void walk(double* __restrict__ P, const long n, const long ld,
                                            const long n_tiles, const double f) {
    const long per_xcd = (n_tiles + 7) / 8;
    const long xcd = blockIdx.x % 8, stride = gridDim.x / 8;
    const long Lend = min(n_tiles, (xcd + 1) * per_xcd);
    long L = xcd * per_xcd + blockIdx.x / 8;
    if (L >= Lend) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave / 2) * 32, wc = (wave % 2) * 64;         // 4 x 2 waves of 32 x 64
    double cur[32], nxt[32];
    auto addr = [&](const long r0, const long c0, const int k, long& gi, long& gj) {
        if (MODE == 0) {                       // frag: x = k / 16, y = (k / 4) % 4, r = k % 4
            const int x = k >> 4, y = (k >> 2) & 3, r = k & 3;
            gi = r0 + wr + 16 * x + (lane >> 4) + 4 * r;
            gj = c0 + wc + 16 * y + (lane & 15);
        } else if (MODE == 1) {                // wide: pairs of columns, 2 rows per load
            const int h = k >> 1, s = k & 1;
            gi = r0 + wr + 2 * h + (lane >> 5);
            gj = c0 + wc + 2 * (lane & 31) + s;
        } else {                               // rows: 1 KB rows, 4 doubles per lane per row pair
            const int q = k >> 2, s = k & 3;   // q: 8 row groups of 4 rows
            gi = r0 + wr + 4 * q + (lane >> 4);
            gj = c0 + wc + 4 * (lane & 15) + s;
        }
    };
    auto load = [&](double (&t)[32], const long r0, const long c0, const bool diag) {
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                t[k] = (gi < n && gj < n && (!diag || gj <= gi))
                           ? __builtin_nontemporal_load(&P[gi * ld + gj]) : 0.0;
            }
        } else if (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 32; k += 2) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                if (gi < n && gj + 1 < n) {
                    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(&P[gi * ld + gj]));
                    t[k] = v.x;
                    t[k + 1] = v.y;
                } else {
                    t[k] = t[k + 1] = 0.0;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 32; k += 4) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                if (gi < n && gj + 3 < n) {
                    const d2v* p = reinterpret_cast<const d2v*>(&P[gi * ld + gj]);
                    const d2v a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1);
                    t[k] = a.x;
                    t[k + 1] = a.y;
                    t[k + 2] = b.x;
                    t[k + 3] = b.y;
                } else {
                    t[k] = t[k + 1] = t[k + 2] = t[k + 3] = 0.0;
                }
            }
        }
    };
    auto store = [&](const double (&t)[32], const long r0, const long c0, const bool diag) {
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                if (gi < n && gj < n && (!diag || gj <= gi)) P[gi * ld + gj] = t[k] * f;
            }
        } else if (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 32; k += 2) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                if (gi < n && gj + 1 < n)
                    *reinterpret_cast<double2*>(&P[gi * ld + gj]) = double2{t[k] * f, t[k + 1] * f};
            }
        } else {
#pragma unroll
            for (int k = 0; k < 32; k += 4) {
                long gi, gj;
                addr(r0, c0, k, gi, gj);
                if (gi < n && gj + 3 < n) {
                    double2* p = reinterpret_cast<double2*>(&P[gi * ld + gj]);
                    p[0] = double2{t[k] * f, t[k + 1] * f};
                    p[1] = double2{t[k + 2] * f, t[k + 3] * f};
                }
            }
        }
    };
    long ti, tj;
    tile_rc(L, ti, tj);
    load(cur, ti * kTile, tj * kTile, ti == tj);
    for (;;) {
        const long Ln = L + stride;
        const bool more = Ln < Lend;
        long tin = 0, tjn = 0;
        if (more) {
            tile_rc(Ln, tin, tjn);
            load(nxt, tin * kTile, tjn * kTile, tin == tjn);
        }
        store(cur, ti * kTile, tj * kTile, ti == tj);
        if (!more) break;
#pragma unroll
        for (int k = 0; k < 32; ++k) cur[k] = nxt[k];
        L = Ln;
        ti = tin;
        tj = tjn;
    }
}

int main(int argc, char** argv) {
    const long n = 30003, ld = 30080;                 // C4: n = 3 + 3 * 10,000; rows padded
    const long nt = (n + kTile - 1) / kTile, n_tiles = nt * (nt + 1) / 2;
    double* P;
    CK(hipMalloc(&P, (size_t)n * ld * sizeof(double)));
    CK(hipMemset(P, 0, (size_t)n * ld * sizeof(double)));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus / 8 * 8;
    const double bytes = 16.0 * (double)n * (double)(n + 1) / 2.0;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[3] = {"frag (8 B lanes, 4 x 128 B rows / load)", "wide (16 B lanes, 2 x 512 B rows / load)",
                            "rows (2 x 16 B lanes, 4 x 256 B / load pair)"};
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    for (int round = 0; round < 2; ++round)
        for (int m = 0; m < 3; ++m) {
            float best = 1e30f, sum = 0.0f;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(a));
                if (m == 0) walk<0><<<grid, 512>>>(P, n, ld, n_tiles, 1.0);
                if (m == 1) walk<1><<<grid, 512>>>(P, n, ld, n_tiles, 1.0);
                if (m == 2) walk<2><<<grid, 512>>>(P, n, ld, n_tiles, 1.0);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
                sum += ms;
            }
            std::printf("round %d %-45s best %.3f ms  avg %.3f ms  %.2f TB/s (algorithmic %.2f GB)\n", round,
                        names[m], best, sum / reps, bytes / (best * 1e-3) / 1e12, bytes / 1e9);
        }
    CK(hipFree(P));
    return 0;
}
