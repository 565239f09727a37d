// Probe: phase timing of finalize_deferred_kernel on synthetic, self-consistent
// inputs (n = 2^20).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
// -ffp-contract=off tools/fin_probe.hip -o tools/fin_probe
#define SLAM_FIN_PROBE
#include "../slam-robot_simu_amd/csrc/pf_kernels.inl"
#include <cstdio>
#include <vector>
#include <random>
using namespace slam;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
template <typename T> T* dev(size_t n) { T* p; (void)hipMalloc(&p, n * sizeof(T)); (void)hipMemset(p, 0, n * sizeof(T)); return p; }
int main() {
    const int64_t n = 1 << 20, nb = n / kPartPer;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<double> w(n), pmax(nb), leaf((kPartPer / 128) * nb), ps(11 * nb);
    std::vector<int64_t> pidx(nb);
    std::vector<double> ppre(nb);
    for (auto& v : w) { double u = U(g); v = u * u * u * u * 1e-20; }
    for (int64_t b = 0; b < nb; ++b) {
        double m = -1; int64_t mi = 0;
        for (int k = 0; k < kPartPer; ++k) if (w[b * kPartPer + k] > m) { m = w[b * kPartPer + k]; mi = b * kPartPer + k; }
        pmax[b] = m; pidx[b] = mi;
        double pr = -1; for (int64_t i = b * kPartPer; i < mi; ++i) pr = w[i] > pr ? w[i] : pr;
        ppre[b] = pr;
        for (int L = 0; L < kPartPer / 128; ++L) {
            double r[8];
            for (int k = 0; k < 8; ++k) { r[k] = w[b * kPartPer + L * 128 + k]; for (int j = 1; j < 16; ++j) r[k] += w[b * kPartPer + L * 128 + k + 8 * j]; }
            leaf[(kPartPer / 128) * b + L] = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        }
        for (int j = 0; j < 11; ++j) ps[j * nb + b] = U(g);
    }
    DeferParts dp;
    dp.pmax = dev<double>(nb); dp.pidx = dev<int64_t>(nb); dp.leaf = dev<double>((kPartPer / 128) * nb);
    for (int j = 0; j < 11; ++j) { dp.ps[j] = dev<double>(nb); CK(hipMemcpy(dp.ps[j], &ps[j * nb], nb * 8, hipMemcpyHostToDevice)); }
    CK(hipMemcpy(dp.pmax, pmax.data(), nb * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp.pidx, pidx.data(), nb * 8, hipMemcpyHostToDevice));
    dp.ppre = dev<double>(nb); CK(hipMemcpy(dp.ppre, ppre.data(), nb * 8, hipMemcpyHostToDevice));
    for (int j = 0; j < 3; ++j) dp.pxe[j] = dev<double>(nb);
    CK(hipMemcpy(dp.leaf, leaf.data(), leaf.size() * 8, hipMemcpyHostToDevice));
    double* w_un = dev<double>(n); CK(hipMemcpy(w_un, w.data(), n * 8, hipMemcpyHostToDevice));
    double *s_cur = dev<double>(1), *xs = dev<double>(n), *ys = dev<double>(n), *ts = dev<double>(n), *refp = dev<double>(4), *boff = dev<double>(nb + 1);
    int32_t* flags = dev<int32_t>(kFlagWords);
    int32_t* tl = dev<int32_t>(4); int32_t* to = dev<int32_t>(4);
    StepIO io; io.ctl = dev<double>(2 * 64); io.z = dev<double>(2); io.ofs = dev<double>(64); io.res = dev<slam_pf_result>(64); io.ctr = dev<int32_t>(4);
    int rate = 0; CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int rep = 0; rep < 6; ++rep) {
        int32_t z4[4] = {0, 0, 0, 0};
        CK(hipMemcpy(io.ctr, z4, 16, hipMemcpyHostToDevice));
        int32_t fl = rep & 1;     // odd reps: next step resamples (prefix pass)
        CK(hipMemcpy(flags, &fl, 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        finalize_deferred_kernel<<<1, kFinThreads>>>(n, dp, w_un, s_cur, tl, to, 0, 0, xs, ys, ts, refp, flags, (rep & 1) ? 1e30 : -1.0, io, -1, 1.0 / n, boff);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        long long st[16]; CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_fin_probe), sizeof(st)));
        slam_pf_result r; CK(hipMemcpy(&r, io.res, sizeof(r), hipMemcpyDeviceToHost));
        printf("rep %d total %.1f us | phases(us):", rep, ms * 1e3);
        for (int k = 1; k <= 5; ++k) printf(" %.2f", (st[k] - st[k - 1]) * 1e3 / rate);

        printf(" | max_idx %lld ess %.4g\n", (long long)r.max_idx, r.ess);
    }
    return 0;
}
