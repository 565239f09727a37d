// Host AddressSanitizer / UBSan run of the C-ABI (VERDICT r3 item
// 10): `make -C slam-robot_simu_amd asan` builds libslam_hip_asan.so with the
// host side instrumented (-Xarch_host -fsanitize=address,undefined) and this
// driver against it, then runs it.  It needs no GPU: it walks every entry
// point's argument checks and error returns (NULL handles and arguments, bad
// sizes, a create on a machine with no device), and the host-only code paths
// -- the MT19937 jump-ahead (Berlekamp-Massey, x^n mod phi), the glibc log
// restatement with its libm table probe, the shard split -- checking their
// results.  Any sanitizer report aborts the run (halt_on_error).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/slam_hip.h"

static int g_fail = 0, g_checks = 0;

#define CHECK(cond, ...)                                                         \
    do {                                                                         \
        ++g_checks;                                                              \
        if (!(cond)) {                                                           \
            ++g_fail;                                                            \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);            \
            std::fprintf(stderr, __VA_ARGS__);                                   \
            std::fprintf(stderr, "\n");                                          \
        }                                                                        \
    } while (0)

// an error return with a message behind it
#define EXPECT_ERR(call)                                                         \
    do {                                                                         \
        const int rc_ = (call);                                                  \
        const char* m_ = slam_last_error();                                      \
        CHECK(rc_ < 0 && m_ && m_[0], "%s returned %d (%s)", #call, rc_, m_ ? m_ : "null"); \
    } while (0)

static uint32_t mt_next(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

int main() {
    CHECK(slam_version() >= 10000, "version %d", slam_version());
    int ndev = -1;
    const int rc_dev = slam_device_count(&ndev);
    std::printf("slam_device_count rc %d n %d (%s)\n", rc_dev, ndev, rc_dev ? slam_last_error() : "");
    EXPECT_ERR(slam_device_count(nullptr));

    // ---- particle filter: argument checks and a create without a device
    slam_pf_config cfg{};
    cfg.dt = 0.1;
    cfg.ess_threshold = 10.0;
    cfg.r_cov[0] = cfg.r_cov[3] = 0.04;
    cfg.motion = SLAM_MOTION_VELOCITY;
    cfg.likelihood = SLAM_LIK_LOGSUM;
    std::vector<double> lm(40, 1.0), buf(1 << 12, 0.0);
    slam_pf* pf = nullptr;
    EXPECT_ERR(slam_pf_create(nullptr, 1000, 20, lm.data(), 0, &pf));
    EXPECT_ERR(slam_pf_create(&cfg, 0, 20, lm.data(), 0, &pf));
    EXPECT_ERR(slam_pf_create(&cfg, 1000, -1, lm.data(), 0, &pf));
    EXPECT_ERR(slam_pf_create(&cfg, 1000, 20, nullptr, 0, &pf));
    slam_pf_config bad = cfg;
    bad.motion = 7;
    EXPECT_ERR(slam_pf_create(&bad, 1000, 20, lm.data(), 0, &pf));
    bad = cfg;
    bad.likelihood = 9;
    EXPECT_ERR(slam_pf_create(&bad, 1000, 20, lm.data(), 0, &pf));
    if (ndev <= 0) {
        EXPECT_ERR(slam_pf_create(&cfg, 1000, 20, lm.data(), 0, &pf));
        CHECK(pf == nullptr, "no handle without a device");
    }
    CHECK(slam_pf_destroy(nullptr) == 0, "destroy(NULL) is a no-op");
    slam_pf_result res{};
    double ms = 0.0;
    int32_t i32 = 0;
    int64_t i64 = 0;
    EXPECT_ERR(slam_pf_set_state(nullptr, buf.data(), buf.data(), buf.data(), buf.data()));
    EXPECT_ERR(slam_pf_get_state(nullptr, buf.data(), buf.data(), buf.data(), buf.data()));
    EXPECT_ERR(slam_pf_set_landmarks(nullptr, lm.data()));
    EXPECT_ERR(slam_pf_step(nullptr, buf.data(), buf.data(), nullptr, NAN, &res));
    EXPECT_ERR(slam_pf_resample(nullptr, 0.5, 1, &i32));
    EXPECT_ERR(slam_pf_predict(nullptr, buf.data(), nullptr));
    EXPECT_ERR(slam_pf_update(nullptr, buf.data(), &res));
    EXPECT_ERR(slam_pf_resample_indices(nullptr, 0.5, &i64, &i32));
    EXPECT_ERR(slam_pf_weight_sum(nullptr, &ms));
    EXPECT_ERR(slam_pf_load_observations(nullptr, 4, buf.data()));
    EXPECT_ERR(slam_pf_run(nullptr, 0, 4, buf.data(), &res));
    EXPECT_ERR(slam_pf_enable_timing(nullptr, 1));
    EXPECT_ERR(slam_pf_timing(nullptr, 0, &ms, &i64));
    EXPECT_ERR(slam_pf_set_graphs(nullptr, 1));
    EXPECT_ERR(slam_pf_prepare_graphs(nullptr, &ms));
    EXPECT_ERR(slam_pf_set_scan_merged(nullptr, 1));
    EXPECT_ERR(slam_pf_set_resample_next(nullptr, 1));
    EXPECT_ERR(slam_pf_set_ess_band(nullptr, 1e-9));
    EXPECT_ERR(slam_pf_set_stream(nullptr, nullptr, 0));
    EXPECT_ERR(slam_pf_load_truth(nullptr, 4, buf.data()));
    EXPECT_ERR(slam_pf_step_truth(nullptr, buf.data(), buf.data(), buf.data(), &res));
    EXPECT_ERR(slam_debug_pair_normals(0, 0, -1, 0, 0, buf.data()));

    // ---- the sharded filter
    int64_t gb = -1, nl = -1, sum = 0;
    for (int32_t world : {1, 2, 3, 8}) {
        const int64_t n = 8 * 1048576 + 5 * 8192 + 17;
        sum = 0;
        for (int32_t r = 0; r < world; ++r) {
            CHECK(slam_dist_shard_range(n, world, r, &gb, &nl) == 0, "shard_range %d/%d", r, world);
            CHECK(gb == sum, "contiguous shards (%lld != %lld)", (long long)gb, (long long)sum);
            if (r + 1 < world) CHECK(nl % 8192 == 0, "whole np.sum buffers but the last");
            sum += nl;
        }
        CHECK(sum == n, "shards cover the filter");
    }
    EXPECT_ERR(slam_dist_shard_range(100, 0, 0, &gb, &nl));
    EXPECT_ERR(slam_dist_shard_range(100, 2, 2, &gb, &nl));
    CHECK(slam_dist_handle_size(&i64) == 0 && i64 > 0, "handle size %lld", (long long)i64);
    slam_dist* dd = nullptr;
    EXPECT_ERR(slam_dist_create(nullptr, 1, 1, 0, &dd));
    EXPECT_ERR(slam_dist_run(nullptr, 0, 1, buf.data(), &res));
    EXPECT_ERR(slam_dist_prepare_graphs(nullptr, &ms));
    EXPECT_ERR(slam_dist_connect(nullptr, buf.data()));
    EXPECT_ERR(slam_dist_step(nullptr, buf.data(), buf.data(), &res));
    EXPECT_ERR(slam_dist_set_merged(nullptr, 1, &i32));
    CHECK(slam_dist_destroy(nullptr) == 0, "dist destroy(NULL)");
    EXPECT_ERR(slam_pf_create_dist_shard(&cfg, 0, 100, 0, 20, lm.data(), 0, &pf));

    // ---- EKF, EKF-SLAM, graph
    slam_ekf* ekf = nullptr;
    EXPECT_ERR(slam_ekf_create(nullptr, 16, 0, &ekf));
    EXPECT_ERR(slam_ekf_set_state(nullptr, buf.data(), buf.data()));
    EXPECT_ERR(slam_ekf_get_state(nullptr, buf.data(), buf.data()));
    EXPECT_ERR(slam_ekf_run(nullptr, 2, buf.data(), buf.data(), buf.data()));
    EXPECT_ERR(slam_ekf_synchronize(nullptr));
    CHECK(slam_ekf_destroy(nullptr) == 0, "ekf destroy(NULL)");
    slam_ekfslam* eks = nullptr;
    EXPECT_ERR(slam_ekfslam_create(nullptr, 10, 0, &eks));
    EXPECT_ERR(slam_ekfslam_predict(nullptr, buf.data()));
    EXPECT_ERR(slam_ekfslam_get_rows(nullptr, 1, &i64, buf.data()));
    CHECK(slam_ekfslam_destroy(nullptr) == 0, "ekfslam destroy(NULL)");
    slam_graph* gr = nullptr;
    EXPECT_ERR(slam_graph_create(nullptr, 0, &gr));
    EXPECT_ERR(slam_graph_update(nullptr, buf.data()));
    EXPECT_ERR(slam_graph_optimize(nullptr, 0.01, 4, buf.data(), &i32));
    EXPECT_ERR(slam_graph_cond_info(nullptr, buf.data()));
    EXPECT_ERR(slam_graph_get_bsr(nullptr, &i64, nullptr, nullptr, nullptr));
    CHECK(slam_graph_destroy(nullptr) == 0, "graph destroy(NULL)");
    EXPECT_ERR(slam_graph_pair_halves(-1, nullptr, 4, 0, &i64, nullptr));
    EXPECT_ERR(slam_error_ellipse(-1, buf.data(), 1.0, 0, buf.data(), 0));
    EXPECT_ERR(slam_scan_noise(-1, buf.data(), buf.data(), 0.1, 0.1, 0.1, buf.data(), 0));
    EXPECT_ERR(slam_motion_velocity(nullptr, 1, buf.data(), 1.0, 0.1, buf.data(), buf.data(), 0));
    slam_comm* cm = nullptr;
    EXPECT_ERR(slam_comm_create(nullptr, 1, 0, 0, &cm));
    EXPECT_ERR(slam_comm_all_gather_host(nullptr, buf.data(), buf.data(), 8));
    CHECK(slam_comm_destroy(nullptr) == 0, "comm destroy(NULL)");

    // ---- MT19937 (host): the jump-ahead window against the recurrence
    std::vector<uint32_t> win(624), out(624);
    uint32_t s = 5489u;
    win[0] = s;
    for (int i = 1; i < 624; ++i) win[i] = s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
    for (uint64_t J : {uint64_t(1), uint64_t(623), uint64_t(624), uint64_t(1000), uint64_t(40000)}) {
        std::vector<uint32_t> seq(win);
        seq.reserve(624 + J);
        for (uint64_t k = 624; k < 624 + J; ++k)
            seq.push_back(mt_next(seq[k - 624], seq[k - 623], seq[k - 227]));
        const int rc = slam_mt_jump_window(win.data(), J, out.data());
        CHECK(rc == 0, "jump_window(%llu) rc %d: %s", (unsigned long long)J, rc, slam_last_error());
        bool ok = (out[0] & 0x80000000u) == (seq[J] & 0x80000000u);   // word 0: top bit only
        for (int j = 1; j < 624; ++j) ok = ok && out[j] == seq[J + j];
        CHECK(ok, "jump_window(%llu) differs from the recurrence", (unsigned long long)J);
    }
    EXPECT_ERR(slam_mt_jump_window(nullptr, 10, out.data()));
    slam_mt* mt = nullptr;
    EXPECT_ERR(slam_mt_create(nullptr, 0, 0, 0.0, 0, &mt));
    EXPECT_ERR(slam_mt_random_sample(nullptr, 4, buf.data()));
    CHECK(slam_mt_destroy(nullptr) == 0, "mt destroy(NULL)");

    // ---- glibc log restatement (host): bit-exact against this process's log()
    std::vector<double> x, y;
    for (int i = 0; i < 4096; ++i) x.push_back(std::ldexp(1.0 + i / 4096.0, (i % 61) - 30));
    x.push_back(1.0);
    x.push_back(0x1p-1074);
    x.push_back(0.5 + 0x1p-53);
    y.resize(x.size());
    const int rcl = slam_glibc_log((int64_t)x.size(), x.data(), y.data());
    CHECK(rcl == 0, "glibc_log rc %d: %s", rcl, slam_last_error());
    if (rcl == 0) {
        int bad_bits = 0;
        for (size_t i = 0; i < x.size(); ++i) {
            const double ref = std::log(x[i]);
            bad_bits += std::memcmp(&y[i], &ref, 8) != 0;
        }
        CHECK(bad_bits == 0, "glibc_log: %d of %zu differ from log()", bad_bits, x.size());
    }
    EXPECT_ERR(slam_glibc_log(4, nullptr, y.data()));

    std::printf("capi_asan_driver: %d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
