// motion_api.hip -- MotionModel (motion_model.py:14-86) on a batch of poses.
//
// The reference applies sample_motion_model_velocity to one (3,1) pose per
// call (motion_model.py:31-62) or its noise-free form (:64-86).  Here one lane
// takes one pose; a batch of N poses with the standard normals of N
// consecutive moveWithNoise calls (draw order v, w, gamma per call,
// :46-48) gives N calls' results in one launch.  The arithmetic follows the
// reference operation by operation (-ffp-contract=off): sin/cos of the two
// headings are evaluated directly (not by angle addition as in the PF step
// kernel), so the result is within the sin/cos ulp of NumPy's.
#include <mutex>

#include "common.hpp"

namespace slam {

struct MotionConst {
    double dt;
    double a[6];
};

// motion_model.py:31-62 (noise != nullptr) / :64-86 (noise == nullptr)
__global__ __launch_bounds__(256) void motion_velocity_kernel(const int64_t n,
                                                              const double* __restrict__ poses,
                                                              const double v, const double w,
                                                              const double* __restrict__ noise,
                                                              const MotionConst mc,
                                                              double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = poses[3 * i], y = poses[3 * i + 1], th = poses[3 * i + 2];
    double xn, yn, tn;
    if (noise) {
        const double v2 = v * v, w2 = w * w;                       // :40-41
        const double sv = (mc.a[0] * v2) + (mc.a[1] * w2);         // :43-45
        const double sw = (mc.a[2] * v2) + (mc.a[3] * w2);
        const double sg = (mc.a[4] * v2) + (mc.a[5] * w2);
        // :46-48 np.random.normal(0, sigma**2) = 0 + sigma**2 * g (legacy)
        const double vh = v + (0.0 + (sv * sv) * noise[3 * i]);
        const double wh = w + (0.0 + (sw * sw) * noise[3 * i + 1]);
        const double gh = 0.0 + (sg * sg) * noise[3 * i + 2];
        const double a = vh / wh;                                  // :50-51
        const double b = wh * mc.dt;
        double s0, c0, s1, c1;
        fast_sincos(th, &s0, &c0);
        fast_sincos(th + b, &s1, &c1);
        xn = (x - (a * s0)) + (a * s1);                            // :54-56
        yn = (y + (a * c0)) - (a * c1);
        tn = wrap_angle(th + (wh + gh) * mc.dt);
    } else {
        const double a = v / w;                                    // :73-76
        const double b = wrap_angle(w * mc.dt);
        const double ya = wrap_angle(th + b);
        double s0, c0, s1, c1;
        fast_sincos(th, &s0, &c0);
        fast_sincos(ya, &s1, &c1);
        xn = x + a * (-s0 + s1);                                   // :78-80
        yn = y + a * (c0 - c1);
        tn = ya;
    }
    out[3 * i] = xn;
    out[3 * i + 1] = yn;
    out[3 * i + 2] = tn;
}

namespace {

// grow-only device scratch per device for the one-shot entry point
struct MotionScratch {
    std::mutex mu;
    int device = -1;
    size_t cap = 0;      // poses
    double* buf = nullptr;
    hipStream_t stream = nullptr;
};

MotionScratch& scratch_for(int device) {
    static MotionScratch s[64];
    return s[device & 63];
}

}  // namespace
}  // namespace slam

using namespace slam;

extern "C" int slam_motion_velocity(const double* params, int64_t n, const double* poses, double v,
                                    double w, const double* normals, double* out, int device) {
    SLAM_ARG_CHECK(params && poses && out && n >= 0, "slam_motion_velocity: NULL argument");
    if (n == 0) return SLAM_OK;
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev && device < 64, "slam_motion_velocity: no such HIP device");
    MotionScratch& sc = scratch_for(device);
    std::lock_guard<std::mutex> lock(sc.mu);
    SLAM_HIP_TRY(hipSetDevice(device));
    if (!sc.stream) SLAM_HIP_TRY(hipStreamCreateWithFlags(&sc.stream, hipStreamNonBlocking));
    const size_t need = (size_t)n;
    if (need > sc.cap) {
        if (sc.buf) (void)hipFree(sc.buf);
        sc.buf = nullptr;
        sc.cap = 0;
        SLAM_HIP_TRY(hipMalloc(&sc.buf, sizeof(double) * 9 * need));   // poses, noise, out
        sc.cap = need;
    }
    double* d_pose = sc.buf;
    double* d_noise = sc.buf + 3 * sc.cap;
    double* d_out = sc.buf + 6 * sc.cap;
    const size_t bytes = sizeof(double) * 3 * need;
    SLAM_HIP_TRY(hipMemcpyAsync(d_pose, poses, bytes, hipMemcpyHostToDevice, sc.stream));
    if (normals) SLAM_HIP_TRY(hipMemcpyAsync(d_noise, normals, bytes, hipMemcpyHostToDevice, sc.stream));
    MotionConst mc;
    mc.dt = params[0];
    for (int k = 0; k < 6; ++k) mc.a[k] = params[1 + k];
    const unsigned grid = (unsigned)((n + 255) / 256);
    motion_velocity_kernel<<<grid, 256, 0, sc.stream>>>(n, d_pose, v, w, normals ? d_noise : nullptr,
                                                         mc, d_out);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(out, d_out, bytes, hipMemcpyDeviceToHost, sc.stream));
    SLAM_HIP_TRY(hipStreamSynchronize(sc.stream));
    return SLAM_OK;
}
