// sensor_api.hip -- ScanSensor.scan (graph_based_slam.py:128-172) over a batch
// of robot poses x landmarks.
//
// The reference scans one pose at a time: world2robot of every landmark
// (mylib/transform.py:31-35), distance (np.linalg.norm), direction (arctan2),
// orientation (BASE_ANG - yaw), the fan-shaped field-of-view test (:155-159),
// and, per detected landmark in landmark order, three np.random.normal draws
// (:163-165).  Here one lane takes one (pose, landmark) pair:
//   slam_scan_detect: the noise-free observation and the detection flag;
//   slam_scan_noise:  the noisy observation of each detected pair from the
//                     standard normals of the reference's draw order
//                     (np.random.normal(loc, scale) = loc + scale * gauss).
// cos / sin of the robot yaw come from the caller (NumPy's, one per pose), so
// the rotation is the reference's to the rounding of its 2x2 product; the
// direction is the device atan2 (within an ulp of the C library's).
#include <mutex>

#include "common.hpp"

namespace slam {

// per (pose p, landmark i), p-major: flag + (dist, dir, orient)
__global__ __launch_bounds__(256) void scan_detect_kernel(
    const int64_t np_, const int64_t nl, const double* __restrict__ poses,
    const double* __restrict__ yaw_cs, const double* __restrict__ lm, const double range,
    const double tan_scan, int32_t* __restrict__ detect, double* __restrict__ obs) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= np_ * nl) return;
    const int64_t p = k / nl, i = k - p * nl;
    const double c = yaw_cs[3 * p], s = yaw_cs[3 * p + 1], orient = yaw_cs[3 * p + 2];
    const double dx = lm[2 * i] - poses[3 * p];             // world - origin (transform.py:32)
    const double dy = lm[2 * i + 1] - poses[3 * p + 1];
    const double rx = fma(-s, dy, c * dx);                  // rot @ diff.T (:33-35)
    const double ry = fma(c, dy, s * dx);
    const double d = sqrt(rx * rx + ry * ry);               // np.linalg.norm(axis=1) (:150)
    const double dir = atan2(ry, rx);                       // :151
    detect[k] = (d <= range && ry >= fabs(rx) * tan_scan) ? 1 : 0;   // :155-159
    obs[3 * k] = d;
    obs[3 * k + 1] = dir;
    obs[3 * k + 2] = orient;                                 // :152
}

// :163-165 for n detected observations: d + (d R_dist) g0, limit_angle(dir +
// R_dir g1), limit_angle(orient + R_orient g2)
__global__ __launch_bounds__(256) void scan_noise_kernel(const int64_t n,
                                                         const double* __restrict__ clean,
                                                         const double* __restrict__ g,
                                                         const double r_dist, const double r_dir,
                                                         const double r_orient,
                                                         double* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double d = clean[3 * k], dir = clean[3 * k + 1], ori = clean[3 * k + 2];
    out[3 * k] = d + (d * r_dist) * g[3 * k];
    out[3 * k + 1] = wrap_angle(dir + r_dir * g[3 * k + 1]);
    out[3 * k + 2] = wrap_angle(ori + r_orient * g[3 * k + 2]);
}

namespace {

struct SensorScratch {
    std::mutex mu;
    size_t cap = 0;      // bytes
    char* buf = nullptr;
    hipStream_t stream = nullptr;
};

SensorScratch& sensor_scratch(int device) {
    static SensorScratch s[64];
    return s[device & 63];
}

int sensor_begin(SensorScratch& sc, int device, size_t bytes) {
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev && device < 64, "scan sensor: no such HIP device");
    SLAM_HIP_TRY(hipSetDevice(device));
    if (!sc.stream) SLAM_HIP_TRY(hipStreamCreateWithFlags(&sc.stream, hipStreamNonBlocking));
    if (bytes > sc.cap) {
        if (sc.buf) (void)hipFree(sc.buf);
        sc.buf = nullptr;
        sc.cap = 0;
        SLAM_HIP_TRY(hipMalloc(&sc.buf, bytes));
        sc.cap = bytes;
    }
    return SLAM_OK;
}

size_t al256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace
}  // namespace slam

using namespace slam;

extern "C" {

int slam_scan_detect(int64_t n_poses, const double* poses, const double* yaw_cs, int64_t n_landmarks,
                     const double* landmarks, double range, double tan_scan, int32_t* detect,
                     double* obs, int device) {
    SLAM_ARG_CHECK(n_poses >= 0 && n_landmarks >= 0 && (poses && yaw_cs && landmarks && detect && obs ||
                                                         n_poses * n_landmarks == 0),
                   "slam_scan_detect: bad arguments");
    const int64_t n = n_poses * n_landmarks;
    if (n == 0) return SLAM_OK;
    SensorScratch& sc = sensor_scratch(device);
    std::lock_guard<std::mutex> lock(sc.mu);
    const size_t bp = al256(24 * n_poses), bl = al256(16 * n_landmarks), bd = al256(4 * n),
                 bo = al256(24 * n);
    int rc = sensor_begin(sc, device, 2 * bp + bl + bd + bo);
    if (rc) return rc;
    double* d_pose = (double*)sc.buf;
    double* d_cs = (double*)(sc.buf + bp);
    double* d_lm = (double*)(sc.buf + 2 * bp);
    int32_t* d_det = (int32_t*)(sc.buf + 2 * bp + bl);
    double* d_obs = (double*)(sc.buf + 2 * bp + bl + bd);
    SLAM_HIP_TRY(hipMemcpyAsync(d_pose, poses, 24 * n_poses, hipMemcpyHostToDevice, sc.stream));
    SLAM_HIP_TRY(hipMemcpyAsync(d_cs, yaw_cs, 24 * n_poses, hipMemcpyHostToDevice, sc.stream));
    SLAM_HIP_TRY(hipMemcpyAsync(d_lm, landmarks, 16 * n_landmarks, hipMemcpyHostToDevice, sc.stream));
    scan_detect_kernel<<<(unsigned)((n + 255) / 256), 256, 0, sc.stream>>>(
        n_poses, n_landmarks, d_pose, d_cs, d_lm, range, tan_scan, d_det, d_obs);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(detect, d_det, 4 * n, hipMemcpyDeviceToHost, sc.stream));
    SLAM_HIP_TRY(hipMemcpyAsync(obs, d_obs, 24 * n, hipMemcpyDeviceToHost, sc.stream));
    SLAM_HIP_TRY(hipStreamSynchronize(sc.stream));
    return SLAM_OK;
}

int slam_scan_noise(int64_t n, const double* clean, const double* normals, double r_dist,
                    double r_dir, double r_orient, double* out, int device) {
    SLAM_ARG_CHECK(n >= 0 && (clean && normals && out || n == 0), "slam_scan_noise: bad arguments");
    if (n == 0) return SLAM_OK;
    SensorScratch& sc = sensor_scratch(device);
    std::lock_guard<std::mutex> lock(sc.mu);
    const size_t b = al256(24 * n);
    int rc = sensor_begin(sc, device, 3 * b);
    if (rc) return rc;
    double* d_c = (double*)sc.buf;
    double* d_g = (double*)(sc.buf + b);
    double* d_o = (double*)(sc.buf + 2 * b);
    SLAM_HIP_TRY(hipMemcpyAsync(d_c, clean, 24 * n, hipMemcpyHostToDevice, sc.stream));
    SLAM_HIP_TRY(hipMemcpyAsync(d_g, normals, 24 * n, hipMemcpyHostToDevice, sc.stream));
    scan_noise_kernel<<<(unsigned)((n + 255) / 256), 256, 0, sc.stream>>>(n, d_c, d_g, r_dist, r_dir,
                                                                          r_orient, d_o);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(out, d_o, 24 * n, hipMemcpyDeviceToHost, sc.stream));
    SLAM_HIP_TRY(hipStreamSynchronize(sc.stream));
    return SLAM_OK;
}

}  // extern "C"
