// api_common.hip -- version, thread-local error text, device query.
#include "common.hpp"

namespace slam {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace slam

extern "C" {

int slam_version(void) { return 10000; }  // 1.0.0

const char* slam_last_error(void) { return slam::g_last_error.c_str(); }

int slam_device_count(int* n) {
    SLAM_ARG_CHECK(n != nullptr, "slam_device_count: n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *n = c;
    return SLAM_OK;
}

}  // extern "C"
