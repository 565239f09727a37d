// comm_api.hip -- RCCL communicator of the multi-GPU particle filter.
//
// RCCL (the NCCL API on ROCm) is loaded with dlopen when the first
// communicator is created, so libslam_hip.so has no link-time RCCL
// dependency; a process that already holds an RCCL (PyTorch ships one under
// the same soname, librccl.so.1) shares that instance.  The communicator is
// used to bootstrap the sharded filter's peer-memory exchange (slam_dist_*)
// and for the fixed-size all-gather of the per-step reduction records when the
// filter runs in its RCCL mode.
#include <dlfcn.h>

#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "comm.hpp"
#include "common.hpp"

namespace slam {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    void* dl = nullptr;
};

namespace {

std::mutex g_rccl_mu;
Rccl g_rccl;
bool g_rccl_tried = false;
std::string g_rccl_err;

const Rccl* rccl_load() {
    std::lock_guard<std::mutex> lock(g_rccl_mu);
    if (g_rccl.dl) return &g_rccl;
    if (g_rccl_tried) return nullptr;
    g_rccl_tried = true;
    void* dl = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);      // already in the process
    if (!dl) dl = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!dl) dl = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!dl) {
        g_rccl_err = std::string("dlopen(librccl.so.1): ") + dlerror();
        return nullptr;
    }
    Rccl r;
    r.dl = dl;
#define SLAM_SYM(field, name)                                               \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(dl, name));         \
    if (!r.field) {                                                         \
        g_rccl_err = std::string("RCCL symbol missing: ") + name;           \
        return nullptr;                                                     \
    }
    SLAM_SYM(get_unique_id, "ncclGetUniqueId");
    SLAM_SYM(comm_init_rank, "ncclCommInitRank");
    SLAM_SYM(comm_destroy, "ncclCommDestroy");
    SLAM_SYM(all_gather, "ncclAllGather");
    SLAM_SYM(send, "ncclSend");
    SLAM_SYM(recv, "ncclRecv");
    SLAM_SYM(group_start, "ncclGroupStart");
    SLAM_SYM(group_end, "ncclGroupEnd");
    SLAM_SYM(error_string, "ncclGetErrorString");
#undef SLAM_SYM
    g_rccl = r;
    return &g_rccl;
}

int rccl_fail(const Rccl* api, ncclResult_t r, const char* what) {
    return fail(SLAM_ERR_COMM, std::string(what) + ": " + (api ? api->error_string(r) : "RCCL"));
}

}  // namespace

int comm_all_gather(const Comm& c, const void* send, void* recv, size_t bytes, hipStream_t stream) {
    if (c.world == 1) {
        if (send != recv)
            SLAM_HIP_TRY(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, stream));
        return SLAM_OK;
    }
    if (!c.nccl) return fail(SLAM_ERR_COMM, "comm_all_gather: no RCCL communicator");
    const ncclResult_t r =
        c.api->all_gather(send, recv, bytes, ncclUint8, (ncclComm_t)c.nccl, stream);
    if (r != ncclSuccess) return rccl_fail(c.api, r, "ncclAllGather");
    return SLAM_OK;
}

int comm_exchange(const Comm& c, const std::vector<const void*>& send_ptr,
                  const std::vector<size_t>& send_bytes, const std::vector<void*>& recv_ptr,
                  const std::vector<size_t>& recv_bytes, hipStream_t stream) {
    if (c.world == 1) return SLAM_OK;
    if (!c.nccl) return fail(SLAM_ERR_COMM, "comm_exchange: no RCCL communicator");
    ncclResult_t r = c.api->group_start();
    if (r != ncclSuccess) return rccl_fail(c.api, r, "ncclGroupStart");
    for (int p = 0; p < c.world; ++p) {
        if (p == c.rank) continue;
        if (send_bytes[p] &&
            (r = c.api->send(send_ptr[p], send_bytes[p], ncclUint8, p, (ncclComm_t)c.nccl, stream)) !=
                ncclSuccess)
            break;
        if (recv_bytes[p] &&
            (r = c.api->recv(recv_ptr[p], recv_bytes[p], ncclUint8, p, (ncclComm_t)c.nccl, stream)) !=
                ncclSuccess)
            break;
    }
    const ncclResult_t e = c.api->group_end();
    if (r != ncclSuccess) return rccl_fail(c.api, r, "ncclSend/ncclRecv");
    if (e != ncclSuccess) return rccl_fail(c.api, e, "ncclGroupEnd");
    return SLAM_OK;
}

}  // namespace slam

using namespace slam;

extern "C" {

int slam_comm_unique_id(uint8_t* id_out) {
    SLAM_ARG_CHECK(id_out, "slam_comm_unique_id: NULL argument");
    const Rccl* api = rccl_load();
    if (!api) return fail(SLAM_ERR_COMM, "RCCL unavailable: " + g_rccl_err);
    ncclUniqueId id;
    const ncclResult_t r = api->get_unique_id(&id);
    if (r != ncclSuccess) return rccl_fail(api, r, "ncclGetUniqueId");
    std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return SLAM_OK;
}

int slam_comm_create(const uint8_t* id, int32_t world, int32_t rank, int device, slam_comm** out) {
    SLAM_ARG_CHECK(id && out && world >= 1 && rank >= 0 && rank < world,
                   "slam_comm_create: bad argument");
    *out = nullptr;
    int ndev = 0;
    SLAM_HIP_TRY(hipGetDeviceCount(&ndev));
    SLAM_ARG_CHECK(device >= 0 && device < ndev, "slam_comm_create: no such HIP device");
    const Rccl* api = rccl_load();
    if (!api) return fail(SLAM_ERR_COMM, "RCCL unavailable: " + g_rccl_err);
    SLAM_HIP_TRY(hipSetDevice(device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t nc = nullptr;
    const ncclResult_t r = api->comm_init_rank(&nc, world, uid, rank);
    if (r != ncclSuccess) return rccl_fail(api, r, "ncclCommInitRank");
    slam_comm* h = new slam_comm();
    h->c.world = world;
    h->c.rank = rank;
    h->c.device = device;
    h->c.nccl = nc;
    h->c.api = api;
    *out = h;
    return SLAM_OK;
}

int slam_comm_destroy(slam_comm* h) {
    if (!h) return SLAM_OK;
    if (h->c.nccl && h->c.api) {
        (void)hipSetDevice(h->c.device);
        (void)h->c.api->comm_destroy((ncclComm_t)h->c.nccl);
    }
    delete h;
    return SLAM_OK;
}

int slam_comm_info(slam_comm* h, int32_t* world, int32_t* rank) {
    SLAM_ARG_CHECK(h, "slam_comm_info: NULL handle");
    if (world) *world = h->c.world;
    if (rank) *rank = h->c.rank;
    return SLAM_OK;
}

// all-gather of a host buffer (bootstrap data, e.g. peer-memory handles):
// recv (host, world * bytes) <- send (host, bytes) of every rank, rank order.
int slam_comm_all_gather_host(slam_comm* h, const void* send, void* recv, int64_t bytes) {
    SLAM_ARG_CHECK(h && send && recv && bytes > 0, "slam_comm_all_gather_host: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->c.device));
    void* d = nullptr;
    SLAM_HIP_TRY(hipMalloc(&d, (size_t)bytes * (h->c.world + 1)));
    char* dsend = (char*)d + (size_t)bytes * h->c.world;
    hipStream_t s = nullptr;
    int rc = SLAM_OK;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(d);
        return fail(SLAM_ERR_HIP, "slam_comm_all_gather_host: stream creation failed");
    }
    if (hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
        rc = fail(SLAM_ERR_HIP, "slam_comm_all_gather_host: upload failed");
    if (!rc) rc = comm_all_gather(h->c, dsend, d, (size_t)bytes, s);
    if (!rc && hipMemcpyAsync(recv, d, (size_t)bytes * h->c.world, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(SLAM_ERR_HIP, "slam_comm_all_gather_host: download failed");
    if (!rc && hipStreamSynchronize(s) != hipSuccess)
        rc = fail(SLAM_ERR_HIP, "slam_comm_all_gather_host: synchronize failed");
    (void)hipStreamDestroy(s);
    (void)hipFree(d);
    return rc;
}

}  // extern "C"
