// comm.hpp -- the multi-GPU exchange layer of libslam_hip.so.
//
// One process per GPU.  Collectives go through RCCL (NCCL API; over xGMI on
// an MI355X node), loaded at run time with dlopen: the library has no link-time
// RCCL dependency, and a process that already holds an RCCL (e.g. the one
// PyTorch ships, same soname) shares it.  A communicator is either an RCCL
// communicator (one rank of world) or a LOCAL one: several ranks held by the
// same process (tests; several shards on one GPU), whose collectives are
// device copies between the shards' buffers on one stream.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include <hip/hip_runtime.h>

namespace slam {

struct Rccl;   // dlopen'd RCCL entry points (comm_api.hip)

struct Comm {
    int world = 1;
    int rank = 0;
    int device = 0;
    void* nccl = nullptr;        // ncclComm_t (RCCL communicator), or nullptr for LOCAL
    const Rccl* api = nullptr;
    bool local = false;          // LOCAL: every rank lives in this process
};

// Collectives on `stream` (enqueued; asynchronous; graph-capturable for RCCL).
// all_gather: recv[rank * bytes .. +bytes] <- send of every rank.
int comm_all_gather(const Comm& c, const void* send, void* recv, size_t bytes, hipStream_t stream);
// grouped point-to-point: for every peer p != rank, send send_bytes[p] from
// send_ptr[p] and receive recv_bytes[p] into recv_ptr[p].
int comm_exchange(const Comm& c, const std::vector<const void*>& send_ptr,
                  const std::vector<size_t>& send_bytes, const std::vector<void*>& recv_ptr,
                  const std::vector<size_t>& recv_bytes, hipStream_t stream);

}  // namespace slam

// the C-ABI's communicator handle (slam_hip.h: slam_comm)
struct slam_comm {
    slam::Comm c;
};
