// fs2_comm.hpp -- RCCL (over xGMI) plumbing for particle sharding.
//
// One process per GPU; each rank owns a contiguous block of particles.  Per
// scan the ranks exchange two small records (weight totals, then normalised
// statistics) with ncclAllGather on the handle's stream; resampling moves
// particle maps between neighbouring ranks with grouped ncclSend/ncclRecv.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/fs2.h"

namespace fs2comm {

struct Comm {
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0;
};

inline int nccl_fail(ncclResult_t r, std::string *err, const char *what) {
    if (err) *err = std::string(what) + ": " + ncclGetErrorString(r);
    return FS2_ERR_COMM;
}

inline int unique_id(uint8_t out[128], std::string *err) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return nccl_fail(r, err, "ncclGetUniqueId");
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return FS2_OK;
}

inline int create(const uint8_t id_bytes[128], int world, int rank, Comm **out, std::string *err) {
    ncclUniqueId id;
    std::memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
    Comm *c = new Comm();
    c->world = world;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, err, "ncclCommInitRank");
    }
    *out = c;
    return FS2_OK;
}

inline void destroy(Comm *c) {
    if (!c) return;
    if (c->comm) ncclCommDestroy(c->comm);
    delete c;
}

inline int allgather_bytes(Comm *c, const void *send, void *recv, size_t bytes, hipStream_t s,
                           std::string *err) {
    ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, c->comm, s);
    if (r != ncclSuccess) return nccl_fail(r, err, "ncclAllGather");
    return FS2_OK;
}

}  // namespace fs2comm
