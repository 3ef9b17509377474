// fs2_comm.hpp -- transports for particle sharding.
//
// One rank per GPU; rank r owns the contiguous block of global particles
// [N*r/G, N*(r+1)/G).  Per scan the ranks exchange small records (weight
// totals, normalised statistics) with an all-gather; a resample moves the
// particles whose output range crosses a shard boundary with grouped
// point-to-point transfers.
//
//   RcclTransport   production: ncclAllGather / ncclSend / ncclRecv on the
//                   handle's stream (RCCL over xGMI); one process per GPU.
//   LocalTransport  G ranks as threads of one process (device-to-device
//                   copies + a host barrier).  Exercises every sharded code
//                   path on a single GPU (tests/test_gpu_sharded.py).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fs2.h"

namespace fs2comm {

struct Xfer {
    int peer;
    void *buf;
    size_t bytes;
};

class Transport {
  public:
    virtual ~Transport() {}
    virtual int world() const = 0;
    virtual int rank() const = 0;
    // recv holds world() * bytes, rank order
    virtual int allgather(const void *send, void *recv, size_t bytes, hipStream_t s,
                          std::string *err) = 0;
    // grouped point-to-point: every rank lists what it sends to and receives from each peer
    virtual int exchange(const std::vector<Xfer> &sends, const std::vector<Xfer> &recvs,
                         hipStream_t s, std::string *err) = 0;
};

// ------------------------------------------------------------------ RCCL ---

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

class RcclTransport : public Transport {
  public:
    ncclComm_t comm = nullptr;
    int G = 1, r = 0;
    ~RcclTransport() override {
        if (comm) ncclCommDestroy(comm);
    }
    int world() const override { return G; }
    int rank() const override { return r; }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t s,
                  std::string *err) override {
        ncclResult_t e = ncclAllGather(send, recv, bytes, ncclUint8, comm, s);
        return e == ncclSuccess ? FS2_OK : nccl_fail(e, err, "ncclAllGather");
    }
    int exchange(const std::vector<Xfer> &sends, const std::vector<Xfer> &recvs, hipStream_t s,
                 std::string *err) override {
        ncclResult_t e = ncclGroupStart();
        if (e != ncclSuccess) return nccl_fail(e, err, "ncclGroupStart");
        for (const Xfer &x : sends)
            if (x.bytes && (e = ncclSend(x.buf, x.bytes, ncclUint8, x.peer, comm, s)) != ncclSuccess)
                break;
        if (e == ncclSuccess)
            for (const Xfer &x : recvs)
                if (x.bytes && (e = ncclRecv(x.buf, x.bytes, ncclUint8, x.peer, comm, s)) != ncclSuccess)
                    break;
        ncclResult_t e2 = ncclGroupEnd();
        if (e != ncclSuccess) return nccl_fail(e, err, "ncclSend/ncclRecv");
        return e2 == ncclSuccess ? FS2_OK : nccl_fail(e2, err, "ncclGroupEnd");
    }
};

inline int create_rccl(const uint8_t id_bytes[128], int world, int rank, Transport **out,
                       std::string *err) {
    ncclUniqueId id;
    std::memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
    auto *t = new RcclTransport();
    t->G = world;
    t->r = rank;
    ncclResult_t e = ncclCommInitRank(&t->comm, world, id, rank);
    if (e != ncclSuccess) {
        t->comm = nullptr;
        delete t;
        return nccl_fail(e, err, "ncclCommInitRank");
    }
    *out = t;
    return FS2_OK;
}

// ----------------------------------------------------------------- local ---

struct LocalGroup {
    int G;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const void *> send_ptr;
    std::vector<std::vector<Xfer>> sends;   // per rank: its sends
    explicit LocalGroup(int g) : G(g), send_ptr(g), sends(g) {}

    // all ranks rendezvous; false on timeout (a rank failed or never arrived)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == G) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        return cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen; });
    }
};

inline std::mutex &registry_mu() {
    static std::mutex m;
    return m;
}
inline std::map<std::string, std::weak_ptr<LocalGroup>> &registry() {
    static std::map<std::string, std::weak_ptr<LocalGroup>> r;
    return r;
}

class LocalTransport : public Transport {
  public:
    std::shared_ptr<LocalGroup> grp;
    int r = 0;
    int world() const override { return grp->G; }
    int rank() const override { return r; }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t s,
                  std::string *err) override {
        if (hipStreamSynchronize(s) != hipSuccess) return fail(err, "stream sync");
        grp->send_ptr[r] = send;
        if (!grp->barrier()) return fail(err, "allgather rendezvous timed out");
        for (int p = 0; p < grp->G; ++p)
            if (hipMemcpyAsync((char *)recv + (size_t)p * bytes, grp->send_ptr[p], bytes,
                               hipMemcpyDeviceToDevice, s) != hipSuccess)
                return fail(err, "allgather copy");
        if (hipStreamSynchronize(s) != hipSuccess) return fail(err, "stream sync");
        if (!grp->barrier()) return fail(err, "allgather completion timed out");
        return FS2_OK;
    }
    int exchange(const std::vector<Xfer> &sends, const std::vector<Xfer> &recvs, hipStream_t s,
                 std::string *err) override {
        if (hipStreamSynchronize(s) != hipSuccess) return fail(err, "stream sync");
        grp->sends[r] = sends;
        if (!grp->barrier()) return fail(err, "exchange rendezvous timed out");
        for (const Xfer &x : recvs) {
            if (!x.bytes) continue;
            const Xfer *match = nullptr;
            for (const Xfer &y : grp->sends[x.peer])
                if (y.peer == r) match = &y;
            if (!match || match->bytes != x.bytes) return fail(err, "exchange size mismatch");
            if (hipMemcpyAsync(x.buf, match->buf, x.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return fail(err, "exchange copy");
        }
        if (hipStreamSynchronize(s) != hipSuccess) return fail(err, "stream sync");
        if (!grp->barrier()) return fail(err, "exchange completion timed out");
        return FS2_OK;
    }

  private:
    static int fail(std::string *err, const char *what) {
        if (err) *err = std::string("local transport: ") + what;
        return FS2_ERR_COMM;
    }
};

inline int create_local(const uint8_t key[128], int world, int rank, Transport **out,
                        std::string *err) {
    const std::string k(reinterpret_cast<const char *>(key), 128);
    std::lock_guard<std::mutex> lk(registry_mu());
    auto &reg = registry();
    std::shared_ptr<LocalGroup> g = reg[k].lock();
    if (!g) {
        g = std::make_shared<LocalGroup>(world);
        reg[k] = g;
    }
    if (g->G != world) {
        if (err) *err = "local transport: world size mismatch for group key";
        return FS2_ERR_ARG;
    }
    auto *t = new LocalTransport();
    t->grp = g;
    t->r = rank;
    *out = t;
    return FS2_OK;
}

}  // namespace fs2comm
