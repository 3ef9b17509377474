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
//   ShmTransport    G ranks as processes of one host (several may share a GPU),
//                   stream-ordered like RCCL: pinned staging copies around one
//                   host function per collective that moves the bytes through a
//                   POSIX shared-memory segment behind a process barrier
//                   (tests/test_gpu_sharded_procs.py).
#pragma once

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
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
    // a failure inside a stream-ordered collective (after the call returned), else FS2_OK
    virtual int status(std::string *) { return FS2_OK; }
    // page_refs mode, at creation (no collective in flight): every rank's base of one
    // device allocation (hipMalloc base), mapped into this process -- peers[r] for
    // rank r, this rank's own base at peers[rank()]; unmapped with the transport
    virtual int share(void *base, void **peers, std::string *err) = 0;
    void unshare() { close_handles(); }
    // ranks are threads of one process (their handles are closed one after another)
    virtual bool in_process() const { return false; }

  protected:
    // a host-side rendezvous of every rank (creation-time use only)
    virtual bool host_barrier(std::string *err) = 0;
    std::vector<void *> opened_;     // IPC mappings to close
    // The ranks open each other's handles one rank at a time (a rendezvous between
    // turns): on ROCm 7.2 with dmabuf IPC, processes that all sat in
    // hipIpcOpenMemHandle at once never returned (8 processes on one GPU,
    // FS2_TRACE).  Every rank takes every turn's rendezvous, whatever its own
    // opens did.
    int open_handles(const std::vector<hipIpcMemHandle_t> &hs, void *base, void **peers, std::string *err) {
        const bool tr = std::getenv("FS2_TRACE") != nullptr;
        int rc = FS2_OK;
        for (int turn = 0; turn < (int)hs.size(); ++turn) {
            if (turn == rank()) {
                for (int p = 0; p < (int)hs.size() && rc == FS2_OK; ++p) {
                    if (p == rank()) {
                        peers[p] = base;
                        continue;
                    }
                    void *q = nullptr;
                    if (tr) std::fprintf(stderr, "[fs2 rank %d] open handle of rank %d\n", rank(), p);
                    if (hipIpcOpenMemHandle(&q, hs[p], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                        (void)hipGetLastError();     // reported here, not by the next launch
                        if (err) *err = "hipIpcOpenMemHandle failed (page references across ranks)";
                        rc = FS2_ERR_COMM;
                        break;
                    }
                    opened_.push_back(q);
                    peers[p] = q;
                }
            }
            std::string berr;
            if (!host_barrier(&berr)) {
                if (err) *err = berr;
                return FS2_ERR_COMM;
            }
        }
        return rc;
    }
    void close_handles() {
        for (void *q : opened_) hipIpcCloseMemHandle(q);
        opened_.clear();
    }
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
    bool failed_ = false;             // an IPC handle exchange failed: the communicator is unusable
    int status(std::string *err) override {
        if (!failed_) return FS2_OK;
        if (err) *err = "rccl transport: the IPC handle exchange failed";
        return FS2_ERR_COMM;
    }
    ~RcclTransport() override {
        close_handles();
        if (comm) ncclCommDestroy(comm);
    }
    // (a rank whose handle or mappings fail still takes part in the exchange; it
    // returns the failure, fs2_api's agreement turns the mode off on every rank)
    int share(void *base, void **peers, std::string *err) override {
        hipIpcMemHandle_t mine;
        const bool got = hipIpcGetMemHandle(&mine, base) == hipSuccess;
        if (!got) {
            (void)hipGetLastError();
            std::memset(&mine, 0, sizeof mine);
        }
        std::vector<hipIpcMemHandle_t> hs(G);
        char *d = nullptr;
        hipStream_t s = nullptr;
        int rc = FS2_OK;
        if (hipMalloc(&d, sizeof(hipIpcMemHandle_t) * (G + 1)) != hipSuccess ||
            hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            rc = FS2_ERR_COMM;
            if (err) *err = "IPC handle exchange buffers";
        }
        if (!rc && hipMemcpy(d, &mine, sizeof mine, hipMemcpyHostToDevice) != hipSuccess) rc = FS2_ERR_COMM;
        if (!rc) {
            ncclResult_t e = ncclAllGather(d, d + sizeof mine, sizeof mine, ncclUint8, comm, s);
            if (e != ncclSuccess) rc = nccl_fail(e, err, "ncclAllGather (IPC handles)");
        }
        if (!rc && (hipStreamSynchronize(s) != hipSuccess ||
                    hipMemcpy(hs.data(), d + sizeof mine, sizeof mine * G, hipMemcpyDeviceToHost) != hipSuccess))
            rc = FS2_ERR_COMM;
        if (s) hipStreamDestroy(s);
        hipFree(d);
        if (rc) {
            failed_ = true;           // the exchange itself: the communicator is unusable
            return rc;
        }
        if (!got) {
            if (err) *err = "hipIpcGetMemHandle failed";
            return FS2_ERR_COMM;
        }
        return open_handles(hs, base, peers, err);
    }
    int world() const override { return G; }
    int rank() const override { return r; }
  protected:
    bool host_barrier(std::string *err) override {
        char *d = nullptr;
        hipStream_t s = nullptr;
        bool ok = hipMalloc(&d, (size_t)G + 1) == hipSuccess &&
                  hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
                  ncclAllGather(d, d + 1, 1, ncclUint8, comm, s) == ncclSuccess && hipStreamSynchronize(s) == hipSuccess;
        if (s) hipStreamDestroy(s);
        hipFree(d);
        if (!ok) {
            (void)hipGetLastError();
            failed_ = true;
            if (err) *err = "rccl transport: rendezvous failed";
        }
        return ok;
    }
  public:
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

    bool in_process() const override { return true; }

  protected:
    bool host_barrier(std::string *err) override {
        if (grp->barrier()) return true;
        if (err) *err = "local transport: rendezvous timed out";
        return false;
    }

  public:
    // ranks are threads of this process: the bases themselves
    int share(void *base, void **peers, std::string *err) override {
        grp->send_ptr[r] = base;
        if (!grp->barrier()) return fail(err, "share rendezvous timed out");
        for (int p = 0; p < grp->G; ++p) peers[p] = const_cast<void *>(grp->send_ptr[p]);
        if (!grp->barrier()) return fail(err, "share completion timed out");
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

// ------------------------------------------------------------------- shm ---
//
// Segment: a header (barriers, per-rank round counts), one all-gather slot per
// rank and a mailbox per ordered pair of ranks (`chunk` bytes + a 64-byte
// header naming the transfer's size and round).  A collective is
//   hipMemcpyAsync  device -> this process's pinned staging
//   hipLaunchHostFunc  staging -> segment, barrier, segment -> staging, barrier
//   hipMemcpyAsync  pinned staging -> device
// on the caller's stream; the host function runs when the stream reaches it,
// so the bytes it moves are the ones the kernels before it produced, and the
// kernels after it see what arrived -- the ordering RCCL's kernels give, without
// a host-side stream sync.  Transfers larger than a mailbox go in rounds; every
// rank runs max over ranks of its own round count (agreed through the header).

constexpr uint64_t kShmMagic = 0x66733273686d3031ull;   // "fs2shm01"
constexpr size_t kShmAgCap = 16384;                     // all-gather bytes per rank (ChainSummary, RankRecordX)
constexpr size_t kShmHeader = 4096;
constexpr size_t kShmBoxHeader = 64;
constexpr int kShmMaxRanks = 16;                        // >= fs2::kMaxRanks (static_assert in fs2_api.hip)

struct ShmBarrier {
    std::atomic<uint32_t> count;
    std::atomic<uint32_t> gen;
    char pad[56];
};

struct ShmHeader {
    std::atomic<uint64_t> magic;
    int32_t G;
    int32_t pad0;
    uint64_t chunk;
    std::atomic<uint32_t> failed;          // some rank timed out or saw a size mismatch
    char pad1[36];
    ShmBarrier attach;                     // creation
    ShmBarrier bar;                        // collectives (host functions)
    std::atomic<int64_t> need[kShmMaxRanks];  // rounds the current exchange needs, per rank
};
static_assert(sizeof(ShmHeader) <= kShmHeader, "shm header");
static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<int64_t>::is_always_lock_free &&
                  std::atomic<uint64_t>::is_always_lock_free,
              "process-shared atomics must be lock-free");

struct ShmBox {
    int64_t total;                         // bytes of the whole transfer
    int64_t round;
    char pad[kShmBoxHeader - 16];
};

inline size_t shm_segment_bytes(int G, size_t chunk) {
    return kShmHeader + (size_t)G * kShmAgCap + (size_t)G * G * (kShmBoxHeader + chunk);
}

class ShmTransport : public Transport {
  public:
    int G = 1, r = 0;
    char *seg = nullptr;
    size_t seg_bytes = 0;
    ShmHeader *hdr = nullptr;
    size_t chunk = 0;
    std::chrono::milliseconds timeout{60000};
    char *ag_send = nullptr, *ag_recv = nullptr;          // pinned
    std::vector<char *> xs, xr;                           // pinned, per peer
    std::vector<size_t> xs_cap, xr_cap;
    std::mutex fmu;
    std::string fmsg;                                     // first failure seen by a host function
    std::atomic<int> failed{0};

    ~ShmTransport() override {
        close_handles();
        if (ag_send) hipHostFree(ag_send);
        if (ag_recv) hipHostFree(ag_recv);
        for (char *p : xs) if (p) hipHostFree(p);
        for (char *p : xr) if (p) hipHostFree(p);
        if (seg) munmap(seg, seg_bytes);
    }
    int world() const override { return G; }
    int rank() const override { return r; }

    char *slot(int p) const { return seg + kShmHeader + (size_t)p * kShmAgCap; }
    ShmBox *box(int from, int to) const {
        return reinterpret_cast<ShmBox *>(seg + kShmHeader + (size_t)G * kShmAgCap +
                                          ((size_t)from * G + to) * (kShmBoxHeader + chunk));
    }
    char *box_data(int from, int to) const { return reinterpret_cast<char *>(box(from, to)) + kShmBoxHeader; }

    // sense-counting barrier over the segment; false when a rank failed or the
    // wait exceeded the timeout (then every rank's later waits fail at once)
    bool wait(ShmBarrier &b) {
        if (hdr->failed.load(std::memory_order_acquire)) return false;
        const uint32_t g = b.gen.load(std::memory_order_acquire);
        if (b.count.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)G - 1) {
            b.count.store(0, std::memory_order_relaxed);
            b.gen.store(g + 1, std::memory_order_release);
            return true;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned it = 0;; ++it) {
            if (b.gen.load(std::memory_order_acquire) != g) return true;
            if ((it & 255u) == 255u) {
                if (hdr->failed.load(std::memory_order_acquire)) return false;
                const auto dt = std::chrono::steady_clock::now() - t0;
                if (dt > timeout) {
                    hdr->failed.store(1, std::memory_order_release);
                    return false;
                }
                if (dt > std::chrono::milliseconds(2)) std::this_thread::sleep_for(std::chrono::microseconds(20));
                else std::this_thread::yield();
            } else {
                __builtin_ia32_pause();
            }
        }
    }
    void note_fail(const char *what) {
        std::lock_guard<std::mutex> lk(fmu);
        if (!failed.exchange(1)) fmsg = std::string("shm transport: ") + what;
        hdr->failed.store(1, std::memory_order_release);
    }
    int status(std::string *err) override {
        if (!failed.load() && !hdr->failed.load(std::memory_order_acquire)) return FS2_OK;
        std::lock_guard<std::mutex> lk(fmu);
        if (err) *err = fmsg.empty() ? std::string("shm transport: another rank failed") : fmsg;
        return FS2_ERR_COMM;
    }

  protected:
    bool host_barrier(std::string *err) override {
        if (wait(hdr->bar)) return true;
        fail(err, "rendezvous failed or timed out");
        return false;
    }

  public:
    // the handles through the all-gather slots, host-side (creation: nothing in flight)
    int share(void *base, void **peers, std::string *err) override {
        if (int rc = status(err)) return rc;
        hipIpcMemHandle_t mine;
        if (hipIpcGetMemHandle(&mine, base) != hipSuccess) return fail(err, "hipIpcGetMemHandle failed");
        std::memcpy(slot(r), &mine, sizeof mine);
        if (!wait(hdr->bar)) return fail(err, "share rendezvous failed or timed out");
        std::vector<hipIpcMemHandle_t> hs(G);
        for (int p = 0; p < G; ++p) std::memcpy(&hs[p], slot(p), sizeof mine);
        if (!wait(hdr->bar)) return fail(err, "share completion failed or timed out");
        return open_handles(hs, base, peers, err);
    }

    int allgather(const void *send, void *recv, size_t bytes, hipStream_t s, std::string *err) override {
        if (int rc = status(err)) return rc;
        if (bytes > kShmAgCap) return fail(err, "all-gather larger than its slot");
        if (hipMemcpyAsync(ag_send, send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
            return fail(err, "all-gather copy to staging");
        auto *op = new AgOp{this, bytes};
        if (hipLaunchHostFunc(s, &ShmTransport::ag_host, op) != hipSuccess) {
            delete op;
            return fail(err, "hipLaunchHostFunc");
        }
        if (hipMemcpyAsync(recv, ag_recv, bytes * G, hipMemcpyHostToDevice, s) != hipSuccess)
            return fail(err, "all-gather copy from staging");
        return FS2_OK;
    }

    int exchange(const std::vector<Xfer> &sends, const std::vector<Xfer> &recvs, hipStream_t s,
                 std::string *err) override {
        if (int rc = status(err)) return rc;
        auto *op = new XOp{this, std::vector<size_t>(G, 0), std::vector<size_t>(G, 0)};
        int rc = FS2_OK;
        for (const Xfer &x : sends) {
            if (x.peer < 0 || x.peer >= G || x.peer == r) rc = fail(err, "exchange peer out of range");
            else if (x.bytes && !(rc = stage(xs, xs_cap, x.peer, x.bytes, s, err)))
                op->send[x.peer] = x.bytes;
            if (rc) break;
        }
        for (const Xfer &x : recvs) {
            if (rc) break;
            if (x.peer < 0 || x.peer >= G || x.peer == r) rc = fail(err, "exchange peer out of range");
            else if (x.bytes && !(rc = stage(xr, xr_cap, x.peer, x.bytes, s, err)))
                op->recv[x.peer] = x.bytes;
        }
        if (rc) {
            delete op;
            return rc;
        }
        for (const Xfer &x : sends)
            if (x.bytes && hipMemcpyAsync(xs[x.peer], x.buf, x.bytes, hipMemcpyDeviceToHost, s) != hipSuccess) {
                delete op;
                return fail(err, "exchange copy to staging");
            }
        if (hipLaunchHostFunc(s, &ShmTransport::x_host, op) != hipSuccess) {
            delete op;
            return fail(err, "hipLaunchHostFunc");
        }
        for (const Xfer &x : recvs)
            if (x.bytes && hipMemcpyAsync(x.buf, xr[x.peer], x.bytes, hipMemcpyHostToDevice, s) != hipSuccess)
                return fail(err, "exchange copy from staging");
        return FS2_OK;
    }

  private:
    struct AgOp {
        ShmTransport *t;
        size_t bytes;
    };
    struct XOp {
        ShmTransport *t;
        std::vector<size_t> send, recv;   // bytes per peer
    };
    static int fail(std::string *err, const char *what) {
        if (err) *err = std::string("shm transport: ") + what;
        return FS2_ERR_COMM;
    }
    // pinned staging for one peer; growing drains the stream first (earlier
    // collectives may still copy through the old buffer)
    int stage(std::vector<char *> &v, std::vector<size_t> &cap, int p, size_t bytes, hipStream_t s,
              std::string *err) {
        if (cap[p] >= bytes) return FS2_OK;
        if (hipStreamSynchronize(s) != hipSuccess) return fail(err, "stream sync");
        if (v[p]) hipHostFree(v[p]);
        v[p] = nullptr;
        cap[p] = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 20);
        if (hipHostMalloc((void **)&v[p], want, 0) != hipSuccess) return fail(err, "pinned staging allocation");
        cap[p] = want;
        return FS2_OK;
    }
    static void ag_host(void *u) {
        AgOp *op = static_cast<AgOp *>(u);
        ShmTransport *t = op->t;
        const size_t b = op->bytes;
        delete op;
        std::memcpy(t->slot(t->r), t->ag_send, b);
        if (!t->wait(t->hdr->bar)) return t->note_fail("all-gather rendezvous failed or timed out");
        for (int p = 0; p < t->G; ++p) std::memcpy(t->ag_recv + (size_t)p * b, t->slot(p), b);
        if (!t->wait(t->hdr->bar)) t->note_fail("all-gather completion failed or timed out");
    }
    static void x_host(void *u) {
        XOp *op = static_cast<XOp *>(u);
        ShmTransport *t = op->t;
        const int G = t->G, me = t->r;
        const size_t C = t->chunk;
        int64_t mine = 0;
        for (int p = 0; p < G; ++p)
            mine = std::max<int64_t>(mine, (int64_t)((std::max(op->send[p], op->recv[p]) + C - 1) / C));
        t->hdr->need[me].store(mine, std::memory_order_release);
        int64_t R = 0;
        bool ok = t->wait(t->hdr->bar);
        if (ok) {
            for (int p = 0; p < G; ++p) R = std::max(R, t->hdr->need[p].load(std::memory_order_acquire));
            ok = t->wait(t->hdr->bar);     // need[] is rewritten by the next exchange
        }
        for (int64_t k = 0; ok && k < R; ++k) {
            const size_t off = (size_t)k * C;
            for (int p = 0; p < G; ++p)
                if (op->send[p] > off) {
                    ShmBox *bx = t->box(me, p);
                    bx->total = (int64_t)op->send[p];
                    bx->round = k;
                    std::memcpy(t->box_data(me, p), t->xs[p] + off, std::min(C, op->send[p] - off));
                }
            if (!(ok = t->wait(t->hdr->bar))) break;
            for (int q = 0; q < G; ++q)
                if (op->recv[q] > off) {
                    const ShmBox *bx = t->box(q, me);
                    if (bx->total != (int64_t)op->recv[q] || bx->round != k) {
                        t->note_fail("exchange size mismatch between sender and receiver");
                        ok = false;
                        break;
                    }
                    std::memcpy(t->xr[q] + off, t->box_data(q, me), std::min(C, op->recv[q] - off));
                }
            if (ok) ok = t->wait(t->hdr->bar);
        }
        if (!ok) t->note_fail("exchange rendezvous failed or timed out");
        delete op;
    }
};

inline int create_shm(const uint8_t key[128], int world, int rank, Transport **out, std::string *err) {
    auto bad = [&](const std::string &what) {
        if (err) *err = "shm transport: " + what;
        return FS2_ERR_COMM;
    };
    if (world < 1 || world > kShmMaxRanks) return bad("world size out of range");
    char name[64];
    int k = std::snprintf(name, sizeof name, "/fs2shm.");
    for (int i = 0; i < 16; ++i) k += std::snprintf(name + k, sizeof name - k, "%02x", key[i]);
    long tmo_s = 60;
    if (const char *e = std::getenv("FS2_SHM_TIMEOUT_S")) tmo_s = std::max(1L, std::atol(e));
    size_t chunk = std::min<size_t>(4u << 20, std::max<size_t>(64u << 10, (256u << 20) / ((size_t)world * world)));
    if (const char *e = std::getenv("FS2_SHM_CHUNK")) chunk = std::max<size_t>(4096, std::strtoull(e, nullptr, 10));
    chunk = (chunk + 63) / 64 * 64;
    // creation waits for every rank to start (a process importing its runtime may
    // take a while), so it allows at least a minute whatever the collective timeout
    const long attach_s = std::max(tmo_s, 60L);
    const auto t0 = std::chrono::steady_clock::now();
    const auto deadline = t0 + std::chrono::seconds(attach_s);
    int fd = -1;
    size_t bytes = 0;
    char *seg = nullptr;
    if (rank == 0) {
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) return bad(std::string("shm_open(") + name + ") failed: " + std::strerror(errno));
        bytes = shm_segment_bytes(world, chunk);
        if (ftruncate(fd, (off_t)bytes) != 0) {
            close(fd);
            shm_unlink(name);
            return bad("ftruncate failed");
        }
        seg = (char *)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (seg == MAP_FAILED) {
            shm_unlink(name);
            return bad("mmap failed");
        }
        auto *h = new (seg) ShmHeader();
        h->G = world;
        h->chunk = chunk;
        h->failed.store(0);
        h->attach.count.store(0);
        h->attach.gen.store(0);
        h->bar.count.store(0);
        h->bar.gen.store(0);
        for (auto &v : h->need) v.store(0);
        h->magic.store(kShmMagic, std::memory_order_release);
    } else {
        while ((fd = shm_open(name, O_RDWR, 0)) < 0) {
            if (std::chrono::steady_clock::now() > deadline) return bad("rank 0's segment never appeared");
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
        // the header first (rank 0 may still be sizing the segment), then all of it
        struct stat sb {};
        while (fstat(fd, &sb) != 0 || (size_t)sb.st_size < kShmHeader) {
            if (std::chrono::steady_clock::now() > deadline) {
                close(fd);
                return bad("segment never sized");
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        char *hp = (char *)mmap(nullptr, kShmHeader, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (hp == MAP_FAILED) {
            close(fd);
            return bad("mmap failed");
        }
        auto *h = reinterpret_cast<ShmHeader *>(hp);
        while (h->magic.load(std::memory_order_acquire) != kShmMagic) {
            if (std::chrono::steady_clock::now() > deadline) {
                munmap(hp, kShmHeader);
                close(fd);
                return bad("segment never initialised");
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        const int G0 = h->G;
        chunk = h->chunk;
        munmap(hp, kShmHeader);
        if (G0 != world) {
            close(fd);
            return bad("world size differs from rank 0's");
        }
        bytes = shm_segment_bytes(world, chunk);
        seg = (char *)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (seg == MAP_FAILED) return bad("mmap failed");
    }
    auto *t = new ShmTransport();
    t->G = world;
    t->r = rank;
    t->seg = seg;
    t->seg_bytes = bytes;
    t->hdr = reinterpret_cast<ShmHeader *>(seg);
    t->chunk = chunk;
    t->timeout = std::chrono::milliseconds(attach_s * 1000);
    t->xs.assign(world, nullptr);
    t->xr.assign(world, nullptr);
    t->xs_cap.assign(world, 0);
    t->xr_cap.assign(world, 0);
    if (hipHostMalloc((void **)&t->ag_send, kShmAgCap, 0) != hipSuccess ||
        hipHostMalloc((void **)&t->ag_recv, kShmAgCap * world, 0) != hipSuccess) {
        t->hdr->failed.store(1);
        if (rank == 0) shm_unlink(name);
        delete t;
        return bad("pinned staging allocation failed");
    }
    // every rank mapped the segment: its name is no longer needed (nothing stays
    // behind in /dev/shm, whatever happens to the processes later)
    const bool ok = t->wait(t->hdr->attach);
    t->timeout = std::chrono::milliseconds(tmo_s * 1000);
    if (rank == 0) shm_unlink(name);
    if (!ok) {
        delete t;
        return bad("ranks did not all attach in time");
    }
    *out = t;
    return FS2_OK;
}

}  // namespace fs2comm
