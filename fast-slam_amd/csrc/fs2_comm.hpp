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
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
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

// One physical chunk of an allocation that grows in place (fs2_api.hip GrowMem):
// the chunks are mapped back to back from the allocation's base.
struct VmChunk {
    hipMemGenericAllocationHandle_t hd;
    size_t bytes;
};

// ---- file descriptors between the processes of one host (page_refs) ----
//
// A rank's pools are VMM chunks exported as POSIX file descriptors
// (hipMemExportToShareableHandle) and handed to the other ranks over Unix
// SOCK_SEQPACKET sockets in the abstract namespace (SCM_RIGHTS), named from the
// group key and the rank.  hipIpcOpenMemHandle is not used between processes:
// the runtime's own dmabuf IPC did not complete an open in a process that had
// exported an allocation itself (profiles/r05_ipc_probe.txt), and every rank
// exports its pools and opens the others'.
namespace uds {
inline bool name(const std::string &key, int rank, sockaddr_un *a, socklen_t *len) {
    std::memset(a, 0, sizeof *a);
    a->sun_family = AF_UNIX;
    const int k = std::snprintf(a->sun_path + 1, sizeof a->sun_path - 1, "fs2vm.%s.%d", key.c_str(), rank);
    if (k <= 0 || k >= (int)sizeof a->sun_path - 1) return false;
    *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + k);
    return true;
}
inline int listen_on(const std::string &key, int rank) {
    sockaddr_un a;
    socklen_t len;
    if (!name(key, rank, &a, &len)) return -1;
    const int fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    if (bind(fd, (sockaddr *)&a, len) != 0 || listen(fd, 64) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}
inline bool wait_fd(int fd, short ev, int ms) {
    pollfd p{fd, ev, 0};
    return poll(&p, 1, ms) == 1 && (p.revents & ev);
}
// the connected peer runs under this process's user (SO_PEERCRED)
inline bool peer_is_us(int fd) {
    ucred cr{};
    socklen_t len = sizeof cr;
    return getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &len) == 0 && len == sizeof cr && cr.uid == getuid();
}
inline int accept_one(int lfd, int ms) {
    if (!wait_fd(lfd, POLLIN, ms)) return -1;
    return accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
}
inline int connect_to(const std::string &key, int rank, int ms) {
    sockaddr_un a;
    socklen_t len;
    if (!name(key, rank, &a, &len)) return -1;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const int fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
        if (fd < 0) return -1;
        if (connect(fd, (sockaddr *)&a, len) == 0) return fd;
        close(fd);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms)) return -1;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}
// one message: `len` bytes and up to 250 descriptors
inline bool send_msg(int fd, const void *buf, size_t len, const int *fds, int nfd) {
    iovec io{const_cast<void *>(buf), len};
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    std::vector<char> ctl;
    if (nfd > 0) {
        ctl.assign(CMSG_SPACE(sizeof(int) * (size_t)nfd), 0);
        m.msg_control = ctl.data();
        m.msg_controllen = ctl.size();
        cmsghdr *c = CMSG_FIRSTHDR(&m);
        c->cmsg_level = SOL_SOCKET;
        c->cmsg_type = SCM_RIGHTS;
        c->cmsg_len = CMSG_LEN(sizeof(int) * (size_t)nfd);
        std::memcpy(CMSG_DATA(c), fds, sizeof(int) * (size_t)nfd);
    }
    return sendmsg(fd, &m, MSG_NOSIGNAL) == (ssize_t)len;
}
inline ssize_t recv_msg(int fd, void *buf, size_t len, int *fds, int maxfd, int *nfd, int ms) {
    *nfd = 0;
    if (!wait_fd(fd, POLLIN, ms)) return -1;
    iovec io{buf, len};
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    std::vector<char> ctl(CMSG_SPACE(sizeof(int) * (size_t)std::max(maxfd, 1)), 0);
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    const ssize_t n = recvmsg(fd, &m, MSG_CMSG_CLOEXEC);
    if (n < 0) return n;
    for (cmsghdr *c = CMSG_FIRSTHDR(&m); c; c = CMSG_NXTHDR(&m, c))
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) {
            const int k = (int)((c->cmsg_len - CMSG_LEN(0)) / sizeof(int));
            for (int i = 0; i < k; ++i) {
                int f;
                std::memcpy(&f, CMSG_DATA(c) + sizeof(int) * (size_t)i, sizeof f);
                if (*nfd < maxfd) fds[(*nfd)++] = f;
                else close(f);
            }
        }
    return n;
}
}  // namespace uds

// hipMemImportFromShareableHandle takes a pointer to the descriptor on the HIP 7.0
// runtime PyTorch's wheel brings (the descriptor itself crashes it) and the
// descriptor itself on ROCm 7.2 (a pointer is refused there): profiles/r05_ipc_probe.txt.
// Only those two measured ABIs are used; any other runtime version fails the
// import cleanly (page_refs then falls back to the page transfer on every rank)
// rather than probing with a value the runtime might dereference.
enum class FdAbi { pointer, value, unknown };
inline FdAbi fd_abi(int ver) {
    if (ver >= 70000000 && ver < 70100000) return FdAbi::pointer;     // 7.0.x (measured: 7.0.51831)
    if (ver >= 70200000 && ver < 70300000) return FdAbi::value;       // 7.2.x (measured: 7.2.26015, ROCm 7.2.0)
    return FdAbi::unknown;
}
inline hipError_t import_fd(hipMemGenericAllocationHandle_t *hd, int fd) {
    static const int ver = [] {
        int v = 0;
        return hipRuntimeGetVersion(&v) == hipSuccess ? v : 0;
    }();
    int f = fd;
    switch (fd_abi(ver)) {
    case FdAbi::pointer:
        return hipMemImportFromShareableHandle(hd, &f, hipMemHandleTypePosixFileDescriptor);
    case FdAbi::value:
        return hipMemImportFromShareableHandle(hd, (void *)(intptr_t)fd, hipMemHandleTypePosixFileDescriptor);
    default:
        return hipErrorNotSupported;
    }
}

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
    // page_refs mode, ranks that are processes: every rank's allocation made of VMM
    // `chunks` (exportable as POSIX descriptors) from `base`, mapped into this
    // process for `device` (peers[rank()] = base).  The descriptors go over Unix
    // sockets one rank at a time (a rendezvous between turns); every rank takes
    // every turn whatever its own imports did.
    virtual int share_vm(const std::vector<VmChunk> &chunks, void *base, int device, void **peers,
                         std::string *err) {
        return share_vm_uds(chunks, base, device, peers, err);
    }
    void unshare() { close_handles(); }
    std::string group_key;          // hex of the group key / unique id: names the ranks' sockets
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
    struct VmImport {
        char *base;
        size_t bytes;
        std::vector<hipMemGenericAllocationHandle_t> hds;
    };
    std::vector<VmImport> vm_opened_;     // peers' chunks mapped here
    int lfd_ = -1;                       // this rank's listening socket (share_vm_uds)
    void close_handles() {
        for (void *q : opened_) (void)hipIpcCloseMemHandle(q);
        opened_.clear();
        for (auto &v : vm_opened_) {
            if (v.base) {
                (void)hipMemUnmap(v.base, v.bytes);
                (void)hipMemAddressFree(v.base, v.bytes);
            }
            for (auto hd : v.hds) (void)hipMemRelease(hd);
        }
        vm_opened_.clear();
    }
    void close_listener() {
        if (lfd_ >= 0) close(lfd_);
        lfd_ = -1;
    }
    // the peer's chunks (descriptors, sizes) mapped back to back into a fresh range
    int map_peer(const std::vector<int> &fds, const std::vector<uint64_t> &sizes, int device, void **out) {
        VmImport v{nullptr, 0, {}};
        for (uint64_t b : sizes) v.bytes += b;
        bool ok = fds.size() == sizes.size() && v.bytes > 0;
        for (size_t k = 0; ok && k < fds.size(); ++k) {
            hipMemGenericAllocationHandle_t hd{};
            ok = import_fd(&hd, fds[k]) == hipSuccess;
            if (ok) v.hds.push_back(hd);
        }
        void *p = nullptr;
        ok = ok && hipMemAddressReserve(&p, v.bytes, 0, nullptr, 0) == hipSuccess;
        if (ok) v.base = (char *)p;
        size_t off = 0, mapped = 0;
        for (size_t k = 0; ok && k < v.hds.size(); ++k) {
            ok = hipMemMap(v.base + off, sizes[k], 0, v.hds[k], 0) == hipSuccess;
            if (ok) mapped = off + sizes[k];
            off += sizes[k];
        }
        if (ok) {
            hipMemAccessDesc ad{};
            ad.location.type = hipMemLocationTypeDevice;
            ad.location.id = device;
            ad.flags = hipMemAccessFlagsProtReadWrite;
            ok = hipMemSetAccess(v.base, v.bytes, &ad, 1) == hipSuccess;
        }
        for (int f : fds) close(f);
        if (!ok) {
            (void)hipGetLastError();
            if (v.base) {
                if (mapped) (void)hipMemUnmap(v.base, mapped);
                (void)hipMemAddressFree(v.base, v.bytes);
            }
            for (auto hd : v.hds) (void)hipMemRelease(hd);
            return FS2_ERR_COMM;
        }
        *out = v.base;
        vm_opened_.push_back(std::move(v));
        return FS2_OK;
    }
    int share_vm_uds(const std::vector<VmChunk> &chunks, void *base, int device, void **peers, std::string *err) {
        const int G = world(), me = rank();
        const int ms = 60000;
        int rc = FS2_OK;
        auto note = [&](const char *what) {
            if (rc == FS2_OK && err) *err = std::string("page_refs (VMM descriptors): ") + what;
            rc = FS2_ERR_COMM;
        };
        // this rank's chunks as descriptors (closed at the end: the peers hold their own)
        std::vector<int> mine;
        std::vector<uint64_t> sizes;
        for (const VmChunk &c : chunks) {
            int fd = -1;
            if (hipMemExportToShareableHandle(&fd, c.hd, hipMemHandleTypePosixFileDescriptor, 0) != hipSuccess) {
                (void)hipGetLastError();
                note("hipMemExportToShareableHandle failed");
                break;
            }
            mine.push_back(fd);
            sizes.push_back(c.bytes);
        }
        if (lfd_ < 0) lfd_ = uds::listen_on(group_key, me);
        if (lfd_ < 0) note("listening socket");
        std::string berr;
        if (!host_barrier(&berr)) {
            for (int f : mine) close(f);
            if (err) *err = berr;
            return FS2_ERR_COMM;
        }
        const bool have = rc == FS2_OK;
        for (int turn = 0; turn < G; ++turn) {
            if (turn == me) {
                peers[me] = base;
                // serve every other rank: its rank, then the sizes, then the descriptors
                // (an empty table when this rank has nothing to give: its peers fail).
                // Only a process of this user that names a rank of the group not yet
                // served gets anything: any other connection is closed unanswered and
                // does not take a peer's place (the socket name is visible in
                // /proc/net/unix).
                std::vector<uint8_t> served((size_t)G, 0);
                const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
                for (int k = 0; k < G - 1;) {
                    const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                                         deadline - std::chrono::steady_clock::now()).count();
                    const int c = (lfd_ >= 0 && left > 0) ? uds::accept_one(lfd_, left) : -1;
                    if (c < 0) {
                        note("accept");
                        break;
                    }
                    int32_t who = -1;
                    int nf = 0;
                    const bool got = uds::recv_msg(c, &who, sizeof who, nullptr, 0, &nf, std::max(left, 1)) ==
                                     (ssize_t)sizeof who;
                    if (!got || !uds::peer_is_us(c) || who < 0 || who >= G || who == me || served[(size_t)who]) {
                        close(c);
                        continue;
                    }
                    served[(size_t)who] = 1;
                    ++k;
                    std::vector<uint64_t> hdr(1 + sizes.size());
                    hdr[0] = have ? sizes.size() : 0;
                    for (size_t i = 0; have && i < sizes.size(); ++i) hdr[1 + i] = sizes[i];
                    if (!uds::send_msg(c, hdr.data(), sizeof(uint64_t) * (have ? hdr.size() : 1), nullptr, 0))
                        note("send sizes");
                    for (size_t i = 0; have && i < mine.size(); i += 200) {
                        const int n = (int)std::min<size_t>(200, mine.size() - i);
                        const uint32_t cnt = (uint32_t)n;
                        if (!uds::send_msg(c, &cnt, sizeof cnt, mine.data() + i, n)) note("send descriptors");
                    }
                    close(c);
                }
            } else {
                const int c = uds::connect_to(group_key, turn, ms);
                bool ok = c >= 0;
                const int32_t who = me;
                ok = ok && uds::send_msg(c, &who, sizeof who, nullptr, 0);
                std::vector<uint64_t> hdr(1 + 65536);
                int nf = 0;
                const ssize_t hn = ok ? uds::recv_msg(c, hdr.data(), sizeof(uint64_t) * hdr.size(), nullptr, 0, &nf, ms) : -1;
                ok = ok && hn >= (ssize_t)sizeof(uint64_t) && hdr[0] > 0 &&
                     hn == (ssize_t)(sizeof(uint64_t) * (1 + hdr[0]));
                std::vector<int> fds;
                std::vector<uint64_t> psz;
                if (ok) psz.assign(hdr.begin() + 1, hdr.begin() + 1 + (ptrdiff_t)hdr[0]);
                while (ok && fds.size() < psz.size()) {
                    uint32_t cnt = 0;
                    int got[256];
                    const ssize_t n = uds::recv_msg(c, &cnt, sizeof cnt, got, 256, &nf, ms);
                    ok = n == (ssize_t)sizeof cnt && (int)cnt == nf;
                    for (int i = 0; i < nf; ++i) fds.push_back(got[i]);
                }
                if (c >= 0) close(c);
                void *q = nullptr;
                if (ok && map_peer(fds, psz, device, &q) == FS2_OK) {
                    peers[turn] = q;
                } else {
                    if (!ok)
                        for (int f : fds) close(f);
                    note("importing a peer's chunks");
                }
            }
            if (!host_barrier(&berr)) {
                for (int f : mine) close(f);
                if (err) *err = berr;
                return FS2_ERR_COMM;
            }
        }
        for (int f : mine) close(f);
        return rc;
    }
};

// ------------------------------------------------------------------ RCCL ---

inline int nccl_fail(ncclResult_t r, std::string *err, const char *what) {
    if (err) *err = std::string(what) + ": " + ncclGetErrorString(r);
    return FS2_ERR_COMM;
}

// a digest of the whole group key / unique id in hex (names the ranks' sockets):
// two FNV-1a passes with different offsets
inline std::string key_hex(const uint8_t key[128]) {
    uint64_t a = 0xcbf29ce484222325ull, b = 0x84222325cbf29ce4ull;
    for (int i = 0; i < 128; ++i) {
        a = (a ^ key[i]) * 0x100000001b3ull;
        b = (b ^ key[127 - i]) * 0x100000001b3ull;
    }
    char s[40];
    std::snprintf(s, sizeof s, "%016llx%016llx", (unsigned long long)a, (unsigned long long)b);
    return std::string(s);
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
        close_listener();
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
    t->group_key = key_hex(id_bytes);
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
    int share_vm(const std::vector<VmChunk> &, void *base, int, void **peers, std::string *err) override {
        return share(base, peers, err);
    }
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
        close_listener();
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
    t->group_key = key_hex(key);
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
