// ipc_probe.hip -- host-side probe of cross-process device-memory sharing on one
// GPU (VERDICT r04 "what's weak" #2: hipIpcOpenMemHandle of a peer's 17 GB page
// pool never returned).  Built as a shared library and driven by
// scripts/ipc_probe.py, which runs the exporter and the importer as separate
// processes (each loads the chosen HIP runtime first, as the product shim does),
// passes the handle (and, for VMM, the file descriptor) over a Unix socket and
// watches the importer with a time limit.
//
// mode 0: hipMalloc + hipIpcGetMemHandle / hipIpcOpenMemHandle (the page_refs
//         path of round 4);
// mode 1 / 2: hipMemCreate with a POSIX file-descriptor handle type, exported with
//         hipMemExportToShareableHandle, imported with
//         hipMemImportFromShareableHandle and mapped into a reserved range.
//
// The exporter fills the allocation with 0x5A; the importer reads back bytes at
// the start, the middle and the end.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace {
hipMemGenericAllocationHandle_t g_vh{};
void *g_base = nullptr;
size_t g_bytes = 0, g_res = 0;
int g_mode = -1;

hipMemAllocationProp vm_prop(int fd_type) {
    hipMemAllocationProp p{};
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    if (fd_type) p.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
    return p;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int check_pattern(const char *base, size_t bytes) {
    const size_t offs[3] = {0, bytes / 2, bytes - 64};
    for (size_t o : offs) {
        unsigned char b[64];
        if (hipMemcpy(b, base + o, 64, hipMemcpyDeviceToHost) != hipSuccess) return -10;
        for (unsigned char c : b)
            if (c != 0x5A) return -11;
    }
    return 0;
}
}  // namespace

extern "C" {

// Allocates `bytes`, fills it, exports it.  handle_out: 64 bytes (hipIpcMemHandle_t),
// fd_out: the POSIX fd (mode 1).  base_out / range_out: what hipMemGetAddressRange
// says of the exported pointer (is it the allocation base?).  Returns 0 or an error.
int probe_export(int mode, size_t bytes, void *handle_out, int *fd_out, void **base_out, size_t *range_out,
                 double *ms_out) {
    const auto t0 = std::chrono::steady_clock::now();
    g_mode = mode;
    if (hipSetDevice(0) != hipSuccess) return -1;
    if (mode == 0) {
        if (hipMalloc(&g_base, bytes) != hipSuccess) return -2;
        g_bytes = bytes;
        if (hipMemset(g_base, 0x5A, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -3;
        hipDeviceptr_t b = nullptr;
        size_t r = 0;
        if (hipMemGetAddressRange(&b, &r, g_base) != hipSuccess) return -4;
        *base_out = (void *)b;
        *range_out = r;
        hipIpcMemHandle_t hd;
        if (hipIpcGetMemHandle(&hd, g_base) != hipSuccess) return -5;
        std::memcpy(handle_out, &hd, sizeof hd);
    } else {
        hipMemAllocationProp p = vm_prop(1);
        size_t gran = 0;
        if (hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityRecommended) != hipSuccess) return -6;
        g_bytes = (bytes + gran - 1) / gran * gran;
        if (hipMemCreate(&g_vh, g_bytes, &p, 0) != hipSuccess) return -7;
        g_res = g_bytes;
        if (hipMemAddressReserve(&g_base, g_res, 0, nullptr, 0) != hipSuccess) return -8;
        if (hipMemMap(g_base, g_bytes, 0, g_vh, 0) != hipSuccess) return -9;
        hipMemAccessDesc ad{};
        ad.location = p.location;
        ad.flags = hipMemAccessFlagsProtReadWrite;
        if (hipMemSetAccess(g_base, g_bytes, &ad, 1) != hipSuccess) return -12;
        if (hipMemset(g_base, 0x5A, g_bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -3;
        *base_out = g_base;
        *range_out = g_bytes;
        int fd = -1;
        const hipError_t e = hipMemExportToShareableHandle(&fd, g_vh, hipMemHandleTypePosixFileDescriptor, 0);
        if (e != hipSuccess) {
            std::fprintf(stderr, "export: %s\n", hipGetErrorString(e));
            return -13;
        }
        *fd_out = fd;
    }
    *ms_out = ms_since(t0);
    return 0;
}

// Opens the peer's allocation, checks the pattern, closes it.  ms_out[0]: the open
// (or import + map + access), ms_out[1]: the check.
int probe_import(int mode, const void *handle, int fd, size_t bytes, double *ms_out) {
    if (hipSetDevice(0) != hipSuccess) return -1;
    hipFree(nullptr);                          // runtime initialised before the timed open
    auto t0 = std::chrono::steady_clock::now();
    int rc = 0;
    if (mode == 0) {
        hipIpcMemHandle_t hd;
        std::memcpy(&hd, handle, sizeof hd);
        void *p = nullptr;
        std::fprintf(stderr, "import: hipIpcOpenMemHandle ...\n");
        std::fflush(stderr);
        const hipError_t e = hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess);
        ms_out[0] = ms_since(t0);
        if (e != hipSuccess) {
            std::fprintf(stderr, "import: %s\n", hipGetErrorString(e));
            return -20;
        }
        t0 = std::chrono::steady_clock::now();
        rc = check_pattern((const char *)p, bytes);
        ms_out[1] = ms_since(t0);
        hipIpcCloseMemHandle(p);
    } else {
        hipMemGenericAllocationHandle_t vh{};
        std::fprintf(stderr, "import: hipMemImportFromShareableHandle ...\n");
        std::fflush(stderr);
        // mode 1: the fd by value (CUDA's convention); mode 2: a pointer to it
        int fdv = fd;
        hipError_t e = hipMemImportFromShareableHandle(&vh, mode == 2 ? (void *)&fdv : (void *)(intptr_t)fd,
                                                       hipMemHandleTypePosixFileDescriptor);
        if (e != hipSuccess) {
            std::fprintf(stderr, "import: %s\n", hipGetErrorString(e));
            return -21;
        }
        void *p = nullptr;
        if (hipMemAddressReserve(&p, bytes, 0, nullptr, 0) != hipSuccess) return -22;
        if (hipMemMap(p, bytes, 0, vh, 0) != hipSuccess) return -23;
        hipMemAccessDesc ad{};
        ad.location = vm_prop(0).location;
        ad.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(p, bytes, &ad, 1);
        ms_out[0] = ms_since(t0);
        if (e != hipSuccess) {
            std::fprintf(stderr, "import access: %s\n", hipGetErrorString(e));
            return -24;
        }
        t0 = std::chrono::steady_clock::now();
        rc = check_pattern((const char *)p, bytes);
        ms_out[1] = ms_since(t0);
        hipMemUnmap(p, bytes);
        hipMemAddressFree(p, bytes);
        hipMemRelease(vh);
    }
    return rc;
}

// A plain allocation the process keeps (memory pressure on the device), touched.
int probe_ballast(size_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return -1;
    return hipMemset(p, 1, bytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}

// (the "hip" exporter: a HIP call per loop iteration while the importer opens)
void probe_poke(void) { hipDeviceSynchronize(); }

void probe_release(void) {
    hipDeviceSynchronize();
    if (g_mode == 0 && g_base) hipFree(g_base);
    if (g_mode >= 1 && g_base) {
        hipMemUnmap(g_base, g_bytes);
        hipMemAddressFree(g_base, g_res);
        hipMemRelease(g_vh);
    }
    g_base = nullptr;
}

}  // extern "C"
