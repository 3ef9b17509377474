// ubench_gridbar.hip -- cost of a device-wide barrier inside one cooperative
// launch vs a kernel boundary, on gfx950 (8 XCDs, per-XCD L2).
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_gridbar scripts/ubench_gridbar.hip
//   scripts/ubench_gridbar [K]
//
// Prints, per variant, microseconds per barrier (or per kernel) averaged over K:
//   empty_kernels   K empty 1024-thread kernels of `grid` workgroups back to back
//   atomic_barrier  one cooperative kernel, K barriers (agent-scope atomic counter,
//                   release on arrival, relaxed polling, acquire after)
//   atomic_barrier_data  the same with every workgroup storing 4 KB before each
//                   barrier and reading a neighbour's 4 KB after it
//   cg_grid_sync    cooperative_groups::this_grid().sync()
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(1024) void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

__device__ __forceinline__ bool gbar(unsigned *cnt, unsigned target, int *err) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s at 100 MHz
                *err = 1;
                ok = false;
                break;
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system-wide compiler + hw acquire (agent scope below)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(1024) void k_atomic_bar(unsigned *cnt, unsigned base, int K, int *err, double *data,
                                                     int with_data) {
    const unsigned G = gridDim.x;
    double acc = 0.0;
    for (int k = 0; k < K; ++k) {
        if (with_data) {
            double *mine = data + (size_t)blockIdx.x * 512;
            if (threadIdx.x < 512) mine[threadIdx.x] = (double)(k + threadIdx.x);
        }
        if (!gbar(cnt, base + (unsigned)(k + 1) * G, err)) return;
        if (with_data) {
            const double *other = data + (size_t)((blockIdx.x + 1) % G) * 512;
            if (threadIdx.x < 512) acc += other[threadIdx.x];
        }
    }
    if (with_data && acc == -1.0) err[1] = 1;
}

__global__ __launch_bounds__(1024) void k_cg_sync(int K) {
    namespace cg = cooperative_groups;
    cg::grid_group g = cg::this_grid();
    for (int k = 0; k < K; ++k) g.sync();
}

// "last workgroup done": every workgroup stores a partial, releases it (agent
// scope) and counts itself in; the last one acquires and reads every partial.
__global__ __launch_bounds__(1024) void k_lastdone(double *part, unsigned *cnt, unsigned base, double *out,
                                                   int fence) {
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        part[blockIdx.x] = (double)blockIdx.x;
        unsigned prev;
        if (fence) {
            prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = (prev - base == gridDim.x - 1);
    }
    __syncthreads();
    if (s_last) {
        double v = 0.0;
        for (unsigned k = threadIdx.x; k < gridDim.x; k += 1024) v += part[k];
        if (v == -1.0) out[0] = v;
    }
}

__global__ __launch_bounds__(256) void k_dirty(double *p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (double)i;
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 200;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int grid = prop.multiProcessorCount;
    int per = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_atomic_bar, 1024, 0));
    std::printf("device %s CUs %d coop %d blocks/CU(1024 thr) %d\n", prop.name, grid, prop.cooperativeLaunch, per);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned *cnt;
    int *err;
    double *data;
    CK(hipMalloc(&cnt, 4));
    CK(hipMalloc(&err, 8));
    CK(hipMalloc(&data, (size_t)grid * 512 * 8));
    CK(hipMemset(cnt, 0, 4));
    CK(hipMemset(err, 0, 8));
    float ms = 0;
    // empty kernels
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(1024), 0, s, nullptr);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
    }
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("empty_kernels        %8.2f us each\n", ms * 1e3 / K);
    unsigned base = 0;
    for (int wd = 0; wd < 2; ++wd) {
        for (int rep = 0; rep < 2; ++rep) {
            void *args[] = {&cnt, &base, (void *)&K, &err, &data, &wd};
            CK(hipEventRecord(e0, s));
            CK(hipLaunchCooperativeKernel((const void *)k_atomic_bar, dim3(grid), dim3(1024), args, 0, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            base += (unsigned)K * grid;
        }
        CK(hipEventElapsedTime(&ms, e0, e1));
        int herr[2];
        CK(hipMemcpy(herr, err, 8, hipMemcpyDeviceToHost));
        std::printf("%-20s %8.2f us each (err %d)\n", wd ? "atomic_barrier_data" : "atomic_barrier", ms * 1e3 / K,
                    herr[0]);
    }
    for (int rep = 0; rep < 2; ++rep) {
        int KK = K;
        void *args[] = {&KK};
        CK(hipEventRecord(e0, s));
        CK(hipLaunchCooperativeKernel((const void *)k_cg_sync, dim3(grid), dim3(1024), args, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
    }
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("cg_grid_sync         %8.2f us each\n", ms * 1e3 / K);
    // one cooperative launch of 0 barriers: the launch itself
    for (int rep = 0; rep < 2; ++rep) {
        int K0 = 0, wd = 0;
        void *args[] = {&cnt, &base, &K0, &err, &data, &wd};
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 20; ++k)
            CK(hipLaunchCooperativeKernel((const void *)k_atomic_bar, dim3(grid), dim3(1024), args, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
    }
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("coop_launch_empty    %8.2f us each\n", ms * 1e3 / 20);
    // last-done pattern over G workgroups, with / without the acq_rel counter, after
    // a kernel leaving ~256 MB of writes behind (dirty lines in the L2s)
    double *part, *out, *big;
    const size_t nbig = (size_t)32 << 20;
    CK(hipMalloc(&part, 8 * 4096 * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMalloc(&big, nbig * 8));
    unsigned lbase = 0;
    CK(hipMemset(cnt, 0, 4));
    for (int G : {977, 3907}) {
        for (int fence = 0; fence < 2; ++fence) {
            for (int dirty = 0; dirty < 2; ++dirty) {
                float tot = 0;
                for (int rep = 0; rep < 6; ++rep) {
                    if (dirty) hipLaunchKernelGGL(k_dirty, dim3(4096), dim3(256), 0, s, big, nbig);
                    CK(hipEventRecord(e0, s));
                    hipLaunchKernelGGL(k_lastdone, dim3(G), dim3(1024), 0, s, part, cnt, lbase, out, fence);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    lbase += G;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep >= 2) tot += ms;
                }
                std::printf("lastdone G=%4d fence=%d dirty=%d %8.2f us per launch\n", G, fence, dirty, tot * 1e3 / 4);
            }
        }
    }
    return 0;
}
