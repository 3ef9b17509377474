// Layout microbenchmark for the association pass: read 16 B per (particle, slot)
// for S slots of N particles and reduce, in three layouts.
//   soa   : [slot][particle] float4            (lanes coalesced, 1 KiB per wave-instruction)
//   aos   : [particle][slot] float4, lane = particle, 4 consecutive slots per step
//   aosdma: same layout, teams of 4 lanes load one particle's 64 B; global_load_lds
//           stages [particle][sub] in LDS; each lane reads its 4 slots back
// hipcc --offload-arch=gfx950 -O3 ubench_layout.hip -o ubench_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_soa(const float4 *d, int64_t n, int S, float *out) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float acc = 0.f;
    for (int j = 0; j < S; j += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = d[(int64_t)(j + u) * n + i];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    out[i] = acc;
}

__global__ __launch_bounds__(256) void k_aos(const float4 *d, int64_t n, int S, float *out) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 *p = d + i * S;
    float acc = 0.f;
    for (int j = 0; j < S; j += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = p[j + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    out[i] = acc;
}

__global__ __launch_bounds__(256) void k_aosdma(const float4 *d, int64_t n, int S, float *out) {
    __shared__ __attribute__((aligned(16))) float4 st[2][4][256];   // [buf][wave][64 particles x 4 subs]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wbase = (int64_t)blockIdx.x * 256 + wv * 64;
    const int64_t i = wbase + lane;
    float acc = 0.f;
    auto issue = [&](int j, int b) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t part = wbase + 16 * r + (lane >> 2);
            const float4 *src = d + part * S + j + (lane & 3);
            __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)&st[b][wv][r * 64], 16, 0, 0);
        }
    };
    issue(0, 0);
    for (int j = 0; j < S; j += 4) {
        const int b = (j >> 2) & 1;
        if (j + 4 < S) issue(j + 4, b ^ 1);
        if (j + 4 < S) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = st[b][wv][lane * 4 + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x * v[u].y + v[u].z;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (i < n) out[i] = acc;
}

// FETCH_SIZE calibration for the access shapes of k_candidates: the descriptor
// stream ([row][particle] 8-byte entries, 512 B per wave-instruction) and page
// opens (one random 128-byte line per lane, read as 8 x 16 B), each byte
// fetched exactly once (a bijective line permutation over a table far beyond L2
// and the Infinity Cache).
__global__ __launch_bounds__(256) void k_desc8(const uint2 *d, int64_t n, int rows, unsigned *out) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    unsigned acc = 0;
    for (int r = 0; r < rows; r += 4) {
        uint2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = d[(int64_t)(r + u) * n + i];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x ^ v[u].y;
    }
    out[i] = acc;
}

__global__ __launch_bounds__(256) void k_lines128(const float4 *d, int64_t n, int per, int64_t nlines, float *out) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float acc = 0.f;
    for (int r = 0; r < per; ++r) {
        const uint64_t line = ((uint64_t)(i * per + r) * 2654435761ull) & (uint64_t)(nlines - 1);
        const float4 *p = d + line * 8;
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    out[i] = acc;
}

int main() {
    const int64_t n = 1 << 20;
    const int S = 512;
    const size_t bytes = (size_t)n * S * 16;
    float4 *d;
    float *o;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, n * 4));
    CK(hipMemset(d, 0, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char *names[3] = {"soa", "aos", "aosdma"};
    for (int rep = 0; rep < 3; ++rep)
        for (int k = 0; k < 3; ++k) {
            CK(hipEventRecord(a));
            for (int it = 0; it < 5; ++it) {
                if (k == 0) hipLaunchKernelGGL(k_soa, dim3(n / 256), dim3(256), 0, 0, d, n, S, o);
                if (k == 1) hipLaunchKernelGGL(k_aos, dim3(n / 256), dim3(256), 0, 0, d, n, S, o);
                if (k == 2) hipLaunchKernelGGL(k_aosdma, dim3(n / 256), dim3(256), 0, 0, d, n, S, o);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ms /= 5;
            printf("%-7s rep %d: %.3f ms  %.0f GB/s\n", names[k], rep, ms, bytes / (ms * 1e-3) / 1e9);
        }
    {   // calibration kernels (run once each after a warm-up)
        const int rows = 512;
        hipLaunchKernelGGL(k_desc8, dim3(n / 256), dim3(256), 0, 0, (const uint2 *)d, n, rows, (unsigned *)o);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_desc8, dim3(n / 256), dim3(256), 0, 0, (const uint2 *)d, n, rows, (unsigned *)o);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("desc8   : %.3f ms  %.0f GB/s (%zu B)\n", ms, (double)n * rows * 8 / (ms * 1e-3) / 1e9,
               (size_t)n * rows * 8);
        const int per = 8;
        const int64_t nlines = (int64_t)bytes / 128;        // 2^26 lines = 8 GiB
        hipLaunchKernelGGL(k_lines128, dim3(n / 256), dim3(256), 0, 0, d, n, per, nlines, o);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_lines128, dim3(n / 256), dim3(256), 0, 0, d, n, per, nlines, o);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("lines128: %.3f ms  %.0f GB/s (%zu B)\n", ms, (double)n * per * 128 / (ms * 1e-3) / 1e9,
               (size_t)n * per * 128);
    }
    return 0;
}
