// ubench_lines.hip -- throughput of random 128-byte line reads on gfx950, the
// access pattern of k_candidates' page opens and k_update's record reads.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_lines scripts/ubench_lines.hip
//   scripts/ubench_lines
//
// Variants (each reads 2^23 random 128 B lines = 1 GiB, hashed line indices):
//   lane      one lane per line, 8 x 16 B loads per lane (k_candidates' form)
//   lane2     the same with two lines in flight per lane
//   coop      8 lanes per line, one 16 B load each (whole lines per instruction)
//   rec48     one lane per 48-byte record (3 x 16 B), records at 48 B stride
//   rec48c    the same records, 3 lanes per record (21 records per instruction)
//   lanloc    as lane, but each wave instruction's 64 lines lie in one 2 MiB region
// over a pool of 8 GiB and of 256 MiB (TLB reach), plus a 4-lines-per-lane
// variant of lane.  Prints GB/s of the lines' bytes.
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

__device__ __forceinline__ uint64_t hline(uint64_t k, uint64_t mask) { return (k * 2654435761ull) & mask; }

// one lane per line, `per` lines per lane, one at a time
__global__ __launch_bounds__(256) void k_lane(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    for (int r = 0; r < per; ++r) {
        const float4 *p = d + hline((uint64_t)(i * per + r), mask) * 8;
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    if (acc == 1234.5f) out[i] = acc;
}

// one lane per line, two lines in flight
__global__ __launch_bounds__(256) void k_lane2(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    for (int r = 0; r < per; r += 2) {
        const float4 *p = d + hline((uint64_t)(i * per + r), mask) * 8;
        const float4 *q = d + hline((uint64_t)(i * per + r + 1), mask) * 8;
        float4 v[8], w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = q[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x * v[u].y + v[u].z + w[u].x * w[u].y + w[u].z;
    }
    if (acc == 1234.5f) out[i] = acc;
}

// 8 lanes per line: lane group g of the wave reads line (8 * wave_line + g)
__global__ __launch_bounds__(256) void k_coop(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t grp = t >> 3;          // one group of 8 lanes per line
    const int sub = (int)(t & 7);
    float acc = 0.f;
    for (int r = 0; r < 8 * per; ++r) {  // the same lines per group of 8 as 8 lanes of k_lane
        const float4 *p = d + hline((uint64_t)(grp * 8 * per + r), mask) * 8;
        const float4 v = p[sub];
        acc += v.x * v.y + v.z;
    }
    if (acc == 1234.5f) out[t] = acc;
}

// one lane per 48-byte record (k_update's record reads)
__global__ __launch_bounds__(256) void k_rec48(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t nrec = (mask + 1) * 128 / 48;
    float acc = 0.f;
    for (int r = 0; r < per; ++r) {
        const uint64_t rec = ((uint64_t)(i * per + r) * 2654435761ull) % nrec;
        const float4 *p = reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(d) + rec * 48);
        float4 v[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) v[u] = p[u];
#pragma unroll
        for (int u = 0; u < 3; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    if (acc == 1234.5f) out[i] = acc;
}

// 3 lanes per 48-byte record, 21 records per wave instruction (lane 63 idle)
__global__ __launch_bounds__(256) void k_rec48coop(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int lane = (int)(t & 63);
    const int64_t wave = t >> 6;
    const uint64_t nrec = (mask + 1) * 128 / 48;
    float acc = 0.f;
    if (lane < 63) {
        const int k = lane / 3, c = lane % 3;
        // the wave reads the records 64 lanes x per of k_rec48 would: 21 per step
        const int64_t total = 64 * (int64_t)per;
        for (int64_t f = k; f < total; f += 21) {
            const uint64_t rec = ((uint64_t)(wave * total + f) * 2654435761ull) % nrec;
            const float4 v = reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(d) + rec * 48)[c];
            acc += v.x * v.y + v.z;
        }
    }
    if (acc == 1234.5f) out[t] = acc;
}

// one lane per line as k_lane, but the wave's 64 lines lie in one 2 MiB region
// (one translation per instruction instead of up to 64)
__global__ __launch_bounds__(256) void k_lane_local(const float4 *d, int64_t nl, int per, uint64_t mask, float *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int lane = (int)(i & 63);
    const int64_t wave = i >> 6;
    float acc = 0.f;
    for (int r = 0; r < per; ++r) {
        const uint64_t region = hline((uint64_t)(wave * per + r), mask >> 14);   // 2^14 lines = 2 MiB
        const uint64_t line = (region << 14) | (((uint64_t)lane * 2654435761ull + (uint64_t)r * 977ull) & 16383ull);
        const float4 *p = d + line * 8;
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x * v[u].y + v[u].z;
    }
    if (acc == 1234.5f) out[i] = acc;
}

int main() {
    const size_t big = (size_t)8 << 30;
    float4 *d;
    float *o;
    CK(hipMalloc(&d, big));
    CK(hipMalloc(&o, (size_t)64 << 20));
    CK(hipMemset(d, 0, big));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int64_t lines = (int64_t)1 << 23;   // 1 GiB of lines read per launch
    for (size_t pool : {big, (size_t)256 << 20}) {
        const uint64_t mask = pool / 128 - 1;
        for (int per : {4, 8}) {
            const int64_t lanes = lines / per;
            struct V {
                const char *name;
                void (*k)(const float4 *, int64_t, int, uint64_t, float *);
                int64_t threads;
                double bytes;
            } vs[] = {{"lane", k_lane, lanes, (double)lines * 128},
                      {"lane2", k_lane2, lanes, (double)lines * 128},
                      {"coop", k_coop, lanes, (double)lines * 128},
                      {"rec48", k_rec48, lanes, (double)lanes * per * 48},
                      {"rec48c", k_rec48coop, lanes, (double)lanes * per * 48},
                      {"lanloc", k_lane_local, lanes, (double)lines * 128}};
            for (const V &v : vs) {
                const unsigned grid = (unsigned)(v.threads / 256);
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipEventRecord(a));
                    hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, d, lines, per, mask, o);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                }
                CK(hipGetLastError());
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                std::printf("pool %5zu MiB  per %d  %-6s %8.3f ms  %7.0f GB/s\n", pool >> 20, per, v.name, ms,
                            v.bytes / (ms * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
