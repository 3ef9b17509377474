// VMM growth probe: reserve a range, map chunks one after another at its end,
// in a few variants, printing every call's status (what gm_grow in fs2_api.hip
// relies on).  hipcc --offload-arch=gfx950 -O2 scripts/vmm_probe.hip -o scripts/vmm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define P(x) do { hipError_t e_ = (x); std::printf("  %-70s %s\n", #x, hipGetErrorString(e_)); if (e_ != hipSuccess) ok = false; } while (0)

__global__ void touch(char *p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 1;
}

static bool variant(int v, size_t gran_kind) {
    bool ok = true;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    P(hipMemGetAllocationGranularity(&gran, &prop, gran_kind ? hipMemAllocationGranularityRecommended
                                                            : hipMemAllocationGranularityMinimum));
    std::printf("variant %d granularity %zu (%s)\n", v, gran, gran_kind ? "recommended" : "minimum");
    const size_t reserve = 1ull << 32;
    void *base = nullptr;
    // v2: one reservation per chunk, each at the end of the last (address hint)
    std::vector<std::pair<void *, size_t>> res;
    if (v == 2) {
        P(hipMemAddressReserve(&base, 64ull << 20, 0, nullptr, 0));
        res.push_back({base, 64ull << 20});
    } else {
        P(hipMemAddressReserve(&base, reserve, 0, nullptr, 0));
    }
    size_t mapped = 0;
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> ch;
    const size_t steps[3] = {64ull << 20, 96ull << 20, 160ull << 20};
    for (int k = 0; k < 3 && ok; ++k) {
        const size_t want = (mapped + steps[k] + gran - 1) / gran * gran, delta = want - mapped;
        if (v == 2 && k > 0) {
            void *q = nullptr;
            P(hipMemAddressReserve(&q, delta, 0, (char *)base + mapped, 0));
            std::printf("  hint %p got %p (%s)\n", (void *)((char *)base + mapped), q,
                        q == (char *)base + mapped ? "adjacent" : "elsewhere");
            if (q) res.push_back({q, delta});
            if (q != (char *)base + mapped) { ok = false; break; }
        }
        hipMemGenericAllocationHandle_t h{};
        P(hipMemCreate(&h, delta, &prop, 0));
        P(hipMemMap((char *)base + mapped, delta, 0, h, 0));
        hipMemAccessDesc ad{};
        ad.location = prop.location;
        ad.flags = hipMemAccessFlagsProtReadWrite;
        if (v != 1) P(hipMemSetAccess((char *)base + mapped, delta, &ad, 1));      // the new chunk
        else P(hipMemSetAccess(base, want, &ad, 1));                               // everything mapped
        ch.push_back({h, delta});
        mapped = want;
        hipLaunchKernelGGL(touch, dim3(1024), dim3(256), 0, 0, (char *)base, mapped);
        P(hipDeviceSynchronize());
        std::printf("  mapped %zu MiB\n", mapped >> 20);
    }
    size_t off = mapped;
    for (auto it = ch.rbegin(); it != ch.rend(); ++it) {
        off -= it->second;
        P(hipMemUnmap((char *)base + off, it->second));
        P(hipMemRelease(it->first));
    }
    if (v == 2) {
        for (auto &q : res) P(hipMemAddressFree(q.first, q.second));
    } else {
        P(hipMemAddressFree(base, reserve));
    }
    return ok;
}

int main() {
    int r = 0;
    for (int g = 0; g < 2; ++g)
        for (int v = 0; v < 3; ++v) r |= variant(v, g) ? 0 : (1 << (3 * g + v));
    std::printf("result mask %d (0: every variant worked)\n", r);
    return 0;
}
