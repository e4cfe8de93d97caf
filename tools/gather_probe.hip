// Random-gather ceiling of the MI355X for k_reconcile's access mix (measurement tool, not
// product code). Per "link" it issues the uniformly random gathers k_reconcile issues on
// config 2 against tables of the same sizes — one 16-B pod slot over a 16 MB table and
// `pct` 4-B parsed-percentage words over a 4.3 MB table — with nothing else in the kernel,
// so the time is the chip's rate for that request mix. Both tables fit the Infinity Cache;
// what separates them is the 4 MiB L2 of each XCD.
//
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o kube-dtn_amd/bin/gather_probe
//   gather_probe [links=10000000] [reps=10]
// Prints one JSON line per mode: links, gathers, ms (median), G gathers/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

constexpr int LPT = 4;   // links per thread, gathers of all four issued before any is used

// mode bit 0: pod slot gather (16 B); bit 1: `pct` percentage gathers; bit 2: the pod slot as
// 8 B (an 8 MB table), bit 3: as 4 B (4 MB)
__global__ void __launch_bounds__(256) k_probe(const uint4* pod, uint32_t pod_n, const uint32_t* pct,
                                               uint32_t pct_n, uint32_t links, int mode, int npct,
                                               uint32_t* sink) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    uint4 p[LPT];
    uint32_t q[LPT][9];
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
        const uint32_t i = t * LPT + k;
        const bool on = i < links;
        p[k] = make_uint4(0, 0, 0, 0);
        if (on && (mode & 1)) p[k] = pod[mix(i * 2 + 1) % pod_n];
        if (on && (mode & 4)) {
            const uint2 v = reinterpret_cast<const uint2*>(pod)[mix(i * 2 + 1) % pod_n];
            p[k] = make_uint4(v.x, v.y, 0, 0);
        }
        if (on && (mode & 8)) p[k].x = reinterpret_cast<const uint32_t*>(pod)[mix(i * 2 + 1) % pod_n];
#pragma unroll
        for (int f = 0; f < 9; ++f) {
            q[k][f] = 0;
            if (on && (mode & 2) && f < npct) q[k][f] = pct[mix(i * 16 + f + 3) % pct_n];
        }
    }
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
        acc += p[k].x ^ p[k].y ^ p[k].z ^ p[k].w;
#pragma unroll
        for (int f = 0; f < 9; ++f) acc += q[k][f];
    }
    if (acc == 0x12345678u) sink[t] = acc;   // keeps the loads; (almost) never stores
}

int main(int argc, char** argv) {
    const uint32_t links = argc > 1 ? (uint32_t)std::atoll(argv[1]) : 10000000u;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
    const uint32_t pod_n = 1000000, pct_n = 1070000;        // config 2: 1M pods, 1.07M prop strings
    uint4* pod;
    uint32_t *pct, *sink;
    CK(hipMalloc(&pod, (size_t)pod_n * 16));
    CK(hipMalloc(&pct, (size_t)pct_n * 4));
    CK(hipMalloc(&sink, (size_t)links * 4));
    CK(hipMemset(pod, 1, (size_t)pod_n * 16));
    CK(hipMemset(pct, 1, (size_t)pct_n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint32_t grid = (links + 256 * LPT - 1) / (256 * LPT);
    struct Mode { const char* name; int mode, npct; };
    const Mode modes[] = {{"pod", 1, 0}, {"pct4.5", 2, 0}, {"pod+pct4.5", 3, 0}, {"pct9", 2, 9}, {"pod+pct9", 3, 9},
                          {"pod8", 4, 0}, {"pod8+pct4.5", 6, 0}, {"pod4", 8, 0}, {"pod4+pct4.5", 10, 0}};
    for (const Mode& m : modes) {
        std::vector<float> ms;
        for (int r = 0; r < reps + 2; ++r) {
            // pct4.5: 4 or 5 of the nine fields per link (the config-2 mean of non-empty ones)
            const int np = m.npct ? m.npct : 4 + (r & 1);
            CK(hipEventRecord(a));
            k_probe<<<grid, 256>>>(pod, pod_n, pct, pct_n, links, m.mode, np, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float x;
            CK(hipEventElapsedTime(&x, a, b));
            if (r >= 2) ms.push_back(x);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        const double per_link = ((m.mode & 13) ? 1.0 : 0.0) + ((m.mode & 2) ? (m.npct ? m.npct : 4.5) : 0.0);
        const double g = per_link * links;
        std::printf("{\"mode\": \"%s\", \"links\": %u, \"gathers\": %.0f, \"ms\": %.4f, \"G_gathers_per_s\": %.2f}\n",
                    m.name, links, g, med, g / (med * 1e-3) / 1e9);
    }
    CK(hipFree(pod));
    CK(hipFree(pct));
    CK(hipFree(sink));
    return 0;
}
