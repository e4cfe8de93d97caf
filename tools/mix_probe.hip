// mix_probe — does the per-CU vector-memory path overlap k_reconcile's streaming pass with its
// random gathers, or add them up? (profiling tool, not product code)
//
// One synthetic "record" per thread-iteration, shaped like a config-2 AddLinks entry of
// k_reconcile (per-unit bytes): 19 coalesced dword loads of columns (AoSoA tile
// rows, non-temporal) and 23 coalesced dword stores of outputs (idx + resolved + qdisc), plus
// the random lanes the lookups make — one 16-B slot from a 16 MB table (the peer's pod slot,
// an Infinity-Cache hit), 3 dwords from a 4 MB table (cold parsed percentages, the peer-IP
// predicate word) and 3 dwords from a 64 KB table (hot parsed values). Kernels:
//   stream   the loads and stores only
//   gather   the random lanes only (ids from a hash of the record index)
//   mix      both, the ids taken from the loaded columns (the dependency k_reconcile has;
//            the columns hold random words)
//   mix_ind  both, ids from the hash (no load → gather dependency)
// 10M records (config 2), 256-thread workgroups held to 4 per CU by 28 KB of LDS like
// k_reconcile. One JSON line per kernel (best of 5).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mix_probe tools/mix_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int BLOCK = 256, NLOAD = 19, NSTORE = 23;
constexpr uint32_t BIG = 1u << 20, MID = 1u << 20, HOT = 1u << 14;   // 16 MB of uint4, 4 MB / 64 KB of dwords

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}

template <bool STREAM, bool GATHER, bool DEP>
__global__ void __launch_bounds__(BLOCK) k_mix(const uint32_t* __restrict__ cols, uint32_t* __restrict__ outc, uint32_t n,
                                               const uint4* __restrict__ big, const uint32_t* __restrict__ mid,
                                               const uint32_t* __restrict__ hot, uint32_t* sink) {
    __shared__ uint32_t lds[7040];                                // 28 KB: 4 workgroups per CU
    if (threadIdx.x == 0) lds[0] = 0;
    const uint32_t nt = gridDim.x * BLOCK;
    uint32_t acc = 0;
    for (uint32_t r = blockIdx.x * BLOCK + threadIdx.x; r < n; r += nt) {
        const uint32_t tile = r >> 6, lane = r & 63u;
        const uint32_t* row = cols + (size_t)tile * (NLOAD * 64) + lane;
        uint32_t c[NLOAD];
        if constexpr (STREAM) {
#pragma unroll
            for (int k = 0; k < NLOAD; ++k) c[k] = __builtin_nontemporal_load(row + k * 64);
        } else {
#pragma unroll
            for (int k = 0; k < NLOAD; ++k) c[k] = r * (k + 1);
        }
        uint32_t v = 0;
        if constexpr (GATHER) {
            const uint32_t h0 = DEP ? c[2] : mix32(r), h1 = DEP ? c[5] : mix32(r + 1), h2 = DEP ? c[8] : mix32(r + 2);
            const uint32_t h3 = DEP ? c[11] : mix32(r + 3), h4 = DEP ? c[14] : mix32(r + 4), h5 = DEP ? c[17] : mix32(r + 5);
            const uint32_t h6 = DEP ? c[3] : mix32(r + 6);
            const uint4 s = big[mix32(h0) & (BIG - 1)];
            v = s.x ^ s.w ^ mid[mix32(h1) & (MID - 1)] ^ mid[mix32(h2) & (MID - 1)] ^ mid[mix32(h3) & (MID - 1)] ^
                hot[mix32(h4) & (HOT - 1)] ^ hot[mix32(h5) & (HOT - 1)] ^ hot[mix32(h6) & (HOT - 1)];
        }
        uint32_t x = v;
#pragma unroll
        for (int k = 0; k < NLOAD; ++k) x += c[k];
        if constexpr (STREAM) {
            uint32_t* o = outc + (size_t)tile * (NSTORE * 64) + lane;
#pragma unroll
            for (int k = 0; k < NSTORE; ++k) __builtin_nontemporal_store(x + k, o + k * 64);
        } else {
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc + lds[0];
}

// random column contents (a memset would make every dependent id the same address)
__global__ void k_fill(uint32_t* a, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = mix32((uint32_t)i * 0x9E3779B9u + 0x7F4A7C15u);
}

int main() {
    int ncu = 0;
    CK(hipSetDevice(0));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t n = 10u << 20;                                      // ~10M records (config 2)
    uint32_t *cols, *outc, *mid, *hot, *sink;
    uint4* big;
    CK(hipMalloc(&cols, (size_t)n * NLOAD * 4));
    CK(hipMalloc(&outc, (size_t)n * NSTORE * 4));
    CK(hipMalloc(&big, (size_t)BIG * 16));
    CK(hipMalloc(&mid, (size_t)MID * 4));
    CK(hipMalloc(&hot, (size_t)HOT * 4));
    CK(hipMalloc(&sink, 64));
    k_fill<<<1024, 256>>>(cols, (uint64_t)n * NLOAD);
    CK(hipMemset(big, 1, (size_t)BIG * 16));
    CK(hipMemset(mid, 2, (size_t)MID * 4));
    CK(hipMemset(hot, 3, (size_t)HOT * 4));
    const uint32_t grid = ncu * 4 * 8;                                 // 8 rounds of the resident slots
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern) -> int {
        kern<<<grid, BLOCK>>>(cols, outc, n, big, mid, hot, sink);
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            kern<<<grid, BLOCK>>>(cols, outc, n, big, mid, hot, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        std::printf("{\"kernel\": \"%s\", \"records\": %u, \"ms\": %.4f, \"stream_TBps\": %.2f}\n", name, n, best,
                    (double)n * (NLOAD + NSTORE) * 4 / (best * 1e-3) / 1e12);
        return 0;
    };
    if (run("stream", k_mix<true, false, false>)) return 1;
    if (run("gather", k_mix<false, true, false>)) return 1;
    if (run("mix", k_mix<true, true, true>)) return 1;
    if (run("mix_ind", k_mix<true, true, false>)) return 1;
    return 0;
}
