// vmem_probe — vector-memory pipe rates on MI355X for the access shapes k_reconcile uses
// (profiling tool, not product): coalesced streaming with dword vs dwordx4 loads per lane,
// and random dword / dwordx4 gathers. Prints one JSON line per kernel: bytes/s and VMEM
// wave-instructions/s per CU, to tell a per-instruction cost from a per-byte one.
//   hipcc --offload-arch=gfx950 -O3 -o tools/vmem_probe tools/vmem_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int BLOCK = 256;

__global__ void __launch_bounds__(BLOCK) k_stream_d1(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
    const uint64_t nt = (uint64_t)gridDim.x * BLOCK, t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t s = 0;
    for (uint64_t i = t; i < n; i += 16 * nt) {
        uint32_t v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = i + k * nt < n ? __builtin_nontemporal_load(a + i + k * nt) : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k) s ^= v[k];
    }
    if (s == 0x12345678u) out[t] = s;
}

__global__ void __launch_bounds__(BLOCK) k_stream_d4(const uint4* __restrict__ a, uint64_t n4, uint32_t* out) {
    const uint64_t nt = (uint64_t)gridDim.x * BLOCK, t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t s = 0;
    for (uint64_t i = t; i < n4; i += 4 * nt) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i + k * nt < n4 ? a[i + k * nt] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) s ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (s == 0x12345678u) out[t] = s;
}

// G gathers per thread of one dword from tab[ids[...]] (ids read coalesced)
template <int G>
__global__ void __launch_bounds__(BLOCK) k_gather_d1(const uint32_t* __restrict__ ids, uint64_t n, const uint32_t* __restrict__ tab,
                                                     uint32_t* out) {
    const uint64_t nt = (uint64_t)gridDim.x * BLOCK, t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t s = 0;
    for (uint64_t i = t; i < n; i += G * nt) {
        uint32_t id[G], v[G];
#pragma unroll
        for (int k = 0; k < G; ++k) id[k] = i + k * nt < n ? ids[i + k * nt] : 0u;
#pragma unroll
        for (int k = 0; k < G; ++k) v[k] = tab[id[k]];
#pragma unroll
        for (int k = 0; k < G; ++k) s ^= v[k];
    }
    if (s == 0x12345678u) out[t] = s;
}

template <int G>
__global__ void __launch_bounds__(BLOCK) k_gather_d4(const uint32_t* __restrict__ ids, uint64_t n, const uint4* __restrict__ tab,
                                                     uint32_t* out) {
    const uint64_t nt = (uint64_t)gridDim.x * BLOCK, t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t s = 0;
    for (uint64_t i = t; i < n; i += G * nt) {
        uint32_t id[G];
        uint4 v[G];
#pragma unroll
        for (int k = 0; k < G; ++k) id[k] = i + k * nt < n ? ids[i + k * nt] : 0u;
#pragma unroll
        for (int k = 0; k < G; ++k) v[k] = tab[id[k]];
#pragma unroll
        for (int k = 0; k < G; ++k) s ^= v[k].x ^ v[k].w;
    }
    if (s == 0x12345678u) out[t] = s;
}

int main() {
    int dev = 0, ncu = 0;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t nbytes = 1ull << 30, n = nbytes / 4;
    uint32_t *a, *out, *ids, *tab;
    CK(hipMalloc(&a, nbytes));
    CK(hipMemset(a, 1, nbytes));
    const uint32_t grid = ncu * 8;                         // 8 workgroups (32 waves) per CU
    CK(hipMalloc(&out, (size_t)grid * BLOCK * 4));
    const uint64_t ng = 64ull << 20;                        // 64M gather ids
    CK(hipMalloc(&ids, ng * 4));
    const uint32_t tab_small = 1u << 20, tab_big = 4u << 20;   // 4 MB of dwords, 64 MB of uint4
    CK(hipMalloc(&tab, (size_t)tab_big * 16));
    CK(hipMemset(tab, 3, (size_t)tab_big * 16));
    std::vector<uint32_t> h(ng);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < ng; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint32_t)x; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, double instr, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"vmem_instr_per_cu_per_us\": %.2f}\n", name, best,
                    bytes / (best * 1e-3) / 1e9, instr / ncu / (best * 1e3));
        return 0;
    };
    timeit("stream_dword", nbytes, n / 64.0, [&] { k_stream_d1<<<grid, BLOCK>>>(a, n, out); });
    timeit("stream_dwordx4", nbytes, n / 4 / 64.0, [&] { k_stream_d4<<<grid, BLOCK>>>((const uint4*)a, n / 4, out); });
    for (uint64_t i = 0; i < ng; ++i) h[i] &= tab_small - 1;
    CK(hipMemcpy(ids, h.data(), ng * 4, hipMemcpyHostToDevice));
    timeit("gather_dword_4MB", ng * 8.0, 2 * ng / 64.0, [&] { k_gather_d1<8><<<grid, BLOCK>>>(ids, ng, tab, out); });
    for (uint64_t i = 0; i < ng; ++i) h[i] = (uint32_t)(h[i] * 2654435761u) & (tab_big - 1);
    CK(hipMemcpy(ids, h.data(), ng * 4, hipMemcpyHostToDevice));
    timeit("gather_dwordx4_64MB", ng * 20.0, 2 * ng / 64.0, [&] { k_gather_d4<8><<<grid, BLOCK>>>(ids, ng, (const uint4*)tab, out); });
    for (uint64_t i = 0; i < ng; ++i) h[i] = (uint32_t)(i / 64 * 8) & (tab_small - 1);   // 64 lanes on 8 dwords: one line
    CK(hipMemcpy(ids, h.data(), ng * 4, hipMemcpyHostToDevice));
    timeit("gather_dword_same_line", ng * 8.0, 2 * ng / 64.0, [&] { k_gather_d1<8><<<grid, BLOCK>>>(ids, ng, tab, out); });
    return 0;
}
