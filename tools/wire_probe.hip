// wire_probe — what a Link entry's string gathers cost under three string-table layouts
// (profiling tool, not product code). Shaped like config 2's wire encoding: 10M entries, each
// with 3 random key strings (a 12M-string dictionary, 5-23 bytes), 2 hot key strings and 6
// random property strings (a 1M-string dictionary, 3-10 bytes). Kernels (gathers only, the
// bytes folded into a sink; one JSON line each, best of 5):
//   tab8       {offset, length} table, then the string's bytes from the arena (one or two
//              16-B loads) — the product's k_wire_write
//   inline     key strings from a 24-B {length, 23 bytes} table, property strings from a 16-B
//              {length, 15 bytes} table (one gather per string)
//   len4       the length word of the 8-B table only — the product's k_wire_entry_sizes
//   len1       a 1-byte length table
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/wire_probe tools/wire_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int BLOCK = 256, NK = 5, NP = 6;
constexpr uint32_t D = 12u << 20, P = 1u << 20, N = 10u << 20;

struct Ent {
    const uint32_t* kid;     // [NK][N]
    const uint32_t* pid;     // [NP][N]
};

__device__ __forceinline__ uint32_t fold16(const uint8_t* a, uint32_t b, uint32_t len) {
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    const uint32_t* a32 = reinterpret_cast<const uint32_t*>(a) + (b >> 2);
    const uint32_t sh = b & 3u, nw = (sh + len + 3u) >> 2;
    const u32x4a A = *reinterpret_cast<const u32x4a*>(a32);
    u32x4a B = {0u, 0u, 0u, 0u};
    if (nw > 4u) B = *reinterpret_cast<const u32x4a*>(a32 + 4);
    return A.x ^ A.y ^ A.z ^ A.w ^ B.x ^ B.y ^ B.z ^ B.w;
}

__global__ void __launch_bounds__(BLOCK) k_tab8(Ent e, const uint2* kt, const uint8_t* ka, const uint2* pt,
                                                 const uint8_t* pa, uint32_t* sink) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= N) return;
    uint32_t id[NK + NP];
#pragma unroll
    for (int k = 0; k < NK; ++k) id[k] = e.kid[(size_t)k * N + i];
#pragma unroll
    for (int k = 0; k < NP; ++k) id[NK + k] = e.pid[(size_t)k * N + i];
    uint2 r[NK + NP];
#pragma unroll
    for (int k = 0; k < NK + NP; ++k) r[k] = k < NK ? kt[id[k]] : pt[id[k]];
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < NK + NP; ++k) x ^= fold16(k < NK ? ka : pa, r[k].x, r[k].y);
    if (x == 0x9E3779B9u) sink[0] = x;
}

__global__ void __launch_bounds__(BLOCK) k_inline(Ent e, const uint2* kt, const uint8_t* ka, const uint32_t* k24,
                                                   const uint4* p16, uint32_t* sink) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= N) return;
    uint32_t id[NK + NP];
#pragma unroll
    for (int k = 0; k < NK; ++k) id[k] = e.kid[(size_t)k * N + i];
#pragma unroll
    for (int k = 0; k < NP; ++k) id[NK + k] = e.pid[(size_t)k * N + i];
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const uint32_t* q = k24 + (size_t)id[k] * 6;
        const uint4 a = *reinterpret_cast<const uint4*>(q);
        const uint2 b = *reinterpret_cast<const uint2*>(q + 4);
        x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y;
        if ((a.x & 0xFFu) == 0xFFu) {                       // long: offset in word 1
            const uint2 r = kt[id[k]];
            x ^= fold16(ka, r.x, r.y);
        }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint4 a = p16[id[NK + k]];
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (x == 0x9E3779B9u) sink[0] = x;
}

template <bool BYTE>
__global__ void __launch_bounds__(BLOCK) k_len(Ent e, const uint2* kt, const uint2* pt, const uint8_t* kl,
                                                const uint8_t* pl, uint32_t* out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= N) return;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const uint32_t id = e.kid[(size_t)k * N + i];
        s += BYTE ? kl[id] : reinterpret_cast<const uint32_t*>(kt)[2 * (size_t)id + 1];
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint32_t id = e.pid[(size_t)k * N + i];
        s += BYTE ? pl[id] : reinterpret_cast<const uint32_t*>(pt)[2 * (size_t)id + 1];
    }
    out[i] = s;
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}

int main() {
    // dictionaries: key strings 5-23 bytes, property strings 3-10 bytes
    std::vector<uint2> kt(D), pt(P);
    std::vector<uint32_t> k24((size_t)D * 6);
    std::vector<uint4> p16(P);
    std::vector<uint8_t> kl(D), pl(P);
    std::vector<uint8_t> ka, pa;
    ka.reserve((size_t)D * 15);
    for (uint32_t s = 0; s < D; ++s) {
        const uint32_t len = 5 + rnd() % 19;
        kt[s] = make_uint2((uint32_t)ka.size(), len);
        kl[s] = (uint8_t)len;
        uint8_t* w = reinterpret_cast<uint8_t*>(&k24[(size_t)s * 6]);
        w[0] = (uint8_t)len;
        for (uint32_t c = 0; c < len; ++c) {
            const uint8_t b = (uint8_t)('a' + rnd() % 26);
            ka.push_back(b);
            w[1 + c] = b;
        }
    }
    for (int k = 0; k < 64; ++k) ka.push_back(0);
    for (uint32_t s = 0; s < P; ++s) {
        const uint32_t len = 3 + rnd() % 8;
        pt[s] = make_uint2((uint32_t)pa.size(), len);
        pl[s] = (uint8_t)len;
        uint8_t* w = reinterpret_cast<uint8_t*>(&p16[s]);
        w[0] = (uint8_t)len;
        for (uint32_t c = 0; c < len; ++c) {
            const uint8_t b = (uint8_t)('0' + rnd() % 10);
            pa.push_back(b);
            w[1 + c] = b;
        }
    }
    for (int k = 0; k < 64; ++k) pa.push_back(0);
    std::vector<uint32_t> kid((size_t)NK * N), pid((size_t)NP * N);
    for (uint32_t i = 0; i < N; ++i) {
        kid[i] = rnd() % D;                                   // peer_pod
        kid[(size_t)N + i] = rnd() % D;                       // local_ip
        kid[2 * (size_t)N + i] = rnd() % D;                   // peer_ip
        kid[3 * (size_t)N + i] = rnd() % 16;                  // local_intf (hot)
        kid[4 * (size_t)N + i] = rnd() % 16;                  // peer_intf (hot)
        for (int k = 0; k < NP; ++k) pid[(size_t)k * N + i] = rnd() % P;
    }
    CK(hipSetDevice(0));
    auto up = [&](const void* h, size_t n, void** d) -> int {
        CK(hipMalloc(d, n));
        CK(hipMemcpy(*d, h, n, hipMemcpyHostToDevice));
        return 0;
    };
    void *dkt, *dpt, *dk24, *dp16, *dkl, *dpl, *dka, *dpa, *dkid, *dpid, *dout;
    if (up(kt.data(), kt.size() * 8, &dkt) || up(pt.data(), pt.size() * 8, &dpt) ||
        up(k24.data(), k24.size() * 4, &dk24) || up(p16.data(), p16.size() * 16, &dp16) ||
        up(kl.data(), kl.size(), &dkl) || up(pl.data(), pl.size(), &dpl) || up(ka.data(), ka.size(), &dka) ||
        up(pa.data(), pa.size(), &dpa) || up(kid.data(), kid.size() * 4, &dkid) || up(pid.data(), pid.size() * 4, &dpid))
        return 1;
    CK(hipMalloc(&dout, (size_t)N * 4));
    Ent e{(const uint32_t*)dkid, (const uint32_t*)dpid};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t grid = (N + BLOCK - 1) / BLOCK;
    auto run = [&](const char* name, auto launch) -> int {
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
        std::printf("{\"kernel\": \"%s\", \"entries\": %u, \"ms\": %.4f}\n", name, N, best);
        return 0;
    };
    if (run("tab8", [&] { k_tab8<<<grid, BLOCK>>>(e, (const uint2*)dkt, (const uint8_t*)dka, (const uint2*)dpt,
                                                  (const uint8_t*)dpa, (uint32_t*)dout); }))
        return 1;
    if (run("inline", [&] { k_inline<<<grid, BLOCK>>>(e, (const uint2*)dkt, (const uint8_t*)dka, (const uint32_t*)dk24,
                                                      (const uint4*)dp16, (uint32_t*)dout); }))
        return 1;
    if (run("len4", [&] { k_len<false><<<grid, BLOCK>>>(e, (const uint2*)dkt, (const uint2*)dpt, (const uint8_t*)dkl,
                                                         (const uint8_t*)dpl, (uint32_t*)dout); }))
        return 1;
    if (run("len1", [&] { k_len<true><<<grid, BLOCK>>>(e, (const uint2*)dkt, (const uint2*)dpt, (const uint8_t*)dkl,
                                                        (const uint8_t*)dpl, (uint32_t*)dout); }))
        return 1;
    return 0;
}
