// Device-to-host copy engines on MI355X (profiling tool, not product code): a D2H copy of
// `mb` MB from device memory into page-locked host memory (hipHostMalloc), timed as
//   hip      hipMemcpyAsync on a non-blocking stream (the runtime picks blit kernels or SDMA)
//   sdma:k   hsa_amd_memory_async_copy_on_engine split over k SDMA engines (force_copy_on_sdma)
// and the same for host-to-device. One JSON line per variant.
//   hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.cpp -o /tmp/sdma_probe -lhsa-runtime64
//   /tmp/sdma_probe [mb=48] [reps=20]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        auto _e = (x);                                                             \
        if (_e != 0) {                                                             \
            std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e); \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? std::atoi(argv[1]) : 48;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const size_t n = mb << 20;
    CK(hipSetDevice(0));
    void *dev = nullptr, *host = nullptr;
    CK(hipMalloc(&dev, n));
    CK(hipHostMalloc(&host, n, hipHostMallocDefault));
    CK(hipMemset(dev, 1, n));
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int dir = 0; dir < 2; ++dir) {                  // 0: D2H, 1: H2D
        void* dst = dir ? dev : host;
        void* src = dir ? host : dev;
        const hipMemcpyKind kind = dir ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
        CK(hipMemcpyAsync(dst, src, n, kind, s));
        CK(hipStreamSynchronize(s));
        double t0 = now();
        for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dst, src, n, kind, s));
        CK(hipStreamSynchronize(s));
        double dt = (now() - t0) / reps;
        std::printf("{\"dir\": \"%s\", \"path\": \"hip\", \"MB\": %zu, \"ms\": %.4f, \"GBps\": %.2f}\n",
                    dir ? "h2d" : "d2h", mb, dt * 1e3, n / dt / 1e9);
    }
    CK(hsa_init());
    CK(hsa_iterate_agents(find_agents, nullptr));
    for (int dir = 0; dir < 2; ++dir) {
        hsa_agent_t da = dir ? g_gpu : g_cpu, sa = dir ? g_cpu : g_gpu;
        uint32_t mask = 0;
        hsa_status_t st = hsa_amd_memory_copy_engine_status(da, sa, &mask);
        uint32_t pref = 0;
        (void)hsa_amd_memory_get_preferred_copy_engine(da, sa, &pref);
        std::printf("{\"dir\": \"%s\", \"engines_status\": %d, \"mask\": \"0x%x\", \"preferred\": \"0x%x\"}\n",
                    dir ? "h2d" : "d2h", (int)st, mask, pref);
        std::vector<int> eng;
        for (int b = 0; b < 16; ++b)
            if (mask & (1u << b)) eng.push_back(b);
        char* dst = static_cast<char*>(dir ? dev : host);
        char* src = static_cast<char*>(dir ? host : dev);
        for (size_t k : {1, 2, 4}) {
            if (k > eng.size()) break;
            hsa_signal_t sig;
            CK(hsa_signal_create(1, 0, nullptr, &sig));
            double best = 1e9;
            for (int r = 0; r < reps + 1; ++r) {
                hsa_signal_store_relaxed(sig, (hsa_signal_value_t)k);
                double t0 = now();
                const size_t part = (n / k + 4095) & ~(size_t)4095;
                for (size_t i = 0; i < k; ++i) {
                    const size_t o = i * part, len = o >= n ? 0 : (o + part > n ? n - o : part);
                    CK(hsa_amd_memory_async_copy_on_engine(dst + o, da, src + o, sa, len, 0, nullptr, sig,
                                                           (hsa_amd_sdma_engine_id_t)(1u << eng[i]), true));
                }
                while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {
                }
                double dt = now() - t0;
                if (r) best = dt < best ? dt : best;
            }
            std::printf("{\"dir\": \"%s\", \"path\": \"sdma:%zu\", \"MB\": %zu, \"best_ms\": %.4f, \"GBps\": %.2f}\n",
                        dir ? "h2d" : "d2h", k, mb, best * 1e3, n / best / 1e9);
            CK(hsa_signal_destroy(sig));
        }
    }
    // every engine alone, and each engine's D2H beside a concurrent HIP host-to-device copy
    // (the pipelined resident loop: epoch k's download beside epoch k+1's delta upload)
    void *dev2 = nullptr, *host2 = nullptr;
    CK(hipMalloc(&dev2, n));
    CK(hipHostMalloc(&host2, n, hipHostMallocDefault));
    for (int dir = 0; dir < 2; ++dir) {
        hsa_agent_t da = dir ? g_gpu : g_cpu, sa = dir ? g_cpu : g_gpu;
        uint32_t mask = 0;
        (void)hsa_amd_memory_copy_engine_status(da, sa, &mask);
        char* dst = static_cast<char*>(dir ? dev : host);
        char* src = static_cast<char*>(dir ? host : dev);
        for (int b = 0; b < 16; ++b) {
            if (!(mask & (1u << b))) continue;
            for (int duplex = 0; duplex < (dir ? 1 : 2); ++duplex) {
                hsa_signal_t sig;
                CK(hsa_signal_create(1, 0, nullptr, &sig));
                std::vector<double> t;
                for (int r = 0; r < reps + 1; ++r) {
                    hsa_signal_store_relaxed(sig, 1);
                    double t0 = now();
                    if (duplex) CK(hipMemcpyAsync(dev2, host2, n, hipMemcpyHostToDevice, s));
                    CK(hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, n, 0, nullptr, sig,
                                                           (hsa_amd_sdma_engine_id_t)(1u << b), true));
                    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX,
                                                     HSA_WAIT_STATE_ACTIVE) != 0) {
                    }
                    if (duplex) CK(hipStreamSynchronize(s));
                    if (r) t.push_back(now() - t0);
                }
                std::sort(t.begin(), t.end());
                std::printf("{\"dir\": \"%s\", \"path\": \"engine 0x%x%s\", \"MB\": %zu, \"median_ms\": %.4f, "
                            "\"best_ms\": %.4f, \"GBps_median\": %.2f}\n",
                            dir ? "h2d" : "d2h", 1u << b, duplex ? " + hip h2d beside" : "", mb, t[t.size() / 2] * 1e3,
                            t[0] * 1e3, n / t[t.size() / 2] / 1e9);
                CK(hsa_signal_destroy(sig));
            }
        }
    }
    CK(hipHostFree(host2));
    CK(hipFree(dev2));
    CK(hipHostFree(host));
    CK(hipFree(dev));
    return 0;
}
