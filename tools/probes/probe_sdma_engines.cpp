// Host-side duration of hsa_amd_memory_async_copy_on_engine per SDMA engine,
// first use vs later uses (H2D, pinned host -> device, 6 MB): is the post-sync
// frame-upload stall of the Tracker2D bench the lazy set-up of an SDMA engine's
// queue on its first copy? Then hipMemcpyAsync after device syncs on 4 streams.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>

static hsa_agent_t g_gpu{}, g_cpu{};
static int g_ngpu = 0;
static hsa_status_t pick(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_ngpu++ == 0) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
    hipSetDevice(0);
    hipFree(nullptr);
    hsa_init();
    hsa_iterate_agents(pick, nullptr);
    const size_t n = 6u << 20;
    void *h = nullptr, *d = nullptr;
    hipHostMalloc(&h, n, 0);
    hipMalloc(&d, n);
    hsa_signal_t sig;
    hsa_signal_create(1, 0, nullptr, &sig);
    uint32_t avail = 0, pref = 0;
    hsa_amd_memory_copy_engine_status(g_gpu, g_cpu, &avail);
    hsa_amd_memory_get_preferred_copy_engine(g_gpu, g_cpu, &pref);
    printf("{\"gpus\": %d, \"h2d_engines_available\": \"0x%x\", \"preferred\": \"0x%x\", \"rounds\": [", g_ngpu, avail, pref);
    for (int round = 0; round < 3; round++) {
        printf("%s[", round ? ", " : "");
        bool first = true;
        for (int e = 0; e < 16; e++) {
            if (!(avail & (1u << e))) continue;
            hsa_signal_store_relaxed(sig, 1);
            const double t0 = now_ms();
            const hsa_status_t st = hsa_amd_memory_async_copy_on_engine(d, g_gpu, h, g_cpu, n, 0, nullptr, sig,
                                                                        (hsa_amd_sdma_engine_id_t)(1u << e), true);
            const double t1 = now_ms();
            if (st == HSA_STATUS_SUCCESS) hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            const double t2 = now_ms();
            printf("%s{\"engine\": %d, \"status\": %d, \"call_ms\": %.3f, \"done_ms\": %.3f}", first ? "" : ", ", e, (int)st,
                   t1 - t0, t2 - t0);
            first = false;
        }
        printf("]");
    }
    printf("], \"hip\": [");
    hipStream_t s[4];
    for (auto &x : s) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    for (int round = 0; round < 6; round++) {
        hipDeviceSynchronize();
        printf("%s[", round ? ", " : "");
        for (int i = 0; i < 4; i++) {
            const double t0 = now_ms();
            hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s[i]);
            printf("%s%.3f", i ? ", " : "", now_ms() - t0);
        }
        printf("]");
    }
    printf("]}\n");
    hipDeviceSynchronize();
    return 0;
}
