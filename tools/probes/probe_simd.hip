// Wave -> SIMD placement probe for gfx950: 512 workgroups of 256 threads with
// the LK single-tile kernel's LDS footprint (2 workgroups per CU), every wave
// records HW_ID / XCC_ID; the host reports how co-resident workgroups' waves
// share SIMDs (whether both workgroups' wave 0 land on one SIMD).
// Build: hipcc -O2 --offload-arch=gfx950 probe_simd.hip -o probe_simd
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <string>
#include <tuple>
#include <vector>

__global__ void k(unsigned *out, int lds_touch) {
    extern __shared__ unsigned sm[];
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    if (threadIdx.x == 0) sm[lds_touch] = hw;
    const long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < 200000) __builtin_amdgcn_s_sleep(10);
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        out[(blockIdx.x * 4 + w) * 2] = hw;
        out[(blockIdx.x * 4 + w) * 2 + 1] = xcc;
    }
}

int main() {
    const int nwg = 512, lds = 58816;
    unsigned *d;
    (void)hipMalloc(&d, nwg * 4 * 2 * sizeof(unsigned));
    (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(nwg), dim3(256), lds, 0, d, 5);
    std::vector<unsigned> h(nwg * 8);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::map<std::tuple<unsigned, unsigned, unsigned>, std::vector<int>> cu;  // (xcc, se/sh, cu) -> wgs
    int same0 = 0, pairs = 0, fixed_map = 0;
    for (int g = 0; g < nwg; g++) {
        const unsigned hw = h[g * 8], xcc = h[g * 8 + 1];
        cu[{xcc, (hw >> 12) & 0xf, (hw >> 8) & 0xf}].push_back(g);
        bool f = true;
        for (int w = 0; w < 4; w++) f &= ((h[(g * 4 + w) * 2] >> 4) & 3) == (unsigned)w;
        fixed_map += f;
    }
    std::map<std::string, int> rel;  // (A's simd sequence, B's) pattern counts
    for (auto &kv : cu)
        if (kv.second.size() == 2) {
            char buf[64];
            const int a = kv.second[0], b = kv.second[1];
            snprintf(buf, sizeof buf, "%u%u%u%u-%u%u%u%u", (h[(a * 4) * 2] >> 4) & 3, (h[(a * 4 + 1) * 2] >> 4) & 3,
                     (h[(a * 4 + 2) * 2] >> 4) & 3, (h[(a * 4 + 3) * 2] >> 4) & 3, (h[(b * 4) * 2] >> 4) & 3,
                     (h[(b * 4 + 1) * 2] >> 4) & 3, (h[(b * 4 + 2) * 2] >> 4) & 3, (h[(b * 4 + 3) * 2] >> 4) & 3);
            rel[buf]++;
        }
    for (auto &kv : rel) printf("pattern %s: %d\n", kv.first.c_str(), kv.second);
    std::map<int, int> hist;
    for (auto &kv : cu) {
        hist[(int)kv.second.size()]++;
        if (kv.second.size() == 2) {
            pairs++;
            const int a = kv.second[0], b = kv.second[1];
            same0 += ((h[a * 8] >> 4) & 3) == ((h[b * 8] >> 4) & 3);
        }
    }
    printf("{\"cus\": %zu, \"wgs_per_cu_hist\": {", cu.size());
    bool first = true;
    for (auto &kv : hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"wave_i_on_simd_i\": %d, \"cu_pairs\": %d, \"pairs_wave0_same_simd\": %d}\n", fixed_map, pairs, same0);
    for (int g = 0; g < 8; g++) {
        printf("wg %d:", g);
        for (int w = 0; w < 4; w++) printf(" simd%u", (h[(g * 4 + w) * 2] >> 4) & 3);
        printf(" cu %u se %u xcc %u\n", (h[g * 8] >> 8) & 0xf, (h[g * 8] >> 13) & 7, h[g * 8 + 1]);
    }
    return 0;
}
