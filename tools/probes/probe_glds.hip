// Probe: LDS layout written by global_load_lds_ubyte / _ushort / _dword on gfx950,
// and the latency of a dependent v_add_f32 chain (one wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int SZ>
__global__ void k_glds(const unsigned char *__restrict__ g, unsigned char *out) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xEE;
    __syncthreads();
    const unsigned char *src = g + threadIdx.x * SZ;
    auto gp = (const void __attribute__((address_space(1))) *)src;
    auto lp = (void __attribute__((address_space(3))) *)(lds);
    if constexpr (SZ == 1) __builtin_amdgcn_global_load_lds(gp, lp, 1, 0, 0);
    if constexpr (SZ == 2) __builtin_amdgcn_global_load_lds(gp, lp, 2, 0, 0);
    if constexpr (SZ == 4) __builtin_amdgcn_global_load_lds(gp, lp, 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}

__global__ void k_chain(const float *in, float *out, long long *cyc, int n) {
    float acc = 0.f;
    const float a = in[threadIdx.x];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
        acc = acc + a;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    std::vector<unsigned char> h(4096);
    for (int i = 0; i < 4096; i++) h[i] = (unsigned char)(i * 7 + 3);
    unsigned char *d, *o;
    hipMalloc(&d, 4096);
    hipMalloc(&o, 512);
    hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
    std::vector<unsigned char> r(512);
    auto show = [&](const char *name) {
        hipMemcpy(r.data(), o, 512, hipMemcpyDeviceToHost);
        printf("%s:", name);
        for (int i = 0; i < 24; i++) printf(" %02x", r[i]);
        printf("  | expect bytes of g:");
        for (int i = 0; i < 8; i++) printf(" %02x", h[i]);
        printf("\n");
    };
    k_glds<1><<<1, 64>>>(d, o);
    show("ubyte");
    k_glds<2><<<1, 64>>>(d, o);
    show("ushort");
    k_glds<4><<<1, 64>>>(d, o);
    show("dword");
    float *fi, *fo;
    long long *cy;
    hipMalloc(&fi, 256 * 4);
    hipMalloc(&fo, 256 * 4);
    hipMalloc(&cy, 8);
    hipMemset(fi, 0, 256 * 4);
    for (int n : {100, 1000}) {
        k_chain<<<1, 64>>>(fi, fo, cy, n);
        long long c;
        hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
        printf("dependent v_add_f32 chain: %.2f cycles/add (n=%d)\n", (double)c / (8.0 * n), n);
    }
    return 0;
}
