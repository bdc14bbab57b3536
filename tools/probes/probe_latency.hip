// Latency probe for the one-wave LK iteration design: cycles per step of
// dependent chains of the instruction kinds the iteration uses, measured by a
// single wave (s_memtime = shader clock). Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/probe_latency tools/probes/probe_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 64
#define STAMP(t) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory")

__global__ void probe(unsigned long long *out, int seed) {
    __shared__ int lds[256];
    int v = threadIdx.x + seed;
    float f = (float)v;
    unsigned long long t0, t1;
    lds[threadIdx.x] = v;
    __syncthreads();
    int k = 0;
    // 0: dependent v_add_u32
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_add_u32 %0, %0, %0" : "+v"(v));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 1: independent v_add_u32 (4 chains)
    int a = v, b = v + 1, c = v + 2, d = v + 3;
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N / 4; i++)
        asm volatile("v_add_u32 %0, %0, %0\n\tv_add_u32 %1, %1, %1\n\tv_add_u32 %2, %2, %2\n\tv_add_u32 %3, %3, %3"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    STAMP(t1);
    out[k++] = t1 - t0;
    v = a + b + c + d;
    // 2: dependent f32 add
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_add_f32 %0, %0, %0" : "+v"(f));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 3: dependent DPP row_shr:1 add
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 4: dependent DPP row_bcast:15 add
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(v));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 5: 4 interleaved scans (6 steps each) x (N/6)
    a = v; b = v + 1; c = v + 2; d = v + 3;
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N / 6; i++) {
#define SC(x, ctl, rm) asm volatile("v_add_u32_dpp %0, %0, %0 " ctl " row_mask:" rm " bank_mask:0xf" : "+v"(x))
        SC(a, "row_shr:1", "0xf"); SC(b, "row_shr:1", "0xf"); SC(c, "row_shr:1", "0xf"); SC(d, "row_shr:1", "0xf");
        SC(a, "row_shr:2", "0xf"); SC(b, "row_shr:2", "0xf"); SC(c, "row_shr:2", "0xf"); SC(d, "row_shr:2", "0xf");
        SC(a, "row_shr:4", "0xf"); SC(b, "row_shr:4", "0xf"); SC(c, "row_shr:4", "0xf"); SC(d, "row_shr:4", "0xf");
        SC(a, "row_shr:8", "0xf"); SC(b, "row_shr:8", "0xf"); SC(c, "row_shr:8", "0xf"); SC(d, "row_shr:8", "0xf");
        SC(a, "row_bcast:15", "0xa"); SC(b, "row_bcast:15", "0xa"); SC(c, "row_bcast:15", "0xa"); SC(d, "row_bcast:15", "0xa");
        SC(a, "row_bcast:31", "0xc"); SC(b, "row_bcast:31", "0xc"); SC(c, "row_bcast:31", "0xc"); SC(d, "row_bcast:31", "0xc");
    }
    STAMP(t1);
    out[k++] = t1 - t0;
    v = a ^ b ^ c ^ d;
    // 6: dependent v_readlane -> s_add -> v_add (VALU->SALU->VALU round trip)
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) {
        int s = __builtin_amdgcn_readlane(v, 63);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));
        v += s;
    }
    STAMP(t1);
    out[k++] = t1 - t0;
    // 7: dependent LDS write -> read round trip
    STAMP(t0);
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        lds[threadIdx.x] = v;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        v = lds[(threadIdx.x + 1) & 63] + 1;
    }
    STAMP(t1);
    out[k++] = t1 - t0;
    // 8: dependent LDS read (pointer chase)
    int p = threadIdx.x & 63;
    STAMP(t0);
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        asm volatile("" : "+v"(p));
        p = lds[p] & 63;
    }
    STAMP(t1);
    out[k++] = t1 - t0;
    // 9: dependent f64 mul+add
    double dd = (double)f;
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(dd));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 10: dependent v_dot2_i32_i16 accumulate
    int acc = v;
    STAMP(t0);
#pragma unroll
    for (int i = 0; i < N; i++) asm volatile("v_dot2c_i32_i16 %0, %1, %1" : "+v"(acc) : "v"(v));
    STAMP(t1);
    out[k++] = t1 - t0;
    // 11: dependent v_readfirstlane -> s_cmp -> s_cbranch (uniform branch on VALU value)
    STAMP(t0);
#pragma unroll 1
    for (int i = 0; i < N; i++) {
        int s = __builtin_amdgcn_readfirstlane(v);
        asm volatile("" : "+s"(s));
        if (s == 0x7fffffff) asm volatile("v_add_u32 %0, 3, %0" : "+v"(v));
        asm volatile("v_add_u32 %0, 1, %0" : "+v"(v));
    }
    STAMP(t1);
    out[k++] = t1 - t0;
    // 12: empty stamp pair
    STAMP(t0);
    STAMP(t1);
    out[k++] = t1 - t0;
    if (v == 0x12345 && f == 1.f && acc == 7 && dd == 2.0 && p == 99) out[63] = 1;
}

int main() {
    unsigned long long *d, h[64];
    hipMalloc(&d, sizeof(h));
    const char *names[] = {"v_add_u32 dep",        "v_add_u32 4-indep",      "v_add_f32 dep",
                           "dpp row_shr dep",      "dpp row_bcast15 dep",    "4 scans interleaved (per DPP op)",
                           "readlane->salu->valu", "lds write->read rt",     "lds read chase",
                           "v_fma_f64 dep",        "v_dot2c dep",            "readfirstlane->branch",
                           "stamp overhead"};
    const int per[] = {N, N, N, N, N, (N / 6) * 24, N, N, N, N, N, N, 1};
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, rep);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    }
    for (int i = 0; i < 13; i++) printf("%-36s %8.2f cycles/op\n", names[i], (double)h[i] / per[i]);
    return 0;
}
