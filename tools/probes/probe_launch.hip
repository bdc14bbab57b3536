// Launch-gap probe for gfx950: back-to-back launches on one stream of
//  (a) an empty kernel with an 8-B kernarg, (b) an empty kernel with a 2-KB
//  kernarg (the LK launch's size), (c) a kernel that writes 2.75 MB (a 1080p
//  pyramid), (d) the same as (b)/(c) captured into a hipGraph of 100 launches.
// Prints microseconds per launch. Build: hipcc -O2 --offload-arch=gfx950.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Big {
    int v[512];
};

__global__ void k_small(int *p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}
__global__ void k_big(Big b, int *p) {
    if (p && threadIdx.x == 1023) p[0] = b.v[blockIdx.x & 511];
}
__global__ void k_write(uint4 *p, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = make_uint4(i, i, i, i);
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                          \
        }                                                                      \
    } while (0)

template <class F>
static double timed(hipStream_t s, int n, F f) {
    for (int i = 0; i < 20; i++) f();
    (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    (void)hipStreamSynchronize(s);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint4 *buf;
    const int n16 = 2754000 / 16;
    CK(hipMalloc(&buf, (size_t)n16 * 16));
    Big b{};
    const int N = 2000;
    double a = timed(s, N, [&] { hipLaunchKernelGGL(k_small, dim3(512), dim3(256), 0, s, (int *)nullptr); });
    double bb = timed(s, N, [&] { hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s, b, (int *)nullptr); });
    double c = timed(s, N, [&] { hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, s, buf, n16); });
    // graph of 100 launches of k_big
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s, b, (int *)nullptr);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    double d = timed(s, 50, [&] { (void)hipGraphLaunch(ge, s); }) / 100.0;
    hipGraph_t g2;
    hipGraphExec_t ge2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, s, buf, n16);
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    double e = timed(s, 50, [&] { (void)hipGraphLaunch(ge2, s); }) / 100.0;
    printf("{\"empty_small_kernarg_us\": %.2f, \"empty_2KB_kernarg_us\": %.2f, \"write_2.75MB_us\": %.2f, "
           "\"graph_empty_2KB_us\": %.2f, \"graph_write_2.75MB_us\": %.2f}\n", a, bb, c, d, e);
    return 0;
}
