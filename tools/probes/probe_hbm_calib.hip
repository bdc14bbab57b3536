// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// Tracker2D kernels use (MI355X_MICROARCH.md: FETCH_SIZE is exact only for
// calibrated patterns). Each kernel moves a KNOWN byte count through a buffer
// larger than the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read_u8(const unsigned char *__restrict__ p, size_t n, unsigned *out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
    if (acc == 0x12345678u) *out = acc;
}
__global__ void read_x4(const uint4 *__restrict__ p, size_t n, unsigned *out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i].x ^ p[i].w;
    if (acc == 0x12345678u) *out = acc;
}
__global__ void write_u8(unsigned char *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (unsigned char)i;
}
__global__ void write_x4(uint4 *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((unsigned)i, 1, 2, 3);
}

int main() {
    const size_t bytes = 1ull << 30;  // 1 GiB, 4x the Infinity Cache
    unsigned char *a, *b;
    unsigned *o;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&o, 4);
    hipMemset(a, 1, bytes);
    hipMemset(b, 2, bytes);
    for (int r = 0; r < 2; r++) {
        read_u8<<<4096, 256>>>(a, bytes, o);
        read_x4<<<4096, 256>>>((const uint4 *)b, bytes / 16, o);
        write_u8<<<4096, 256>>>(a, bytes);
        write_x4<<<4096, 256>>>((uint4 *)b, bytes / 16);
    }
    hipDeviceSynchronize();
    printf("moved %zu bytes per kernel\n", bytes);
    return 0;
}
