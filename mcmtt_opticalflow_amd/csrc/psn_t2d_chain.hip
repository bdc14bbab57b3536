// Device step of the Tracker2D backward chain (include/psn_t2d_device.h):
// CPSNWhere_Tracker2D::LocalSearchKLT (psn_where/PSNWhere_Tracker2D.cpp:452-554)
// and the chain bookkeeping of Track2D_BackwardFeatureTracking (:787-811), one
// workgroup of 128 lanes per detection (<= 100 points, one point per lane).
//
// LocalSearchKLT, step by step (the host version is
// mcmtt_opticalflow_amd/host/tracker2d_flow.cpp):
//   1. d_i = nextPts_i - prevPts_i in float, widened to double; a vector
//      "moves" unless |d_i| < 0.1 (:477-490);
//   2. fewer than half moving -> the box stays, no inliers (:493-496);
//   3. sort dx and dy (:499-500); the mode of each is the first sorted value
//      with the most neighbours closer than window = 0.2 * box.w (:502-537);
//   4. inliers = moving vectors within `window` of the mode, in point order
//      (:540-546); box += mode (:549-553).
// Ordered compactions are lane-ordered prefix sums, the sort a bitonic
// network; every comparison and sum uses the host's double arithmetic.
#include <hip/hip_runtime.h>

#include "psn_lk.h"
#include "psn_t2d_device.h"

namespace psn {
namespace {

constexpr int kLanes = 128;

// inclusive prefix sum over the workgroup (2 waves)
__device__ int block_incl_scan(int v, int *tmp) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) tmp[wid] = v;
    __syncthreads();
    const int add = wid ? tmp[0] : 0;
    __syncthreads();
    return v + add;
}

__device__ void bitonic128(double *a) {
    for (int size = 2; size <= kLanes; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const int t = threadIdx.x;
            if (t < kLanes / 2) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const double x = a[lo], y = a[hi];
                if ((x > y) == up) {
                    a[lo] = y;
                    a[hi] = x;
                }
            }
            __syncthreads();
        }
}

__global__ __launch_bounds__(kLanes) void chain_step_kernel(psn_t2d_chain_dev C, int step) {
    __shared__ double sdx[kLanes], sdy[kLanes];  // moving vectors, then sorted
    __shared__ double mvx[kLanes], mvy[kLanes];  // moving vectors in point order
    __shared__ int midx[kLanes], inl[kLanes];
    __shared__ int tmp[4];
    __shared__ int red[2][kLanes];
    const int k = blockIdx.x, t = threadIdx.x;
    const int n = C.cnt[k];
    if (n <= 0) return;  // chain stopped earlier (or no features)
    const size_t pb = (size_t)k * C.cap * 2;
    const double bx = C.boxes[4 * k], by = C.boxes[4 * k + 1], bw = C.boxes[4 * k + 2], bh = C.boxes[4 * k + 3];

    // 1. moving vectors (cv::Point2f difference, then PSN_Point2D)
    double mx = 0.0, my = 0.0;
    bool moving = false;
    if (t < n) {
        const float dxf = C.nxt[pb + 2 * t] - C.cur[pb + 2 * t];
        const float dyf = C.nxt[pb + 2 * t + 1] - C.cur[pb + 2 * t + 1];
        mx = (double)dxf;
        my = (double)dyf;
        moving = !(sqrt(mx * mx + my * my) < 0.1 * 1.0);
    }
    const int pos = block_incl_scan(moving ? 1 : 0, tmp);
    __shared__ int nmov;
    if (t == kLanes - 1) nmov = pos;
    if (moving) {
        mvx[pos - 1] = mx;
        mvy[pos - 1] = my;
        midx[pos - 1] = t;
    }
    __syncthreads();
    const int M = nmov;
    int ninl = 0;
    double estx = 0.0, esty = 0.0;
    if (!((double)M < (double)n * 0.5)) {  // 2. enough moving vectors
        // 3. sorted copies, mode by neighbour counting
        sdx[t] = t < M ? mvx[t] : __builtin_inf();
        sdy[t] = t < M ? mvy[t] : __builtin_inf();
        __syncthreads();
        bitonic128(sdx);
        bitonic128(sdy);
        const double ws = bw * 0.2 * 1.0;
        int nx = 0, ny = 0;
        if (t < M) {
            const double vx = sdx[t], vy = sdy[t];
            for (int c = 0; c < M; c++) {
                if (fabs(vx - sdx[c]) < ws) nx++;
                if (fabs(vy - sdy[c]) < ws) ny++;
            }
        }
        // first maximum in sorted order: the smallest index with the largest count
        red[0][t] = t < M ? (nx << 8) | (kLanes - 1 - t) : -1;
        red[1][t] = t < M ? (ny << 8) | (kLanes - 1 - t) : -1;
        __syncthreads();
        for (int s = kLanes / 2; s > 0; s >>= 1) {
            if (t < s) {
                red[0][t] = max(red[0][t], red[0][t + s]);
                red[1][t] = max(red[1][t], red[1][t + s]);
            }
            __syncthreads();
        }
        estx = sdx[kLanes - 1 - (red[0][0] & 0xff)];
        esty = sdy[kLanes - 1 - (red[1][0] & 0xff)];
        // 4. inliers in point order
        bool in = false;
        if (t < M) {
            const double ex = mvx[t] - estx, ey = mvy[t] - esty;
            in = sqrt(ex * ex + ey * ey) < ws;
        }
        const int ip = block_incl_scan(in ? 1 : 0, tmp);
        __shared__ int ninl_s;
        if (t == kLanes - 1) ninl_s = ip;
        if (in) inl[ip - 1] = midx[t];
        __syncthreads();
        ninl = ninl_s;
    }
    if (ninl < 4) {  // :788 the chain stops here
        if (t == 0) C.cnt[k] = 0;
        return;
    }
    const int S = PSN_T2D_CHAIN_STEPS;
    if (t == 0) {
        double *ob = C.out_boxes + ((size_t)k * S + step) * 4;
        ob[0] = bx + estx;
        ob[1] = by + esty;
        ob[2] = bw;
        ob[3] = bh;
        C.cnt[k] = (C.last_step && step >= C.last_step[k]) ? 0 : ninl;  // no older frame: the chain ends
        C.nsteps[k] = step;
        if (step == 1) C.set_cnt[k * S] = ninl;
        C.set_cnt[k * S + step] = ninl;
    }
    if (t < ninl) {
        const int i = inl[t];
        const float px = C.nxt[pb + 2 * i], py = C.nxt[pb + 2 * i + 1];
        C.next_in[pb + 2 * t] = px;
        C.next_in[pb + 2 * t + 1] = py;
        float *srow = C.sets + ((size_t)k * S + step) * C.cap * 2;
        srow[2 * t] = px;
        srow[2 * t + 1] = py;
        if (step == 1) {
            float *s0 = C.sets + (size_t)k * S * C.cap * 2;
            s0[2 * t] = C.cur[pb + 2 * i];
            s0[2 * t + 1] = C.cur[pb + 2 * i + 1];
        }
    }
}

// Detections whose feature count fails the reference's minimum (:744) get no
// chain: their count becomes 0, so their workgroups exit at once.
__global__ void gate_counts_kernel(int *cnt, int n, int min_count, const int *last_step) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (cnt[i] < min_count || (last_step && last_step[i] < 1))) cnt[i] = 0;
}

// The start of a frame's device chain, one workgroup per detection: its step and
// set counters cleared; a detection with enough features (:744) gets set 0 = its
// features at t -- the tracker features the reference keeps when no chain step
// finds 4 inliers (:815-818; step 1 overwrites set 0 with its inliers when it
// does), which the next frame's forward call reads -- then the gate.
__global__ __launch_bounds__(128) void chain_begin_kernel(psn_t2d_chain_dev C, int min_count) {
    const int k = blockIdx.x, t = threadIdx.x;
    const int S = PSN_T2D_CHAIN_STEPS;
    const int n = C.cnt[k];
    const bool valid = n >= min_count;
    const int m = valid ? min(n, C.cap) : 0;
    const size_t pb = (size_t)k * C.cap * 2;
    float *s0 = C.sets + (size_t)k * S * C.cap * 2;
    for (int i = t; i < m; i += blockDim.x) {
        s0[2 * i] = C.cur[pb + 2 * i];
        s0[2 * i + 1] = C.cur[pb + 2 * i + 1];
    }
    __syncthreads();  // every lane has read cnt[k] before lane 0 gates it
    if (t == 0) {
        C.nsteps[k] = 0;
        C.set_cnt[(size_t)k * S] = m;
        for (int s = 1; s < S; s++) C.set_cnt[(size_t)k * S + s] = 0;
        if (!valid || (C.last_step && C.last_step[k] < 1)) C.cnt[k] = 0;
    }
}

// HBM <-> a mapped pinned host block: 16-B accesses over the bus, grid-strided.
__global__ __launch_bounds__(256) void copy_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src, size_t n16,
                                                     uint8_t *__restrict__ dtail, const uint8_t *__restrict__ stail,
                                                     int ntail) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

}  // namespace
}  // namespace psn

// One copy kernel between HBM and a mapped pinned host block (either side).
static int copy_mapped(void *dst, const void *src, size_t bytes, hipStream_t stream) {
    const size_t n16 = bytes / 16;
    const int ntail = (int)(bytes % 16);
    const int grid = (int)std::max<size_t>(1, std::min<size_t>((n16 + 255) / 256, 512));
    hipLaunchKernelGGL(psn::copy_kernel, dim3(grid), dim3(256), 0, stream, (uint4 *)dst, (const uint4 *)src, n16,
                       (uint8_t *)dst + n16 * 16, (const uint8_t *)src + n16 * 16, ntail);
    return hipGetLastError() == hipSuccess ? PSN_LK_OK : PSN_LK_ERR_HIP;
}

// The device address of a pinned host block (hipHostMalloc'd memory is mapped).
static void *mapped(const void *h) {
    void *p = nullptr;
    return hipHostGetDevicePointer(&p, const_cast<void *>(h), 0) == hipSuccess ? p : nullptr;
}

extern "C" int psn_t2d_upload_device(void *d_dst, const void *h_src, size_t bytes, void *stream) {
    if (bytes == 0) return PSN_LK_OK;
    if (!d_dst || !h_src || ((uintptr_t)d_dst & 15) || ((uintptr_t)h_src & 15)) return PSN_LK_ERR_ARG;
    const void *src = mapped(h_src);
    return src ? copy_mapped(d_dst, src, bytes, (hipStream_t)stream) : PSN_LK_ERR_ARG;
}

extern "C" int psn_t2d_download_device(void *h_dst, const void *d_src, size_t bytes, void *stream) {
    if (bytes == 0) return PSN_LK_OK;
    if (!h_dst || !d_src || ((uintptr_t)h_dst & 15) || ((uintptr_t)d_src & 15)) return PSN_LK_ERR_ARG;
    void *dst = mapped(h_dst);
    return dst ? copy_mapped(dst, d_src, bytes, (hipStream_t)stream) : PSN_LK_ERR_ARG;
}

extern "C" int psn_t2d_gate_counts_device(int *d_cnt, int n, int min_count, const int *d_last_step, void *stream) {
    if (n < 0 || (n > 0 && !d_cnt)) return PSN_LK_ERR_ARG;
    if (n == 0) return PSN_LK_OK;
    hipLaunchKernelGGL(psn::gate_counts_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, d_cnt, n,
                       min_count, d_last_step);
    return hipGetLastError() == hipSuccess ? PSN_LK_OK : PSN_LK_ERR_HIP;
}

extern "C" int psn_t2d_chain_begin_device(const psn_t2d_chain_dev *c, int min_count, void *stream) {
    if (!c || c->ndet < 0 || c->cap <= 0 || c->cap > 128 || (c->ndet > 0 && (!c->cnt || !c->cur || !c->sets ||
                                                                             !c->set_cnt || !c->nsteps)))
        return PSN_LK_ERR_ARG;
    if (c->ndet == 0) return PSN_LK_OK;
    hipLaunchKernelGGL(psn::chain_begin_kernel, dim3(c->ndet), dim3(128), 0, (hipStream_t)stream, *c, min_count);
    return hipGetLastError() == hipSuccess ? PSN_LK_OK : PSN_LK_ERR_HIP;
}

extern "C" int psn_t2d_chain_step_device(const psn_t2d_chain_dev *c, int step, void *stream) {
    if (!c || c->ndet < 0 || c->cap <= 0 || c->cap > 128 || step < 1 || step >= PSN_T2D_CHAIN_STEPS)
        return PSN_LK_ERR_ARG;
    if (c->ndet == 0) return PSN_LK_OK;
    hipLaunchKernelGGL(psn::chain_step_kernel, dim3(c->ndet), dim3(psn::kLanes), 0, (hipStream_t)stream, *c, step);
    return hipGetLastError() == hipSuccess ? PSN_LK_OK : PSN_LK_ERR_HIP;
}
