// GridFAST feature extraction for the backward chain of CPSNWhere_Tracker2D
// (psn_where/PSNWhere_Tracker2D.cpp:142, :734-757): FAST-9/16 corners
// (threshold 10, non-max suppression) of OpenCV 2.4.6's
// GridAdaptedFeatureDetector over a 4 x 4 grid with at most 1000/16 keypoints
// per cell, masked by the detection box, then the shuffle + cap to 100 points.
//
// The reference runs a full-frame FAST per detection and masks afterwards.
// Only positions inside the box can survive the mask, and a cell's FAST only
// reads its own sub-image, so here each (detection, cell) workgroup evaluates
// exactly the box part of the cell's detection region (3 px inside the cell):
// scores on that region plus a 1-px ring (clipped to the cell's detection
// region; outside it a score is 0, as in FAST_t's zeroed score rows), strict
// 8-neighbour non-max, then keepStrongest by a 256-bin score histogram. The
// work per detection scales with its box, not with the frame.
//
// Definitions of the reference's unspecified choices (same in the oracle,
// oracle/gridfast_oracle.c): keepStrongest ties at the cut go to the earlier
// keypoint in row-major order, kept keypoints stay in row-major order, cells
// in grid order; random_shuffle = order by a seeded 32-bit hash per candidate.
//
// Memory: byte tiles of the frame through LDS (HBM-bound integer work, no MFMA).
#include <hip/hip_runtime.h>

#include "psn_gridfast.h"

namespace psn {

namespace {

constexpr int kGfThreads = 256;

// fast.cpp makeOffsets(16): circle (dx, dy)
__constant__ signed char kCircDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ signed char kCircDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

// a run of >= 9 set bits in the circular 16-bit mask m
__device__ __forceinline__ bool arc9(unsigned m) {
    unsigned d = m | (m << 16);
    unsigned a = d & (d >> 1);  // runs of 2
    a &= a >> 2;                // 4
    a &= a >> 4;                // 8
    a &= d >> 8;                // 9
    return a != 0;
}

// FAST-9/16 at tile position (tx, ty) (centre pixel): 0 = no corner, else
// response + 1. cornerScore<16> in closed form: max(t, max over 9-arcs of
// min(v - x), max over 9-arcs of min(x - v)) - 1 (fast_score.cpp).
__device__ int fast_resp1(const uint8_t *pix, int pc, int ty, int tx, int t, int nonmax) {
    const int v = pix[ty * pc + tx];
    int e[16];
    unsigned br = 0, dk = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        e[k] = (int)pix[(ty + kCircDy[k]) * pc + tx + kCircDx[k]] - v;
        br |= (unsigned)(e[k] > t) << k;
        dk |= (unsigned)(e[k] < -t) << k;
    }
    if (!arc9(br) && !arc9(dk)) return 0;
    if (!nonmax) return 1;
    // sliding minima / maxima over the 9-arcs starting at each k
    int best = t;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int mn = e[k], mx = e[k];
#pragma unroll
        for (int m = 1; m < 9; m++) {
            const int x = e[(k + m) & 15];
            mn = min(mn, x);
            mx = max(mx, x);
        }
        best = max(best, max(mn, -mx));
    }
    return best;  // response best - 1, stored + 1
}

// block-wide exclusive scan of one int per thread; returns the total in *tot
__device__ int block_scan_excl(int v, int *scratch, int *tot) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    int base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kGfThreads / 64; w++) {
        const int s = scratch[w];
        if (w < wid) base += s;
        all += s;
    }
    __syncthreads();
    *tot = all;
    return base + x - v;
}

}  // namespace

// q / d for 0 <= q < 2^24 by a float reciprocal and one correction step
__device__ __forceinline__ int fdiv(int q, int d, float inv) {
    int y = (int)((float)q * inv);
    const int r = q - y * d;
    if (r >= d) y++;
    else if (r < 0) y--;
    return y;
}

// One workgroup per (cell, roi): the cell's keypoints inside the roi after
// keepStrongest, in row-major order. Dynamic LDS (host-sized for the widest
// region of the launch, A.rw_max, and the strip height A.strip):
//   pix   (strip + 8) x pc  bytes   frame rows of the strip + FAST radius + 1
//   sco   (strip + 2) x sc  bytes   responses + 1 (0 = no corner) with a 1-px ring
//   ks    strip x rw_max    bytes   keypoint responses + 1 of the strip
//   list  A.list_cap u32            keypoints of the region in row-major order
//                                   (x | y << 12 | response << 24; single pass)
// Single pass when the region's keypoints surely fit the list (non-max: no
// two keypoints are 8-neighbours, so at most ceil(W/2) * ceil(H/2)): FAST,
// non-max and the score histogram while collecting, then keepStrongest over
// the list. Otherwise two passes over the frame (histogram, then selection).
__global__ __launch_bounds__(kGfThreads) void gridfast_cell_kernel(GridFastArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
    __shared__ int hist[256];
    __shared__ int scratch[8];
    __shared__ int sel[2];  // threshold response (-1: keep all), ties to keep

    const int SH = A.strip, PC = (A.rw_max + 8 + 3) & ~3, SC = A.rw_max + 2;
    uint8_t *pix = gsm;
    uint8_t *sco = pix + (SH + 8) * PC;
    uint8_t *ks = sco + (((SH + 2) * SC + 15) & ~15);
    uint32_t *list = (uint32_t *)(ks + ((SH * A.rw_max + 15) & ~15));

    const int cell = blockIdx.x, r = blockIdx.y;
    const int ci = cell / A.grid_cols, cj = cell - ci * A.grid_cols;
    const int ncell = A.grid_rows * A.grid_cols;
    const int tid = threadIdx.x;
    // cell = sub-image rows [cy0, cy1), cols [cx0, cx1); FAST detects 3 px inside
    const int cy0 = (ci * A.h) / A.grid_rows, cy1 = ((ci + 1) * A.h) / A.grid_rows;
    const int cx0 = (cj * A.w) / A.grid_cols, cx1 = ((cj + 1) * A.w) / A.grid_cols;
    const int dy0 = cy0 + 3, dy1 = cy1 - 3, dx0 = cx0 + 3, dx1 = cx1 - 3;
    const int4 roi = A.rois[r];
    const uint8_t *img = A.roi_img[r];
    const int ax0 = max(dx0, roi.x), ax1 = min(dx1, roi.x + roi.z);
    const int ay0 = max(dy0, roi.y), ay1 = min(dy1, roi.y + roi.w);
    int *cnt = A.cell_cnt + (size_t)r * ncell + cell;
    uint32_t *out = A.cell_kp + ((size_t)r * ncell + cell) * A.per_cell;
    if (ax0 >= ax1 || ay0 >= ay1 || roi.z <= 0 || roi.w <= 0) {
        if (tid == 0) *cnt = 0;
        return;
    }
    const int RW = ax1 - ax0, RH = ay1 - ay0;
    const int SW = RW + 2, PW = RW + 8;
    const float invSW = 1.f / (float)SW, invRW = 1.f / (float)RW;
    const bool single = A.nonmax && ((RW + 1) / 2) * ((RH + 1) / 2) <= A.list_cap;

    for (int i = tid; i < 256; i += kGfThreads) hist[i] = 0;
    int tie_run = 0, kept_run = 0, nlist = 0;

    // ordered keep-selection over n row-major items (thread runs): item i has
    // response resp(i) (< 0: none); kept items go to `out` in order
    auto select_run = [&](int n, int T, int need, auto resp, auto coord) {
        const int run = (n + kGfThreads - 1) / kGfThreads;
        const int p0 = min(n, tid * run), p1 = min(n, p0 + run);
        int ties = 0;
        if (T >= 0)
            for (int p = p0; p < p1; p++) ties += resp(p) == T;
        int tie_tot;
        const int tie_base = tie_run + block_scan_excl(ties, scratch, &tie_tot);
        int keep = 0;
        for (int p = p0, tb = tie_base; p < p1; p++) {
            const int s = resp(p);
            if (s < 0) continue;
            if (s > T) keep++;
            else if (s == T) keep += tb++ < need;
        }
        int kept_tot;
        int pos = kept_run + block_scan_excl(keep, scratch, &kept_tot);
        for (int p = p0, tb = tie_base; p < p1; p++) {
            const int s = resp(p);
            if (s < 0) continue;
            bool k = s > T;
            if (s == T) k = tb++ < need;
            if (k) out[pos++] = coord(p);
        }
        tie_run += tie_tot;
        kept_run += kept_tot;
    };

    const int npass = single ? 1 : 2;
    for (int pass = 0; pass < npass; pass++) {
        if (pass == 1) {
            if (tid == 0) {
                int total = 0;
                for (int s = 0; s < 256; s++) total += hist[s];
                int T = -1, need = 0;
                if (total > A.per_cell) {
                    int cum = 0;
                    for (int s = 255; s >= 0; s--) {
                        if (cum + hist[s] >= A.per_cell) {
                            T = s;
                            need = A.per_cell - cum;
                            break;
                        }
                        cum += hist[s];
                    }
                }
                sel[0] = T;
                sel[1] = need;
            }
            __syncthreads();
        }
        const int T = pass ? sel[0] : 0, need = pass ? sel[1] : 0;
        for (int y0 = ay0; y0 < ay1; y0 += SH) {
            const int sh = min(SH, ay1 - y0);
            // pixels rows [y0 - 4, y0 + sh + 4), cols [ax0 - 4, ax1 + 4), clamped
            // into the image (clamped values are never read by a computed score)
            __syncthreads();  // previous strip's readers are done
            {  // every thread issues up to 16 loads before its first LDS store
                const int n = (sh + 8) * PW;
                const float invPW = 1.f / (float)PW;
                for (int b0 = 0; b0 < n; b0 += 16 * kGfThreads) {
                    uint8_t v[16];
                    int dst[16];
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        const int q = b0 + k * kGfThreads + tid;
                        dst[k] = -1;
                        if (q < n) {
                            const int yy = fdiv(q, PW, invPW), xx = q - yy * PW;
                            v[k] = img[(size_t)clampi(y0 - 4 + yy, 0, A.h - 1) * A.pitch + clampi(ax0 - 4 + xx, 0, A.w - 1)];
                            dst[k] = yy * PC + xx;
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 16; k++)
                        if (dst[k] >= 0) pix[dst[k]] = v[k];
                }
            }
            __syncthreads();
            // responses at rows [y0 - 1, y0 + sh + 1), cols [ax0 - 1, ax1 + 1)
            for (int q = tid; q < (sh + 2) * SW; q += kGfThreads) {
                const int yy = fdiv(q, SW, invSW), xx = q - yy * SW;
                const int gy = y0 - 1 + yy, gx = ax0 - 1 + xx;
                int v = 0;
                if (gy >= dy0 && gy < dy1 && gx >= dx0 && gx < dx1) v = fast_resp1(pix, PC, yy + 3, xx + 3, A.threshold, A.nonmax);
                sco[yy * SC + xx] = (uint8_t)v;
            }
            __syncthreads();
            // keypoints of the strip (strict 8-neighbour maximum of the response)
            for (int q = tid; q < sh * RW; q += kGfThreads) {
                const int yy = fdiv(q, RW, invRW), xx = q - yy * RW;
                const uint8_t *c = sco + (yy + 1) * SC + xx + 1;
                const int v = c[0];
                bool kp = v != 0;
                if (kp && A.nonmax) {
                    // FAST_t compares responses, a non-corner counting as 0
                    const int nb = max(max(max(c[-1], c[1]), max(c[-SC - 1], c[-SC])),
                                       max(max(c[-SC + 1], c[SC - 1]), max(c[SC], c[SC + 1])));
                    kp = v - 1 > max(nb - 1, 0);
                }
                ks[q] = kp ? (uint8_t)v : 0;
                if (kp && pass == 0) atomicAdd(&hist[v - 1], 1);
            }
            __syncthreads();
            if (single) {  // append the strip's keypoints to the list, in order
                const int n = sh * RW, run = (n + kGfThreads - 1) / kGfThreads;
                const int p0 = min(n, tid * run), p1 = min(n, p0 + run);
                int m = 0;
                for (int p = p0; p < p1; p++) m += ks[p] != 0;
                int tot;
                int pos = nlist + block_scan_excl(m, scratch, &tot);
                for (int p = p0; p < p1; p++) {
                    const int v = ks[p];
                    if (!v) continue;
                    const int yy = fdiv(p, RW, invRW), xx = p - yy * RW;
                    list[pos++] = (uint32_t)(ax0 + xx) | ((uint32_t)(y0 + yy) << 12) | ((uint32_t)(v - 1) << 24);
                }
                nlist += tot;
                continue;
            }
            if (pass == 0) continue;
            select_run(sh * RW, T, need, [&](int p) { return (int)ks[p] - 1; },
                       [&](int p) {
                           const int yy = fdiv(p, RW, invRW), xx = p - yy * RW;
                           return (uint32_t)(ax0 + xx) | ((uint32_t)(y0 + yy) << 16);
                       });
        }
        __syncthreads();
    }
    if (single) {  // keepStrongest over the collected list
        if (tid == 0) {
            int T = -1, need = 0;
            if (nlist > A.per_cell) {
                int cum = 0;
                for (int s = 255; s >= 0; s--) {
                    if (cum + hist[s] >= A.per_cell) {
                        T = s;
                        need = A.per_cell - cum;
                        break;
                    }
                    cum += hist[s];
                }
            }
            sel[0] = T;
            sel[1] = need;
        }
        __syncthreads();
        select_run(nlist, sel[0], sel[1], [&](int p) { return (int)(list[p] >> 24); },
                   [&](int p) { return (list[p] & 0xfffu) | (((list[p] >> 12) & 0xfffu) << 16); });
    }
    if (tid == 0) *cnt = kept_run;
}

// One workgroup per roi: the cells' keypoints concatenated in grid order,
// ordered by the seeded hash key, the first `cap` out. Keys are unique
// (hash << 32 | candidate index). Only the `cap` smallest are needed: a 256-bin
// histogram of the hashes' top byte finds the bin b holding the cap-th key,
// the keys of bins <= b (about cap + n / 256) are ranked against each other
// (a key's position = the number of smaller keys in that set, which holds
// every smaller key of all n), and a key of rank < cap is written at its rank.
// A set larger than kGfRankMax (cap near n) takes a bitonic sort of all keys.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

constexpr int kGfRankMax = 512;
static_assert(kGfThreads == 256, "one histogram bin per thread");

__global__ __launch_bounds__(kGfThreads) void gridfast_select_kernel(GridFastArgs A) {
    __shared__ unsigned long long key[kGfMaxTotal];
    __shared__ uint32_t cand[kGfMaxTotal];
    __shared__ unsigned long long small[kGfRankMax];
    __shared__ int off[257];
    __shared__ int hist[256];
    __shared__ int nsmall, bsel;
    const int r = blockIdx.x, tid = threadIdx.x;
    const int ncell = A.grid_rows * A.grid_cols;
    const int *cnt = A.cell_cnt + (size_t)r * ncell;
    if (tid == 0) {
        int s = 0;
        for (int c = 0; c < ncell; c++) {
            off[c] = s;
            s += cnt[c];
        }
        off[ncell] = s;
        nsmall = 0;
    }
    hist[tid] = 0;  // kGfThreads == 256 bins
    __syncthreads();
    const int n = off[ncell];
    const int m = min(n, A.cap);
    float *o = A.out_xy + (size_t)r * A.cap * 2;
    if (tid == 0) {
        A.out_count[r] = m;
        if (A.out_total) A.out_total[r] = n;
    }
    if (m <= 0) return;
    const uint32_t h0 = mix32(A.seed + 0x9e3779b9u * (uint32_t)(A.roi_key[r] + 1));
    for (int c = 0; c < ncell; c++) {
        const uint32_t *src = A.cell_kp + ((size_t)r * ncell + c) * A.per_cell;
        for (int j = tid; j < off[c + 1] - off[c]; j += kGfThreads) cand[off[c] + j] = src[j];
    }
    for (int k = tid; k < n; k += kGfThreads) {
        const uint32_t h = mix32(h0 ^ (uint32_t)k);
        key[k] = ((unsigned long long)h << 32) | (uint32_t)k;
        atomicAdd(&hist[h >> 24], 1);
    }
    __syncthreads();
    if (tid < 64) {  // bin of the m-th smallest key: wave-wide scan of 4 bins per lane
        const int b4 = hist[4 * tid] + hist[4 * tid + 1] + hist[4 * tid + 2] + hist[4 * tid + 3];
        int x = b4;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d, 64);
            if (tid >= d) x += y;
        }
        const unsigned long long hit = __ballot(x >= m);  // x: bins [0, 4 tid + 4)
        const int lane = __ffsll((long long)hit) - 1;
        if (tid == lane) {
            int cum = x - b4, b = 4 * tid;
            while (cum + hist[b] < m) cum += hist[b++];
            bsel = b;
        }
    }
    __syncthreads();
    const uint32_t bmax = (uint32_t)bsel;
    for (int k = tid; k < n; k += kGfThreads) {
        const unsigned long long q = key[k];
        if ((uint32_t)(q >> 56) <= bmax) {
            const int i = atomicAdd(&nsmall, 1);
            if (i < kGfRankMax) small[i] = q;
        }
    }
    __syncthreads();
    const int ns = nsmall;
    if (ns <= kGfRankMax) {
        for (int i = tid; i < ns; i += kGfThreads) {
            const unsigned long long q = small[i];
            int rank = 0;
            for (int j = 0; j < ns; j++) rank += small[j] < q;
            if (rank < m) {
                const uint32_t p = cand[(uint32_t)q];
                o[2 * rank] = (float)(p & 0xffffu);
                o[2 * rank + 1] = (float)(p >> 16);
            }
        }
        return;
    }
    int P = 1;
    while (P < n) P <<= 1;
    for (int k = n + tid; k < P; k += kGfThreads) key[k] = ~0ull;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < P / 2; t += kGfThreads) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = key[lo], b = key[hi];
                if ((a > b) == up) {
                    key[lo] = b;
                    key[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < m; i += kGfThreads) {
        const uint32_t p = cand[(uint32_t)key[i]];
        o[2 * i] = (float)(p & 0xffffu);
        o[2 * i + 1] = (float)(p >> 16);
    }
}

int gridfast_lds_bytes(int rw_max, int strip, int list_cap) {
    const int pc = (rw_max + 8 + 3) & ~3, sc = rw_max + 2;
    return (strip + 8) * pc + (((strip + 2) * sc + 15) & ~15) + ((strip * rw_max + 15) & ~15) + 4 * list_cap;
}

// Raises the per-cell kernel's dynamic-LDS limit on the current device; called
// by lk_kernels_init at every context creation (per device, no shared state).
hipError_t gridfast_kernels_init() {
    return hipFuncSetAttribute((const void *)gridfast_cell_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kGfMaxLds);
}

hipError_t launch_gridfast(const GridFastArgs &a, hipStream_t s) {
    if (a.nroi <= 0) return hipSuccess;
    const int lds = gridfast_lds_bytes(a.rw_max, a.strip, a.list_cap);
    hipLaunchKernelGGL(gridfast_cell_kernel, dim3(a.grid_rows * a.grid_cols, a.nroi), dim3(kGfThreads), lds, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gridfast_select_kernel, dim3(a.nroi), dim3(kGfThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace psn
