// HIP kernels for gfx950 (CDNA4) of the Tracker2D pyramidal-LK path.
//
//   pyramid_kernel  ingest (gray copy or BGR->gray) + all pyrDown levels of one
//                   frame in ONE launch: each workgroup owns a tile of the top
//                   level and recomputes its halo through the levels in LDS.
//                   Replaces cv::cvtColor/resize (PSNWhere_Tracker2D.cpp:257-262)
//                   and buildOpticalFlowPyramid inside every calcOpticalFlowPyrLK
//                   call (:776-782, :871-877).
//   lk_kernel       LKTrackerInvoker over all levels for one point per
//                   workgroup: I patch + Scharr + bilinear window staged in LDS,
//                   J window staged in LDS with a margin, per-iteration 2x2 solve.
//
// Numerics follow OpenCV 2.4.6 exactly (integer fixed-point bilinear, float
// normal equations). The float sums reproduce the SSE2 build's summation
// ORDER (4 lanes for A, 2x4 lanes for b, scalar tail): the per-pixel products
// are computed by all lanes in parallel into LDS, laid out "chain-major", and
// each SSE2 lane / tail chain is summed sequentially by one lane. The result is
// bit-identical to oracle/lk_oracle.c. MFMA is not used: the work is a batch of
// tiny 2x2 solves, not a contraction.
#include <float.h>

#include "psn_lk_kernels.h"

namespace psn {

#define PSN_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

// Diagnostic build (-DPSN_LK_STAMPS): shader-clock stamps of workgroup phases.
#ifdef PSN_LK_STAMPS
#define LK_STAMP(slot)                                                                                   \
    do {                                                                                                 \
        if (threadIdx.x == 0 && A.stamps) A.stamps[(size_t)blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define LK_COUNT(slot, v)                                                          \
    do {                                                                           \
        if (threadIdx.x == 0 && A.stamps) A.stamps[(size_t)blockIdx.x * 64 + (slot)] = (v); \
    } while (0)
#else
#define LK_STAMP(slot) \
    do {              \
    } while (0)
#define LK_COUNT(slot, v) \
    do {                 \
    } while (0)
#endif

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// cvRound(double) on SSE2 (round half to even) of a float value.
__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int cv_floor(float v) { return (int)floorf(v); }

// ---------------------------------------------------------------------------
// Pyramid
// ---------------------------------------------------------------------------

// Region of level l (l < top) that a top-level tile needs, per axis:
// start = 2^(top-l)*t0 - 2*(2^(top-l)-1), size = 2^(top-l)*T + 3*(2^(top-l)-1).
__host__ __device__ inline int pyr_region_n(int top, int l, int T) {
    int sp = 1 << (top - l);
    return sp * T + 3 * (sp - 1);
}
__host__ __device__ inline int pyr_lds_off(int top, int l, int T) {
    int off = 0;
    for (int m = 0; m < l; m++) {
        int n = pyr_region_n(top, m, T);
        off += align16(n * n);
    }
    return off;
}
__host__ __device__ inline int pyr_lds_bytes(int top, int T) {
    if (top == 0) return 0;
    int n0 = pyr_region_n(top, 0, T), n1 = pyr_region_n(top, 1, T);
    return pyr_lds_off(top, top, T) + align16(2 * n0 * n1);
}

__device__ __forceinline__ uint8_t load_src(const PyrBuildArgs &a, int y, int x) {
    const uint8_t *row = a.src + (size_t)y * a.src_stride;
    if (a.channels == 1) return row[x];
    const uint8_t *p = row + 3 * x;  // BGR: RGB2Gray<uchar> with B2Y=1868, G2Y=9617, R2Y=4899
    return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
}

// One top-level tile (bx, by) of a multi-level build (top >= 1) by NT threads.
// Called by pyramid_kernel and, for a deferred build fused into an LK launch,
// by LK workgroups that have finished their point (lk_kernel_st epilogue).
template <int NT>
__device__ __forceinline__ void pyr_tile(const PyrBuildArgs &a, int bx, int by, uint8_t *smem) {
    const int tid = threadIdx.x;
    const int top = a.nlevels - 1;
    const int W0 = a.lv[0].w, H0 = a.lv[0].h;
    const int T = a.tile;
    const int topx = bx * T, topy = by * T;
    const int n0 = pyr_region_n(top, 0, T);
    const int span = 1 << top;
    const int s0x = span * topx - 2 * (span - 1), s0y = span * topy - 2 * (span - 1);
    int16_t *Ht = (int16_t *)(smem + pyr_lds_off(top, top, T));

    // level-0 region, reflect-101 applied for every position
    {
        uint8_t *B0 = smem;
        const bool interior = s0x >= 0 && s0y >= 0 && s0x + n0 <= W0 && s0y + n0 <= H0;
        for (int idx = tid; idx < n0 * n0; idx += NT) {
            int yy = idx / n0, xx = idx - yy * n0;
            int gy = s0y + yy, gx = s0x + xx;
            if (!interior) {
                gy = refl101(gy, H0);
                gx = refl101(gx, W0);
            }
            B0[idx] = load_src(a, gy, gx);
        }
        __syncthreads();
        // own level-0 tile
        const int own = span * T, d = 2 * (span - 1);
        const int ox = topx * span, oy = topy * span;
        uint8_t *dst = a.lv[0].p;
        const int pitch = a.lv[0].pitch;
        for (int idx = tid; idx < own * own; idx += NT) {
            int yy = idx / own, xx = idx - yy * own;
            int gy = oy + yy, gx = ox + xx;
            if (gy < H0 && gx < W0) dst[(size_t)gy * pitch + gx] = B0[(yy + d) * n0 + xx + d];
        }
    }

    for (int l = 1; l <= top; l++) {
        const int sp = 1 << (top - l);
        const int nl = (l == top) ? T : pyr_region_n(top, l, T);
        const int np = pyr_region_n(top, l - 1, T);
        const int slx = sp * topx - 2 * (sp - 1), sly = sp * topy - 2 * (sp - 1);
        const int Wl = a.lv[l].w, Hl = a.lv[l].h;
        const uint8_t *Bp = smem + pyr_lds_off(top, l - 1, T);
        // horizontal [1 4 6 4 1] over the previous region (rows np, cols nl)
        for (int idx = tid; idx < np * nl; idx += NT) {
            int r = idx / nl, c = idx - r * nl;
            const uint8_t *q = Bp + r * np + 2 * c;
            Ht[idx] = (int16_t)(q[0] + q[4] + 4 * (q[1] + q[3]) + 6 * q[2]);
        }
        __syncthreads();
        if (l < top) {
            uint8_t *Bl = smem + pyr_lds_off(top, l, T);
            for (int idx = tid; idx < nl * nl; idx += NT) {
                int yy = idx / nl, xx = idx - yy * nl;
                int gy = sly + yy, gx = slx + xx;
                if ((unsigned)gy < (unsigned)Hl && (unsigned)gx < (unsigned)Wl) {
                    const int16_t *c = Ht + 2 * yy * nl + xx;
                    int v = c[0] + c[4 * nl] + 4 * (c[nl] + c[3 * nl]) + 6 * c[2 * nl];
                    Bl[idx] = (uint8_t)((v + 128) >> 8);
                }
            }
            __syncthreads();
            const bool border = slx < 0 || sly < 0 || slx + nl > Wl || sly + nl > Hl;
            if (border) {  // positions outside the level: copy their reflect-101 source
                for (int idx = tid; idx < nl * nl; idx += NT) {
                    int yy = idx / nl, xx = idx - yy * nl;
                    int gy = sly + yy, gx = slx + xx;
                    if ((unsigned)gy >= (unsigned)Hl || (unsigned)gx >= (unsigned)Wl) {
                        int ry = refl101(gy, Hl) - sly, rx = refl101(gx, Wl) - slx;
                        Bl[idx] = Bl[ry * nl + rx];
                    }
                }
                __syncthreads();
            }
            const int own = sp * T, d = 2 * (sp - 1);
            const int ox = topx * sp, oy = topy * sp;
            uint8_t *dst = a.lv[l].p;
            const int pitch = a.lv[l].pitch;
            for (int idx = tid; idx < own * own; idx += NT) {
                int yy = idx / own, xx = idx - yy * own;
                int gy = oy + yy, gx = ox + xx;
                if (gy < Hl && gx < Wl) dst[(size_t)gy * pitch + gx] = Bl[(yy + d) * nl + xx + d];
            }
        } else {
            uint8_t *dst = a.lv[l].p;
            const int pitch = a.lv[l].pitch;
            for (int idx = tid; idx < T * T; idx += NT) {
                int yy = idx / T, xx = idx - yy * T;
                int gy = topy + yy, gx = topx + xx;
                if (gy < Hl && gx < Wl) {
                    const int16_t *c = Ht + 2 * yy * nl + xx;
                    int v = c[0] + c[4 * nl] + 4 * (c[nl] + c[3 * nl]) + 6 * c[2 * nl];
                    dst[(size_t)gy * pitch + gx] = (uint8_t)((v + 128) >> 8);
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void pyramid_kernel(PyrBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.nlevels == 1) {  // single level: ingest only, 64x64 tiles
        const int W0 = a.lv[0].w, H0 = a.lv[0].h;
        const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
        for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
            int gy = y0 + (idx >> 6), gx = x0 + (idx & 63);
            if (gy < H0 && gx < W0) a.lv[0].p[(size_t)gy * a.lv[0].pitch + gx] = load_src(a, gy, gx);
        }
        return;
    }
    pyr_tile<256>(a, blockIdx.x, blockIdx.y, smem);
}

void pyramid_grid(const PyrBuildArgs &a, int &tiles_x, int &tiles_y, int &lds_bytes) {
    const int top = a.nlevels - 1;
    if (top == 0) {
        tiles_x = (a.lv[0].w + 63) / 64;
        tiles_y = (a.lv[0].h + 63) / 64;
        lds_bytes = 0;
    } else {
        tiles_x = (a.lv[top].w + a.tile - 1) / a.tile;
        tiles_y = (a.lv[top].h + a.tile - 1) / a.tile;
        lds_bytes = pyr_lds_bytes(top, a.tile);
    }
}

hipError_t launch_pyramid(const PyrBuildArgs &a, hipStream_t s) {
    int tx, ty, lds;
    pyramid_grid(a, tx, ty, lds);
    hipLaunchKernelGGL(pyramid_kernel, dim3(tx, ty), dim3(256), lds, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LK
// ---------------------------------------------------------------------------
//
// Float sums. OpenCV accumulates A11/A12/A22 and b1/b2 as float sums of
// integer products, in the SSE2 build's lane order. Two exact ways to get the
// same bits:
//  * fast path: every term is an integer; if sum|t| <= 2^24, every partial
//    sum in ANY order is an integer <= 2^24 and therefore exact in float, so
//    the ordered float sum equals the integer sum. Integer sums are reduced
//    across the workgroup (DPP), |t| sums saturate at 2^30.
//  * otherwise: the per-pixel float products are laid out chain-major in LDS
//    and each SSE2 lane / scalar tail chain is summed sequentially by one lane.

constexpr unsigned kSatCap = 1u << 30;
constexpr int kExact = 1 << 24;

__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ unsigned sat_add(unsigned a, unsigned b) { return min(a + b, kSatCap); }
__device__ __forceinline__ unsigned wave_sum_sat(unsigned v) {
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = sat_add(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Workgroup sums of (wrapping int, wrapping int, saturating, saturating) -- or
// with SAT0 the first one saturating too. Results are uniform.
template <int NT, bool SAT0>
__device__ __forceinline__ void block_reduce4(int &v0, int &v1, unsigned &v2, unsigned &v3, int *scratch) {
    v0 = SAT0 ? (int)wave_sum_sat((unsigned)v0) : wave_sum(v0);
    v1 = wave_sum(v1);
    v2 = wave_sum_sat(v2);
    v3 = wave_sum_sat(v3);
    if constexpr (NT > 64) {
        const int wid = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            scratch[4 * wid + 0] = v0;
            scratch[4 * wid + 1] = v1;
            scratch[4 * wid + 2] = (int)v2;
            scratch[4 * wid + 3] = (int)v3;
        }
        __syncthreads();
        int a0 = 0, a1 = 0;
        unsigned a2 = 0, a3 = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            a0 = SAT0 ? (int)sat_add((unsigned)a0, (unsigned)scratch[4 * w]) : a0 + scratch[4 * w];
            a1 += scratch[4 * w + 1];
            a2 = sat_add(a2, (unsigned)scratch[4 * w + 2]);
            a3 = sat_add(a3, (unsigned)scratch[4 * w + 3]);
        }
        __syncthreads();
        v0 = a0;
        v1 = a1;
        v2 = a2;
        v3 = a3;
    }
}

// Per-thread walk over a PW-wide region in steps of NT elements.
struct Walk {
    int x, y, sx, sy, pw;
    __device__ __forceinline__ void init(int tid, int nt, int pw_) {
        pw = pw_;
        x = tid % pw;
        y = tid / pw;
        sx = nt % pw;
        sy = nt / pw;
    }
    __device__ __forceinline__ void step() {
        x += sx;
        y += sy;
        if (x >= pw) {
            x -= pw;
            y++;
        }
    }
};

// Stage u8 regions of pyramid levels into LDS with reflect-101 addressing and
// up to 2*K loads in flight per thread (two regions are loaded together so
// their memory latencies overlap).
template <int NT, int K>
struct Stager {
    uint8_t *dst;
    const uint8_t *src;
    int pitch, lw, lh, gy0, gx0, n;
    bool interior;
    Walk wk;
    int off;  // uniform batch offset
    __device__ __forceinline__ void init(uint8_t *d, const LevelDev &L, int gy0_, int gx0_, int PW, int PH) {
        dst = d;
        src = L.p;
        pitch = L.pitch;
        lw = L.w;
        lh = L.h;
        gy0 = gy0_;
        gx0 = gx0_;
        n = PW * PH;
        interior = gy0 >= 0 && gx0 >= 0 && gy0 + PH <= lh && gx0 + PW <= lw;
        wk.init(threadIdx.x, NT, PW);
        off = 0;
    }
    __device__ __forceinline__ bool more() const { return off < n; }
    __device__ __forceinline__ void load(uint8_t (&v)[K]) const {
        Walk w = wk;
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (off + k * NT + (int)threadIdx.x < n) {
                int gy = gy0 + w.y, gx = gx0 + w.x;
                if (!interior) {
                    gy = refl101(gy, lh);
                    gx = refl101(gx, lw);
                }
                v[k] = src[(size_t)gy * pitch + gx];
            }
            w.step();
        }
    }
    __device__ __forceinline__ void store(const uint8_t (&v)[K]) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int idx = off + k * NT + (int)threadIdx.x;
            if (idx < n) dst[idx] = v[k];
            wk.step();
        }
        off += K * NT;
    }
};

template <int NT>
__device__ __forceinline__ void stage_one(uint8_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH) {
    Stager<NT, 16> a;
    a.init(dst, L, gy0, gx0, PW, PH);
    while (a.more()) {
        uint8_t v[16];
        a.load(v);
        a.store(v);
    }
}

template <int NT>
__device__ __forceinline__ void stage_two(uint8_t *da, const LevelDev &La, int ya, int xa, int PWa, int PHa,
                                          uint8_t *db, const LevelDev &Lb, int yb, int xb, int PWb, int PHb) {
    Stager<NT, 12> a, b;
    a.init(da, La, ya, xa, PWa, PHa);
    b.init(db, Lb, yb, xb, PWb, PHb);
    while (a.more() || b.more()) {
        uint8_t va[12], vb[12];
        const bool ma = a.more(), mb = b.more();
        if (ma) a.load(va);
        if (mb) b.load(vb);
        if (ma) a.store(va);
        if (mb) b.store(vb);
    }
}

// Sequential float sum of `len` LDS floats (16-B aligned), in order.
__device__ __forceinline__ float chain_sum(const float *p, int len, float acc) {
    const float4 *p4 = (const float4 *)p;
    int i = 0;
#pragma unroll 4
    for (; i + 4 <= len; i += 4) {
        const float4 v = p4[i >> 2];
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
    }
    for (; i < len; i++) acc = acc + p[i];
    return acc;
}

__device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// Chain-major LDS layout of one tile (th rows) -- see the file header.
// A: 4 SSE2 lanes (lane = x&3, 4-pixel steps) then the scalar tail.
struct ChainA {
    int nA, tA, SA, P;  // lane stride, plane size (floats)
    __device__ __forceinline__ ChainA(int w, int th, bool sse) {
        nA = sse ? w / 4 : 0;
        tA = w - 4 * nA;
        SA = round4(th * nA);
        P = 4 * SA + round4(th * tA);
    }
    __device__ __forceinline__ int pos(int yl, int x) const {
        return x < 4 * nA ? (x & 3) * SA + yl * nA + (x >> 2) : 4 * SA + yl * tA + (x - 4 * nA);
    }
};
// b: 8-pixel steps; pixel k = x&7 feeds lane group g = k&3 (qb0 lanes 0-1:
// k=0,4; qb0 2-3: k=1,5; qb1 0-1: k=2,6; qb1 2-3: k=3,7), ordered (row, step,
// k>>2); then the scalar tail.
struct ChainB {
    int nB, tB, SB, P;
    __device__ __forceinline__ ChainB(int w, int th, bool sse) {
        nB = sse ? w / 8 : 0;
        tB = w - 8 * nB;
        SB = round4(th * 2 * nB);
        P = 4 * SB + round4(th * tB);
    }
    __device__ __forceinline__ int pos(int yl, int x) const {
        return x < 8 * nB ? (x & 3) * SB + yl * 2 * nB + 2 * (x >> 3) + ((x >> 2) & 1)
                          : 4 * SB + yl * tB + (x - 8 * nB);
    }
};

__device__ __forceinline__ void bilin_weights(float fx, float fy, int &w00, int &w01, int &w10, int &w11) {
    w00 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fx), __fsub_rn(1.f, fy)), 16384.f));
    w01 = cv_round(__fmul_rn(__fmul_rn(fx, __fsub_rn(1.f, fy)), 16384.f));
    w10 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fx), fy), 16384.f));
    w11 = (1 << 14) - w00 - w01 - w10;
}

template <int NT>
__global__ __launch_bounds__(NT) void lk_kernel(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int g = blockIdx.x;
    int qi = 0;
    while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
    const LkQueryDev &Q = A.q[qi];
    const int pi = Q.pt_begin + (g - Q.wg_begin);
    const int w = Q.win_w, h = Q.win_h;
    const int TR = Q.tile_rows;
    const int maxL = Q.max_level;
    const int flags = Q.flags;
    const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
    const int JRW = lk_jreg_w(w), JRH = lk_jreg_h(h);
    const int PW = w + 3, DW = w + 1;

    int16_t *Iw = (int16_t *)smem;
    short2 *Dw = (short2 *)(smem + lk_off_dw(w, h));
    uint8_t *JR = smem + lk_off_jr(w, h);
    float *RED = (float *)(smem + lk_off_red(w, h));
    int *REDI = (int *)(RED + 48);  // 16 ints of block-reduce scratch
    uint8_t *Pimg = smem + lk_off_tile(w, h);
    short2 *Dg = (short2 *)(Pimg + lk_tile_pimg_bytes(w, TR));
    float *Prod = (float *)((uint8_t *)Dg + lk_tile_dg_bytes(w, TR));

    const float hwx = __fmul_rn((float)(w - 1), 0.5f), hwy = __fmul_rn((float)(h - 1), 0.5f);
    const float px0 = A.prev[2 * pi], py0 = A.prev[2 * pi + 1];
    float NPx = 0.f, NPy = 0.f;
    if (flags & PSN_LK_USE_INITIAL_FLOW) {
        NPx = A.next[2 * pi];
        NPy = A.next[2 * pi + 1];
    }
    int status = 1;
    float errv = 0.f;
    const float FLT_SCALE = 1.f / (1 << 20);

    for (int level = maxL; level >= 0; level--) {
        const LevelDev I = A.slots[Q.prev_slot * kMaxLevels + level];
        const LevelDev J = A.slots[Q.next_slot * kMaxLevels + level];
        const int cols = I.w, rows = I.h;
        const float scale = ldexpf(1.f, -level);
        float px = __fmul_rn(px0, scale), py = __fmul_rn(py0, scale);
        float nx, ny;
        if (level == maxL) {
            if (flags & PSN_LK_USE_INITIAL_FLOW) {
                nx = __fmul_rn(NPx, scale);
                ny = __fmul_rn(NPy, scale);
            } else {
                nx = px;
                ny = py;
            }
        } else {
            nx = __fmul_rn(NPx, 2.f);
            ny = __fmul_rn(NPy, 2.f);
        }
        NPx = nx;
        NPy = ny;
        px = __fsub_rn(px, hwx);
        py = __fsub_rn(py, hwy);
        const int ipx = cv_floor(px), ipy = cv_floor(py);
        if (ipx < -w || ipx >= cols || ipy < -h || ipy >= rows) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            continue;
        }
        int iw00, iw01, iw10, iw11;
        bilin_weights(__fsub_rn(px, (float)ipx), __fsub_rn(py, (float)ipy), iw00, iw01, iw10, iw11);

        // J region for the first iteration, fetched together with the I patch
        nx = __fsub_rn(nx, hwx);
        ny = __fsub_rn(ny, hwy);
        int jr_x0 = cv_floor(nx) - kJMargin, jr_y0 = cv_floor(ny) - kJMargin;
        bool jr_valid = false;

        // ---- A-phase: I window, Scharr, structure tensor ----
        int sA11 = 0, sA12 = 0;
        unsigned aA12 = 0, sA22 = 0;
        for (int r0 = 0; r0 < h; r0 += TR) {
            const int th = min(TR, h - r0);
            if (r0 > 0) __syncthreads();  // previous tile's Pimg/Dg readers are done
            if (r0 == 0) {
                stage_two<NT>(Pimg, I, ipy - 1, ipx - 1, PW, th + 3, JR, J, jr_y0, jr_x0, JRW, JRH);
                jr_valid = true;
            } else {
                stage_one<NT>(Pimg, I, ipy + r0 - 1, ipx - 1, PW, th + 3);
            }
            __syncthreads();
            {  // Scharr on (th+1) x (w+1) positions; zero outside the image
                Walk wk;
                wk.init(tid, NT, DW);
                for (int idx = tid; idx < (th + 1) * DW; idx += NT, wk.step()) {
                    const int yy = wk.y, xx = wk.x;
                    const int gy = ipy + r0 + yy, gx = ipx + xx;
                    short2 d = make_short2(0, 0);
                    if ((unsigned)gy < (unsigned)rows && (unsigned)gx < (unsigned)cols) {
                        const uint8_t *p = Pimg + yy * PW + xx;
                        const int v0l = 3 * (p[0] + p[2 * PW]) + 10 * p[PW];
                        const int v0r = 3 * (p[2] + p[2 * PW + 2]) + 10 * p[PW + 2];
                        const int v1l = p[2 * PW] - p[0];
                        const int v1c = p[2 * PW + 1] - p[1];
                        const int v1r = p[2 * PW + 2] - p[2];
                        d.x = (short)(v0r - v0l);
                        d.y = (short)(3 * (v1l + v1r) + 10 * v1c);
                    }
                    Dg[idx] = d;
                }
            }
            __syncthreads();
            {  // bilinear I / Ix / Iy window rows; integer structure-tensor sums
                Walk wk;
                wk.init(tid, NT, w);
                for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                    const int yl = wk.y, x = wk.x;
                    const uint8_t *p = Pimg + (yl + 1) * PW + x + 1;
                    const int ival = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[PW] * iw10 + p[PW + 1] * iw11, 9);
                    const short2 *d = Dg + yl * DW + x;
                    const int ixv = PSN_DESCALE(d[0].x * iw00 + d[1].x * iw01 + d[DW].x * iw10 + d[DW + 1].x * iw11, 14);
                    const int iyv = PSN_DESCALE(d[0].y * iw00 + d[1].y * iw01 + d[DW].y * iw10 + d[DW + 1].y * iw11, 14);
                    const int y = r0 + yl;
                    Iw[y * w + x] = (int16_t)ival;
                    Dw[y * w + x] = make_short2((short)ixv, (short)iyv);
                    const int xy = ixv * iyv;
                    sA11 = (int)sat_add((unsigned)sA11, (unsigned)(ixv * ixv));
                    sA12 += xy;
                    aA12 = sat_add(aA12, (unsigned)abs(xy));
                    sA22 = sat_add(sA22, (unsigned)(iyv * iyv));
                }
            }
        }
        __syncthreads();  // Iw / Dw complete
        block_reduce4<NT, true>(sA11, sA12, aA12, sA22, REDI);
        const bool ex11 = sA11 <= kExact, ex12 = aA12 <= (unsigned)kExact, ex22 = sA22 <= (unsigned)kExact;
        float A11 = (float)sA11, A12 = (float)sA12, A22 = (float)sA22;
        if (!(ex11 && ex12 && ex22)) {
            // ordered float chains over (float)(Ix*Ix), (float)(Ix*Iy), (float)(Iy*Iy)
            float acc = 0.f;
            for (int r0 = 0; r0 < h; r0 += TR) {
                const int th = min(TR, h - r0);
                const ChainA C(w, th, sse);
                if (r0 > 0) __syncthreads();
                Walk wk;
                wk.init(tid, NT, w);
                for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                    const short2 d = Dw[(r0 + wk.y) * w + wk.x];
                    const int pos = C.pos(wk.y, wk.x);
                    Prod[pos] = (float)(d.x * d.x);
                    Prod[C.P + pos] = (float)(d.x * d.y);
                    Prod[2 * C.P + pos] = (float)(d.y * d.y);
                }
                __syncthreads();
                if (tid < 15) {
                    const int ch = tid % 5, s = tid / 5;
                    const int base = ch < 4 ? ch * C.SA : 4 * C.SA;
                    const int len = ch < 4 ? th * C.nA : th * C.tA;
                    acc = chain_sum(Prod + s * C.P + base, len, acc);
                }
            }
            if (tid < 15) RED[tid] = acc;
            __syncthreads();
            float s3[3];
#pragma unroll
            for (int s = 0; s < 3; s++) {
                float tail = RED[s * 5 + 4];
                if (sse) {
                    const float q = __fadd_rn(__fadd_rn(__fadd_rn(RED[s * 5 + 0], RED[s * 5 + 1]), RED[s * 5 + 2]), RED[s * 5 + 3]);
                    tail = __fadd_rn(tail, q);
                }
                s3[s] = tail;
            }
            if (!ex11) A11 = s3[0];
            if (!ex12) A12 = s3[1];
            if (!ex22) A22 = s3[2];
        }
        A11 = __fmul_rn(A11, FLT_SCALE);
        A12 = __fmul_rn(A12, FLT_SCALE);
        A22 = __fmul_rn(A22, FLT_SCALE);
        float D = __fsub_rn(__fmul_rn(A11, A22), __fmul_rn(A12, A12));
        {
            const float dd = __fsub_rn(A11, A22);
            const float t = __fadd_rn(__fmul_rn(dd, dd), __fmul_rn(__fmul_rn(4.f, A12), A12));
            const float minEig = __fdiv_rn(__fsub_rn(__fadd_rn(A22, A11), sqrtf(t)), (float)(2 * w * h));
            if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = minEig;
            if (minEig < Q.min_eig || D < FLT_EPSILON) {
                if (level == 0) status = 0;
                __syncthreads();
                continue;
            }
        }
        D = __fdiv_rn(1.f, D);
        float pdx = 0.f, pdy = 0.f;

        for (int j = 0; j < Q.max_count; j++) {
            const int inx = cv_floor(nx), iny = cv_floor(ny);
            if (inx < -w || inx >= cols || iny < -h || iny >= rows) {
                if (level == 0) status = 0;
                break;
            }
            bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), iw00, iw01, iw10, iw11);
            if (!(jr_valid && inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW && iny + h + 1 <= jr_y0 + JRH)) {
                jr_x0 = inx - kJMargin;
                jr_y0 = iny - kJMargin;
                jr_valid = true;
                __syncthreads();
                stage_one<NT>(JR, J, jr_y0, jr_x0, JRW, JRH);
                __syncthreads();
            }
            const uint8_t *jb = JR + (iny - jr_y0) * JRW + (inx - jr_x0);
            int s1 = 0, s2 = 0;
            unsigned a1 = 0, a2 = 0;
            {
                Walk wk;
                wk.init(tid, NT, w);
                for (int idx = tid; idx < w * h; idx += NT, wk.step()) {
                    const uint8_t *p = jb + wk.y * JRW + wk.x;
                    const int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                    const int diff = jv - Iw[idx];
                    const short2 d = Dw[idx];
                    const int t1 = diff * d.x, t2 = diff * d.y;
                    s1 += t1;
                    s2 += t2;
                    a1 = sat_add(a1, (unsigned)abs(t1));
                    a2 = sat_add(a2, (unsigned)abs(t2));
                }
            }
            block_reduce4<NT, false>(s1, s2, a1, a2, REDI);
            float b1, b2;
            if (a1 <= (unsigned)kExact && a2 <= (unsigned)kExact) {
                b1 = (float)s1;
                b2 = (float)s2;
            } else {
                float bacc = 0.f;
                for (int r0 = 0; r0 < h; r0 += TR) {
                    const int th = min(TR, h - r0);
                    const ChainB C(w, th, sse);
                    __syncthreads();  // chain lanes done with the previous tile / reduce scratch
                    Walk wk;
                    wk.init(tid, NT, w);
                    for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                        const int y = r0 + wk.y;
                        const uint8_t *p = jb + y * JRW + wk.x;
                        const int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                        const int diff = jv - Iw[y * w + wk.x];
                        const short2 d = Dw[y * w + wk.x];
                        const int pos = C.pos(wk.y, wk.x);
                        Prod[pos] = (float)(diff * d.x);
                        Prod[C.P + pos] = (float)(diff * d.y);
                    }
                    __syncthreads();
                    if (tid < 10) {
                        const int ch = tid % 5, s = tid / 5;
                        const int base = ch < 4 ? ch * C.SB : 4 * C.SB;
                        const int len = ch < 4 ? th * 2 * C.nB : th * C.tB;
                        bacc = chain_sum(Prod + s * C.P + base, len, bacc);
                    }
                }
                if (tid < 10) RED[16 + tid] = bacc;
                __syncthreads();
                b1 = RED[16 + 4];
                b2 = RED[16 + 9];
                if (sse) {
                    // bbuf = qb0 + qb1; b1 += bbuf[0] + bbuf[2]; b2 += bbuf[1] + bbuf[3]
                    const float bb0 = __fadd_rn(RED[16 + 0], RED[16 + 2]);
                    const float bb2 = __fadd_rn(RED[16 + 1], RED[16 + 3]);
                    const float bb1 = __fadd_rn(RED[16 + 5], RED[16 + 7]);
                    const float bb3 = __fadd_rn(RED[16 + 6], RED[16 + 8]);
                    b1 = __fadd_rn(b1, __fadd_rn(bb0, bb2));
                    b2 = __fadd_rn(b2, __fadd_rn(bb1, bb3));
                }
                __syncthreads();  // RED read by all before any later write
            }
            b1 = __fmul_rn(b1, FLT_SCALE);
            b2 = __fmul_rn(b2, FLT_SCALE);
            const float dx = __fmul_rn(__fsub_rn(__fmul_rn(A12, b2), __fmul_rn(A22, b1)), D);
            const float dy = __fmul_rn(__fsub_rn(__fmul_rn(A12, b1), __fmul_rn(A11, b2)), D);
            nx = __fadd_rn(nx, dx);
            ny = __fadd_rn(ny, dy);
            NPx = __fadd_rn(nx, hwx);
            NPy = __fadd_rn(ny, hwy);
            const double dd = __dadd_rn(__dmul_rn((double)dx, (double)dx), __dmul_rn((double)dy, (double)dy));
            if (dd <= Q.eps2) break;
            if (j > 0 && (double)fabsf(__fadd_rn(dx, pdx)) < 0.01 && (double)fabsf(__fadd_rn(dy, pdy)) < 0.01) {
                NPx = __fsub_rn(NPx, __fmul_rn(dx, 0.5f));
                NPy = __fsub_rn(NPy, __fmul_rn(dy, 0.5f));
                break;
            }
            pdx = dx;
            pdy = dy;
        }

        if (level == 0 && status && A.err && (flags & PSN_LK_GET_MIN_EIGENVALS) == 0) {
            const float qx = __fsub_rn(NPx, hwx), qy = __fsub_rn(NPy, hwy);
            const int iqx = cv_floor(qx), iqy = cv_floor(qy);
            if (iqx < -w || iqx >= cols || iqy < -h || iqy >= rows) {
                status = 0;
                __syncthreads();
                continue;
            }
            bilin_weights(__fsub_rn(qx, (float)iqx), __fsub_rn(qy, (float)iqy), iw00, iw01, iw10, iw11);
            if (!(jr_valid && iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                jr_x0 = iqx - kJMargin;
                jr_y0 = iqy - kJMargin;
                jr_valid = true;
                __syncthreads();
                stage_one<NT>(JR, J, jr_y0, jr_x0, JRW, JRH);
                __syncthreads();
            }
            const uint8_t *jb = JR + (iqy - jr_y0) * JRW + (iqx - jr_x0);
            int e0 = 0, e1 = 0;
            unsigned e2 = 0, e3 = 0;
            {
                Walk wk;
                wk.init(tid, NT, w);
                for (int idx = tid; idx < w * h; idx += NT, wk.step()) {
                    const uint8_t *p = jb + wk.y * JRW + wk.x;
                    const int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                    e2 = sat_add(e2, (unsigned)abs(jv - Iw[idx]));
                }
            }
            block_reduce4<NT, false>(e0, e1, e2, e3, REDI);
            float errval;
            if (e2 <= (unsigned)kExact) {
                // every partial sum of errval += |diff| is an integer <= 2^24: exact
                errval = (float)e2;
            } else {
                float eacc = 0.f;
                for (int r0 = 0; r0 < h; r0 += TR) {
                    const int th = min(TR, h - r0);
                    __syncthreads();
                    Walk wk;
                    wk.init(tid, NT, w);
                    for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                        const int y = r0 + wk.y;
                        const uint8_t *p = jb + y * JRW + wk.x;
                        const int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                        Prod[idx] = (float)abs(jv - Iw[y * w + wk.x]);
                    }
                    __syncthreads();
                    if (tid == 0) eacc = chain_sum(Prod, th * w, eacc);
                }
                if (tid == 0) RED[32] = eacc;
                __syncthreads();
                errval = RED[32];
            }
            errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * w * h));
        }
        __syncthreads();  // LDS reuse by the next level
    }

    if (tid == 0) {
        A.next[2 * pi] = NPx;
        A.next[2 * pi + 1] = NPy;
        A.status[pi] = (uint8_t)status;
        if (A.err) A.err[pi] = errv;
    }
}

// ---------------------------------------------------------------------------
// Single-tile LK kernel: the whole window (I, Ix, Iy in registers, product planes in LDS)
// is LDS-resident. Per iteration: ONE fused pass computes the J bilinear
// window, the b-products (written chain-major into a double-buffered plane)
// and their integer sums; one barrier exchanges the per-wave DPP sums; if the
// exact-integer condition fails, EVERY wave sums the 10 float chains itself
// (lanes 0-9, software-pipelined 16-float LDS reads) and reads the results
// with readlane, so no second barrier is needed. Double buffering of the
// planes and of the reduce scratch keeps one barrier per iteration race-free:
// a wave can be at most one iteration ahead of the slowest one.
// ---------------------------------------------------------------------------

__device__ __forceinline__ float add16(float acc, const float4 &a, const float4 &b, const float4 &c, const float4 &d) {
    acc = acc + a.x; acc = acc + a.y; acc = acc + a.z; acc = acc + a.w;
    acc = acc + b.x; acc = acc + b.y; acc = acc + b.z; acc = acc + b.w;
    acc = acc + c.x; acc = acc + c.y; acc = acc + c.z; acc = acc + c.w;
    acc = acc + d.x; acc = acc + d.y; acc = acc + d.z; acc = acc + d.w;
    return acc;
}

// Ordered float sum of nb*16 LDS floats (zero padding is exact: the running
// sum of integer-valued floats starting at +0 is never -0).
__device__ __forceinline__ float chain_sum16(const float *p, int nb) {
    float acc = 0.f;
    if (nb <= 0) return acc;
    const float4 *q = (const float4 *)p;
    float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
    for (int b = 1; b < nb; b++) {
        const float4 c0 = q[4 * b], c1 = q[4 * b + 1], c2 = q[4 * b + 2], c3 = q[4 * b + 3];
        acc = add16(acc, a0, a1, a2, a3);
        a0 = c0;
        a1 = c1;
        a2 = c2;
        a3 = c3;
    }
    return add16(acc, a0, a1, a2, a3);
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Chain-major geometry of a w x h window, regions padded to 16 floats.
struct ChainGeo {
    int nL, tL;      // per-row terms in each SSE2 lane chain / in the tail chain
    int S, T, P;     // lane-region stride, tail-region stride, plane size (floats)
    int lenL, lenT;  // chain lengths
};
__device__ __forceinline__ ChainGeo chain_geo_A(int w, int h, bool sse) {
    ChainGeo g;
    const int nA = sse ? w / 4 : 0;
    g.nL = nA;
    g.tL = w - 4 * nA;
    g.lenL = h * nA;
    g.lenT = h * g.tL;
    g.S = round16i(g.lenL);
    g.T = round16i(g.lenT + 1);
    g.P = lk_st_planeA(w, h, sse);
    return g;
}
__device__ __forceinline__ ChainGeo chain_geo_B(int w, int h, bool sse) {
    ChainGeo g;
    const int nB = sse ? w / 8 : 0;
    g.nL = 2 * nB;
    g.tL = w - 8 * nB;
    g.lenL = h * 2 * nB;
    g.lenT = h * g.tL;
    g.S = round16i(g.lenL);
    g.T = round16i(g.lenT + 1);
    g.P = lk_st_planeB(w, h, sse);
    return g;
}
__device__ __forceinline__ int posA(const ChainGeo &g, int y, int x) {
    const int nA = g.nL;
    return x < 4 * nA ? (x & 3) * g.S + y * nA + (x >> 2) : 4 * g.S + y * g.tL + (x - 4 * nA);
}
__device__ __forceinline__ int posB(const ChainGeo &g, int y, int x) {
    const int n8 = 4 * g.nL;  // 8*nB
    return x < n8 ? (x & 3) * g.S + y * g.nL + 2 * (x >> 3) + ((x >> 2) & 1) : 4 * g.S + y * g.tL + (x - n8);
}
// Zero the padding slots of `np` planes (never product positions).
template <int NT>
__device__ __forceinline__ void zero_pads(float *plane0, const ChainGeo &g, int np) {
    for (int k = threadIdx.x; k < np * 80; k += NT) {
        const int pl = k / 80, c = (k >> 4) % 5, o = k & 15;
        const int len = c < 4 ? g.lenL : g.lenT;
        const int stride = c < 4 ? g.S : g.T;
        if (o < stride - len) plane0[pl * g.P + c * g.S + len + o] = 0.f;
    }
}

// Workgroup sums of (s1 wrapping, s2 wrapping, a saturating): DPP within each
// wave, then the waves' totals through LDS scratch `ri` and ONE barrier (the
// caller's phase barrier). Results are uniform.
template <int NT>
__device__ __forceinline__ void block_sums4(int &s1, int &s2, int &s3, unsigned &a, int *ri) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    s3 = wave_sum(s3);
    a = wave_sum_sat(a);
    if constexpr (NT > 64) {
        const int wid = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            ri[4 * wid + 0] = s1;
            ri[4 * wid + 1] = s2;
            ri[4 * wid + 2] = s3;
            ri[4 * wid + 3] = (int)a;
        }
        __syncthreads();
        int t1 = 0, t2 = 0, t3 = 0;
        unsigned ta = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; k++) {
            t1 += ri[4 * k];
            t2 += ri[4 * k + 1];
            t3 += ri[4 * k + 2];
            ta = sat_add(ta, (unsigned)ri[4 * k + 3]);
        }
        s1 = t1;
        s2 = t2;
        s3 = t3;
        a = ta;
    } else {
        __syncthreads();
    }
}

template <int NT>
__device__ __forceinline__ void block_sums3(int &s1, int &s2, unsigned &a, int *ri) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    a = wave_sum_sat(a);
    if constexpr (NT > 64) {
        const int wid = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            ri[4 * wid + 0] = s1;
            ri[4 * wid + 1] = s2;
            ri[4 * wid + 2] = (int)a;
        }
        __syncthreads();
        int t1 = 0, t2 = 0;
        unsigned ta = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; k++) {
            t1 += ri[4 * k];
            t2 += ri[4 * k + 1];
            ta = sat_add(ta, (unsigned)ri[4 * k + 2]);
        }
        s1 = t1;
        s2 = t2;
        a = ta;
    } else {
        __syncthreads();  // single wave: orders this phase's LDS writes before the next phase's reads
    }
}

typedef const void __attribute__((address_space(1))) *gptr_t;
typedef void __attribute__((address_space(3))) *lptr_t;

// Asynchronous LDS-DMA gather of a PW x PH u8 region of a pyramid level
// (reflect-101 addressing) into LDS, one dword per pixel. Wave w issues the
// 64-pixel chunks w, w+NW, ...; completion = s_waitcnt vmcnt(0) + barrier.
template <int NT>
__device__ __forceinline__ void dma_region(uint32_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH) {
    const int n = PW * PH;
    const bool interior = gy0 >= 0 && gx0 >= 0 && gy0 + PH <= L.h && gx0 + PW <= L.w;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    Walk wk;
    wk.init(threadIdx.x, NT, PW);
    for (int c0 = wid * 64; c0 < n; c0 += NT, wk.step()) {
        if (c0 + lane < n) {
            int gy = gy0 + wk.y, gx = gx0 + wk.x;
            if (!interior) {
                gy = refl101(gy, L.h);
                gx = refl101(gx, L.w);
            }
            const uint8_t *src = L.p + (size_t)gy * L.pitch + gx;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + c0), 1, 0, 0);
        }
    }
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ LevelDev tbl_level(const int *tbl, int pyr, int level) {
    const int *e = tbl + (pyr * kMaxLevels + level) * 8;
    LevelDev L;
    L.p = (uint8_t *)(((uint64_t)(uint32_t)e[1] << 32) | (uint32_t)e[0]);
    L.w = e[2];
    L.h = e[3];
    L.pitch = e[4];
    L.pad_ = 0;
    return L;
}

// Register-staged load of a PW x PH u8 region into LDS (one dword per pixel,
// row stride PW): the loads are issued by load() and written by store(), so
// the memory latency overlaps whatever the caller does in between. Interior
// regions move aligned dwords (4 pixels per load); regions that cross the
// image border gather single bytes through reflect-101. Up to KJ*NT elements
// are in flight; any remainder is moved synchronously by store().
constexpr int KJ = 8;
template <int NT>
struct JStage {
    int v[KJ];
    const uint8_t *src;
    int pitch, lw, lh, gy0, gx0, PW, PH, ax0, ndw, n;
    bool interior;
    __device__ __forceinline__ void fetch(int e, int &out) const {
        if (interior) {  // element = aligned dword d of row y
            const int y = e / ndw, d = e - y * ndw;
            out = *(const __attribute__((address_space(1))) int *)(src + (size_t)(gy0 + y) * pitch + ax0 + 4 * d);
        } else {
            const int y = e / PW, x = e - y * PW;
            out = src[(size_t)refl101(gy0 + y, lh) * pitch + refl101(gx0 + x, lw)];
        }
    }
    __device__ __forceinline__ void put(uint32_t *dst, int e, int val) const {
        if (interior) {
            const int y = e / ndw, d = e - y * ndw;
            const int x0 = ax0 + 4 * d - gx0;  // region column of byte 0
            uint32_t *row = dst + y * PW;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int x = x0 + b;
                if (x >= 0 && x < PW) row[x] = (uint32_t)(val >> (8 * b)) & 0xff;
            }
        } else {
            dst[e] = (uint32_t)val;
        }
    }
    __device__ __forceinline__ void load(const LevelDev &L, int y0, int x0, int pw, int ph) {
        src = L.p;
        pitch = L.pitch;
        lw = L.w;
        lh = L.h;
        gy0 = y0;
        gx0 = x0;
        PW = pw;
        PH = ph;
        interior = y0 >= 0 && x0 >= 0 && y0 + ph <= lh && x0 + pw <= lw;
        ax0 = x0 & ~3;
        ndw = (x0 - ax0 + pw + 3) >> 2;
        n = interior ? ph * ndw : ph * pw;
        // dword loads may read up to 3 bytes past the region's row end: they stay
        // inside the row's 256-B padded pitch or the next row, never past the slot
#pragma unroll
        for (int k = 0; k < KJ; k++) {
            const int e = threadIdx.x + k * NT;
            if (e < n) fetch(e, v[k]);
        }
    }
    __device__ __forceinline__ void store(uint32_t *dst) const {
#pragma unroll
        for (int k = 0; k < KJ; k++) {
            const int e = threadIdx.x + k * NT;
            if (e < n) put(dst, e, v[k]);
        }
        for (int e = threadIdx.x + KJ * NT; e < n; e += NT) {
            int t;
            fetch(e, t);
            put(dst, e, t);
        }
    }
};

template <int NT, int EPT>
__global__ __launch_bounds__(NT) void lk_kernel_st(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int g = blockIdx.x;
    int qi = 0;
    while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
    const LkQueryDev &Q = A.q[qi];
    const int pi = Q.pt_begin + (g - Q.wg_begin);
    const int w = Q.win_w, h = Q.win_h, wh = w * h;
    const int maxL = Q.max_level;
    const int flags = Q.flags;
    const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
    const int JRW = lk_jreg_w(w), JRH = lk_jreg_h(h);
    const int PW = w + 3, DW = w + 1;

    const LkStLayout lay(w, h, sse, maxL + 1);
    int *TBL = (int *)(smem + lay.tbl);
    int *RI = (int *)(smem + lay.ri);  // [4][16]: iterations (x2), A-phase, err
    uint32_t *JR = (uint32_t *)(smem + lay.jr);
    short2 *Dg = (short2 *)(smem + lay.dg);
    float *PA = (float *)(smem + lay.pa);
    float *PB = (float *)(smem + lay.pb);
    const ChainGeo GA = chain_geo_A(w, h, sse), GB = chain_geo_B(w, h, sse);

    // ---- per-thread window pixels (fixed for the whole kernel). Idle lanes
    // (pixel index >= w*h) read pixel 0, carry zero gradients and write their
    // zero products into a pad slot of the chain planes: branch-free loops.
    int ofsJ[EPT], ofsP[EPT], ofsD[EPT], posA_[EPT], posB_[EPT], ofsE[EPT];
    bool ev[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
        const int idx = tid + k * NT;
        ev[k] = idx < wh;
        const int i = ev[k] ? idx : 0;
        const int y = i / w, x = i - (i / w) * w;
        ofsJ[k] = y * JRW + x;
        ofsP[k] = (y + 1) * PW + x + 1;
        ofsD[k] = y * DW + x;
        posA_[k] = ev[k] ? posA(GA, y, x) : 4 * GA.S + GA.lenT;
        posB_[k] = ev[k] ? posB(GB, y, x) : 4 * GB.S + GB.lenT;
        ofsE[k] = ev[k] ? idx : round16i(wh);  // err plane (row-major): idle lanes write past the end
    }

    // ---- prologue: level table -> LDS, zero chain padding once ----
    if (tid < 2 * (maxL + 1) * 8) {
        const int pyr = tid / ((maxL + 1) * 8), rem = tid % ((maxL + 1) * 8), lvl = rem / 8, f = rem % 8;
        const int slot = pyr == 0 ? Q.prev_slot : Q.next_slot;
        const int *src = (const int *)&A.slots[slot * kMaxLevels + lvl];
        if (f < 6) TBL[(pyr * kMaxLevels + lvl) * 8 + f] = src[f];
    }
    zero_pads<NT>(PA, GA, 3);
    zero_pads<NT>(PB, GB, 2);
    zero_pads<NT>(PB + 2 * GB.P, GB, 2);
    __syncthreads();

    const float hwx = __fmul_rn((float)(w - 1), 0.5f), hwy = __fmul_rn((float)(h - 1), 0.5f);
    const float px0 = A.prev[2 * pi], py0 = A.prev[2 * pi + 1];
    float NPx = 0.f, NPy = 0.f;
    if (flags & PSN_LK_USE_INITIAL_FLOW) {
        NPx = A.next[2 * pi];
        NPy = A.next[2 * pi + 1];
    }

    // ---- prologue LDS-DMA: the I patch of EVERY level + the coarsest J region ----
    for (int l = 0; l <= maxL; l++) {
        const LevelDev I = tbl_level(TBL, 0, l);
        const float sc = ldexpf(1.f, -l);
        const int ipx = cv_floor(__fsub_rn(__fmul_rn(px0, sc), hwx)), ipy = cv_floor(__fsub_rn(__fmul_rn(py0, sc), hwy));
        if (ipx < -w || ipx >= I.w || ipy < -h || ipy >= I.h) continue;
        dma_region<NT>((uint32_t *)(smem + lay.pim + l * lay.pim_stride), I, ipy - 1, ipx - 1, PW, h + 3);
    }
    int jr_x0, jr_y0;
    {
        const float sc = ldexpf(1.f, -maxL);
        float nx0 = (flags & PSN_LK_USE_INITIAL_FLOW) ? __fmul_rn(NPx, sc) : __fmul_rn(px0, sc);
        float ny0 = (flags & PSN_LK_USE_INITIAL_FLOW) ? __fmul_rn(NPy, sc) : __fmul_rn(py0, sc);
        jr_x0 = cv_floor(__fsub_rn(nx0, hwx)) - kJMargin;
        jr_y0 = cv_floor(__fsub_rn(ny0, hwy)) - kJMargin;
        dma_region<NT>(JR, tbl_level(TBL, 1, maxL), jr_y0, jr_x0, JRW, JRH);
    }
    dma_wait();
    __syncthreads();

    int status = 1;
    float errv = 0.f;
    const float FLT_SCALE = 1.f / (1 << 20);
    LK_STAMP(60);
#ifdef PSN_LK_STAMPS
    unsigned long long acc_ph[6] = {0, 0, 0, 0, 0, 0}, t_ph = 0;
#define PH_BEGIN() t_ph = __builtin_amdgcn_s_memtime()
#define PH_MARK(i)                                                  \
    do {                                                            \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        acc_ph[i] += t_ - t_ph;                                     \
        t_ph = t_;                                                  \
    } while (0)
#define PH_COUNT(i) acc_ph[i]++
#else
#define PH_BEGIN() \
    do {           \
    } while (0)
#define PH_MARK(i) \
    do {           \
    } while (0)
#define PH_COUNT(i) \
    do {            \
    } while (0)
#endif
    JStage<NT> js;

    for (int level = maxL; level >= 0; level--) {
        LK_STAMP(level * 10 + 0);
        const LevelDev I = tbl_level(TBL, 0, level);
        const LevelDev J = tbl_level(TBL, 1, level);
        const int cols = I.w, rows = I.h;
        const float scale = ldexpf(1.f, -level);
        float px = __fmul_rn(px0, scale), py = __fmul_rn(py0, scale);
        float nx, ny;
        if (level == maxL) {
            if (flags & PSN_LK_USE_INITIAL_FLOW) {
                nx = __fmul_rn(NPx, scale);
                ny = __fmul_rn(NPy, scale);
            } else {
                nx = px;
                ny = py;
            }
        } else {
            nx = __fmul_rn(NPx, 2.f);
            ny = __fmul_rn(NPy, 2.f);
        }
        NPx = nx;
        NPy = ny;
        px = __fsub_rn(px, hwx);
        py = __fsub_rn(py, hwy);
        const int ipx = cv_floor(px), ipy = cv_floor(py);
        if (ipx < -w || ipx >= cols || ipy < -h || ipy >= rows) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
            continue;
        }
        int iw00, iw01, iw10, iw11;
        bilin_weights(__fsub_rn(px, (float)ipx), __fsub_rn(py, (float)ipy), iw00, iw01, iw10, iw11);
        nx = __fsub_rn(nx, hwx);
        ny = __fsub_rn(ny, hwy);
        const bool new_jr = level < maxL;
        if (new_jr) {  // J region of this level: loads in flight during the A-phase
            jr_x0 = cv_floor(nx) - kJMargin;
            jr_y0 = cv_floor(ny) - kJMargin;
            js.load(J, jr_y0, jr_x0, JRW, JRH);
        }
        LK_STAMP(level * 10 + 1);

        // ---- A-phase: Scharr of the staged I patch, bilinear window, tensor ----
        const uint32_t *P = (const uint32_t *)(smem + lay.pim + level * lay.pim_stride);
        {
            Walk wk;
            wk.init(tid, NT, DW);
            for (int idx = tid; idx < (h + 1) * DW; idx += NT, wk.step()) {
                const int gy = ipy + wk.y, gx = ipx + wk.x;
                short2 d = make_short2(0, 0);
                if ((unsigned)gy < (unsigned)rows && (unsigned)gx < (unsigned)cols) {
                    const uint32_t *p = P + wk.y * PW + wk.x;
                    const int a0 = p[0], a1 = p[1], a2 = p[2];
                    const int b0 = p[PW], b2 = p[PW + 2];
                    const int c0 = p[2 * PW], c1 = p[2 * PW + 1], c2 = p[2 * PW + 2];
                    d.x = (short)(3 * (a2 + c2) + 10 * b2 - 3 * (a0 + c0) - 10 * b0);
                    d.y = (short)(3 * ((c0 - a0) + (c2 - a2)) + 10 * (c1 - a1));
                }
                Dg[idx] = d;
            }
        }
        __syncthreads();
        LK_STAMP(level * 10 + 2);
        int Iw_[EPT], Ix_[EPT], Iy_[EPT];
        int sA11 = 0, sA12 = 0, sA22 = 0;
        unsigned aA = 0;  // saturating sum of |every A term|
#pragma unroll
        for (int k = 0; k < EPT; k++) {
            const uint32_t *p = P + ofsP[k];
            Iw_[k] = PSN_DESCALE((int)p[0] * iw00 + (int)p[1] * iw01 + (int)p[PW] * iw10 + (int)p[PW + 1] * iw11, 9);
            const short2 *d = Dg + ofsD[k];
            const short2 d00 = d[0], d01 = d[1], d10 = d[DW], d11 = d[DW + 1];
            const int ix = PSN_DESCALE(d00.x * iw00 + d01.x * iw01 + d10.x * iw10 + d11.x * iw11, 14);
            const int iy = PSN_DESCALE(d00.y * iw00 + d01.y * iw01 + d10.y * iw10 + d11.y * iw11, 14);
            Ix_[k] = ev[k] ? ix : 0;
            Iy_[k] = ev[k] ? iy : 0;
            const int xx2 = Ix_[k] * Ix_[k], xy = Ix_[k] * Iy_[k], yy2 = Iy_[k] * Iy_[k];
            PA[posA_[k]] = (float)xx2;
            PA[GA.P + posA_[k]] = (float)xy;
            PA[2 * GA.P + posA_[k]] = (float)yy2;
            sA11 += xx2;
            sA12 += xy;
            sA22 += yy2;
            aA = sat_add(aA, sat_add(sat_add((unsigned)xx2, (unsigned)abs(xy)), (unsigned)yy2));
        }
        if (new_jr) js.store(JR);  // published by the barrier below
        LK_STAMP(level * 10 + 3);
        block_sums4<NT>(sA11, sA12, sA22, aA, RI + 32);
        LK_STAMP(level * 10 + 4);
        float A11, A12, A22;
        if (aA <= (unsigned)kExact) {
            // every term and every partial sum of the three sums is an integer
            // <= 2^24: exact in float, so any summation order gives these values
            A11 = (float)sA11;
            A12 = (float)sA12;
            A22 = (float)sA22;
        } else {
            float acc = 0.f;
            if (lane < 15) {
                const int ch = lane % 5, s = lane / 5;
                const int base = s * GA.P + (ch < 4 ? ch * GA.S : 4 * GA.S);
                const int nb = (ch < 4 ? GA.S : GA.T) >> 4;
                acc = chain_sum16(PA + base, nb);
            }
            float s3[3];
#pragma unroll
            for (int s = 0; s < 3; s++) {
                float tail = readlane_f(acc, s * 5 + 4);
                if (sse) {
                    const float q = __fadd_rn(__fadd_rn(__fadd_rn(readlane_f(acc, s * 5 + 0), readlane_f(acc, s * 5 + 1)),
                                                        readlane_f(acc, s * 5 + 2)), readlane_f(acc, s * 5 + 3));
                    tail = __fadd_rn(tail, q);
                }
                s3[s] = tail;
            }
            A11 = s3[0];
            A12 = s3[1];
            A22 = s3[2];
        }
        LK_STAMP(level * 10 + 5);
        A11 = __fmul_rn(A11, FLT_SCALE);
        A12 = __fmul_rn(A12, FLT_SCALE);
        A22 = __fmul_rn(A22, FLT_SCALE);
        float D = __fsub_rn(__fmul_rn(A11, A22), __fmul_rn(A12, A12));
        {
            const float dd = __fsub_rn(A11, A22);
            const float t = __fadd_rn(__fmul_rn(dd, dd), __fmul_rn(__fmul_rn(4.f, A12), A12));
            const float minEig = __fdiv_rn(__fsub_rn(__fadd_rn(A22, A11), sqrtf(t)), (float)(2 * wh));
            if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = minEig;
            if (minEig < Q.min_eig || D < FLT_EPSILON) {
                if (level == 0) status = 0;
                continue;
            }
        }
        D = __fdiv_rn(1.f, D);
        float pdx = 0.f, pdy = 0.f;
        LK_STAMP(level * 10 + 6);
        int jdone = 0;

        for (int j = 0; j < Q.max_count; j++) {
            jdone = j + 1;
            PH_BEGIN();
            const int inx = cv_floor(nx), iny = cv_floor(ny);
            if (inx < -w || inx >= cols || iny < -h || iny >= rows) {
                if (level == 0) status = 0;
                break;
            }
            bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), iw00, iw01, iw10, iw11);
            if (!(inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW && iny + h + 1 <= jr_y0 + JRH)) {
                // every wave's JR reads of iteration j-1 precede that iteration's
                // barrier, which this wave has passed
                jr_x0 = inx - kJMargin;
                jr_y0 = iny - kJMargin;
                js.load(J, jr_y0, jr_x0, JRW, JRH);
                js.store(JR);
                __syncthreads();
                PH_COUNT(5);
            }
            const uint32_t *jb = JR + (iny - jr_y0) * JRW + (inx - jr_x0);
            float *pb = PB + (j & 1) * 2 * GB.P;
            int s1 = 0, s2 = 0;
            unsigned a = 0;
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint32_t *p = jb + ofsJ[k];
                const int jv = PSN_DESCALE((int)p[0] * iw00 + (int)p[1] * iw01 + (int)p[JRW] * iw10 + (int)p[JRW + 1] * iw11, 9);
                const int diff = jv - Iw_[k];
                const int t1 = diff * Ix_[k], t2 = diff * Iy_[k];
                pb[posB_[k]] = (float)t1;
                pb[GB.P + posB_[k]] = (float)t2;
                s1 += t1;
                s2 += t2;
                a = sat_add(a, sat_add((unsigned)abs(t1), (unsigned)abs(t2)));
            }
            PH_MARK(0);
            block_sums3<NT>(s1, s2, a, RI + 16 * (j & 1));  // the iteration's barrier
            PH_MARK(1);
            float b1, b2;
            if (a <= (unsigned)kExact) {
                b1 = (float)s1;
                b2 = (float)s2;
            } else {
                float acc = 0.f;
                if (lane < 10) {
                    const int ch = lane % 5, s = lane / 5;
                    const int base = s * GB.P + (ch < 4 ? ch * GB.S : 4 * GB.S);
                    const int nb = (ch < 4 ? GB.S : GB.T) >> 4;
                    acc = chain_sum16(pb + base, nb);
                }
                b1 = readlane_f(acc, 4);
                b2 = readlane_f(acc, 9);
                if (sse) {
                    // bbuf = qb0 + qb1; b1 += bbuf[0] + bbuf[2]; b2 += bbuf[1] + bbuf[3]
                    const float bb0 = __fadd_rn(readlane_f(acc, 0), readlane_f(acc, 2));
                    const float bb2 = __fadd_rn(readlane_f(acc, 1), readlane_f(acc, 3));
                    const float bb1 = __fadd_rn(readlane_f(acc, 5), readlane_f(acc, 7));
                    const float bb3 = __fadd_rn(readlane_f(acc, 6), readlane_f(acc, 8));
                    b1 = __fadd_rn(b1, __fadd_rn(bb0, bb2));
                    b2 = __fadd_rn(b2, __fadd_rn(bb1, bb3));
                }
                PH_COUNT(4);
            }
            PH_MARK(2);
            b1 = __fmul_rn(b1, FLT_SCALE);
            b2 = __fmul_rn(b2, FLT_SCALE);
            const float dx = __fmul_rn(__fsub_rn(__fmul_rn(A12, b2), __fmul_rn(A22, b1)), D);
            const float dy = __fmul_rn(__fsub_rn(__fmul_rn(A12, b1), __fmul_rn(A11, b2)), D);
            nx = __fadd_rn(nx, dx);
            ny = __fadd_rn(ny, dy);
            NPx = __fadd_rn(nx, hwx);
            NPy = __fadd_rn(ny, hwy);
            const double dd = __dadd_rn(__dmul_rn((double)dx, (double)dx), __dmul_rn((double)dy, (double)dy));
            PH_MARK(3);
            if (dd <= Q.eps2) break;
            if (j > 0 && (double)fabsf(__fadd_rn(dx, pdx)) < 0.01 && (double)fabsf(__fadd_rn(dy, pdy)) < 0.01) {
                NPx = __fsub_rn(NPx, __fmul_rn(dx, 0.5f));
                NPy = __fsub_rn(NPy, __fmul_rn(dy, 0.5f));
                break;
            }
            pdx = dx;
            pdy = dy;
        }
        LK_STAMP(level * 10 + 7);
        LK_COUNT(level * 10 + 8, jdone);
        (void)jdone;

        if (level == 0 && status && A.err && (flags & PSN_LK_GET_MIN_EIGENVALS) == 0) {
            const float qx = __fsub_rn(NPx, hwx), qy = __fsub_rn(NPy, hwy);
            const int iqx = cv_floor(qx), iqy = cv_floor(qy);
            if (iqx < -w || iqx >= cols || iqy < -h || iqy >= rows) {
                status = 0;
                continue;
            }
            bilin_weights(__fsub_rn(qx, (float)iqx), __fsub_rn(qy, (float)iqy), iw00, iw01, iw10, iw11);
            __syncthreads();  // every wave is done with PA (A chains) and JR (last products)
            if (!(iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                jr_x0 = iqx - kJMargin;
                jr_y0 = iqy - kJMargin;
                js.load(J, jr_y0, jr_x0, JRW, JRH);
                js.store(JR);
                __syncthreads();
            }
            const uint32_t *jb = JR + (iqy - jr_y0) * JRW + (iqx - jr_x0);
            int e1 = 0, e2 = 0;
            unsigned ea = 0;
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint32_t *p = jb + ofsJ[k];
                const int jv = PSN_DESCALE((int)p[0] * iw00 + (int)p[1] * iw01 + (int)p[JRW] * iw10 + (int)p[JRW + 1] * iw11, 9);
                const int ad = ev[k] ? abs(jv - Iw_[k]) : 0;
                PA[ofsE[k]] = (float)ad;  // row-major, for the sequential fallback
                ea = sat_add(ea, (unsigned)ad);
            }
            for (int k = wh + tid; k < round16i(wh); k += NT) PA[k] = 0.f;
            block_sums3<NT>(e1, e2, ea, RI + 48);
            float errval;
            if (ea <= (unsigned)kExact) {
                errval = (float)ea;  // every partial sum of errval += |diff| is an exact integer
            } else {
                float acc = 0.f;
                if (lane == 0) acc = chain_sum16(PA, round16i(wh) >> 4);
                errval = readlane_f(acc, 0);
            }
            errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * wh));
        }
    }

    LK_STAMP(61);
#ifdef PSN_LK_STAMPS
    for (int i = 0; i < 6; i++) LK_COUNT(40 + i, acc_ph[i]);
#endif
    if (tid == 0) {
        A.next[2 * pi] = NPx;
        A.next[2 * pi + 1] = NPy;
        A.status[pi] = (uint8_t)status;
        if (A.err) A.err[pi] = errv;
    }
    if (A.pyr_ntiles > 0) {
        // fused next-frame ingest: this workgroup's point is done, so it pulls
        // pyramid tiles while slower points keep iterating (fills the tail of
        // the launch instead of a concurrent kernel on a second stream)
        int *tile_slot = RI + 60;
        for (;;) {
            __syncthreads();  // every wave is done with LDS (LK state / previous tile)
            if (tid == 0) tile_slot[0] = (int)atomicAdd(&A.pyr_ctr[0], 1u);
            __syncthreads();
            const int tile = tile_slot[0];
            if (tile >= A.pyr_ntiles) break;
            const int by = tile / A.pyr_tiles_x, bx = tile - by * A.pyr_tiles_x;
            // the tile's LDS starts past the reduce scratch that holds tile_slot
            pyr_tile<NT>(A.pyr, bx, by, smem + lay.jr);
        }
        if (tid == 0) {
            // the last workgroup to finish resets the counters for the next launch;
            // every workgroup has stopped pulling tiles before it counts itself done
            __threadfence();
            const unsigned done = atomicAdd(&A.pyr_ctr[1], 1u);
            if (done == (unsigned)A.total_wgs - 1) {
                A.pyr_ctr[0] = 0;
                A.pyr_ctr[1] = 0;
            }
        }
    }
}
#undef PH_BEGIN
#undef PH_MARK
#undef PH_COUNT

hipError_t launch_lk(const LkLaunchArgs &a, int total_wgs, int threads, int lds_bytes, bool single_tile, hipStream_t s) {
    if (total_wgs <= 0) return hipSuccess;
    const dim3 grid(total_wgs);
    if (single_tile) {
        // threads encodes (workgroup size, pixels per thread): NT * 10 + EPT
        switch (threads) {
            case 642: hipLaunchKernelGGL((lk_kernel_st<64, 2>), grid, dim3(64), lds_bytes, s, a); break;
            case 644: hipLaunchKernelGGL((lk_kernel_st<64, 4>), grid, dim3(64), lds_bytes, s, a); break;
            case 1282: hipLaunchKernelGGL((lk_kernel_st<128, 2>), grid, dim3(128), lds_bytes, s, a); break;
            case 1284: hipLaunchKernelGGL((lk_kernel_st<128, 4>), grid, dim3(128), lds_bytes, s, a); break;
            case 2562: hipLaunchKernelGGL((lk_kernel_st<256, 2>), grid, dim3(256), lds_bytes, s, a); break;
            default: hipLaunchKernelGGL((lk_kernel_st<256, 4>), grid, dim3(256), lds_bytes, s, a); break;
        }
    } else {
        switch (threads) {
            case 64: hipLaunchKernelGGL(lk_kernel<64>, grid, dim3(64), lds_bytes, s, a); break;
            case 128: hipLaunchKernelGGL(lk_kernel<128>, grid, dim3(128), lds_bytes, s, a); break;
            default: hipLaunchKernelGGL(lk_kernel<256>, grid, dim3(256), lds_bytes, s, a); break;
        }
    }
    return hipGetLastError();
}

hipError_t lk_kernels_init() {
    const int max_lds = 160 * 1024;
    hipError_t e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    const void *st[] = {(const void *)lk_kernel_st<64, 2>,  (const void *)lk_kernel_st<64, 4>,
                        (const void *)lk_kernel_st<128, 2>, (const void *)lk_kernel_st<128, 4>,
                        (const void *)lk_kernel_st<256, 2>, (const void *)lk_kernel_st<256, 4>};
    for (const void *f : st)
        if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)pyramid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace psn
