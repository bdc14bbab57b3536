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

__global__ __launch_bounds__(256) void pyramid_kernel(PyrBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int top = a.nlevels - 1;
    const int W0 = a.lv[0].w, H0 = a.lv[0].h;

    if (top == 0) {  // single level: ingest only, 64x64 tiles
        const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
        for (int idx = tid; idx < 64 * 64; idx += 256) {
            int gy = y0 + (idx >> 6), gx = x0 + (idx & 63);
            if (gy < H0 && gx < W0) a.lv[0].p[(size_t)gy * a.lv[0].pitch + gx] = load_src(a, gy, gx);
        }
        return;
    }

    const int T = a.tile;
    const int topx = blockIdx.x * T, topy = blockIdx.y * T;
    const int n0 = pyr_region_n(top, 0, T);
    const int span = 1 << top;
    const int s0x = span * topx - 2 * (span - 1), s0y = span * topy - 2 * (span - 1);
    int16_t *Ht = (int16_t *)(smem + pyr_lds_off(top, top, T));

    // level-0 region, reflect-101 applied for every position
    {
        uint8_t *B0 = smem;
        const bool interior = s0x >= 0 && s0y >= 0 && s0x + n0 <= W0 && s0y + n0 <= H0;
        for (int idx = tid; idx < n0 * n0; idx += 256) {
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
        for (int idx = tid; idx < own * own; idx += 256) {
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
        for (int idx = tid; idx < np * nl; idx += 256) {
            int r = idx / nl, c = idx - r * nl;
            const uint8_t *q = Bp + r * np + 2 * c;
            Ht[idx] = (int16_t)(q[0] + q[4] + 4 * (q[1] + q[3]) + 6 * q[2]);
        }
        __syncthreads();
        if (l < top) {
            uint8_t *Bl = smem + pyr_lds_off(top, l, T);
            for (int idx = tid; idx < nl * nl; idx += 256) {
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
                for (int idx = tid; idx < nl * nl; idx += 256) {
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
            for (int idx = tid; idx < own * own; idx += 256) {
                int yy = idx / own, xx = idx - yy * own;
                int gy = oy + yy, gx = ox + xx;
                if (gy < Hl && gx < Wl) dst[(size_t)gy * pitch + gx] = Bl[(yy + d) * nl + xx + d];
            }
        } else {
            uint8_t *dst = a.lv[l].p;
            const int pitch = a.lv[l].pitch;
            for (int idx = tid; idx < T * T; idx += 256) {
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

hipError_t launch_pyramid(const PyrBuildArgs &a, hipStream_t s) {
    const int top = a.nlevels - 1;
    dim3 grid;
    int lds = 0;
    if (top == 0) {
        grid = dim3((a.lv[0].w + 63) / 64, (a.lv[0].h + 63) / 64);
    } else {
        grid = dim3((a.lv[top].w + a.tile - 1) / a.tile, (a.lv[top].h + a.tile - 1) / a.tile);
        lds = pyr_lds_bytes(top, a.tile);
    }
    hipLaunchKernelGGL(pyramid_kernel, grid, dim3(256), lds, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LK
// ---------------------------------------------------------------------------

// Chain-major position of window pixel (yl, x) inside a tile of `th` rows.
// A-phase (SSE2): 4 lanes over 4-pixel steps (lane = x&3), then a scalar tail.
__device__ __forceinline__ int chainA_pos(int yl, int x, int th, int nA, int tA) {
    if (x < 4 * nA) return (x & 3) * th * nA + yl * nA + (x >> 2);
    return 4 * th * nA + yl * tA + (x - 4 * nA);
}
// b-phase (SSE2): 8-pixel steps; pixel k = x&7 feeds lane group g = k&3
// (qb0 lanes 0-1: k=0,4; qb0 2-3: k=1,5; qb1 0-1: k=2,6; qb1 2-3: k=3,7), in
// order (row, step, k>>2); then a scalar tail.
__device__ __forceinline__ int chainB_pos(int yl, int x, int th, int nB, int tB) {
    if (x < 8 * nB) return (x & 3) * th * 2 * nB + yl * 2 * nB + 2 * (x >> 3) + ((x >> 2) & 1);
    return 4 * th * 2 * nB + yl * tB + (x - 8 * nB);
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
    const int nA = sse ? w / 4 : 0, tA = w - 4 * nA;
    const int nB = sse ? w / 8 : 0, tB = w - 8 * nB;
    const int JRW = lk_jreg_w(w), JRH = lk_jreg_h(h);

    int16_t *Iw = (int16_t *)smem;
    short2 *Dw = (short2 *)(smem + lk_off_dw(w, h));
    uint8_t *JR = smem + lk_off_jr(w, h);
    float *RED = (float *)(smem + lk_off_red(w, h));
    int *REDI = (int *)(RED + 48);
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

    // thread -> (row, col) walk of a w-wide tile
    const int t_x0 = tid % w, t_y0 = tid / w;
    const int s_x = NT % w, s_y = NT / w;

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
        float fa = __fsub_rn(px, (float)ipx), fb = __fsub_rn(py, (float)ipy);
        int iw00 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), __fsub_rn(1.f, fb)), 16384.f));
        int iw01 = cv_round(__fmul_rn(__fmul_rn(fa, __fsub_rn(1.f, fb)), 16384.f));
        int iw10 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), fb), 16384.f));
        int iw11 = (1 << 14) - iw00 - iw01 - iw10;

        // ---- A-phase: I window, Scharr, structure tensor ----
        float acc = 0.f;
        for (int r0 = 0; r0 < h; r0 += TR) {
            const int th = min(TR, h - r0);
            {  // stage I rows ipy+r0-1 .. +th+1, cols ipx-1 .. ipx+w+1 (reflect-101)
                const int PW = w + 3, PH = th + 3;
                const int gy0 = ipy + r0 - 1, gx0 = ipx - 1;
                const bool interior = gy0 >= 0 && gx0 >= 0 && gy0 + PH <= rows && gx0 + PW <= cols;
                for (int idx = tid; idx < PW * PH; idx += NT) {
                    int yy = idx / PW, xx = idx - yy * PW;
                    int gy = gy0 + yy, gx = gx0 + xx;
                    if (!interior) {
                        gy = refl101(gy, rows);
                        gx = refl101(gx, cols);
                    }
                    Pimg[idx] = I.p[(size_t)gy * I.pitch + gx];
                }
            }
            __syncthreads();
            {  // Scharr on (th+1) x (w+1) positions; zero outside the image
                const int PW = w + 3, DW = w + 1;
                for (int idx = tid; idx < (th + 1) * DW; idx += NT) {
                    int yy = idx / DW, xx = idx - yy * DW;
                    int gy = ipy + r0 + yy, gx = ipx + xx;
                    short2 d = make_short2(0, 0);
                    if ((unsigned)gy < (unsigned)rows && (unsigned)gx < (unsigned)cols) {
                        const uint8_t *p = Pimg + yy * PW + xx;
                        int v0l = 3 * (p[0] + p[2 * PW]) + 10 * p[PW];
                        int v0r = 3 * (p[2] + p[2 * PW + 2]) + 10 * p[PW + 2];
                        int v1l = p[2 * PW] - p[0];
                        int v1c = p[2 * PW + 1] - p[1];
                        int v1r = p[2 * PW + 2] - p[2];
                        d.x = (short)(v0r - v0l);
                        d.y = (short)(3 * (v1l + v1r) + 10 * v1c);
                    }
                    Dg[idx] = d;
                }
            }
            __syncthreads();
            {  // bilinear I / Ix / Iy window rows + A products (chain-major)
                const int PW = w + 3, DW = w + 1, thw = th * w;
                int x = t_x0, yl = t_y0;
                while (yl < th) {
                    const uint8_t *p = Pimg + (yl + 1) * PW + x + 1;
                    int ival = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[PW] * iw10 + p[PW + 1] * iw11, 9);
                    const short2 *d = Dg + yl * DW + x;
                    int ixv = PSN_DESCALE(d[0].x * iw00 + d[1].x * iw01 + d[DW].x * iw10 + d[DW + 1].x * iw11, 14);
                    int iyv = PSN_DESCALE(d[0].y * iw00 + d[1].y * iw01 + d[DW].y * iw10 + d[DW + 1].y * iw11, 14);
                    const int y = r0 + yl;
                    Iw[y * w + x] = (int16_t)ival;
                    Dw[y * w + x] = make_short2((short)ixv, (short)iyv);
                    const int pos = chainA_pos(yl, x, th, nA, tA);
                    Prod[pos] = (float)(ixv * ixv);
                    Prod[thw + pos] = (float)(ixv * iyv);
                    Prod[2 * thw + pos] = (float)(iyv * iyv);
                    x += s_x;
                    yl += s_y;
                    if (x >= w) {
                        x -= w;
                        yl++;
                    }
                }
            }
            __syncthreads();
            if (tid < 15) {  // lane = (chain ch, sum s): sequential float sums
                const int ch = tid % 5, s = tid / 5;
                const int len = ch < 4 ? th * nA : th * tA;
                const float *pp = Prod + s * th * w + (ch < 4 ? ch * th * nA : 4 * th * nA);
                for (int i = 0; i < len; i++) acc = acc + pp[i];
            }
            // the next tile's Prod/Dg writes follow the next __syncthreads()
        }
        if (tid < 15) RED[tid] = acc;
        __syncthreads();
        float A11, A12, A22;
        {
            float s3[3];
#pragma unroll
            for (int s = 0; s < 3; s++) {
                float tail = RED[s * 5 + 4];
                if (sse) {
                    float q = __fadd_rn(__fadd_rn(__fadd_rn(RED[s * 5 + 0], RED[s * 5 + 1]), RED[s * 5 + 2]), RED[s * 5 + 3]);
                    tail = __fadd_rn(tail, q);
                }
                s3[s] = tail;
            }
            A11 = __fmul_rn(s3[0], FLT_SCALE);
            A12 = __fmul_rn(s3[1], FLT_SCALE);
            A22 = __fmul_rn(s3[2], FLT_SCALE);
        }
        float D = __fsub_rn(__fmul_rn(A11, A22), __fmul_rn(A12, A12));
        {
            float dd = __fsub_rn(A11, A22);
            float t = __fadd_rn(__fmul_rn(dd, dd), __fmul_rn(__fmul_rn(4.f, A12), A12));
            float minEig = __fdiv_rn(__fsub_rn(__fadd_rn(A22, A11), sqrtf(t)), (float)(2 * w * h));
            if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = minEig;
            if (minEig < Q.min_eig || D < FLT_EPSILON) {
                if (level == 0) status = 0;
                continue;
            }
        }
        D = __fdiv_rn(1.f, D);
        nx = __fsub_rn(nx, hwx);
        ny = __fsub_rn(ny, hwy);
        float pdx = 0.f, pdy = 0.f;
        bool jr_valid = false;
        int jr_x0 = 0, jr_y0 = 0;

        for (int j = 0; j < Q.max_count; j++) {
            const int inx = cv_floor(nx), iny = cv_floor(ny);
            if (inx < -w || inx >= cols || iny < -h || iny >= rows) {
                if (level == 0) status = 0;
                break;
            }
            fa = __fsub_rn(nx, (float)inx);
            fb = __fsub_rn(ny, (float)iny);
            iw00 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), __fsub_rn(1.f, fb)), 16384.f));
            iw01 = cv_round(__fmul_rn(__fmul_rn(fa, __fsub_rn(1.f, fb)), 16384.f));
            iw10 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), fb), 16384.f));
            iw11 = (1 << 14) - iw00 - iw01 - iw10;

            if (!(jr_valid && inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW && iny + h + 1 <= jr_y0 + JRH)) {
                jr_x0 = inx - kJMargin;
                jr_y0 = iny - kJMargin;
                jr_valid = true;
                const bool interior = jr_x0 >= 0 && jr_y0 >= 0 && jr_x0 + JRW <= cols && jr_y0 + JRH <= rows;
                for (int idx = tid; idx < JRW * JRH; idx += NT) {
                    int yy = idx / JRW, xx = idx - yy * JRW;
                    int gy = jr_y0 + yy, gx = jr_x0 + xx;
                    if (!interior) {
                        gy = refl101(gy, rows);
                        gx = refl101(gx, cols);
                    }
                    JR[idx] = J.p[(size_t)gy * J.pitch + gx];
                }
                __syncthreads();
            }

            float bacc = 0.f;
            for (int r0 = 0; r0 < h; r0 += TR) {
                const int th = min(TR, h - r0), thw = th * w;
                if (r0 > 0) __syncthreads();  // chain lanes done with the previous tile
                {
                    const uint8_t *jb = JR + (iny - jr_y0) * JRW + (inx - jr_x0);
                    int x = t_x0, yl = t_y0;
                    while (yl < th) {
                        const int y = r0 + yl;
                        const uint8_t *p = jb + y * JRW + x;
                        int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                        int diff = jv - Iw[y * w + x];
                        short2 d = Dw[y * w + x];
                        const int pos = chainB_pos(yl, x, th, nB, tB);
                        Prod[pos] = (float)(diff * d.x);
                        Prod[thw + pos] = (float)(diff * d.y);
                        x += s_x;
                        yl += s_y;
                        if (x >= w) {
                            x -= w;
                            yl++;
                        }
                    }
                }
                __syncthreads();
                if (tid < 10) {
                    const int ch = tid % 5, s = tid / 5;
                    const int len = ch < 4 ? th * 2 * nB : th * tB;
                    const float *pp = Prod + s * thw + (ch < 4 ? ch * th * 2 * nB : 4 * th * 2 * nB);
                    for (int i = 0; i < len; i++) bacc = bacc + pp[i];
                }
            }
            if (tid < 10) RED[16 + tid] = bacc;
            __syncthreads();
            float b1 = RED[16 + 4], b2 = RED[16 + 9];
            if (sse) {
                // bbuf = qb0 + qb1; b1 += bbuf[0] + bbuf[2]; b2 += bbuf[1] + bbuf[3]
                float bb0 = __fadd_rn(RED[16 + 0], RED[16 + 2]);
                float bb2 = __fadd_rn(RED[16 + 1], RED[16 + 3]);
                float bb1 = __fadd_rn(RED[16 + 5], RED[16 + 7]);
                float bb3 = __fadd_rn(RED[16 + 6], RED[16 + 8]);
                b1 = __fadd_rn(b1, __fadd_rn(bb0, bb2));
                b2 = __fadd_rn(b2, __fadd_rn(bb1, bb3));
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
                continue;
            }
            fa = __fsub_rn(qx, (float)iqx);
            fb = __fsub_rn(qy, (float)iqy);
            iw00 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), __fsub_rn(1.f, fb)), 16384.f));
            iw01 = cv_round(__fmul_rn(__fmul_rn(fa, __fsub_rn(1.f, fb)), 16384.f));
            iw10 = cv_round(__fmul_rn(__fmul_rn(__fsub_rn(1.f, fa), fb), 16384.f));
            iw11 = (1 << 14) - iw00 - iw01 - iw10;
            __syncthreads();  // every lane is past its last read of JR / RED
            if (!(jr_valid && iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                jr_x0 = iqx - kJMargin;
                jr_y0 = iqy - kJMargin;
                jr_valid = true;
                const bool interior = jr_x0 >= 0 && jr_y0 >= 0 && jr_x0 + JRW <= cols && jr_y0 + JRH <= rows;
                for (int idx = tid; idx < JRW * JRH; idx += NT) {
                    int yy = idx / JRW, xx = idx - yy * JRW;
                    int gy = jr_y0 + yy, gx = jr_x0 + xx;
                    if (!interior) {
                        gy = refl101(gy, rows);
                        gx = refl101(gx, cols);
                    }
                    JR[idx] = J.p[(size_t)gy * J.pitch + gx];
                }
            }
            if (tid == 0) REDI[0] = 0;
            __syncthreads();
            const uint8_t *jb = JR + (iqy - jr_y0) * JRW + (iqx - jr_x0);
            int isum = 0;
            {
                int x = t_x0, y = t_y0;
                while (y < h) {
                    const uint8_t *p = jb + y * JRW + x;
                    int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                    isum += abs(jv - Iw[y * w + x]);
                    x += s_x;
                    y += s_y;
                    if (x >= w) {
                        x -= w;
                        y++;
                    }
                }
            }
            atomicAdd(REDI, isum);
            __syncthreads();
            const int total = REDI[0];
            float errval;
            if (total <= (1 << 24)) {
                // every partial sum of the sequential float chain is an integer
                // <= 2^24, hence exact: the chain equals the integer total
                errval = (float)total;
            } else {
                // sequential row-major chain (errval += |diff|), tiled through Prod
                float eacc = 0.f;
                for (int r0 = 0; r0 < h; r0 += TR) {
                    const int th = min(TR, h - r0);
                    if (r0 > 0) __syncthreads();
                    for (int idx = tid; idx < th * w; idx += NT) {
                        int yl = idx / w, x = idx - yl * w, y = r0 + yl;
                        const uint8_t *p = jb + y * JRW + x;
                        int jv = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[JRW] * iw10 + p[JRW + 1] * iw11, 9);
                        Prod[idx] = (float)abs(jv - Iw[y * w + x]);
                    }
                    __syncthreads();
                    if (tid == 0)
                        for (int i = 0; i < th * w; i++) eacc = eacc + Prod[i];
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

hipError_t launch_lk(const LkLaunchArgs &a, int total_wgs, int threads, int lds_bytes, hipStream_t s) {
    if (total_wgs <= 0) return hipSuccess;
    switch (threads) {
        case 64:
            hipLaunchKernelGGL(lk_kernel<64>, dim3(total_wgs), dim3(64), lds_bytes, s, a);
            break;
        case 128:
            hipLaunchKernelGGL(lk_kernel<128>, dim3(total_wgs), dim3(128), lds_bytes, s, a);
            break;
        default:
            hipLaunchKernelGGL(lk_kernel<256>, dim3(total_wgs), dim3(256), lds_bytes, s, a);
            break;
    }
    return hipGetLastError();
}

hipError_t lk_kernels_init() {
    const int max_lds = 160 * 1024;
    hipError_t e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)lk_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)pyramid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace psn
