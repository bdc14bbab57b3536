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
#include <limits.h>

#include <type_traits>

#include "psn_gridfast.h"
#include "psn_lk_kernels.h"
#include "psn_lk_device.h"
#include "psn_lk_bx.h"

namespace psn {


// Diagnostic build (-DPSN_LK_STAMPS): shader-clock stamps of workgroup phases.
#ifdef PSN_LK_STAMPS
// ordered: the stamp is taken where it stands in program order (issue time)
#define LK_STAMP(slot)                                                                            \
    do {                                                                                          \
        unsigned long long t_s;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_s) : : "memory");             \
        if (threadIdx.x == 0 && A.stamps) A.stamps[(size_t)blockIdx.x * 64 + (slot)] = t_s;      \
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


// ---------------------------------------------------------------------------
// Pyramid
// ---------------------------------------------------------------------------

// (the LDS plan of a tile, pyr_lds_bytes, and its build-time guards: psn_lk_kernels.h)

__device__ __forceinline__ uint8_t load_src(const PyrBuildArgs &a, int y, int x) {
    const uint8_t *row = a.src + (size_t)y * a.src_stride;
    if (a.channels == 1) return row[x];
    const uint8_t *p = row + 3 * x;  // BGR: RGB2Gray<uchar> with B2Y=1868, G2Y=9617, R2Y=4899
    return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
}

// One top-level tile (bx, by) of a multi-level build (top >= 1) by NT threads
// laid out 16 wide (no index divisions). The tile recomputes its halo through
// the levels in LDS: level-0 region (dword loads for interior gray tiles,
// reflect-101 byte gathers otherwise), then per level a horizontal [1 4 6 4 1]
// pass into int16 and a vertical pass with (sum + 128) >> 8; region positions
// outside a level take their reflect-101 source. Each level's own tile goes
// out as dword stores. Called by pyramid_kernel and, for a deferred build
// fused into an LK launch, by the LK launch's workgroups (pyr_tail).
template <int NT>
__device__ __forceinline__ void pyr_tile(const PyrBuildArgs &a, int bx, int by, uint8_t *smem) {
    constexpr int TX = 16, TY = NT / 16;
    const int tx = threadIdx.x & (TX - 1), ty = threadIdx.x / TX;
    const int top = a.nlevels - 1;
    const int W0 = a.lv[0].w, H0 = a.lv[0].h;
    const int T = a.tile;
    const int topx = bx * T, topy = by * T;
    const int n0 = pyr_region_n(top, 0, T);
    const int span = 1 << top;
    const int s0x = span * topx - 2 * (span - 1), s0y = span * topy - 2 * (span - 1);
    const int ax = s0x & ~3, off0 = s0x - ax, S0 = pyr_s0(n0);
    uint8_t *B0 = smem;
    int16_t *Ht = (int16_t *)(smem + pyr_lds_off(top, top, T));

    // level-0 region
    {
        const int m = (off0 + n0 + 3) >> 2;  // dwords per row
        const bool dw = s0x >= 0 && s0y >= 0 && ax + 4 * m <= W0 && s0y + n0 <= H0 &&
                        ((uintptr_t)a.src & 3) == 0 && (a.src_stride & 3) == 0;
        if (dw && a.channels == 1) {
            for (int r = ty; r < n0; r += TY) {
                const uint32_t *srow = (const uint32_t *)(a.src + (size_t)(s0y + r) * a.src_stride + ax);
                for (int d = tx; d < m; d += TX) *(uint32_t *)(B0 + r * S0 + 4 * d) = srow[d];
            }
        } else if (dw) {
            // BGR interior region: 4 pixels = 3 aligned dwords -> RGB2Gray<uchar> -> one dword
            for (int r = ty; r < n0; r += TY) {
                const uint32_t *srow = (const uint32_t *)(a.src + (size_t)(s0y + r) * a.src_stride + 3 * ax);
                for (int d = tx; d < m; d += TX) {
                    const uint32_t w0 = srow[3 * d], w1 = srow[3 * d + 1], w2 = srow[3 * d + 2];
                    const uint32_t bgr[12] = {w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255, w0 >> 24,
                                              w1 & 255, (w1 >> 8) & 255, (w1 >> 16) & 255, w1 >> 24,
                                              w2 & 255, (w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24};
                    uint32_t out = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        out |= ((bgr[3 * k] * 1868 + bgr[3 * k + 1] * 9617 + bgr[3 * k + 2] * 4899 + (1 << 13)) >> 14)
                               << (8 * k);
                    *(uint32_t *)(B0 + r * S0 + 4 * d) = out;
                }
            }
        } else {
            for (int r = ty; r < n0; r += TY) {
                const int gy = refl101(s0y + r, H0);
                for (int c = tx; c < n0; c += TX) B0[r * S0 + off0 + c] = load_src(a, gy, refl101(s0x + c, W0));
            }
        }
    }
    __syncthreads();
    // own level-0 tile
    {
        const int own = span * T, d0 = 2 * (span - 1);
        const int ox = topx * span, oy = topy * span;
        uint8_t *dst = a.lv[0].p;
        const int pitch = a.lv[0].pitch;
        for (int r = ty; r < own && oy + r < H0; r += TY) {
            const uint8_t *srow = B0 + (r + d0) * S0 + off0 + d0;
            uint8_t *drow = dst + (size_t)(oy + r) * pitch + ox;
            for (int q = tx; q < own / 4; q += TX) {
                const uint8_t *sp4 = srow + 4 * q;
                if (ox + 4 * q + 4 <= W0) {
                    *(uint32_t *)(drow + 4 * q) =
                        sp4[0] | ((uint32_t)sp4[1] << 8) | ((uint32_t)sp4[2] << 16) | ((uint32_t)sp4[3] << 24);
                } else {
                    for (int b = 0; b < 4; b++)
                        if (ox + 4 * q + b < W0) drow[4 * q + b] = sp4[b];
                }
            }
        }
    }

    for (int l = 1; l <= top; l++) {
        const int sp = 1 << (top - l);
        const int nl = (l == top) ? T : pyr_region_n(top, l, T);
        const int np = pyr_region_n(top, l - 1, T);
        const int slx = sp * topx - 2 * (sp - 1), sly = sp * topy - 2 * (sp - 1);
        const int Wl = a.lv[l].w, Hl = a.lv[l].h;
        const uint8_t *Bp = l == 1 ? B0 + off0 : smem + pyr_lds_off(top, l - 1, T);
        const int Sp = l == 1 ? S0 : np;
        // horizontal [1 4 6 4 1] over the previous region (rows np, cols nl)
        for (int r = ty; r < np; r += TY)
            for (int c = tx; c < nl; c += TX) {
                const uint8_t *q = Bp + r * Sp + 2 * c;
                Ht[r * nl + c] = (int16_t)(q[0] + q[4] + 4 * (q[1] + q[3]) + 6 * q[2]);
            }
        __syncthreads();
        if (l < top) {
            uint8_t *Bl = smem + pyr_lds_off(top, l, T);
            for (int r = ty; r < nl; r += TY)
                for (int c = tx; c < nl; c += TX) {
                    const int gy = sly + r, gx = slx + c;
                    if ((unsigned)gy < (unsigned)Hl && (unsigned)gx < (unsigned)Wl) {
                        const int16_t *cc = Ht + 2 * r * nl + c;
                        const int v = cc[0] + cc[4 * nl] + 4 * (cc[nl] + cc[3 * nl]) + 6 * cc[2 * nl];
                        Bl[r * nl + c] = (uint8_t)((v + 128) >> 8);
                    }
                }
            __syncthreads();
            const bool border = slx < 0 || sly < 0 || slx + nl > Wl || sly + nl > Hl;
            if (border) {  // positions outside the level: copy their reflect-101 source
                for (int r = ty; r < nl; r += TY)
                    for (int c = tx; c < nl; c += TX) {
                        const int gy = sly + r, gx = slx + c;
                        if ((unsigned)gy >= (unsigned)Hl || (unsigned)gx >= (unsigned)Wl) {
                            const int ry = refl101(gy, Hl) - sly, rx = refl101(gx, Wl) - slx;
                            Bl[r * nl + c] = Bl[ry * nl + rx];
                        }
                    }
                __syncthreads();
            }
            const int own = sp * T, d = 2 * (sp - 1);
            const int ox = topx * sp, oy = topy * sp;
            uint8_t *dst = a.lv[l].p;
            const int pitch = a.lv[l].pitch;
            for (int r = ty; r < own && oy + r < Hl; r += TY) {
                const uint8_t *srow = Bl + (r + d) * nl + d;
                uint8_t *drow = dst + (size_t)(oy + r) * pitch + ox;
                for (int q = tx; q < own / 4; q += TX) {
                    const uint8_t *sp4 = srow + 4 * q;
                    if (ox + 4 * q + 4 <= Wl) {
                        *(uint32_t *)(drow + 4 * q) =
                            sp4[0] | ((uint32_t)sp4[1] << 8) | ((uint32_t)sp4[2] << 16) | ((uint32_t)sp4[3] << 24);
                    } else {
                        for (int b = 0; b < 4; b++)
                            if (ox + 4 * q + b < Wl) drow[4 * q + b] = sp4[b];
                    }
                }
            }
        } else {
            uint8_t *dst = a.lv[l].p;
            const int pitch = a.lv[l].pitch;
            for (int r = ty; r < T; r += TY)
                for (int c = tx; c < T; c += TX) {
                    const int gy = topy + r, gx = topx + c;
                    if (gy < Hl && gx < Wl) {
                        const int16_t *cc = Ht + 2 * r * nl + c;
                        const int v = cc[0] + cc[4 * nl] + 4 * (cc[nl] + cc[3 * nl]) + 6 * cc[2 * nl];
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
    // XCD-aware tile order (as lk_kernel_bx): runs of consecutive row-major tiles
    // share one XCD's L2, so the halo a tile re-reads of its neighbours is an L2 hit
    const int n = gridDim.x * gridDim.y, t = xcd_remap((int)(blockIdx.y * gridDim.x + blockIdx.x), n);
    pyr_tile<256>(a, t % gridDim.x, t / gridDim.x, smem);
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


template <int NT>
__global__ __launch_bounds__(NT) void lk_kernel(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int g = blockIdx.x;
    int qi = 0;
    while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
    const LkQueryDev &Q = A.q[qi];
    const int pi = lk_query_point(Q, A.counts, A.count_stride, g);
    if (pi < 0) return;  // past the query's device count
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
            if (sums_exact(a1, s1) && sums_exact(a2, s2)) {  // subset-sum bound (see sums_exact)
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

// Element walk of a region with m elements per row: this thread's first
// element (row, column) and the per-NT step (computed once per kernel).
struct JWalk {
    int ey0, ex0, sy, sx, m;
};
__device__ __forceinline__ JWalk jwalk_t(int t, int m, int nt, unsigned mg) {
    JWalk wk;
    wk.m = m;
    wk.ey0 = qdiv(t, mg);
    wk.ex0 = t - wk.ey0 * m;
    wk.sy = qdiv(nt, mg);
    wk.sx = nt - wk.sy * m;
    return wk;
}
__device__ __forceinline__ JWalk jwalk(int m, int nt) {
    JWalk wk;
    wk.m = m;
    wk.ey0 = threadIdx.x / m;
    wk.ex0 = threadIdx.x - wk.ey0 * m;
    wk.sy = nt / m;
    wk.sx = nt - wk.sy * m;
    return wk;
}

// Register-staged load of a J region into LDS in PAIR format: dword c of a
// row holds J[c] | J[c+1] << 16, so one LDS read feeds one packed dot
// (v_dot2_i32_i16) half of the bilinear interpolation. load() issues the
// global loads and store() writes LDS, so the memory latency overlaps whatever
// the caller does in between (the next level's region is prefetched at its
// predicted position while this level iterates). The region origin is a
// multiple of 4 columns: interior regions move 8 bytes per element (two
// aligned dwords) and write 4 pairs with one 16-B LDS store; regions that cross
// the image border gather the 2 bytes of each pair through reflect-101. KJ*NT
// elements are held in registers; the rest move synchronously in store().
// With cs > 0 the region is written COLUMN-major (pair (r, c) at c * cs + r),
// the layout of the one-wave iteration kernel.
constexpr int KJ = 4;
template <int NT>
struct JPStage {
    uint2 v[KJ];
    const uint8_t *src;
    int pitch, lw, lh, gy0, gx0, PW, PH;
    int cs = 0;
    bool interior;
    JWalk wk;
    __device__ __forceinline__ void setup(const LevelDev &L, int y0, int x0, int pw, int ph, const JWalk &wi,
                                          const JWalk &wb) {
        src = L.p;
        pitch = L.pitch;
        lw = L.w;
        lh = L.h;
        gy0 = y0;
        gx0 = x0;
        PW = pw;
        PH = ph;
        interior = y0 >= 0 && x0 >= 0 && y0 + ph <= lh && x0 + pw <= lw;
        wk = interior ? wi : wb;
    }
    __device__ __forceinline__ void step(int &y, int &x) const {
        x += wk.sx;
        y += wk.sy;
        if (x >= wk.m) {
            x -= wk.m;
            y++;
        }
    }
    __device__ __forceinline__ void fetch(int y, int x, uint2 &out) const {
        typedef const __attribute__((address_space(1))) unsigned gu32;
        if (interior) {
            // bytes 4x .. 4x+7 of the row (the last element reads 4 bytes past the
            // region: inside the 256-B padded pitch, the next row, or the slot slack)
            gu32 *q = (gu32 *)(src + (size_t)(gy0 + y) * pitch + gx0 + 4 * x);
            out.x = q[0];
            out.y = q[1];
        } else {
            const uint8_t *row = src + (size_t)refl101(gy0 + y, lh) * pitch;
            out.x = row[refl101(gx0 + x, lw)];
            out.y = row[refl101(gx0 + x + 1, lw)];
        }
    }
    __device__ __forceinline__ void put(uint32_t *dst, int y, int x, const uint2 &val) const {
        if (interior) {
            uint4 q;
            q.x = __builtin_amdgcn_perm(val.y, val.x, 0x0c010c00u);  // J[4x]   | J[4x+1] << 16
            q.y = __builtin_amdgcn_perm(val.y, val.x, 0x0c020c01u);
            q.z = __builtin_amdgcn_perm(val.y, val.x, 0x0c030c02u);
            q.w = __builtin_amdgcn_perm(val.y, val.x, 0x0c040c03u);  // J[4x+3] | J[4x+4] << 16
            if (cs > 0) {
                uint32_t *d = dst + 4 * x * cs + y;
                d[0] = q.x;
                d[cs] = q.y;
                d[2 * cs] = q.z;
                d[3 * cs] = q.w;
            } else {
                *(uint4 *)(dst + y * PW + 4 * x) = q;
            }
        } else {
            dst[cs > 0 ? x * cs + y : y * PW + x] = val.x | (val.y << 16);
        }
    }
    __device__ __forceinline__ void load(const LevelDev &L, int y0, int x0, int pw, int ph, const JWalk &wi,
                                         const JWalk &wb) {
        setup(L, y0, x0, pw, ph, wi, wb);
        int y = wk.ey0, x = wk.ex0;
#pragma unroll
        for (int k = 0; k < KJ; k++) {
            if (y < PH) fetch(y, x, v[k]);
            step(y, x);
        }
    }
    __device__ __forceinline__ void store(uint32_t *dst) const {
        int y = wk.ey0, x = wk.ex0;
#pragma unroll
        for (int k = 0; k < KJ; k++) {
            if (y < PH) put(dst, y, x, v[k]);
            step(y, x);
        }
        while (y < PH) {
            uint2 t;
            fetch(y, x, t);
            put(dst, y, x, t);
            step(y, x);
        }
    }
    // synchronous load + store (restage inside the iterations)
    __device__ __forceinline__ void copy(uint32_t *dst, const LevelDev &L, int y0, int x0, int pw, int ph,
                                         const JWalk &wi, const JWalk &wb) {
        setup(L, y0, x0, pw, ph, wi, wb);
        int y = wk.ey0, x = wk.ex0;
        while (y < PH) {
            uint2 t;
            fetch(y, x, t);
            put(dst, y, x, t);
            step(y, x);
        }
    }
};

// Level table in LDS (single-tile kernel): entry (pyramid s, level l) = 8 ints
// {ptr lo, ptr hi, w, h, pitch}; s = 0 the I (prev) pyramid, 1 the J (next).
__device__ __forceinline__ void tbl_put(int *tbl, int s, int l, const LevelDev &L) {
    int *e = tbl + (s * kMaxLevels + l) * 8;
    const unsigned long long pv = (unsigned long long)L.p;
    *(int4 *)e = make_int4((int)(unsigned)pv, (int)(unsigned)(pv >> 32), L.w, L.h);
    e[4] = L.pitch;
}
__device__ __forceinline__ LevelDev tbl_get(const int *tbl, int s, int l) {
    const int *e = tbl + (s * kMaxLevels + l) * 8;
    const int4 a = *(const int4 *)e;
    LevelDev L;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane(a.x), hi = (unsigned)__builtin_amdgcn_readfirstlane(a.y);
    L.p = (uint8_t *)(((unsigned long long)hi << 32) | lo);
    L.w = __builtin_amdgcn_readfirstlane(a.z);
    L.h = __builtin_amdgcn_readfirstlane(a.w);
    L.pitch = __builtin_amdgcn_readfirstlane(e[4]);
    L.pad_ = 0;
    return L;
}

// Three simultaneous 64-lane sums (DPP, interleaved); a is clamped per lane to
// 2^25 first so its total cannot wrap. Results are uniform.
__device__ __forceinline__ void wave_sum3(int &s1, int &s2, unsigned &a) {
    a = min(a, 1u << 25);
#define PSN_DPP3(ctl, rm)                                                   \
    s1 += __builtin_amdgcn_update_dpp(0, s1, ctl, rm, 0xf, false);          \
    s2 += __builtin_amdgcn_update_dpp(0, s2, ctl, rm, 0xf, false);          \
    a += (unsigned)__builtin_amdgcn_update_dpp(0, (int)a, ctl, rm, 0xf, false)
    PSN_DPP3(0x111, 0xf);
    PSN_DPP3(0x112, 0xf);
    PSN_DPP3(0x114, 0xf);
    PSN_DPP3(0x118, 0xf);
    PSN_DPP3(0x142, 0xa);
    PSN_DPP3(0x143, 0xc);
#undef PSN_DPP3
    s1 = __builtin_amdgcn_readlane(s1, 63);
    s2 = __builtin_amdgcn_readlane(s2, 63);
    a = (unsigned)__builtin_amdgcn_readlane((int)a, 63);
}

// Four simultaneous 64-lane sums (one-wave iterations): s1, s2 and the
// per-lane sum|t1|, sum|t2|, clamped per lane to 2^25 + 1 first (a clamped lane
// alone fails the exactness test below; totals stay below 2^31).
__device__ __forceinline__ void wave_sum4(int &s1, int &s2, unsigned &a1, unsigned &a2) {
    a1 = min(a1, (1u << 25) + 1u);
    a2 = min(a2, (1u << 25) + 1u);
#define PSN_DPP4(ctl, rm)                                                   \
    s1 += __builtin_amdgcn_update_dpp(0, s1, ctl, rm, 0xf, false);          \
    s2 += __builtin_amdgcn_update_dpp(0, s2, ctl, rm, 0xf, false);          \
    a1 += (unsigned)__builtin_amdgcn_update_dpp(0, (int)a1, ctl, rm, 0xf, false); \
    a2 += (unsigned)__builtin_amdgcn_update_dpp(0, (int)a2, ctl, rm, 0xf, false)
    PSN_DPP4(0x111, 0xf);
    PSN_DPP4(0x112, 0xf);
    PSN_DPP4(0x114, 0xf);
    PSN_DPP4(0x118, 0xf);
    PSN_DPP4(0x142, 0xa);
    PSN_DPP4(0x143, 0xc);
#undef PSN_DPP4
    s1 = __builtin_amdgcn_readlane(s1, 63);
    s2 = __builtin_amdgcn_readlane(s2, 63);
    a1 = (unsigned)__builtin_amdgcn_readlane((int)a1, 63);
    a2 = (unsigned)__builtin_amdgcn_readlane((int)a2, 63);
}
// Level geometry of the I window (prevPt/2^l - halfWin): top-left, validity and weights.
struct IGeo {
    int ipx, ipy, w00, w01, w10, w11;
    bool valid;
};
__device__ __forceinline__ IGeo i_geo(float px0, float py0, float hwx, float hwy, int level, int w, int h, int cols,
                                      int rows) {
    IGeo gg;
    const float scale = ldexpf(1.f, -level);
    const float px = __fsub_rn(__fmul_rn(px0, scale), hwx), py = __fsub_rn(__fmul_rn(py0, scale), hwy);
    gg.ipx = cv_floor(px);
    gg.ipy = cv_floor(py);
    gg.valid = !(gg.ipx < -w || gg.ipx >= cols || gg.ipy < -h || gg.ipy >= rows);
    bilin_weights(__fsub_rn(px, (float)gg.ipx), __fsub_rn(py, (float)gg.ipy), gg.w00, gg.w01, gg.w10, gg.w11);
    return gg;
}

// Fused next-frame ingest (PSN_LK_OVERLAP_FUSED): helper workgroups, and LK
// workgroups whose point is done, pull top-level pyramid tiles from a work
// counter while slower points keep iterating. Every workgroup of the launch
// counts itself done once it stopped pulling; the last one resets the counters
// for the next launch on the stream.
template <int NT>
__device__ __forceinline__ void pyr_tail(const LkLaunchArgs &A, uint8_t *smem) {
    int *tile_slot = (int *)(smem + 2 * kMaxLevels * 8 * 4) + kStRiTile;  // inside the scratch area
    __builtin_amdgcn_s_setprio(0);
    for (;;) {
        __syncthreads();  // every wave is done with LDS (LK state / previous tile)
        if (threadIdx.x == 0) tile_slot[0] = (int)atomicAdd(&A.pyr_ctr[0], 1u);
        __syncthreads();
        const int tile = tile_slot[0];
        if (tile >= A.pyr_ntiles) break;
        const int by = tile / A.pyr_tiles_x, bx = tile - by * A.pyr_tiles_x;
        pyr_tile<NT>(A.pyr, bx, by, smem + kStScratchBytes);  // past the scratch holding tile_slot
    }
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned done = atomicAdd(&A.pyr_ctr[1], 1u);
        if (done == (unsigned)A.total_wgs - 1) {
            A.pyr_ctr[0] = 0;
            A.pyr_ctr[1] = 0;
        }
    }
}

// Solver table of one level from the A sums (a11, a22 saturating, s12 wrapping)
// and the 15 ordered chain sums c (sum s = 0..2: chains 5s..5s+3 the SSE2 lanes,
// 5s+4 the tail; used only when the sum is not exact as an integer):
// {A11, A12, A22, 1/D, minEig, ok} as LKTrackerInvoker computes them.
__device__ __forceinline__ void st_level_table(float *lv, unsigned a11, int s12, unsigned a22, float c0, float c1,
                                               float c2, float c3, float c4, float c5, float c6, float c7, float c8,
                                               float c9, float c10, float c11, float c12, float c13, float c14,
                                               bool sse, int wh, float min_eig) {
    // a sum whose every term and every partial sum (in any order) is an
    // integer <= 2^24 is exact in float: its integer value; otherwise the
    // ordered chains, combined in the SSE2 build's order
    float s0 = c4, s1 = c9, s2 = c14;
    if (sse) {
        s0 = __fadd_rn(s0, __fadd_rn(__fadd_rn(__fadd_rn(c0, c1), c2), c3));
        s1 = __fadd_rn(s1, __fadd_rn(__fadd_rn(__fadd_rn(c5, c6), c7), c8));
        s2 = __fadd_rn(s2, __fadd_rn(__fadd_rn(__fadd_rn(c10, c11), c12), c13));
    }
    float A11 = a11 <= (unsigned)kExact ? (float)a11 : s0;
    float A12 = ((a11 + a22) >> 1) <= (unsigned)kExact ? (float)s12 : s1;
    float A22 = a22 <= (unsigned)kExact ? (float)a22 : s2;
    const float FLT_SCALE = 1.f / (1 << 20);
    A11 = __fmul_rn(A11, FLT_SCALE);
    A12 = __fmul_rn(A12, FLT_SCALE);
    A22 = __fmul_rn(A22, FLT_SCALE);
    const float D = __fsub_rn(__fmul_rn(A11, A22), __fmul_rn(A12, A12));
    const float dd = __fsub_rn(A11, A22);
    const float t = __fadd_rn(__fmul_rn(dd, dd), __fmul_rn(__fmul_rn(4.f, A12), A12));
    const float minEig = __fdiv_rn(__fsub_rn(__fadd_rn(A22, A11), sqrtf(t)), (float)(2 * wh));
    const bool ok = !(minEig < min_eig || D < FLT_EPSILON);
    lv[0] = A11;
    lv[1] = A12;
    lv[2] = A22;
    lv[3] = ok ? __fdiv_rn(1.f, D) : 0.f;
    lv[4] = minEig;
    lv[5] = ok ? 1.f : 0.f;
}

// Diagnostic stamps of the single-tile kernel (PSN_LK_STAMPS): 60 start, 50
// prologue landed, 51 Scharr of all levels, 52 A products + reduction, 53
// solver table; per level L*10+0 start, +1 J staged, +2 window loaded, +7
// iterations done, +8 iteration count; 40..45 accumulated iteration phases.
template <int NT, int EPT, int E, int OCC = 1>
__global__ __launch_bounds__(NT, OCC) void lk_kernel_st(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = blockIdx.x;
    if (A.poison_lds) lds_poison<NT>(smem, A.poison_lds);
    if (A.pyr_ntiles > 0 && g >= A.lk_wgs) {  // fused-build helper: tiles only
        pyr_tail<NT>(A, smem);
        return;
    }
    int qi = 0;
    while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
    const LkQueryDev &Q = A.q[qi];
    const int pi = lk_query_point(Q, A.counts, A.count_stride, g);
    if (pi < 0) return;  // past the query's device count
    const int w = Q.win_w, h = Q.win_h, wh = w * h;
    const int maxL = Q.max_level, nlev = maxL + 1;
    const int flags = Q.flags;
    const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
    const int JRW = st_jreg_w(w), JRH = st_jreg_h(h);
    const int PW = w + 3, DW = w + 1;
    const int RS = lk_pat_rs(w);  // I patch row stride (bytes)

    // overlapped A phase (one-wave builds at two workgroups per CU): the prologue
    // computes the coarsest level only; waves 1-3 compute the finer levels while
    // wave 0 iterates (the per-level barriers order their tables before use)
    // (not the 4-row build: its VGPRs would pass 170, one workgroup less per CU)
    const bool ovl = E > 4 && OCC == 1 && Q.st_ovl != 0;
    const int lo = ovl ? maxL : 0;  // the prologue's levels: lo..maxL
    const LkStLayout lay(w, h, sse, nlev, E > 0, ovl);
    int *RI = (int *)(smem + lay.ri);
    float *LV = (float *)(smem + lay.lv);
    uint32_t *JP = (uint32_t *)(smem + lay.jp);
    float *R = (float *)(smem + lay.r);    // b chain planes / err row (iterations)
    float *RA = (float *)(smem + lay.ra);  // A-phase chain planes (prologue; == R outside the one-wave layout)
    const ChainGeo GA = chain_geo_A(w, h, sse), GB = chain_geo_B(w, h, sse);

    // ---- per-thread window pixels (fixed for the whole kernel). Idle lanes
    // (pixel index >= w*h) read pixel 0, carry zero gradients and write their
    // zero products into a pad slot of the chain planes: branch-free loops.
    int ofsJ[EPT], ofsP[EPT], ofsD[EPT], posA_[EPT], posB_[EPT], ofsE[EPT], pix[EPT];
    bool ev[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
        const int idx = tid + k * NT;
        ev[k] = idx < wh;
        const int i = ev[k] ? idx : 0;
        const int y = qdiv(i, Q.dv_w), x = i - y * w;
        pix[k] = i;
        ofsJ[k] = y * JRW + x;
        ofsP[k] = (y + 1) * RS + x + 1;
        ofsD[k] = y * DW + x;
        posA_[k] = ev[k] ? posA(GA, y, x) : 4 * GA.S + GA.lenT;
        posB_[k] = ev[k] ? posB(GB, y, x) : 4 * GB.S + GB.lenT;
        ofsE[k] = ev[k] ? idx : round16i(wh);  // err plane (row-major): idle lanes write past the end
    }

    // the point's waves outrank fused pyramid-tile waves sharing their SIMDs
    if (A.pyr_ntiles > 0) __builtin_amdgcn_s_setprio(2);
    // ---- prologue: zero the A planes' chain padding (ordered by the barrier
    // after the DMA); level geometry comes from the kernel arguments ----
    zero_pads<NT>(RA, GA, 3 * nlev);
    const JWalk wk_int = jwalk_t(tid, JRW >> 2, NT, Q.dv_jrw4), wk_bord = jwalk_t(tid, JRW, NT, Q.dv_jrw);  // J staging walks
    LK_STAMP(60);

    const float hwx = __fmul_rn((float)(w - 1), 0.5f), hwy = __fmul_rn((float)(h - 1), 0.5f);
    const float px0 = A.prev[2 * pi], py0 = A.prev[2 * pi + 1];
    float NPx = 0.f, NPy = 0.f;
    if (flags & PSN_LK_USE_INITIAL_FLOW) {
        NPx = A.next[2 * pi];
        NPy = A.next[2 * pi + 1];
    }
#ifdef PSN_LK_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // point landed
    LK_STAMP(58);
#endif

    // ---- the I patch of every level by LDS-DMA; the coarsest J region into registers ----
#pragma unroll
    for (int l = 0; l < kStMaxLev; l++) {
        if (l > maxL) break;
        if (l < lo) continue;
        const LevelDev I = ring_level(A.ring, Q.prev_slot, l);
        const IGeo gg = i_geo(px0, py0, hwx, hwy, l, w, h, I.w, I.h);
        if (!gg.valid) continue;
        dma_patch<NT>(smem + lay.pim + l * lay.pim_stride, I, gg.ipy - 1, gg.ipx - 1, PW, h + 3, lk_pat_m(w), Q.dv_pm);
    }
    LK_STAMP(62);
    // level table for the level loops (ordered by the barrier below)
    int *TBL = (int *)(smem + lay.tbl);
    if (tid < 2 * kStMaxLev) {
        const int ts = tid >= kStMaxLev ? 1 : 0, tl = tid - ts * kStMaxLev;
        LevelDev L = ring_level(A.ring, ts ? Q.next_slot : Q.prev_slot, 0);
#pragma unroll
        for (int l = 1; l < kStMaxLev; l++)
            if (tl == l) L = ring_level(A.ring, ts ? Q.next_slot : Q.prev_slot, l);
        tbl_put(TBL, ts, tl, L);
    }
    LK_STAMP(63);
    JPStage<NT> pf;  // prefetched J region of level pf_level at (pf_y0, pf_x0)
    int pf_level, pf_x0, pf_y0;
    {
        const float sc = ldexpf(1.f, -maxL);
        const float nx0 = (flags & PSN_LK_USE_INITIAL_FLOW) ? __fmul_rn(NPx, sc) : __fmul_rn(px0, sc);
        const float ny0 = (flags & PSN_LK_USE_INITIAL_FLOW) ? __fmul_rn(NPy, sc) : __fmul_rn(py0, sc);
        pf_x0 = (cv_floor(__fsub_rn(nx0, hwx)) - kStJMargin) & ~3;
        pf_y0 = cv_floor(__fsub_rn(ny0, hwy)) - kStJMargin;
        pf_level = maxL;
        pf.load(ring_level_u(A.ring, Q.next_slot, maxL), pf_y0, pf_x0, JRW, JRH, wk_int, wk_bord);
    }
    LK_STAMP(59);
    dma_wait();
    __syncthreads();
    LK_STAMP(50);

    // ---- A phase for ALL levels at once (the I window does not depend on the
    // flow): Scharr of every patch; window values, tensor products and sums;
    // one reduction barrier; wave 0 sums the float chains of every level in
    // parallel lanes and writes the per-level solver table LV ----
#pragma unroll
    for (int l = 0; l < kStMaxLev; l++) {
        if (l > maxL) break;
        if (l < lo) continue;
        const LevelDev I = ring_level(A.ring, Q.prev_slot, l);
        const IGeo gg = i_geo(px0, py0, hwx, hwy, l, w, h, I.w, I.h);
        if (!gg.valid) continue;
        const uint8_t *P = smem + lay.pim + l * lay.pim_stride + ((gg.ipx - 1) & 3);
        short2 *Dg = (short2 *)(smem + lay.dg + l * lay.dg_stride);
        Walk wk;
        wk.init_m(tid, NT, DW, Q.dv_dw);
        for (int idx = tid; idx < (h + 1) * DW; idx += NT, wk.step()) {
            const int gy = gg.ipy + wk.y, gx = gg.ipx + wk.x;
            short2 d = make_short2(0, 0);
            if ((unsigned)gy < (unsigned)I.h && (unsigned)gx < (unsigned)I.w) {
                const uint8_t *p = P + wk.y * RS + wk.x;
                const int a0 = p[0], a1 = p[1], a2 = p[2];
                const int b0 = p[RS], b2 = p[RS + 2];
                const int c0 = p[2 * RS], c1 = p[2 * RS + 1], c2 = p[2 * RS + 2];
                d.x = (short)(3 * (a2 + c2) + 10 * b2 - 3 * (a0 + c0) - 10 * b0);
                d.y = (short)(3 * ((c0 - a0) + (c2 - a2)) + 10 * (c1 - a1));
            }
            Dg[idx] = d;
        }
    }
    __syncthreads();
    LK_STAMP(51);
#pragma unroll
    for (int l = 0; l < kStMaxLev; l++) {
        if (l > maxL) break;
        if (l < lo) continue;
        const LevelDev I = ring_level(A.ring, Q.prev_slot, l);
        const IGeo gg = i_geo(px0, py0, hwx, hwy, l, w, h, I.w, I.h);
        // Per-sum exactness: A11 (terms >= 0) is exact when s11 <= 2^24, A22 when
        // s22 <= 2^24, A12 when sum|xy| <= (s11 + s22) / 2 <= 2^24; s11 and s22
        // are reduced saturating, s12 wrapping
        unsigned s11 = 0, s22 = 0;
        int s12 = 0;
        if (gg.valid) {
            const uint8_t *P = smem + lay.pim + l * lay.pim_stride + ((gg.ipx - 1) & 3);
            const short2 *Dg = (const short2 *)(smem + lay.dg + l * lay.dg_stride);
            int2 *IW = (int2 *)(smem + lay.iw + l * lay.iw_stride);
            float *PA = RA + l * 3 * GA.P;
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint8_t *p = P + ofsP[k];
                const int iw = PSN_DESCALE(__mul24((int)p[0], gg.w00) + __mul24((int)p[1], gg.w01) +
                                               __mul24((int)p[RS], gg.w10) + __mul24((int)p[RS + 1], gg.w11), 9);
                const short2 *d = Dg + ofsD[k];
                const short2 d00 = d[0], d01 = d[1], d10 = d[DW], d11 = d[DW + 1];
                int ix = PSN_DESCALE(__mul24((int)d00.x, gg.w00) + __mul24((int)d01.x, gg.w01) +
                                         __mul24((int)d10.x, gg.w10) + __mul24((int)d11.x, gg.w11), 14);
                int iy = PSN_DESCALE(__mul24((int)d00.y, gg.w00) + __mul24((int)d01.y, gg.w01) +
                                         __mul24((int)d10.y, gg.w10) + __mul24((int)d11.y, gg.w11), 14);
                if (ev[k]) IW[pix[k]] = make_int2(iw, (ix & 0xffff) | (iy << 16));
                ix = ev[k] ? ix : 0;
                iy = ev[k] ? iy : 0;
                const int xx2 = __mul24(ix, ix), xy = __mul24(ix, iy), yy2 = __mul24(iy, iy);
                PA[posA_[k]] = (float)xx2;
                PA[GA.P + posA_[k]] = (float)xy;
                PA[2 * GA.P + posA_[k]] = (float)yy2;
                s11 += (unsigned)xx2;  // per thread <= 4 * 4080^2 < 2^30
                s12 += xy;
                s22 += (unsigned)yy2;
            }
        }
        s11 = wave_sum_sat(s11);
        s12 = wave_sum(s12);
        s22 = wave_sum_sat(s22);
        if (lane == 0) {
            int *ra = RI + kStRiA + l * 4 * 8 + wid;
            ra[0] = (int)s11;
            ra[8] = s12;
            ra[16] = (int)s22;
        }
    }
    __syncthreads();
    LK_STAMP(52);
    if (wid == 0) {
        float *CH = (float *)RI;  // 15 chain results per level (the iteration scratch is still unused)
        // chain pass: slot q -> (level q/15, sum (q%15)/5, chain q%5); two slots per lane
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const int q = lane + 64 * half;
            const int l = q / 15, r = q - 15 * (q / 15);
            if (l <= maxL && l >= lo) {
                unsigned a11 = 0, a22 = 0;
#pragma unroll
                for (int ww = 0; ww < NW; ww++) {
                    a11 = sat_add(a11, (unsigned)RI[kStRiA + l * 32 + ww]);
                    a22 = sat_add(a22, (unsigned)RI[kStRiA + l * 32 + 16 + ww]);
                }
                const int s = r / 5, ch = r - 5 * (r / 5);
                const unsigned bound = s == 0 ? a11 : s == 2 ? a22 : (a11 + a22) >> 1;
                float acc = 0.f;
                if (bound > (unsigned)kExact) {
                    const int base = (l * 3 + s) * GA.P + (ch < 4 ? ch * GA.S : 4 * GA.S);
                    const int nb = (ch < 4 ? GA.S : GA.T) >> 4;
                    acc = chain_sum16(RA + base, nb);
                }
                CH[q] = acc;
            }
        }
        // CH written by other lanes of this wave: LDS executes a wave's accesses in
        // order; the clobber keeps the compiler from hoisting the reads
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane <= maxL && lane >= lo) {
            const int l = lane;
            unsigned a11 = 0, a22 = 0;
            int s12 = 0;
#pragma unroll
            for (int ww = 0; ww < NW; ww++) {
                const int *ra = RI + kStRiA + l * 32 + ww;
                a11 = sat_add(a11, (unsigned)ra[0]);
                s12 += ra[8];
                a22 = sat_add(a22, (unsigned)ra[16]);
            }
            const float *c = CH + l * 15;
            st_level_table(LV + l * kStLvFloats, a11, s12, a22, c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8],
                           c[9], c[10], c[11], c[12], c[13], c[14], sse, wh, Q.min_eig);
        }
    }
    __syncthreads();  // LV published; the A planes in R are dead from here
    LK_STAMP(53);
    zero_pads<NT>(R, GB, 4);  // b planes (2 buffers x 2 sums) now own R; ordered by the first iteration's barrier

    int status = 1;
    float errv = 0.f;
    const float FLT_SCALE = 1.f / (1 << 20);
#ifdef PSN_LK_STAMPS
    unsigned long long acc_ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_ph = 0;
// ordered stamps: every earlier instruction has issued and every LDS access landed
#define PH_STAMP(t) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory")
#define PH_BEGIN() PH_STAMP(t_ph)
#define PH_MARK(i)                                                  \
    do {                                                            \
        unsigned long long t_;                                      \
        PH_STAMP(t_);                                               \
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
    int jr_x0 = 0, jr_y0 = 0;

    if constexpr (E > 0) {
        // ---- one-wave iterations: wave 0 runs the LK iterations of every level
        // with no workgroup barrier inside the loop; waves 1..NW-1 meanwhile
        // stage the next level's J region (predicted start) into the other
        // half of the double-buffered, column-major J region. ----
        const int JRHc = st_jrh_cm(h);
        uint32_t *const JPB0 = JP, *const JPB1 = JP + st_jp_cm_dw(w, h);
        // lane -> (window column, row group): columns sorted by SSE2 chain class
        // (class c < 4: x = c, c+4, ... < n8; class 4 = the scalar tail)
        const int G = Q.ow_g, RG = Q.ow_rg;
        const int n8 = sse ? (w / 8) * 8 : 0, cw = n8 / 4;
        const int cr = qdiv(lane, Q.dv_g), gi = lane - cr * G;
        const bool lane_on = cr < w;
        const int ccl = qdiv(cr, sse ? Q.dv_cw : 0u);  // chain class of an SSE2 column
        const int colx = !lane_on ? 0 : (cr < n8 ? ccl + 4 * (cr - ccl * cw) : cr);
        const int oy0 = gi * RG;
        const int lane_off = colx * JRHc + oy0;
        // class c occupies lanes (last[c-1], last[c]]; empty classes repeat the previous bound
        const int last4 = w * G - 1;
        // this lane ends class cls_end (it publishes the class's scans), or -1; with
        // no tail columns (w % 8 == 0) the last lane ends class 3 and the empty class
        // 4 alike and publishes both (class 4's sums are then 0)
        int cls_end = -1;
        bool end3 = false;
        if (lane == last4) {
            cls_end = 4;
            end3 = n8 > 0 && n8 == w;
        }
        if (n8 > 0)
            for (int c = 0; c < 4; c++)
                if (lane == (c + 1) * cw * G - 1 && lane != last4) cls_end = c;
        int4 *CSX = (int4 *)(RI + kStRiIt + 16);  // 5 x int4 class scans
        if (n8 == 0 && tid < 4) CSX[tid] = make_int4(0, 0, 0, 0);  // ordered by the first level barrier
        // loop constants pinned in registers (not re-read from the kernel arguments)
        double eps2 = Q.eps2;
        int maxc = Q.max_count;
        asm volatile("" : "+v"(eps2), "+s"(maxc));
        const int th = max(tid - 64, 0);
        const JWalk wkh_int = jwalk_t(th, JRW >> 2, NT - 64, Q.dv_jrw4), wkh_bord = jwalk_t(th, JRW, NT - 64, Q.dv_jrw);
        const JWalk wk0_int = jwalk_t(lane, JRW >> 2, 64, Q.dv_jrw4), wk0_bord = jwalk_t(lane, JRW, 64, Q.dv_jrw);
        pf.cs = JRHc;
        // overlapped A phase of level l by ONE wave (no barrier: a wave's LDS
        // accesses complete in order): I patch by LDS-DMA, Scharr plane, window
        // values and A products, the 15 ordered chains when a sum is inexact, and
        // the level's solver table -- the prologue's arithmetic, one wave wide
        auto a_level_wave = [&](int l) {
            const LevelDev I = tbl_get(TBL, 0, l);
            const IGeo gg = i_geo(px0, py0, hwx, hwy, l, w, h, I.w, I.h);
            if (!gg.valid) return;
            uint8_t *const pim = smem + lay.pim + l * lay.pim_stride;
            dma_patch_t<64>(pim, I, gg.ipy - 1, gg.ipx - 1, PW, h + 3, lk_pat_m(w), Q.dv_pm, lane);
            dma_wait();
            const uint8_t *P = pim + ((gg.ipx - 1) & 3);
            short2 *Dg = (short2 *)(smem + lay.dg + l * lay.dg_stride);
            {
                Walk wk;
                wk.init_m(lane, 64, DW, Q.dv_dw);
                for (int idx = lane; idx < (h + 1) * DW; idx += 64, wk.step()) {
                    const int gy = gg.ipy + wk.y, gx = gg.ipx + wk.x;
                    short2 d = make_short2(0, 0);
                    if ((unsigned)gy < (unsigned)I.h && (unsigned)gx < (unsigned)I.w) {
                        const uint8_t *p = P + wk.y * RS + wk.x;
                        const int a0 = p[0], a1 = p[1], a2 = p[2];
                        const int b0 = p[RS], b2 = p[RS + 2];
                        const int c0 = p[2 * RS], c1 = p[2 * RS + 1], c2 = p[2 * RS + 2];
                        d.x = (short)(3 * (a2 + c2) + 10 * b2 - 3 * (a0 + c0) - 10 * b0);
                        d.y = (short)(3 * ((c0 - a0) + (c2 - a2)) + 10 * (c1 - a1));
                    }
                    Dg[idx] = d;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            int2 *IW = (int2 *)(smem + lay.iw + l * lay.iw_stride);
            float *PA = RA + l * 3 * GA.P;
            unsigned s11 = 0, s22 = 0;  // per lane <= 16 * 4080^2 < 2^30
            int s12 = 0;
            for (int i0 = 0; i0 < wh; i0 += 64) {
                const int idx = i0 + lane;
                const bool v = idx < wh;
                const int i = v ? idx : 0;
                const int y = qdiv(i, Q.dv_w), x = i - y * w;
                const uint8_t *p = P + (y + 1) * RS + x + 1;
                const int iw = PSN_DESCALE(__mul24((int)p[0], gg.w00) + __mul24((int)p[1], gg.w01) +
                                               __mul24((int)p[RS], gg.w10) + __mul24((int)p[RS + 1], gg.w11), 9);
                const short2 *d = Dg + y * DW + x;
                const short2 d00 = d[0], d01 = d[1], d10 = d[DW], d11 = d[DW + 1];
                int ix = PSN_DESCALE(__mul24((int)d00.x, gg.w00) + __mul24((int)d01.x, gg.w01) +
                                         __mul24((int)d10.x, gg.w10) + __mul24((int)d11.x, gg.w11), 14);
                int iy = PSN_DESCALE(__mul24((int)d00.y, gg.w00) + __mul24((int)d01.y, gg.w01) +
                                         __mul24((int)d10.y, gg.w10) + __mul24((int)d11.y, gg.w11), 14);
                if (v) IW[i] = make_int2(iw, (ix & 0xffff) | (iy << 16));
                ix = v ? ix : 0;
                iy = v ? iy : 0;
                const int xx2 = __mul24(ix, ix), xy = __mul24(ix, iy), yy2 = __mul24(iy, iy);
                const int pos = v ? posA(GA, y, x) : 4 * GA.S + GA.lenT;
                PA[pos] = (float)xx2;
                PA[GA.P + pos] = (float)xy;
                PA[2 * GA.P + pos] = (float)yy2;
                s11 += (unsigned)xx2;
                s12 += xy;
                s22 += (unsigned)yy2;
            }
            s11 = wave_sum_sat(s11);
            s12 = wave_sum(s12);
            s22 = wave_sum_sat(s22);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float acc = 0.f;
            if (lane < 15) {
                const int sm = lane / 5, ch = lane - 5 * sm;
                const unsigned bound = sm == 0 ? s11 : sm == 2 ? s22 : (s11 + s22) >> 1;
                if (bound > (unsigned)kExact) {
                    const int base = sm * GA.P + (ch < 4 ? ch * GA.S : 4 * GA.S);
                    acc = chain_sum16(PA + base, (ch < 4 ? GA.S : GA.T) >> 4);
                }
            }
            float c[15];
#pragma unroll
            for (int k = 0; k < 15; k++) c[k] = readlane_f(acc, k);
            if (lane == 0)
                st_level_table(LV + l * kStLvFloats, s11, s12, s22, c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7],
                               c[8], c[9], c[10], c[11], c[12], c[13], c[14], sse, wh, Q.min_eig);
        };
        LK_STAMP(54);
        bool pf_regs = true;  // the prefetched region is still in registers (prologue) vs already in LDS
        int buf = 0;
        float *XCH = (float *)(RI + kStRiIt);  // wave 0 -> all: NPx, NPy at the end of a level

        for (int level = maxL; level >= 0; level--) {
            LK_STAMP(level * 10 + 0);
            const LevelDev I = tbl_get(TBL, 0, level);
            const LevelDev J = tbl_get(TBL, 1, level);
            const int cols = I.w, rows = I.h;
            const float scale = ldexpf(1.f, -level);
            float nx, ny;
            if (level == maxL) {
                if (flags & PSN_LK_USE_INITIAL_FLOW) {
                    nx = __fmul_rn(NPx, scale);
                    ny = __fmul_rn(NPy, scale);
                } else {
                    nx = __fmul_rn(px0, scale);
                    ny = __fmul_rn(py0, scale);
                }
            } else {
                nx = __fmul_rn(NPx, 2.f);
                ny = __fmul_rn(NPy, 2.f);
            }
            NPx = nx;
            NPy = ny;
            const IGeo gg = i_geo(px0, py0, hwx, hwy, level, w, h, cols, rows);
            const float *lv = LV + level * kStLvFloats;
            const bool run = gg.valid && lv[5] != 0.f;
            if (!gg.valid) {
                if (level == 0) {
                    status = 0;
                    errv = 0.f;
                }
            } else {
                if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = lv[4];
                if (!run && level == 0) status = 0;
            }
            nx = __fsub_rn(nx, hwx);
            ny = __fsub_rn(ny, hwy);
            uint32_t *const JC = buf ? JPB1 : JPB0;
            if (run) {
                const int inx0 = __builtin_amdgcn_readfirstlane(cv_floor(nx));
                const int iny0 = __builtin_amdgcn_readfirstlane(cv_floor(ny));
                if (pf_level == level && inx0 >= pf_x0 && iny0 >= pf_y0 && inx0 + w + 1 <= pf_x0 + JRW &&
                    iny0 + h + 1 <= pf_y0 + JRH) {
                    if (pf_regs) {
                        LK_STAMP(55);
                        pf.store(JC);
                        LK_STAMP(56);
                    }
                    jr_x0 = pf_x0;
                    jr_y0 = pf_y0;
                } else {
                    JPStage<NT> cp;
                    cp.cs = JRHc;
                    jr_x0 = (inx0 - kStJMargin) & ~3;
                    jr_y0 = iny0 - kStJMargin;
                    cp.copy(JC, J, jr_y0, jr_x0, JRW, JRH, wk_int, wk_bord);
                }
            }
            pf_regs = false;
            __syncthreads();  // JC complete; every wave is past the previous level
            LK_STAMP(level * 10 + 1);
            // next level's region at its predicted start (2 x this start)
            pf_level = level > 0 ? level - 1 : -1;
            pf_x0 = __builtin_amdgcn_readfirstlane((cv_floor(__fsub_rn(__fmul_rn(NPx, 2.f), hwx)) - kStJMargin) & ~3);
            pf_y0 = __builtin_amdgcn_readfirstlane(cv_floor(__fsub_rn(__fmul_rn(NPy, 2.f), hwy)) - kStJMargin);

            if (wid != 0) {
                if (ovl && level == maxL) {  // the finer levels' A phase: wave k takes levels maxL - k, maxL - k - 3, ...
                    for (int l = maxL - wid; l >= 0; l -= NW - 1) a_level_wave(l);
#ifdef PSN_LK_STAMPS
                    unsigned long long t_s;  // wave k's A phase done: slot 59 - 10 k
                    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_s) : : "memory");
                    if (lane == 0 && wid < 4 && A.stamps) A.stamps[(size_t)blockIdx.x * 64 + 59 - 10 * wid] = t_s;
#endif
                }
                if (level > 0) {
                    JPStage<NT> cp;
                    cp.cs = JRHc;
                    cp.copy(buf ? JPB0 : JPB1, tbl_get(TBL, 1, level - 1), pf_y0, pf_x0, JRW, JRH,
                            wkh_int, wkh_bord);
                }
            } else if (run) {
                const float A11 = lv[0], A12 = lv[1], A22 = lv[2], D = lv[3];
                // the lane's window rows, two rows per dword (int16 halves): I, Ix,
                // Iy, |Ix| + |Iy|; rows past the window carry zero gradients
                constexpr int E2 = (E + 1) / 2;
                unsigned IxP[E2], IyP[E2], AxP[E2], AyP[E2];
                int Cw[2 * E2];  // 256 - 512 * I: the bilinear sum plus Cw, >> 9, is J* - I*
                int Iw_[E];
                {
                    const int2 *IW = (const int2 *)(smem + lay.iw + level * lay.iw_stride);
                    int iw[2 * E2], ix[2 * E2], iy[2 * E2];
#pragma unroll
                    for (int k = 0; k < 2 * E2; k++) {
                        const int y = oy0 + k;
                        const bool v = k < E && lane_on && k < RG && y < h;
                        const int2 t = IW[v ? y * w + colx : 0];
                        iw[k] = k < E ? t.x : 0;
                        ix[k] = v ? (int)(short)(t.y & 0xffff) : 0;
                        iy[k] = v ? (t.y >> 16) : 0;
                        if (k < E) Iw_[k] = t.x;
                    }
#pragma unroll
                    for (int q = 0; q < E2; q++) {
                        Cw[2 * q] = 256 - 512 * iw[2 * q];
                        Cw[2 * q + 1] = 256 - 512 * iw[2 * q + 1];
                        IxP[q] = pack_w(ix[2 * q], ix[2 * q + 1]);
                        IyP[q] = pack_w(iy[2 * q], iy[2 * q + 1]);
                        AxP[q] = pack_w(abs(ix[2 * q]), abs(ix[2 * q + 1]));
                        AyP[q] = pack_w(abs(iy[2 * q]), abs(iy[2 * q + 1]));
                    }
                }
                LK_STAMP(level * 10 + 2);
                float pdx = 0.f, pdy = 0.f;
                int jdone = 0;
                unsigned dP[E2];
                // diffs J - I of the lane's rows at offset (ox, oy) of the region
                // (packed pairs into dP) and the lane's s1, s2, sum|t1|, sum|t2|
                auto products = [&](int ox, int oy, unsigned W0, unsigned W1, int &s1, int &s2, unsigned &a,
                                    unsigned &a2) {
                    const uint32_t *jb = JC + __mul24(ox, JRHc) + oy + lane_off;
                    unsigned rr[2 * E2 + 1];
#pragma unroll
                    for (int k = 0; k <= 2 * E2; k++) rr[k] = jb[k];
                    s1 = 0;
                    s2 = 0;
                    a = 0;
                    a2 = 0;
#pragma unroll
                    for (int q = 0; q < E2; q++) {
                        // (sum + 256) >> 9 - I == (sum + 256 - 512 I) >> 9: the diffs directly
                        const int d0 = sdot2v(rr[2 * q + 1], W1, sdot2v(rr[2 * q], W0, Cw[2 * q])) >> 9;
                        const int d1 = sdot2v(rr[2 * q + 2], W1, sdot2v(rr[2 * q + 1], W0, Cw[2 * q + 1])) >> 9;
                        const s16x2 d = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((unsigned)d1, (unsigned)d0, 0x05040100u));
                        dP[q] = __builtin_bit_cast(unsigned, d);
                        s1 = sdot2(dP[q], IxP[q], s1);
                        s2 = sdot2(dP[q], IyP[q], s2);
                        const s16x2 ad = __builtin_elementwise_max(d, (s16x2)0 - d);
                        a = udot2(__builtin_bit_cast(unsigned, ad), AxP[q], a);  // per lane < 2^29
                        a2 = udot2(__builtin_bit_cast(unsigned, ad), AyP[q], a2);
                    }
                };
                for (int j = 0; j < maxc; j++) {
                    jdone = j + 1;
                    PH_BEGIN();
                    const int inx = cv_floor(nx), iny = cv_floor(ny);
                    int iw00, iw01, iw10, iw11;
                    bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), iw00, iw01, iw10, iw11);
                    const unsigned W0 = pack_w(iw00, iw01), W1 = pack_w(iw10, iw11);
                    // speculative: the offsets are clamped into the region, the
                    // bounds / region tests below decide whether the sums count
                    const int ox = min(max(inx - jr_x0, 0), JRW - w - 1), oy = min(max(iny - jr_y0, 0), JRH - h - 1);
                    int s1, s2;
                    unsigned a, a2;
                    products(ox, oy, W0, W1, s1, s2, a, a2);
                    int sinx = __builtin_amdgcn_readfirstlane(inx), siny = __builtin_amdgcn_readfirstlane(iny);
                    // keep the (rarely taken) branches below the products: the
                    // conditions formally depend on them
                    asm volatile("; order %2 %3 %4 %5" : "+s"(sinx), "+s"(siny) : "v"(s1), "v"(s2), "v"(a), "v"(a2));
                    if (sinx < -w || sinx >= cols || siny < -h || siny >= rows) {
                        if (level == 0) status = 0;
                        break;
                    }
                    if (!(sinx >= jr_x0 && siny >= jr_y0 && sinx + w + 1 <= jr_x0 + JRW && siny + h + 1 <= jr_y0 + JRH)) {
                        // restage by this wave alone (the other waves never read JC)
                        JPStage<NT> cp;
                        cp.cs = JRHc;
                        jr_x0 = __builtin_amdgcn_readfirstlane((sinx - kStJMargin) & ~3);
                        jr_y0 = __builtin_amdgcn_readfirstlane(siny - kStJMargin);
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        cp.copy(JC, J, jr_y0, jr_x0, JRW, JRH, wk0_int, wk0_bord);
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        products(sinx - jr_x0, siny - jr_y0, W0, W1, s1, s2, a, a2);
                        PH_COUNT(5);
                    }
                    PH_MARK(0);
                    const int l1 = s1, l2 = s2;  // the lane's own sums (class path)
                    const unsigned la1 = a, la2 = a2;
                    wave_sum4(s1, s2, a, a2);
                    PH_MARK(1);
                    float b1, b2;
                    if (sums_exact(a, s1) && sums_exact(a2, s2)) {
                        // every partial sum in any order is an integer of magnitude <= 2^24
                        b1 = (float)s1;
                        b2 = (float)s2;
                    } else {
                        PH_COUNT(6);
                        // per SSE2 chain class: inclusive scans of the lanes' sums and
                        // of sum|t1|, sum|t2|; class-end lanes publish to LDS
                        unsigned a1 = min(la1, (1u << 25) + 1u);  // a clamped lane fails its class
                        a2 = min(la2, (1u << 25) + 1u);
                        const int c1 = wave_scan(l1), c2 = wave_scan(l2);
                        a1 = (unsigned)wave_scan((int)a1);
                        a2 = (unsigned)wave_scan((int)a2);
                        if (cls_end >= 0) CSX[cls_end] = make_int4(c1, c2, (int)a1, (int)a2);
                        if (end3) CSX[3] = make_int4(c1, c2, (int)a1, (int)a2);
                        int S1[5], S2[5];
                        bool exact = true;
                        int4 pv = make_int4(0, 0, 0, 0);
#pragma unroll
                        for (int c = 0; c < 5; c++) {
                            const int4 cv = CSX[c];  // classes 0-3 stay zero without SSE2 lanes
                            S1[c] = cv.x - pv.x;     // wrapping: exact whenever the class passes
                            S2[c] = cv.y - pv.y;
                            exact = exact && sums_exact((unsigned)(cv.z - pv.z), S1[c]) &&
                                    sums_exact((unsigned)(cv.w - pv.w), S2[c]);
                            pv = cv;
                        }
                        if (exact) {
                            // every chain's partial sums are integers <= 2^24: each chain
                            // sum is its integer sum; combine in the SSE2 build's order
                            b1 = (float)S1[4];
                            b2 = (float)S2[4];
                            if (sse) {
                                b1 = __fadd_rn(b1, __fadd_rn(__fadd_rn((float)S1[0], (float)S1[2]),
                                                             __fadd_rn((float)S1[1], (float)S1[3])));
                                b2 = __fadd_rn(b2, __fadd_rn(__fadd_rn((float)S2[0], (float)S2[2]),
                                                             __fadd_rn((float)S2[1], (float)S2[3])));
                            }
                        } else {
                            // ordered float chains: products chain-major into R, one lane per chain
#pragma unroll
                            for (int k = 0; k < E; k++) {
                                const int y = oy0 + k;
                                if (lane_on && k < RG && y < h) {
                                    const int d = (int)(short)(k & 1 ? dP[k >> 1] >> 16 : dP[k >> 1] & 0xffff);
                                    const int gx = (int)(short)(k & 1 ? IxP[k >> 1] >> 16 : IxP[k >> 1] & 0xffff);
                                    const int gy = (int)(short)(k & 1 ? IyP[k >> 1] >> 16 : IyP[k >> 1] & 0xffff);
                                    const int pos = posB(GB, y, colx);
                                    R[pos] = (float)__mul24(d, gx);
                                    R[GB.P + pos] = (float)__mul24(d, gy);
                                }
                            }
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            float acc = 0.f;
                            if (lane < 10) {
                                const int ch = lane % 5, s = lane / 5;
                                const int base = s * GB.P + (ch < 4 ? ch * GB.S : 4 * GB.S);
                                const int nb = (ch < 4 ? GB.S : GB.T) >> 4;
                                acc = chain_sum16(R + base, nb);
                            }
                            b1 = readlane_f(acc, 4);
                            b2 = readlane_f(acc, 9);
                            if (sse) {
                                const float bb0 = __fadd_rn(readlane_f(acc, 0), readlane_f(acc, 2));
                                const float bb2 = __fadd_rn(readlane_f(acc, 1), readlane_f(acc, 3));
                                const float bb1 = __fadd_rn(readlane_f(acc, 5), readlane_f(acc, 7));
                                const float bb3 = __fadd_rn(readlane_f(acc, 6), readlane_f(acc, 8));
                                b1 = __fadd_rn(b1, __fadd_rn(bb0, bb2));
                                b2 = __fadd_rn(b2, __fadd_rn(bb1, bb3));
                            }
                            PH_COUNT(4);
                        }
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // CSX / R reads done before the next writes
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
                    if (dd <= eps2) break;
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
                    } else {
                        int iw00, iw01, iw10, iw11;
                        bilin_weights(__fsub_rn(qx, (float)iqx), __fsub_rn(qy, (float)iqy), iw00, iw01, iw10, iw11);
                        if (!(iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                            JPStage<NT> cp;
                            cp.cs = JRHc;
                            jr_x0 = (iqx - kStJMargin) & ~3;
                            jr_y0 = iqy - kStJMargin;
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            cp.copy(JC, J, jr_y0, jr_x0, JRW, JRH, wk0_int, wk0_bord);
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        }
                        const unsigned W0 = pack_w(iw00, iw01), W1 = pack_w(iw10, iw11);
                        const uint32_t *jb = JC + (iqx - jr_x0) * JRHc + (iqy - jr_y0) + lane_off;
                        unsigned ea = 0;
                        int ad[E];
#pragma unroll
                        for (int k = 0; k < E; k++) {
                            const int jv = sdot2(jb[k + 1], W1, sdot2(jb[k], W0, 1 << 8)) >> 9;
                            const int y = oy0 + k;
                            ad[k] = (lane_on && k < RG && y < h) ? abs(jv - Iw_[k]) : 0;
                            ea += (unsigned)ad[k];
                        }
                        ea = (unsigned)__builtin_amdgcn_readlane(wave_scan((int)ea), 63);
                        float errval;
                        if (ea <= (unsigned)kExact) {
                            errval = (float)ea;  // every partial sum of errval += |diff| is an exact integer
                        } else {  // row-major order, one lane
#pragma unroll
                            for (int k = 0; k < E; k++) {
                                const int y = oy0 + k;
                                if (lane_on && k < RG && y < h) R[y * w + colx] = (float)ad[k];
                            }
                            for (int k = wh + lane; k < round16i(wh); k += 64) R[k] = 0.f;
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            float acc = 0.f;
                            if (lane == 0) acc = chain_sum16(R, round16i(wh) >> 4);
                            errval = readlane_f(acc, 0);
                        }
                        errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * wh));
                    }
                }
            }
            if (tid == 0) {
                XCH[0] = NPx;
                XCH[1] = NPy;
            }
            __syncthreads();  // wave 0 done with JC; the next level's region staged
            NPx = XCH[0];
            NPy = XCH[1];
            buf ^= 1;
        }
    } else {
    for (int level = maxL; level >= 0; level--) {
        LK_STAMP(level * 10 + 0);
        const LevelDev I = tbl_get(TBL, 0, level);
        const LevelDev J = tbl_get(TBL, 1, level);
        const int cols = I.w, rows = I.h;
        const float scale = ldexpf(1.f, -level);
        float nx, ny;
        if (level == maxL) {
            if (flags & PSN_LK_USE_INITIAL_FLOW) {
                nx = __fmul_rn(NPx, scale);
                ny = __fmul_rn(NPy, scale);
            } else {
                nx = __fmul_rn(px0, scale);
                ny = __fmul_rn(py0, scale);
            }
        } else {
            nx = __fmul_rn(NPx, 2.f);
            ny = __fmul_rn(NPy, 2.f);
        }
        NPx = nx;
        NPy = ny;
        const IGeo gg = i_geo(px0, py0, hwx, hwy, level, w, h, cols, rows);
        const float *lv = LV + level * kStLvFloats;
        const bool run = gg.valid && lv[5] != 0.f;
        if (!gg.valid) {
            if (level == 0) {
                status = 0;
                errv = 0.f;
            }
        } else {
            if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = lv[4];
            if (!run && level == 0) status = 0;
        }
        nx = __fsub_rn(nx, hwx);
        ny = __fsub_rn(ny, hwy);
        if (run) {
            // this level's J region: the prefetched registers if they cover the start
            const int inx0 = cv_floor(nx), iny0 = cv_floor(ny);
            if (pf_level == level && inx0 >= pf_x0 && iny0 >= pf_y0 && inx0 + w + 1 <= pf_x0 + JRW &&
                iny0 + h + 1 <= pf_y0 + JRH) {
                pf.store(JP);
                jr_x0 = pf_x0;
                jr_y0 = pf_y0;
            } else {
                JPStage<NT> cp;
                jr_x0 = (inx0 - kStJMargin) & ~3;
                jr_y0 = iny0 - kStJMargin;
                cp.copy(JP, J, jr_y0, jr_x0, JRW, JRH, wk_int, wk_bord);
            }
        }
        pf_level = -1;
        if (level > 0) {  // prefetch the next level's region at its predicted start (2 x this start)
            pf_x0 = (cv_floor(__fsub_rn(__fmul_rn(NPx, 2.f), hwx)) - kStJMargin) & ~3;
            pf_y0 = cv_floor(__fsub_rn(__fmul_rn(NPy, 2.f), hwy)) - kStJMargin;
            pf_level = level - 1;
            pf.load(tbl_get(TBL, 1, level - 1), pf_y0, pf_x0, JRW, JRH, wk_int, wk_bord);
        }
        if (!run) continue;
        __syncthreads();  // JP published (every wave finished the previous level's reads)
        LK_STAMP(level * 10 + 1);

        const float A11 = lv[0], A12 = lv[1], A22 = lv[2], D = lv[3];
        int Iw_[EPT], Ix_[EPT], Iy_[EPT];
        unsigned Sxy[EPT];
        {
            const int2 *IW = (const int2 *)(smem + lay.iw + level * lay.iw_stride);
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const int2 t = IW[pix[k]];
                Iw_[k] = t.x;
                Ix_[k] = ev[k] ? (int)(short)(t.y & 0xffff) : 0;
                Iy_[k] = ev[k] ? (t.y >> 16) : 0;
                Sxy[k] = (unsigned)(abs(Ix_[k]) + abs(Iy_[k]));
            }
        }
        LK_STAMP(level * 10 + 2);
        float pdx = 0.f, pdy = 0.f;
        int jdone = 0;

        for (int j = 0; j < Q.max_count; j++) {
            jdone = j + 1;
            PH_BEGIN();
            const int inx = cv_floor(nx), iny = cv_floor(ny);
            if (inx < -w || inx >= cols || iny < -h || iny >= rows) {
                if (level == 0) status = 0;
                break;
            }
            int iw00, iw01, iw10, iw11;
            bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), iw00, iw01, iw10, iw11);
            if (!(inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW && iny + h + 1 <= jr_y0 + JRH)) {
                // every wave's JP reads of iteration j-1 precede that iteration's
                // barrier, which this wave has passed
                JPStage<NT> cp;
                jr_x0 = (inx - kStJMargin) & ~3;
                jr_y0 = iny - kStJMargin;
                cp.copy(JP, J, jr_y0, jr_x0, JRW, JRH, wk_int, wk_bord);
                __syncthreads();
                PH_COUNT(5);
            }
            const unsigned W0 = pack_w(iw00, iw01), W1 = pack_w(iw10, iw11);
            const uint32_t *jb = JP + (iny - jr_y0) * JRW + (inx - jr_x0);
            float *pb = R + (j & 1) * 2 * GB.P;
            int s1 = 0, s2 = 0;
            unsigned a = 0;
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint32_t *p = jb + ofsJ[k];
                const int jv = sdot2(p[JRW], W1, sdot2(p[0], W0, 1 << 8)) >> 9;
                const int diff = jv - Iw_[k];
                const int t1 = __mul24(diff, Ix_[k]), t2 = __mul24(diff, Iy_[k]);
                pb[posB_[k]] = (float)t1;
                pb[GB.P + posB_[k]] = (float)t2;
                s1 += t1;
                s2 += t2;
                a += (unsigned)__mul24(abs(diff), (int)Sxy[k]);  // |t1| + |t2| (both factors < 2^14); per thread < 2^30
            }
            PH_MARK(0);
            block_sums3<NT>(s1, s2, a, RI + kStRiIt + 32 * (j & 1));  // the iteration's barrier
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
            int iw00, iw01, iw10, iw11;
            bilin_weights(__fsub_rn(qx, (float)iqx), __fsub_rn(qy, (float)iqy), iw00, iw01, iw10, iw11);
            __syncthreads();  // every wave is done with R (last products) and JP
            if (!(iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                JPStage<NT> cp;
                jr_x0 = (iqx - kStJMargin) & ~3;
                jr_y0 = iqy - kStJMargin;
                cp.copy(JP, J, jr_y0, jr_x0, JRW, JRH, wk_int, wk_bord);
                __syncthreads();
            }
            const unsigned W0 = pack_w(iw00, iw01), W1 = pack_w(iw10, iw11);
            const uint32_t *jb = JP + (iqy - jr_y0) * JRW + (iqx - jr_x0);
            int e1 = 0, e2 = 0;
            unsigned ea = 0;
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint32_t *p = jb + ofsJ[k];
                const int jv = sdot2(p[JRW], W1, sdot2(p[0], W0, 1 << 8)) >> 9;
                const int ad = ev[k] ? abs(jv - Iw_[k]) : 0;
                R[ofsE[k]] = (float)ad;  // row-major, for the sequential fallback
                ea += (unsigned)ad;
            }
            for (int k = wh + tid; k < round16i(wh); k += NT) R[k] = 0.f;
            block_sums3<NT>(e1, e2, ea, RI + kStRiErr);
            float errval;
            if (ea <= (unsigned)kExact) {
                errval = (float)ea;  // every partial sum of errval += |diff| is an exact integer
            } else {
                float acc = 0.f;
                if (lane == 0) acc = chain_sum16(R, round16i(wh) >> 4);
                errval = readlane_f(acc, 0);
            }
            errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * wh));
        }
    }
    }  // legacy multi-wave iterations

    LK_STAMP(61);
#ifdef PSN_LK_STAMPS
    for (int i = 0; i < 8; i++) LK_COUNT(40 + i, acc_ph[i]);
#endif
    if (tid == 0) {
        A.next[2 * pi] = NPx;
        A.next[2 * pi + 1] = NPy;
        A.status[pi] = (uint8_t)status;
        if (A.err) A.err[pi] = errv;
    }
    if (A.pyr_ntiles > 0) pyr_tail<NT>(A, smem);
}
#undef PH_BEGIN
#undef PH_MARK
#undef PH_COUNT

// ---------------------------------------------------------------------------
// lk_kernel_bx -- box windows (Tracker2D: (int)box.w x (int)box.w backward,
// PSNWhere_Tracker2D.cpp:776-782; box w x h forward, :871-877) above the
// single-tile kernel's size. Workgroup = one point, 4 waves. The window is cut
// into units of 4 pixels (row y, quad q) in row-major order and thread t owns
// the CONTIGUOUS units [t*UPT, t*UPT + UPT): for every SSE2 lane chain (x & 3,
// pixels below the 8- resp. 4-pixel-step bound) and the scalar tail chain the
// thread's terms are one contiguous run of the chain, in chain order. Window
// values (256 - 512 I, Ix, Iy) stay in registers for the whole level; the I
// patch and the J region are LDS bytes (J pairs for the packed-dot bilinear are
// formed with v_perm from two dwords per row).
// Exactness of every float sum (A11, A12, A22 per level; b1, b2 per iteration),
// decided per chain: a run's total and its maximum / minimum prefix go through
// a block scan (DPP within a wave, one LDS record per wave, ONE barrier); when
// every prefix of every chain is an integer of magnitude <= 2^24 and every term
// is exact, each chain's float sum IS its integer sum and the chains combine in
// float in the SSE2 build's order. Otherwise the ordered float chains: terms
// chain-major into LDS planes, row tile by row tile, one lane per chain.
// ---------------------------------------------------------------------------
// Diagnostic phase clocks (PSN_LK_STAMPS, thread 0's view): accumulated
// s_memtime ticks per phase, written as stamps[wg][0..15] at the end.
#ifdef PSN_LK_STAMPS
#define BX_CLK(t) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory")
#define BX_BEGIN() BX_CLK(bx_t)
#define BX_MARK(i)                    \
    do {                              \
        unsigned long long t_;        \
        BX_CLK(t_);                   \
        bx_acc[i] += t_ - bx_t;       \
        bx_t = t_;                    \
    } while (0)
#define BX_COUNT(i) bx_acc[i]++
#else
#define BX_BEGIN() \
    do {           \
    } while (0)
#define BX_MARK(i) \
    do {           \
    } while (0)
#define BX_COUNT(i) \
    do {            \
    } while (0)
#endif
template <int UPT, bool NOTAIL>
__global__ __launch_bounds__(kBxNT, bx_occupancy(UPT, NOTAIL)) void lk_kernel_bx(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    static_assert(UPT % 2 == 0, "units are processed in pairs");
    constexpr int NT = kBxNT;
    const int tid = threadIdx.x, lane = tid & 63;
    if (A.poison_lds) lds_poison<NT>(smem, A.poison_lds);
    const int g = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    int qi = 0;
    while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
    const LkQueryDev &Q = A.q[qi];
    const int pi = lk_query_point(Q, A.counts, A.count_stride, g);
    if (pi < 0) return;  // past the query's device count
    const int w = Q.win_w, h = Q.win_h;
    const int maxL = Q.max_level, flags = Q.flags;
    const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
    const int QW = bx_qw(w), U = h * QW;
    const int nqB = sse ? (w / 8) * 2 : 0, n8 = 4 * nqB, tB = w - n8;   // b: 8-pixel steps
    const int nqA = sse ? w / 4 : 0, nA4 = 4 * nqA, tA = w - nA4;        // A: 4-pixel steps
    const int PM = bx_pm(w), JRW = st_jreg_w(w), JRH = st_jreg_h(h), JRP = bx_jrp(w), JRP4 = JRP >> 2;
    const BxLayout lay(w, h, UPT);
    int *X = (int *)smem;                      // chain-check records, two parities
    float *RS = (float *)(X + kBxXInts);       // serial-chain results (wave 0 -> all)
    int *EP = (int *)(RS + 16);                // err partial sums per wave
    // b-fallback tile hand-off flags (PSN_BX_FLAGS): ready[3], consumed[3], and
    // FLG[6] = a hand-off wait ran out of its bound (never expected: the point is
    // then reported failed, see the result writes)
    volatile int *FLG = (volatile int *)(RS + 24);
    if (threadIdx.x < 7) FLG[threadIdx.x] = threadIdx.x < 6 ? -1 : 0;  // ordered by the first level barrier
    int fb_epoch = 0;
    uint8_t *JR = smem + lay.jr;
    const uint32_t *JR32 = (const uint32_t *)JR;
    uint8_t *UN = smem + lay.un;
    const uint32_t *P32 = (const uint32_t *)UN;
    float *PL = (float *)UN;

    const int u0 = tid * UPT;
    const int y0 = u0 / QW, q0 = u0 - y0 * QW;
    // per unit of the thread: the byte offset of its J dwords in the region (row
    // y * JRP + 4 q; 0 past the window, where the gradients are zero), two units
    // per register (the b pass adds a half to the iteration's base: SDWA), and
    // whether it is an SSE2 unit of the b chains (bit k)
    unsigned UB[UPT / 2];
    unsigned sseB = 0;
    {
        int y = y0, q = q0;
#pragma unroll
        for (int k = 0; k < UPT; k++) {
            const unsigned o = u0 + k < U ? (unsigned)(y * JRP + 4 * q) : 0u;
            if (k & 1)
                UB[k >> 1] |= o << 16;
            else
                UB[k >> 1] = o;
            sseB |= (unsigned)(q < nqB) << k;
            if (++q == QW) {
                q = 0;
                y++;
            }
        }
    }

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
    int par = 0;
#ifdef PSN_LK_STAMPS
    unsigned long long bx_acc[16] = {}, bx_t = 0, bx_t0 = 0, bx_r0 = 0;
    BX_CLK(bx_t0);
    bx_t = bx_t0;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(bx_r0) : : "memory");  // 100 MHz
#endif

    unsigned IP[UPT][2], XP[UPT][2], YP[UPT][2];  // I, Ix, Iy as packed 16-bit pairs (pixels 0,1 and 2,3)
    int gmax = 0;              // max |Ix|, |Iy| of the thread's pixels
    unsigned nwin = 0;         // window passes (A phase + iterations) over the levels: the sample count / (w*h)

    for (int level = maxL; level >= 0; level--) {
        const LevelDev I = ring_level_u(A.ring, Q.prev_slot, level);
        const LevelDev J = ring_level_u(A.ring, Q.next_slot, level);
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
        int jr_x0 = (cv_floor(nx) - kStJMargin) & ~3, jr_y0 = cv_floor(ny) - kStJMargin;

        __syncthreads();  // the previous level is done with LDS
        dma_patch<NT>(UN, I, ipy - 1, ipx - 1, w + 3, h + 3, PM, Q.dv_bxpm);
        dma_wait();
        // the J region moves while the A phase reads the I patch: waited for
        // before the A publish barrier, which makes it visible to every wave
        dma_patch<NT>(JR, J, jr_y0, jr_x0, JRW, JRH, JRP4, Q.dv_bxjr);
        barrier_inflight();  // the I patch (waited above) for every wave; J still moving
        BX_MARK(0);  // level setup + staging
        bx_prio_lo();

        // ---- A phase: Scharr + bilinear window values of the thread's units from
        // the I patch bytes; the 15 A chains (sum x class) as runs ----
        float A11, A12, A22;
        nwin++;
        {
            const int sh = (ipx - 1) & 3;
            int T11[5] = {0, 0, 0, 0, 0}, T22[5] = {0, 0, 0, 0, 0}, T12[5] = {0, 0, 0, 0, 0};
            int M12[5] = {0, 0, 0, 0, 0}, m12[5] = {0, 0, 0, 0, 0};
            int gmx = 0, gmn = 0;  // max / min gradient of the thread's pixels
            // every derivative the window reads inside the image (columns ipx .. ipx +
            // 4 QW + 1, rows ipy .. ipy + h): no border masks (uniform)
            const bool interior = ipx >= 0 && ipy >= 0 && ipx + 4 * QW + 2 <= cols && ipy + h + 1 <= rows;
            const int c256 = 1 << 8, c8192 = 1 << 13;  // scalar accumulators of the VOP3 v_dot2
            auto apass = [&](auto inner) {
            constexpr bool IN = decltype(inner)::value;
            int y = y0, q = q0;
            asm volatile("" : "+v"(y), "+v"(q));  // opaque: no per-unit address hoisting (VGPRs)
#pragma unroll
            for (int k = 0; k < UPT; k++) {
                const bool uv = u0 + k < U;
                const int yy = uv ? y : 0, qq = uv ? q : 0;
                bx_unit<IN, NOTAIL>(P32, PM, sh, yy, qq, uv, w, ipx, ipy, cols, rows, iw00, iw01, iw10, iw11, c256,
                                    c8192, IP[k], XP[k], YP[k], gmx, gmn);
                // materialize the unit's results here: no sinking of its arithmetic
                // past later units (which would keep its patch bytes live)
                asm volatile("" : "+v"(IP[k][0]), "+v"(IP[k][1]), "+v"(XP[k][0]), "+v"(XP[k][1]), "+v"(YP[k][0]),
                             "+v"(YP[k][1]), "+v"(gmx), "+v"(gmn));
                if (++q == QW) {
                    q = 0;
                    y++;
                }
                __builtin_amdgcn_sched_barrier(0);  // one unit at a time (register pressure)
            }
            };
            if (interior)
                apass(std::true_type());
            else
                apass(std::false_type());
            gmax = max(gmx, -gmn);
            // A products of the window values, units in pairs (a second pass keeps
            // the Scharr temporaries and the chain runs apart): v_mad_i32_i16 on the
            // packed gradient halves, one v_max3 / v_min3 per two A12 prefixes
            int q = q0;
            asm volatile("" : "+v"(q));
#pragma unroll
            for (int k = 0; k < UPT; k += 2) {
                unsigned xs[2][2], ys[2][2], xt[2][2], yt[2][2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    // SSE2 unit: pixel i feeds lane chain i; else the tail chain, row-major
                    // (branch-free: the other chain's gradients are masked to zero)
                    const unsigned ms = (NOTAIL || q < nqA) ? ~0u : 0u;
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        xs[u][hh] = XP[k + u][hh] & ms;
                        ys[u][hh] = YP[k + u][hh] & ms;
                        xt[u][hh] = XP[k + u][hh] & ~ms;
                        yt[u][hh] = YP[k + u][hh] & ~ms;
                    }
                    if (++q == QW) q = 0;
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int hh = i >> 1;
                    int ta, tb;
                    if (i & 1) {
                        T11[i] = mad16p<1, 1>(xs[1][hh], xs[1][hh], mad16p<1, 1>(xs[0][hh], xs[0][hh], T11[i]));
                        T22[i] = mad16p<1, 1>(ys[1][hh], ys[1][hh], mad16p<1, 1>(ys[0][hh], ys[0][hh], T22[i]));
                        ta = mad16p<1, 1>(xs[0][hh], ys[0][hh], T12[i]);
                        tb = mad16p<1, 1>(xs[1][hh], ys[1][hh], ta);
                    } else {
                        T11[i] = mad16p<0, 0>(xs[1][hh], xs[1][hh], mad16p<0, 0>(xs[0][hh], xs[0][hh], T11[i]));
                        T22[i] = mad16p<0, 0>(ys[1][hh], ys[1][hh], mad16p<0, 0>(ys[0][hh], ys[0][hh], T22[i]));
                        ta = mad16p<0, 0>(xs[0][hh], ys[0][hh], T12[i]);
                        tb = mad16p<0, 0>(xs[1][hh], ys[1][hh], ta);
                    }
                    run2(T12[i], M12[i], m12[i], ta, tb);
                }
                if (!NOTAIL) {  // the tail chain: unit k's pixels 0-3, then unit k+1's
#pragma unroll
                    for (int u = 0; u < 2; u++)
#pragma unroll
                        for (int hh = 0; hh < 2; hh++) {
                            T11[4] = mad16p<1, 1>(xt[u][hh], xt[u][hh], mad16p<0, 0>(xt[u][hh], xt[u][hh], T11[4]));
                            T22[4] = mad16p<1, 1>(yt[u][hh], yt[u][hh], mad16p<0, 0>(yt[u][hh], yt[u][hh], T22[4]));
                            const int ta = mad16p<0, 0>(xt[u][hh], yt[u][hh], T12[4]);
                            const int tb = mad16p<1, 1>(xt[u][hh], yt[u][hh], ta);
                            run2(T12[4], M12[4], m12[4], ta, tb);
                        }
                }
                asm volatile("" : "+v"(T11[0]), "+v"(T11[1]), "+v"(T11[2]), "+v"(T11[3]), "+v"(T11[4]), "+v"(T22[0]),
                             "+v"(T22[1]), "+v"(T22[2]), "+v"(T22[3]), "+v"(T22[4]));
                asm volatile("" : "+v"(T12[0]), "+v"(T12[1]), "+v"(T12[2]), "+v"(T12[3]), "+v"(T12[4]), "+v"(M12[0]),
                             "+v"(M12[1]), "+v"(M12[2]), "+v"(M12[3]), "+v"(M12[4]));
                asm volatile("" : "+v"(m12[0]), "+v"(m12[1]), "+v"(m12[2]), "+v"(m12[3]), "+v"(m12[4]));
            }
            // A11 / A22 terms are >= 0: the maximum prefix is the total
            int T[15], M[15], m[15];
#pragma unroll
            for (int c = 0; c < 5; c++) {
                T[c] = T11[c], M[c] = T11[c], m[c] = 0;
                T[5 + c] = T12[c], M[5 + c] = M12[c], m[5 + c] = m12[c];
                T[10 + c] = T22[c], M[10 + c] = T22[c], m[10 + c] = 0;
            }
            BX_MARK(1);  // A window values + runs
            bx_prio_hi();
            int *rec = X + par * 4 * kBxRecInts;
            par ^= 1;
            bx_publish<15>(T, rec, NOTAIL || tA == 0);
            dma_wait();  // this thread's J region loads (the barrier: every thread's)
            __syncthreads();
            bx_check<15>(T, M, m, false, rec, NOTAIL || tA == 0);
            __syncthreads();
            int tot, h0, base0;
            const bool exact = bx_eval<15>(rec, tot, h0, base0);
            float s3[3];
            if (exact) {
#pragma unroll
                for (int s = 0; s < 3; s++) {
                    float t = rl_f(tot, 5 * s + 4);
                    if (sse)
                        t = __fadd_rn(t, __fadd_rn(__fadd_rn(__fadd_rn(rl_f(tot, 5 * s), rl_f(tot, 5 * s + 1)),
                                                             rl_f(tot, 5 * s + 2)), rl_f(tot, 5 * s + 3)));
                    s3[s] = t;
                }
            } else {
                // ordered float chains from half wave h0 on (every earlier prefix is an
                // exact integer: the chains start from base0): tiles of HW half waves
                // (the units of threads 32g..), products chain-major into 3 planes,
                // double-buffered: the threads of the next tile write its products
                // while the chain lanes (lanes 0-14 of wave 0; lane c holds chain c's
                // base0) sum the current one
                // the fallback's thread roles from an opaque copy of the thread id: computed
                // here, not hoisted to the kernel start and spilled across the loops
                int ftid = (int)threadIdx.x;
                asm volatile("" : "+v"(ftid));
                const int HW = Q.bx_hw, PCA = 3 * bx_pc(UPT) * HW;
                const bool chl = ftid < 15;  // wave 0: its tiles are written first, so it rarely writes while it sums
                const int cl = chl ? ftid : 0, cs = cl / 5, cc = cl - 5 * cs;
                float acc = (float)base0;  // |base0| <= 2^24: exact
                const int g_last = (U - 1) / (32 * UPT);
                auto geoA = [&](int g, int &sa, int &ta, int &nsse, int &ntail) {
                    const int ua = 32 * UPT * g, ub = min(ua + 32 * UPT * HW, U);
                    sa = (ua / QW) * nqA + min(ua % QW, nqA);
                    ta = (ua / QW) * tA + min(max(4 * (ua % QW) - nA4, 0), tA);
                    nsse = (ub / QW) * nqA + min(ub % QW, nqA) - sa;
                    ntail = (ub / QW) * tA + min(max(4 * (ub % QW) - nA4, 0), tA) - ta;
                };
                auto unitA = [&](int yk, int qk, bool uv, unsigned x0, unsigned x1, unsigned y0_, unsigned y1_, float *buf,
                                 int S, int P, int sa, int ta) {
                    if (!uv) return;
                    unsigned xp[2] = {x0, x1}, yp[2] = {y0_, y1_};
                    asm volatile("" : "+v"(xp[0]), "+v"(xp[1]), "+v"(yp[0]), "+v"(yp[1]));
                    const bool su = NOTAIL || qk < nqA;
                    const int base = su ? yk * nqA + qk - sa : 4 * S + yk * tA + 4 * qk - nA4 - ta;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        // pixels past the window width write a dummy slot past the buffers
                        const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                        const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                        const bool on = 4 * qk + i < w;
                        float *d1 = on ? buf + (su ? i * S + base : base + i) : PL + 2 * PCA;
                        const int pp = on ? P : 1;
                        d1[0] = (float)__mul24(gx, gx);
                        d1[pp] = (float)__mul24(gx, gy);
                        d1[2 * pp] = (float)__mul24(gy, gy);
                    }
                };
                // half-wave tiles: the whole wave writes one (as the b fallback's write_tile)
                constexpr int K1 = UPT / 2;
                const bool split = HW == 1 && (UPT & 1) == 0;
                auto swp = [](unsigned a, unsigned b, bool first) {
                    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
                    return first ? r[0] : r[1];
                };
                // no-tail build: the tile's half picked at compile time, the unit's plane
                // slot from its index in the tile (as the b fallback's write_tile_nt)
                auto writeA_nt = [&](int g, float *buf, auto lowerT) {
                    constexpr bool lower = decltype(lowerT)::value;
                    if ((ftid >> 6) != (g >> 1)) return;
                    int sa, ta, nsse, ntail;
                    geoA(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    const bool up = (ftid & 32) != 0;
                    const int ub = lower ? (up ? (ftid ^ 32) * UPT + K1 : ftid * UPT) : (up ? ftid * UPT + K1 : (ftid ^ 32) * UPT);
                    const int rel = ub - 32 * UPT * g;
                    auto pick = [](unsigned a, unsigned b) {
                        auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
                        return lower ? r[0] : r[1];
                    };
#pragma unroll
                    for (int k = 0; k < K1; k++) {
                        unsigned xp[2] = {pick(XP[k][0], XP[K1 + k][0]), pick(XP[k][1], XP[K1 + k][1])};
                        unsigned yp[2] = {pick(YP[k][0], YP[K1 + k][0]), pick(YP[k][1], YP[K1 + k][1])};
                        if (ub + k < U) {
                            asm volatile("" : "+v"(xp[0]), "+v"(xp[1]), "+v"(yp[0]), "+v"(yp[1]));
                            float *d1 = buf + rel + k;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                                const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                                d1[i * S] = (float)__mul24(gx, gx);
                                d1[i * S + P] = (float)__mul24(gx, gy);
                                d1[i * S + 2 * P] = (float)__mul24(gy, gy);
                            }
                        }
                    }
                };
                auto writeA = [&](int g, float *buf) {
                    if constexpr (NOTAIL) {
                        if (HW == 1) {  // (split: UPT is even)
                            if (g & 1)
                                writeA_nt(g, buf, std::false_type());
                            else
                                writeA_nt(g, buf, std::true_type());
                            return;
                        }
                    }
                    int sa, ta, nsse, ntail;
                    if (split) {
                        if ((ftid >> 6) != (g >> 1)) return;
                        geoA(g, sa, ta, nsse, ntail);
                        const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                        const bool lower = (g & 1) == 0, own = ((ftid >> 5) & 1) == (g & 1);
                        const int ub = (own ? ftid : ftid ^ 32) * UPT + (lower == own ? 0 : K1);
                        int yk = ub / QW, qk = ub - yk * QW;
                        asm volatile("" : "+v"(yk), "+v"(qk));
#pragma unroll
                        for (int k = 0; k < K1; k++) {
                            unitA(yk, qk, ub + k < U, swp(XP[k][0], XP[K1 + k][0], lower), swp(XP[k][1], XP[K1 + k][1], lower),
                                  swp(YP[k][0], YP[K1 + k][0], lower), swp(YP[k][1], YP[K1 + k][1], lower), buf, S, P, sa, ta);
                            if (++qk == QW) {
                                qk = 0;
                                yk++;
                            }
                        }
                        return;
                    }
                    if ((ftid >> 5) < g || (ftid >> 5) >= g + HW) return;
                    geoA(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    if constexpr (NOTAIL && UPT <= 8) {  // the thread's own units, slots from their index
                        const int rel = u0 - 32 * UPT * g;
#pragma unroll
                        for (int k = 0; k < UPT; k++) {
                            if (u0 + k >= U) break;
                            unsigned xp[2] = {XP[k][0], XP[k][1]}, yp[2] = {YP[k][0], YP[k][1]};
                            asm volatile("" : "+v"(xp[0]), "+v"(xp[1]), "+v"(yp[0]), "+v"(yp[1]));
                            float *d1 = buf + rel + k;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                                const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                                d1[i * S] = (float)__mul24(gx, gx);
                                d1[i * S + P] = (float)__mul24(gx, gy);
                                d1[i * S + 2 * P] = (float)__mul24(gy, gy);
                            }
                        }
                        return;
                    }
                    int yk = y0, qk = q0;
                    asm volatile("" : "+v"(yk), "+v"(qk));
#pragma unroll
                    for (int k = 0; k < UPT; k++) {
                        unitA(yk, qk, u0 + k < U, XP[k][0], XP[k][1], YP[k][0], YP[k][1], buf, S, P, sa, ta);
                        if (++qk == QW) {
                            qk = 0;
                            yk++;
                        }
                    }
                };
                auto padA = [&](int g, float *buf) {  // chain lanes: zero their region's pad
                    if (!chl) return;
                    int sa, ta, nsse, ntail;
                    geoA(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    const int len = cc < 4 ? nsse : ntail;
                    float *rg = buf + cs * P + cc * S;
                    for (int i = len; i < ((len + 15) & ~15); i++) rg[i] = 0.f;
                };
                // the I patch under PL was consumed before the publish barrier
                writeA(h0, PL);
                padA(h0, PL);
                __syncthreads();
                for (int g = h0, t = 0; g <= g_last; g += HW, t ^= 1) {
                    float *cur = PL + t * PCA, *nxt = PL + (t ^ 1) * PCA;
                    if (g + HW <= g_last) writeA(g + HW, nxt);
                    if ((ftid >> 6) == 0) {
                        int sa, ta, nsse, ntail;
                        geoA(g, sa, ta, nsse, ntail);
                        const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                        const int len = chl ? (cc < 4 ? nsse : ntail) : 0;
                        // (no-tail: every chain lane's length is nsse)
                        const int nbmax = NOTAIL ? (nsse + 15) >> 4 : __builtin_amdgcn_readlane(wave_max_scan((len + 15) >> 4), 63);
                        // (no-tail: the tail-chain lanes keep acc = 0)
                        if (chl && (!NOTAIL || cc < 4)) acc = chain_sum_pl<NOTAIL>(cur + cs * P + cc * S, len, nbmax, acc);
                        if (g + HW <= g_last) padA(g + HW, nxt);
                    }
                    __syncthreads();
                }
                if (ftid < 64) {  // wave 0 combines in the SSE2 build's order
                    const int av = __float_as_int(acc);
#pragma unroll
                    for (int s = 0; s < 3; s++) {
                        float t = __int_as_float(__builtin_amdgcn_readlane(av, 5 * s + 4));
                        if (sse) {
                            const float c0 = __int_as_float(__builtin_amdgcn_readlane(av, 5 * s));
                            const float c1 = __int_as_float(__builtin_amdgcn_readlane(av, 5 * s + 1));
                            const float c2 = __int_as_float(__builtin_amdgcn_readlane(av, 5 * s + 2));
                            const float c3 = __int_as_float(__builtin_amdgcn_readlane(av, 5 * s + 3));
                            t = __fadd_rn(t, __fadd_rn(__fadd_rn(__fadd_rn(c0, c1), c2), c3));
                        }
                        if (ftid == 0) RS[s] = t;
                    }
                }
                __syncthreads();
                s3[0] = RS[0];
                s3[1] = RS[1];
                s3[2] = RS[2];
            }
            BX_MARK(2);  // A publish / eval / serial chains
            A11 = __fmul_rn(s3[0], FLT_SCALE);
            A12 = __fmul_rn(s3[1], FLT_SCALE);
            A22 = __fmul_rn(s3[2], FLT_SCALE);
        }
        float D = __fsub_rn(__fmul_rn(A11, A22), __fmul_rn(A12, A12));
        {
            const float dd = __fsub_rn(A11, A22);
            const float t = __fadd_rn(__fmul_rn(dd, dd), __fmul_rn(__fmul_rn(4.f, A12), A12));
            const float minEig = __fdiv_rn(__fsub_rn(__fadd_rn(A22, A11), sqrtf(t)), (float)(2 * w * h));
            if (flags & PSN_LK_GET_MIN_EIGENVALS) errv = minEig;
            if (minEig < Q.min_eig || D < FLT_EPSILON) {
                if (level == 0) status = 0;
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
            int w00, w01, w10, w11;
            bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), w00, w01, w10, w11);
            if (!(inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW && iny + h + 1 <= jr_y0 + JRH)) {
                // every wave's J reads of the previous iteration precede its barrier
                jr_x0 = (inx - kStJMargin) & ~3;
                jr_y0 = iny - kStJMargin;
                dma_patch<NT>(JR, J, jr_y0, jr_x0, JRW, JRH, JRP4, Q.dv_bxjr);
                dma_wait();
                __syncthreads();
            }
            BX_MARK(3);  // iteration head (restage)
            bx_prio_lo();
            BX_COUNT(10);
            nwin++;
            const unsigned W0 = pack_w(w00, w01), W1 = pack_w(w10, w11);
            const int ox = inx - jr_x0, oy = iny - jr_y0, sj = ox & 3;
            const unsigned s0 = bx_sel(sj, 0), s1 = bx_sel(sj, 1), s2 = bx_sel(sj, 2), s3 = bx_sel(sj, 3);
            int T1[5] = {0, 0, 0, 0, 0}, M1[5] = {0, 0, 0, 0, 0}, m1[5] = {0, 0, 0, 0, 0};
            int T2[5] = {0, 0, 0, 0, 0}, M2[5] = {0, 0, 0, 0, 0}, m2[5] = {0, 0, 0, 0, 0};
            int dmx = 0, dmn = 0;  // max / min d of the thread's pixels (when tracked)
            const int c256 = opaque256();
            // every term d * g is an exact float unless |g| > 2^24 / 8160 (|d| <= 8160):
            // below that in the whole wave, the pass keeps no max |d|
            const bool dtrack = __ballot(gmax > kExact / 8160) != 0ull;
            auto bmain = [&](auto trk) {
                // the iteration's byte offsets of rows oy and oy + 1 in LDS, opaque
                // scalars (the J region's constant offset stays inside them: one
                // SDWA add per row and unit, not two adds and a constant)
                unsigned jo0 = (unsigned)((const uint8_t *)(JR32 + oy * JRP4 + (ox >> 2)) - smem);
                unsigned jo1 = jo0 + 4u * (unsigned)JRP4;
                asm volatile("" : "+s"(jo0), "+s"(jo1));
                // units in pairs (UPT is even): each chain takes its two terms by
                // v_mad_i32_i16 (gradient half, product and sum in one) and one
                // v_max3 / v_min3 of the two new prefixes
#pragma unroll
                for (int k = 0; k < UPT; k += 2) {
                    int d[2][4], ms[2];
                    asm volatile("" : "+v"(UB[k >> 1]));  // opaque per iteration: its halves stay packed
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const unsigned o = u ? UB[k >> 1] >> 16 : UB[k >> 1] & 0xffffu;
                        bx_diffs2((const uint32_t *)(smem + jo0 + o), (const uint32_t *)(smem + jo1 + o), W0, W1, s0, s1, s2,
                                  s3, IP[k + u], d[u], c256);
                        ms[u] = -(int)((sseB >> (k + u)) & 1u);  // SSE2 unit -> lane chains 0-3, else the tail chain
                    }
                    if constexpr (decltype(trk)::value) {
#pragma unroll
                        for (int u = 0; u < 2; u++) {
                            dmx = max(dmx, max(d[u][0], d[u][1]));
                            dmx = max(dmx, max(d[u][2], d[u][3]));
                            dmn = min(dmn, min(d[u][0], d[u][1]));
                            dmn = min(dmn, min(d[u][2], d[u][3]));
                        }
                    }
                    if (NOTAIL) {  // every unit feeds lane chains 0-3
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int h = i >> 1;
                            int ta, tb;
                            if (i & 1) {
                                ta = mad16<1>(d[0][i], XP[k][h], T1[i]);
                                tb = mad16<1>(d[1][i], XP[k + 1][h], ta);
                            } else {
                                ta = mad16<0>(d[0][i], XP[k][h], T1[i]);
                                tb = mad16<0>(d[1][i], XP[k + 1][h], ta);
                            }
                            run2(T1[i], M1[i], m1[i], ta, tb);
                            if (i & 1) {
                                ta = mad16<1>(d[0][i], YP[k][h], T2[i]);
                                tb = mad16<1>(d[1][i], YP[k + 1][h], ta);
                            } else {
                                ta = mad16<0>(d[0][i], YP[k][h], T2[i]);
                                tb = mad16<0>(d[1][i], YP[k + 1][h], ta);
                            }
                            run2(T2[i], M2[i], m2[i], ta, tb);
                        }
                    } else {
                        // branch-free: the other chain gets zero terms (masked d); the tail
                        // chain first (unit k's pixels 0-3, then unit k+1's, in order)
#pragma unroll
                        for (int u = 0; u < 2; u++) {
                            const unsigned *xp = XP[k + u], *yp = YP[k + u];
                            const int nm = ~ms[u];
                            int a0 = mad16<0>(d[u][0] & nm, xp[0], T1[4]);
                            int a1 = mad16<1>(d[u][1] & nm, xp[0], a0);
                            run2(T1[4], M1[4], m1[4], a0, a1);
                            a0 = mad16<0>(d[u][2] & nm, xp[1], T1[4]);
                            a1 = mad16<1>(d[u][3] & nm, xp[1], a0);
                            run2(T1[4], M1[4], m1[4], a0, a1);
                            a0 = mad16<0>(d[u][0] & nm, yp[0], T2[4]);
                            a1 = mad16<1>(d[u][1] & nm, yp[0], a0);
                            run2(T2[4], M2[4], m2[4], a0, a1);
                            a0 = mad16<0>(d[u][2] & nm, yp[1], T2[4]);
                            a1 = mad16<1>(d[u][3] & nm, yp[1], a0);
                            run2(T2[4], M2[4], m2[4], a0, a1);
                        }
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int h = i >> 1;
                            const int e0 = d[0][i] & ms[0], e1 = d[1][i] & ms[1];
                            int ta, tb;
                            if (i & 1) {
                                ta = mad16<1>(e0, XP[k][h], T1[i]);
                                tb = mad16<1>(e1, XP[k + 1][h], ta);
                            } else {
                                ta = mad16<0>(e0, XP[k][h], T1[i]);
                                tb = mad16<0>(e1, XP[k + 1][h], ta);
                            }
                            run2(T1[i], M1[i], m1[i], ta, tb);
                            if (i & 1) {
                                ta = mad16<1>(e0, YP[k][h], T2[i]);
                                tb = mad16<1>(e1, YP[k + 1][h], ta);
                            } else {
                                ta = mad16<0>(e0, YP[k][h], T2[i]);
                                tb = mad16<0>(e1, YP[k + 1][h], ta);
                            }
                            run2(T2[i], M2[i], m2[i], ta, tb);
                        }
                    }
                    // materialize the runs per unit pair (no sinking across pairs)
                    asm volatile("" : "+v"(T1[0]), "+v"(T1[1]), "+v"(T1[2]), "+v"(T1[3]), "+v"(T1[4]), "+v"(M1[0]),
                                 "+v"(M1[1]), "+v"(M1[2]), "+v"(M1[3]), "+v"(M1[4]));
                    asm volatile("" : "+v"(m1[0]), "+v"(m1[1]), "+v"(m1[2]), "+v"(m1[3]), "+v"(m1[4]), "+v"(T2[0]),
                                 "+v"(T2[1]), "+v"(T2[2]), "+v"(T2[3]), "+v"(T2[4]));
                    asm volatile("" : "+v"(M2[0]), "+v"(M2[1]), "+v"(M2[2]), "+v"(M2[3]), "+v"(M2[4]), "+v"(m2[0]),
                                 "+v"(m2[1]), "+v"(m2[2]), "+v"(m2[3]), "+v"(m2[4]), "+v"(dmx), "+v"(dmn));
                }
            };
            if (dtrack)
                bmain(std::true_type());
            else
                bmain(std::false_type());
            const int dmax = max(dmx, -dmn);
            // masked pixels carry zero gradients but any d: only real terms count
            const bool bad = (long long)dmax * gmax > (long long)kExact;
            int T[10], M[10], m[10];
#pragma unroll
            for (int c = 0; c < 5; c++) {
                T[c] = T1[c], M[c] = M1[c], m[c] = m1[c];
                T[5 + c] = T2[c], M[5 + c] = M2[c], m[5 + c] = m2[c];
            }
            BX_MARK(4);  // b main pass
            bx_prio_hi();
            int *rec = X + par * 4 * kBxRecInts;
            par ^= 1;
            bx_publish<10>(T, rec, NOTAIL || tB == 0);
            BX_MARK(9);  // b publish (this wave's scans and records)
            __syncthreads();
            bx_check<10>(T, M, m, bad, rec, NOTAIL || tB == 0);
            __syncthreads();
            int tot, h0, base0;
            float b1, b2;
            const bool bex = bx_eval<10>(rec, tot, h0, base0);
            BX_MARK(5);  // b publish + barrier + eval
            if (bex) {
                b1 = rl_f(tot, 4);
                b2 = rl_f(tot, 9);
                if (sse) {
                    b1 = __fadd_rn(b1, __fadd_rn(__fadd_rn(rl_f(tot, 0), rl_f(tot, 2)), __fadd_rn(rl_f(tot, 1), rl_f(tot, 3))));
                    b2 = __fadd_rn(b2, __fadd_rn(__fadd_rn(rl_f(tot, 5), rl_f(tot, 7)), __fadd_rn(rl_f(tot, 6), rl_f(tot, 8))));
                }
            } else {
                // ordered float chains from half wave h0 on, tiles of 32 threads' units,
                // double-buffered: the threads of tile g+1 write its products while the
                // chain lanes (wave 0, lanes 0-9, starting from the exact prefixes
                // base0) sum tile g
                // thread roles from an opaque copy of the thread id (see the A fallback)
                int ftid = (int)threadIdx.x;
                asm volatile("" : "+v"(ftid));
                const int HW = Q.bx_hw, PC = bx_pc(UPT) * HW;
                const bool chl = ftid < 10;  // wave 0 (as in the A fallback)
                const int cl = chl ? ftid : 0, cs = cl / 5, cc = cl - 5 * cs;
                float acc = (float)base0;
                const int g_last = (U - 1) / (32 * UPT);
                auto tile_geo = [&](int g, int &sa, int &ta, int &nsse, int &ntail) {
                    const int ua = 32 * UPT * g, ub = min(ua + 32 * UPT * HW, U);
                    sa = (ua / QW) * nqB + min(ua % QW, nqB);
                    ta = (ua / QW) * tB + min(max(4 * (ua % QW) - n8, 0), tB);
                    nsse = (ub / QW) * nqB + min(ub % QW, nqB) - sa;
                    ntail = (ub / QW) * tB + min(max(4 * (ub % QW) - n8, 0), tB) - ta;
                };
                // one unit's b products into the tile's chain regions
                auto tile_unit = [&](int yk, int qk, bool uv, const unsigned (&ip)[2], const unsigned (&xp)[2],
                                     const unsigned (&yp)[2], float *buf, int S, int P, int sa, int ta, int zf) {
                    if (!uv) return;
                    int d[4];
                    bx_diffs(JR32 + (oy + yk) * JRP4 + (ox >> 2) + qk, JRP4, W0, W1, s0, s1, s2, s3, ip, d, zf);
                    const bool su = NOTAIL || qk < nqB;
                    const int base = su ? yk * nqB + qk - sa : 4 * S + yk * tB + 4 * qk - n8 - ta;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        // pixels past the window width write a dummy slot past the buffers (branch-free)
                        const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                        const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                        const bool on = 4 * qk + i < w;
                        float *d1 = on ? buf + (su ? i * S + base : base + i) : PL + 6 * PC;  // past 3 buffers
                        d1[0] = (float)__mul24(d[i], gx);
                        d1[on ? P : 1] = (float)__mul24(d[i], gy);
                    }
                };
                // Half-wave tiles (HW = 1): the whole wave writes one tile, K1 = UPT/2
                // unit slots per lane. v_permlane32_swap of unit registers k and K1 + k
                // gives, as its first result, lower lane l's unit k on lane l and its
                // unit K1 + k on lane l + 32 (a lower-half tile), as its second, upper
                // lane l + 32's unit K1 + k there and its unit k on lane l (an upper-half
                // tile): both halves run one instruction stream.
                constexpr int K1 = UPT / 2;
                const bool split = HW == 1 && (UPT & 1) == 0;
                auto swp = [](unsigned a, unsigned b, bool first) {
                    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
                    return first ? r[0] : r[1];
                };
                auto write_tile = [&](int g, float *buf) {
                    const int zf = opaque256();  // per tile: no diff constants hoisted out of the tile loop
                    int sa, ta, nsse, ntail;
                    if (split) {
                        if ((ftid >> 6) != (g >> 1)) return;
                        tile_geo(g, sa, ta, nsse, ntail);
                        const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                        const bool lower = (g & 1) == 0, own = ((ftid >> 5) & 1) == (g & 1);
                        const int ub = (own ? ftid : ftid ^ 32) * UPT + (lower == own ? 0 : K1);
                        int yk = ub / QW, qk = ub - yk * QW;
                        asm volatile("" : "+v"(yk), "+v"(qk));
#pragma unroll
                        for (int k = 0; k < K1; k++) {
                            const unsigned ip[2] = {swp(IP[k][0], IP[K1 + k][0], lower), swp(IP[k][1], IP[K1 + k][1], lower)};
                            const unsigned xp[2] = {swp(XP[k][0], XP[K1 + k][0], lower), swp(XP[k][1], XP[K1 + k][1], lower)};
                            const unsigned yp[2] = {swp(YP[k][0], YP[K1 + k][0], lower), swp(YP[k][1], YP[K1 + k][1], lower)};
                            tile_unit(yk, qk, ub + k < U, ip, xp, yp, buf, S, P, sa, ta, zf);
                            if (++qk == QW) {
                                qk = 0;
                                yk++;
                            }
                        }
                        return;
                    }
                    if ((ftid >> 5) < g || (ftid >> 5) >= g + HW) return;
                    tile_geo(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    if constexpr (NOTAIL && UPT <= 8) {  // the thread's own units: offsets from UB, slots from their index
                        unsigned fo0 = (unsigned)((const uint8_t *)(JR32 + oy * JRP4 + (ox >> 2)) - smem);
                        unsigned fo1 = fo0 + 4u * (unsigned)JRP4;
                        asm volatile("" : "+s"(fo0), "+s"(fo1));
                        const int rel = u0 - 32 * UPT * g;
#pragma unroll
                        for (int k = 0; k < UPT; k++) {
                            if (u0 + k >= U) break;
                            // opaque copies: nothing of the unit is hoisted out of the tile loop
                            unsigned ubk = UB[k >> 1], ip[2] = {IP[k][0], IP[k][1]}, xp[2] = {XP[k][0], XP[k][1]},
                                     yp[2] = {YP[k][0], YP[k][1]};
                            asm volatile("" : "+v"(ubk), "+v"(ip[0]), "+v"(ip[1]), "+v"(xp[0]), "+v"(xp[1]), "+v"(yp[0]),
                                         "+v"(yp[1]));
                            const unsigned off = (k & 1) ? ubk >> 16 : ubk & 0xffffu;
                            int d[4];
                            bx_diffs2((const uint32_t *)(smem + fo0 + off), (const uint32_t *)(smem + fo1 + off), W0, W1, s0,
                                      s1, s2, s3, ip, d, zf);
                            float *d1 = buf + rel + k;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                                const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                                d1[i * S] = (float)__mul24(d[i], gx);
                                d1[i * S + P] = (float)__mul24(d[i], gy);
                            }
                        }
                        return;
                    }
                    int yk = y0, qk = q0;
                    asm volatile("" : "+v"(yk), "+v"(qk));
#pragma unroll
                    for (int k = 0; k < UPT; k++) {
                        tile_unit(yk, qk, u0 + k < U, IP[k], XP[k], YP[k], buf, S, P, sa, ta, zf);
                        if (++qk == QW) {
                            qk = 0;
                            yk++;
                        }
                    }
                };
                // No-tail build, half-wave tiles: the unit's J dwords from its packed
                // offset (UB, swapped like the window values) and its plane slot from its
                // index in the tile (every quad is an SSE2 quad, every pixel inside the
                // window); the tile's half picked at compile time (no select per value)
                unsigned fo0 = (unsigned)((const uint8_t *)(JR32 + oy * JRP4 + (ox >> 2)) - smem);
                unsigned fo1 = fo0 + 4u * (unsigned)JRP4;
                asm volatile("" : "+s"(fo0), "+s"(fo1));
                auto write_tile_nt = [&](int g, float *buf, auto lowerT) {
                    constexpr bool lower = decltype(lowerT)::value;
                    const int zf = opaque256();
                    int sa, ta, nsse, ntail;
                    tile_geo(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    const bool up = (ftid & 32) != 0;
                    // lower tile: lane l < 32 its unit k, lane l + 32 lane l's unit K1 + k;
                    // upper tile: lane l < 32 lane l + 32's unit k, lane l + 32 its unit K1 + k
                    const int ub = lower ? (up ? (ftid ^ 32) * UPT + K1 : ftid * UPT) : (up ? ftid * UPT + K1 : (ftid ^ 32) * UPT);
                    const int rel = ub - 32 * UPT * g;
                    auto pick = [](unsigned a, unsigned b) {
                        auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
                        return lower ? r[0] : r[1];
                    };
                    auto uoff = [&](int k) { return (k & 1) ? UB[k >> 1] >> 16 : UB[k >> 1] & 0xffffu; };
#pragma unroll
                    for (int k = 0; k < K1; k++) {
                        const unsigned ip[2] = {pick(IP[k][0], IP[K1 + k][0]), pick(IP[k][1], IP[K1 + k][1])};
                        const unsigned xp[2] = {pick(XP[k][0], XP[K1 + k][0]), pick(XP[k][1], XP[K1 + k][1])};
                        const unsigned yp[2] = {pick(YP[k][0], YP[K1 + k][0]), pick(YP[k][1], YP[K1 + k][1])};
                        const unsigned off = pick(uoff(k), uoff(K1 + k));
                        if (ub + k < U) {
                            int d[4];
                            bx_diffs2((const uint32_t *)(smem + fo0 + off), (const uint32_t *)(smem + fo1 + off), W0, W1, s0,
                                      s1, s2, s3, ip, d, zf);
                            float *d1 = buf + rel + k;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int gx = (i & 1) ? hi16(xp[i >> 1]) : lo16(xp[i >> 1]);
                                const int gy = (i & 1) ? hi16(yp[i >> 1]) : lo16(yp[i >> 1]);
                                d1[i * S] = (float)__mul24(d[i], gx);
                                d1[i * S + P] = (float)__mul24(d[i], gy);
                            }
                        }
                    }
                };
                auto pad_tile = [&](int g, float *buf) {  // chain lanes: zero their region's pad
                    if (!chl) return;
                    int sa, ta, nsse, ntail;
                    tile_geo(g, sa, ta, nsse, ntail);
                    const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                    const int len = cc < 4 ? nsse : ntail;
                    float *rg = buf + cs * P + cc * S;
                    for (int i = len; i < ((len + 15) & ~15); i++) rg[i] = 0.f;
                };
#if PSN_BX_FLAGS
                if (split) {
                    // Three tile buffers, handed over through LDS flags instead of a
                    // workgroup barrier per tile: wave w writes its tiles 2w, 2w+1 as
                    // soon as their buffers are free (tile g waits for the chain lanes
                    // to finish tile g - 3), wave 0 first writes its own tiles, then
                    // its chain lanes sum tile after tile as each one is flagged ready.
                    // No cycle: tile g's writer waits only for tiles of lower waves.
                    const int ep = ++fb_epoch, wv = ftid >> 6, fl = ftid & 63;
                    auto tag = [&](int g) { return ep * 16 + g; };
                    auto spin = [&](int idx, int want) {
                        for (int n = 0; n < (1 << 22); n++) {  // (a bound: never a hang)
                            if (__builtin_amdgcn_readfirstlane(FLG[idx]) == want) break;
                            __builtin_amdgcn_s_sleep(1);
                        }
                        // the bound ran out: the tile may be half written, fail the point
                        if (__builtin_amdgcn_readfirstlane(FLG[idx]) != want) FLG[6] = 1;
                        asm volatile("" ::: "memory");
                    };
                    for (int g = max(h0, 2 * wv); g <= min(2 * wv + 1, g_last); g++) {
                        const int b = (g - h0) % 3;
                        if (g - h0 >= 3) spin(3 + b, tag(g - 3));
                        if constexpr (NOTAIL) {
                            if (g & 1)
                                write_tile_nt(g, PL + b * 2 * PC, std::false_type());
                            else
                                write_tile_nt(g, PL + b * 2 * PC, std::true_type());
                        } else {
                            write_tile(g, PL + b * 2 * PC);
                        }
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if (fl == 0) FLG[b] = tag(g);
                    }
                    BX_MARK(6);  // serial b: own tiles' products
                    if (wv == 0) {
                        for (int g = h0; g <= g_last; g++) {
                            const int b = (g - h0) % 3;
                            spin(b, tag(g));
                            float *cur = PL + b * 2 * PC;
                            int sa, ta, nsse, ntail;
                            tile_geo(g, sa, ta, nsse, ntail);
                            const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                            const int len = chl ? (cc < 4 ? nsse : ntail) : 0;
                            if (chl) {  // zero this chain's pad (its writer never touches it)
                                float *rg = cur + cs * P + cc * S;
                                for (int i = len; i < ((len + 15) & ~15); i++) rg[i] = 0.f;
                            }
                            const int nbmax = NOTAIL ? (nsse + 15) >> 4 : __builtin_amdgcn_readlane(wave_max_scan((len + 15) >> 4), 63);
                            if (chl && (!NOTAIL || cc < 4)) acc = chain_sum_pl<NOTAIL>(cur + cs * P + cc * S, len, nbmax, acc);
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            if (fl == 0) FLG[3 + b] = tag(g);
                        }
                    }
                } else
#endif
                {
                write_tile(h0, PL);
                pad_tile(h0, PL);
                __syncthreads();
                BX_MARK(6);  // serial b: first tile's products
                for (int g = h0, t = 0; g <= g_last; g += HW, t ^= 1) {  // tile = half waves g .. g+HW-1
                    float *cur = PL + t * 2 * PC, *nxt = PL + (t ^ 1) * 2 * PC;
                    if (g + HW <= g_last) write_tile(g + HW, nxt);
#ifdef PSN_LK_STAMPS
                    unsigned long long tc0, tc1, tc2;
                    BX_CLK(tc0);
#endif
                    if ((ftid >> 6) == 0) {
                        int sa, ta, nsse, ntail;
                        tile_geo(g, sa, ta, nsse, ntail);
                        const int S = bx_region(nsse), P = 4 * S + bx_region(ntail);
                        const int len = chl ? (cc < 4 ? nsse : ntail) : 0;
                        // (no-tail: every chain lane's length is nsse)
                        const int nbmax = NOTAIL ? (nsse + 15) >> 4 : __builtin_amdgcn_readlane(wave_max_scan((len + 15) >> 4), 63);
                        // (no-tail: the tail-chain lanes keep acc = 0)
                        if (chl && (!NOTAIL || cc < 4)) acc = chain_sum_pl<NOTAIL>(cur + cs * P + cc * S, len, nbmax, acc);
                        if (g + HW <= g_last) pad_tile(g + HW, nxt);
                    }
#ifdef PSN_LK_STAMPS
                    BX_CLK(tc1);
#endif
                    __syncthreads();
#ifdef PSN_LK_STAMPS
                    BX_CLK(tc2);
                    bx_acc[12] += tc1 - tc0;  // (chain lane 0's view) chain sums incl. its own tile writes
                    bx_acc[13] += tc2 - tc1;  // barrier wait
                    bx_acc[14]++;
#endif
                }
                }
                BX_MARK(7);  // serial b: pipelined products + chains
                BX_COUNT(11);
                if (ftid < 64) {  // wave 0 combines in the SSE2 build's order
                    const int a = __float_as_int(acc);
                    float r1 = __int_as_float(__builtin_amdgcn_readlane(a, 4));
                    float r2 = __int_as_float(__builtin_amdgcn_readlane(a, 9));
                    if (sse) {
                        const float bb0 = __fadd_rn(__int_as_float(__builtin_amdgcn_readlane(a, 0)),
                                                    __int_as_float(__builtin_amdgcn_readlane(a, 2)));
                        const float bb2 = __fadd_rn(__int_as_float(__builtin_amdgcn_readlane(a, 1)),
                                                    __int_as_float(__builtin_amdgcn_readlane(a, 3)));
                        const float bb1 = __fadd_rn(__int_as_float(__builtin_amdgcn_readlane(a, 5)),
                                                    __int_as_float(__builtin_amdgcn_readlane(a, 7)));
                        const float bb3 = __fadd_rn(__int_as_float(__builtin_amdgcn_readlane(a, 6)),
                                                    __int_as_float(__builtin_amdgcn_readlane(a, 8)));
                        r1 = __fadd_rn(r1, __fadd_rn(bb0, bb2));
                        r2 = __fadd_rn(r2, __fadd_rn(bb1, bb3));
                    }
                    if (ftid == 0) {
                        RS[4] = r1;
                        RS[5] = r2;
                    }
                }
                __syncthreads();
                b1 = RS[4];
                b2 = RS[5];
            }
            BX_MARK(8);  // b results
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
            int w00, w01, w10, w11;
            bilin_weights(__fsub_rn(qx, (float)iqx), __fsub_rn(qy, (float)iqy), w00, w01, w10, w11);
            if (!(iqx >= jr_x0 && iqy >= jr_y0 && iqx + w + 1 <= jr_x0 + JRW && iqy + h + 1 <= jr_y0 + JRH)) {
                __syncthreads();  // a serial b pass may still read nothing of JR, but be safe
                jr_x0 = (iqx - kStJMargin) & ~3;
                jr_y0 = iqy - kStJMargin;
                dma_patch<NT>(JR, J, jr_y0, jr_x0, JRW, JRH, JRP4, Q.dv_bxjr);
                dma_wait();
                __syncthreads();
            }
            const unsigned W0 = pack_w(w00, w01), W1 = pack_w(w10, w11);
            const int ox = iqx - jr_x0, oy = iqy - jr_y0, sj = ox & 3;
            const unsigned s0 = bx_sel(sj, 0), s1 = bx_sel(sj, 1), s2 = bx_sel(sj, 2), s3 = bx_sel(sj, 3);
            unsigned e = 0;
            {
                int y = y0, q = q0;
            asm volatile("" : "+v"(y), "+v"(q));  // opaque: no per-unit address hoisting (VGPRs)
#pragma unroll
                for (int k = 0; k < UPT; k++) {
                    const bool uv = u0 + k < U;
                    int d[4];
                    bx_diffs(JR32 + (oy + (uv ? y : 0)) * JRP4 + (ox >> 2) + (uv ? q : 0), JRP4, W0, W1, s0, s1, s2, s3, IP[k], d, 256);
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if (uv && 4 * q + i < w) e += (unsigned)abs(d[i]);
                    if (++q == QW) {
                        q = 0;
                        y++;
                    }
                    __builtin_amdgcn_sched_barrier(0);  // one unit at a time (register pressure)
                }
            }
            e = (unsigned)wave_sum((int)e);  // <= 64 * 48 * 8160 < 2^31
            if (lane == 0) EP[tid >> 6] = (int)e;
            __syncthreads();
            const unsigned et = (unsigned)EP[0] + (unsigned)EP[1] + (unsigned)EP[2] + (unsigned)EP[3];
            float errval;
            if (et <= (unsigned)kExact) {
                errval = (float)et;  // every partial sum of errval += |diff| is an exact integer
            } else {  // row-major order, one lane, row tiles
                const int TR = Q.bx_tre;
                float acc = 0.f;
                for (int r0 = 0; r0 < h; r0 += TR) {
                    const int tr = min(TR, h - r0);
                    __syncthreads();
                    int yk = y0, qk = q0;
                    asm volatile("" : "+v"(yk), "+v"(qk));
#pragma unroll
                    for (int k = 0; k < UPT; k++) {
                        if (u0 + k < U && yk >= r0 && yk < r0 + tr) {
                            int d[4];
                            bx_diffs(JR32 + (oy + (yk)) * JRP4 + (ox >> 2) + (qk), JRP4, W0, W1, s0, s1, s2, s3, IP[k], d, 256);
#pragma unroll
                            for (int i = 0; i < 4; i++)
                                if (4 * qk + i < w) PL[(yk - r0) * w + 4 * qk + i] = (float)abs(d[i]);
                        }
                        if (++qk == QW) {
                            qk = 0;
                            yk++;
                        }
                    }
                    __syncthreads();
                    if (tid == 0) acc = chain_sum(PL, tr * w, acc);
                }
                if (tid == 0) RS[8] = acc;
                __syncthreads();
                errval = RS[8];
            }
            errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * w * h));
        }
    }

#ifdef PSN_LK_STAMPS
    {
        unsigned long long t_end;
        BX_CLK(t_end);
        bx_acc[15] = t_end - bx_t0;
        unsigned long long r1;
        unsigned hwid, xcc;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1) : : "memory");
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (tid == 0 && A.stamps) {  // thread 0: also the chain lane of the tile stamps 12-14
            for (int i = 0; i < 16; i++) A.stamps[(size_t)g * 64 + i] = bx_acc[i];
            // residency: realtime (100 MHz) start / end and the CU it ran on
            A.stamps[(size_t)g * 64 + 16] = bx_r0;
            A.stamps[(size_t)g * 64 + 17] = r1;
            A.stamps[(size_t)g * 64 + 18] = ((unsigned long long)xcc << 32) | hwid;
        }
    }
#endif
    if (tid == 0) {
        if (FLG[6]) {  // a fallback hand-off timed out: the sums may be wrong -- say so
            NPx = NPy = errv = __builtin_nanf("");
            status = 0;
        }
        A.next[2 * pi] = NPx;
        A.next[2 * pi + 1] = NPy;
        A.status[pi] = (uint8_t)status;
        if (A.err) A.err[pi] = errv;
        if (A.samples) atomicAdd(A.samples, (unsigned long long)nwin * (unsigned)(w * h));
    }
}

hipError_t launch_lk_bx(const LkLaunchArgs &a, int total_wgs, int upt, bool notail, int lds_bytes, hipStream_t s) {
    if (total_wgs <= 0) return hipSuccess;
    const dim3 grid(total_wgs), block(kBxNT);
#define PSN_BX_CASE(U)                                                                              \
    case U:                                                                                         \
        if (notail)                                                                                 \
            hipLaunchKernelGGL((lk_kernel_bx<U, true>), grid, block, lds_bytes, s, a);              \
        else                                                                                        \
            hipLaunchKernelGGL((lk_kernel_bx<U, false>), grid, block, lds_bytes, s, a);             \
        break;
    switch (upt) {
        PSN_BX_CASE(4)
        PSN_BX_CASE(8)
        PSN_BX_CASE(10)
        PSN_BX_CASE(12)
        PSN_BX_CASE(16)
        default: return hipErrorInvalidValue;
    }
#undef PSN_BX_CASE
    return hipGetLastError();
}

hipError_t launch_lk(const LkLaunchArgs &a, int total_wgs, int threads, int lds_bytes, bool single_tile, hipStream_t s) {
    if (total_wgs <= 0) return hipSuccess;
    const dim3 grid(total_wgs);
    if (single_tile) {
        // threads encodes (workgroup size, pixels per thread, one-wave rows): E * 1000 + NT * 10 + EPT
        switch (threads) {
            case 642: hipLaunchKernelGGL((lk_kernel_st<64, 2, 0>), grid, dim3(64), lds_bytes, s, a); break;
            case 644: hipLaunchKernelGGL((lk_kernel_st<64, 4, 0>), grid, dim3(64), lds_bytes, s, a); break;
            case 1282: hipLaunchKernelGGL((lk_kernel_st<128, 2, 0>), grid, dim3(128), lds_bytes, s, a); break;
            case 1284: hipLaunchKernelGGL((lk_kernel_st<128, 4, 0>), grid, dim3(128), lds_bytes, s, a); break;
            case 2562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 0>), grid, dim3(256), lds_bytes, s, a); break;
            case 5121: hipLaunchKernelGGL((lk_kernel_st<512, 1, 0>), grid, dim3(512), lds_bytes, s, a); break;
            case 5122: hipLaunchKernelGGL((lk_kernel_st<512, 2, 0>), grid, dim3(512), lds_bytes, s, a); break;
            case 6562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 4>), grid, dim3(256), lds_bytes, s, a); break;
            case 9562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 7>), grid, dim3(256), lds_bytes, s, a); break;
            case 10562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 8>), grid, dim3(256), lds_bytes, s, a); break;
            case 10564: hipLaunchKernelGGL((lk_kernel_st<256, 4, 8>), grid, dim3(256), lds_bytes, s, a); break;
            case 18562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 16>), grid, dim3(256), lds_bytes, s, a); break;
            case 18564: hipLaunchKernelGGL((lk_kernel_st<256, 4, 16>), grid, dim3(256), lds_bytes, s, a); break;
            case 2564: hipLaunchKernelGGL((lk_kernel_st<256, 4, 0>), grid, dim3(256), lds_bytes, s, a); break;
            // one-wave kernels held to 168 VGPRs: three workgroups per CU when the
            // launch has more points than two per CU can hold (+200000)
            case 206562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 4, 3>), grid, dim3(256), lds_bytes, s, a); break;
            case 209562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 7, 3>), grid, dim3(256), lds_bytes, s, a); break;
            case 210562: hipLaunchKernelGGL((lk_kernel_st<256, 2, 8, 3>), grid, dim3(256), lds_bytes, s, a); break;
            default: return hipErrorInvalidValue;
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
    const void *st[] = {(const void *)lk_kernel_st<64, 2, 0>,   (const void *)lk_kernel_st<64, 4, 0>,
                        (const void *)lk_kernel_st<128, 2, 0>,  (const void *)lk_kernel_st<128, 4, 0>,
                        (const void *)lk_kernel_st<256, 2, 0>,  (const void *)lk_kernel_st<256, 4, 0>,
                        (const void *)lk_kernel_st<512, 1, 0>,  (const void *)lk_kernel_st<512, 2, 0>,
                        (const void *)lk_kernel_st<256, 2, 4>,  (const void *)lk_kernel_st<256, 2, 7>,
                        (const void *)lk_kernel_st<256, 2, 8>,  (const void *)lk_kernel_st<256, 4, 8>,
                        (const void *)lk_kernel_st<256, 2, 16>, (const void *)lk_kernel_st<256, 4, 16>,
                        (const void *)lk_kernel_st<256, 2, 4, 3>,  (const void *)lk_kernel_st<256, 2, 7, 3>,
                        (const void *)lk_kernel_st<256, 2, 8, 3>};
    for (const void *f : st)
        if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void *)pyramid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    const void *bx[] = {(const void *)lk_kernel_bx<4, false>, (const void *)lk_kernel_bx<8, false>,
                        (const void *)lk_kernel_bx<10, false>, (const void *)lk_kernel_bx<12, false>,
                        (const void *)lk_kernel_bx<4, true>, (const void *)lk_kernel_bx<8, true>,
                        (const void *)lk_kernel_bx<10, true>, (const void *)lk_kernel_bx<12, true>,
                        (const void *)lk_kernel_bx<16, false>, (const void *)lk_kernel_bx<16, true>};
    for (const void *f : bx)
        if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds)) != hipSuccess) return e;
    if ((e = lg_kernels_init()) != hipSuccess) return e;
    return gridfast_kernels_init();
}

}  // namespace psn
