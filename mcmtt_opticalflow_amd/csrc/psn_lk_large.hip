// lk_kernel_lg: LKTrackerInvoker (OpenCV 2.4.6, reached from
// PSNWhere_Tracker2D.cpp:776-782 backward and :871-877 forward) for windows the
// LDS-resident kernels cannot hold -- Tracker2D box windows of any size
// (forward w x h, backward w x w; e.g. 100x250 at 1080p, 128x320 at 4K).
//
// One workgroup per point, the grid striding over the launch's points; each
// workgroup owns an HBM slot for the window values of the current level
// ({I*, Ix* | Iy* << 16}, 8 B per window pixel, written once per level by the A
// phase and streamed by every iteration -- L2 / MALL resident for Tracker2D box
// sizes). LDS holds only one row band of the I patch, its Scharr plane and the
// chain-major product planes of the ordered-sum fallbacks, so several
// workgroups share a CU and hide each other's serial chains. J is read straight
// from the pyramid level (reflect-101 addressing off the image interior).
//
// Arithmetic and summation order are those of lk_kernel (psn_lk_kernels.hip):
// integer window sums with the subset-sum exactness bound, otherwise the SSE2
// chains summed in order, one lane per chain, band by band. Bit-identical to
// oracle/lk_oracle.c.
#include "psn_lk_device.h"

namespace psn {

// bilinear J (DESCALE 9) at a window pixel whose 2x2 taps are inside the level
__device__ __forceinline__ int lg_j_in(const uint8_t *p, int pitch, int w00, int w01, int w10, int w11) {
    return PSN_DESCALE(p[0] * w00 + p[1] * w01 + p[pitch] * w10 + p[pitch + 1] * w11, 9);
}
// the same at level coordinates (gy, gx) with reflect-101 taps (the padded J
// buffer of calcOpticalFlowPyrLK: copyMakeBorder(..., BORDER_REFLECT_101))
__device__ __forceinline__ int lg_j_refl(const LevelDev &J, int gy, int gx, int w00, int w01, int w10, int w11) {
    const uint8_t *r0 = J.p + (long long)refl101(gy, J.h) * J.pitch;
    const uint8_t *r1 = J.p + (long long)refl101(gy + 1, J.h) * J.pitch;
    const int x0 = refl101(gx, J.w), x1 = refl101(gx + 1, J.w);
    return PSN_DESCALE(r0[x0] * w00 + r0[x1] * w01 + r1[x0] * w10 + r1[x1] * w11, 9);
}

// J - I* and the gradients of window pixel (y, x), idx = y * w + x
struct LgIter {
    const uint8_t *jb;  // J at the window origin (interior only)
    LevelDev J;
    int pitch, iny, inx, w00, w01, w10, w11;
    bool in;
    __device__ __forceinline__ int jval(int y, int x) const {
        return in ? lg_j_in(jb + (long long)y * pitch + x, pitch, w00, w01, w10, w11)
                  : lg_j_refl(J, iny + y, inx + x, w00, w01, w10, w11);
    }
};
__device__ __forceinline__ LgIter lg_iter(const LevelDev &J, int inx, int iny, int w, int h, int w00, int w01, int w10,
                                          int w11) {
    LgIter it;
    it.J = J;
    it.pitch = J.pitch;
    it.inx = inx;
    it.iny = iny;
    it.w00 = w00;
    it.w01 = w01;
    it.w10 = w10;
    it.w11 = w11;
    // the taps of every window pixel: columns inx .. inx + w, rows iny .. iny + h
    it.in = inx >= 0 && iny >= 0 && inx + w + 1 <= J.w && iny + h + 1 <= J.h;
    it.jb = it.in ? J.p + (long long)iny * J.pitch + inx : J.p;
    return it;
}
__device__ __forceinline__ int lg_gx(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int lg_gy(int v) { return v >> 16; }

// Diagnostic phase clocks (PSN_LK_STAMPS build, tools/lg_stamps.py): accumulated
// s_memtime ticks per phase of each point, thread 0's view, stamps[point][0..15].
#ifdef PSN_LK_STAMPS
#define LG_CLK(t) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory")
#define LG_MARK(i)                    \
    do {                              \
        unsigned long long t_;        \
        LG_CLK(t_);                   \
        lg_acc[i] += t_ - lg_t;       \
        lg_t = t_;                    \
    } while (0)
#define LG_COUNT(i) lg_acc[i]++
#else
#define LG_MARK(i) \
    do {           \
    } while (0)
#define LG_COUNT(i) \
    do {            \
    } while (0)
#endif

template <int NT>
__global__ __launch_bounds__(NT) void lk_kernel_lg(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    float *RED = (float *)smem;
    int *REDI = (int *)(RED + 48);  // 16 ints of block-reduce scratch
    int2 *WV = A.lg_ws + (long long)blockIdx.x * A.lg_slot;
    const float FLT_SCALE = 1.f / (1 << 20);

    for (int g = blockIdx.x; g < A.lk_wgs; g += gridDim.x) {
        int qi = 0;
        while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
        const LkQueryDev &Q = A.q[qi];
        if (A.counts && g - Q.wg_begin >= A.counts[Q.qidx]) continue;  // past the query's device count
        const int pi = Q.pt_begin + (g - Q.wg_begin);
        const int w = Q.win_w, h = Q.win_h, wh = w * h;
        const int TR = Q.tile_rows;
        const int maxL = Q.max_level, flags = Q.flags;
        const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
        const int PW = w + 3, DW = w + 1;
        uint8_t *Pimg = smem + lg_off_pimg();
        short2 *Dg = (short2 *)(smem + lg_off_dg(w, TR));
        float *Prod = (float *)(smem + lg_off_prod(w, TR));

        const float hwx = __fmul_rn((float)(w - 1), 0.5f), hwy = __fmul_rn((float)(h - 1), 0.5f);
        const float px0 = A.prev[2 * pi], py0 = A.prev[2 * pi + 1];
        float NPx = 0.f, NPy = 0.f;
        if (flags & PSN_LK_USE_INITIAL_FLOW) {
            NPx = A.next[2 * pi];
            NPy = A.next[2 * pi + 1];
        }
        int status = 1;
        float errv = 0.f;
        unsigned nwin = 0;  // window passes (A phase + iterations): the sample count / (w*h)
#ifdef PSN_LK_STAMPS
        unsigned long long lg_acc[16] = {}, lg_t = 0, lg_t0 = 0;
        LG_CLK(lg_t0);
        lg_t = lg_t0;
#endif

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

            // ---- A phase, band by band: I patch rows -> Scharr -> window values
            // into the HBM slot, integer structure-tensor sums ----
            nwin++;
            int sA11 = 0, sA12 = 0;
            unsigned aA12 = 0, sA22 = 0;
            for (int r0 = 0; r0 < h; r0 += TR) {
                const int th = min(TR, h - r0);
                __syncthreads();  // the previous band's (level's, point's) LDS readers are done
                stage_one<NT>(Pimg, I, ipy + r0 - 1, ipx - 1, PW, th + 3);
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
                {
                    Walk wk;
                    wk.init(tid, NT, w);
                    for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                        const int yl = wk.y, x = wk.x;
                        const uint8_t *p = Pimg + (yl + 1) * PW + x + 1;
                        const int ival = PSN_DESCALE(p[0] * iw00 + p[1] * iw01 + p[PW] * iw10 + p[PW + 1] * iw11, 9);
                        const short2 *d = Dg + yl * DW + x;
                        const int ixv = PSN_DESCALE(d[0].x * iw00 + d[1].x * iw01 + d[DW].x * iw10 + d[DW + 1].x * iw11, 14);
                        const int iyv = PSN_DESCALE(d[0].y * iw00 + d[1].y * iw01 + d[DW].y * iw10 + d[DW + 1].y * iw11, 14);
                        WV[r0 * w + idx] = make_int2(ival, (ixv & 0xffff) | (iyv << 16));
                        const int xy = ixv * iyv;
                        sA11 = (int)sat_add((unsigned)sA11, (unsigned)(ixv * ixv));
                        sA12 += xy;
                        aA12 = sat_add(aA12, (unsigned)abs(xy));
                        sA22 = sat_add(sA22, (unsigned)(iyv * iyv));
                    }
                }
            }
            // (the reduce's barrier also publishes the slot's window values to the workgroup)
            block_reduce4<NT, true>(sA11, sA12, aA12, sA22, REDI);
            LG_MARK(0);  // A phase: I bands, Scharr, window values, integer sums
            const bool ex11 = sA11 <= kExact, ex12 = aA12 <= (unsigned)kExact, ex22 = sA22 <= (unsigned)kExact;
            float A11 = (float)sA11, A12 = (float)sA12, A22 = (float)sA22;
            if (!(ex11 && ex12 && ex22)) {
                // ordered float chains over (float)(Ix*Ix), (float)(Ix*Iy), (float)(Iy*Iy)
                float acc = 0.f;
                for (int r0 = 0; r0 < h; r0 += TR) {
                    const int th = min(TR, h - r0);
                    const ChainA C(w, th, sse);
                    __syncthreads();  // chain lanes done with the previous band
                    Walk wk;
                    wk.init(tid, NT, w);
                    for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                        const int v = WV[r0 * w + idx].y;
                        const int gx = lg_gx(v), gy = lg_gy(v);
                        const int pos = C.pos(wk.y, wk.x);
                        Prod[pos] = (float)(gx * gx);
                        Prod[C.P + pos] = (float)(gx * gy);
                        Prod[2 * C.P + pos] = (float)(gy * gy);
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
                __syncthreads();  // RED read by all before any later write
            }
            LG_MARK(1);  // A ordered chains
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
                nwin++;
                int w00, w01, w10, w11;
                bilin_weights(__fsub_rn(nx, (float)inx), __fsub_rn(ny, (float)iny), w00, w01, w10, w11);
                const LgIter it = lg_iter(J, inx, iny, w, h, w00, w01, w10, w11);
                int s1 = 0, s2 = 0;
                unsigned a1 = 0, a2 = 0;
                {
                    Walk wk;
                    wk.init(tid, NT, w);
#pragma unroll 2
                    for (int idx = tid; idx < wh; idx += NT, wk.step()) {
                        const int2 v = WV[idx];
                        const int diff = it.jval(wk.y, wk.x) - v.x;
                        const int t1 = diff * lg_gx(v.y), t2 = diff * lg_gy(v.y);
                        s1 += t1;
                        s2 += t2;
                        a1 = sat_add(a1, (unsigned)abs(t1));
                        a2 = sat_add(a2, (unsigned)abs(t2));
                    }
                }
                LG_MARK(2);  // main pass
                LG_COUNT(10);
                block_reduce4<NT, false>(s1, s2, a1, a2, REDI);
                LG_MARK(3);  // reduce
                float b1, b2;
                if (sums_exact(a1, s1) && sums_exact(a2, s2)) {  // subset-sum bound (see sums_exact)
                    b1 = (float)s1;
                    b2 = (float)s2;
                } else {
                    LG_COUNT(11);
                    float bacc = 0.f;
                    for (int r0 = 0; r0 < h; r0 += TR) {
                        const int th = min(TR, h - r0);
                        const ChainB C(w, th, sse);
                        __syncthreads();  // chain lanes done with the previous band / reduce scratch
                        Walk wk;
                        wk.init(tid, NT, w);
                        for (int idx = tid; idx < th * w; idx += NT, wk.step()) {
                            const int2 v = WV[r0 * w + idx];
                            const int diff = it.jval(r0 + wk.y, wk.x) - v.x;
                            const int pos = C.pos(wk.y, wk.x);
                            Prod[pos] = (float)(diff * lg_gx(v.y));
                            Prod[C.P + pos] = (float)(diff * lg_gy(v.y));
                        }
                        __syncthreads();
                        LG_MARK(4);  // fallback: band products
                        if (tid < 10) {
                            const int ch = tid % 5, s = tid / 5;
                            const int base = ch < 4 ? ch * C.SB : 4 * C.SB;
                            const int len = ch < 4 ? th * 2 * C.nB : th * C.tB;
                            bacc = chain_sum(Prod + s * C.P + base, len, bacc);
                        }
                        LG_MARK(5);  // fallback: chain sums
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
                LG_MARK(6);  // results
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
                const LgIter it = lg_iter(J, iqx, iqy, w, h, w00, w01, w10, w11);
                int e0 = 0, e1 = 0;
                unsigned e2 = 0, e3 = 0;
                {
                    Walk wk;
                    wk.init(tid, NT, w);
                    for (int idx = tid; idx < wh; idx += NT, wk.step())
                        e2 = sat_add(e2, (unsigned)abs(it.jval(wk.y, wk.x) - WV[idx].x));
                }
                block_reduce4<NT, false>(e0, e1, e2, e3, REDI);
                float errval;
                if (e2 <= (unsigned)kExact) {
                    // every partial sum of errval += |diff| is an integer <= 2^24: exact
                    errval = (float)e2;
                } else {  // row-major order, one lane, band by band
                    float eacc = 0.f;
                    for (int r0 = 0; r0 < h; r0 += TR) {
                        const int th = min(TR, h - r0);
                        __syncthreads();
                        Walk wk;
                        wk.init(tid, NT, w);
                        for (int idx = tid; idx < th * w; idx += NT, wk.step())
                            Prod[idx] = (float)abs(it.jval(r0 + wk.y, wk.x) - WV[r0 * w + idx].x);
                        __syncthreads();
                        if (tid == 0) eacc = chain_sum(Prod, th * w, eacc);
                    }
                    if (tid == 0) RED[32] = eacc;
                    __syncthreads();
                    errval = RED[32];
                    __syncthreads();  // RED read by all before any later write
                }
                errv = __fdiv_rn(__fmul_rn(errval, 1.f), (float)(32 * w * h));
            }
        }

#ifdef PSN_LK_STAMPS
        {
            unsigned long long t_end;
            LG_CLK(t_end);
            lg_acc[15] = t_end - lg_t0;
            if (tid == 0 && A.stamps)
                for (int i = 0; i < 16; i++) A.stamps[(size_t)g * 64 + i] = lg_acc[i];
        }
#endif
        if (tid == 0) {
            A.next[2 * pi] = NPx;
            A.next[2 * pi + 1] = NPy;
            A.status[pi] = (uint8_t)status;
            if (A.err) A.err[pi] = errv;
            if (A.samples) atomicAdd(A.samples, (unsigned long long)nwin * (unsigned)wh);
        }
        __syncthreads();  // the next point reuses the slot, the bands and the reduce scratch
    }
}

hipError_t launch_lk_lg(const LkLaunchArgs &a, int grid, int lds_bytes, hipStream_t s) {
    if (grid <= 0 || a.lk_wgs <= 0) return hipSuccess;
    if (!a.lg_ws || a.lg_slot <= 0 || lds_bytes > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lk_kernel_lg<kLgNT>, dim3(grid), dim3(kLgNT), lds_bytes, s, a);
    return hipGetLastError();
}

hipError_t lg_kernels_init() {
    return hipFuncSetAttribute((const void *)lk_kernel_lg<kLgNT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

}  // namespace psn
