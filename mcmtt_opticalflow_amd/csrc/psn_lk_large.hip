// lk_kernel_lg: LKTrackerInvoker (OpenCV 2.4.6, reached from
// PSNWhere_Tracker2D.cpp:776-782 backward and :871-877 forward) for the box
// windows the box kernel cannot hold in registers -- Tracker2D windows of any
// size (forward w x h, backward w x w; PETS-scale 100x250 at 1080p, 128x320 at
// 4K).
//
// The structure of lk_kernel_bx (psn_lk_kernels.hip) with the window values
// streamed instead of register-resident. One workgroup (4 waves) per point, the
// grid striding over the launch's points. The window is cut into quads (row y,
// 4 pixels) in row-major order; thread t owns the CONTIGUOUS quads [t*K, t*K+K),
// so for every SSE2 lane chain and the scalar tail chain its terms form one
// contiguous run of the chain. Per level the A phase writes every quad's window
// values -- (I*, Ix*, Iy*) of 4 pixels as packed 16-bit pairs, 24 B -- into the
// workgroup's HBM slot (laid out [j][t], so thread t's j-th quads are one
// coalesced load), and every iteration streams them back (L2 / MALL resident)
// with the quad's J rows as two aligned dwords per row (packed-dot bilinear as
// in lk_kernel_bx). Exactness of each float sum per chain by the run records
// (total, maximum / minimum prefix) through one block scan; otherwise the
// ordered chains from the first inexact half wave on, over tiles of consecutive
// quads whose products are written chain-major into double-buffered LDS planes
// while wave 0's chain lanes sum the previous tile. LDS holds only the tiles
// (and, in the A phase, one row band of the I patch and its Scharr plane), so
// several workgroups share a CU and hide each other's serial chains.
//
// Bit-identical to oracle/lk_oracle.c (the SSE2 build's summation order, or the
// scalar build's with PSN_LK_ACCUM_SCALAR).
#include "psn_lk_xb.h"

// (PSN_LG_XB, psn_lk_kernels.h: the b fallback by parity records before the
// ordered tiles -- a build parameter, 0 = the tiles only)

namespace psn {

// pair selector: bytes (s, s + 1) of a row's 8-byte window -> J[x] | J[x+1] << 16
__device__ __forceinline__ unsigned lg_sel(int s) { return 0x0c000c00u | ((unsigned)(s + 1) << 16) | (unsigned)s; }

// Window geometry: quads per row, quads, quads per thread; the SSE2 chain split
// of the b sums (8-pixel steps: nB2 quads per row, n8 pixels, tB tail pixels)
// and of the A sums (4-pixel steps: nA quads, tA tail pixels).
struct LgGeo {
    int w, h, QW, NQ, K;
    int nB2, n8, tB, nA, tA;
    float rQW, rK;  // 1 / QW, 1 / K (lg_div)
};
// n / d for 0 <= n < 2^24 (quad indices; the planner keeps windows below 2^22
// quads) by the float reciprocal r = 1 / d and one correction step
__device__ __forceinline__ int lg_div(int n, int d, float r) {
    int t = (int)__fmul_rn((float)n, r);
    const int m = n - t * d;
    t += m < 0 ? -1 : (m >= d ? 1 : 0);
    return t;
}
__device__ __forceinline__ LgGeo lg_geo(int w, int h, bool sse) {
    LgGeo g;
    g.w = w;
    g.h = h;
    g.QW = (w + 3) >> 2;
    g.NQ = h * g.QW;
    g.K = (g.NQ + kLgNT - 1) / kLgNT;
    g.nB2 = sse ? 2 * (w / 8) : 0;
    g.n8 = 4 * g.nB2;
    g.tB = w - g.n8;
    g.nA = sse ? w / 4 : 0;
    g.tA = w - 4 * g.nA;
    g.rQW = __fdiv_rn(1.f, (float)g.QW);
    g.rK = __fdiv_rn(1.f, (float)g.K);
    return g;
}
// terms of the SSE chains (one per SSE quad) and of the tail chain before quad q
__device__ __forceinline__ int lg_sse_before(const LgGeo &g, int q, int nS) {
    const int y = lg_div(q, g.QW, g.rQW);
    return y * nS + min(q - y * g.QW, nS);
}
__device__ __forceinline__ int lg_tail_before(const LgGeo &g, int q, int nS, int t) {
    const int y = lg_div(q, g.QW, g.rQW);
    return y * t + min(max(4 * (q - y * g.QW - nS), 0), t);
}

// One quad's J - I* (4 pixels) at window row y, quad column qx: from the LDS copy
// of the J region (lds), or from the level (in: every tap inside it).
struct LgJ {
    const uint32_t *jl;  // lds: the region's dword holding the window origin
    const uint8_t *jb;   // in: J at the window origin aligned down to a dword
    LevelDev J;
    int inx, iny, pitch, jrp4;
    unsigned W0, W1, s[4];
    int w00, w01, w10, w11;
    bool lds, in;
};
__device__ __forceinline__ LgJ lg_j(const LevelDev &J, int inx, int iny, int w, int h, int w00, int w01, int w10,
                                    int w11, const uint32_t *jr, int jrp4, int jr_x0, int jr_y0) {
    LgJ r;
    r.J = J;
    r.inx = inx;
    r.iny = iny;
    r.pitch = J.pitch;
    r.jrp4 = jrp4;
    r.w00 = w00;
    r.w01 = w01;
    r.w10 = w10;
    r.w11 = w11;
    r.W0 = pack_w(w00, w01);
    r.W1 = pack_w(w10, w11);
    r.lds = jr != nullptr;
    // every tap of the window (columns inx .. inx + w, rows iny .. iny + h) inside the level
    r.in = inx >= 0 && iny >= 0 && inx + w + 1 <= J.w && iny + h + 1 <= J.h;
    int sh = r.in ? (inx & 3) : 0;
    if (r.lds) {
        const int ox = inx - jr_x0;
        sh = ox & 3;
        r.jl = jr + (iny - jr_y0) * jrp4 + (ox >> 2);
    } else {
        r.jl = nullptr;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) r.s[i] = lg_sel(sh + i);
    r.jb = r.in ? J.p + (long long)iny * J.pitch + (inx - sh) : J.p;
    return r;
}
// d[i] = DESCALE(bilinear J, 9) - I of the quad's pixels (ip: I* as packed pairs);
// the diff is folded into the dot product's accumulator: (v + 256 - 512 I) >> 9.
// Taps outside the level take their reflect-101 source (the padded J buffer of
// calcOpticalFlowPyrLK: copyMakeBorder(..., BORDER_REFLECT_101)); the LDS copy
// holds them already (dma_patch).
__device__ __forceinline__ void lg_diffs(const LgJ &J, int y, int qx, const uint2 &ip, int (&d)[4]) {
    const int I[4] = {lo16(ip.x), hi16(ip.x), lo16(ip.y), hi16(ip.y)};
    if (J.lds || J.in) {
        uint32_t a0, a1, b0, b1;
        if (J.lds) {
            const uint32_t *r0 = J.jl + y * J.jrp4 + qx;
            a0 = r0[0];
            a1 = r0[1];
            b0 = r0[J.jrp4];
            b1 = r0[J.jrp4 + 1];
        } else {
            const uint32_t *r0 = (const uint32_t *)(J.jb + (long long)y * J.pitch + 4 * qx);
            const uint32_t *r1 = (const uint32_t *)((const uint8_t *)r0 + J.pitch);
            a0 = r0[0];
            a1 = r0[1];
            b0 = r1[0];
            b1 = r1[1];
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
            d[i] = sdot2(__builtin_amdgcn_perm(b1, b0, J.s[i]), J.W1,
                         sdot2(__builtin_amdgcn_perm(a1, a0, J.s[i]), J.W0, 256 - 512 * I[i])) >> 9;
    } else {  // a window reaching past the level: reflect-101 taps, pixel by pixel
        const uint8_t *r0 = J.J.p + (long long)refl101(J.iny + y, J.J.h) * J.pitch;
        const uint8_t *r1 = J.J.p + (long long)refl101(J.iny + y + 1, J.J.h) * J.pitch;
#pragma unroll 1
        for (int i = 0; i < 4; i++) {
            const int xa = refl101(J.inx + 4 * qx + i, J.J.w), xb = refl101(J.inx + 4 * qx + i + 1, J.J.w);
            d[i] = PSN_DESCALE(r0[xa] * J.w00 + r0[xb] * J.w01 + r1[xa] * J.w10 + r1[xb] * J.w11, 9) - I[i];
        }
    }
}

// LDS tile planes of the ordered-chain fallbacks (psn_lk_kernels.h): per plane 4
// SSE chain regions of up to TQ terms and a tail region of up to 4*TQ terms
// (16-float blocks + 4: conflict-free across the chain lanes' 16-B reads)

// One quad's window values as the fallback writers hold them between tiles.
struct LgQ {
    uint2 ip, xp, yp;
};

// Ordered chains from quad qs on, tile by tile: waves 1-3 write a tile's products
// (one quad per thread: `load(q)` fetches quad q's window values, `store(v, q,
// tile start, buffer)` writes its products), chain lanes (wave 0, lanes < NCH)
// sum the previous tile meanwhile; double-buffered, one barrier per tile, each
// writer's loads for tile g+2 in flight while tile g is summed. `before(q, s, t)`
// gives the SSE / tail chain terms before quad q (uniform); a chain lane zeroes
// the 16-float block holding the end of its region for tile g+2 right after
// summing tile g from the same buffer (the writers fill the block's front a
// barrier later). Returns acc (chain lanes: their chain's sum onto its base).
template <int NPL, int TQ, typename Load, typename Store, typename Before, typename Mark>
__device__ __forceinline__ float lg_tiles(int qs, int NQ, float *buf, int nch, float acc, Load load, Store store,
                                          Before before, Mark mark) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int PL = lg_plane(TQ), SR = lg_sreg(TQ);
    const bool chl = tid < nch;
    const int cs = lane / 5, cc = lane - 5 * cs;
    const int ntiles = (NQ - qs + TQ - 1) / TQ;
    if (ntiles <= 0) return acc;
    auto region = [&](float *b) { return b + cs * PL + (cc < 4 ? cc * SR : 4 * SR); };
    // chain terms before tile boundaries g .. g+3 (uniform), rolled per tile
    int bs[4], bt[4];
#pragma unroll
    for (int i = 0; i < 4; i++) before(min(qs + i * TQ, NQ), bs[i], bt[i]);
    auto pad = [&](int i0, float *b) {  // the tile between boundaries i0, i0 + 1
        if (!chl) return;
        const int len = cc < 4 ? bs[i0 + 1] - bs[i0] : bt[i0 + 1] - bt[i0];
        if (len & 15) {
            float4 *z = (float4 *)(region(b) + (len & ~15));
            const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
            z[0] = zero;
            z[1] = zero;
            z[2] = zero;
            z[3] = zero;
        }
    };
    // writer thread tid (waves 1-3) takes quad tid - 64 of each tile
    auto quad_of = [&](int g) { return tid >= 64 && tid - 64 < TQ ? qs + g * TQ + tid - 64 : NQ; };
    pad(0, buf);
    if (ntiles > 1) pad(1, buf + NPL * PL);
    __syncthreads();
    LgQ v{};
    int q = quad_of(0);
    if (q < NQ) store(load(q), q, qs, buf);
    q = quad_of(1);
    if (q < NQ) v = load(q);
    __syncthreads();
    for (int g = 0; g < ntiles; g++) {
        float *cur = buf + (g & 1) * NPL * PL, *nxt = buf + ((g + 1) & 1) * NPL * PL;
        if (g + 1 < ntiles) {
            if (q < NQ) store(v, q, qs + (g + 1) * TQ, nxt);
            q = quad_of(g + 2);
            if (q < NQ) v = load(q);
        }
        if (tid < 64) {
            const int ns = bs[1] - bs[0], nt = bt[1] - bt[0];
            const int len = chl ? (cc < 4 ? ns : nt) : 0;
            const int nbmax = (max(ns, nt) + 15) >> 4;
            mark(2);
            if (chl) acc = chain_sum_pl<false>(region(cur), len, nbmax, acc);
            mark(3);
            if (g + 2 < ntiles) pad(2, cur);
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            bs[i] = bs[i + 1];
            bt[i] = bt[i + 1];
        }
        before(min(qs + (g + 4) * TQ, NQ), bs[3], bt[3]);
        mark(0);
        __syncthreads();
        mark(1);
    }
    return acc;
}

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

constexpr int kLgMB = 4;  // quads per batch of slot loads in the passes over the window

// Minimum waves per SIMD of the build (__launch_bounds__: k workgroups per CU of
// 256 threads = k waves per SIMD; a build parameter for occupancy A/Bs)
#ifndef PSN_LG_WAVES
#define PSN_LG_WAVES 1
#endif
// TQ: quads per ordered-chain tile (kLgTQs; the planner's choice per query)
template <int TQ>
__global__ __launch_bounds__(kLgNT, PSN_LG_WAVES) void lk_kernel_lg(LkLaunchArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NT = kLgNT;
    const int tid = threadIdx.x, lane = tid & 63;
    if (A.poison_lds) lds_poison<NT>(smem, A.poison_lds);
    int *X = (int *)smem;                 // chain-check records, two parities
    float *RS = (float *)(X + kBxXInts);  // results (wave 0 -> all), err partials
    int *EP = (int *)(RS + 16);
    uint8_t *U = smem + lg_scr_bytes();   // band staging | tile planes
    float *PL = (float *)U;
    uint32_t *JR = (uint32_t *)(U + lg_iter_region(TQ));  // J region (lg_jr), after the b tiles / run records
#if PSN_LG_XB
    int2 *XREC = (int2 *)U;  // b fallback run records [chain][thread]
#endif
    uint8_t *const slot = (uint8_t *)A.lg_ws + (long long)blockIdx.x * A.lg_slot * 8;
    const float FLT_SCALE = 1.f / (1 << 20);
    int par = 0;

    for (int gi = blockIdx.x; gi < A.lk_wgs; gi += gridDim.x) {
        const int g = gi;
        int qi = 0;
        while (qi + 1 < A.nq && g >= A.q[qi + 1].wg_begin) qi++;
        const LkQueryDev &Q = A.q[qi];
        const int pi = lk_query_point(Q, A.counts, A.count_stride, g);
        if (pi < 0) continue;  // past the query's device count
        const int w = Q.win_w, h = Q.win_h, TR = Q.tile_rows;
        const int maxL = Q.max_level, flags = Q.flags;
        const bool sse = (flags & PSN_LK_ACCUM_SCALAR) == 0;
        const LgGeo G = lg_geo(w, h, sse);
        const int K = G.K, QW = G.QW, NQ = G.NQ;
        uint2 *IPs = (uint2 *)slot, *XPs = IPs + NT * K, *YPs = XPs + NT * K;
        const int q0 = min(tid * K, NQ), cnt = min(NQ - q0, K);  // this thread's quads [q0, q0 + cnt)
        const int y0 = q0 / QW, x0 = q0 - y0 * QW;
        const int PM = bx_pm(w);  // I patch dwords per row
        const bool jrm = Q.lg_jr != 0;
        const int JRW = st_jreg_w(w), JRH = st_jreg_h(h), JRP4 = bx_jrp(w) >> 2;
#if PSN_LG_XB
        float *POOL = (float *)((uint8_t *)JR + (jrm ? lg_jr_bytes(w, h) : 0));  // HARD runs' terms
#endif
        uint8_t *Pimg = U;

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
        unsigned long long lg_acc[24] = {}, lg_t = 0, lg_t0 = 0;
        LG_CLK(lg_t0);
        lg_t = lg_t0;
#endif

        for (int level = maxL; level >= 0; level--) {
            const LevelDev I = ring_level_u(A.ring, Q.prev_slot, level);
            const LevelDev J = ring_level_u(A.ring, Q.next_slot, level);
            const int cols = I.w, rows = I.h;
            const float scale = ldexpf(1.f, -level);
            // the LDS copy of the J region around the window (lg_jr): restaged when the
            // window at (inx, iny) leaves it (the A phase's bands and tiles reuse its LDS)
            bool jr_valid = false;
            int jr_x0 = 0, jr_y0 = 0;
            auto window_j = [&](int inx, int iny, int w00, int w01, int w10, int w11) {
                if (jrm && !(jr_valid && inx >= jr_x0 && iny >= jr_y0 && inx + w + 1 <= jr_x0 + JRW &&
                             iny + h + 1 <= jr_y0 + JRH)) {
                    // every reader of the previous copy passed a barrier since
                    jr_x0 = (inx - kStJMargin) & ~3;
                    jr_y0 = iny - kStJMargin;
                    dma_patch<NT>((uint8_t *)JR, J, jr_y0, jr_x0, JRW, JRH, JRP4, Q.dv_bxjr);
                    dma_wait();
                    __syncthreads();
                    jr_valid = true;
                }
                return lg_j(J, inx, iny, w, h, w00, w01, w10, w11, jrm ? JR : nullptr, JRP4, jr_x0, jr_y0);
            };
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
            nwin++;

            // ---- A phase (1): window values, band by band: the band's I patch rows
            // by LDS-DMA, then each quad's Scharr + bilinear values (bx_unit) into
            // the slot ----
            {
                const int sh = (ipx - 1) & 3;
                const bool interior = ipx >= 0 && ipy >= 0 && ipx + 4 * QW + 2 <= cols && ipy + h + 1 <= rows;
                const int c256 = 1 << 8, c8192 = 1 << 13;
                const uint32_t *P32 = (const uint32_t *)Pimg;
                int gdum0 = 0, gdum1 = 0;  // (the A runs below track the gradients)
                auto band = [&](auto inner) {
                    constexpr bool IN = decltype(inner)::value;
                    for (int r0 = 0; r0 < h; r0 += TR) {
                        const int th = min(TR, h - r0);
                        __syncthreads();  // the previous band's (tile's, level's, point's) LDS readers are done
                        dma_rows<NT>(Pimg, I, ipy + r0 - 1, ipx - 1, w + 3, th + 3, PM);
                        dma_wait();
                        __syncthreads();
                        LG_MARK(7);  // band staging
                        Walk wk;
                        wk.init(tid, NT, QW);
                        for (int qb = tid; qb < th * QW; qb += NT, wk.step()) {
                            unsigned ip[2], xp[2], yp[2];
                            bx_unit<IN, false>(P32, PM, sh, wk.y, wk.x, true, w, ipx, ipy + r0, cols, rows, iw00, iw01,
                                               iw10, iw11, c256, c8192, ip, xp, yp, gdum0, gdum1);
                            const int q = (r0 + wk.y) * QW + wk.x, t = lg_div(q, K, G.rK), idx = (q - t * K) * NT + t;
                            IPs[idx] = make_uint2(ip[0], ip[1]);
                            XPs[idx] = make_uint2(xp[0], xp[1]);
                            YPs[idx] = make_uint2(yp[0], yp[1]);
                        }
                        LG_MARK(9);  // band quads
                    }
                };
                if (interior)
                    band(std::true_type());
                else
                    band(std::false_type());
            }
            __syncthreads();  // the window values of every band for every thread
            LG_MARK(0);  // A phase: window values

            // ---- A phase (2): the 15 A chains (sum x class) as runs over the
            // thread's quads, the block check, ordered chains if inexact ----
            float A11, A12, A22;
            int gmax = 0;  // max |Ix|, |Iy| of the thread's pixels (exactness of the b terms)
            {
                int T11[5] = {0, 0, 0, 0, 0}, T22[5] = {0, 0, 0, 0, 0}, T12[5] = {0, 0, 0, 0, 0};
                int M12[5] = {0, 0, 0, 0, 0}, m12[5] = {0, 0, 0, 0, 0};
                int qx = x0;
                auto quad = [&](const uint2 &xp, const uint2 &yp) {
                    const int gx[4] = {lo16(xp.x), hi16(xp.x), lo16(xp.y), hi16(xp.y)};
                    const int gy[4] = {lo16(yp.x), hi16(yp.x), lo16(yp.y), hi16(yp.y)};
                    // (A11 / A22 runs saturate at 2^30: a long run never wraps; a run past 2^25
                    // fails the check below, as it must)
                    if (qx < G.nA) {  // SSE2 quad: pixel i feeds lane chain i
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            T11[i] = (int)sat_add((unsigned)T11[i], (unsigned)(gx[i] * gx[i]));
                            T22[i] = (int)sat_add((unsigned)T22[i], (unsigned)(gy[i] * gy[i]));
                            run_add(T12[i], M12[i], m12[i], gx[i] * gy[i]);
                        }
                    } else {  // the tail chain, in order (pixels past w carry zero gradients)
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            T11[4] = (int)sat_add((unsigned)T11[4], (unsigned)(gx[i] * gx[i]));
                            T22[4] = (int)sat_add((unsigned)T22[4], (unsigned)(gy[i] * gy[i]));
                            run_add(T12[4], M12[4], m12[4], gx[i] * gy[i]);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) gmax = max(gmax, max(abs(gx[i]), abs(gy[i])));
                    if (++qx == QW) qx = 0;
                };
                int k = 0;
                for (; k + kLgMB <= cnt; k += kLgMB) {
                    uint2 xp[kLgMB], yp[kLgMB];
#pragma unroll
                    for (int u = 0; u < kLgMB; u++) {
                        xp[u] = XPs[(k + u) * NT + tid];
                        yp[u] = YPs[(k + u) * NT + tid];
                    }
#pragma unroll
                    for (int u = 0; u < kLgMB; u++) quad(xp[u], yp[u]);
                }
                for (; k < cnt; k++) quad(XPs[k * NT + tid], YPs[k * NT + tid]);
                // A11 / A22 terms are >= 0: the maximum prefix is the total
                int T[15], M[15], m[15];
#pragma unroll
                for (int c = 0; c < 5; c++) {
                    T[c] = T11[c], M[c] = T11[c], m[c] = 0;
                    T[5 + c] = T12[c], M[5 + c] = M12[c], m[5 + c] = m12[c];
                    T[10 + c] = T22[c], M[10 + c] = T22[c], m[10 + c] = 0;
                }
                // a run whose own prefix leaves [-2^25, 2^25] cannot stay exact after any
                // exact start (|start| <= 2^24): flag it (long runs never wrap unseen)
                bool badA = false;
#pragma unroll
                for (int c = 0; c < 15; c++) badA |= M[c] > (1 << 25) || m[c] < -(1 << 25);
                int *rec = X + par * 4 * kBxRecInts;
                par ^= 1;
                bx_publish<15>(T, rec, G.tA == 0);
                __syncthreads();
                bx_check_t<15>(T, M, m, badA, rec, G.tA == 0);
                __syncthreads();
                int tot, h0, base0;
                const bool exact = bx_eval_t<15>(rec, tot, h0, base0);
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
                    // ordered chains from thread h0's run on (every earlier prefix is an
                    // exact integer: the chain lanes start from base0)
                    const int qs = min(h0 * K, NQ);
                    auto geoA = [&](int q, int &bs, int &bt) {
                        bs = lg_sse_before(G, q, G.nA);
                        bt = lg_tail_before(G, q, G.nA, G.tA);
                    };
                    auto loadA = [&](int q) {
                        const int t = lg_div(q, K, G.rK), idx = (q - t * K) * NT + t;
                        LgQ v;
                        v.xp = XPs[idx];
                        v.yp = YPs[idx];
                        return v;
                    };
                    auto storeA = [&](const LgQ &v, int q, int a, float *buf) {
                        const int gx[4] = {lo16(v.xp.x), hi16(v.xp.x), lo16(v.xp.y), hi16(v.xp.y)};
                        const int gy[4] = {lo16(v.yp.x), hi16(v.yp.x), lo16(v.yp.y), hi16(v.yp.y)};
                        const int PLA = lg_plane(TQ), SR = lg_sreg(TQ);
                        const int y = lg_div(q, QW, G.rQW), qx = q - y * QW;
                        if (qx < G.nA) {
                            const int pos = lg_sse_before(G, q, G.nA) - lg_sse_before(G, a, G.nA);
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                float *p = buf + i * SR + pos;
                                p[0] = (float)(gx[i] * gx[i]);
                                p[PLA] = (float)(gx[i] * gy[i]);
                                p[2 * PLA] = (float)(gy[i] * gy[i]);
                            }
                        } else {
                            const int pos = lg_tail_before(G, q, G.nA, G.tA) - lg_tail_before(G, a, G.nA, G.tA);
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                if (4 * qx + i >= w) break;
                                float *p = buf + 4 * SR + pos + i;
                                p[0] = (float)(gx[i] * gx[i]);
                                p[PLA] = (float)(gx[i] * gy[i]);
                                p[2 * PLA] = (float)(gy[i] * gy[i]);
                            }
                        }
                    };
                    float acc = lg_tiles<3, TQ>(qs, NQ, PL, 15, (float)base0, loadA, storeA, geoA, [&](int) {});
                    if (tid < 64) {  // wave 0 combines in the SSE2 build's order
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
                            if (tid == 0) RS[s] = t;
                        }
                    }
                    __syncthreads();
                    s3[0] = RS[0];
                    s3[1] = RS[1];
                    s3[2] = RS[2];
                }
                A11 = __fmul_rn(s3[0], FLT_SCALE);
                A12 = __fmul_rn(s3[1], FLT_SCALE);
                A22 = __fmul_rn(s3[2], FLT_SCALE);
            }
            LG_MARK(1);  // A chains
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
                const LgJ JJ = window_j(inx, iny, w00, w01, w10, w11);
                // ---- main pass: the thread's quads in order, the 10 b chains as runs ----
                int T1[5] = {0, 0, 0, 0, 0}, M1[5] = {0, 0, 0, 0, 0}, m1[5] = {0, 0, 0, 0, 0};
                int T2[5] = {0, 0, 0, 0, 0}, M2[5] = {0, 0, 0, 0, 0}, m2[5] = {0, 0, 0, 0, 0};
                int dmax = 0;
                {
                    int y = y0, qx = x0;
                    auto quad = [&](const uint2 &ip, const uint2 &xp, const uint2 &yp) {
                        int d[4];
                        lg_diffs(JJ, y, qx, ip, d);
                        const int gx[4] = {lo16(xp.x), hi16(xp.x), lo16(xp.y), hi16(xp.y)};
                        const int gy[4] = {lo16(yp.x), hi16(yp.x), lo16(yp.y), hi16(yp.y)};
                        if (qx < G.nB2) {  // SSE2 quad: pixel i feeds lane chain i
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                run_add(T1[i], M1[i], m1[i], __mul24(d[i], gx[i]));
                                run_add(T2[i], M2[i], m2[i], __mul24(d[i], gy[i]));
                            }
                        } else {  // the tail chain, in order (pixels past w: zero gradients)
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                run_add(T1[4], M1[4], m1[4], __mul24(d[i], gx[i]));
                                run_add(T2[4], M2[4], m2[4], __mul24(d[i], gy[i]));
                            }
                        }
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            if (4 * qx + i < w) dmax = max(dmax, abs(d[i]));
                        if (++qx == QW) {
                            qx = 0;
                            y++;
                        }
                    };
                    // batches of kLgMB quads: their slot loads in flight together
                    int k = 0;
                    for (; k + kLgMB <= cnt; k += kLgMB) {
                        uint2 ip[kLgMB], xp[kLgMB], yp[kLgMB];
#pragma unroll
                        for (int u = 0; u < kLgMB; u++) {
                            const int ix = (k + u) * NT + tid;
                            ip[u] = IPs[ix];
                            xp[u] = XPs[ix];
                            yp[u] = YPs[ix];
                        }
#pragma unroll
                        for (int u = 0; u < kLgMB; u++) quad(ip[u], xp[u], yp[u]);
                    }
                    for (; k < cnt; k++) {
                        const int ix = k * NT + tid;
                        quad(IPs[ix], XPs[ix], YPs[ix]);
                    }
                }
                LG_MARK(2);  // main pass
                LG_COUNT(10);
                // every term is an exact float unless |d| * |g| > 2^24; a run past
                // [-2^25, 2^25] (terms < 2^26: seen before any wrap) cannot be exact
                bool bad = (long long)dmax * gmax > (long long)kExact;
                int T[10], M[10], m[10];
#pragma unroll
                for (int c = 0; c < 5; c++) {
                    T[c] = T1[c], M[c] = M1[c], m[c] = m1[c];
                    T[5 + c] = T2[c], M[5 + c] = M2[c], m[5 + c] = m2[c];
                }
#pragma unroll
                for (int c = 0; c < 10; c++) bad |= M[c] > (1 << 25) || m[c] < -(1 << 25);
                int *rec = X + par * 4 * kBxRecInts;
                par ^= 1;
                bx_publish<10>(T, rec, G.tB == 0);
                __syncthreads();
                bx_check_t<10>(T, M, m, bad, rec, G.tB == 0);
                __syncthreads();
                int tot, h0, base0;
                const bool bex = bx_eval_t<10>(rec, tot, h0, base0);
                LG_MARK(3);  // publish / check / eval
                float b1, b2;
                if (bex) {
                    b1 = rl_f(tot, 4);
                    b2 = rl_f(tot, 9);
                    if (sse) {
                        b1 = __fadd_rn(b1, __fadd_rn(__fadd_rn(rl_f(tot, 0), rl_f(tot, 2)), __fadd_rn(rl_f(tot, 1), rl_f(tot, 3))));
                        b2 = __fadd_rn(b2, __fadd_rn(__fadd_rn(rl_f(tot, 5), rl_f(tot, 7)), __fadd_rn(rl_f(tot, 6), rl_f(tot, 8))));
                    }
                } else {
                    LG_COUNT(11);
                    // ordered float chains from thread h0's run on (chain lanes: wave 0,
                    // lanes 0-9, from their exact prefixes base0), tiles of TQ quads
                    const int qs = min(h0 * K, NQ);
                    auto geoB = [&](int q, int &bs, int &bt) {
                        bs = lg_sse_before(G, q, G.nB2);
                        bt = lg_tail_before(G, q, G.nB2, G.tB);
                    };
                    auto loadB = [&](int q) {
                        const int t = lg_div(q, K, G.rK), idx = (q - t * K) * NT + t;
                        LgQ v;
                        v.ip = IPs[idx];
                        v.xp = XPs[idx];
                        v.yp = YPs[idx];
                        return v;
                    };
                    auto storeB = [&](const LgQ &v, int q, int a, float *buf) {
                        const int y = lg_div(q, QW, G.rQW), qx = q - y * QW;
                        int d[4];
                        lg_diffs(JJ, y, qx, v.ip, d);
                        const int gx[4] = {lo16(v.xp.x), hi16(v.xp.x), lo16(v.xp.y), hi16(v.xp.y)};
                        const int gy[4] = {lo16(v.yp.x), hi16(v.yp.x), lo16(v.yp.y), hi16(v.yp.y)};
                        const int PLB = lg_plane(TQ), SR = lg_sreg(TQ);
                        if (qx < G.nB2) {
                            const int pos = lg_sse_before(G, q, G.nB2) - lg_sse_before(G, a, G.nB2);
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                float *p = buf + i * SR + pos;
                                p[0] = (float)__mul24(d[i], gx[i]);
                                p[PLB] = (float)__mul24(d[i], gy[i]);
                            }
                        } else {
                            const int pos = lg_tail_before(G, q, G.nB2, G.tB) - lg_tail_before(G, a, G.nB2, G.tB);
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                if (4 * qx + i >= w) break;
                                float *p = buf + 4 * SR + pos + i;
                                p[0] = (float)__mul24(d[i], gx[i]);
                                p[PLB] = (float)__mul24(d[i], gy[i]);
                            }
                        }
                    };
                    LG_MARK(4);
                    auto markB = [&](int i) {
                        if (i == 0) {
                            LG_MARK(18);  // ordered b chains: pads of the next tile
                            LG_COUNT(14);
                        } else if (i == 1) {
                            LG_MARK(13);  // barrier wait
                        } else if (i == 2) {
                            LG_MARK(16);  // writes, loads, tile geometry
                        } else {
                            LG_MARK(17);  // chain sums
                        }
                    };
                    // ---- parity records (psn_lk_xb.h): every thread's run of every chain
                    // as one record, the chain lanes walk them in order; the ordered
                    // tiles when a term is past 2^24, a prefix past 2^30 or the pool of
                    // HARD runs' terms overflows ----
#if PSN_LG_XB
                    auto xb_b = [&](float &acc_out) -> bool {
                        const int wv = tid >> 6, fs = h0;
                        // exact prefix at the run start per chain (the block scan's exclusive
                        // prefix: wave-exclusive + the earlier waves' totals)
                        int B[10];
#pragma unroll
                        for (int c = 0; c < 10; c++) {
                            const int *r = rec + 8 * c;
                            B[c] = T[c] + (wv > 0 ? r[0] : 0) + (wv > 1 ? r[1] : 0) + (wv > 2 ? r[2] : 0);
                        }
                        // guard (saturating sum of the runs' excursions: every prefix < 2^30,
                        // no int wrap) and the largest |prefix| (the grid of the error bound)
                        int gx = (long long)dmax * gmax > (long long)kExact || K > 64 ? (1 << 30) : 0, mx = 0;
#pragma unroll
                        for (int c = 0; c < 10; c++) {
                            gx = max(gx, max(M[c], -m[c]));
                            mx = max(mx, max(B[c] + M[c], -(B[c] + m[c])));
                        }
                        const unsigned gw = wave_sum_sat((unsigned)gx);
                        const int mw = __builtin_amdgcn_readlane(wave_max_scan(mx), 63);
                        if (lane == 0) {
                            EP[4 + wv] = mw;
                            EP[8 + wv] = (int)gw;
                        }
                        __syncthreads();
                        const unsigned gsum = sat_add(sat_add((unsigned)EP[8], (unsigned)EP[9]), sat_add((unsigned)EP[10], (unsigned)EP[11]));
                        if (gsum >= (1u << 30)) return false;
                        const int MX = max(max(EP[4], EP[5]), max(EP[6], EP[7]));
                        const int umax = MX + (MX >> 3) + 1024 <= (1 << 24) ? 1 : 1 << (31 - __builtin_clz((unsigned)(MX + (MX >> 3) + 1024)) - 23);
                        // keys, term counts, HARD terms
                        const bool mine = tid >= fs && cnt > 0;
                        const int q1 = q0 + cnt, nq = mine ? q1 - fs * K : 0;
                        const int nS = lg_sse_before(G, q1, G.nB2) - lg_sse_before(G, q0, G.nB2);
                        const int nT = lg_tail_before(G, q1, G.nB2, G.tB) - lg_tail_before(G, q0, G.nB2, G.tB);
                        const int ES = nq * (umax >> 1) + 2 * umax, ET = nq * 2 * umax + 2 * umax;
                        int key[10], hard = 0;
#pragma unroll
                        for (int c = 0; c < 10; c++) {
                            const int E = c % 5 == 4 ? ET : ES, n = c % 5 == 4 ? nT : nS;
                            key[c] = mine && n > 0 ? xb_key(B[c] + m[c] - E, B[c] + M[c] + E) : 23;
                            if (key[c] < 0) hard += n;
                        }
                        const int hs = wave_scan(hard);
                        if (lane == 63) EP[12 + wv] = hs;
                        if (tid == 0) EP[3] = 0;  // the replay's failure flag
                        __syncthreads();
                        const int pbase = (wv > 0 ? EP[12] : 0) + (wv > 1 ? EP[13] : 0) + (wv > 2 ? EP[14] : 0);
                        const int ptotal = EP[12] + EP[13] + EP[14] + EP[15];
                        if (ptotal > kLgPoolBytes / 4) return false;
                        LG_MARK(19);  // xb: prefixes, guard, keys, pool scan
                        // replay: each thread's run of every chain; first terms kept, the rest
                        // from two representatives of either parity near B + first term (key
                        // 23: one exact replay); HARD runs' terms into the pool
                        float r0[10], r1[10];
                        int f1[10], R0[10], poff[10];
                        unsigned started = 0;
                        {
                            int o = pbase + hs - hard;
#pragma unroll
                            for (int c = 0; c < 10; c++) {
                                poff[c] = o;
                                if (key[c] < 0) o += c % 5 == 4 ? nT : nS;
                                r0[c] = r1[c] = 0.f;
                                f1[c] = R0[c] = 0;
                            }
                        }
                        auto term = [&](int c, int t) {
                            if (key[c] < 0) {
                                POOL[poff[c]++] = (float)t;
                                return;
                            }
                            const int ks = key[c] - 23, u = 1 << ks;
                            if (!(started & (1u << c))) {
                                started |= 1u << c;
                                f1[c] = t;
                                const int v = B[c] + t;
                                R0[c] = ((v + u) >> (ks + 1)) << (ks + 1);
                                r0[c] = (float)R0[c];
                                r1[c] = (float)(R0[c] + u);
                            } else {
                                const float tf = (float)t;
                                r0[c] = __fadd_rn(r0[c], tf);
                                r1[c] = __fadd_rn(r1[c], tf);
                            }
                        };
                        if (mine) {
                            int y = y0, qx = x0;
                            auto quad = [&](const uint2 &ip, const uint2 &xp, const uint2 &yp) {
                                int d[4];
                                lg_diffs(JJ, y, qx, ip, d);
                                const int gxv[4] = {lo16(xp.x), hi16(xp.x), lo16(xp.y), hi16(xp.y)};
                                const int gyv[4] = {lo16(yp.x), hi16(yp.x), lo16(yp.y), hi16(yp.y)};
                                if (qx < G.nB2) {
#pragma unroll
                                    for (int i = 0; i < 4; i++) {
                                        term(i, __mul24(d[i], gxv[i]));
                                        term(5 + i, __mul24(d[i], gyv[i]));
                                    }
                                } else {
#pragma unroll
                                    for (int i = 0; i < 4; i++) {
                                        if (4 * qx + i >= w) break;
                                        term(4, __mul24(d[i], gxv[i]));
                                        term(9, __mul24(d[i], gyv[i]));
                                    }
                                }
                                if (++qx == QW) {
                                    qx = 0;
                                    y++;
                                }
                            };
                            int k = 0;
                            for (; k + kLgMB <= cnt; k += kLgMB) {
                                uint2 ip[kLgMB], xp[kLgMB], yp[kLgMB];
#pragma unroll
                                for (int u = 0; u < kLgMB; u++) {
                                    const int ix = (k + u) * NT + tid;
                                    ip[u] = IPs[ix];
                                    xp[u] = XPs[ix];
                                    yp[u] = YPs[ix];
                                }
#pragma unroll
                                for (int u = 0; u < kLgMB; u++) quad(ip[u], xp[u], yp[u]);
                            }
                            for (; k < cnt; k++) {
                                const int ix = k * NT + tid;
                                quad(IPs[ix], XPs[ix], YPs[ix]);
                            }
                        }
                        LG_MARK(20);  // xb: replay
                        // records (the b tiles region; its last readers passed a barrier)
                        bool fail = false;
                        if (tid >= fs) {
#pragma unroll
                            for (int c = 0; c < 10; c++) {
                                const int n = c % 5 == 4 ? nT : nS;
                                int2 rv;
                                if (!mine || n == 0) {
                                    rv = xb_rec_hard(0, 0);
                                } else if (key[c] < 0) {
                                    rv = xb_rec_hard(poff[c] - n, n);
                                } else {
                                    const int ks = key[c] - 23;
                                    const int Q0 = ((int)r0[c] - R0[c]) >> ks;
                                    const int D = (((int)r1[c] - R0[c] - (1 << ks)) >> ks) - Q0;
                                    fail |= D < -1 || D > 1;
                                    rv = xb_rec(Q0, f1[c], ks, D);
                                }
                                XREC[c * kXbRecThreads + tid] = rv;
                            }
                        }
                        if (fail) EP[3] = 1;  // (no __syncthreads_or: it takes static LDS)
                        __syncthreads();
                        if (EP[3]) return false;
                        LG_MARK(21);  // xb: records
                        // the walk: chain lane c from the exact prefix before half wave h0
                        if (tid < 10) {
                            const int last = min(kXbRecThreads, (NQ + K - 1) / K);
                            acc_out = xb_walk(XREC + tid * kXbRecThreads, POOL, fs, last, (float)base0);
                        }
                        LG_MARK(22);  // xb: walk
                        return true;
                    };
                    float acc;
                    if (!xb_b(acc)) {
                        __syncthreads();  // every reader of the records / scratch is done
                        acc = lg_tiles<2, TQ>(qs, NQ, PL, 10, (float)base0, loadB, storeB, geoB, markB);
                    }
#else
                    const float acc = lg_tiles<2, TQ>(qs, NQ, PL, 10, (float)base0, loadB, storeB, geoB, markB);
#endif
                    LG_MARK(5);  // ordered b chains
                    if (tid < 64) {  // wave 0 combines in the SSE2 build's order
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
                        if (tid == 0) {
                            RS[4] = r1;
                            RS[5] = r2;
                        }
                    }
                    __syncthreads();
                    b1 = RS[4];
                    b2 = RS[5];
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
                const float qxf = __fsub_rn(NPx, hwx), qyf = __fsub_rn(NPy, hwy);
                const int iqx = cv_floor(qxf), iqy = cv_floor(qyf);
                if (iqx < -w || iqx >= cols || iqy < -h || iqy >= rows) {
                    status = 0;
                    continue;
                }
                int w00, w01, w10, w11;
                bilin_weights(__fsub_rn(qxf, (float)iqx), __fsub_rn(qyf, (float)iqy), w00, w01, w10, w11);
                const LgJ JJ = window_j(iqx, iqy, w00, w01, w10, w11);
                unsigned e = 0;
                {
                    int y = y0, qx = x0;
                    auto quad = [&](const uint2 &ip) {
                        int d[4];
                        lg_diffs(JJ, y, qx, ip, d);
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            if (4 * qx + i < w) e = sat_add(e, (unsigned)abs(d[i]));
                        if (++qx == QW) {
                            qx = 0;
                            y++;
                        }
                    };
                    int k = 0;
                    for (; k + kLgMB <= cnt; k += kLgMB) {
                        uint2 ip[kLgMB];
#pragma unroll
                        for (int u = 0; u < kLgMB; u++) ip[u] = IPs[(k + u) * NT + tid];
#pragma unroll
                        for (int u = 0; u < kLgMB; u++) quad(ip[u]);
                    }
                    for (; k < cnt; k++) quad(IPs[k * NT + tid]);
                }
                e = wave_sum_sat(e);
                if (lane == 0) EP[tid >> 6] = (int)e;
                __syncthreads();
                const unsigned et = sat_add(sat_add((unsigned)EP[0], (unsigned)EP[1]), sat_add((unsigned)EP[2], (unsigned)EP[3]));
                float errval;
                if (et <= (unsigned)kExact) {
                    errval = (float)et;  // every partial sum of errval += |diff| is an exact integer
                } else {  // row-major order, one lane, tiles of kLgTQE quads
                    float acc = 0.f;
                    for (int a = 0; a < NQ; a += kLgTQE) {
                        const int b = min(a + kLgTQE, NQ);
                        const int pa = lg_div(a, QW, G.rQW) * w + 4 * (a - lg_div(a, QW, G.rQW) * QW);  // row-major pixel index of quad a
                        __syncthreads();
                        const int q = a + tid;
                        if (q < b) {
                            const int t = lg_div(q, K, G.rK), idx = (q - t * K) * NT + t;
                            const int y = lg_div(q, QW, G.rQW), qx = q - y * QW;
                            int d[4];
                            lg_diffs(JJ, y, qx, IPs[idx], d);
#pragma unroll
                            for (int i = 0; i < 4; i++)
                                if (4 * qx + i < w) PL[y * w + 4 * qx + i - pa] = (float)abs(d[i]);
                        }
                        __syncthreads();
                        const int pb = b < NQ ? lg_div(b, QW, G.rQW) * w + 4 * (b - lg_div(b, QW, G.rQW) * QW) : w * h;
                        if (tid == 0) acc = chain_sum(PL, pb - pa, acc);
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
            LG_CLK(t_end);
            lg_acc[15] = t_end - lg_t0;
            if (tid == 0 && A.stamps)
                for (int i = 0; i < 24; i++) A.stamps[(size_t)g * 64 + i] = lg_acc[i];
        }
#endif
        if (tid == 0) {
            A.next[2 * pi] = NPx;
            A.next[2 * pi + 1] = NPy;
            A.status[pi] = (uint8_t)status;
            if (A.err) A.err[pi] = errv;
            if (A.samples) atomicAdd(A.samples, (unsigned long long)nwin * (unsigned)(w * h));
        }
        __syncthreads();  // the next point reuses the slot, the LDS and the records
    }
}

hipError_t launch_lk_lg(const LkLaunchArgs &a, int grid, int lds_bytes, int tq, hipStream_t s) {
    if (grid <= 0 || a.lk_wgs <= 0) return hipSuccess;
    if (!a.lg_ws || a.lg_slot <= 0 || lds_bytes > 160 * 1024) return hipErrorInvalidValue;
    switch (tq) {
        case 192: hipLaunchKernelGGL(lk_kernel_lg<192>, dim3(grid), dim3(kLgNT), lds_bytes, s, a); break;
        case 128: hipLaunchKernelGGL(lk_kernel_lg<128>, dim3(grid), dim3(kLgNT), lds_bytes, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t lg_kernels_init() {
    const void *f[2] = {(const void *)lk_kernel_lg<192>, (const void *)lk_kernel_lg<128>};
    for (const void *k : f) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace psn
