// Device helpers shared by the LK kernels of libpsn_lk.so (psn_lk_kernels.hip,
// psn_lk_large.hip): OpenCV 2.4.6 rounding / border rules, workgroup sums, the
// LDS staging walkers and the SSE2 chain layouts. Internal, not installed.
#pragma once

#include <float.h>
#include <limits.h>

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

// Exactness of a float sum of integer terms t in ANY order or chain split:
// every partial sum is a subset sum, inside [-N, P] (P = sum of the positive
// terms, N = sum of |negative terms|), so max(P, N) <= 2^24 makes every
// partial sum an exact float. With A = sum|t| and S = sum t:
// max(P, N) = (A + |S|) / 2. A <= 2^25 also keeps an int32 S unwrapped
// (A is reduced saturating, so a wrapped S comes with a failing A).
__device__ __forceinline__ bool sums_exact(unsigned A, int S) {
    return A + (unsigned)abs(S) <= (2u << 24);
}

__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
// Inclusive prefix sum over the 64 lanes (the wave_sum sequence without the final readlane).
__device__ __forceinline__ int wave_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
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

// n / d for 0 <= n, d < 1024 with mg = div_magic(d) = ceil(2^22 / d): the error
// term n * (mg * d - 2^22) < 2^20 keeps the quotient exact; n * mg < 2^32.
__device__ __forceinline__ int qdiv(int n, unsigned mg) { return (int)(__umul24((unsigned)n, mg) >> 22); }

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
    // the same with the division magic of pw (tid, nt < 1024)
    __device__ __forceinline__ void init_m(int tid, int nt, int pw_, unsigned mg) {
        pw = pw_;
        y = qdiv(tid, mg);
        x = tid - y * pw;
        sy = qdiv(nt, mg);
        sx = nt - sy * pw;
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

// Level descriptor of (slot, level) from the kernel-argument ring geometry.
__device__ __forceinline__ LevelDev ring_level(const RingGeo &r, int slot, int level) {
    LevelDev L;
    L.p = r.base + (long long)slot * r.slot_bytes + r.off[level];
    L.w = r.w[level];
    L.h = r.h[level];
    L.pitch = r.pitch[level];
    L.pad_ = 0;
    return L;
}

// The same for a uniform runtime level: an unrolled select over static
// kernel-argument offsets (the scalar loads issue together, no dependent
// load per level).
__device__ __forceinline__ LevelDev ring_level_u(const RingGeo &r, int slot, int level) {
    LevelDev L = ring_level(r, slot, 0);
#pragma unroll
    for (int l = 1; l < kPyrMaxTop + 1; l++)
        if (level == l) L = ring_level(r, slot, l);
    return L;
}

typedef const void __attribute__((address_space(1))) *gptr_t;
typedef void __attribute__((address_space(3))) *lptr_t;

// Asynchronous LDS-DMA gather of a PW x PH u8 region of a pyramid level
// (reflect-101 addressing) into LDS, one dword per pixel. Wave w issues the
// 64-pixel chunks w, w+NW, ...; completion = s_waitcnt vmcnt(0) + barrier.
template <int NT>
__device__ __forceinline__ void dma_region(uint32_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH,
                                           unsigned mg_pw) {
    const int n = PW * PH;
    const bool interior = gy0 >= 0 && gx0 >= 0 && gy0 + PH <= L.h && gx0 + PW <= L.w;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    Walk wk;
    wk.init_m(threadIdx.x, NT, PW, mg_pw);
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
// The I patch of one level (PH rows, lk_pat_m(w) dwords per row from the
// aligned-down column gx0 & ~3) into LDS bytes: interior patches move as
// aligned dwords by LDS-DMA (lane i of a chunk lands at dst + 4 * i, so the
// chunk of dwords c0.. is contiguous in LDS); patches crossing the image border
// reflect their rows, move the dwords that lie inside the image the same way and
// gather the others' bytes through reflect-101.
// NT threads t = 0..NT-1 of the caller's group (the workgroup, or one wave).
template <int NT>
__device__ __forceinline__ void dma_patch_t(uint8_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH, int m,
                                            unsigned dv_m, int t) {
    const int ax = gx0 & ~3;
    const int n = PH * m;
    const int wid = t >> 6, lane = t & 63;
    if (gy0 >= 0 && gx0 >= 0 && gy0 + PH <= L.h && gx0 + PW <= L.w) {
        // the row's last dword may read up to 6 bytes past the image width:
        // inside the 256-B pitch, the next row, or the ring's slack
        for (int c0 = wid * 64; c0 < n; c0 += NT) {
            const int q = c0 + lane;
            if (q < n) {
                const int r = qdiv(q, dv_m), j = q - r * m;
                const uint8_t *src = L.p + (size_t)(gy0 + r) * L.pitch + ax + 4 * j;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + 4 * c0), 4, 0, 0);
            }
        }
    } else {
        // across the border: reflect-101 rows; dwords whose 4 columns are inside the
        // image still move by LDS-DMA (lanes with such a dword: the DMA writes lane i's
        // dword at dst + 4 * (c0 + i)), the others gather their 4 reflected bytes
        for (int c0 = wid * 64; c0 < n; c0 += NT) {
            const int q = c0 + lane;
            if (q < n) {
                const int r = qdiv(q, dv_m), j = q - r * m;
                const uint8_t *row = L.p + (size_t)refl101(gy0 + r, L.h) * L.pitch;
                const int x = ax + 4 * j;
                if (x >= 0 && x + 4 <= L.w) {
                    __builtin_amdgcn_global_load_lds((gptr_t)(row + x), (lptr_t)(dst + 4 * c0), 4, 0, 0);
                } else {
                    unsigned v = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) v |= (unsigned)row[refl101(x + b, L.w)] << (8 * b);
                    *(unsigned *)(dst + 4 * q) = v;
                }
            }
        }
    }
}
template <int NT>
__device__ __forceinline__ void dma_patch(uint8_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH, int m,
                                          unsigned dv_m) {
    dma_patch_t<NT>(dst, L, gy0, gx0, PW, PH, m, dv_m, (int)threadIdx.x);
}
// dma_patch for rows of any width (no division magic): each thread's (row,
// dword) by a Walk over the PH x m dword grid.
template <int NT>
__device__ __forceinline__ void dma_rows(uint8_t *dst, const LevelDev &L, int gy0, int gx0, int PW, int PH, int m) {
    const int ax = gx0 & ~3;
    const int n = PH * m;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool in = gy0 >= 0 && gx0 >= 0 && gy0 + PH <= L.h && gx0 + PW <= L.w;
    Walk wk;
    wk.init(threadIdx.x, NT, m);
    for (int c0 = wid * 64; c0 < n; c0 += NT, wk.step()) {
        if (c0 + lane >= n) continue;
        const int x = ax + 4 * wk.x;
        if (in) {  // as dma_patch: a row's last dword may read a few bytes past PW
            __builtin_amdgcn_global_load_lds((gptr_t)(L.p + (size_t)(gy0 + wk.y) * L.pitch + x), (lptr_t)(dst + 4 * c0),
                                             4, 0, 0);
        } else {
            const uint8_t *row = L.p + (size_t)refl101(gy0 + wk.y, L.h) * L.pitch;
            if (x >= 0 && x + 4 <= L.w) {
                __builtin_amdgcn_global_load_lds((gptr_t)(row + x), (lptr_t)(dst + 4 * c0), 4, 0, 0);
            } else {
                unsigned v = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) v |= (unsigned)row[refl101(x + b, L.w)] << (8 * b);
                *(unsigned *)(dst + 4 * (c0 + lane)) = v;
            }
        }
    }
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Debug (PSN_LK_VARIANT_POISON_LDS): fill `bytes` of dynamic LDS with 24-bit
// pseudo-random words before the kernel uses it, so a read of LDS the kernel never
// wrote sees the same values on every run instead of what earlier kernels left.
template <int NT>
__device__ __forceinline__ void lds_poison(uint8_t *smem, int bytes) {
    unsigned *p = (unsigned *)smem;
    for (int i = threadIdx.x; i < bytes / 4; i += NT) p[i] = ((unsigned)i * 2654435761u) >> 8;
    __syncthreads();
}
// A workgroup barrier that leaves vector-memory loads in flight (__syncthreads'
// fence would wait for them): every thread's LDS data it orders was already
// waited for (dma_wait / lgkmcnt) by the thread that wrote it. The empty asm
// keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void barrier_inflight() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}


}  // namespace psn
