// Internal (non-ABI) declarations shared by the HIP kernels and the C-ABI host
// code of libpsn_lk.so. Not installed; the public surface is include/psn_lk.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psn_lk.h"

namespace psn {

constexpr int kMaxLevels = PSN_LK_MAX_LEVELS;
constexpr int kMaxQueries = 32;     // queries per LK launch (kernel-argument table)
constexpr int kJMargin = 3;         // J staging margin (px) around the window, each side
constexpr int kPyrMaxTop = 5;       // fused pyramid kernel supports top level <= 5

// One pyramid level in HBM: unpadded u8 plane, rows `pitch` bytes apart.
struct LevelDev {
    uint8_t *p;
    int w, h, pitch;
    int pad_;
};

struct PyrBuildArgs {
    const uint8_t *src;   // level-0 source frame (gray or BGR)
    int src_stride;
    int channels;         // 1 or 3
    int nlevels;          // levels to write (1..kPyrMaxTop+1)
    int tile;             // top-level tile edge
    LevelDev lv[kMaxLevels];
};

struct LkQueryDev {
    int prev_slot, next_slot;
    int wg_begin;         // first workgroup of this query
    int pt_begin;         // first point index in the arrays
    int num_pts;
    int win_w, win_h;
    int max_level;        // effective (truncated) maxLevel
    int max_count;
    int flags;
    int tile_rows;        // window rows per LDS tile (>= win_h: single-tile kernel)
    float min_eig;
    double eps2;
    // division magics (q = n * dv >> 22, exact for n, d < 1024) of the per-query
    // divisors the single-tile kernel needs, and its one-wave lane geometry
    unsigned dv_w, dv_dw, dv_pm, dv_jrw, dv_jrw4, dv_g, dv_cw;
    int ow_g, ow_rg;
    int qidx;             // the caller's query index (LkLaunchArgs::counts)
    // box-window kernel: row tiles of the err-chain fallback
    // and the division magics of its I-patch / J-region dword rows
    int bx_tre;
    union {
        int bx_hw;  // box kernel: half waves per fallback tile
        int lg_jr;  // large-window kernel: 1 = the iterations read J from an LDS copy of its region
        int st_ovl; // single-tile one-wave kernel: 1 = the finer levels' A phase runs beside the iterations
    };
    unsigned dv_bxpm, dv_bxjr;
    // a merged query (sub_pts > 0): sub-queries of sub_pts points each, sub-query
    // j's points from pt_begin + j * sub_pstride, its device count at
    // counts[qidx + j * LkLaunchArgs::count_stride] (the caller's queries k..k+n-1
    // of one plan; 0: one query)
    int sub_pts, sub_pstride;
};
// Workgroup g's point in query Q (g - Q.wg_begin >= 0), or -1 when it is past
// its (sub-)query's device count
__device__ __forceinline__ int lk_query_point(const LkQueryDev &Q, const int *counts, int count_stride, int g) {
    int loc = g - Q.wg_begin;
    if (Q.sub_pts > 0) {
        const int sub = loc / Q.sub_pts;
        loc -= sub * Q.sub_pts;
        if (counts && loc >= counts[Q.qidx + sub * count_stride]) return -1;
        return Q.pt_begin + sub * Q.sub_pstride + loc;
    }
    if (counts && loc >= counts[Q.qidx]) return -1;
    return Q.pt_begin + loc;
}
__host__ __device__ inline unsigned div_magic(int d) { return d > 0 ? ((1u << 22) + (unsigned)d - 1u) / (unsigned)d : 0u; }

// Ring geometry as kernel arguments (every slot has the same level layout):
// level l of slot s starts at base + s * slot_bytes + off[l].
struct RingGeo {
    uint8_t *base;
    long long slot_bytes;
    long long off[kMaxLevels];
    int w[kMaxLevels], h[kMaxLevels], pitch[kMaxLevels];
};

struct LkLaunchArgs {
    const LevelDev *slots;   // [nslots][kMaxLevels]
    RingGeo ring;
    const float *prev;       // (x,y) pairs
    float *next;
    uint8_t *status;
    float *err;              // may be null
    unsigned long long *stamps;  // diagnostic build only (PSN_LK_STAMPS): [wg][64] s_memtime
    unsigned long long *samples; // optional: += sum over levels of w*h*(1 + iterations) per point
    int nq;
    int poison_lds;          // debug (PSN_LK_VARIANT_POISON_LDS): bytes of dynamic LDS the kernel fills with a pattern first
    // optional per-query point counts on the device (<= num_pts, the grid
    // capacity): workgroups past a query's count exit at once (device-side
    // chains whose counts come from a previous kernel)
    const int *counts;
    int count_stride;        // counts of consecutive caller queries are count_stride apart
    LkQueryDev q[kMaxQueries];
    // Deferred pyramid build fused into this launch (single-tile kernel only):
    // workgroups that finish their point pull top-level tiles of `pyr` from
    // the work counter pyr_ctr[0]; pyr_ctr[1] counts finished workgroups and
    // the last one resets both. pyr_ntiles == 0: no fused build.
    // Helper workgroups (blockIdx >= lk_wgs) skip the LK part and pull tiles
    // from the start; total_wgs = lk_wgs + helpers.
    int pyr_ntiles, pyr_tiles_x;
    int total_wgs, lk_wgs;
    unsigned *pyr_ctr;
    PyrBuildArgs pyr;
    // Large-window kernel (lk_kernel_lg): per-workgroup HBM slots of the window
    // values {I*, Ix* | Iy* << 16}, lg_slot int2 apart; the grid strides over
    // the launch's lk_wgs points
    int2 *lg_ws;
    long long lg_slot;
};

// LDS bytes a query needs for a given tile height (shared by host planner and kernel).
__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }
__host__ __device__ inline int lk_jreg_w(int w) { return w + 1 + 2 * kJMargin; }
__host__ __device__ inline int lk_jreg_h(int h) { return h + 1 + 2 * kJMargin; }
__host__ __device__ inline int lk_off_dw(int w, int h) { return align16(2 * w * h); }
__host__ __device__ inline int lk_off_jr(int w, int h) { return lk_off_dw(w, h) + align16(4 * w * h); }
__host__ __device__ inline int lk_off_red(int w, int h) { return lk_off_jr(w, h) + align16(lk_jreg_w(w) * lk_jreg_h(h)); }
constexpr int kRedBytes = 256;
__host__ __device__ inline int lk_off_tile(int w, int h) { return lk_off_red(w, h) + kRedBytes; }
__host__ __device__ inline int lk_tile_pimg_bytes(int w, int tr) { return align16((tr + 3) * (w + 3)); }
__host__ __device__ inline int lk_tile_dg_bytes(int w, int tr) { return align16(4 * (tr + 1) * (w + 1)); }
// 3 planes, each = 5 chain regions rounded up to 4 floats (16-B aligned vector reads)
__host__ __device__ inline int lk_tile_prod_bytes(int w, int tr) { return 12 * (tr * w + 20); }
__host__ __device__ inline int lk_lds_bytes(int w, int h, int tr) {
    return lk_off_tile(w, h) + lk_tile_pimg_bytes(w, tr) + lk_tile_dg_bytes(w, tr) + lk_tile_prod_bytes(w, tr);
}

// Single-tile kernel layout (whole window LDS-resident, double-buffered b products).
__host__ __device__ inline int round16i(int x) { return (x + 15) & ~15; }
__host__ __device__ inline int lk_st_planeA(int w, int h, bool sse) {
    const int n = sse ? w / 4 : 0;
    return 4 * round16i(h * n) + round16i(h * (w - 4 * n) + 1);  // +1: a zero slot for idle lanes
}
__host__ __device__ inline int lk_st_planeB(int w, int h, bool sse) {
    const int n = sse ? w / 8 : 0;
    return 4 * round16i(h * 2 * n) + round16i(h * (w - 8 * n) + 1);
}
// Single-tile kernel LDS layout.
//   scratch: level table (2 pyramids x kMaxLevels x 8 ints), reduce scratch
//     RI (per-iteration regions for iteration parity 0/1 and the err pass: 4
//     ints per wave for up to 8 waves; the fused-build tile index; the A-phase
//     region: 4 sums x kStMaxLev levels x 8 waves), the per-level solver table
//     LV (kStMaxLev x 8 floats);
//   jp: the J region in PAIR format (dword x = J[x] | J[x+1] << 16, rows of
//     st_jreg_w(w) dwords) for the packed-dot bilinear of the iterations;
//   pim: the I patch of every level ((h+3) x (w+3), one dword per pixel as
//     LDS-DMA writes them);
//   dg: Scharr (Ix, Iy) short2 of every level ((h+1) x (w+1));
//   iw: per level and window pixel {Iw, Ix | Iy << 16} (int2);
//   r: A products of every level (3 chain-major planes per level); reused by
//     the double-buffered b products of the iterations and the err plane.
constexpr int kStMaxLev = kPyrMaxTop + 1;
constexpr int kStJMargin = 4;  // J region margin (px) each side; prefetched at the predicted position
constexpr int kStRiIt = 0, kStRiErr = 64, kStRiTile = 96, kStRiA = 128;           // ints
constexpr int kStRiInts = kStRiA + 4 * kStMaxLev * 8;                             // 320
constexpr int kStLvFloats = 8;
constexpr int kStScratchBytes = 2 * kMaxLevels * 8 * 4 + kStRiInts * 4 + kStMaxLev * kStLvFloats * 4;  // 1984
// J region: origin aligned down to 4 columns (one 8-byte load -> 4 pairs -> one
// 16-B LDS write), width a multiple of 4 keeping >= kStJMargin columns each side
__host__ __device__ inline int st_jreg_w(int w) { return (w + 2 * kStJMargin + 4 + 3) & ~3; }
__host__ __device__ inline int st_jreg_h(int h) { return h + 1 + 2 * kStJMargin; }
// One-wave iteration mode: the J region is column-major with an odd column
// stride (LDS banks), double-buffered, each buffer padded for the idle rows of
// the last lanes.
__host__ __device__ inline int st_jrh_cm(int h) { return st_jreg_h(h) | 1; }
__host__ __device__ inline int st_jp_cm_dw(int w, int h) { return (st_jreg_w(w) * st_jrh_cm(h) + 16 + 20) & ~15; }
// Lane geometry of the one-wave mode: window columns of one SSE2 chain class
// on consecutive lanes, G row groups of RG rows per column (G * w <= 64).
__host__ __device__ inline int ow_groups(int w) { return w <= 64 ? 64 / w : 0; }
__host__ __device__ inline int ow_rows(int w, int h) {
    const int G = ow_groups(w);
    return G ? (h + G - 1) / G : 1 << 30;
}
constexpr int kOwMaxRows = 16;
// I patch of a level in LDS: (h + 3) rows of bytes, row stride lk_pat_rs(w) =
// 4 * lk_pat_m(w): the w + 3 patch pixels start at byte (gx0 & 3) of a row, so
// every row moves as lk_pat_m(w) aligned dwords (LDS-DMA).
__host__ __device__ inline int lk_pat_m(int w) { return (w + 3 + 3 + 3) >> 2; }
__host__ __device__ inline int lk_pat_rs(int w) { return 4 * lk_pat_m(w); }
//   one-wave layout (ow): the window values IW of every level, then a union
//     of what only the prologue uses (I patches, Scharr planes, the A-phase
//     float chain planes RA) and what only the iterations use (the two J
//     regions JP, the b chain planes / err row R) -- 49.6 KB at 21x21 with 4
//     levels: three workgroups per CU.
//   overlapped one-wave layout (ow + ovl): no union -- the prologue computes only
//     the coarsest level's A phase; waves 1-3 compute the finer levels' (I
//     patch, Scharr, window values, A chains) while wave 0 iterates, so the I
//     patches, Scharr planes and A planes of every level stay beside the J
//     regions and b planes: 66.6 KB at 21x21 with 4 levels.
struct LkStLayout {
    int tbl, ri, lv, jp, pim, pim_stride, dg, dg_stride, iw, iw_stride, r, ra, total;
    __host__ __device__ LkStLayout(int w, int h, bool sse, int nlev, bool ow = false, bool ovl = false) {
        const int wh = w * h;
        tbl = 0;
        ri = tbl + 2 * kMaxLevels * 8 * 4;
        lv = ri + kStRiInts * 4;
        pim_stride = align16((h + 3) * lk_pat_rs(w));
        dg_stride = align16(4 * (h + 1) * (w + 1));
        iw_stride = align16(8 * wh);
        const int rb_a = 12 * nlev * lk_st_planeA(w, h, sse);
        const int pb = 16 * lk_st_planeB(w, h, sse);
        const int eb = 4 * round16i(wh);
        if (ow && ovl) {
            iw = kStScratchBytes;
            pim = iw + nlev * iw_stride;
            dg = pim + nlev * pim_stride;
            ra = dg + nlev * dg_stride;
            jp = ra + rb_a;
            r = jp + 8 * st_jp_cm_dw(w, h);
            total = r + (pb > eb ? pb : eb);
        } else if (ow) {
            iw = kStScratchBytes;  // fused builds use LDS from kStScratchBytes, after the LK work
            const int u = iw + nlev * iw_stride;
            pim = u;  // prologue view
            dg = pim + nlev * pim_stride;
            ra = dg + nlev * dg_stride;
            const int end_pro = ra + rb_a;
            jp = u;  // iteration view
            r = jp + 8 * st_jp_cm_dw(w, h);
            const int end_it = r + (pb > eb ? pb : eb);
            total = end_pro > end_it ? end_pro : end_it;
        } else {
            jp = kStScratchBytes;  // fused builds use LDS from here
            pim = jp + align16(4 * st_jreg_w(w) * st_jreg_h(h));
            dg = pim + nlev * pim_stride;
            iw = dg + nlev * dg_stride;
            r = iw + nlev * iw_stride;
            ra = r;
            int rb = rb_a;
            if (rb < pb) rb = pb;
            if (rb < eb) rb = eb;
            total = r + rb;
        }
    }
};
// Box-window kernel (lk_kernel_bx, Tracker2D box windows above the single-tile
// size). The window is cut into UNITS of 4 pixels (row y, quad q: x = 4q..4q+3),
// QW = ceil(w/4) per row, in row-major order; thread t owns units
// [t*UPT, t*UPT + UPT). LDS: chain-check scratch | J region (bytes, rows of
// bx_jrp(w)) | a union of the level's I patch (bytes, rows of bx_pm(w) dwords)
// and the row-tiled float chain planes of the ordered-sum fallbacks.
constexpr int kBxNT = 256;
constexpr int kBxMaxUPT = 16;
constexpr int kBxRecInts = 8 * 15 + 4;                 // per wave and chain: {total, max, min prefix, -} at lanes 31 and 63; term flag
constexpr int kBxXInts = 2 * 4 * kBxRecInts;           // two parities x 4 waves
constexpr int kBxScrBytes = (kBxXInts + 32) * 4 + 64;  // + results / err partials
constexpr int kBxMaxLds = 64 * 1024;   // three or four workgroups per CU
constexpr int kBxMaxLds2 = 80 * 1024;  // the two-per-CU builds
constexpr int kBxLdsTarget = 53 * 1024;  // three workgroups per CU
// workgroups per CU of lk_kernel_bx<upt, notail> (its __launch_bounds__): the
// 4-unit build fits 128 VGPRs, so four per CU when the LDS plan allows it; the
// builds whose registers do not fit 168 VGPRs at three per CU (12 units, and 10
// units with the scalar-tail chain: 8-33 spilled VGPRs; 16 units) run two per CU
__host__ __device__ constexpr int bx_occupancy(int upt, bool notail) {
    return upt <= 4 ? 4 : (upt >= 12 || (!notail && upt >= 10)) ? 2 : 3;
}
__host__ __device__ constexpr int bx_lds_target(int upt, bool notail) {
    return bx_occupancy(upt, notail) == 4 ? 40 * 1024 : bx_occupancy(upt, notail) == 3 ? kBxLdsTarget : kBxMaxLds2;
}
// the largest LDS plan of a lk_kernel_bx<upt, notail> launch
__host__ __device__ constexpr int bx_max_lds(int upt, bool notail) {
    return bx_occupancy(upt, notail) == 2 ? kBxMaxLds2 : kBxMaxLds;
}
__host__ __device__ inline int bx_qw(int w) { return (w + 3) >> 2; }
__host__ __device__ inline int bx_pm(int w) { return bx_qw(w) + 2; }      // I patch dwords per row
__host__ __device__ inline int bx_jrp(int w) { return st_jreg_w(w) + 8; }  // J region row pitch (bytes)
__host__ __device__ inline int bx_round4(int x) { return (x + 3) & ~3; }
// One chain region of a fallback plane: n floats rounded to 16, + 4: with a
// region stride of 4 (mod 16) floats the chain lanes' 16-B reads of one plane
// fall into different 4-bank groups (conflict-free).
__host__ __device__ inline int bx_region(int n) { return ((n + 15) & ~15) + 4; }
// Fallback tiles are half-wave unit ranges (32 threads x UPT units): one plane
// (4 SSE2 lane regions + the tail region) holds at most 4*32*UPT terms + padding.
__host__ __device__ inline int bx_pc(int upt) { return 128 * upt + 96; }
struct BxLayout {
    int jr, un, pb, total;
    __host__ __device__ BxLayout(int w, int h, int upt, int hw = 1) {
        jr = align16(kBxScrBytes);
        un = jr + align16(st_jreg_h(h) * bx_jrp(w));
        const int pim = align16((h + 3) * 4 * bx_pm(w));
        const int planes = 24 * bx_pc(upt) * hw;  // tiles of hw half waves, 2 buffers x (A: 3, b: 2) planes
        pb = pim > planes ? pim : planes;
        total = un + pb + 1024;  // slack: the chain sums read up to 5 blocks past a chain (discarded)
    }
};
// Row tiles of the (rare) err chain fallback: one row-major plane.
inline int bx_err_rows(int w, int h, int pb) {
    for (int t = h; t >= 1; t--)
        if (4 * bx_round4(t * w) <= pb) return t;
    return 1;
}

// Large-window kernel (lk_kernel_lg, psn_lk_large.hip: box windows the box kernel
// cannot hold in registers). Per workgroup an HBM slot of the window values
// (3 x 256 x K uint2: I*, Ix*, Iy* of every quad as packed pairs, K quads per
// thread) and LDS: the chain-check records | a union of one row band of the I
// patch + Scharr plane (A phase) and the double-buffered tile planes of the
// ordered-chain fallbacks (A: 3 planes of TQ quads, b: 2 of TQ).
constexpr int kLgNT = 256;
// fallback tile sizes (quads per tile; <= 192: waves 1-3 write a tile, one quad
// per thread): the kernel is built for each, the planner takes the largest whose
// workgroup keeps the J region in LDS within kLgJrMaxLds, else (J from the
// level) kLgTQNoJr
constexpr int kLgTQs[2] = {192, 128};
constexpr int kLgTQNoJr = 128;
constexpr int kLgTQE = 128;  // quads per err fallback tile (one row-major chain)
__host__ __device__ constexpr int lg_sreg(int tq) { return ((tq + 15) & ~15) + 4; }  // SSE chain region (floats)
__host__ __device__ constexpr int lg_plane(int tq) { return 4 * lg_sreg(tq) + ((4 * tq + 15) & ~15) + 4; }
__host__ __device__ constexpr int lg_scr_bytes() { return align16((kBxXInts + 32) * 4); }
__host__ __device__ constexpr int lg_tiles_a_bytes(int tq) { return 2 * 3 * lg_plane(tq) * 4 + 1024; }
// + slack: the chain sums read up to 5 blocks past a chain (discarded)
__host__ __device__ constexpr int lg_tiles_b_bytes(int tq) { return 2 * 2 * lg_plane(tq) * 4 + 1024; }
// A phase band: tr + 3 rows of the I patch, bx_pm(w) dwords each
__host__ __device__ inline int lg_band_bytes(int w, int tr) { return align16((tr + 3) * 4 * bx_pm(w)); }
// J region of the iterations (lg_jr): st_jreg_h(h) rows of bx_jrp(w) bytes, after the b tiles
__host__ __device__ inline int lg_jr_bytes(int w, int h) { return align16(st_jreg_h(h) * bx_jrp(w)); }
// b fallback by parity records (psn_lk_xb.h; build parameter PSN_LG_XB, off by
// default: measured slower than the ordered tiles): 10
// chains x 256 threads of 8-B run records in the b tile region, and a pool of
// the HARD runs' terms after the J region
#ifndef PSN_LG_XB
#define PSN_LG_XB 0
#endif
constexpr int kXbRecBytes = 10 * 256 * 8;
#ifndef PSN_LG_POOL_KB
#define PSN_LG_POOL_KB 8
#endif
constexpr int kLgPoolBytes = PSN_LG_XB ? PSN_LG_POOL_KB * 1024 : 0;
__host__ __device__ constexpr int lg_iter_region(int tq) {
    return !PSN_LG_XB || lg_tiles_b_bytes(tq) > kXbRecBytes + 64 ? lg_tiles_b_bytes(tq) : kXbRecBytes + 64;
}
__host__ __device__ inline int lg_lds_bytes(int w, int h, int tr, bool jr, int tq) {
    int u = lg_band_bytes(w, tr);
    u = u > lg_tiles_a_bytes(tq) ? u : lg_tiles_a_bytes(tq);
    const int it = lg_iter_region(tq) + (jr ? lg_jr_bytes(w, h) : 0) + kLgPoolBytes;
    return lg_scr_bytes() + (u > it ? u : it);
}
#ifndef PSN_LG_JR_MAX_KB
#define PSN_LG_JR_MAX_KB 80
#endif
constexpr int kLgJrMaxLds = PSN_LG_JR_MAX_KB * 1024;  // J region in LDS while the workgroup fits this (80 KB: 2 per CU)
__host__ __device__ inline int lg_quads_per_thread(int w, int h) { return (h * ((w + 3) >> 2) + kLgNT - 1) / kLgNT; }
// window-value slot of one workgroup, in 8-byte units
__host__ __device__ inline long long lg_slot_int2(int w, int h) { return 3LL * kLgNT * lg_quads_per_thread(w, h); }

// ---- pyramid tiles (pyramid_kernel, and the builds fused into lk_kernel_st) ----
// Region of level l (l < top) that a top-level tile needs, per axis:
// start = 2^(top-l)*t0 - 2*(2^(top-l)-1), size = 2^(top-l)*T + 3*(2^(top-l)-1).
__host__ __device__ constexpr int pyr_region_n(int top, int l, int T) {
    return (1 << (top - l)) * T + 3 * ((1 << (top - l)) - 1);
}
// Level-0 region rows in LDS: the region starts at an aligned-down column
// (offset 0..3) so interior rows move as dwords.
__host__ __device__ constexpr int pyr_s0(int n0) { return (n0 + 3 + 3) & ~3; }
__host__ __device__ constexpr int pyr_lds_off(int top, int l, int T) {
    int off = 0;
    for (int m = 0; m < l; m++) {
        const int n = pyr_region_n(top, m, T);
        off += align16(m == 0 ? pyr_s0(n) * n : n * n);
    }
    return off;
}
__host__ __device__ constexpr int pyr_lds_bytes(int top, int T) {
    return top == 0 ? 0 : pyr_lds_off(top, top, T) + align16(2 * pyr_region_n(top, 0, T) * pyr_region_n(top, 1, T));
}
// Top-level tile edge of a build (a build parameter, PSN_PYR_TILE; tops past 4
// take 4)
#ifndef PSN_PYR_TILE
#define PSN_PYR_TILE 8
#endif
constexpr int kPyrTile = PSN_PYR_TILE;
constexpr int kPyrTileDeep = 4;
__host__ __device__ constexpr int pyr_tile_edge(int top) { return top <= 4 ? kPyrTile : kPyrTileDeep; }
// Build-time guards (a bad build parameter fails the compile instead of a launch
// with hipErrorInvalidValue): every top level a context may build, standalone and
// fused behind the single-tile kernel's scratch, fits the CU's LDS.
constexpr int kMaxLdsBytes = 160 * 1024;
__host__ __device__ constexpr bool pyr_tiles_fit(int top) {
    return top > kPyrMaxTop || (kStScratchBytes + pyr_lds_bytes(top, pyr_tile_edge(top)) <= kMaxLdsBytes &&
                                pyr_tiles_fit(top + 1));
}
static_assert(kPyrTile >= 1 && pyr_tiles_fit(1), "PSN_PYR_TILE: a pyramid tile's LDS plan exceeds 160 KB");
// The large-window kernel's LDS plan: its A tiles of every tile size beside the
// records, and the J-region cap
static_assert(lg_scr_bytes() + lg_tiles_a_bytes(kLgTQs[0]) <= kMaxLdsBytes &&
                  lg_scr_bytes() + lg_tiles_a_bytes(kLgTQs[1]) <= kMaxLdsBytes,
              "kLgTQs: a large-window tile plan exceeds 160 KB");
static_assert(kLgJrMaxLds > 0 && kLgJrMaxLds <= kMaxLdsBytes, "PSN_LG_JR_MAX_KB exceeds 160 KB");
static_assert(kBxMaxLds <= kMaxLdsBytes && kBxLdsTarget <= kBxMaxLds && 2 * kBxMaxLds2 <= kMaxLdsBytes,
              "box-kernel LDS caps exceed 160 KB");

constexpr int kStEPTMax = 4;  // window pixels per thread held in registers by the single-tile kernel
constexpr int kStMaxLds = 150 * 1024;

// Launchers (psn_lk_kernels.hip).
hipError_t launch_pyramid(const PyrBuildArgs &a, hipStream_t s);
void pyramid_grid(const PyrBuildArgs &a, int &tiles_x, int &tiles_y, int &lds_bytes);
// threads: tiled kernel = workgroup size; single-tile kernel = NT * 10 + EPT,
// plus 1000 * E for the one-wave iteration mode (E window rows per lane).
hipError_t launch_lk(const LkLaunchArgs &a, int total_wgs, int threads, int lds_bytes, bool single_tile, hipStream_t s);
// Box-window kernel with UPT units per thread (4, 8, 10 or 12).
// notail: every query of the launch sums in the SSE2 order with width % 8 == 0
// (no scalar-tail chain: a build without its per-pixel bookkeeping)
hipError_t launch_lk_bx(const LkLaunchArgs &a, int total_wgs, int upt, bool notail, int lds_bytes, hipStream_t s);
// Large-window kernel (psn_lk_large.hip): `grid` workgroups over a.lk_wgs points.
hipError_t launch_lk_lg(const LkLaunchArgs &a, int grid, int lds_bytes, int tq, hipStream_t s);
hipError_t lg_kernels_init();
hipError_t lk_kernels_init();   // raises the dynamic-LDS limit once

}  // namespace psn
