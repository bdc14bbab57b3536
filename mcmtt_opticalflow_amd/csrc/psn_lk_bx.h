// Device helpers of the box-window LK kernel (lk_kernel_bx, psn_lk_kernels.hip)
// shared with the large-window kernel (lk_kernel_lg, psn_lk_large.hip): packed
// 16-bit dot products, the per-chain exactness records (publish / check / eval),
// the ordered LDS chain sums, the XCD-aware workgroup order. Internal.
#pragma once

#include "psn_lk_device.h"

namespace psn {

// v_dot2_i32_i16: a.lo*b.lo + a.hi*b.hi + c on signed 16-bit halves. Signed
// because iw11 = 2^14 - iw00 - iw01 - iw10 is -1 when the three rounded
// weights overshoot (tiny fractional offsets); pixels (<= 255) are positive.
__device__ __forceinline__ int sdot2(unsigned a, unsigned b, int c) {
    typedef short i16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, b), c, false);
}
__device__ __forceinline__ unsigned pack_w(int lo, int hi) { return ((unsigned)lo & 0xffffu) | ((unsigned)hi << 16); }
// sdot2 in the VOP3 form (separate accumulator input and result: no copy of a
// loop-invariant accumulator into the tied VOP2 destination)
__device__ __forceinline__ int sdot2v(unsigned a, unsigned b, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// v_dot2_u32_u16: a.lo*b.lo + a.hi*b.hi + c on unsigned 16-bit halves.
__device__ __forceinline__ unsigned udot2(unsigned a, unsigned b, unsigned c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c, false);
}
// Inclusive max / min scans over the 64 lanes (the wave_scan DPP sequence):
// lane 31 holds lanes 0-31, lane 63 the whole wave.
__device__ __forceinline__ int wave_max_scan(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ int wave_min_scan(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x142, 0xa, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x143, 0xc, 0xf, false));
    return v;
}

// Exactness of NC chains in three steps around two barriers (per-lane run total
// T, maximum prefix M >= 0 and minimum prefix m <= 0, prefixes relative to the
// run start). bx_publish: one wave scan per chain turns T into the exclusive
// prefix inside the wave, and lanes 31 / 63 record the half-wave / wave totals
// (rec[8c + 4 + wave], rec[8c + wave]). bx_check (after the first barrier):
// each lane adds the earlier waves' totals and tests its own extreme prefixes
// against 2^24; the wave's first failing half wave goes to rec[120 + wave]
// (8: none). bx_eval (after the second barrier): the verdict, chain c's total
// and its exact prefix before the first failing half wave, on lane c. int32 is
// enough: every value up to the first failing prefix is exact, and what a wrap
// past it produces is never read (only the FIRST failure counts).
constexpr int kBxHalfRec = 120;
template <int NC>
__device__ __forceinline__ void bx_publish(int (&T)[NC], int *rec, bool no_tail) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // every chain's scan first (independent DPP chains interleave: no hazard
    // waits between the steps of one scan), then the records in one exec region
    int incl[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) incl[c] = (no_tail && c % 5 == 4) ? 0 : wave_scan(T[c]);
    if (lane == 31 || lane == 63) {
        int *r = rec + wv + (lane == 31 ? 4 : 0);
#pragma unroll
        for (int c = 0; c < NC; c++) r[8 * c] = incl[c];
    }
#pragma unroll
    for (int c = 0; c < NC; c++) T[c] = incl[c] - T[c];
}
// one wave's test (WV: its index, a compile-time constant of the caller's
// scalar switch): the earlier waves' totals, then the extreme prefixes of all
// chains folded by v_max3 / v_min3 into one comparison each
template <int NC, int WV>
__device__ __forceinline__ bool bx_check_wave(const int (&E)[NC], const int (&M)[NC], const int (&m)[NC], const int *rec,
                                              bool no_tail) {
    int hi = 0, lo = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if (no_tail && c % 5 == 4) continue;
        const int *r = rec + 8 * c;
        int p = E[c];
        if (WV > 0) p += r[0];
        if (WV > 1) p += r[1];
        if (WV > 2) p += r[2];
        hi = max(hi, p + M[c]);
        lo = min(lo, p + m[c]);
    }
    return (hi > kExact) | (lo < -kExact);
}
template <int NC>
__device__ __forceinline__ void bx_check(const int (&E)[NC], const int (&M)[NC], const int (&m)[NC], bool bad, int *rec,
                                         bool no_tail) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);  // uniform: a scalar switch
    bool fail;
    switch (wv) {
        case 0: fail = bx_check_wave<NC, 0>(E, M, m, rec, no_tail); break;
        case 1: fail = bx_check_wave<NC, 1>(E, M, m, rec, no_tail); break;
        case 2: fail = bx_check_wave<NC, 2>(E, M, m, rec, no_tail); break;
        default: fail = bx_check_wave<NC, 3>(E, M, m, rec, no_tail); break;
    }
    const unsigned long long f = __ballot(fail | bad);
    if (lane == 0) rec[kBxHalfRec + wv] = f == 0ull ? 8 : 2 * wv + ((unsigned)f == 0u ? 1 : 0);
}
template <int NC>
__device__ __forceinline__ bool bx_eval(const int *rec, int &total, int &h0, int &base0) {
    const int lane = threadIdx.x & 63;
    const int c = lane < NC ? lane : 0;
    const int4 hh = *(const int4 *)(rec + kBxHalfRec);
    h0 = min(min(hh.x, hh.y), min(hh.z, hh.w));
    const int4 t = *(const int4 *)(rec + 8 * c), s = *(const int4 *)(rec + 8 * c + 4);
    total = t.x + t.y + t.z + t.w;
    const int hw = h0 >> 1;
    base0 = (hw > 0 ? t.x : 0) + (hw > 1 ? t.y : 0) + (hw > 2 ? t.z : 0) + (hw > 3 ? t.w : 0);
    if (h0 & 1) base0 += hw == 0 ? s.x : hw == 1 ? s.y : hw == 2 ? s.z : s.w;
    return h0 == 8;
}
// The same test at THREAD granularity (lk_kernel_lg: the ordered chains start at
// the first failing thread's run, not at its half wave; lk_kernel_bx keeps the
// half waves: the failing lane's prefixes kept live past the test spilled
// registers in every build of it): bx_check_t records each
// wave's first failing thread (256: none) and that thread's exact prefix of every
// chain (the block-exclusive prefix: every earlier prefix passed the test, so it
// is an exact integer); bx_eval_t returns the block's first failing thread f and,
// on lane c, chain c's total and its exact prefix before thread f.
constexpr int kBxThrRec = 128;  // [4 waves][16]: the first failing thread's prefixes
template <int NC>
__device__ __forceinline__ void bx_check_t(const int (&E)[NC], const int (&M)[NC], const int (&m)[NC], bool bad, int *rec,
                                           bool no_tail) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    int p[NC];
    int hi = 0, lo = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const int *r = rec + 8 * c;
        p[c] = E[c] + (wv > 0 ? r[0] : 0) + (wv > 1 ? r[1] : 0) + (wv > 2 ? r[2] : 0);
        if (no_tail && c % 5 == 4) continue;
        hi = max(hi, p[c] + M[c]);
        lo = min(lo, p[c] + m[c]);
    }
    const unsigned long long f = __ballot((hi > kExact) | (lo < -kExact) | bad);
    const int fl = f == 0ull ? 64 : __builtin_ctzll(f);
    if (lane == 0) rec[kBxHalfRec + wv] = f == 0ull ? 256 : 64 * wv + fl;
    if (lane == fl) {
#pragma unroll
        for (int c = 0; c < NC; c++) rec[kBxThrRec + 16 * wv + c] = p[c];
    }
}
template <int NC>
__device__ __forceinline__ bool bx_eval_t(const int *rec, int &total, int &f, int &base0) {
    const int lane = threadIdx.x & 63;
    const int c = lane < NC ? lane : 0;
    const int4 hh = *(const int4 *)(rec + kBxHalfRec);
    f = min(min(hh.x, hh.y), min(hh.z, hh.w));
    const int4 t = *(const int4 *)(rec + 8 * c);
    total = t.x + t.y + t.z + t.w;
    base0 = f < 256 ? rec[kBxThrRec + 16 * (f >> 6) + c] : 0;
    return f == 256;
}
__device__ __forceinline__ float rl_f(int v, int lane) { return (float)__builtin_amdgcn_readlane(v, lane); }

// chain-run update with one term
__device__ __forceinline__ void run_add(int &T, int &M, int &m, int t) {
    T += t;
    M = max(M, T);
    m = min(m, T);
}

__device__ __forceinline__ int lo16(unsigned v) { return (int)(short)(v & 0xffffu); }
__device__ __forceinline__ int hi16(unsigned v) { return (int)v >> 16; }
// v_dot2_i32_i16 in the VOP3 form with a scalar accumulator (a constant in an
// SGPR: no copy into a tied VOP2 destination per use)
__device__ __forceinline__ int sdot2k(unsigned a, unsigned b, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
// v_mad_i32_i16: int16 a (low half) x int16 half BH of b + c -- one instruction
// for a chain term's extraction, product and running sum (op_sel picks the half)
template <int BH>
__device__ __forceinline__ int mad16(int a, unsigned b, int c) {
    int r;
    if constexpr (BH)
        asm("v_mad_i32_i16 %0, %1, %2, %3 op_sel:[0,1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else
        asm("v_mad_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// the same with a's half AH: squares and cross products of packed gradient pairs
template <int AH, int BH>
__device__ __forceinline__ int mad16p(unsigned a, unsigned b, int c) {
    int r;
    if constexpr (AH && BH)
        asm("v_mad_i32_i16 %0, %1, %2, %3 op_sel:[1,1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else if constexpr (AH)
        asm("v_mad_i32_i16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else if constexpr (BH)
        asm("v_mad_i32_i16 %0, %1, %2, %3 op_sel:[0,1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else
        asm("v_mad_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// two terms of one chain run: total, maximum and minimum prefix (v_max3 / v_min3)
__device__ __forceinline__ void run2(int &T, int &M, int &m, int ta, int tb) {
    M = max(M, max(ta, tb));
    m = min(m, min(ta, tb));
    T = tb;
}
// an opaque 256 of the caller's loop (one VGPR): the accumulator constant below
// is then not loop-invariant, so no unit's constants are hoisted out of the loop
__device__ __forceinline__ int opaque256() {
    int c;
    asm volatile("v_mov_b32 %0, 256" : "=v"(c));
    return c;
}
// 256 - 512 I of the pair half picked by the scalar selector pair k ((-512, 0) or
// (0, -512)): one VOP3 v_dot2 (separate accumulator: no copy of c per use)
__device__ __forceinline__ int cw_dot(unsigned ip, unsigned k, int c) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(ip), "s"(k), "v"(c));
    return r;
}
// J - I of one unit (4 pixels) from the byte J region: rows jp and jp + JRP4
// (dwords), pairs selected by the uniform v_perm selectors s0..s3, packed-dot
// bilinear with the diff folded into the accumulator constant 256 - 512 I
// (I = the unit's window values, packed pairs ip; one v_dot2 each with the
// selector pairs (-512, 0) / (0, -512) and c256 = 256).
// (rows as two pointers: jp and jq = jp + JRP4)
__device__ __forceinline__ void bx_diffs2(const uint32_t *jp, const uint32_t *jq, unsigned W0, unsigned W1, unsigned s0,
                                          unsigned s1, unsigned s2, unsigned s3, const unsigned (&ip)[2], int (&d)[4],
                                          int c256) {
    const uint32_t a0 = jp[0], a1 = jp[1], b0 = jq[0], b1 = jq[1];
    const unsigned kl = 0x0000fe00u, kh = 0xfe000000u;  // (-512, 0), (0, -512)
    const int cw[4] = {cw_dot(ip[0], kl, c256), cw_dot(ip[0], kh, c256), cw_dot(ip[1], kl, c256), cw_dot(ip[1], kh, c256)};
    d[0] = sdot2(__builtin_amdgcn_perm(b1, b0, s0), W1, sdot2(__builtin_amdgcn_perm(a1, a0, s0), W0, cw[0])) >> 9;
    d[1] = sdot2(__builtin_amdgcn_perm(b1, b0, s1), W1, sdot2(__builtin_amdgcn_perm(a1, a0, s1), W0, cw[1])) >> 9;
    d[2] = sdot2(__builtin_amdgcn_perm(b1, b0, s2), W1, sdot2(__builtin_amdgcn_perm(a1, a0, s2), W0, cw[2])) >> 9;
    d[3] = sdot2(__builtin_amdgcn_perm(b1, b0, s3), W1, sdot2(__builtin_amdgcn_perm(a1, a0, s3), W0, cw[3])) >> 9;
}
__device__ __forceinline__ void bx_diffs(const uint32_t *jp, int JRP4, unsigned W0, unsigned W1, unsigned s0,
                                         unsigned s1, unsigned s2, unsigned s3, const unsigned (&ip)[2], int (&d)[4],
                                         int c256) {
    bx_diffs2(jp, jp + JRP4, W0, W1, s0, s1, s2, s3, ip, d, c256);
}
// pair selector: bytes (sj + i, sj + i + 1) of a row's 8-byte window -> J[x] | J[x+1] << 16
__device__ __forceinline__ unsigned bx_sel(int sj, int i) {
    return 0x0c000c00u | ((unsigned)(sj + i + 1) << 16) | (unsigned)(sj + i);
}

// Window values of one unit (window row yy, quad column qq: 4 pixels) from the
// level's I patch in LDS (rows of PM dwords from the window origin - (1, 1)
// aligned down to a dword, byte shift sh): Scharr derivatives on packed 16-bit
// pairs (zero outside the image unless IN: every derivative the window reads is
// inside), bilinear I*, Ix*, Iy* by v_dot2 (the rounding folded in) as packed
// pairs; gmx / gmn track the unit's gradients (pixels past w and invalid units
// (uv false) give zero gradients). Shared by lk_kernel_bx (register-resident
// units) and lk_kernel_lg (units streamed to its slot).
template <bool IN, bool NOTAIL>
__device__ __forceinline__ void bx_unit(const uint32_t *P32, int PM, int sh, int yy, int qq, bool uv, int w, int ipx,
                                        int ipy, int cols, int rows, int iw00, int iw01, int iw10, int iw11, int c256,
                                        int c8192, unsigned (&IPk)[2], unsigned (&XPk)[2], unsigned (&YPk)[2],
                                        int &gmx, int &gmn) {
    // the unit's 4 x 7-byte patch window as packed 16-bit pairs: even pairs
    // E[r][k] = (byte 2k, byte 2k+1), odd pairs O[r-1][k] = (2k+1, 2k+2) of rows 1, 2
    s16x2 E[4][4], O[2][2];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t *p = P32 + (yy + r) * PM + qq;
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
        E[r][0] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c010c00u));
        E[r][1] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c030c02u));
        E[r][2] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c050c04u));
        E[r][3] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c070c06u));
        if (r == 1 || r == 2) {
            O[r - 1][0] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c020c01u));
            O[r - 1][1] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(hi, lo, 0x0c040c03u));
        }
    }
    // column masks of pixels 2k, 2k+1 (zero derivative outside the image)
    unsigned cm[3];
#pragma unroll
    for (int kk = 0; kk < 3; kk++)
        cm[kk] = IN ? ~0u
                    : ((unsigned)(ipx + 4 * qq + 2 * kk) < (unsigned)cols ? 0xffffu : 0u) |
                          ((unsigned)(ipx + 4 * qq + 2 * kk + 1) < (unsigned)cols ? 0xffff0000u : 0u);
    // Scharr on packed pairs (|values| <= 4080: exact in 16 bits): DX/DY pairs
    // (2k, 2k+1) of the two derivative rows o = 0, 1
    unsigned DXp[2][3], DYp[2][3];
    const s16x2 k3 = {3, 3}, k10 = {10, 10};
#pragma unroll
    for (int o = 0; o < 2; o++) {
        const unsigned rm = IN || (unsigned)(ipy + yy + o) < (unsigned)rows ? ~0u : 0u;
        s16x2 SV[4], DV[4];
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
            SV[kk] = (E[o][kk] + E[o + 2][kk]) * k3 + E[o + 1][kk] * k10;
            DV[kk] = E[o + 2][kk] - E[o][kk];
        }
#pragma unroll
        for (int kk = 0; kk < 3; kk++) {
            const s16x2 dvo = __builtin_bit_cast(
                s16x2, __builtin_amdgcn_alignbyte(__builtin_bit_cast(unsigned, DV[kk + 1]),
                                                  __builtin_bit_cast(unsigned, DV[kk]), 2));
            const s16x2 dx = SV[kk + 1] - SV[kk];
            const s16x2 dy = (DV[kk] + DV[kk + 1]) * k3 + dvo * k10;
            DXp[o][kk] = __builtin_bit_cast(unsigned, dx) & cm[kk] & rm;
            DYp[o][kk] = __builtin_bit_cast(unsigned, dy) & cm[kk] & rm;
        }
    }
    // bilinear window values by v_dot2 on (x, x+1) pairs, rounding folded in
    const unsigned Wa = pack_w(iw00, iw01), Wb = pack_w(iw10, iw11);
    const unsigned b1p[4] = {__builtin_bit_cast(unsigned, O[0][0]), __builtin_bit_cast(unsigned, E[1][1]),
                             __builtin_bit_cast(unsigned, O[0][1]), __builtin_bit_cast(unsigned, E[1][2])};
    const unsigned b2p[4] = {__builtin_bit_cast(unsigned, O[1][0]), __builtin_bit_cast(unsigned, E[2][1]),
                             __builtin_bit_cast(unsigned, O[1][1]), __builtin_bit_cast(unsigned, E[2][2])};
    int ix[4], iy[4], iv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const bool pv = uv && (NOTAIL || 4 * qq + i < w);
        const int h = i >> 1;
        // pairs (i, i+1): even i from the stored pairs, odd i shifted by 16 bits
        const unsigned x0 = (i & 1) ? __builtin_amdgcn_alignbyte(DXp[0][h + 1], DXp[0][h], 2) : DXp[0][h];
        const unsigned x1 = (i & 1) ? __builtin_amdgcn_alignbyte(DXp[1][h + 1], DXp[1][h], 2) : DXp[1][h];
        const unsigned y0_ = (i & 1) ? __builtin_amdgcn_alignbyte(DYp[0][h + 1], DYp[0][h], 2) : DYp[0][h];
        const unsigned y1_ = (i & 1) ? __builtin_amdgcn_alignbyte(DYp[1][h + 1], DYp[1][h], 2) : DYp[1][h];
        iv[i] = sdot2(b2p[i], Wb, sdot2k(b1p[i], Wa, c256)) >> 9;
        const int gx = sdot2(x1, Wb, sdot2k(x0, Wa, c8192)) >> 14;
        const int gy = sdot2(y1_, Wb, sdot2k(y0_, Wa, c8192)) >> 14;
        ix[i] = gx & -(int)pv;
        iy[i] = gy & -(int)pv;
        gmx = max(gmx, max(ix[i], iy[i]));
        gmn = min(gmn, min(ix[i], iy[i]));
    }
    IPk[0] = pack_w(iv[0], iv[1]);
    IPk[1] = pack_w(iv[2], iv[3]);
    XPk[0] = pack_w(ix[0], ix[1]);
    XPk[1] = pack_w(ix[2], ix[3]);
    YPk[0] = pack_w(iy[0], iy[1]);
    YPk[1] = pack_w(iy[2], iy[3]);
}

// Ordered float sum of a zero-padded LDS chain (16-B aligned, ceil(len/16)
// blocks of 16 floats; +0 pads leave an integer-valued sum unchanged) onto acc,
// with one block in flight while one is summed: the LDS latency (~100 cycles)
// hides behind the 16 dependent adds. Blocks go to two register sets with fixed
// roles (the loop is unrolled by 2, so no in-flight register is ever copied); the loads
// and their lgkmcnt waits are inline asm, because as plain loads the compiler
// folds the loop-carried registers back into one load at the top of each step
// and waits there. nbmax = the wave's largest block count (uniform); lanes past
// their own chain keep acc (the blocks they read are discarded).
typedef float bxf4 __attribute__((ext_vector_type(4)));
#define BX_LD(v0, v1, v2, v3, addr, o0, o1, o2, o3)                                                   \
    asm volatile("ds_read_b128 %0, %4 offset:" #o0 "\n\tds_read_b128 %1, %4 offset:" #o1 "\n\t"           \
                 "ds_read_b128 %2, %4 offset:" #o2 "\n\tds_read_b128 %3, %4 offset:" #o3                  \
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)                                              \
                 : "v"(addr)                                                                           \
                 : "memory")
#define BX_WAIT4(v0, v1, v2, v3) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3))
__device__ __forceinline__ float add16m(float acc, const bxf4 &a, const bxf4 &b, const bxf4 &c, const bxf4 &d, bool on) {
    float t = acc;
    t = t + a.x; t = t + a.y; t = t + a.z; t = t + a.w;
    t = t + b.x; t = t + b.y; t = t + b.z; t = t + b.w;
    t = t + c.x; t = t + c.y; t = t + c.z; t = t + c.w;
    t = t + d.x; t = t + d.y; t = t + d.z; t = t + d.w;
    return on ? t : acc;
}
// Wave priority of the latency-critical sections of lk_kernel_bx (from the end of
// a main pass to the start of the next: publish, check, eval, results, solve,
// iteration head; the A publish / eval) over the throughput sections (A window,
// main passes) of the other workgroups on the SIMD; the ordered chains run at 3.
#ifndef PSN_BX_PRIO
#define PSN_BX_PRIO 1
#endif
// b fallback: tiles handed from their writer waves to the chain lanes through
// LDS flags (three buffers) rather than one workgroup barrier per tile
#ifndef PSN_BX_FLAGS
#define PSN_BX_FLAGS 1
#endif
__device__ __forceinline__ void bx_prio_hi() { __builtin_amdgcn_s_setprio(PSN_BX_PRIO); }
__device__ __forceinline__ void bx_prio_lo() { __builtin_amdgcn_s_setprio(0); }
// UNIFORM (no-tail builds): every chain lane has nbmax blocks, so no block is
// masked and the adds carry no select on the dependent chain; an odd last
// block is summed after the loop.
template <bool UNIFORM>
__device__ __forceinline__ float chain_sum_pl(const float *p, int len, int nbmax, float acc) {
    unsigned ad = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float *)p;
    const int nb = (len + 15) >> 4;
    if (nbmax <= 0) return acc;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the counts below are then exact
    // the chain is a dependent add sequence sharing its SIMD with other
    // workgroups' waves: issue it first
    __builtin_amdgcn_s_setprio(3);
    bxf4 a0, a1, a2, a3, c0, c1, c2, c3;
    BX_LD(a0, a1, a2, a3, ad, 0, 16, 32, 48);
    if constexpr (UNIFORM) {
        int b = 0;
        for (; b + 1 < nbmax; b += 2) {
            BX_LD(c0, c1, c2, c3, ad, 64, 80, 96, 112);
            BX_WAIT4(a0, a1, a2, a3);
            acc = add16m(acc, a0, a1, a2, a3, true);
            BX_LD(a0, a1, a2, a3, ad, 128, 144, 160, 176);
            BX_WAIT4(c0, c1, c2, c3);
            acc = add16m(acc, c0, c1, c2, c3, true);
            ad += 128u;
        }
        if (b < nbmax) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : : "memory");
            acc = add16m(acc, a0, a1, a2, a3, true);
        }
    } else {
        for (int b = 0; b < nbmax; b += 2) {
            BX_LD(c0, c1, c2, c3, ad, 64, 80, 96, 112);
            BX_WAIT4(a0, a1, a2, a3);
            acc = add16m(acc, a0, a1, a2, a3, b < nb);
            BX_LD(a0, a1, a2, a3, ad, 128, 144, 160, 176);
            BX_WAIT4(c0, c1, c2, c3);
            acc = add16m(acc, c0, c1, c2, c3, b + 1 < nb);
            ad += 128u;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : : "memory");
    __builtin_amdgcn_s_setprio(PSN_BX_PRIO);
    return acc;
}

// XCD-aware workgroup order (MI355X_MICROARCH.md, workgroup dispatch: blocks are
// dealt round-robin over the 8 XCDs, each with its own L2): hardware block b
// runs logical workgroup xcd_remap(b), so that logical workgroups [x*q, ...) --
// consecutive points of one box, whose windows overlap -- share one XCD's L2.
// A bijection for any n (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, j = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

}  // namespace psn
