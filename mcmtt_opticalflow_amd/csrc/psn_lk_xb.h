// psn_lk_xb.h -- an ordered float chain of the LK sums (LKTrackerInvoker, OpenCV
// 2.4.6: the SSE2 build's lane chains and the scalar tail chain, float sums of
// integer products) evaluated as per-thread PARITY RECORDS, bit for bit the
// sequential sum. Used by lk_kernel_lg's b fallback; CPU model and its proof
// obligations: oracle/chain_model.c oracle_chain_runs (tests/test_chain_model.py).
//
// Every thread of the workgroup owns a contiguous run of each chain's terms and
// knows, from the exactness scan, the run's exact integer start prefix B and its
// local prefix extremes m <= 0 <= M. With s the chain's float value and P the
// exact prefix, |s - P| <= E = (terms since the ordered start) * u_max / 2, u_max
// the grid of the largest |P|. The run's values s + t then lie in
// [B + m - E, B + M + E]:
//   * inside [-2^24, 2^24] (key 23): no step rounds, the run adds its exact total;
//   * inside one binade [2^k, 2^(k+1)) of |v| (key k, grid u = 2^(k-23)): every
//     step rounds to the grid u with ties to even, so once s is on the grid the
//     run moves it by u * (Q0 + D * parity(s / u)), D in {-1, 0, 1} (two starts
//     of opposite parity merge at the first tie) -- a parity function, found by
//     replaying the run in float from two representatives of either parity;
//   * otherwise the run is HARD: its terms are added one by one.
// The walk (one lane per chain, the runs in order) adds each run's FIRST term as
// a float add (s may sit on a finer grid when the key changes) and applies the
// parity function of the rest; HARD runs' terms come from an LDS pool.
#pragma once

#include "psn_lk_bx.h"

namespace psn {

// Key of the value range [lo, hi]: 23 = exact zone, k >= 24 = one binade of |v|
// (k = floor(log2 |v|) on the whole range), -1 = neither. |lo|, |hi| < 2^30.
__device__ __forceinline__ int xb_key(int lo, int hi) {
    if (lo >= -(1 << 24) && hi <= (1 << 24)) return 23;
    if (lo > (1 << 24)) {
        const int k = 31 - __builtin_clz((unsigned)lo);
        return hi < (2 << k) ? k : -1;
    }
    if (hi < -(1 << 24)) {
        const int k = 31 - __builtin_clz((unsigned)-hi);
        return -lo < (2 << k) ? k : -1;
    }
    return -1;
}

// Run record (int2): x = Q0 (units of the grid; key 23: the exact total of the
// run's terms after the first) or, HARD, the pool offset of its terms; y = the
// first term (26-bit signed; HARD: the term count) | (key - 23) << 26 | (D + 1) << 29
// | HARD << 31. A run without terms is a HARD run of 0 terms.
constexpr int kXbChains = 10;
constexpr int kXbRecThreads = 256;
static_assert(kXbRecBytes == kXbChains * kXbRecThreads * 8, "record region");
__device__ __forceinline__ int2 xb_rec(int q0, int f1, int ks, int D) {
    return make_int2(q0, (f1 & 0x3ffffff) | (ks << 26) | ((D + 1) << 29));
}
__device__ __forceinline__ int2 xb_rec_hard(int off, int cnt) { return make_int2(off, (int)(0x80000000u | (unsigned)cnt)); }

// One chain's walk over the records [t0, t1) of the chain's row (stride 1),
// from the exact value s. Serial by nature: one lane per chain.
__device__ __forceinline__ float xb_walk(const int2 *rec, const float *pool, int t0, int t1, float s) {
    for (int t = t0; t < t1; t++) {
        const int2 r = rec[t];
        if (r.y < 0) {  // HARD: its terms in order
            const int cnt = r.y & 0x3ffffff;
            const float *p = pool + r.x;
            for (int i = 0; i < cnt; i++) s = __fadd_rn(s, p[i]);
        } else {
            const int f1 = (r.y << 6) >> 6, ks = (r.y >> 26) & 7, D = ((r.y >> 29) & 3) - 1;
            s = __fadd_rn(s, (float)f1);
            if (ks == 0) {
                s = (float)((int)s + r.x);  // no rounding in [-2^24, 2^24]
            } else {
                const int q = r.x + D * (__float_as_int(s) & 1);  // parity of s / u: the mantissa LSB
                s = __fadd_rn(s, (float)(q << ks));                // lands on a float: exact
            }
        }
    }
    return s;
}

}  // namespace psn
