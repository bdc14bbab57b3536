/*
 * oracle/chain_model.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A CPU model of the binade-run evaluation of an ordered float chain, the
 * algorithm lk_kernel_bx uses when a window sum leaves the exact-integer range
 * (the b sums of LKTrackerInvoker, OpenCV 2.4.6 video/src/lkpyramid.cpp, in the
 * SSE2 build's lane order; see DESIGN.md §3 "binade runs"). It is here so the
 * argument can be tested exhaustively on the CPU against the plain sequential
 * float sum (tests/test_chain_model.py) and so chain statistics of real
 * Tracker2D windows can be collected (oracle_set_chain_log in lk_oracle.c).
 *
 * The chain: s_0 = 0, s_i = fl(s_{i-1} + f_i), f_i floats with integer values
 * (each term is the float conversion of an integer product). Split into
 * segments (one per GPU thread, `seg_off`), waves of `wave` segments.
 *
 *  1. Exact prefixes: B_t = sum of the terms before segment t (exact), the
 *     segment's prefix range [B_t + m_t, B_t + M_t] (m_t <= 0 <= M_t).
 *  2. Error bound: |s_i - P_i| <= E = n * ulp(max |P|) / 2 for every step
 *     (each rounding moves s by at most half an ulp of a value <= max |P| + E).
 *  3. A segment is UNIFORM when every accumulator value v = s_{i-1} + f_i it can
 *     see (its prefix range widened by E + 2u) lies in one binade of |v|
 *     (key k = max(23, floor(log2 |v|)), grid u = 2^(k-23); k = 23 is the exact
 *     range |v| < 2^24, u = 1). Inside a binade, rounding to the grid u is
 *     invariant under shifts by 2u, so for any start s that is a multiple of u
 *     the segment maps s to s + u * Q[parity(s / u)]: a PARITY FUNCTION
 *     (Q0, Q1, p0', p1'), found by running the segment from two guessed starts
 *     (one of each parity) near B_t with real float adds.
 *  4. Runs: maximal groups of consecutive uniform segments with the same key.
 *     The run head's first step is executed as a float add (its incoming s may
 *     come from a finer grid); the rest of the head (Rest) and the following
 *     segments (Full) compose as parity functions. Per wave, one record per
 *     run piece: HEAD (f1, R0, R1) or CONT (R0, R1, a run continuing from the
 *     previous wave); a non-uniform segment is a HARD record (its terms).
 *  5. A serial walk over the records: HEAD s = fl(s + f1), then s += u*R[p];
 *     CONT s += u*R[p]; HARD sequential float adds. p = parity(s / u) = the
 *     mantissa LSB of s (|s| is in binade k there).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "lk_oracle.h"

static int key_of(double a) { /* a >= 0 */
    if (a < 16777216.0) return 23;
    int e;
    frexp(a, &e);
    return e - 1;
}
static int interval_key(double lo, double hi) {
    if (lo > 0) {
        const int a = key_of(lo), b = key_of(hi);
        return a == b ? a : -1;
    }
    if (hi < 0) {
        const int a = key_of(-hi), b = key_of(-lo);
        return a == b ? a : -1;
    }
    return fmax(-lo, hi) < 16777216.0 ? 23 : -1;
}
static unsigned parity_of(float s) {
    uint32_t b;
    memcpy(&b, &s, 4);
    return b & 1u;
}
static double round_to_2u(double x, double u) { return 2.0 * u * nearbyint(x / (2.0 * u)); }

typedef struct {
    long long Q[2];
    int p[2];
} pfun;
static pfun pf_compose(pfun a, pfun b) { /* a then b */
    pfun r;
    for (int i = 0; i < 2; i++) {
        r.Q[i] = a.Q[i] + b.Q[a.p[i]];
        r.p[i] = b.p[a.p[i]];
    }
    return r;
}
/* parity function of terms f[0..n) on grid u, guessed starts near `near` */
static pfun pf_run(const float *f, int n, double near, double u) {
    pfun r;
    for (int p = 0; p < 2; p++) {
        const double g = round_to_2u(near, u) + p * u;
        float s = (float)g;
        for (int i = 0; i < n; i++) s = s + f[i];
        r.Q[p] = (long long)(((double)s - g) / u);
        r.p[p] = u > 1.0 ? (int)parity_of(s) : (int)(((long long)s) & 1);
    }
    return r;
}

float oracle_chain_serial(const float *f, int n) {
    float s = 0.f;
    for (int i = 0; i < n; i++) s = s + f[i];
    return s;
}

float oracle_chain_binade(const float *f, int n, const int *seg_off, int nseg, int wave, int *stats) {
    /* stats: [0] records (HEAD + CONT), [1] HARD segments, [2] HARD terms, [3] max records of one wave,
     * [4] max HARD segments of one wave */
    enum { kMaxSeg = 4096 };
    static __thread int key[kMaxSeg];
    static __thread double B[kMaxSeg + 1];
    if (nseg > kMaxSeg) return NAN;
    double E;
    { /* E = n * ulp(max |P|) / 2, the slack 2^-9 |P| + 1024 covers |v| <= |P| + E */
        double P = 0, mx = 0;
        for (int i = 0; i < n; i++) {
            P += f[i];
            mx = fmax(mx, fabs(P));
        }
        const int kb = key_of(mx * (1.0 + 1.0 / 512) + 1024.0);
        E = kb == 23 ? 0.0 : n * ldexp(1.0, kb - 23) * 0.5;
    }
    B[0] = 0.0;
    for (int t = 0; t < nseg; t++) {
        const int a = seg_off[t], b = seg_off[t + 1];
        double P = B[t], M = B[t], m = B[t];
        for (int i = a; i < b; i++) {
            P += f[i];
            M = fmax(M, P);
            m = fmin(m, P);
        }
        B[t + 1] = P;
        int k = interval_key(m - E, M + E);
        if (k >= 0) {
            const double u = ldexp(1.0, k - 23);
            if (interval_key(m - E - 2 * u, M + E + 2 * u) != k) k = -1;
        }
        key[t] = b > a ? k : (t > 0 ? key[t - 1] : 23); /* empty segments join the run */
    }
    int recs = 0, hard = 0, hard_terms = 0, wrec = 0, whard = 0, max_wrec = 0, max_whard = 0;
    float s = 0.f;
    int t = 0;
    while (t < nseg) {
        if (t % wave == 0) {
            wrec = whard = 0;
        }
        const int a = seg_off[t], b = seg_off[t + 1];
        if (key[t] < 0) { /* HARD */
            for (int i = a; i < b; i++) s = s + f[i];
            hard++;
            hard_terms += b - a;
            whard++;
            max_whard = whard > max_whard ? whard : max_whard;
            t++;
            continue;
        }
        const int k = key[t];
        const double u = ldexp(1.0, k - 23);
        const int head = t == 0 || key[t - 1] != k;
        pfun R;
        int t1 = t + 1;
        if (head) {
            if (b > a) {
                s = s + f[a];
                R = pf_run(f + a + 1, b - a - 1, B[t] + f[a], u);
            } else {
                R = pf_run(f, 0, B[t], u);
            }
        } else {
            R = pf_run(f + a, b - a, B[t], u);
        }
        /* the rest of the run inside this wave */
        while (t1 < nseg && t1 % wave != 0 && key[t1] == k) {
            R = pf_compose(R, pf_run(f + seg_off[t1], seg_off[t1 + 1] - seg_off[t1], B[t1], u));
            t1++;
        }
        const int p = u > 1.0 ? (int)parity_of(s) : 0;
        s = (float)((double)s + u * (double)R.Q[p]);
        recs++;
        wrec++;
        max_wrec = wrec > max_wrec ? wrec : max_wrec;
        t = t1;
    }
    if (stats) {
        stats[0] = recs;
        stats[1] = hard;
        stats[2] = hard_terms;
        stats[3] = max_wrec;
        stats[4] = max_whard;
    }
    return s;
}
