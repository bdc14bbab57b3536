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

/*
 * Per-thread parity records with local HARD runs (the lk_kernel_lg b / A
 * fallback of round 5): the chain from segment fs on,
 * starting at the exact integer value `base` (every earlier prefix exact).
 *   - B_t exact prefix at segment t, (m_t, M_t) its local prefix extremes (0
 *     included), E_t = 8 * (terms from the start of segment fs to the end of t)
 *     + 64: bounds |s - P| for every value of the segment and its representatives
 *     while every |P| + E < 2^28 (ulp <= 16); past that the evaluation aborts
 *     (returns NAN: the caller keeps its ordered tiles).
 *   - key: 23 when [B + m - E, B + M + E] lies in [-2^24, 2^24] (no rounding: the
 *     segment adds its exact total T), k >= 24 when it lies inside one binade of
 *     |v| (grid u = 2^(k-23)), else HARD (its terms summed in order).
 *   - a binade segment is a HEAD when the previous segment is not of key k (or
 *     is HARD): its first term is added explicitly (s may sit on a finer grid),
 *     the rest is a parity function (Q0, D): from a start s on the grid u, the
 *     segment moves s by u * (Q0 + D * parity(s / u)), D in {-1, 0, 1}, found by
 *     replaying it from two representatives of either parity near the start.
 *   - the walk: per segment in order, s from the exact start.
 * stats: [0] records walked, [1] HARD segments, [2] HARD terms, [3] heads,
 * [4] 1 = aborted.
 */
static int key_abs(long long a) { /* a >= 0: 23 for a <= 2^24, else floor(log2 a) */
    if (a <= (1LL << 24)) return 23;
    int k = 63 - __builtin_clzll((unsigned long long)a);
    return k;
}
float oracle_chain_runs(const float *f, const int *seg_off, int nseg, int fs, int base, int *stats) {
    int recs = 0, hard = 0, hterms = 0, heads = 0;
    if (stats) memset(stats, 0, 5 * sizeof(int));
    enum { kMax = 4096 };
    static __thread int key[kMax];
    static __thread long long Bv[kMax + 1];
    if (nseg > kMax) return NAN;
    long long P = base;
    const int a0 = seg_off[fs];
    for (int t = fs; t < nseg; t++) {
        const int a = seg_off[t], b = seg_off[t + 1];
        Bv[t] = P;
        long long m = 0, M = 0, q = 0;
        for (int i = a; i < b; i++) {
            if (fabsf(f[i]) > 16777216.f) {
                if (stats) stats[4] = 1;
                return NAN;
            }
            q += (long long)f[i];
            if (q < m) m = q;
            if (q > M) M = q;
        }
        P += q;
        const long long E = 8LL * (b - a0) + 64;
        const long long lo = Bv[t] + m - E, hi = Bv[t] + M + E;
        if (hi >= (1LL << 28) || lo <= -(1LL << 28)) {
            if (stats) stats[4] = 1;
            return NAN;
        }
        int k;
        if (lo >= -(1LL << 24) && hi <= (1LL << 24))
            k = 23;
        else if (lo > (1LL << 24)) {
            k = key_abs(lo);
            if (key_abs(hi) != k || hi >= (2LL << k)) k = -1;
        } else if (hi < -(1LL << 24)) {
            k = key_abs(-hi);
            if (key_abs(-lo) != k || -lo >= (2LL << k)) k = -1;
        } else
            k = -1;
        key[t] = b > a ? k : (t > fs ? key[t - 1] : 23);
    }
    float s = (float)base;
    for (int t = fs; t < nseg; t++) {
        const int a = seg_off[t], b = seg_off[t + 1];
        if (b == a) continue;
        const int k = key[t];
        recs++;
        if (k < 0) {
            hard++;
            hterms += b - a;
            for (int i = a; i < b; i++) s = s + f[i];
            continue;
        }
        if (k == 23) {
            long long T = 0;
            for (int i = a; i < b; i++) T += (long long)f[i];
            s = (float)((long long)s + T);
            continue;
        }
        const long long u = 1LL << (k - 23);
        const int head = t == fs || key[t - 1] != k;
        int i0 = a;
        long long near = Bv[t];
        if (head) {
            heads++;
            s = s + f[a];
            near += (long long)f[a];
            i0 = a + 1;
        }
        /* representatives: the multiple of 2u nearest `near`, and it + u */
        const long long R0 = (long long)llround((double)near / (double)(2 * u)) * 2 * u;
        float r0 = (float)R0, r1 = (float)(R0 + u);
        for (int i = i0; i < b; i++) {
            r0 = r0 + f[i];
            r1 = r1 + f[i];
        }
        const long long Q0 = ((long long)r0 - R0) / u, Q1 = ((long long)r1 - (R0 + u)) / u;
        const long long D = Q1 - Q0;
        if (D < -1 || D > 1) {
            if (stats) stats[4] = 2;
            return NAN;
        }
        uint32_t bits;
        memcpy(&bits, &s, 4);
        const int p = (int)(bits & 1u);
        s = (float)((long long)s + u * (Q0 + D * p));
    }
    if (stats) {
        stats[0] = recs;
        stats[1] = hard;
        stats[2] = hterms;
        stats[3] = heads;
    }
    return s;
}
