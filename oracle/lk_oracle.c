#include <stdio.h>
/*
 * oracle/lk_oracle.c -- TEST INFRASTRUCTURE ONLY (see lk_oracle.h).
 *
 * A plain-C restatement of the OpenCV 2.4.6 code that
 * CPSNWhere_Tracker2D reaches through cv::calcOpticalFlowPyrLK
 * (psn_where/PSNWhere_Tracker2D.cpp:776-782 and :871-877), plus the ingest
 * step cv::cvtColor(BGR2GRAY) + cv::resize(scale 1.0) (:257, :262).
 *
 * PARITY UNPINNED (no reference fixtures exist; OpenCV 2.4.6 is absent).
 *
 * Built with -O2 -ffp-contract=off so float arithmetic is IEEE single
 * rounding per operation with no FMA contraction, as MSVC x64 (/fp:precise,
 * SSE2 scalar math) evaluates the same expressions.
 */
#include "lk_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Optional per-point statistics (analysis only): iterations run per level and
 * how many b-sums / A-sums stayed within the exact-integer bound 2^24. */
static int *g_iter_log = 0; /* [npts][8] iterations at level l */
void oracle_set_iter_log(int *buf) { g_iter_log = buf; }
/* b-sum exactness classes (analysis only): [0] b-sums evaluated, [1] sum|t1|+sum|t2| <= 2^24,
 * [2] max(sum|t1|, sum|t2|) <= 2^24, [3] every SSE2 chain sum|t| <= 2^24, [4] every chain's
 * every prefix |P| <= 2^24 and every |t| <= 2^24 (sequential float sum == integer sum), [5] every pixel class
 * (SSE2 lane or tail) sum|t1|+|t2| <= 2^24. */
static long long *g_bsum_log = 0;
void oracle_set_bsum_log(long long *buf) { g_bsum_log = buf; }
static long long *g_chain_log = 0;
static int g_chain_upt = 0;
/* the per-thread parity-record model on every fallback evaluation (buf[16..24]:
 * the caller's buffer holds ORACLE_CHAIN_LOG_ENTRIES = 25 entries, lk_oracle.h) */
static int g_chain_log_ext = 0;
static int g_chain_fs = 256, g_chain_ls = -1;
static float g_chain_ser[10];
static float *g_chain_terms[10];
static int g_chain_off[10][257];
static size_t g_chain_cap = 0;
void oracle_set_chain_log(long long *buf, int upt) {
    g_chain_log = buf;
    g_chain_upt = upt;
    g_chain_log_ext = buf != 0;
}
/* lk_kernel_bx's chains of one b-sum evaluation through the binade-run model.
 * buf: [0] evaluations, [1] of them on the exact fast path (every prefix of every
 * chain an exact integer), [2] model != sequential sum (must stay 0), [3] sum over
 * fallback evaluations of the longest serial walk (records + HARD terms) of a
 * chain, [4] its maximum, [5] records, [6] HARD segments, [7] HARD terms, [8] max
 * records of one chain in one wave, [9] max HARD segments of one chain in one
 * wave, [10] fallback evaluations. */
static void chain_classify(const long long *t1, const long long *t2, int w, int h, int sse) {
    const int QW = (w + 3) / 4, U = h * QW, nqB = sse ? (w / 8) * 2 : 0;
    const int need = (U + 255) / 256;
    const int upt = g_chain_upt > 0 ? g_chain_upt : need <= 4 ? 4 : need <= 8 ? 8 : need <= 10 ? 10 : 12;
    float *f = (float *)malloc(sizeof(float) * (size_t)w * h);
    if (g_chain_log_ext && g_chain_cap < (size_t)w * h) {
        for (int i = 0; i < 10; i++) {
            free(g_chain_terms[i]);
            g_chain_terms[i] = (float *)malloc(sizeof(float) * (size_t)w * h);
        }
        g_chain_cap = (size_t)w * h;
    }
    int off[257];
    int exact = 1, walk_max = 0, st[5];
    long long recs = 0, hard = 0, hterms = 0;
    int mrec = 0, mhard = 0, mismatch = 0;
    float res[10];
    for (int cc = 0; cc < 10; cc++) {
        const long long *tv = cc < 5 ? t1 : t2;
        const int c = cc % 5;
        int n = 0;
        for (int t = 0; t < 256; t++) {
            off[t] = n;
            for (int k = 0; k < upt; k++) {
                const int un = t * upt + k;
                if (un >= U) break;
                const int y = un / QW, q = un % QW;
                if (q < nqB) {
                    if (c < 4) f[n++] = (float)tv[y * w + 4 * q + c];
                } else if (c == 4) {
                    for (int i = 0; i < 4; i++)
                        if (4 * q + i < w) f[n++] = (float)tv[y * w + 4 * q + i];
                }
            }
        }
        off[256] = n;
        long long P = 0;
        for (int i = 0; i < n; i++) {
            P += (long long)f[i];
            if (llabs((long long)f[i]) > (1LL << 24) || llabs(P) > (1LL << 24)) exact = 0;
        }
        const float ser = oracle_chain_serial(f, n);
        const float mod = oracle_chain_binade(f, n, off, 256, 64, st);
        if (g_chain_log_ext) { /* [16] evaluations with a fallback, [17] sum of the longest chain walk
                                * (records + HARD terms), [18] aborted, [19] mismatches, [20] serial
                                * terms from the first failing thread (longest chain), [21] HARD terms */
            int fs = 256;
            long long Pq = 0;
            for (int t = 0; t < 256 && fs == 256; t++) {
                long long M = Pq, m = Pq;
                for (int i = off[t]; i < off[t + 1]; i++) {
                    Pq += (long long)f[i];
                    if (Pq > M) M = Pq;
                    if (Pq < m) m = Pq;
                    if (fabsf(f[i]) > 16777216.f) M = 1LL << 30;
                }
                if (M > (1LL << 24) || m < -(1LL << 24)) fs = t;
            }
            if (fs < g_chain_fs) g_chain_fs = fs;
            {   /* [22] last thread whose run leaves |prefix| <= 2^24 - 2^16 (max over chains) */
                int ls = -1;
                long long Pr = 0;
                for (int t = 0; t < 256; t++) {
                    long long M = Pr, m = Pr;
                    for (int i = off[t]; i < off[t + 1]; i++) {
                        Pr += (long long)f[i];
                        if (Pr > M) M = Pr;
                        if (Pr < m) m = Pr;
                        if (fabsf(f[i]) > 16777216.f) M = 1LL << 30;
                    }
                    if (M > (1LL << 24) - (1LL << 16) || m < -((1LL << 24) - (1LL << 16))) ls = t;
                }
                if (ls > g_chain_ls) g_chain_ls = ls;
            }
            g_chain_ser[cc] = ser;
            memcpy(g_chain_terms[cc], f, sizeof(float) * (size_t)n);
            memcpy(g_chain_off[cc], off, sizeof(off));
        }
        {   /* [11] terms after the chain's first inexact step, [12] of them the steps whose
             * accumulator stays below 2^24 - 2^16 in magnitude (exact integer additions),
             * [13] the same in blocks of 16 terms whose every step qualifies */
            float acc = 0.f;
            int first = -1;
            long long P = 0;
            for (int i = 0; i < n; i++) {
                P += (long long)f[i];
                if (first < 0 && (llabs(P) > (1LL << 24) || llabs((long long)f[i]) > (1LL << 24))) first = i;
            }
            if (first >= 0) {
                int blk_ok = 1, blk_n = 0;
                for (int i = 0; i < n; i++) {
                    acc = acc + f[i];
                    if (i < first) continue;
                    const int ok = fabsf(acc) < (float)((1 << 24) - (1 << 16));
                    g_chain_log[11]++;
                    g_chain_log[12] += ok;
                    blk_ok &= ok;
                    if (++blk_n == 16) {
                        if (blk_ok) g_chain_log[13] += 16;
                        blk_ok = 1;
                        blk_n = 0;
                    }
                }
            }
        }
        if (memcmp(&ser, &mod, 4) != 0) mismatch = 1;
        res[cc] = ser;
        recs += st[0];
        hard += st[1];
        hterms += st[2];
        if (st[0] + st[2] > walk_max) walk_max = st[0] + st[2];
        if (st[3] > mrec) mrec = st[3];
        if (st[4] > mhard) mhard = st[4];
    }
    (void)res;
    if (g_chain_log_ext && g_chain_fs < 256) { /* the kernel's fallback: every chain from the first failing thread */
        const int fs = g_chain_fs;
        int walk_max = 0, ser_max = 0;
        g_chain_log[16]++;
        for (int cc = 0; cc < 10; cc++) {
            const float *fc = g_chain_terms[cc];
            const int *oc = g_chain_off[cc];
            long long base = 0;
            for (int i = 0; i < oc[fs]; i++) base += (long long)fc[i];
            int st2[5];
            const float r = oracle_chain_runs(fc, oc, 256, fs, (int)base, st2);
            if (r != r) {
                g_chain_log[18]++;
                continue;
            }
            if (memcmp(&r, &g_chain_ser[cc], 4) != 0) {
                if (g_chain_log[19]++ == 0 && getenv("CHAIN_DUMP")) {
                    FILE *fp = fopen(getenv("CHAIN_DUMP"), "wb");
                    if (fp) {
                        int hdr[3] = {fs, (int)base, oc[256]};
                        fwrite(hdr, 4, 3, fp);
                        fwrite(oc, 4, 257, fp);
                        fwrite(fc, 4, (size_t)oc[256], fp);
                        fclose(fp);
                    }
                }
            }
            if (st2[0] + st2[2] > walk_max) walk_max = st2[0] + st2[2];
            if (oc[256] - oc[fs] > ser_max) ser_max = oc[256] - oc[fs];
            g_chain_log[21] += st2[2];
        }
        g_chain_log[17] += walk_max;
        g_chain_log[20] += ser_max;
        {   /* [22] serial terms of the longest chain from the first failing thread to the
             * end of the last one whose run leaves a prefix above 2^24 - 2^16, [23] threads
             * from the first to that last failing one, [24] threads from the first to the end */
            int cut_max = 0;
            for (int cc = 0; cc < 10; cc++) {
                const int *oc = g_chain_off[cc];
                const int e = g_chain_ls + 1 > fs ? g_chain_ls + 1 : fs;
                if (oc[e] - oc[fs] > cut_max) cut_max = oc[e] - oc[fs];
            }
            g_chain_log[22] += cut_max;
            g_chain_log[23] += g_chain_ls + 1 - fs;
            g_chain_log[24] += 256 - fs;
        }
    }
    g_chain_fs = 256;
    g_chain_ls = -1;
    free(f);
    g_chain_log[0]++;
    g_chain_log[2] += mismatch;
    if (exact) {
        g_chain_log[1]++;
        return;
    }
    g_chain_log[10]++;
    g_chain_log[3] += walk_max;
    if (walk_max > g_chain_log[4]) g_chain_log[4] = walk_max;
    g_chain_log[5] += recs;
    g_chain_log[6] += hard;
    g_chain_log[7] += hterms;
    if (mrec > g_chain_log[8]) g_chain_log[8] = mrec;
    if (mhard > g_chain_log[9]) g_chain_log[9] = mhard;
}
static void bsum_classify(const long long *t1, const long long *t2, int w, int h, int sse) {
    const long long E = 1LL << 24;
    long long a1 = 0, a2 = 0, ca[10] = {0}, p[10] = {0};
    int ok4 = 1;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const int n8 = sse ? (w / 8) * 8 : 0;
            const int c = x < n8 ? (x & 3) : 4;
            const long long u = t1[y * w + x], v = t2[y * w + x];
            a1 += llabs(u);
            a2 += llabs(v);
            ca[c] += llabs(u);
            ca[5 + c] += llabs(v);
            p[c] += u;
            p[5 + c] += v;
            if (llabs(u) > E || llabs(v) > E || llabs(p[c]) > E || llabs(p[5 + c]) > E) ok4 = 0;
        }
    int ok3 = 1;
    for (int c = 0; c < 10; c++)
        if (ca[c] > E) ok3 = 0;
    int ok5 = 1;
    for (int c = 0; c < 5; c++)
        if (ca[c] + ca[5 + c] > E) ok5 = 0;
    g_bsum_log[5] += ok5;
    /* lane model of the one-wave kernel: lane = (column in class order, group of RG rows) */
    {
        const int G = w <= 64 ? 64 / w : 1, RG = (h + G - 1) / G;
        const int n8 = sse ? (w / 8) * 8 : 0, cw = n8 / 4;
        long long la1[64] = {0}, la2[64] = {0};
        int lcls[64];
        for (int l = 0; l < 64; l++) lcls[l] = -1;
        for (int r = 0; r < w && r * G < 64; r++) {
            const int x = r < n8 ? r / cw + 4 * (r % cw) : r;
            const int c = r < n8 ? r / cw : 4;
            for (int g = 0; g < G; g++) {
                const int lane = r * G + g;
                if (lane >= 64) continue;
                lcls[lane] = c;
                for (int k = 0; k < RG; k++) {
                    const int y = g * RG + k;
                    if (y >= h) break;
                    la1[lane] += llabs(t1[y * w + x]);
                    la2[lane] += llabs(t2[y * w + x]);
                }
            }
        }
        /* (B) max lane value x lanes per class */
        long long mx = 0;
        int cnt[5] = {0};
        for (int l = 0; l < 64; l++) {
            if (lcls[l] < 0) continue;
            cnt[lcls[l]]++;
            if (la1[l] > mx) mx = la1[l];
            if (la2[l] > mx) mx = la2[l];
        }
        int mc = 0;
        for (int c = 0; c < 5; c++) mc = cnt[c] > mc ? cnt[c] : mc;
        g_bsum_log[6] += mx * mc <= E;
        /* (D) 16-lane row sums, class bound = rows it touches */
        long long r1[4] = {0}, r2[4] = {0};
        for (int l = 0; l < 64; l++) { r1[l / 16] += la1[l]; r2[l / 16] += la2[l]; }
        int okd = 1;
        for (int c = 0; c < 5; c++) {
            int rlo = 4, rhi = -1;
            for (int l = 0; l < 64; l++) if (lcls[l] == c) { if (l / 16 < rlo) rlo = l / 16; if (l / 16 > rhi) rhi = l / 16; }
            long long b1 = 0, b2 = 0;
            for (int r = rlo; r <= rhi; r++) { b1 += r1[r]; b2 += r2[r]; }
            if (b1 > E || b2 > E) okd = 0;
        }
        g_bsum_log[7] += okd;
    }
    {   /* [8] max(sum of positive terms, sum of |negative terms|) <= 2^24 for b1 and b2:
         * every subset sum (any order, any chain split) is then an exact integer */
        long long P1 = 0, N1 = 0, P2 = 0, N2 = 0;
        for (int i = 0; i < w * h; i++) {
            if (t1[i] > 0) P1 += t1[i]; else N1 -= t1[i];
            if (t2[i] > 0) P2 += t2[i]; else N2 -= t2[i];
        }
        g_bsum_log[8] += P1 <= E && N1 <= E && P2 <= E && N2 <= E;
    }
    {   /* [9] per-mille of the longest chain suffix from the first prefix violation (serial
         * work of a fallback that starts each chain at its first violation); [10] the same
         * for a common start (shortest exact prefix over the chains) */
        const int n8 = sse ? (w / 8) * 8 : 0;
        long long P[10] = {0};
        int first[10], len[10] = {0};
        for (int c = 0; c < 10; c++) first[c] = -1;
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                const int c = x < n8 ? (x & 3) : 4;
                const long long tt[2] = {t1[y * w + x], t2[y * w + x]};
                for (int s = 0; s < 2; s++) {
                    const int cc = 5 * s + c;
                    P[cc] += tt[s];
                    if (first[cc] < 0 && (llabs(tt[s]) > E || llabs(P[cc]) > E)) first[cc] = len[cc];
                    len[cc]++;
                }
            }
        long long worst = 0, common = 0;
        for (int c = 0; c < 10; c++) {
            if (!len[c]) continue;
            const long long suf = first[c] < 0 ? 0 : 1000LL * (len[c] - first[c]) / len[c];
            if (suf > worst) worst = suf;
        }
        int minfirst = 1 << 30;
        for (int c = 0; c < 10; c++)
            if (len[c] && first[c] >= 0) {
                const int f = (int)(1000LL * first[c] / len[c]);
                if (f < minfirst) minfirst = f;
            }
        common = minfirst == (1 << 30) ? 0 : 1000 - minfirst;
        g_bsum_log[9] += worst;
        g_bsum_log[10] += common;
    }
    {   /* [11] passes of a parity-scan evaluation of the float chains (binade of every step
         * guessed from the exact prefix, restarted at the first failed guess), summed over
         * b-sums that need one; [12] such b-sums; [13] max passes of one b-sum; [14] steps
         * whose exact sum reaches 2^27 or more */
        const int n8 = sse ? (w / 8) * 8 : 0;
        int npass_max = 0, need = 0;
        for (int cc = 0; cc < 10; cc++) {
            const int s2 = cc / 5, c = cc % 5;
            long long tv[16384];
            int n = 0;
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++) {
                    const int cx = x < n8 ? (x & 3) : 4;
                    if (cx != c) continue;
                    tv[n++] = (long long)(float)(s2 ? t2[y * w + x] : t1[y * w + x]);
                }
            /* true chain */
            long long st = 0;
            int inexact = 0, passes = 0, pos = 0;
            long long S = 0;
            while (pos < n) {
                passes++;
                long long P = S, s = S;
                int k = pos, fail = -1;
                for (; k < n; k++) {
                    const long long xg = P + tv[k];
                    long long ax = llabs(xg);
                    long long u = 1;
                    while (ax >= (1LL << 24) * u * 2 || (ax >= (1LL << 24) && u == 1 && ax >= (1LL << 24))) {
                        if (ax < (1LL << 24) * 2 * u && u > 1) break;
                        if (ax >= (1LL << 25) * u) u *= 2; else { if (ax >= (1LL << 24)) u = u < 2 ? 2 : u; break; }
                    }
                    /* u_true of the model state */
                    const long long xt = s + tv[k];
                    long long axt = llabs(xt), ut = 1;
                    while (axt >= (1LL << 24) * ut) ut *= 2;
                    if (ut > 1) ut /= 1;
                    /* ulp: 1 below 2^24, 2 in [2^24, 2^25), ... */
                    long long ug = 1;
                    { long long a2x = llabs(xg); while (a2x >= (1LL << 24) * ug) ug *= 2; }
                    if (ug != ut || (s % ut) != 0) { fail = k; break; }
                    if (ax >= (1LL << 27)) g_bsum_log[14]++;
                    /* round xt to a multiple of ut, ties to even */
                    long long r = ((xt % ut) + ut) % ut, base = xt - r;
                    if (2 * r > ut || (2 * r == ut && ((base / ut) & 1))) base += ut;
                    if (ut > 1) inexact = 1;
                    s = base;
                    P += tv[k];
                }
                if (fail < 0) break;
                {   /* the true step at the failure */
                    const long long xt = s + tv[fail];
                    long long axt = llabs(xt), ut = 1;
                    while (axt >= (1LL << 24) * ut) ut *= 2;
                    long long r = ((xt % ut) + ut) % ut, base = xt - r;
                    if (2 * r > ut || (2 * r == ut && ((base / ut) & 1))) base += ut;
                    S = base;
                    pos = fail + 1;
                    inexact = 1;
                }
            }
            (void)st;
            if (inexact) {
                need = 1;
                if (passes > npass_max) npass_max = passes;
            }
        }
        if (need) {
            g_bsum_log[11] += npass_max;
            g_bsum_log[12]++;
            if (npass_max > g_bsum_log[13]) g_bsum_log[13] = npass_max;
        }
    }
    g_bsum_log[0]++;
    g_bsum_log[1] += (a1 + a2) <= E;
    g_bsum_log[2] += (a1 <= E && a2 <= E);
    g_bsum_log[3] += ok3;
    g_bsum_log[4] += ok4;
}

#define W_BITS 14
#define W_BITS1 14
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

/* cv::borderInterpolate(p, len, BORDER_REFLECT_101) [OCV246 core/src/copy.cpp]:
 * "-1 -> 1, len -> len-2", repeated until inside. */
int oracle_refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p; /* -p - 1 + delta, delta = 1 */
        else
            p = 2 * len - 2 - p; /* len - 1 - (p - len) - delta */
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* cv::cvRound(double) on SSE2 = cvtsd2si = round half to even. */
static inline int cv_round(float v) { return (int)rint((double)v); }
static inline int cv_floor(float v) { return (int)floor((double)v); }

/* RGB2Gray<uchar> [OCV246 imgproc/src/color.cpp]: R2Y=4899, G2Y=9617, B2Y=1868,
 * yuv_shift=14, half added through the R table. Called from
 * PSNWhere_Tracker2D.cpp:257 (CV_BGR2GRAY: src[0]=B, src[1]=G, src[2]=R). */
void oracle_bgr2gray(const uint8_t *src, int w, int h, int sstride, uint8_t *dst, int dstride) {
    for (int y = 0; y < h; y++) {
        const uint8_t *s = src + (long)y * sstride;
        uint8_t *d = dst + (long)y * dstride;
        for (int x = 0; x < w; x++)
            d[x] = (uint8_t)((s[3 * x] * 1868 + s[3 * x + 1] * 9617 + s[3 * x + 2] * 4899 + (1 << 13)) >> 14);
    }
}

/* pyrDown_<FixPtCast<uchar,8>> [OCV246 imgproc/src/pyramids.cpp]: separable
 * [1 4 6 4 1]^2, (sum + 128) >> 8, reflect-101 on the SOURCE size. Integer,
 * so the row ring buffer / SSE2 vecOp order is immaterial. */
/* Threads of the full-frame passes (pyrDown, borders, Scharr) inside one
 * calcOpticalFlowPyrLK call (cpu_baseline legs: they scale with the cores as
 * the points do); set per call, 1 outside. Integer row passes: the thread
 * count cannot change a result. */
static int g_rows_threads = 1;
#define ROWS_PAR _Pragma("omp parallel for schedule(static) num_threads(g_rows_threads) if(g_rows_threads > 1)")

void oracle_pyr_down(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dstride) {
    static const int k[5] = {1, 4, 6, 4, 1};
    int dw = (sw + 1) / 2, dh = (sh + 1) / 2;
    int *cx = (int *)malloc(sizeof(int) * 5 * dw);
    for (int x = 0; x < dw; x++)
        for (int j = 0; j < 5; j++) cx[x * 5 + j] = oracle_refl101(2 * x + j - 2, sw);
    ROWS_PAR
    for (int y = 0; y < dh; y++) {
        const uint8_t *rows[5];
        for (int i = 0; i < 5; i++) rows[i] = src + (long)oracle_refl101(2 * y + i - 2, sh) * sstride;
        for (int x = 0; x < dw; x++) {
            int acc = 0;
            for (int i = 0; i < 5; i++) {
                int r = 0;
                for (int j = 0; j < 5; j++) r += k[j] * rows[i][cx[x * 5 + j]];
                acc += k[i] * r;
            }
            dst[(long)y * dstride + x] = (uint8_t)((acc + 128) >> 8);
        }
    }
    free(cx);
}

/* calcSharrDeriv [OCV246 video/src/lkpyramid.cpp]: vertical (3,10,3) / (-1,0,1)
 * pass with reflect-101 rows, horizontal pass with reflect-101 columns of the
 * filtered rows; interleaved int16 (Ix, Iy). */
void oracle_scharr(const uint8_t *src, int w, int h, int sstride, int16_t *dst, int dstride) {
    ROWS_PAR
    for (int y = 0; y < h; y++) {
        int *t0 = (int *)malloc(sizeof(int) * 2 * (w + 2)), *t1 = t0 + w + 2;
        const uint8_t *s0 = src + (long)(y > 0 ? y - 1 : h > 1 ? 1 : 0) * sstride;
        const uint8_t *s1 = src + (long)y * sstride;
        const uint8_t *s2 = src + (long)(y < h - 1 ? y + 1 : h > 1 ? h - 2 : 0) * sstride;
        for (int x = 0; x < w; x++) {
            t0[x + 1] = (s0[x] + s2[x]) * 3 + s1[x] * 10;
            t1[x + 1] = s2[x] - s0[x];
        }
        int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
        t0[0] = t0[x0 + 1];
        t0[w + 1] = t0[x1 + 1];
        t1[0] = t1[x0 + 1];
        t1[w + 1] = t1[x1 + 1];
        int16_t *d = dst + (long)y * dstride;
        for (int x = 0; x < w; x++) {
            d[2 * x] = (int16_t)(t0[x + 2] - t0[x]);
            d[2 * x + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
        }
        free(t0);
    }
}

/* buildOpticalFlowPyramid's stop rule [OCV246 video/src/lkpyramid.cpp]: after
 * level `l` is built, sz = ((w+1)/2, (h+1)/2); stop (maxLevel = l) when
 * sz.width <= winW || sz.height <= winH. */
int oracle_effective_max_level(int w, int h, int win_w, int win_h, int max_level) {
    int sw = w, sh = h;
    for (int level = 0; level <= max_level; level++) {
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win_w || sh <= win_h) return level;
    }
    return max_level;
}

void oracle_level_size(int w, int h, int level, int *lw, int *lh) {
    for (int l = 0; l < level; l++) {
        w = (w + 1) / 2;
        h = (h + 1) / 2;
    }
    *lw = w;
    *lh = h;
}

long oracle_level_offset(int w, int h, int level) {
    long off = 0;
    for (int l = 0; l < level; l++) {
        off += (long)w * h;
        w = (w + 1) / 2;
        h = (h + 1) / 2;
    }
    return off;
}

/* Level 0 = the image (its reflect-101 border is applied on read), level l+1 =
 * pyrDown(level l) on the level's own ROI (BORDER_ISOLATED in 2.4.6). */
void oracle_build_pyramid(const uint8_t *img, int w, int h, int stride, int nlevels, uint8_t *pyr) {
    for (int y = 0; y < h; y++) memcpy(pyr + (long)y * w, img + (long)y * stride, (size_t)w);
    int lw = w, lh = h;
    long off = 0;
    for (int l = 1; l < nlevels; l++) {
        int nw = (lw + 1) / 2, nh = (lh + 1) / 2;
        oracle_pyr_down(pyr + off, lw, lh, lw, pyr + off + (long)lw * lh, nw);
        off += (long)lw * lh;
        lw = nw;
        lh = nh;
    }
}

/* A level as calcOpticalFlowPyrLK sees it: I and J padded by winSize with
 * reflect-101 (copyMakeBorder(..., BORDER_REFLECT_101), buildOpticalFlowPyramid)
 * and the Scharr plane of I padded by winSize with zeros
 * (copyMakeBorder(derivI, ..., BORDER_CONSTANT|BORDER_ISOLATED)). Pointers
 * address the ROI origin; strides are in elements. */
typedef struct {
    const uint8_t *I, *J;
    const int16_t *dI;
    int stepI, dstep; /* dstep in int16 elements (2 per pixel) */
    int cols, rows;
} level_view;

/* copyMakeBorder(src, dst, bh, bh, bw, bw, BORDER_REFLECT_101) */
static void pad_reflect(const uint8_t *src, int cols, int rows, int bw, int bh, uint8_t *dst) {
    int dcols = cols + 2 * bw;
    int *tab = (int *)malloc(sizeof(int) * dcols);
    for (int x = 0; x < dcols; x++) tab[x] = oracle_refl101(x - bw, cols);
    ROWS_PAR
    for (int y = 0; y < rows + 2 * bh; y++) {
        const uint8_t *s = src + (long)oracle_refl101(y - bh, rows) * cols;
        uint8_t *d = dst + (long)y * dcols;
        memcpy(d + bw, s, (size_t)cols);
        for (int x = 0; x < bw; x++) d[x] = s[tab[x]];
        for (int x = bw + cols; x < dcols; x++) d[x] = s[tab[x]];
    }
    free(tab);
}

/* Scharr of `src` into a zero-bordered interleaved int16 buffer. */
static void scharr_padded(const uint8_t *src, int cols, int rows, int bw, int bh, int16_t *dst) {
    int dcols = cols + 2 * bw;
    ROWS_PAR
    for (int y = 0; y < rows + 2 * bh; y++) memset(dst + (long)y * 2 * dcols, 0, sizeof(int16_t) * 2 * (size_t)dcols);
    oracle_scharr(src, cols, rows, cols, dst + ((long)bh * dcols + bw) * 2, 2 * dcols);
}

#define BILIN(p, s, w00, w01, w10, w11) ((p)[0] * (w00) + (p)[1] * (w01) + (p)[s] * (w10) + (p)[(s) + 1] * (w11))
#define BILIN_D(p, s, c, w00, w01, w10, w11) \
    ((p)[c] * (w00) + (p)[2 + (c)] * (w01) + (p)[(s) + (c)] * (w10) + (p)[(s) + 2 + (c)] * (w11))

/* LKTrackerInvoker::operator() [OCV246 video/src/lkpyramid.cpp] for one point at
 * one level. nextPts/status/err are the shared output arrays. The SSE2 build
 * keeps 4 float lanes for A (4-pixel steps) and 2x4 lanes for b (8-pixel
 * steps) next to a scalar tail; both are reproduced literally (accum == SSE2). */
static void lk_point_level(const level_view *lv, int level, int max_level, const float *prev_pts,
                           float *next_pts, uint8_t *status, float *err, int i, int win_w,
                           int win_h, int max_count, double eps2, int flags, float min_eig_thr,
                           int accum, int16_t *ibuf /* 3*win_w*win_h */) {
    const float hwx = (float)(win_w - 1) * 0.5f, hwy = (float)(win_h - 1) * 0.5f;
    const float scale = (float)(1. / (1 << level));
    const int cols = lv->cols, rows = lv->rows;
    const int sse = accum == ORACLE_ACCUM_SSE2;
    const int exact = accum == ORACLE_ACCUM_EXACT;
    const int stepI = lv->stepI, dstep = lv->dstep;
    int16_t *Iw = ibuf, *dIw = ibuf + win_w * win_h; /* dIw interleaved (Ix, Iy) */

    float px = prev_pts[2 * i] * scale, py = prev_pts[2 * i + 1] * scale;
    float nx, ny;
    if (level == max_level) {
        if (flags & ORACLE_USE_INITIAL_FLOW) {
            nx = next_pts[2 * i] * scale;
            ny = next_pts[2 * i + 1] * scale;
        } else {
            nx = px;
            ny = py;
        }
    } else {
        nx = next_pts[2 * i] * 2.f;
        ny = next_pts[2 * i + 1] * 2.f;
    }
    next_pts[2 * i] = nx;
    next_pts[2 * i + 1] = ny;

    px -= hwx;
    py -= hwy;
    int ipx = cv_floor(px), ipy = cv_floor(py);
    if (ipx < -win_w || ipx >= cols || ipy < -win_h || ipy >= rows) {
        if (level == 0) {
            status[i] = 0;
            if (err) err[i] = 0;
        }
        return;
    }

    float a = px - (float)ipx, b = py - (float)ipy;
    int iw00 = cv_round((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
    int iw01 = cv_round(a * (1.f - b) * (float)(1 << W_BITS));
    int iw10 = cv_round((1.f - a) * b * (float)(1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

    float A11 = 0, A12 = 0, A22 = 0;
    float qA11[4] = {0, 0, 0, 0}, qA12[4] = {0, 0, 0, 0}, qA22[4] = {0, 0, 0, 0};
    long long eA11 = 0, eA12 = 0, eA22 = 0;
    for (int y = 0; y < win_h; y++) {
        const uint8_t *src = lv->I + (long)(y + ipy) * stepI + ipx;
        const int16_t *dsrc = lv->dI + (long)(y + ipy) * dstep + 2 * ipx;
        int16_t *Iptr = Iw + y * win_w, *dIptr = dIw + 2 * y * win_w;
        int x = 0;
        if (sse) {
            for (; x <= win_w - 4; x += 4) {
                int ixv[4], iyv[4];
                for (int k = 0; k < 4; k++) {
                    Iptr[x + k] = (int16_t)DESCALE(BILIN(src + x + k, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5);
                    ixv[k] = DESCALE(BILIN_D(dsrc + 2 * (x + k), dstep, 0, iw00, iw01, iw10, iw11), W_BITS1);
                    iyv[k] = DESCALE(BILIN_D(dsrc + 2 * (x + k), dstep, 1, iw00, iw01, iw10, iw11), W_BITS1);
                    dIptr[2 * (x + k)] = (int16_t)ixv[k];
                    dIptr[2 * (x + k) + 1] = (int16_t)iyv[k];
                }
                for (int k = 0; k < 4; k++) {
                    float fx = (float)ixv[k], fy = (float)iyv[k];
                    qA22[k] += fy * fy;
                    qA12[k] += fx * fy;
                    qA11[k] += fx * fx;
                }
            }
        }
        for (; x < win_w; x++) {
            int ival = DESCALE(BILIN(src + x, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5);
            int ixval = DESCALE(BILIN_D(dsrc + 2 * x, dstep, 0, iw00, iw01, iw10, iw11), W_BITS1);
            int iyval = DESCALE(BILIN_D(dsrc + 2 * x, dstep, 1, iw00, iw01, iw10, iw11), W_BITS1);
            Iptr[x] = (int16_t)ival;
            dIptr[2 * x] = (int16_t)ixval;
            dIptr[2 * x + 1] = (int16_t)iyval;
            if (exact) {
                eA11 += (long long)ixval * ixval;
                eA12 += (long long)ixval * iyval;
                eA22 += (long long)iyval * iyval;
                continue;
            }
            A11 += (float)(ixval * ixval);
            A12 += (float)(ixval * iyval);
            A22 += (float)(iyval * iyval);
        }
    }
    if (exact) {
        A11 = (float)eA11;
        A12 = (float)eA12;
        A22 = (float)eA22;
    }
    if (sse) {
        A11 += qA11[0] + qA11[1] + qA11[2] + qA11[3];
        A12 += qA12[0] + qA12[1] + qA12[2] + qA12[3];
        A22 += qA22[0] + qA22[1] + qA22[2] + qA22[3];
    }

    const float FLT_SCALE = 1.f / (1 << 20);
    A11 *= FLT_SCALE;
    A12 *= FLT_SCALE;
    A22 *= FLT_SCALE;

    float D = A11 * A22 - A12 * A12;
    float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win_w * win_h);

    if (err && (flags & ORACLE_GET_MIN_EIGENVALS) != 0) err[i] = minEig;

    if (minEig < min_eig_thr || D < FLT_EPSILON) {
        if (level == 0) status[i] = 0;
        return;
    }

    D = 1.f / D;
    nx -= hwx;
    ny -= hwy;
    float pdx = 0.f, pdy = 0.f;

    for (int j = 0; j < max_count; j++) {
        if (g_iter_log) g_iter_log[i * 8 + level]++;
        int inx = cv_floor(nx), iny = cv_floor(ny);
        if (inx < -win_w || inx >= cols || iny < -win_h || iny >= rows) {
            if (level == 0) status[i] = 0;
            break;
        }
        a = nx - (float)inx;
        b = ny - (float)iny;
        iw00 = cv_round((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
        iw01 = cv_round(a * (1.f - b) * (float)(1 << W_BITS));
        iw10 = cv_round((1.f - a) * b * (float)(1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        float b1 = 0, b2 = 0;
        float qb0[4] = {0, 0, 0, 0}, qb1[4] = {0, 0, 0, 0};
        long long eb1 = 0, eb2 = 0;
        if (g_bsum_log || g_chain_log) {
            long long *t1 = (long long *)malloc(sizeof(long long) * 2 * win_w * win_h), *t2 = t1 + win_w * win_h;
            for (int y = 0; y < win_h; y++)
                for (int x = 0; x < win_w; x++) {
                    const uint8_t *Jp = lv->J + (long)(y + iny) * stepI + inx + x;
                    const int d = DESCALE(BILIN(Jp, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5) - Iw[y * win_w + x];
                    t1[y * win_w + x] = (long long)d * dIw[2 * (y * win_w + x)];
                    t2[y * win_w + x] = (long long)d * dIw[2 * (y * win_w + x) + 1];
                }
            if (g_bsum_log) bsum_classify(t1, t2, win_w, win_h, sse);
            if (g_chain_log) chain_classify(t1, t2, win_w, win_h, sse);
            free(t1);
        }
        for (int y = 0; y < win_h; y++) {
            const uint8_t *Jptr = lv->J + (long)(y + iny) * stepI + inx;
            const int16_t *Iptr = Iw + y * win_w, *dIptr = dIw + 2 * y * win_w;
            int x = 0;
            if (sse) {
                for (; x <= win_w - 8; x += 8) {
                    int d[8];
                    for (int k = 0; k < 8; k++)
                        d[k] = DESCALE(BILIN(Jptr + x + k, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5) - Iptr[x + k];
                    const int16_t *g = dIptr + 2 * x;
                    /* diff0 = pixels 0..3: lanes qb0 <- (0,1), qb1 <- (2,3) */
                    qb0[0] += (float)(g[0] * d[0]);
                    qb0[1] += (float)(g[1] * d[0]);
                    qb0[2] += (float)(g[2] * d[1]);
                    qb0[3] += (float)(g[3] * d[1]);
                    qb1[0] += (float)(g[4] * d[2]);
                    qb1[1] += (float)(g[5] * d[2]);
                    qb1[2] += (float)(g[6] * d[3]);
                    qb1[3] += (float)(g[7] * d[3]);
                    /* diff1 = pixels 4..7: qb0 <- (4,5), qb1 <- (6,7) */
                    qb0[0] += (float)(g[8] * d[4]);
                    qb0[1] += (float)(g[9] * d[4]);
                    qb0[2] += (float)(g[10] * d[5]);
                    qb0[3] += (float)(g[11] * d[5]);
                    qb1[0] += (float)(g[12] * d[6]);
                    qb1[1] += (float)(g[13] * d[6]);
                    qb1[2] += (float)(g[14] * d[7]);
                    qb1[3] += (float)(g[15] * d[7]);
                }
            }
            for (; x < win_w; x++) {
                int diff = DESCALE(BILIN(Jptr + x, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5) - Iptr[x];
                if (exact) {
                    eb1 += (long long)diff * dIptr[2 * x];
                    eb2 += (long long)diff * dIptr[2 * x + 1];
                    continue;
                }
                b1 += (float)(diff * dIptr[2 * x]);
                b2 += (float)(diff * dIptr[2 * x + 1]);
            }
        }
        if (exact) {
            b1 = (float)eb1;
            b2 = (float)eb2;
        }
        if (sse) {
            float bb[4];
            for (int k = 0; k < 4; k++) bb[k] = qb0[k] + qb1[k];
            b1 += bb[0] + bb[2];
            b2 += bb[1] + bb[3];
        }
        b1 *= FLT_SCALE;
        b2 *= FLT_SCALE;

        float dx = (float)((A12 * b2 - A22 * b1) * D);
        float dy = (float)((A12 * b1 - A11 * b2) * D);
        nx += dx;
        ny += dy;
        next_pts[2 * i] = nx + hwx;
        next_pts[2 * i + 1] = ny + hwy;

        if ((double)dx * (double)dx + (double)dy * (double)dy <= eps2) break;
        if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
            next_pts[2 * i] -= dx * 0.5f;
            next_pts[2 * i + 1] -= dy * 0.5f;
            break;
        }
        pdx = dx;
        pdy = dy;
    }

    if (status[i] && err && level == 0 && (flags & ORACLE_GET_MIN_EIGENVALS) == 0) {
        float qx = next_pts[2 * i] - hwx, qy = next_pts[2 * i + 1] - hwy;
        int iqx = cv_floor(qx), iqy = cv_floor(qy);
        if (iqx < -win_w || iqx >= cols || iqy < -win_h || iqy >= rows) {
            status[i] = 0;
            return;
        }
        float aa = qx - (float)iqx, bb = qy - (float)iqy;
        iw00 = cv_round((1.f - aa) * (1.f - bb) * (float)(1 << W_BITS));
        iw01 = cv_round(aa * (1.f - bb) * (float)(1 << W_BITS));
        iw10 = cv_round((1.f - aa) * bb * (float)(1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        float errval = 0.f;
        long long eerr = 0;
        for (int y = 0; y < win_h; y++) {
            const uint8_t *Jptr = lv->J + (long)(y + iqy) * stepI + iqx;
            const int16_t *Iptr = Iw + y * win_w;
            for (int x = 0; x < win_w; x++) {
                int diff = DESCALE(BILIN(Jptr + x, stepI, iw00, iw01, iw10, iw11), W_BITS1 - 5) - Iptr[x];
                if (exact)
                    eerr += diff < 0 ? -diff : diff;
                else
                    errval += fabsf((float)diff);
            }
        }
        if (exact) errval = (float)eerr;
        err[i] = errval * 1.f / (float)(32 * win_w * win_h);
    }
}

/* calcOpticalFlowPyrLK body [OCV246]: criteria clamp, status=1, then for
 * level = maxLevel..0 { calcSharrDeriv(prevPyr[level]) + zero border;
 * parallel_for_ over points (LKTrackerInvoker) }. */
int oracle_lk_track_pyr(const uint8_t *prev_pyr, const uint8_t *next_pyr, int w, int h,
                        const float *prev_pts, float *next_pts, uint8_t *status, float *err,
                        int npts, int win_w, int win_h, int max_level, int term_type,
                        int max_count, double epsilon, int flags, double min_eig_threshold,
                        int accum_mode, int nthreads) {
    if (win_w <= 2 || win_h <= 2 || max_level < 0) return -2;
    if (npts <= 0) return 0;
    if ((term_type & 1) == 0)
        max_count = 30;
    else
        max_count = max_count < 0 ? 0 : max_count > 100 ? 100 : max_count;
    if ((term_type & 2) == 0)
        epsilon = 0.01;
    else
        epsilon = epsilon < 0. ? 0. : epsilon > 10. ? 10. : epsilon;
    double eps2 = epsilon * epsilon;
    float min_eig_thr = (float)min_eig_threshold;

    for (int i = 0; i < npts; i++) status[i] = 1;
    if (err)
        for (int i = 0; i < npts; i++) err[i] = 0.f;

    size_t pad_px = (size_t)(w + 2 * win_w) * (h + 2 * win_h);
    uint8_t *Ipad = (uint8_t *)malloc(pad_px), *Jpad = (uint8_t *)malloc(pad_px);
    int16_t *Dpad = (int16_t *)malloc(sizeof(int16_t) * 2 * pad_px);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
    (void)nthreads;
#endif
    g_rows_threads = nthreads;
    for (int level = max_level; level >= 0; level--) {
        int cols, rows;
        oracle_level_size(w, h, level, &cols, &rows);
        const uint8_t *I = prev_pyr + oracle_level_offset(w, h, level);
        const uint8_t *J = next_pyr + oracle_level_offset(w, h, level);
        int pc = cols + 2 * win_w;
        pad_reflect(I, cols, rows, win_w, win_h, Ipad);
        pad_reflect(J, cols, rows, win_w, win_h, Jpad);
        scharr_padded(I, cols, rows, win_w, win_h, Dpad);
        level_view lv = {Ipad + (long)win_h * pc + win_w, Jpad + (long)win_h * pc + win_w,
                         Dpad + ((long)win_h * pc + win_w) * 2, pc, 2 * pc, cols, rows};
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
        {
            int16_t *ibuf = (int16_t *)malloc(sizeof(int16_t) * 3 * (size_t)win_w * win_h);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
            for (int i = 0; i < npts; i++)
                lk_point_level(&lv, level, max_level, prev_pts, next_pts, status, err, i, win_w, win_h,
                               max_count, eps2, flags, min_eig_thr, accum_mode, ibuf);
            free(ibuf);
        }
    }
    free(Ipad);
    free(Jpad);
    free(Dpad);
    g_rows_threads = 1;
    return 0;
}

int oracle_calc_optical_flow_pyr_lk(const uint8_t *prev_img, const uint8_t *next_img, int w, int h,
                                    int stride, const float *prev_pts, float *next_pts,
                                    uint8_t *status, float *err, int npts, int win_w, int win_h,
                                    int max_level, int term_type, int max_count, double epsilon,
                                    int flags, double min_eig_threshold, int accum_mode,
                                    int nthreads) {
    if (win_w <= 2 || win_h <= 2 || max_level < 0) return -2;
    if (npts <= 0) return 0;
    int ml = oracle_effective_max_level(w, h, win_w, win_h, max_level);
    long total = oracle_level_offset(w, h, ml + 1);
    uint8_t *pp = (uint8_t *)malloc((size_t)total), *np = (uint8_t *)malloc((size_t)total);
#ifdef _OPENMP
    g_rows_threads = nthreads > 0 ? nthreads : omp_get_max_threads();
#endif
    oracle_build_pyramid(prev_img, w, h, stride, ml + 1, pp);
    oracle_build_pyramid(next_img, w, h, stride, ml + 1, np);
    g_rows_threads = 1;
    int rc = oracle_lk_track_pyr(pp, np, w, h, prev_pts, next_pts, status, err, npts, win_w, win_h, ml,
                                 term_type, max_count, epsilon, flags, min_eig_threshold, accum_mode,
                                 nthreads);
    free(pp);
    free(np);
    return rc;
}
