/*
 * oracle/gridfast_oracle.c -- TEST INFRASTRUCTURE ONLY (linked into
 * liblk_oracle.so; only tests/ and bench.py's cpu_baseline leg load it).
 *
 * CPU restatement of the feature extraction CPSNWhere_Tracker2D runs for
 * every detection before its backward LK chain:
 *   m_detector = cv::FeatureDetector::create("GridFAST")      PSNWhere_Tracker2D.cpp:142
 *   mask(rectROI) = 255; m_detector->detect(gray, kps, mask)  :734-742
 *   if (kps.size() < 4) continue;                              :744
 *   std::random_shuffle(kps); first min(n, 100) points         :752-757
 * OpenCV 2.4.6 ("GridFAST" = GridAdaptedFeatureDetector(FastFeatureDetector
 * (threshold 10, nonmaxSuppression true), maxTotalKeypoints 1000, 4 x 4 grid),
 * modules/features2d/src/{detectors.cpp, fast.cpp, fast_score.cpp,
 * keypoint.cpp}) is not vendored in the reference and absent here: PARITY
 * UNPINNED, restated from the published algorithm and pinned by the
 * known-answer tests in tests/test_gridfast.py.
 *
 * Written the way OpenCV computes it (a different formulation from the HIP
 * kernel, which never runs a per-cell sub-image pass): every grid cell is a
 * sub-image of its own, FAST_t<16> runs on it with the 3-row score ring and the
 * early-exit cornerScore<16>, the mask filters afterwards
 * (KeyPointsFilter::runByPixelsMask), keepStrongest() trims each cell.
 *
 * The reference's two non-deterministic steps get a fixed definition (see
 * include/psn_lk.h, psn_gridfast_detect):
 *   - keepStrongest's std::nth_element leaves ties at the cut unspecified:
 *     here the earlier keypoint in detection (row-major) order wins, and the
 *     kept keypoints stay in detection order;
 *   - std::random_shuffle is unseeded: here the candidates are ordered by a
 *     seeded 32-bit hash of (seed, roi, index) -- a uniform random permutation
 *     of the same set -- and the first `cap` are taken.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lk_oracle.h"

/* fast.cpp makeOffsets(pixel, step, 16): the Bresenham circle of radius 3. */
static const int kCircle16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                     {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                     {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

/* fast_score.cpp cornerScore<16> (scalar build). */
static int corner_score16(const uint8_t *ptr, const int pixel[25], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[25];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        a = a < d[k + 3] ? a : d[k + 3];
        if (a <= a0) continue;
        for (int m = 4; m <= 8; m++) a = a < d[k + m] ? a : d[k + m];
        int t = a < d[k] ? a : d[k];
        a0 = a0 > t ? a0 : t;
        t = a < d[k + 9] ? a : d[k + 9];
        a0 = a0 > t ? a0 : t;
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int m = 3; m <= 5; m++) b = b > d[k + m] ? b : d[k + m];
        if (b >= b0) continue;
        for (int m = 6; m <= 8; m++) b = b > d[k + m] ? b : d[k + m];
        int t = b > d[k] ? b : d[k];
        b0 = b0 < t ? b0 : t;
        t = b > d[k + 9] ? b : d[k + 9];
        b0 = b0 < t ? b0 : t;
    }
    return -b0 - 1;
}

/* fast.cpp FAST_t<16>: keypoints of a w x h image in detection order
 * (row-major); kx/ky/kr receive up to `cap` entries, the count is returned. */
int oracle_fast16(const uint8_t *img, int w, int h, int stride, int threshold, int nonmax, int *kx, int *ky,
                  int *kr, int cap) {
    const int K = 8, N = 25;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kCircle16[k][0] + kCircle16[k][1] * stride;
    for (int k = 16; k < N; k++) pixel[k] = pixel[k - 16];
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (w < 1) return 0;
    uint8_t *buf[3];
    int *cpbuf[3];
    uint8_t *bufmem = (uint8_t *)calloc((size_t)w * 3, 1);
    int *cpmem = (int *)calloc((size_t)(w + 1) * 3, sizeof(int));
    for (int i = 0; i < 3; i++) {
        buf[i] = bufmem + (size_t)w * i;
        cpbuf[i] = cpmem + (size_t)(w + 1) * i + 1;
    }
    int n = 0;
    for (int i = 3; i < h - 2; i++) {
        const uint8_t *ptr = img + (size_t)i * stride + 3;
        uint8_t *curr = buf[(i - 3) % 3];
        int *cornerpos = cpbuf[(i - 3) % 3];
        int ncorners = 0;
        memset(curr, 0, (size_t)w);
        if (i < h - 3) {
            for (int j = 3; j < w - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t *t = tab - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                int corner = 0;
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                corner = 1;
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (!corner && (d & 2)) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                corner = 1;
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (corner) {
                    cornerpos[ncorners++] = j;
                    if (nonmax) curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t *prev = buf[(i - 4 + 3) % 3];
        const uint8_t *pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (!nonmax || (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                            score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                            score > curr[j] && score > curr[j + 1])) {
                if (n < cap) {
                    kx[n] = j;
                    ky[n] = i - 1;
                    kr[n] = nonmax ? score : 0;
                }
                n++;
            }
        }
    }
    free(bufmem);
    free(cpmem);
    return n;
}

/* detectors.cpp GridAdaptedFeatureDetector::detectImpl with the FAST detector
 * and a mask that is 255 exactly on the rect (rx, ry, rw, rh) (the reference's
 * m_matMaskForFeature(rectROI) = 255). Keypoints in cell order, each cell's
 * in detection order after keepStrongest (ties: earlier wins). Returns the
 * keypoint count; out_xy / out_resp receive up to `cap` entries. */
int oracle_gridfast(const uint8_t *img, int w, int h, int stride, int rx, int ry, int rw, int rh, int threshold,
                    int nonmax, int max_total, int grid_rows, int grid_cols, float *out_xy, int *out_resp, int cap) {
    if (w <= 0 || h <= 0 || grid_rows <= 0 || grid_cols <= 0 || max_total < grid_rows * grid_cols) return 0;
    const int per_cell = max_total / (grid_rows * grid_cols);
    const int scap = w * h;
    int *kx = (int *)malloc(sizeof(int) * (size_t)scap), *ky = (int *)malloc(sizeof(int) * (size_t)scap);
    int *kr = (int *)malloc(sizeof(int) * (size_t)scap);
    int *keep = (int *)malloc(sizeof(int) * (size_t)scap);
    int n = 0;
    for (int i = 0; i < grid_rows; i++) {
        const int r0 = (i * h) / grid_rows, r1 = ((i + 1) * h) / grid_rows;
        for (int j = 0; j < grid_cols; j++) {
            const int c0 = (j * w) / grid_cols, c1 = ((j + 1) * w) / grid_cols;
            int m = oracle_fast16(img + (size_t)r0 * stride + c0, c1 - c0, r1 - r0, stride, threshold, nonmax, kx,
                                  ky, kr, scap);
            /* KeyPointsFilter::runByPixelsMask on the cell's sub-mask */
            int k2 = 0;
            for (int k = 0; k < m; k++) {
                const int gx = kx[k] + c0, gy = ky[k] + r0;
                if (gx >= rx && gx < rx + rw && gy >= ry && gy < ry + rh) {
                    kx[k2] = gx;
                    ky[k2] = gy;
                    kr[k2] = kr[k];
                    k2++;
                }
            }
            m = k2;
            /* keepStrongest(per_cell): the per_cell largest |response|, ties to
             * the earlier keypoint; survivors keep detection order */
            for (int k = 0; k < m; k++) keep[k] = 1;
            if (m > per_cell) {
                for (int k = 0; k < m; k++) {
                    int rank = 0;  /* keypoints ranked before k */
                    for (int q = 0; q < m; q++)
                        if (abs(kr[q]) > abs(kr[k]) || (abs(kr[q]) == abs(kr[k]) && q < k)) rank++;
                    keep[k] = rank < per_cell;
                }
            }
            for (int k = 0; k < m; k++) {
                if (!keep[k]) continue;
                if (n < cap) {
                    out_xy[2 * n] = (float)kx[k];
                    out_xy[2 * n + 1] = (float)ky[k];
                    if (out_resp) out_resp[n] = kr[k];
                }
                n++;
            }
        }
    }
    free(kx);
    free(ky);
    free(kr);
    free(keep);
    return n;
}

/* The seeded shuffle key of candidate k of roi `roi` (lowbias32 mixing). */
static uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
uint32_t oracle_gridfast_key(uint32_t seed, uint32_t roi, uint32_t k) {
    return mix32(mix32(seed + 0x9e3779b9u * (roi + 1u)) ^ k);
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* random_shuffle + cap (PSNWhere_Tracker2D.cpp:752-757) with the seeded
 * definition above: the first min(n, cap) candidates in key order. */
int oracle_gridfast_select(const float *cand_xy, int n, uint32_t seed, int roi, int cap, float *out_xy) {
    uint64_t *key = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
    for (int k = 0; k < n; k++) key[k] = ((uint64_t)oracle_gridfast_key(seed, (uint32_t)roi, (uint32_t)k) << 32) | (uint32_t)k;
    qsort(key, (size_t)n, sizeof(uint64_t), cmp_u64);
    const int m = n < cap ? n : cap;
    for (int i = 0; i < m; i++) {
        const int k = (int)(key[i] & 0xffffffffu);
        out_xy[2 * i] = cand_xy[2 * k];
        out_xy[2 * i + 1] = cand_xy[2 * k + 1];
    }
    free(key);
    return m;
}
