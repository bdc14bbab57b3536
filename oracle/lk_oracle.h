/*
 * oracle/lk_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the OpenCV 2.4.6 pyramidal Lucas-Kanade path that
 * CPSNWhere_Tracker2D calls (psn_where/PSNWhere_Tracker2D.cpp:776-782 backward,
 * :871-877 forward). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * PARITY UNPINNED: the arithmetic lives in OpenCV 2.4.6 (pinned by
 * $(OPENCV_246) and the *246.lib names, psn_where/PSN_Where.vcxproj:97,104,
 * 124-125,151,175-176), which is not vendored in the reference and is absent
 * from this image; the reference ships no tests, fixtures or golden vectors.
 * The restatement follows OpenCV 2.4.6's published algorithm
 * (modules/video/src/lkpyramid.cpp, modules/imgproc/src/pyramids.cpp,
 * color.cpp) and is pinned by self-made known-answer tests (tests/).
 */
#ifndef PSN_LK_ORACLE_H
#define PSN_LK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Accumulation order of the float normal-equation sums.
 * 0 = the SSE2 build of OpenCV 2.4.6 (x64/x86 prebuilt libs the reference
 *     links): 4-lane partial sums for A, 8-pixel/2x4-lane for b, scalar tail.
 * 1 = the scalar (no-SIMD) build: one sequential float chain per sum. */
#define ORACLE_ACCUM_SSE2 0
#define ORACLE_ACCUM_SCALAR 1
/* analysis only (no reference counterpart): A / b / err window sums as exact
 * int64 integers, each converted to float once -- the order-free sums SURVEY
 * Appendix A names "int64_exact"; its distance from the SSE2 order is measured
 * in tests/test_oracle.py::test_exact_sums_vs_sse2_order */
#define ORACLE_ACCUM_EXACT 2

/* cv::OPTFLOW_* flag values (OpenCV 2.4.6 video/tracking.hpp) */
#define ORACLE_USE_INITIAL_FLOW 4
#define ORACLE_GET_MIN_EIGENVALS 8

int oracle_refl101(int p, int len);

/* cv::cvtColor(CV_BGR2GRAY) for CV_8UC3 (PSNWhere_Tracker2D.cpp:257). */
void oracle_bgr2gray(const uint8_t *src, int w, int h, int sstride, uint8_t *dst, int dstride);

/* cv::pyrDown, BORDER_REFLECT_101, dst size ((w+1)/2, (h+1)/2). */
void oracle_pyr_down(const uint8_t *src, int sw, int sh, int sstride, uint8_t *dst, int dstride);

/* calcSharrDeriv: interleaved int16 (Ix, Iy), reflect-101 inside the image. */
void oracle_scharr(const uint8_t *src, int w, int h, int sstride, int16_t *dst, int dstride_elems);

/* Level truncation of buildOpticalFlowPyramid: effective maxLevel. */
int oracle_effective_max_level(int w, int h, int win_w, int win_h, int max_level);

/* Pyramid of `nlevels` u8 planes packed contiguously (level l at offset
 * oracle_level_offset(w,h,l), pitch = level width). */
long oracle_level_offset(int w, int h, int level);
void oracle_level_size(int w, int h, int level, int *lw, int *lh);
void oracle_build_pyramid(const uint8_t *img, int w, int h, int stride, int nlevels, uint8_t *pyr);

/* LK over prebuilt pyramids (packed as above); derivatives are computed per
 * level inside, as calcOpticalFlowPyrLK does. `max_level` must already be the
 * effective (truncated) level; both pyramids must hold >= max_level+1 levels.
 * Returns 0, or -2 when winSize <= 2 (CV_Assert). */
int oracle_lk_track_pyr(const uint8_t *prev_pyr, const uint8_t *next_pyr, int w, int h,
                        const float *prev_pts, float *next_pts, uint8_t *status, float *err,
                        int npts, int win_w, int win_h, int max_level, int term_type,
                        int max_count, double epsilon, int flags, double min_eig_threshold,
                        int accum_mode, int nthreads);

/* One-shot cv::calcOpticalFlowPyrLK(prev, next, ...) with the reference call
 * schedule: both pyramids (and the Scharr planes) rebuilt inside the call. */
int oracle_calc_optical_flow_pyr_lk(const uint8_t *prev_img, const uint8_t *next_img, int w, int h,
                                    int stride, const float *prev_pts, float *next_pts,
                                    uint8_t *status, float *err, int npts, int win_w, int win_h,
                                    int max_level, int term_type, int max_count, double epsilon,
                                    int flags, double min_eig_threshold, int accum_mode,
                                    int nthreads);

/* Analysis hook: when set, counts LK iterations per point and level into
 * buf[i*8 + level] (caller zeroes it). Single-threaded use only. */
void oracle_set_iter_log(int *buf);
void oracle_set_bsum_log(long long *buf);
/* Analysis hook: every b-sum evaluation is cut into lk_kernel_bx's chains
 * (units of 4 px, `upt` units per thread, 256 threads) and evaluated with the
 * binade-run model (chain_model.c); buf[0..15] collects statistics (see
 * chain_classify in lk_oracle.c) and buf[16..24] the per-thread parity-record
 * model, so buf holds at least ORACLE_CHAIN_LOG_ENTRIES entries. upt = 0 picks
 * the kernel's UPT. */
#define ORACLE_CHAIN_LOG_ENTRIES 25
void oracle_set_chain_log(long long *buf, int upt);

/* ---- Binade-run model of an ordered float chain (oracle/chain_model.c) ---- */
float oracle_chain_serial(const float *f, int n);
float oracle_chain_binade(const float *f, int n, const int *seg_off, int nseg, int wave, int *stats);
/* Per-thread parity records with local HARD segments (lk_kernel_lg fallback): the
 * chain from segment fs on, from the exact value base; NAN = aborted. */
float oracle_chain_runs(const float *f, const int *seg_off, int nseg, int fs, int base, int *stats);

/* ---- GridFAST feature extraction (oracle/gridfast_oracle.c) ----
 * FeatureDetector::create("GridFAST")->detect(gray, kps, mask(rect) = 255)
 * and the shuffle + cap of PSNWhere_Tracker2D.cpp:734-757 (definitions of the
 * reference's unspecified tie order and unseeded shuffle: gridfast_oracle.c). */
int oracle_fast16(const uint8_t *img, int w, int h, int stride, int threshold, int nonmax, int *kx, int *ky,
                  int *kr, int cap);
int oracle_gridfast(const uint8_t *img, int w, int h, int stride, int rx, int ry, int rw, int rh, int threshold,
                    int nonmax, int max_total, int grid_rows, int grid_cols, float *out_xy, int *out_resp, int cap);
uint32_t oracle_gridfast_key(uint32_t seed, uint32_t roi, uint32_t k);
int oracle_gridfast_select(const float *cand_xy, int n, uint32_t seed, int roi, int cap, float *out_xy);

/* ---- JPEG decode (oracle/jpeg_oracle.c): cv::imread's libjpeg baseline path ---- */
int oracle_jpeg_info(const uint8_t *data, size_t n, int *w, int *h, int *ncomp);
int oracle_jpeg_decode_bgr(const uint8_t *data, size_t n, uint8_t *out_bgr, int out_stride);

#ifdef __cplusplus
}
#endif
#endif
