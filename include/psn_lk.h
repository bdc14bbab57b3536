/*
 * include/psn_lk.h -- C ABI of the MI355X-native Tracker2D optical-flow path.
 *
 * Replaces, for CPSNWhere_Tracker2D (psn_where/PSNWhere_Tracker2D.{h,cpp}),
 * the two OpenCV 2.4.6 calls
 *   cv::calcOpticalFlowPyrLK(curr, prev, ...)  backward, PSNWhere_Tracker2D.cpp:776-782
 *   cv::calcOpticalFlowPyrLK(prev, curr, ...)  forward,  PSNWhere_Tracker2D.cpp:871-877
 * and the per-frame gray ring buffer they read
 *   cvtColor(BGR2GRAY) + resize(scale 1.0) into m_vecPtGrayFrameBuffer,
 *   PSNWhere_Tracker2D.cpp:256-263 (ingest), :310-316 (rotation), .h:187.
 *
 * Plain C: pointers and sizes only, no C++/torch types. Every entry point
 * returns 0 (PSN_LK_OK) or a negative PSN_LK_ERR_*; no exception or abort
 * crosses the boundary (the reference's failure modes were assert() at
 * PSNWhere_Tracker2D.cpp:253 and OpenCV's CV_Assert(winSize > 2)).
 *
 * Threading: a context is single-threaded and owns one HIP stream; distinct
 * contexts (one per camera) may be driven concurrently, on one or several
 * devices. Device memory is owned by the context; host arrays are only
 * accessed during the call (host-array entry points are synchronous).
 */
#ifndef PSN_LK_H
#define PSN_LK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSN_LK_ABI_VERSION 5

#define PSN_LK_OK 0
#define PSN_LK_ERR_ARG (-1)
#define PSN_LK_ERR_WINSIZE (-2)     /* CV_Assert(winSize.width > 2 && winSize.height > 2) */
#define PSN_LK_ERR_HIP (-3)         /* HIP runtime failure; see psn_lk_last_error */
#define PSN_LK_ERR_NOMEM (-4)
#define PSN_LK_ERR_SLOT (-5)        /* ring slot out of range or never filled */
#define PSN_LK_ERR_LEVEL_CAP (-6)   /* query needs more pyramid levels than the ring holds */
#define PSN_LK_ERR_COMM (-7)        /* RCCL failure */
#define PSN_LK_ERR_UNSUPPORTED (-8) /* window wider than PSN_LK_MAX_WIN_WIDTH or of 2^24+ px (or a feature this build lacks) */

/* flags: OpenCV 2.4.6 values (video/tracking.hpp) + one accumulation-order bit */
#define PSN_LK_USE_INITIAL_FLOW 4      /* cv::OPTFLOW_USE_INITIAL_FLOW */
#define PSN_LK_GET_MIN_EIGENVALS 8     /* cv::OPTFLOW_LK_GET_MIN_EIGENVALS */
#define PSN_LK_ACCUM_SCALAR 0x100      /* float sums in the scalar build's order (default: SSE2 build) */

/* cv::TermCriteria type bits */
#define PSN_LK_TERM_COUNT 1
#define PSN_LK_TERM_EPS 2

#define PSN_LK_MAX_LEVELS 8
/* Window limits: widths up to PSN_LK_MAX_WIN_WIDTH (one window row band of the
 * large-window kernel in LDS) and h * ceil(w/4) < 2^22 quads (about 2^24 px);
 * psn_lk_window_supported() is the window predicate psn_lk_track checks after
 * winSize > 2 (else PSN_LK_ERR_UNSUPPORTED); the only other UNSUPPORTED exit, the
 * large-window planner's 160-KB LDS guard, is unreachable for a supported window.
 * Tracker2D passes box.w x box.h (PSNWhere_Tracker2D.cpp:871-877) and box.w x
 * box.w (:776-782) uncapped: a forward window of a box inside a frame of < 2^24 px
 * is always supported, but a backward box.w x box.w window is not when box.w >
 * 4096 (4097^2 > 2^24): the Tracker2D host checks the same predicate up front and
 * flags such a box; the frame then fails (PSN_LK_ERR_UNSUPPORTED, before any
 * launch) only when that box's backward chain would actually run, i.e. it holds
 * at least the chain's minimum of 4 features. */
#define PSN_LK_MAX_WIN_WIDTH 6400
#define PSN_LK_MAX_WIN_QUADS (1L << 22)

/* Arguments of cv::calcOpticalFlowPyrLK after prevImg/nextImg/points. The
 * reference passes only winSize and leaves the rest at their defaults
 * (PSNWhere_Tracker2D.cpp:782, :877); psn_lk_default_params() fills them. */
typedef struct psn_lk_params {
    int win_w, win_h;           /* winSize (default 21x21) */
    int max_level;              /* maxLevel (default 3), truncated per buildOpticalFlowPyramid */
    int term_type;              /* COUNT|EPS */
    int max_count;              /* default 30, clamped to [0,100] */
    double epsilon;             /* default 0.01, clamped to [0,10], squared */
    int flags;                  /* PSN_LK_* flags above (default 0) */
    double min_eig_threshold;   /* default 1e-4 */
} psn_lk_params;

/* One calcOpticalFlowPyrLK call on two ring slots over a contiguous range of
 * the point arrays: points [first_pt, first_pt + num_pts). Several queries
 * (e.g. one per detection box, each with its own window) run in ONE launch. */
typedef struct psn_lk_query {
    int prev_slot;              /* prevImg: pyramid of this ring slot */
    int next_slot;              /* nextImg */
    int first_pt;
    int num_pts;
    psn_lk_params params;
} psn_lk_query;

typedef struct psn_lk_ctx psn_lk_ctx;

/* cv::calcOpticalFlowPyrLK defaults. */
void psn_lk_default_params(psn_lk_params *p);

/* Effective maxLevel of buildOpticalFlowPyramid for an image/window (the
 * level-count truncation rule). Returns < 0 on bad arguments. */
int psn_lk_effective_max_level(int width, int height, int win_w, int win_h, int max_level);

/* 1 when an LK window of w x h px is within the window limits above
 * (w <= PSN_LK_MAX_WIN_WIDTH and h * ceil(w/4) < PSN_LK_MAX_WIN_QUADS), else 0:
 * the predicate psn_lk_track applies after winSize > 2, and the one the
 * Tracker2D host applies to each chain's box.w x box.w and each forward box. */
int psn_lk_window_supported(int w, int h);

/* Per-camera context (replaces CPSNWhere_Tracker2D::Initialize's ring setup,
 * PSNWhere_Tracker2D.cpp:129-139): a device ring of `ring_slots` pyramids of
 * max_level_cap+1 levels for width x height gray frames. */
int psn_lk_create(int device, int width, int height, int ring_slots, int max_level_cap, psn_lk_ctx **out);
void psn_lk_destroy(psn_lk_ctx *ctx);
const char *psn_lk_last_error(psn_lk_ctx *ctx);

/* Use an external HIP stream (hipStream_t as void*); NULL restores the
 * context's own stream. */
int psn_lk_set_stream(psn_lk_ctx *ctx, void *hip_stream);
void *psn_lk_get_stream(psn_lk_ctx *ctx);
int psn_lk_sync(psn_lk_ctx *ctx);

/* Ingest one frame into ring slot `slot` and build its pyramid on device
 * (replaces cvtColor(BGR2GRAY) + resize + the per-call pyramid rebuilds,
 * PSNWhere_Tracker2D.cpp:257-262). channels: 1 (gray) or 3 (BGR).
 * _device: `dev` is a device pointer; the call is asynchronous on the
 * context stream. Host variant copies and returns after enqueueing. */
int psn_lk_push_frame(psn_lk_ctx *ctx, int slot, const uint8_t *host, int stride, int channels);
int psn_lk_push_frame_device(psn_lk_ctx *ctx, int slot, const uint8_t *dev, int stride, int channels);

/* Asynchronous host-frame ingest: the frame is copied (hipMemcpy2DAsync, a copy
 * engine when `host` is pinned) into a staging buffer owned by `slot` and the
 * pyramid is built from it, both on the context's ingest stream, after every
 * LK / GridFAST launch that read the slot's previous frame; LK launches that
 * read the slot wait for the build (slot events, as in STREAM overlap mode,
 * whatever mode the context is in). Returns once enqueued: `host` must stay
 * valid and unchanged until psn_lk_sync, or until a later call that reads the
 * slot has completed. Used to overlap frame t+1's upload with frame t's LK. */
int psn_lk_push_frame_async(psn_lk_ctx *ctx, int slot, const uint8_t *host, int stride, int channels);

/* The same from a compressed frame: a baseline JPEG (include/psn_jpeg.h) of
 * the context's size is decoded on the device (cv::imread, main.cpp:144) into
 * the slot's staging buffer and its pyramid built from the BGR result, all on
 * the ingest stream; `jpeg` is copied before the call returns. */
int psn_lk_push_frame_jpeg(psn_lk_ctx *ctx, int slot, const uint8_t *jpeg, size_t len);

/* Ingest overlap modes (default OFF: builds run on the context stream).
 * STREAM: psn_lk_push_frame* builds the pyramid on the context's internal
 *   ingest stream, ordered only against earlier LK launches that read the same
 *   slot; LK launches wait for the builds of the slots they read. A device
 *   source frame must already be complete when psn_lk_push_frame_device is
 *   called (it is not ordered after the context stream).
 * FUSED: psn_lk_push_frame_device defers the build; the next psn_lk_track*
 *   launch that does not read that slot runs it in its own tail (workgroups
 *   whose point has converged pull pyramid tiles), so frame t+1's ingest costs
 *   no extra launch and no cross-stream wait. Any other call (a track reading
 *   the slot, another push, read_level, sync, set_stream, destroy) runs a
 *   pending build first as its own launch. The device source frame must stay
 *   valid until then. Host-frame pushes are never deferred.
 * Results are identical in every mode. */
#define PSN_LK_OVERLAP_OFF 0
#define PSN_LK_OVERLAP_STREAM 1
#define PSN_LK_OVERLAP_FUSED 2
int psn_lk_set_ingest_overlap(psn_lk_ctx *ctx, int mode);

/* Batched LK (replaces cv::calcOpticalFlowPyrLK at PSNWhere_Tracker2D.cpp:776-782
 * and :871-877). next_xy is written for EVERY point, including status==0 ones,
 * as OpenCV does (the backward path feeds all of them to LocalSearchKLT,
 * :787). err may be NULL. With PSN_LK_USE_INITIAL_FLOW, next_xy is read first.
 * Host variant: synchronous. _device variant: device pointers, async. */
int psn_lk_track(psn_lk_ctx *ctx, const psn_lk_query *q, int nq, const float *prev_xy, float *next_xy,
                 uint8_t *status, float *err);
int psn_lk_track_device(psn_lk_ctx *ctx, const psn_lk_query *q, int nq, const float *d_prev_xy,
                        float *d_next_xy, uint8_t *d_status, float *d_err);

/* The same with per-query point counts that live on the device (e.g. written
 * by a previous kernel on the context stream): query i processes points
 * [first_pt, first_pt + d_counts[i]) with d_counts[i] <= num_pts (num_pts =
 * the capacity the launch is sized for); outputs past the count are not
 * written. Used by the device-side backward chain (psn_t2d_*). */
int psn_lk_track_device_counted(psn_lk_ctx *ctx, const psn_lk_query *q, int nq, const int *d_counts,
                                const float *d_prev_xy, float *d_next_xy, uint8_t *d_status, float *d_err);
/* The same with query i's count at d_counts[i * count_stride] (e.g. one
 * counter of a per-detection record array). */
int psn_lk_track_device_counted_strided(psn_lk_ctx *ctx, const psn_lk_query *q, int nq, const int *d_counts,
                                        int count_stride, const float *d_prev_xy, float *d_next_xy, uint8_t *d_status,
                                        float *d_err);

/* One-shot cv::calcOpticalFlowPyrLK(prevImg, nextImg, prevPts, nextPts, status,
 * err, winSize, maxLevel, criteria, flags, minEigThreshold) on two host gray
 * images of the context's size, using two scratch slots of the context. */
int psn_calc_optical_flow_pyr_lk(psn_lk_ctx *ctx, const uint8_t *prev_img, const uint8_t *next_img,
                                 int stride, const float *prev_pts, float *next_pts, uint8_t *status,
                                 float *err, int npts, const psn_lk_params *params);

/* Copy pyramid level `level` of `slot` back to host (parity / debugging). */
int psn_lk_read_level(psn_lk_ctx *ctx, int slot, int level, uint8_t *host, int stride);
int psn_lk_level_size(psn_lk_ctx *ctx, int level, int *w, int *h);

/* Device-side kernel timing with HIP events recorded on the context stream
 * around every `every`-th psn_lk_push_frame* build launch (pyramid kernel)
 * and psn_lk_track* call (LK launch, including a fused build). `capacity` =
 * timed calls of each kind kept in an event ring (0 disables); every >= 1
 * (each event pair costs a few microseconds of GPU time, so sampling keeps
 * the measurement from slowing the measured loop). psn_lk_timing_stats waits
 * for the recorded events, returns the number of timed calls and their summed
 * milliseconds, and resets. */
int psn_lk_enable_timing(psn_lk_ctx *ctx, int capacity, int every);
int psn_lk_timing_stats(psn_lk_ctx *ctx, int *n_push, double *push_ms, int *n_track, double *track_ms);
/* Per timed track call since psn_lk_enable_timing (before psn_lk_timing_stats,
 * which resets the counts): its duration in ms (HIP events on the stream it
 * was launched on) and the kernel it ran: tag = 10 * UPT + (no-tail build) for
 * lk_kernel_bx<UPT, no-tail>, 1 = lk_kernel_st, 2 = lk_kernel (row-tiled),
 * 3 = lk_kernel_lg (large windows); a call whose queries went to several
 * launches (one per window class) gets 1000 + the tag of the launch with the
 * most window pixels. *n = the calls written (<= cap). */
int psn_lk_timing_launches(psn_lk_ctx *ctx, int cap, double *ms, int *tag, int *n);

/* Kernel-variant selection for tests and experiments (never read from the
 * environment: a product context always runs the planner's choice). Applies
 * to launches planned after the call. Results are identical in every variant.
 *   PSN_LK_VARIANT_THREADS     0 = planner; 64/128/256 tiled-kernel workgroup,
 *                              64..512 single-tile workgroup size
 *   PSN_LK_VARIANT_GENERIC     1 = always the row-tiled kernel
 *   PSN_LK_VARIANT_ONEWAVE     0 = multi-wave iterations in the single-tile kernel
 *   PSN_LK_VARIANT_BOX         0 = box windows run the row-tiled kernel, not lk_kernel_bx
 *   PSN_LK_VARIANT_TILED_LDS   LDS budget (bytes) of a row-tiled workgroup
 *   PSN_LK_VARIANT_FUSED_HELPERS  tile-only workgroups per fused-ingest launch
 *   PSN_LK_VARIANT_LARGE       1 = every query runs the large-window kernel (lk_kernel_lg)
 *   PSN_LK_VARIANT_LG_LDS      LDS budget (bytes) of a large-window workgroup (its row bands)
 *   PSN_LK_VARIANT_LG_JR       0 = the large-window kernel reads J from the level, never
 *                              from an LDS copy of the window's J region
 *   PSN_LK_VARIANT_ST_OVL      0 = the single-tile kernel computes every level's A phase
 *                              in its prologue (1: waves 1-3 compute the finer levels'
 *                              beside wave 0's iterations when the layout fits)
 *   PSN_LK_VARIANT_POISON_LDS  1 = LK launches (single-tile, box, large) fill their LDS
 *                              with pseudo-random words first (tests: a read of unwritten
 *                              LDS shows up)
 * Queries are split into one launch per window class (single-tile / box kernel
 * per units-per-thread and tail build / row-tiled / large), each sized for its
 * own windows. */
#define PSN_LK_VARIANT_THREADS 1
#define PSN_LK_VARIANT_GENERIC 2
#define PSN_LK_VARIANT_ONEWAVE 3
#define PSN_LK_VARIANT_BOX 4
#define PSN_LK_VARIANT_TILED_LDS 5
#define PSN_LK_VARIANT_FUSED_HELPERS 6
#define PSN_LK_VARIANT_LARGE 7
#define PSN_LK_VARIANT_LG_LDS 8
#define PSN_LK_VARIANT_LG_JR 9
#define PSN_LK_VARIANT_ST_OVL 10
#define PSN_LK_VARIANT_POISON_LDS 11
int psn_lk_debug_set_variant(psn_lk_ctx *ctx, int key, int value);

/* Window-sample counter (SURVEY 8(d)'s compute figure): while on, every box-
 * window LK launch (lk_kernel_bx, lk_kernel_lg) adds, per point, sum over levels of
 * w * h * (1 + iterations) to a device counter. _count_samples(ctx, 1) zeroes
 * and enables it (device-wide sync), 0 disables; _read_samples syncs the
 * device and returns the count. Test / benchmark instrumentation. */
int psn_lk_debug_count_samples(psn_lk_ctx *ctx, int on);
int psn_lk_debug_read_samples(psn_lk_ctx *ctx, unsigned long long *out);

/* Diagnostic builds only (libpsn_lk_stamps.so, -DPSN_LK_STAMPS): record
 * shader-clock stamps of every LK workgroup's phases into a device buffer of
 * 64 u64 per workgroup. Returns PSN_LK_ERR_UNSUPPORTED in product builds. */
int psn_lk_debug_set_stamps(psn_lk_ctx *ctx, void *d_stamps);

/* ---- GridFAST feature extraction on a ring slot's frame ----
 * Replaces, per detection of the backward chain (PSNWhere_Tracker2D.cpp:734-757):
 *   m_matMaskForFeature(rectROI) = 255;
 *   m_detector->detect(gray, newKeypoints, m_matMaskForFeature);   // "GridFAST", :142
 *   std::random_shuffle(newKeypoints); currFeatures = first min(n, 100) points
 * FeatureDetector::create("GridFAST") in OpenCV 2.4.6 = GridAdaptedFeatureDetector
 * (FastFeatureDetector(threshold 10, nonmaxSuppression true), maxTotalKeypoints
 * 1000, 4 x 4 grid); psn_gridfast_default_params() fills those values and
 * cap = PSN_2D_FEATURE_MAX_NUM_TRACK (100).
 * rois: nroi x {x, y, w, h} ints = rectROI (box.cropWithSize(cols, rows).cv(),
 * :736), clipped to the image here; an empty roi yields no keypoints.
 * Outputs per roi i: out_total[i] = newKeypoints.size() (the caller's
 * "< PSN_2D_FEATURE_MIN_NUM_TRACK" test, :744; nullable), out_count[i] =
 * min(total, cap), out_xy[i * cap * 2 ...] the points.
 * Fixed choices where the reference is unspecified: keepStrongest ties at a
 * cell's cut keep the earlier keypoint in row-major order; random_shuffle is
 * replaced by ordering the candidates by a hash of (seed, roi index, candidate
 * index) -- a seeded uniform permutation; same seed, same points.
 * Limits: grid cells <= 256, max_total <= 4096, cell width <= 1030 px.
 * Host variant synchronous; _device variant async with device out pointers. */
typedef struct psn_gridfast_params {
    int threshold;  /* FAST threshold (default 10), clamped to [0, 255] */
    int nonmax;     /* nonmaxSuppression (default 1) */
    int max_total;  /* maxTotalKeypoints (default 1000); per cell = max_total / cells */
    int grid_rows;  /* default 4 */
    int grid_cols;  /* default 4 */
    int cap;        /* points kept after the shuffle (default 100) */
} psn_gridfast_params;
void psn_gridfast_default_params(psn_gridfast_params *p);
int psn_gridfast_detect(psn_lk_ctx *ctx, int slot, const int *rois, int nroi, const psn_gridfast_params *p,
                        uint32_t seed, float *out_xy, int *out_count, int *out_total);
int psn_gridfast_detect_device(psn_lk_ctx *ctx, int slot, const int *rois, int nroi, const psn_gridfast_params *p,
                               uint32_t seed, float *d_out_xy, int *d_out_count, int *d_out_total);
/* Several frames' detections at once (PSNWhere_Tracker2D.cpp:734-757 run per
 * camera): set i = nrois[i] rois on ring slot slots[i]; the sets' rois lie
 * consecutively in `rois` and their outputs consecutively in the out arrays.
 * Same results as nset psn_gridfast_detect_device calls at consecutive output
 * offsets (the shuffle key is the roi's index within its set), in as few
 * launches as kGfMaxRois (64) rois per launch allow. Async, device pointers. */
int psn_gridfast_detect_device_sets(psn_lk_ctx *ctx, int nset, const int *slots, const int *nrois, const int *rois,
                                    const psn_gridfast_params *p, uint32_t seed, float *d_out_xy, int *d_out_count,
                                    int *d_out_total);

/* ---- multi-GPU: per-camera tracklet slots all-gathered over RCCL/xGMI ----
 * Replaces the in-process std::vector<stTrack2DResult> hand-off into
 * CPSNWhere_Associator3D::Run (psn_where/PSNWhere.cpp:253, 264, 269). */
typedef struct psn_comm psn_comm;
#define PSN_COMM_UNIQUE_ID_BYTES 128
int psn_comm_get_unique_id(void *id_out /* PSN_COMM_UNIQUE_ID_BYTES */);
int psn_comm_init(int nranks, int rank, int device, const void *unique_id, psn_comm **out);
int psn_comm_allgather(psn_comm *comm, const void *d_send, void *d_recv, size_t bytes_per_rank, void *hip_stream);
void psn_comm_destroy(psn_comm *comm);

int psn_lk_abi_version(void);

/* ---- runtime binding (no reference counterpart: process plumbing) ----
 * libpsn_lk binds the ROCm runtime by soname (libamdhip64.so.7,
 * libhsa-runtime64.so.1, librccl.so.1 from its RUNPATH /opt/rocm/lib). When it
 * loads, it also gives those objects their unversioned names (and maps
 * libamd_comgr.so.3 from the same directory), so a library loaded later that
 * asks for "libamdhip64.so" (PyTorch-ROCm's do) binds to the same runtime
 * instead of mapping a second HIP/HSA runtime. Writes a JSON object into buf:
 * the file each runtime symbol resolves to, the HIP runtime / RCCL versions, a
 * bit mask of the unversioned names bound, and the HIP version built against. */
int psn_lk_runtime_info(char *buf, int len);

/* Wall time (ms) the first psn_lk_create on `device` spent setting up the
 * device's SDMA engines (one 4-KB copy per engine each way, so a later frame
 * upload never lands on an engine whose queue ROCr has yet to create);
 * PSN_LK_ERR_ARG when no context was created on the device yet. The warm-up is
 * skipped (about 0 ms) when the environment sets PSN_LK_SDMA_WARMUP=0, or when
 * no HSA agent matches the HIP device (several agents on its PCI function and
 * none with its UUID); psn_lk_create succeeds either way. */
int psn_lk_sdma_warmup_ms(int device, double *ms);

#ifdef __cplusplus
}
#endif
#endif /* PSN_LK_H */
