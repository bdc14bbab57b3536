/*
 * include/psn_tracker2d.h -- C ABI of the Tracker2D flow stage (host side).
 *
 * The per-frame 2D tracklet propagation of CPSNWhere_Tracker2D that sits
 * directly on the optical-flow path, built on libpsn_lk.so:
 *   - ingest + 4-slot ring rotation      PSNWhere_Tracker2D.cpp:256-263, :310-316
 *   - backward feature tracking chain    :690-838 (LK call :776-782)
 *   - forward tracking + matching score  :851-1025 (LK call :871-877)
 *   - LocalSearchKLT                      :452-554
 *   - BoxMatchingCost                     :600-613
 *   - PSN_Rect arithmetic                 PSNWhere_Types.h:112-182
 * The LK calls of one frame are batched into as few launches as the chain
 * dependencies allow (backward step 1 and the forward calls share a launch).
 *
 * After the flow: Track2D_MatchingAndUpdating (:1038-1164) -- the
 * assignment, the tracker update and life cycle -- and ResultWithTracker
 * (:1231-1257), which produce the stTrack2DResult handed to Associator3D.
 * psn_t2d_group_* runs the whole per-frame CPSNWhere_Tracker2D::Run of several
 * cameras (CPSNWhere::TrackPeople's camera loop, PSNWhere.cpp:257-266) with
 * every camera's LK work batched into the same launches.
 *
 * Out of this stage (the caller's, as in the reference): the detection height
 * gate and the 3D location/height estimate (camera calibration, :711-718; the
 * caller passes them in the detection records).
 *
 * Plain C, fixed-capacity records (the reference caps a detection at
 * PSN_2D_FEATURE_MAX_NUM_TRACK = 100 points, :13, and the chain at
 * PSN_2D_BACKTRACKING_INTERVAL = 4 frames, :16). Returns 0 or a negative
 * PSN_T2D_ERR_* / PSN_LK_ERR_* code.
 */
#ifndef PSN_TRACKER2D_H
#define PSN_TRACKER2D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSN_T2D_MAX_FEATURES 100 /* PSN_2D_FEATURE_MAX_NUM_TRACK */
#define PSN_T2D_MIN_FEATURES 4   /* PSN_2D_FEATURE_MIN_NUM_TRACK */
#define PSN_T2D_INTERVAL 4       /* PSN_2D_BACKTRACKING_INTERVAL (ring slots) */
#define PSN_T2D_MAX_BOXES 16     /* tracker box history kept in the C record */

#define PSN_T2D_ERR_CAPACITY (-20) /* a fixed-capacity record would overflow */
#define PSN_T2D_ABI_VERSION 2
int psn_t2d_abi_version(void);

/* PSN_Rect: double x, y, w, h (PSNWhere_Types.h:112) */
typedef struct psn_rect {
    double x, y, w, h;
} psn_rect;

/* PSN_Rect methods (PSNWhere_Types.h:131-182), for parity tests. */
int psn_rect_overlap(psn_rect a, psn_rect b);
double psn_rect_distance(psn_rect a, psn_rect b);
double psn_rect_overlapped_area(psn_rect a, psn_rect b);
int psn_rect_contain(psn_rect a, float px, float py);
void psn_rect_center(psn_rect a, double *cx, double *cy);

/* CPSNWhere_Tracker2D::BoxMatchingCost (PSNWhere_Tracker2D.cpp:600-613). */
double psn_t2d_box_matching_cost(psn_rect a, psn_rect b);

/* CPSNWhere_Tracker2D::LocalSearchKLT (PSNWhere_Tracker2D.cpp:455-554):
 * box shift = the mode of the flow vectors (pre -> cur); inlier_idx gets the
 * indices of the inlier points (capacity n), *n_inliers their count. */
int psn_t2d_local_search_klt(psn_rect pre_box, const float *pre_xy, const float *cur_xy, int n, psn_rect *out_box,
                             int *inlier_idx, int *n_inliers);

/* One camera's flow stage: owns a psn_lk context with a ring of 4 pyramids. */
typedef struct psn_t2d psn_t2d;
int psn_t2d_create(int device, unsigned cam_id, int width, int height, psn_t2d **out);
void psn_t2d_destroy(psn_t2d *t);
const char *psn_t2d_last_error(psn_t2d *t);
/* Where the backward chain's LocalSearchKLT steps run: 1 (default) on the
 * device -- every chain step's LK launch and LocalSearchKLT kernel enqueued
 * back to back, one host sync per frame -- or 0 on the host between launches.
 * Results are identical. */
int psn_t2d_set_device_chain(psn_t2d *t, int on);
/* ingest frame t into the ring's newest slot (cvtColor + resize, :256-263) */
int psn_t2d_push_frame(psn_t2d *t, const uint8_t *frame, int stride, int channels);
/* the same from a frame already in device memory (complete on the context's
 * stream order; psn_lk_push_frame_device semantics) */
int psn_t2d_push_frame_device(psn_t2d *t, const uint8_t *dev_frame, int stride, int channels);
/* the flow stage's LK context (a psn_lk_ctx * of include/psn_lk.h: stream,
 * kernel timing with psn_lk_enable_timing) */
void *psn_t2d_lk_context(psn_t2d *t);
/* end of Run: the oldest slot becomes the next frame's slot (:310-316) */
int psn_t2d_rotate(psn_t2d *t);

/* stDetectedObject of the backward chain (PSNWhere_Tracker2D.h:17-29). */
typedef struct psn_t2d_detection {
    psn_rect box;                                   /* in: detection box (height-validated) */
    psn_rect head;                                  /* in: stDetection::vecPartBoxes.front() (tracker heads) */
    double location[3];                             /* in: 3D foot location (EstimateDetectionHeight, :711-718) */
    double height;                                  /* in: 3D height, mm */
    int num_features;                               /* in: points at t after shuffle + cap */
    float features[PSN_T2D_MAX_FEATURES][2];        /* in */
    int valid;                                      /* out: >= 4 points (kept in m_vecDetection2D) */
    int overlap_other;                              /* out: bOverlapWithOtherDetection */
    int num_boxes;                                  /* out: boxes[0] = box, then back-propagated */
    psn_rect boxes[PSN_T2D_INTERVAL];
    int num_sets;                                   /* out: vecvecTrackedFeatures, current -> past */
    int set_count[PSN_T2D_INTERVAL];
    float sets[PSN_T2D_INTERVAL][PSN_T2D_MAX_FEATURES][2];
} psn_t2d_detection;

/* stTracker2D (.h:31-47): the fields the forward step and the update read and write. */
typedef struct psn_t2d_tracker {
    unsigned id;                                    /* m_nNewTrackerID at creation (:1119) */
    unsigned time_start, time_end, time_last_update;
    unsigned duration;                              /* in */
    int num_boxes;                                  /* in/out: box history, oldest first */
    psn_rect boxes[PSN_T2D_MAX_BOXES];
    psn_rect heads[PSN_T2D_MAX_BOXES];              /* in/out: one per box; the forward step repeats the last (:896) */
    double last_position[3];                        /* lastPosition (the matched detection's location) */
    double height;
    double confidence;
    int num_features;                               /* in/out: featurePoints */
    float features[PSN_T2D_MAX_FEATURES][2];
    int num_tracked;                                /* out: trackedPoints */
    float tracked[PSN_T2D_MAX_FEATURES][2];
    int updated;                                    /* out: >= 4 points tracked, box pushed */
} psn_t2d_tracker;

/* ---- stTrack2DResult: the Tracker2D -> Associator3D hand-off ----
 * stObject2DInfo (PSNWhere_Types.h:190-198) and stTrack2DResult (:200-209)
 * as plain C records with caller-owned arrays (cap_* = capacity, used by the
 * readers; matMatchingCost is not part of either format). */
typedef struct psn_object2d {
    unsigned id;
    psn_rect box, head;
    double score;
    int num_prev;                                   /* featurePointsPrev */
    float prev[PSN_T2D_MAX_FEATURES][2];
    int num_curr;                                   /* featurePointsCurr */
    float curr[PSN_T2D_MAX_FEATURES][2];
} psn_object2d;

typedef struct psn_track2d_result {
    unsigned cam_id, frame_idx;
    int num_objects, cap_objects;
    psn_object2d *objects;
    int num_detection_rects, cap_detection_rects;
    psn_rect *detection_rects;
    int num_tracker_rects, cap_tracker_rects;
    psn_rect *tracker_rects;
} psn_track2d_result;

/* Feature extraction of the backward chain (PSNWhere_Tracker2D.cpp:734-757) on
 * frame t (call after psn_t2d_push_frame): GridFAST (psn_gridfast_detect with
 * the "GridFAST" defaults) masked by each detection's rectROI =
 * box.cropWithSize(width, height).cv() (:736), shuffled by `seed` (the
 * reference's unseeded std::random_shuffle, :752) and capped at
 * PSN_T2D_MAX_FEATURES. Fills dets[i].features / num_features; a detection
 * with fewer than PSN_T2D_MIN_FEATURES points is skipped by the backward step
 * (:744). */
int psn_t2d_detect_features(psn_t2d *t, psn_t2d_detection *dets, int ndet, uint32_t seed);

/* Track2D_BackwardFeatureTracking for all detections (batched per chain step). */
int psn_t2d_backward(psn_t2d *t, psn_t2d_detection *dets, int ndet);
/* Track2D_ForwardTrackingAndGetMatchingScore: cost is [valid dets][ntrk]
 * row-major (matchingCostArray), +inf where not matched. */
int psn_t2d_forward(psn_t2d *t, psn_t2d_tracker *trk, int ntrk, const psn_t2d_detection *dets, int ndet,
                    float *cost);
/* Both, with backward step 1 and the forward calls in one LK launch; results
 * identical to psn_t2d_backward followed by psn_t2d_forward. */
int psn_t2d_track_frame(psn_t2d *t, psn_t2d_detection *dets, int ndet, psn_t2d_tracker *trk, int ntrk,
                        float *cost);
/* psn_t2d_detect_features + psn_t2d_track_frame in one device pass (device
 * chain mode; otherwise the two calls): the forward LK runs first, on its own
 * stream; GridFAST writes every detection's features straight into the
 * backward chains' inputs and detections below the feature minimum (:744) are
 * gated on the device; one host sync. dets[i].features / num_features are
 * written (the points GridFAST kept), as psn_t2d_detect_features does; the
 * rest as psn_t2d_track_frame. Identical results. */
int psn_t2d_track_frame_detect(psn_t2d *t, psn_t2d_detection *dets, int ndet, uint32_t seed, psn_t2d_tracker *trk,
                               int ntrk, float *cost);

/* ---- after the flow: matching, tracker update, result (:1038-1164, :1231-1257) ---- */

/* The assignment of Track2D_MatchingAndUpdating (:1040-1064 + CPSNWhere_Hungarian::Match):
 * cost = [rows x cols] row-major (the forward step's matchingCostArray);
 * non-finite entries become max(finite) + 100, the reference's Munkres
 * (psn_t2d_hungarian_match) matches the matrix, and pairs at that substitute
 * cost are dropped. match[r] = the column matched to row r, or -1. Ties break
 * as the reference's row-major Munkres breaks them. */
int psn_t2d_assign(const float *cost, int rows, int cols, int *match);

/* CPSNWhere_Hungarian Initialize(std::vector<float>, rows, cols) + Match()
 * (helpers/PSNWhere_Hungarian.cpp:67-89, :212-359) on [rows x cols] float
 * costs: non-finite entries become FLT_MAX - (sum of the finite ones), rows and
 * columns without a finite entry are condensed out, the square is padded to its
 * minimum line cover, Munkres steps 1-6 in float32 (row-major scans), and the
 * starred pairs of finite original cost are returned in row-major order:
 * out_rows/out_cols/out_costs (capacity min(rows, cols)), *n_out pairs
 * (stMatchInfo rows / cols / matchCosts). A NaN cost or an empty matrix gives
 * no pairs (the reference's Initialize leaves the matcher uninitialised). */
int psn_t2d_hungarian_match(const float *cost, int rows, int cols, int *out_rows, int *out_cols, float *out_costs,
                            int *n_out);

/* ResultWithTracker (:1231-1257): id, last box and head, score 0,
 * featurePointsPrev = features, featurePointsCurr = tracked. */
int psn_t2d_result_with_tracker(const psn_t2d_tracker *trk, psn_object2d *out);

/* Track2D_MatchingAndUpdating (:1038-1164) on caller-owned records: dets =
 * the backward step's records (the valid ones are m_vecDetection2D, in order),
 * trk = m_queueActiveTracker2D after psn_t2d_forward, cost = its [valid dets x
 * ntrk] matrix, match = per valid detection the tracker index or -1 (NULL:
 * psn_t2d_assign(cost)). Validation (3D distance <= 600 mm, height difference
 * <= 400 mm, duration <= 3) uses the records' location / height. out_trk
 * receives the new active queue (matched trackers in detection order, then
 * one new tracker per unmatched valid detection, ids from *next_id);
 * result->objects the packed objects in the same order (result capacity
 * cap_objects), result->frame_idx = frame_idx, no detection / tracker rects
 * (the reference never fills them). */
int psn_t2d_matching_and_updating(const psn_t2d_detection *dets, int ndet, const psn_t2d_tracker *trk, int ntrk,
                                  const float *cost, const int *match, unsigned frame_idx, unsigned *next_id,
                                  psn_t2d_tracker *out_trk, int cap_trk, int *n_out, psn_track2d_result *result);

/* CPSNWhere_Tracker2D::FilePrintResult (PSNWhere_Tracker2D.cpp:1268-1334):
 * writes <dir>/track2D_result_cam%d_frame%04d.txt in the reference's text
 * format ("%f" fields; dir must end with a separator, as RESULT_SAVE_PATH
 * "tracklets/" does). Returns 0 or PSN_LK_ERR_ARG (cannot open). */
int psn_t2d_write_result_txt(const char *dir, const psn_track2d_result *r);
/* psn::Read2DTrackResultWithTxt (PSNWhere_Utils.cpp:1148-1237): parses that
 * file (values pass through float, as the reference's fscanf "%f" does).
 * Returns 0, PSN_LK_ERR_ARG (cannot open / malformed) or PSN_T2D_ERR_CAPACITY. */
int psn_t2d_read_result_txt(const char *dir, unsigned cam_id, unsigned frame_idx, psn_track2d_result *r);

/* ---- CPSNWhere_Tracker2D::Run over several cameras, batched ----
 * One group = C cameras on one device (camera c = index c, cam_ids[c] its
 * camID). Per frame:
 *   psn_t2d_group_push_frame(g, c, frame t)    for every camera (async upload;
 *                                              up to 2 frames per camera may be
 *                                              staged, adopted in push order)
 *   psn_t2d_group_launch(g, t, dets, ...)      enqueue the frame's device work
 *   [psn_t2d_group_push_frame(g, c, frame t+1) may overlap it here]
 *   psn_t2d_group_complete(g, dets, results)   wait; matching, update, results
 * (psn_t2d_group_run = launch + complete). dets[c] / ndet[c]: camera c's
 * height-validated detections with head box and 3D estimate; with
 * PSN_T2D_FEATURES_GIVEN their features (after shuffle + cap), with
 * PSN_T2D_FEATURES_GRIDFAST the group runs GridFAST on the device and writes
 * them. The backward outputs are written into dets as psn_t2d_track_frame does;
 * results[c] receives camera c's stTrack2DResult (caller-owned arrays). The
 * dets arrays must stay valid from launch to complete; host frames until the
 * next complete (pinned memory makes the upload asynchronous). */
typedef struct psn_t2d_group psn_t2d_group;
#define PSN_T2D_FEATURES_GIVEN 0
#define PSN_T2D_FEATURES_GRIDFAST 1
int psn_t2d_group_create(int device, int ncams, const unsigned *cam_ids, int width, int height, psn_t2d_group **out);
void psn_t2d_group_destroy(psn_t2d_group *g);
const char *psn_t2d_group_last_error(psn_t2d_group *g);
void *psn_t2d_group_lk_context(psn_t2d_group *g);
int psn_t2d_group_push_frame(psn_t2d_group *g, int cam, const uint8_t *frame, int stride, int channels);
int psn_t2d_group_push_frame_device(psn_t2d_group *g, int cam, const uint8_t *dev_frame, int stride, int channels);
/* the camera's frame as a baseline JPEG file (decoded on the device, psn_lk_push_frame_jpeg) */
int psn_t2d_group_push_frame_jpeg(psn_t2d_group *g, int cam, const uint8_t *jpeg, size_t len);
int psn_t2d_group_launch(psn_t2d_group *g, unsigned frame_idx, psn_t2d_detection *const *dets, const int *ndet,
                         int feature_mode, uint32_t seed);
int psn_t2d_group_complete(psn_t2d_group *g, psn_t2d_detection *const *dets, const int *ndet,
                           psn_track2d_result *results);
int psn_t2d_group_run(psn_t2d_group *g, unsigned frame_idx, psn_t2d_detection *const *dets, const int *ndet,
                      int feature_mode, uint32_t seed, psn_track2d_result *results);
/* psn_t2d_group_complete of frame t that also launches frame t+1: as soon as
 * frame t's device work is done, frame t+1's features (next_dets, feature_mode,
 * seed) and backward chains are enqueued, and the GPU runs them while the host
 * matches frame t (the chains read only frame t+1's detections and the image
 * ring, never frame t's trackers); frame t+1's forward calls follow frame t's
 * tracker update. Results are those of complete(t) + launch(t+1). Frame t+1 of
 * every camera must be staged (push_frame) before this call; the next call must
 * be psn_t2d_group_launch(g, next_frame_idx, next_dets, next_ndet, feature_mode,
 * .), which then only confirms the frame, and next_dets must stay valid until
 * that frame's complete. A pipelined driver (frames uploaded two ahead: frame
 * t+2 moves while frame t runs):
 *   push(0); push(1); launch(0); push(2); complete_next(0 -> 1); launch(1); push(3); complete_next(1 -> 2); ...
 * If only the next frame cannot be launched (e.g. a detection whose window the
 * LK cannot run), this frame's results are still written to dets / results and
 * that error is returned; the next frame is not in flight, its images stay
 * staged, and a plain psn_t2d_group_launch of it (fixed detections) follows. */
int psn_t2d_group_complete_next(psn_t2d_group *g, psn_t2d_detection *const *dets, const int *ndet,
                                psn_track2d_result *results, unsigned next_frame_idx,
                                psn_t2d_detection *const *next_dets, const int *next_ndet, int feature_mode,
                                uint32_t seed);
/* diagnostic: host microseconds accumulated since the last call from the entry
 * of each complete to its phases (result copies + next chains enqueued, device
 * work done, unpacked, matched and updated, next forward calls enqueued), and
 * out6[5] = the number of completes */
int psn_t2d_group_debug_host_times(psn_t2d_group *g, double *out6);
/* diagnostic: host microseconds accumulated since the last call by the parts of
 * the completes' matching phase, over all cameras: overlap flags (:824-835),
 * forward matching costs + majority gate (:906-1022), assignment (:1038-1060),
 * tracker update + results (:1062-1164) */
int psn_t2d_group_debug_host_match_times(psn_t2d_group *g, double *out4);
/* camera c's active trackers (m_queueActiveTracker2D) after the last complete */
int psn_t2d_group_trackers(psn_t2d_group *g, int cam, psn_t2d_tracker *out, int cap, int *n);

/* Fixed-size binary slot of one camera's result for the per-frame RCCL
 * all-gather into Associator3D (psn_comm_allgather, psn_lk.h): exact (no
 * text rounding), little-endian, self-describing:
 *   u32 magic 'PT2R', u32 version 1, u32 cam_id, u32 frame_idx,
 *   u32 nobj, u32 ndet, u32 ntrk, u32 bytes_used,
 *   nobj x {u32 id, u32 num_prev, u32 num_curr, u32 pad, f64 box[4], f64 head[4],
 *           f64 score, f32 prev[num_prev][2], f32 curr[num_curr][2]} (8-B aligned),
 *   ndet x f64[4], ntrk x f64[4].
 * psn_t2d_result_slot_bytes(max objects, max rects) sizes a slot. */
size_t psn_t2d_result_slot_bytes(int max_objects, int max_rects);
int psn_t2d_pack_result(const psn_track2d_result *r, void *slot, size_t slot_bytes);
int psn_t2d_unpack_result(const void *slot, size_t slot_bytes, psn_track2d_result *r);

#ifdef __cplusplus
}
#endif

#endif /* PSN_TRACKER2D_H */
