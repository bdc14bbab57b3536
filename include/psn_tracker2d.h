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
 * Out of this stage (the caller's, as in the reference): the detection height
 * gate (camera calibration, :711-715), GridFAST feature detection + shuffle
 * (:735-758; the caller passes each detection's points), the Hungarian
 * matching and tracker life cycle (:1038-1182).
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
/* ingest frame t into the ring's newest slot (cvtColor + resize, :256-263) */
int psn_t2d_push_frame(psn_t2d *t, const uint8_t *frame, int stride, int channels);
/* end of Run: the oldest slot becomes the next frame's slot (:310-316) */
int psn_t2d_rotate(psn_t2d *t);

/* stDetectedObject of the backward chain (PSNWhere_Tracker2D.h:17-29). */
typedef struct psn_t2d_detection {
    psn_rect box;                                   /* in: detection box (height-validated) */
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

/* stTracker2D fields the forward step reads and writes (.h:31-47). */
typedef struct psn_t2d_tracker {
    unsigned duration;                              /* in */
    int num_boxes;                                  /* in/out: box history, oldest first */
    psn_rect boxes[PSN_T2D_MAX_BOXES];
    int num_features;                               /* in/out: featurePoints */
    float features[PSN_T2D_MAX_FEATURES][2];
    int num_tracked;                                /* out: trackedPoints */
    float tracked[PSN_T2D_MAX_FEATURES][2];
    int updated;                                    /* out: >= 4 points tracked, box pushed */
} psn_t2d_tracker;

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

#ifdef __cplusplus
}
#endif

#endif /* PSN_TRACKER2D_H */
