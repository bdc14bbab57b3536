/*
 * include/psn_t2d_device.h -- device-side step of the Tracker2D backward
 * chain (part of libpsn_lk.so; driven by libpsn_tracker2d.so).
 *
 * CPSNWhere_Tracker2D::Track2D_BackwardFeatureTracking (PSNWhere_Tracker2D.cpp:
 * 763-811) runs, per detection, up to 3 chained LK calls; after each one
 * LocalSearchKLT (:452-554) shifts the box by the mode of the flow vectors and
 * keeps the inliers, which feed the next LK call. Here that step runs on the
 * device for every detection at once, right after the (counted) LK launch of
 * the chain step, so the 3 steps of a frame need no host round trip:
 * psn_lk_track_device_counted reads the per-detection counts this kernel
 * writes. Arithmetic is the reference's (cv::Point2f differences in float,
 * PSN_Point2D / PSN_Rect in IEEE double, correctly rounded sqrt).
 */
#ifndef PSN_T2D_DEVICE_H
#define PSN_T2D_DEVICE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSN_T2D_CHAIN_CAP 100  /* PSN_2D_FEATURE_MAX_NUM_TRACK */
#define PSN_T2D_CHAIN_STEPS 4  /* PSN_2D_BACKTRACKING_INTERVAL: boxes / point sets per detection */

/* Device buffers of the chains of one frame (all device pointers):
 *   boxes    [ndet][4]       detection box (x, y, w, h) LocalSearchKLT searches around
 *   cur      [ndet][cap][2]  input points of this step (the LK prevPts)
 *   nxt      [ndet][cap][2]  the LK nextPts of this step (every point, status ignored: :787)
 *   cnt      [ndet]          in: points of this step (0 = chain stopped);
 *                            out: inliers kept, 0 when fewer than 4 (:788)
 *   next_in  [ndet][cap][2]  out: the inliers' nextPts = the next step's input
 *   out_boxes[ndet][steps][4] out: box pushed at step s in row s (row 0 = the host's detection box)
 *   sets     [ndet][steps][cap][2], set_cnt [ndet][steps]
 *                            out: vecvecTrackedFeatures; step 1 writes row 0 (inliers at t)
 *                            and row 1, step s row s
 *   nsteps   [ndet]          out: last step that kept >= 4 inliers
 *   last_step[ndet]          in, nullable: the chain's last step (the ring of the
 *                            detection's camera holds frames back to t - last_step);
 *                            at that step the count is cleared after the results */
typedef struct psn_t2d_chain_dev {
    int ndet, cap;
    const double *boxes;
    const float *cur, *nxt;
    int *cnt;
    float *next_in;
    double *out_boxes;
    float *sets;
    int *set_cnt;
    int *nsteps;
    const int *last_step;
} psn_t2d_chain_dev;

/* LocalSearchKLT + inlier compaction of chain step `step` (1..3) for every
 * detection, asynchronous on `hip_stream`. Returns 0 or a PSN_LK_ERR_* code. */
int psn_t2d_chain_step_device(const psn_t2d_chain_dev *c, int step, void *hip_stream);

/* d_cnt[i] = 0 where d_cnt[i] < min_count (the reference skips detections with
 * fewer than PSN_2D_FEATURE_MIN_NUM_TRACK features, :744) or where
 * d_last_step[i] < 1 (nullable: no frame t-1 in that camera's ring), asynchronous. */
int psn_t2d_gate_counts_device(int *d_cnt, int n, int min_count, const int *d_last_step, void *hip_stream);
/* The start of a frame's device chain (one launch): per detection k < c->ndet
 * the step / set counters cleared, set 0 = its features at t (c->cur, the
 * first min(cnt, cap) points) with set_cnt[k * STEPS] = that count when
 * cnt[k] >= min_count, then the gate of psn_t2d_gate_counts_device. Set 0 is
 * what the detection's tracker carries into the next frame's forward call:
 * its step-1 inliers, or these features when no step keeps 4 inliers. */
int psn_t2d_chain_begin_device(const psn_t2d_chain_dev *c, int min_count, void *hip_stream);

/* d_dst[0, bytes) = h_src[0, bytes) by a kernel that reads the pinned host block
 * (hipHostMalloc'd, coherent; both pointers 16-B aligned) over the bus, asynchronous on
 * `hip_stream`. The Tracker2D pass inputs (chain boxes / counts / points,
 * forward inputs: kilobytes) go up this way: a runtime copy of a small pinned
 * block can hold the calling thread until the engine's earlier work drains
 * (measured: 7-9 ms host stalls, the first copies after a device sync). */
int psn_t2d_upload_device(void *d_dst, const void *h_src, size_t bytes, void *hip_stream);
/* h_dst[0, bytes) = d_src[0, bytes): the kernel writes the pinned host block
 * (hipHostMalloc'd, coherent; both pointers 16-B aligned) over the bus,
 * asynchronous on `hip_stream` (the pass's result copies). */
int psn_t2d_download_device(void *h_dst, const void *d_src, size_t bytes, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* PSN_T2D_DEVICE_H */
