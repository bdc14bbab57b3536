/*
 * include/psn_sgsmooth.h -- C ABI of the batched Savitzky-Golay trajectory
 * smoother on MI355X (part of libpsn_lk.so).
 *
 * Replaces, for many series at once, the reference's online smoother
 * CPSNWhere_SGSmooth (psn_where/PSNWhere_SGSmooth.{h,cpp}): span / degree as its
 * constructor (defaults SGS_DEFAULT_SPAN 9, SGS_DEFAULT_DEGREE 1,
 * PSNWhere_SGSmooth.h:14-15), one Insert(newData) (:33-37, :91-103) per
 * series per call, the smoothed values it refreshes returned. The reference
 * keeps one smoother per trajectory coordinate (PSNWhere_Types.h:350); here a
 * series has `dims` coordinates (2 for tracked image points, 3 for 3D
 * trajectories) smoothed independently with the reference's arithmetic (IEEE
 * double, the reference's summation orders; Qsets from its CalculateQ,
 * :133-224). Used as the post-filter of the tracked points' trajectories
 * (BASELINE configs[4]).
 *
 * Device state per series: the last `span` raw values of each coordinate, the
 * length and the current Q window -- enough to produce every value an Insert
 * changes (an Insert refreshes positions >= refreshPos >= length - span).
 * Returns 0 or a negative PSN_LK_ERR_* code (psn_lk.h).
 */
#ifndef PSN_SGSMOOTH_H
#define PSN_SGSMOOTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSN_SG_DEFAULT_SPAN 9
#define PSN_SG_DEFAULT_DEGREE 1
#define PSN_SG_MAX_SPAN 63

typedef struct psn_sg psn_sg;

/* nseries independent series of `dims` (1..4) coordinates; span 1..63, degree >= 0. */
int psn_sg_create(int device, int nseries, int dims, int span, int degree, psn_sg **out);
void psn_sg_destroy(psn_sg *sg);
/* Empty every series (a new CPSNWhere_SGSmooth per series). */
int psn_sg_reset(psn_sg *sg);
/* Use an external HIP stream (hipStream_t as void*); NULL = the smoother's own. */
int psn_sg_set_stream(psn_sg *sg, void *hip_stream);

/* Insert(newData) on every series whose active flag is set (d_active NULL =
 * all): in = nseries rows of `dims` floats, rows `in_stride` floats apart
 * (e.g. the LK next_xy array, stride 2). Per series i:
 *   refresh[i] = Insert's return value (the first smoothed position that
 *                changed), or -1 for an inactive series;
 *   out[(i * span + k) * dims + d] = smoothed value of coordinate d at
 *                position refresh[i] + k, k < length[i] - refresh[i] (<= span).
 * _device: device pointers, asynchronous on the smoother's stream. */
int psn_sg_insert_device(psn_sg *sg, const float *d_in, int in_stride, const uint8_t *d_active, int *d_refresh,
                         double *d_out);
int psn_sg_insert(psn_sg *sg, const float *in, int in_stride, const uint8_t *active, int *refresh, double *out);
/* Current length (inserted values) of every series (host array of nseries). */
int psn_sg_lengths(psn_sg *sg, int *lengths);

#ifdef __cplusplus
}
#endif
#endif /* PSN_SGSMOOTH_H */
