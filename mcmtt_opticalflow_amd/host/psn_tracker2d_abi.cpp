// C ABI of include/psn_tracker2d.h over psn::Tracker2DFlow (tracker2d_flow.hpp).
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "psn_tracker2d.h"
#include "tracker2d_flow.hpp"

struct psn_t2d {
    psn::Tracker2DFlow flow;
    std::string err;
};

namespace {

psn::Rect to_rect(const psn_rect &r) { return psn::Rect(r.x, r.y, r.w, r.h); }
psn_rect from_rect(const psn::Rect &r) { return psn_rect{r.x, r.y, r.w, r.h}; }

std::vector<psn::Point2f> to_points(const float (*xy)[2], int n) {
    std::vector<psn::Point2f> v((size_t)n);
    for (int i = 0; i < n; i++) v[(size_t)i] = psn::Point2f{xy[i][0], xy[i][1]};
    return v;
}

int put_points(const std::vector<psn::Point2f> &v, float (*xy)[2], int *n) {
    if (v.size() > PSN_T2D_MAX_FEATURES) return PSN_T2D_ERR_CAPACITY;
    for (size_t i = 0; i < v.size(); i++) {
        xy[i][0] = v[i].x;
        xy[i][1] = v[i].y;
    }
    *n = (int)v.size();
    return 0;
}

int detections_in(const psn_t2d_detection *dets, int ndet, std::vector<psn::Detection> &d,
                  std::vector<std::vector<psn::Point2f>> &f) {
    d.resize((size_t)ndet);
    f.resize((size_t)ndet);
    for (int i = 0; i < ndet; i++) {
        if (dets[i].num_features < 0 || dets[i].num_features > PSN_T2D_MAX_FEATURES) return PSN_T2D_ERR_CAPACITY;
        d[(size_t)i].box = to_rect(dets[i].box);
        f[(size_t)i] = to_points(dets[i].features, dets[i].num_features);
    }
    return 0;
}

int detections_out(const std::vector<psn::DetectedObject> &objs, psn_t2d_detection *dets, int ndet) {
    for (int i = 0; i < ndet; i++) {
        dets[i].valid = 0;
        dets[i].overlap_other = 0;
        dets[i].num_boxes = 0;
        dets[i].num_sets = 0;
    }
    for (const psn::DetectedObject &o : objs) {
        psn_t2d_detection &r = dets[o.id];
        r.valid = 1;
        r.overlap_other = o.bOverlapWithOtherDetection ? 1 : 0;
        if (o.boxes.size() > PSN_T2D_INTERVAL || o.vecvecTrackedFeatures.size() > PSN_T2D_INTERVAL)
            return PSN_T2D_ERR_CAPACITY;
        r.num_boxes = (int)o.boxes.size();
        for (size_t b = 0; b < o.boxes.size(); b++) r.boxes[b] = from_rect(o.boxes[b]);
        r.num_sets = (int)o.vecvecTrackedFeatures.size();
        for (size_t s = 0; s < o.vecvecTrackedFeatures.size(); s++) {
            int rc = put_points(o.vecvecTrackedFeatures[s], r.sets[s], &r.set_count[s]);
            if (rc) return rc;
        }
    }
    return 0;
}

// m_vecDetection2D from the records the backward step marked valid
std::vector<psn::DetectedObject> valid_objects(const psn_t2d_detection *dets, int ndet) {
    std::vector<psn::DetectedObject> v;
    for (int i = 0; i < ndet; i++) {
        if (!dets[i].valid) continue;
        psn::DetectedObject o;
        o.id = (unsigned)i;
        o.detection.box = to_rect(dets[i].box);
        for (int b = 0; b < dets[i].num_boxes; b++) o.boxes.push_back(to_rect(dets[i].boxes[b]));
        v.push_back(std::move(o));
    }
    return v;
}

int trackers_in(const psn_t2d_tracker *trk, int ntrk, std::vector<psn::Tracker2D> &t) {
    t.resize((size_t)ntrk);
    for (int i = 0; i < ntrk; i++) {
        const psn_t2d_tracker &r = trk[i];
        // an active tracker has duration == #boxes (the forward step then pushes one
        // and indexes boxes[duration] down, :936-941)
        if (r.num_boxes < 1 || r.num_boxes >= PSN_T2D_MAX_BOXES || r.num_features < 0 ||
            r.num_features > PSN_T2D_MAX_FEATURES || r.duration != (unsigned)r.num_boxes)
            return PSN_LK_ERR_ARG;
        psn::Tracker2D &o = t[(size_t)i];
        o.duration = r.duration;
        for (int b = 0; b < r.num_boxes; b++) o.boxes.push_back(to_rect(r.boxes[b]));
        o.heads.assign(o.boxes.size(), psn::Rect());
        o.featurePoints = to_points(r.features, r.num_features);
    }
    return 0;
}

int trackers_out(const std::vector<psn::Tracker2D> &t, psn_t2d_tracker *trk, int ntrk) {
    for (int i = 0; i < ntrk; i++) {
        const psn::Tracker2D &o = t[(size_t)i];
        psn_t2d_tracker &r = trk[i];
        if (o.boxes.size() > PSN_T2D_MAX_BOXES) return PSN_T2D_ERR_CAPACITY;
        r.updated = (int)o.boxes.size() > r.num_boxes ? 1 : 0;
        r.num_boxes = (int)o.boxes.size();
        for (size_t b = 0; b < o.boxes.size(); b++) r.boxes[b] = from_rect(o.boxes[b]);
        int rc = put_points(o.featurePoints, r.features, &r.num_features);
        if (rc) return rc;
        rc = put_points(o.trackedPoints, r.tracked, &r.num_tracked);
        if (rc) return rc;
    }
    return 0;
}

int set(psn_t2d *t, int rc) {
    if (rc && t) t->err = t->flow.last_error().empty() ? ("error " + std::to_string(rc)) : t->flow.last_error();
    return rc;
}

}  // namespace

extern "C" {

int psn_rect_overlap(psn_rect a, psn_rect b) { return to_rect(a).overlap(to_rect(b)) ? 1 : 0; }
double psn_rect_distance(psn_rect a, psn_rect b) { return to_rect(a).distance(to_rect(b)); }
double psn_rect_overlapped_area(psn_rect a, psn_rect b) { return to_rect(a).overlappedArea(to_rect(b)); }
int psn_rect_contain(psn_rect a, float px, float py) { return to_rect(a).contain(psn::Point2f{px, py}) ? 1 : 0; }
void psn_rect_center(psn_rect a, double *cx, double *cy) {
    const psn::Point2D c = to_rect(a).center();
    if (cx) *cx = c.x;
    if (cy) *cy = c.y;
}

double psn_t2d_box_matching_cost(psn_rect a, psn_rect b) { return psn::BoxMatchingCost(to_rect(a), to_rect(b)); }

int psn_t2d_local_search_klt(psn_rect pre_box, const float *pre_xy, const float *cur_xy, int n, psn_rect *out_box,
                             int *inlier_idx, int *n_inliers) {
    if (n < 0 || (n > 0 && (!pre_xy || !cur_xy)) || !out_box || !n_inliers || (n > 0 && !inlier_idx))
        return PSN_LK_ERR_ARG;
    std::vector<psn::Point2f> pre((size_t)n), cur((size_t)n);
    for (int i = 0; i < n; i++) {
        pre[(size_t)i] = psn::Point2f{pre_xy[2 * i], pre_xy[2 * i + 1]};
        cur[(size_t)i] = psn::Point2f{cur_xy[2 * i], cur_xy[2 * i + 1]};
    }
    std::vector<size_t> inl;
    *out_box = from_rect(psn::LocalSearchKLT(to_rect(pre_box), pre, cur, inl));
    for (size_t i = 0; i < inl.size(); i++) inlier_idx[i] = (int)inl[i];
    *n_inliers = (int)inl.size();
    return 0;
}

int psn_t2d_create(int device, unsigned cam_id, int width, int height, psn_t2d **out) {
    if (!out) return PSN_LK_ERR_ARG;
    *out = nullptr;
    psn_t2d *t = new (std::nothrow) psn_t2d();
    if (!t) return PSN_LK_ERR_NOMEM;
    const int rc = t->flow.Initialize(cam_id, width, height, device);
    if (rc) {
        delete t;
        return rc;
    }
    *out = t;
    return 0;
}

void psn_t2d_destroy(psn_t2d *t) { delete t; }

const char *psn_t2d_last_error(psn_t2d *t) { return t ? t->err.c_str() : "null context"; }

int psn_t2d_set_device_chain(psn_t2d *t, int on) {
    if (!t) return PSN_LK_ERR_ARG;
    t->flow.SetDeviceChain(on != 0);
    return 0;
}

int psn_t2d_push_frame(psn_t2d *t, const uint8_t *frame, int stride, int channels) {
    if (!t) return PSN_LK_ERR_ARG;
    return set(t, t->flow.PushFrame(frame, stride, channels));
}

int psn_t2d_push_frame_device(psn_t2d *t, const uint8_t *dev_frame, int stride, int channels) {
    if (!t || !dev_frame) return PSN_LK_ERR_ARG;
    return set(t, t->flow.PushFrameDevice(dev_frame, stride, channels));
}

void *psn_t2d_lk_context(psn_t2d *t) { return t ? (void *)t->flow.LkContext() : nullptr; }

int psn_t2d_rotate(psn_t2d *t) {
    if (!t) return PSN_LK_ERR_ARG;
    t->flow.RotateRing();
    return 0;
}

int psn_t2d_detect_features(psn_t2d *t, psn_t2d_detection *dets, int ndet, uint32_t seed) {
    if (!t || ndet < 0 || (ndet > 0 && !dets)) return PSN_LK_ERR_ARG;
    std::vector<psn::Detection> d((size_t)ndet);
    for (int i = 0; i < ndet; i++) d[(size_t)i].box = to_rect(dets[i].box);
    std::vector<std::vector<psn::Point2f>> f;
    const int rc = t->flow.DetectFeatures(d, seed, f);
    if (rc) return set(t, rc);
    for (int i = 0; i < ndet; i++) {
        const int r = put_points(f[(size_t)i], dets[i].features, &dets[i].num_features);
        if (r) return r;
    }
    return 0;
}

int psn_t2d_backward(psn_t2d *t, psn_t2d_detection *dets, int ndet) {
    if (!t || ndet < 0 || (ndet > 0 && !dets)) return PSN_LK_ERR_ARG;
    std::vector<psn::Detection> d;
    std::vector<std::vector<psn::Point2f>> f;
    int rc = detections_in(dets, ndet, d, f);
    if (rc) return rc;
    std::vector<psn::DetectedObject> objs;
    rc = t->flow.BackwardFeatureTracking(d, f, objs);
    if (rc) return set(t, rc);
    return detections_out(objs, dets, ndet);
}

int psn_t2d_forward(psn_t2d *t, psn_t2d_tracker *trk, int ntrk, const psn_t2d_detection *dets, int ndet,
                    float *cost) {
    if (!t || ntrk < 0 || ndet < 0 || (ntrk > 0 && !trk) || (ndet > 0 && !dets)) return PSN_LK_ERR_ARG;
    std::vector<psn::Tracker2D> tr;
    int rc = trackers_in(trk, ntrk, tr);
    if (rc) return rc;
    std::vector<psn::Tracker2D *> ptr;
    for (psn::Tracker2D &x : tr) ptr.push_back(&x);
    const std::vector<psn::DetectedObject> objs = valid_objects(dets, ndet);
    std::vector<float> c;
    rc = t->flow.ForwardTrackingAndGetMatchingScore(ptr, objs, c);
    if (rc) return set(t, rc);
    if (cost && !c.empty()) std::memcpy(cost, c.data(), c.size() * sizeof(float));
    return trackers_out(tr, trk, ntrk);
}

int psn_t2d_track_frame(psn_t2d *t, psn_t2d_detection *dets, int ndet, psn_t2d_tracker *trk, int ntrk,
                        float *cost) {
    if (!t || ntrk < 0 || ndet < 0 || (ntrk > 0 && !trk) || (ndet > 0 && !dets)) return PSN_LK_ERR_ARG;
    std::vector<psn::Detection> d;
    std::vector<std::vector<psn::Point2f>> f;
    int rc = detections_in(dets, ndet, d, f);
    if (rc) return rc;
    std::vector<psn::Tracker2D> tr;
    rc = trackers_in(trk, ntrk, tr);
    if (rc) return rc;
    std::vector<psn::Tracker2D *> ptr;
    for (psn::Tracker2D &x : tr) ptr.push_back(&x);
    std::vector<psn::DetectedObject> objs;
    std::vector<float> c;
    rc = t->flow.TrackFrame(d, f, objs, ptr, c);
    if (rc) return set(t, rc);
    rc = detections_out(objs, dets, ndet);
    if (rc) return rc;
    if (cost && !c.empty()) std::memcpy(cost, c.data(), c.size() * sizeof(float));
    return trackers_out(tr, trk, ntrk);
}

int psn_t2d_track_frame_detect(psn_t2d *t, psn_t2d_detection *dets, int ndet, uint32_t seed, psn_t2d_tracker *trk,
                               int ntrk, float *cost) {
    if (!t || ntrk < 0 || ndet < 0 || (ntrk > 0 && !trk) || (ndet > 0 && !dets)) return PSN_LK_ERR_ARG;
    std::vector<psn::Detection> d((size_t)ndet);
    for (int i = 0; i < ndet; i++) d[(size_t)i].box = to_rect(dets[i].box);
    std::vector<psn::Tracker2D> tr;
    int rc = trackers_in(trk, ntrk, tr);
    if (rc) return rc;
    std::vector<psn::Tracker2D *> ptr;
    for (psn::Tracker2D &x : tr) ptr.push_back(&x);
    std::vector<std::vector<psn::Point2f>> f;
    std::vector<psn::DetectedObject> objs;
    std::vector<float> c;
    rc = t->flow.TrackFrameDetect(d, seed, f, objs, ptr, c);
    if (rc) return set(t, rc);
    for (int i = 0; i < ndet; i++) {
        rc = put_points(f[(size_t)i], dets[i].features, &dets[i].num_features);
        if (rc) return rc;
    }
    rc = detections_out(objs, dets, ndet);
    if (rc) return rc;
    if (cost && !c.empty()) std::memcpy(cost, c.data(), c.size() * sizeof(float));
    return trackers_out(tr, trk, ntrk);
}

}  // extern "C"
