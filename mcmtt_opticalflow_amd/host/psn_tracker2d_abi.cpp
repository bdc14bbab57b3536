// C ABI of include/psn_tracker2d.h over psn::Tracker2DFlow (tracker2d_flow.hpp).
#include <algorithm>
#include <cstring>
#include <list>
#include <new>
#include <string>
#include <vector>

#include "psn_tracker2d.h"
#include "tracker2d_flow.hpp"

struct psn_t2d {
    psn::Tracker2DFlow flow;
    std::string err;
};

struct psn_t2d_group {
    psn::Tracker2DFlow flow;
    // two frames' io: the current frame's, and the next frame's once its chains
    // are launched ahead (psn_t2d_group_complete_next)
    std::vector<psn::Tracker2DFlow::CamFrame> iob[2];
    std::vector<psn::Tracker2DFlow::CamFrame> &io() { return iob[cur]; }
    int cur = 0;
    int feature_mode = PSN_T2D_FEATURES_GIVEN;
    bool launched = false;
    bool ahead = false;  // the next frame's chains are in flight
    unsigned ahead_frame = 0;
    int ahead_mode = PSN_T2D_FEATURES_GIVEN;
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

// stDetection + the caller's 3D estimate of a detection record
psn::Detection detection_of(const psn_t2d_detection &r) {
    psn::Detection d;
    d.box = to_rect(r.box);
    d.vecPartBoxes.assign(1, to_rect(r.head));
    for (int k = 0; k < 3; k++) d.location[k] = r.location[k];
    d.height = r.height;
    return d;
}

int detections_in(const psn_t2d_detection *dets, int ndet, std::vector<psn::Detection> &d,
                  std::vector<std::vector<psn::Point2f>> &f, bool with_features = true) {
    d.resize((size_t)ndet);
    f.resize((size_t)ndet);
    for (int i = 0; i < ndet; i++) {
        d[(size_t)i] = detection_of(dets[i]);
        if (!with_features) continue;
        if (dets[i].num_features < 0 || dets[i].num_features > PSN_T2D_MAX_FEATURES) return PSN_T2D_ERR_CAPACITY;
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
        o.detection = detection_of(dets[i]);
        for (int k = 0; k < 3; k++) o.location[k] = dets[i].location[k];
        o.height = dets[i].height;
        o.bOverlapWithOtherDetection = dets[i].overlap_other != 0;
        for (int b = 0; b < dets[i].num_boxes; b++) o.boxes.push_back(to_rect(dets[i].boxes[b]));
        for (int s2 = 0; s2 < dets[i].num_sets && s2 < PSN_T2D_INTERVAL; s2++)
            o.vecvecTrackedFeatures.push_back(to_points(dets[i].sets[s2], dets[i].set_count[s2]));
        v.push_back(std::move(o));
    }
    return v;
}

int tracker_of(const psn_t2d_tracker &r, psn::Tracker2D &o) {
    if (r.num_boxes < 1 || r.num_boxes > PSN_T2D_MAX_BOXES || r.num_features < 0 ||
        r.num_features > PSN_T2D_MAX_FEATURES || r.num_tracked < 0 || r.num_tracked > PSN_T2D_MAX_FEATURES)
        return PSN_LK_ERR_ARG;
    o = psn::Tracker2D();
    o.id = r.id;
    o.timeStart = r.time_start;
    o.timeEnd = r.time_end;
    o.timeLastUpdate = r.time_last_update;
    o.duration = r.duration;
    o.confidence = r.confidence;
    for (int b = 0; b < r.num_boxes; b++) {
        o.boxes.push_back(to_rect(r.boxes[b]));
        o.heads.push_back(to_rect(r.heads[b]));
    }
    o.featurePoints = to_points(r.features, r.num_features);
    o.trackedPoints = to_points(r.tracked, r.num_tracked);
    for (int k = 0; k < 3; k++) o.lastPosition[k] = r.last_position[k];
    o.height = r.height;
    return 0;
}

int record_of(const psn::Tracker2D &o, psn_t2d_tracker &r) {
    if (o.boxes.size() > PSN_T2D_MAX_BOXES || o.heads.size() != o.boxes.size()) return PSN_T2D_ERR_CAPACITY;
    r.id = o.id;
    r.time_start = o.timeStart;
    r.time_end = o.timeEnd;
    r.time_last_update = o.timeLastUpdate;
    r.duration = o.duration;
    r.confidence = o.confidence;
    r.num_boxes = (int)o.boxes.size();
    for (size_t b = 0; b < o.boxes.size(); b++) {
        r.boxes[b] = from_rect(o.boxes[b]);
        r.heads[b] = from_rect(o.heads[b]);
    }
    for (int k = 0; k < 3; k++) r.last_position[k] = o.lastPosition[k];
    r.height = o.height;
    int rc = put_points(o.featurePoints, r.features, &r.num_features);
    if (rc) return rc;
    return put_points(o.trackedPoints, r.tracked, &r.num_tracked);
}

int trackers_in(const psn_t2d_tracker *trk, int ntrk, std::vector<psn::Tracker2D> &t) {
    t.resize((size_t)ntrk);
    for (int i = 0; i < ntrk; i++) {
        // an active tracker has duration == #boxes (the forward step then pushes one
        // and indexes boxes[duration] down, :936-941)
        if (trk[i].num_boxes >= PSN_T2D_MAX_BOXES || trk[i].duration != (unsigned)trk[i].num_boxes)
            return PSN_LK_ERR_ARG;
        const int rc = tracker_of(trk[i], t[(size_t)i]);
        if (rc) return rc;
        t[(size_t)i].trackedPoints.clear();
    }
    return 0;
}

int trackers_out(const std::vector<psn::Tracker2D> &t, psn_t2d_tracker *trk, int ntrk) {
    for (int i = 0; i < ntrk; i++) {
        psn_t2d_tracker &r = trk[i];
        const int before = r.num_boxes;
        const int rc = record_of(t[(size_t)i], r);
        if (rc) return rc;
        r.updated = r.num_boxes > before ? 1 : 0;
    }
    return 0;
}

int object_out(const psn::Object2DInfo &o, psn_object2d &r) {
    r.id = o.id;
    r.box = from_rect(o.box);
    r.head = from_rect(o.head);
    r.score = o.score;
    const int rc = put_points(o.featurePointsPrev, r.prev, &r.num_prev);
    return rc ? rc : put_points(o.featurePointsCurr, r.curr, &r.num_curr);
}

int result_out(const psn::Track2DResult &res, psn_track2d_result *r) {
    if (!r || (int)res.object2DInfos.size() > std::max(r->cap_objects, 0) ||
        (!res.object2DInfos.empty() && !r->objects))
        return PSN_T2D_ERR_CAPACITY;
    r->cam_id = res.camID;
    r->frame_idx = res.frameIdx;
    r->num_objects = (int)res.object2DInfos.size();
    for (size_t i = 0; i < res.object2DInfos.size(); i++) {
        const int rc = object_out(res.object2DInfos[i], r->objects[i]);
        if (rc) return rc;
    }
    r->num_detection_rects = 0;  // never filled by the reference (vecDetectionRects / vecTrackerRects)
    r->num_tracker_rects = 0;
    return 0;
}

int set(psn_t2d *t, int rc) {
    if (rc && t) t->err = t->flow.last_error().empty() ? ("error " + std::to_string(rc)) : t->flow.last_error();
    return rc;
}

}  // namespace

extern "C" {

int psn_t2d_abi_version(void) { return PSN_T2D_ABI_VERSION; }

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

int psn_t2d_assign(const float *cost, int rows, int cols, int *match) {
    if (rows < 0 || cols < 0 || (rows > 0 && !match) || (rows > 0 && cols > 0 && !cost)) return PSN_LK_ERR_ARG;
    std::vector<float> c;
    if (rows > 0 && cols > 0) c.assign(cost, cost + (size_t)rows * cols);
    const std::vector<int> m = psn::AssignDetections(c, (size_t)rows, (size_t)cols);
    for (int r = 0; r < rows; r++) match[r] = m[(size_t)r];
    return 0;
}

int psn_t2d_hungarian_match(const float *cost, int rows, int cols, int *out_rows, int *out_cols, float *out_costs,
                            int *n_out) {
    if (rows < 0 || cols < 0 || !n_out || (rows > 0 && cols > 0 && (!cost || !out_rows || !out_cols || !out_costs)))
        return PSN_LK_ERR_ARG;
    *n_out = 0;
    std::vector<float> c;
    if (rows > 0 && cols > 0) c.assign(cost, cost + (size_t)rows * cols);
    std::vector<int> r, k;
    std::vector<float> v;
    if (!psn::HungarianMatch(c, (size_t)rows, (size_t)cols, r, k, v)) return PSN_LK_ERR_ARG;
    for (size_t i = 0; i < r.size(); i++) {
        out_rows[i] = r[i];
        out_cols[i] = k[i];
        out_costs[i] = v[i];
    }
    *n_out = (int)r.size();
    return 0;
}

int psn_t2d_result_with_tracker(const psn_t2d_tracker *trk, psn_object2d *out) {
    if (!trk || !out) return PSN_LK_ERR_ARG;
    psn::Tracker2D t;
    int rc = tracker_of(*trk, t);
    if (rc) return rc;
    psn::Object2DInfo o;
    psn::ResultWithTracker(t, o);
    return object_out(o, *out);
}

int psn_t2d_matching_and_updating(const psn_t2d_detection *dets, int ndet, const psn_t2d_tracker *trk, int ntrk,
                                  const float *cost, const int *match, unsigned frame_idx, unsigned *next_id,
                                  psn_t2d_tracker *out_trk, int cap_trk, int *n_out, psn_track2d_result *result) {
    if (ndet < 0 || ntrk < 0 || (ndet > 0 && !dets) || (ntrk > 0 && !trk) || !next_id || !n_out || !result ||
        cap_trk < 0 || (cap_trk > 0 && !out_trk))
        return PSN_LK_ERR_ARG;
    std::vector<psn::DetectedObject> objs = valid_objects(dets, ndet);
    for (const psn::DetectedObject &o : objs)
        if (o.vecvecTrackedFeatures.empty()) return PSN_LK_ERR_ARG;  // a valid detection has its features at t
    if (!objs.empty() && ntrk > 0 && !cost && !match) return PSN_LK_ERR_ARG;
    std::list<psn::Tracker2D> storage;
    std::deque<psn::Tracker2D *> active;
    for (int i = 0; i < ntrk; i++) {
        storage.emplace_back();
        const int rc = tracker_of(trk[i], storage.back());
        if (rc) return rc;
        active.push_back(&storage.back());
    }
    std::vector<int> m(objs.size(), -1);
    if (match) {
        // an assignment: each tracker at most once (the Hungarian's output never
        // repeats a column; a repeat would update and enqueue one tracker twice)
        std::vector<char> taken((size_t)ntrk, 0);
        for (size_t d = 0; d < objs.size(); d++) {
            if (match[d] < -1 || match[d] >= ntrk) return PSN_LK_ERR_ARG;
            if (match[d] >= 0 && taken[(size_t)match[d]]++) return PSN_LK_ERR_ARG;
            m[d] = match[d];
        }
    } else if (ntrk > 0 && !objs.empty()) {
        m = psn::AssignDetections(std::vector<float>(cost, cost + objs.size() * (size_t)ntrk), objs.size(), (size_t)ntrk);
    }
    psn::Track2DResult res;
    res.camID = result->cam_id;
    psn::MatchingAndUpdating(objs, active, storage, m, frame_idx, *next_id, res);
    if ((int)active.size() > cap_trk) return PSN_T2D_ERR_CAPACITY;
    for (size_t i = 0; i < active.size(); i++) {
        const int rc = record_of(*active[i], out_trk[i]);
        if (rc) return rc;
        out_trk[i].updated = 0;
    }
    *n_out = (int)active.size();
    return result_out(res, result);
}

// ---- psn_t2d_group: CPSNWhere_Tracker2D::Run of several cameras ----

int psn_t2d_group_create(int device, int ncams, const unsigned *cam_ids, int width, int height, psn_t2d_group **out) {
    if (!out || ncams <= 0 || !cam_ids) return PSN_LK_ERR_ARG;
    *out = nullptr;
    psn_t2d_group *g = new (std::nothrow) psn_t2d_group();
    if (!g) return PSN_LK_ERR_NOMEM;
    const int rc = g->flow.InitializeCameras(std::vector<unsigned>(cam_ids, cam_ids + ncams), width, height, device);
    if (rc) {
        delete g;
        return rc;
    }
    g->iob[0].resize((size_t)ncams);
    g->iob[1].resize((size_t)ncams);
    *out = g;
    return 0;
}

void psn_t2d_group_destroy(psn_t2d_group *g) { delete g; }

const char *psn_t2d_group_last_error(psn_t2d_group *g) { return g ? g->err.c_str() : "null context"; }

void *psn_t2d_group_lk_context(psn_t2d_group *g) { return g ? (void *)g->flow.LkContext() : nullptr; }

static int gset(psn_t2d_group *g, int rc) {
    if (rc) g->err = g->flow.last_error().empty() ? ("error " + std::to_string(rc)) : g->flow.last_error();
    return rc;
}

int psn_t2d_group_push_frame(psn_t2d_group *g, int cam, const uint8_t *frame, int stride, int channels) {
    if (!g || cam < 0 || (size_t)cam >= g->io().size() || !frame) return PSN_LK_ERR_ARG;
    return gset(g, g->flow.StageFrame((size_t)cam, frame, stride, channels, false));
}

int psn_t2d_group_push_frame_device(psn_t2d_group *g, int cam, const uint8_t *dev_frame, int stride, int channels) {
    if (!g || cam < 0 || (size_t)cam >= g->io().size() || !dev_frame) return PSN_LK_ERR_ARG;
    return gset(g, g->flow.StageFrame((size_t)cam, dev_frame, stride, channels, true));
}

int psn_t2d_group_push_frame_jpeg(psn_t2d_group *g, int cam, const uint8_t *jpeg, size_t len) {
    if (!g || cam < 0 || (size_t)cam >= g->io().size() || !jpeg) return PSN_LK_ERR_ARG;
    return gset(g, g->flow.StageFrameJpeg((size_t)cam, jpeg, len));
}

int psn_t2d_group_launch(psn_t2d_group *g, unsigned frame_idx, psn_t2d_detection *const *dets, const int *ndet,
                         int feature_mode, uint32_t seed) {
    if (!g || !ndet || !dets || (feature_mode != PSN_T2D_FEATURES_GIVEN && feature_mode != PSN_T2D_FEATURES_GRIDFAST) ||
        g->launched)
        return PSN_LK_ERR_ARG;
    if (g->ahead) {  // the frame announced by complete_next: its detections are in io() already
        if (frame_idx != g->ahead_frame || feature_mode != g->ahead_mode) return PSN_LK_ERR_ARG;
        for (size_t c = 0; c < g->io().size(); c++)
            if (ndet[c] < 0 || (size_t)ndet[c] != g->io()[c].dets.size()) return PSN_LK_ERR_ARG;
    } else {
        for (size_t c = 0; c < g->io().size(); c++) {
            if (ndet[c] < 0 || (ndet[c] > 0 && !dets[c])) return PSN_LK_ERR_ARG;
            psn::Tracker2DFlow::CamFrame &f = g->io()[c];
            const int rc = detections_in(dets[c], ndet[c], f.dets, f.features, feature_mode == PSN_T2D_FEATURES_GIVEN);
            if (rc) return rc;
        }
    }
    g->feature_mode = feature_mode;
    const int rc = g->flow.RunLaunch(frame_idx, g->io(), feature_mode == PSN_T2D_FEATURES_GRIDFAST, seed);
    g->ahead = false;
    if (rc) return gset(g, rc);
    g->launched = true;
    return 0;
}

// results of the current frame (after RunComplete) into the caller's records
static int group_outputs(psn_t2d_group *g, psn_t2d_detection *const *dets, const int *ndet,
                         psn_track2d_result *results) {
    for (size_t c = 0; c < g->io().size(); c++) {
        psn::Tracker2DFlow::CamFrame &f = g->io()[c];
        if ((size_t)ndet[c] != f.dets.size()) return PSN_LK_ERR_ARG;
        int rc = 0;
        if (g->feature_mode == PSN_T2D_FEATURES_GRIDFAST)
            for (int i = 0; i < ndet[c]; i++) {
                rc = put_points(f.features[(size_t)i], dets[c][i].features, &dets[c][i].num_features);
                if (rc) return rc;
            }
        rc = detections_out(f.objects, dets[c], ndet[c]);
        if (!rc) rc = result_out(f.result, &results[c]);
        if (rc) return rc;
    }
    return 0;
}

int psn_t2d_group_complete(psn_t2d_group *g, psn_t2d_detection *const *dets, const int *ndet,
                           psn_track2d_result *results) {
    if (!g || !ndet || !dets || !results || !g->launched) return PSN_LK_ERR_ARG;
    g->launched = false;
    const int rc = g->flow.RunComplete(g->io());
    if (rc) return gset(g, rc);
    return group_outputs(g, dets, ndet, results);
}

int psn_t2d_group_complete_next(psn_t2d_group *g, psn_t2d_detection *const *dets, const int *ndet,
                                psn_track2d_result *results, unsigned next_frame_idx,
                                psn_t2d_detection *const *next_dets, const int *next_ndet, int feature_mode,
                                uint32_t seed) {
    if (!g || !ndet || !dets || !results || !g->launched || !next_ndet || !next_dets ||
        (feature_mode != PSN_T2D_FEATURES_GIVEN && feature_mode != PSN_T2D_FEATURES_GRIDFAST))
        return PSN_LK_ERR_ARG;
    std::vector<psn::Tracker2DFlow::CamFrame> &nx = g->iob[g->cur ^ 1];
    for (size_t c = 0; c < nx.size(); c++) {
        if (next_ndet[c] < 0 || (next_ndet[c] > 0 && !next_dets[c])) return PSN_LK_ERR_ARG;
        const int rc = detections_in(next_dets[c], next_ndet[c], nx[c].dets, nx[c].features,
                                     feature_mode == PSN_T2D_FEATURES_GIVEN);
        if (rc) return rc;
    }
    g->launched = false;
    const int rc = g->flow.RunComplete(g->io(), &nx, next_frame_idx, feature_mode == PSN_T2D_FEATURES_GRIDFAST, seed);
    if (rc && g->flow.FrameCompleted()) {
        // only the next frame failed to launch: this frame's results are still
        // delivered, and that frame (staged again) is for a plain launch
        const int orc = group_outputs(g, dets, ndet, results);
        gset(g, rc);
        g->err = "next frame " + std::to_string(next_frame_idx) + " not launched: " + g->err;
        return orc ? orc : rc;
    }
    if (rc) return gset(g, rc);
    const int orc = group_outputs(g, dets, ndet, results);
    g->cur ^= 1;  // the next frame's io, launched ahead
    g->ahead = true;
    g->ahead_frame = next_frame_idx;
    g->ahead_mode = feature_mode;
    return orc;
}

int psn_t2d_group_run(psn_t2d_group *g, unsigned frame_idx, psn_t2d_detection *const *dets, const int *ndet,
                      int feature_mode, uint32_t seed, psn_track2d_result *results) {
    const int rc = psn_t2d_group_launch(g, frame_idx, dets, ndet, feature_mode, seed);
    return rc ? rc : psn_t2d_group_complete(g, dets, ndet, results);
}

int psn_t2d_group_debug_host_times(psn_t2d_group *g, double *out6) {
    if (!g || !out6) return PSN_LK_ERR_ARG;
    g->flow.HostTimes(out6);
    return 0;
}

int psn_t2d_group_debug_host_match_times(psn_t2d_group *g, double *out4) {
    if (!g || !out4) return PSN_LK_ERR_ARG;
    g->flow.HostMatchTimes(out4);
    return 0;
}

int psn_t2d_group_trackers(psn_t2d_group *g, int cam, psn_t2d_tracker *out, int cap, int *n) {
    if (!g || cam < 0 || (size_t)cam >= g->io().size() || !n || cap < 0 || (cap > 0 && !out)) return PSN_LK_ERR_ARG;
    const std::deque<psn::Tracker2D *> &a = g->flow.ActiveTrackers((size_t)cam);
    *n = (int)a.size();
    if ((int)a.size() > cap) return PSN_T2D_ERR_CAPACITY;
    for (size_t i = 0; i < a.size(); i++) {
        const int rc = record_of(*a[i], out[i]);
        if (rc) return rc;
        out[i].updated = 0;
    }
    return 0;
}

}  // extern "C"
