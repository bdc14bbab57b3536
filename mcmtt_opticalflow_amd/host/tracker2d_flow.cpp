// Tracker2D flow stage (see tracker2d_flow.hpp). Reference lines cited are in
// psn_where/PSNWhere_Tracker2D.cpp unless noted.
#include "tracker2d_flow.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "psn_t2d_device.h"

namespace psn {

// :452-554. Vectors with |d| >= 0.1 px vote; if fewer than half the points
// move, the box stays put with no inliers. Otherwise the mode of dx and of dy
// (most neighbours within 0.2 box widths, first maximum in sorted order) is
// the box shift and the inliers are the moving vectors within that window of
// the mode, in point order.
Rect LocalSearchKLT(Rect preBox, const std::vector<Point2f> &preFeatures, const std::vector<Point2f> &curFeatures,
                    std::vector<size_t> &inlierFeatureIndex) {
    const double kMinMovement = 0.1, kNeighborRatio = 0.2;
    const size_t numFeatures = preFeatures.size();
    size_t numMoving = 0;
    inlierFeatureIndex.clear();
    std::vector<Point2D> vecMoving;
    std::vector<size_t> vecMovingIdx;
    std::vector<double> vecDx, vecDy;
    for (size_t i = 0; i < numFeatures; i++) {
        // cv::Point2f difference (float), then widened to PSN_Point2D
        const Point2f d{curFeatures[i].x - preFeatures[i].x, curFeatures[i].y - preFeatures[i].y};
        const Point2D mv(d);
        if (mv.norm_L2() < kMinMovement * kFlowScale) continue;
        vecMoving.push_back(mv);
        vecMovingIdx.push_back(i);
        vecDx.push_back(mv.x);
        vecDy.push_back(mv.y);
        numMoving++;
    }
    if ((double)numMoving < (double)numFeatures * 0.5) return preBox;
    std::sort(vecDx.begin(), vecDx.end());
    std::sort(vecDy.begin(), vecDy.end());
    const double windowSize = preBox.w * kNeighborRatio * kFlowScale;
    size_t maxX = 0, maxY = 0;
    Point2D est(0.0, 0.0);
    for (size_t d = 0; d < numMoving; d++) {
        size_t nx = 0, ny = 0;
        for (size_t c = 0; c < numMoving; c++) {
            if (std::abs(vecDx[d] - vecDx[c]) < windowSize) nx++;
            if (std::abs(vecDy[d] - vecDy[c]) < windowSize) ny++;
        }
        if (maxX < nx) {
            est.x = vecDx[d];
            maxX = nx;
        }
        if (maxY < ny) {
            est.y = vecDy[d];
            maxY = ny;
        }
    }
    for (size_t v = 0; v < numMoving; v++)
        if ((vecMoving[v] - est).norm_L2() < windowSize) inlierFeatureIndex.push_back(vecMovingIdx[v]);
    Rect box = preBox;
    box.x += est.x;
    box.y += est.y;
    return box;
}

// :600-613
double BoxMatchingCost(const Rect &box1, const Rect &box2) {
    const double nom = (box1.center() - box2.center()).norm_L2();
    const double den = (box1.w + box2.w) / 2.0;
    return (nom * nom) / (den * den);
}

// :1231-1257 (PSN_2D_DEBUG_DISPLAY_SCALE = 1.0: the float scaling is exact)
void ResultWithTracker(const Tracker2D &tracker, Object2DInfo &out) {
    const float s = 1.0f;
    out.featurePointsPrev = tracker.featurePoints;
    out.featurePointsCurr = tracker.trackedPoints;
    out.id = tracker.id;
    const Rect &b = tracker.boxes.back(), &h = tracker.heads.back();
    out.box = Rect(b.x * s, b.y * s, b.w * s, b.h * s);
    out.head = Rect(h.x * s, h.y * s, h.w * s, h.h * s);
    out.score = 0;
    for (size_t i = 0; i < out.featurePointsPrev.size(); i++) {
        out.featurePointsPrev[i].x *= s;
        out.featurePointsPrev[i].y *= s;
        if (i >= out.featurePointsCurr.size()) continue;
        out.featurePointsCurr[i].x *= s;
        out.featurePointsCurr[i].y *= s;
    }
}

int Tracker2DFlow::fail(int rc, const char *what) {
    err_ = std::string(what) + ": " + (lk_ ? psn_lk_last_error(lk_) : "no context") + " (" + std::to_string(rc) + ")";
    return rc;
}

int Tracker2DFlow::Initialize(unsigned camID, int width, int height, int device) {
    Finalize();
    if (const char *e = std::getenv("PSN_T2D_HOST_CHAIN")) device_chain_ = std::atoi(e) == 0;
    camID_ = camID;
    width_ = width;
    height_ = height;
    // 4 slots of full pyramids; the reference's default maxLevel 3 needs 4 levels
    const int rc = psn_lk_create(device, width, height, kT2dInterval, 3, &lk_);
    if (rc) {
        lk_ = nullptr;
        err_ = "psn_lk_create failed (" + std::to_string(rc) + ")";
        return rc;
    }
    for (int i = 0; i < kT2dInterval; i++) {
        ring_[i] = i;
        filled_[i] = false;
    }
    hipStream_t fs = nullptr;
    hipEvent_t ev = nullptr;
    if (hipStreamCreateWithFlags(&fs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        err_ = "forward stream / event";
        return PSN_LK_ERR_HIP;
    }
    fwd_stream_ = fs;
    ev_in_ = ev;
    return PSN_LK_OK;
}

// Device and pinned-host buffers of the device-side chain (grown on demand).
struct Tracker2DFlow::DeviceBuffers {
    size_t nchains = 0, nfwd_pts = 0, nfwd_jobs = 0;
    float *d_in = nullptr, *d_out = nullptr, *d_buf[2] = {nullptr, nullptr}, *d_err = nullptr;
    uint8_t *d_status = nullptr;
    double *d_boxes = nullptr, *d_obox = nullptr;
    float *d_sets = nullptr;
    int *d_cnt = nullptr, *d_setcnt = nullptr, *d_nsteps = nullptr, *d_tot = nullptr;
    // pinned staging: inputs, then results
    float *h_in = nullptr, *h_fwd_out = nullptr, *h_sets = nullptr;
    uint8_t *h_fwd_st = nullptr;
    double *h_boxes = nullptr, *h_obox = nullptr;
    int *h_cnt = nullptr, *h_setcnt = nullptr, *h_nsteps = nullptr, *h_rawcnt = nullptr;
    // the chain's results live in one block per side, [nsteps | set counts | boxes | sets], so that
    // one memset clears the counters and one copy returns every used byte
    char *d_res = nullptr, *h_res = nullptr;
    size_t res_sets_off = 0;
    void carve(char *base, double *&obox, float *&sets, int *&setcnt, int *&nsteps, size_t K, size_t S) const {
        nsteps = (int *)base;
        setcnt = nsteps + K;
        obox = (double *)(base + res_box_off(K, S));
        sets = (float *)(base + res_sets_off);
    }
    static size_t res_box_off(size_t K, size_t S) { return (K * (1 + S) * 4 + 255) & ~(size_t)255; }
    void release() {
        for (void *p : {(void *)d_in, (void *)d_out, (void *)d_buf[0], (void *)d_buf[1], (void *)d_err, (void *)d_status,
                        (void *)d_boxes, (void *)d_res, (void *)d_cnt, (void *)d_tot})
            if (p) (void)hipFree(p);
        for (void *p : {(void *)h_in, (void *)h_fwd_out, (void *)h_fwd_st, (void *)h_boxes, (void *)h_res,
                        (void *)h_cnt, (void *)h_rawcnt})
            if (p) (void)hipHostFree(p);
        *this = DeviceBuffers();
    }
};

void Tracker2DFlow::Finalize() {
    if (dev_) {
        if (lk_) psn_lk_sync(lk_);
        dev_->release();
        delete dev_;
        dev_ = nullptr;
    }
    if (fwd_stream_) {
        (void)hipStreamSynchronize((hipStream_t)fwd_stream_);
        (void)hipStreamDestroy((hipStream_t)fwd_stream_);
        fwd_stream_ = nullptr;
    }
    if (ev_in_) (void)hipEventDestroy((hipEvent_t)ev_in_);
    ev_in_ = nullptr;
    if (lk_) psn_lk_destroy(lk_);
    lk_ = nullptr;
}

int Tracker2DFlow::EnsureDevice(size_t nchains, size_t nfwd_pts, size_t nfwd_jobs) {
    if (!dev_) dev_ = new DeviceBuffers();
    DeviceBuffers &b = *dev_;
    if (b.nchains >= nchains && b.nfwd_pts >= nfwd_pts && b.nfwd_jobs >= nfwd_jobs && b.d_in) return PSN_LK_OK;
    if (lk_) psn_lk_sync(lk_);
    b.release();
    const size_t K = std::max<size_t>(nchains, 16), F = std::max<size_t>(nfwd_pts, 1024), J = std::max<size_t>(nfwd_jobs, 16);
    const size_t cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS, npt = K * cap + F;
    bool ok = true;
    auto dm = [&](void **p, size_t bytes) { ok = ok && hipMalloc(p, bytes) == hipSuccess; };
    auto hm = [&](void **p, size_t bytes) { ok = ok && hipHostMalloc(p, bytes, hipHostMallocDefault) == hipSuccess; };
    dm((void **)&b.d_in, npt * 8);
    dm((void **)&b.d_out, npt * 8);
    dm((void **)&b.d_buf[0], K * cap * 8);
    dm((void **)&b.d_buf[1], K * cap * 8);
    dm((void **)&b.d_err, npt * 4);
    dm((void **)&b.d_status, npt);
    dm((void **)&b.d_boxes, K * 4 * 8);
    b.res_sets_off = DeviceBuffers::res_box_off(K, S) + K * S * 4 * 8;
    const size_t res_bytes = b.res_sets_off + K * S * cap * 8;
    dm((void **)&b.d_res, res_bytes);
    dm((void **)&b.d_cnt, (K + J) * 4);
    dm((void **)&b.d_tot, K * 4);
    hm((void **)&b.h_in, npt * 8);
    hm((void **)&b.h_fwd_out, F * 8);
    hm((void **)&b.h_fwd_st, F);
    hm((void **)&b.h_boxes, K * 4 * 8);
    hm((void **)&b.h_res, res_bytes);
    hm((void **)&b.h_cnt, (K + J) * 4);
    hm((void **)&b.h_rawcnt, K * 4);
    if (!ok) {
        b.release();
        err_ = "device-chain buffers: allocation failed";
        return PSN_LK_ERR_NOMEM;
    }
    b.carve(b.d_res, b.d_obox, b.d_sets, b.d_setcnt, b.d_nsteps, K, S);
    b.carve(b.h_res, b.h_obox, b.h_sets, b.h_setcnt, b.h_nsteps, K, S);
    b.nchains = K;
    b.nfwd_pts = F;
    b.nfwd_jobs = J;
    return PSN_LK_OK;
}

// The backward chains of a frame on the device (:763-811): per step one
// counted LK launch over every chain (capacity PSN_T2D_CHAIN_CAP points each;
// a stopped chain's count is 0 so its workgroups exit at once) and one
// LocalSearchKLT + inlier-compaction kernel writing the next step's points and
// counts. The forward calls ride in step 1's launch. Everything is enqueued on
// the LK context stream; the host waits once, for the packed results.
int Tracker2DFlow::ChainsOnDevice(std::vector<Chain> &chains, std::vector<DetectedObject> &out, std::vector<Job> *fwd) {
    const size_t K = chains.size(), cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS;
    size_t F = 0;
    const size_t J = fwd ? fwd->size() : 0;
    for (size_t j = 0; j < J; j++) F += (*fwd)[j].in->size();
    if (K == 0 && F == 0 && J == 0) return PSN_LK_OK;
    int rc = EnsureDevice(K, F, J);
    if (rc) return rc;
    DeviceBuffers &b = *dev_;
    hipStream_t st = (hipStream_t)psn_lk_get_stream(lk_);
    // inputs: chain k's points at k*cap, then the forward jobs' points
    for (size_t k = 0; k < K; k++) {
        const Chain &c = chains[k];
        const Rect box = out[c.obj].detection.box.scale(kFlowScale);
        b.h_boxes[4 * k] = box.x;
        b.h_boxes[4 * k + 1] = box.y;
        b.h_boxes[4 * k + 2] = box.w;
        b.h_boxes[4 * k + 3] = box.h;
        for (size_t i = 0; i < c.curr.size(); i++) {
            b.h_in[2 * (k * cap + i)] = c.curr[i].x;
            b.h_in[2 * (k * cap + i) + 1] = c.curr[i].y;
        }
        b.h_cnt[k] = (int)c.curr.size();
    }
    size_t o = K * cap;
    for (size_t j = 0; j < J; j++) {
        const std::vector<Point2f> &pts = *(*fwd)[j].in;
        for (size_t i = 0; i < pts.size(); i++, o++) {
            b.h_in[2 * o] = pts[i].x;
            b.h_in[2 * o + 1] = pts[i].y;
        }
        b.h_cnt[K + j] = (int)pts.size();
    }
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            err_ = std::string(what) + ": " + hipGetErrorString(e);
            rc = PSN_LK_ERR_HIP;
        }
    };
    chk(hipMemcpyAsync(b.d_in, b.h_in, (K * cap + F) * 8, hipMemcpyHostToDevice, st), "chain inputs");
    chk(hipMemcpyAsync(b.d_boxes, b.h_boxes, std::max<size_t>(K, 1) * 32, hipMemcpyHostToDevice, st), "chain boxes");
    chk(hipMemcpyAsync(b.d_cnt, b.h_cnt, (K + J) * 4, hipMemcpyHostToDevice, st), "chain counts");
    chk(hipMemsetAsync(b.d_nsteps, 0, b.nchains * (1 + S) * 4, st), "chain steps and set counts");
    if (rc) return rc;
    psn_t2d_chain_dev cd{};
    cd.ndet = (int)K;
    cd.cap = (int)cap;
    cd.boxes = b.d_boxes;
    cd.cnt = b.d_cnt;
    cd.out_boxes = b.d_obox;
    cd.sets = b.d_sets;
    cd.set_cnt = b.d_setcnt;
    cd.nsteps = b.d_nsteps;
    const bool step1 = StepAvailable(1);
    for (int step = 1; step < (int)S && (step == 1 || (K && StepAvailable(step))); step++) {
        queries_.clear();
        if (step > 1 || step1)
            for (size_t k = 0; k < K; k++) {
                psn_lk_query q;
                q.prev_slot = ring_[kT2dInterval - step];
                q.next_slot = ring_[kT2dInterval - 1 - step];
                q.first_pt = (int)(k * cap);
                q.num_pts = (int)cap;
                psn_lk_default_params(&q.params);
                q.params.win_w = q.params.win_h = (int)(b.h_boxes[4 * k + 2] * kWinSizeRatio);
                queries_.push_back(q);
            }
        const size_t nb = queries_.size();
        if (step == 1 && J) {
            // the forward calls (Track2D_ForwardTrackingAndGetMatchingScore) are independent of the
            // backward chain: their launch runs on the forward stream, beside the chain's launches
            fwd_queries_.clear();
            for (size_t j = 0, off = K * cap; j < J; j++) {
                const Job &jb = (*fwd)[j];
                psn_lk_query q;
                q.prev_slot = jb.prev_slot;
                q.next_slot = jb.next_slot;
                q.first_pt = (int)off;
                q.num_pts = (int)jb.in->size();
                psn_lk_default_params(&q.params);
                q.params.win_w = jb.win_w;
                q.params.win_h = jb.win_h;
                fwd_queries_.push_back(q);
                off += jb.in->size();
            }
            hipStream_t fs = (hipStream_t)fwd_stream_;
            chk(hipEventRecord((hipEvent_t)ev_in_, st), "inputs event");
            chk(hipStreamWaitEvent(fs, (hipEvent_t)ev_in_, 0), "forward wait");
            if (rc) return rc;
            rc = psn_lk_set_stream(lk_, fs);
            if (!rc)
                rc = psn_lk_track_device_counted(lk_, fwd_queries_.data(), (int)J, b.d_cnt + K, b.d_in, b.d_out,
                                                 b.d_status, b.d_err);
            const int rs = psn_lk_set_stream(lk_, st);
            if (rc || rs) return fail(rc ? rc : rs, "forward launch");
            if (F) {
                chk(hipMemcpyAsync(b.h_fwd_out, b.d_out + 2 * K * cap, F * 8, hipMemcpyDeviceToHost, fs), "forward points");
                chk(hipMemcpyAsync(b.h_fwd_st, b.d_status + K * cap, F, hipMemcpyDeviceToHost, fs), "forward status");
            }
        }
        if (queries_.empty()) break;
        const float *in = step == 1 ? b.d_in : b.d_buf[step & 1];
        rc = rc ? rc
                : psn_lk_track_device_counted(lk_, queries_.data(), (int)queries_.size(), b.d_cnt, in, b.d_out,
                                              b.d_status, b.d_err);
        if (rc) return fail(rc, "psn_lk_track_device_counted");
        if (nb == 0) break;
        cd.cur = in;
        cd.nxt = b.d_out;
        cd.next_in = b.d_buf[(step + 1) & 1];
        rc = psn_t2d_chain_step_device(&cd, step, st);
        if (rc) return fail(rc, "psn_t2d_chain_step_device");
    }
    if (K) {
        chk(hipMemcpyAsync(b.h_res, b.d_res, b.res_sets_off + K * S * cap * 8, hipMemcpyDeviceToHost, st), "chain results");
    }
    chk(hipStreamSynchronize(st), "chain sync");
    chk(hipStreamSynchronize((hipStream_t)fwd_stream_), "forward sync");
    if (rc) return rc;
    for (size_t k = 0; k < K; k++) {
        DetectedObject &ob = out[chains[k].obj];
        const int ns = b.h_nsteps[k];
        for (int s2 = 1; s2 <= ns; s2++) {
            const double *r = b.h_obox + (k * S + s2) * 4;
            ob.boxes.push_back(Rect(r[0], r[1], r[2], r[3]).scale(1.0 / kFlowScale));
        }
        for (int r = 0; ns > 0 && r <= ns; r++) {
            const int n = b.h_setcnt[k * S + r];
            const float *p = b.h_sets + (k * S + r) * cap * 2;
            std::vector<Point2f> v((size_t)n);
            for (int i = 0; i < n; i++) v[(size_t)i] = Point2f{p[2 * i], p[2 * i + 1]};
            ob.vecvecTrackedFeatures.push_back(std::move(v));
        }
        chains[k].active = false;
    }
    for (size_t j = 0, off = 0; j < J; j++) {
        Job &jb = (*fwd)[j];
        const size_t m = jb.in->size();
        jb.out->resize(m);
        jb.status->resize(m);
        for (size_t i = 0; i < m; i++, off++) {
            (*jb.out)[i] = Point2f{b.h_fwd_out[2 * off], b.h_fwd_out[2 * off + 1]};
            (*jb.status)[i] = b.h_fwd_st[off];
        }
    }
    return PSN_LK_OK;
}

int Tracker2DFlow::PushFrame(const uint8_t *frame, int stride, int channels) {
    if (!lk_) return PSN_LK_ERR_ARG;
    const int slot = ring_[kT2dInterval - 1];
    const int rc = psn_lk_push_frame(lk_, slot, frame, stride, channels);
    if (rc) return fail(rc, "psn_lk_push_frame");
    filled_[slot] = true;
    return PSN_LK_OK;
}

int Tracker2DFlow::PushFrameDevice(const uint8_t *dev, int stride, int channels) {
    if (!lk_) return PSN_LK_ERR_ARG;
    const int slot = ring_[kT2dInterval - 1];
    const int rc = psn_lk_push_frame_device(lk_, slot, dev, stride, channels);
    if (rc) return fail(rc, "psn_lk_push_frame_device");
    filled_[slot] = true;
    return PSN_LK_OK;
}

int Tracker2DFlow::DetectFeatures(const std::vector<Detection> &dets, uint32_t seed,
                                  std::vector<std::vector<Point2f>> &features) {
    if (!lk_) return PSN_LK_ERR_ARG;
    const size_t n = dets.size();
    features.assign(n, {});
    if (n == 0) return PSN_LK_OK;
    std::vector<int> rois(4 * n), cnt(n), tot(n);
    for (size_t i = 0; i < n; i++) {
        // cv::Rect((int)x, (int)y, (int)w, (int)h) of the cropped, scaled box
        const Rect r = dets[i].box.scale(kFlowScale).cropWithSize(width_, height_);
        rois[4 * i] = (int)r.x;
        rois[4 * i + 1] = (int)r.y;
        rois[4 * i + 2] = (int)r.w;
        rois[4 * i + 3] = (int)r.h;
    }
    psn_gridfast_params p;
    psn_gridfast_default_params(&p);
    p.cap = (int)kT2dMaxFeatures;
    gf_xy_.resize(2 * n * kT2dMaxFeatures);
    const int rc = psn_gridfast_detect(lk_, ring_[kT2dInterval - 1], rois.data(), (int)n, &p, seed, gf_xy_.data(),
                                       cnt.data(), tot.data());
    if (rc) return fail(rc, "psn_gridfast_detect");
    for (size_t i = 0; i < n; i++) {
        const float *xy = gf_xy_.data() + 2 * kT2dMaxFeatures * i;
        features[i].resize((size_t)cnt[i]);
        for (int k = 0; k < cnt[i]; k++) features[i][(size_t)k] = Point2f{xy[2 * k], xy[2 * k + 1]};
    }
    return PSN_LK_OK;
}

void Tracker2DFlow::RotateRing() { std::rotate(ring_, ring_ + 1, ring_ + kT2dInterval); }

// One launch for all jobs: points concatenated, one query per job. err is
// requested as the reference does (:781, :876): its bounds re-check can clear
// status.
int Tracker2DFlow::RunJobs(std::vector<Job> &jobs) {
    size_t n = 0;
    queries_.clear();
    for (const Job &j : jobs) {
        psn_lk_query q;
        q.prev_slot = j.prev_slot;
        q.next_slot = j.next_slot;
        q.first_pt = (int)n;
        q.num_pts = (int)j.in->size();
        psn_lk_default_params(&q.params);  // maxLevel 3, (COUNT|EPS, 30, 0.01), minEig 1e-4
        q.params.win_w = j.win_w;
        q.params.win_h = j.win_h;
        queries_.push_back(q);
        n += j.in->size();
    }
    if (queries_.empty()) return PSN_LK_OK;
    xy_in_.resize(2 * n);
    xy_out_.resize(2 * n);
    err_out_.resize(n);
    st_out_.resize(n);
    size_t o = 0;
    for (const Job &j : jobs)
        for (const Point2f &p : *j.in) {
            xy_in_[2 * o] = p.x;
            xy_in_[2 * o + 1] = p.y;
            o++;
        }
    const int rc = psn_lk_track(lk_, queries_.data(), (int)queries_.size(), xy_in_.data(), xy_out_.data(),
                                st_out_.data(), err_out_.data());
    if (rc) return fail(rc, "psn_lk_track");
    o = 0;
    for (Job &j : jobs) {
        const size_t m = j.in->size();
        j.out->resize(m);
        j.status->resize(m);
        for (size_t i = 0; i < m; i++, o++) {
            (*j.out)[i] = Point2f{xy_out_[2 * o], xy_out_[2 * o + 1]};
            (*j.status)[i] = st_out_[o];
        }
    }
    return PSN_LK_OK;
}

// ---------------------------------------------------------------------------
// Backward chain (:690-838)
// ---------------------------------------------------------------------------

void Tracker2DFlow::BackwardBegin(const std::vector<Detection> &dets,
                                  const std::vector<std::vector<Point2f>> &features, std::vector<DetectedObject> &out,
                                  std::vector<Chain> &chains) {
    out.clear();
    chains.clear();
    for (size_t i = 0; i < dets.size(); i++) {
        DetectedObject o;
        o.id = (unsigned)i;  // detectionID counts every detection past the height gate (:718)
        o.detection = dets[i];
        o.boxes.push_back(dets[i].box);
        const std::vector<Point2f> &f = features[i];
        if (f.size() < kT2dMinFeatures) continue;  // :744
        Chain c;
        c.curr.assign(f.begin(), f.begin() + std::min(f.size(), kT2dMaxFeatures));  // :753-757
        c.obj = out.size();
        c.active = true;
        out.push_back(std::move(o));
        chains.push_back(std::move(c));
    }
}

// step s tracks frame t-s+1 -> t-s; it exists while the older ring slot holds a frame
bool Tracker2DFlow::StepAvailable(int step) const {
    return step < kT2dInterval && filled_[ring_[kT2dInterval - 1 - step]];
}

void Tracker2DFlow::BackwardJobs(int step, std::vector<Chain> &chains, const std::vector<DetectedObject> &out,
                                 std::vector<Job> &jobs) {
    for (Chain &c : chains) {
        if (!c.active) continue;
        const Rect box = out[c.obj].detection.box.scale(kFlowScale);
        const int win = (int)(box.w * kWinSizeRatio);  // square window of the box width (:782)
        jobs.push_back(Job{ring_[kT2dInterval - step], ring_[kT2dInterval - 1 - step], win, win, &c.curr, &c.prev,
                           &c.status});
    }
}

void Tracker2DFlow::BackwardStepDone(std::vector<Chain> &chains, std::vector<DetectedObject> &out) {
    std::vector<size_t> inl;
    for (Chain &c : chains) {
        if (!c.active) continue;
        DetectedObject &o = out[c.obj];
        // status is ignored: every nextPts value feeds LocalSearchKLT (:787)
        const Rect newRect = LocalSearchKLT(o.detection.box.scale(kFlowScale), c.curr, c.prev, inl);
        if (inl.size() < kT2dMinFeatures) {  // :788
            c.active = false;
            continue;
        }
        o.boxes.push_back(newRect.scale(1.0 / kFlowScale));
        if (o.vecvecTrackedFeatures.empty()) {
            std::vector<Point2f> cur;
            for (size_t k : inl) cur.push_back(c.curr[k]);
            o.vecvecTrackedFeatures.push_back(cur);
        }
        std::vector<Point2f> next;
        next.reserve(inl.size());
        for (size_t k : inl) next.push_back(c.prev[k]);
        o.vecvecTrackedFeatures.push_back(next);
        c.curr.swap(next);
    }
}

void Tracker2DFlow::BackwardEnd(std::vector<Chain> &chains, std::vector<DetectedObject> &out) {
    for (Chain &c : chains)
        if (out[c.obj].vecvecTrackedFeatures.empty()) out[c.obj].vecvecTrackedFeatures.push_back(c.curr);  // :815-818
    // overlap flags (:824-835)
    for (size_t a = 0; a < out.size(); a++) {
        if (out[a].bOverlapWithOtherDetection) continue;
        for (size_t b = a + 1; b < out.size(); b++)
            if (out[a].detection.box.overlap(out[b].detection.box)) {
                out[a].bOverlapWithOtherDetection = true;
                break;
            }
    }
}

int Tracker2DFlow::BackwardFeatureTracking(const std::vector<Detection> &dets,
                                           const std::vector<std::vector<Point2f>> &features,
                                           std::vector<DetectedObject> &out) {
    if (!lk_ || features.size() != dets.size()) return PSN_LK_ERR_ARG;
    std::vector<Chain> chains;
    BackwardBegin(dets, features, out, chains);
    if (device_chain_) {
        const int rc = ChainsOnDevice(chains, out, nullptr);
        if (rc) return rc;
        BackwardEnd(chains, out);
        return PSN_LK_OK;
    }
    std::vector<Job> jobs;
    for (int step = 1; StepAvailable(step); step++) {
        jobs.clear();
        BackwardJobs(step, chains, out, jobs);
        if (jobs.empty()) break;
        int rc = RunJobs(jobs);
        if (rc) return rc;
        BackwardStepDone(chains, out);
    }
    BackwardEnd(chains, out);
    return PSN_LK_OK;
}

// ---------------------------------------------------------------------------
// Forward tracking + matching score (:851-1025)
// ---------------------------------------------------------------------------

void Tracker2DFlow::ForwardJobs(const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                                std::vector<Job> &jobs) {
    status.assign(trackers.size(), {});
    for (size_t t = 0; t < trackers.size(); t++) {
        Tracker2D *tr = trackers[t];
        tr->trackedPoints.clear();
        const Rect cur = tr->boxes.back().scale(kFlowScale);
        jobs.push_back(Job{ring_[kT2dInterval - 2], ring_[kT2dInterval - 1], (int)(cur.w * kWinSizeRatio),
                           (int)(cur.h * kWinSizeRatio), &tr->featurePoints, &tr->trackedPoints, &status[t]});
    }
}

void Tracker2DFlow::ForwardDone(const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                                const std::vector<DetectedObject> &dets, std::vector<float> &cost) {
    const double kBoxMaxDistance = 1.0, kMinOverlapRatio = 0.3, kMaxCenterDiffRatio = 0.5, kMajority = 0.5;
    const size_t T = trackers.size(), D = dets.size();
    const float inf = std::numeric_limits<float>::infinity();
    cost.assign(D * T, inf);
    std::vector<std::deque<int>> inBox(D);
    std::vector<size_t> inl;
    for (size_t t = 0; t < T; t++) {
        Tracker2D *tr = trackers[t];
        std::vector<Point2f> vPrev, vCurr;
        for (size_t i = 0; i < status[t].size(); i++) {  // keep status == 1 (:883-888)
            if (!status[t][i]) continue;
            vPrev.push_back(tr->featurePoints[i]);
            vCurr.push_back(tr->trackedPoints[i]);
        }
        if (vCurr.size() < kT2dMinFeatures) continue;  // :889 (featurePoints kept, trackedPoints = raw output)
        Rect newBox = LocalSearchKLT(tr->boxes.back().scale(kFlowScale), vPrev, vCurr, inl);
        newBox = newBox.scale(1.0 / kFlowScale);
        tr->boxes.push_back(newBox);
        tr->heads.push_back(tr->heads.empty() ? Rect() : tr->heads.back());
        for (size_t d = 0; d < D; d++) {
            const DetectedObject &det = dets[d];
            const size_t pos = d * T + t;
            if (!newBox.overlap(det.detection.box)) continue;
            for (const Point2f &p : tr->trackedPoints)  // the raw LK output (:914-918)
                if (det.detection.box.contain(p)) inBox[d].push_back((int)t);
            double boxCost = 0.0;
            const size_t len = std::min((size_t)kT2dInterval, std::min(tr->boxes.size(), det.boxes.size()));
            size_t tb = (size_t)tr->duration;  // duration = #boxes - 1
            for (size_t b = 0; b < len; b++, tb--) {
                const Rect &db = det.boxes[b], &trb = tr->boxes[tb];
                if (!db.overlap(trb) || kBoxMaxDistance < db.distance(trb) ||
                    kMinOverlapRatio > db.overlappedArea(trb) / std::min(db.area(), trb.area()) ||
                    kMaxCenterDiffRatio * std::max(db.w, trb.w) < (db.center() - trb.center()).norm_L2()) {
                    boxCost = std::numeric_limits<double>::infinity();
                    break;
                }
                boxCost += BoxMatchingCost(trb, db);
            }
            if (std::numeric_limits<double>::infinity() == boxCost) continue;
            boxCost /= (double)len;
            cost[pos] = (float)boxCost;
        }
        tr->featurePoints = vPrev;  // :977-978
        tr->trackedPoints = vCurr;
    }
    // feature-point majority check (:982-1022), run lengths as the reference counts them
    for (size_t d = 0; d < D; d++) {
        const std::deque<int> &f = inBox[d];
        if (f.empty()) continue;
        int nMajor = 0, nCur = 0;
        int major = f.front(), cur = f.front();
        for (size_t k = 0; k < f.size(); k++) {
            if (cur == f[k]) {
                nCur++;
                continue;
            }
            if (nCur > nMajor) {
                major = cur;
                nMajor = nCur;
            }
            cur = f[k];
            nCur = 0;
        }
        (void)major;
        if (f.front() == cur) nMajor = nCur;  // sole tracker
        if ((double)nMajor > (double)f.size() * kMajority) continue;
        for (size_t t = 0; t < T; t++) cost[d * T + t] = inf;
    }
}

int Tracker2DFlow::ForwardTrackingAndGetMatchingScore(const std::vector<Tracker2D *> &trackers,
                                                      const std::vector<DetectedObject> &dets,
                                                      std::vector<float> &cost) {
    if (!lk_) return PSN_LK_ERR_ARG;
    std::vector<std::vector<uint8_t>> status;
    std::vector<Job> jobs;
    if (!trackers.empty() && !StepAvailable(1)) return PSN_LK_ERR_SLOT;  // no frame t-1
    ForwardJobs(trackers, status, jobs);
    int rc = RunJobs(jobs);
    if (rc) return rc;
    ForwardDone(trackers, status, dets, cost);
    return PSN_LK_OK;
}

// GridFAST + backward chains + forward in one device pass (device chain mode):
// the forward launch goes first on its own stream; GridFAST writes every
// detection's features straight into the chain inputs (the host never sees
// them before the chains run); counts below the minimum are gated to 0 on the
// device; one sync at the end. Results are those of DetectFeatures +
// TrackFrame.
int Tracker2DFlow::TrackFrameDetect(const std::vector<Detection> &dets, uint32_t seed,
                                    std::vector<std::vector<Point2f>> &features, std::vector<DetectedObject> &out,
                                    const std::vector<Tracker2D *> &trackers, std::vector<float> &cost) {
    if (!lk_) return PSN_LK_ERR_ARG;
    if (!device_chain_) {
        const int rc = DetectFeatures(dets, seed, features);
        return rc ? rc : TrackFrame(dets, features, out, trackers, cost);
    }
    if (!trackers.empty() && !StepAvailable(1)) return PSN_LK_ERR_SLOT;
    const size_t K = dets.size(), cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS;
    std::vector<std::vector<uint8_t>> fstatus;
    std::vector<Job> fwd;
    ForwardJobs(trackers, fstatus, fwd);
    const size_t J = fwd.size();
    size_t F = 0;
    for (const Job &jb : fwd) F += jb.in->size();
    int rc = EnsureDevice(K, F, J);
    if (rc) return rc;
    DeviceBuffers &b = *dev_;
    hipStream_t st = (hipStream_t)psn_lk_get_stream(lk_), fs = (hipStream_t)fwd_stream_;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            err_ = std::string(what) + ": " + hipGetErrorString(e);
            rc = PSN_LK_ERR_HIP;
        }
    };
    // 1. the forward calls, first, on the forward stream (after frame t's ingest)
    if (J) {
        size_t o = K * cap;
        fwd_queries_.clear();
        for (size_t j = 0; j < J; j++) {
            const std::vector<Point2f> &pts = *fwd[j].in;
            psn_lk_query q;
            q.prev_slot = fwd[j].prev_slot;
            q.next_slot = fwd[j].next_slot;
            q.first_pt = (int)o;
            q.num_pts = (int)pts.size();
            psn_lk_default_params(&q.params);
            q.params.win_w = fwd[j].win_w;
            q.params.win_h = fwd[j].win_h;
            fwd_queries_.push_back(q);
            for (size_t i = 0; i < pts.size(); i++, o++) {
                b.h_in[2 * o] = pts[i].x;
                b.h_in[2 * o + 1] = pts[i].y;
            }
            b.h_cnt[K + j] = (int)pts.size();
        }
        chk(hipEventRecord((hipEvent_t)ev_in_, st), "ingest event");
        chk(hipStreamWaitEvent(fs, (hipEvent_t)ev_in_, 0), "forward wait");
        chk(hipMemcpyAsync(b.d_in + 2 * K * cap, b.h_in + 2 * K * cap, F * 8, hipMemcpyHostToDevice, fs), "forward inputs");
        chk(hipMemcpyAsync(b.d_cnt + K, b.h_cnt + K, J * 4, hipMemcpyHostToDevice, fs), "forward counts");
        if (rc) return rc;
        rc = psn_lk_set_stream(lk_, fs);
        if (!rc)
            rc = psn_lk_track_device_counted(lk_, fwd_queries_.data(), (int)J, b.d_cnt + K, b.d_in, b.d_out, b.d_status,
                                             b.d_err);
        const int rs = psn_lk_set_stream(lk_, st);
        if (rc || rs) return fail(rc ? rc : rs, "forward launch");
        if (F) {
            chk(hipMemcpyAsync(b.h_fwd_out, b.d_out + 2 * K * cap, F * 8, hipMemcpyDeviceToHost, fs), "forward points");
            chk(hipMemcpyAsync(b.h_fwd_st, b.d_status + K * cap, F, hipMemcpyDeviceToHost, fs), "forward status");
        }
    }
    // 2. GridFAST of every detection into the chain inputs, then the chains
    if (K) {
        std::vector<int> rois(4 * K);
        for (size_t i = 0; i < K; i++) {
            const Rect r = dets[i].box.scale(kFlowScale).cropWithSize(width_, height_);
            rois[4 * i] = (int)r.x;
            rois[4 * i + 1] = (int)r.y;
            rois[4 * i + 2] = (int)r.w;
            rois[4 * i + 3] = (int)r.h;
            const Rect box = dets[i].box.scale(kFlowScale);
            b.h_boxes[4 * i] = box.x;
            b.h_boxes[4 * i + 1] = box.y;
            b.h_boxes[4 * i + 2] = box.w;
            b.h_boxes[4 * i + 3] = box.h;
        }
        psn_gridfast_params p;
        psn_gridfast_default_params(&p);
        p.cap = (int)cap;  // kT2dMaxFeatures
        rc = psn_gridfast_detect_device(lk_, ring_[kT2dInterval - 1], rois.data(), (int)K, &p, seed, b.d_in, b.d_cnt,
                                        b.d_tot);
        if (rc) return fail(rc, "psn_gridfast_detect_device");
        chk(hipMemcpyAsync(b.h_rawcnt, b.d_cnt, K * 4, hipMemcpyDeviceToHost, st), "feature counts");
        chk(hipMemcpyAsync(b.h_in, b.d_in, K * cap * 8, hipMemcpyDeviceToHost, st), "features");
        if (!rc) rc = psn_t2d_gate_counts_device(b.d_cnt, (int)K, (int)kT2dMinFeatures, st);
        chk(hipMemcpyAsync(b.d_boxes, b.h_boxes, K * 32, hipMemcpyHostToDevice, st), "chain boxes");
        chk(hipMemsetAsync(b.d_nsteps, 0, b.nchains * (1 + S) * 4, st), "chain steps and set counts");
        if (rc) return rc;
        psn_t2d_chain_dev cd{};
        cd.ndet = (int)K;
        cd.cap = (int)cap;
        cd.boxes = b.d_boxes;
        cd.cnt = b.d_cnt;
        cd.out_boxes = b.d_obox;
        cd.sets = b.d_sets;
        cd.set_cnt = b.d_setcnt;
        cd.nsteps = b.d_nsteps;
        for (int step = 1; step < (int)S && StepAvailable(step); step++) {
            queries_.clear();
            for (size_t k = 0; k < K; k++) {
                psn_lk_query q;
                q.prev_slot = ring_[kT2dInterval - step];
                q.next_slot = ring_[kT2dInterval - 1 - step];
                q.first_pt = (int)(k * cap);
                q.num_pts = (int)cap;
                psn_lk_default_params(&q.params);
                q.params.win_w = q.params.win_h = (int)(b.h_boxes[4 * k + 2] * kWinSizeRatio);
                queries_.push_back(q);
            }
            const float *in = step == 1 ? b.d_in : b.d_buf[step & 1];
            rc = psn_lk_track_device_counted(lk_, queries_.data(), (int)K, b.d_cnt, in, b.d_out, b.d_status, b.d_err);
            if (rc) return fail(rc, "psn_lk_track_device_counted");
            cd.cur = in;
            cd.nxt = b.d_out;
            cd.next_in = b.d_buf[(step + 1) & 1];
            rc = psn_t2d_chain_step_device(&cd, step, st);
            if (rc) return fail(rc, "psn_t2d_chain_step_device");
        }
        chk(hipMemcpyAsync(b.h_res, b.d_res, b.res_sets_off + K * S * cap * 8, hipMemcpyDeviceToHost, st), "chain results");
    }
    chk(hipStreamSynchronize(st), "chain sync");
    chk(hipStreamSynchronize(fs), "forward sync");
    if (rc) return rc;
    // 3. host: features, the valid detections' objects and chains, forward matching
    features.assign(K, {});
    for (size_t i = 0; i < K; i++) {
        const int n = b.h_rawcnt[i];
        const float *xy = b.h_in + 2 * cap * i;
        features[i].resize((size_t)n);
        for (int k = 0; k < n; k++) features[i][(size_t)k] = Point2f{xy[2 * k], xy[2 * k + 1]};
    }
    std::vector<Chain> chains;
    BackwardBegin(dets, features, out, chains);  // valid detections, in order
    for (Chain &c : chains) {
        DetectedObject &ob = out[c.obj];
        const size_t k = ob.id;  // the detection index = its device chain
        const int ns = b.h_nsteps[k];
        for (int s2 = 1; s2 <= ns; s2++) {
            const double *r = b.h_obox + (k * S + s2) * 4;
            ob.boxes.push_back(Rect(r[0], r[1], r[2], r[3]).scale(1.0 / kFlowScale));
        }
        for (int r = 0; ns > 0 && r <= ns; r++) {
            const int n = b.h_setcnt[k * S + r];
            const float *pp = b.h_sets + (k * S + r) * cap * 2;
            std::vector<Point2f> v((size_t)n);
            for (int i = 0; i < n; i++) v[(size_t)i] = Point2f{pp[2 * i], pp[2 * i + 1]};
            ob.vecvecTrackedFeatures.push_back(std::move(v));
        }
        c.active = false;
    }
    for (size_t j = 0, off = 0; j < J; j++) {
        Job &jb = fwd[j];
        const size_t m = jb.in->size();
        jb.out->resize(m);
        jb.status->resize(m);
        for (size_t i = 0; i < m; i++, off++) {
            (*jb.out)[i] = Point2f{b.h_fwd_out[2 * off], b.h_fwd_out[2 * off + 1]};
            (*jb.status)[i] = b.h_fwd_st[off];
        }
    }
    BackwardEnd(chains, out);
    ForwardDone(trackers, fstatus, out, cost);
    return PSN_LK_OK;
}

int Tracker2DFlow::TrackFrame(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                              std::vector<DetectedObject> &out, const std::vector<Tracker2D *> &trackers,
                              std::vector<float> &cost) {
    if (!lk_ || features.size() != dets.size()) return PSN_LK_ERR_ARG;
    if (!trackers.empty() && !StepAvailable(1)) return PSN_LK_ERR_SLOT;
    std::vector<Chain> chains;
    BackwardBegin(dets, features, out, chains);
    std::vector<std::vector<uint8_t>> fstatus;
    std::vector<Job> jobs;
    if (device_chain_) {
        ForwardJobs(trackers, fstatus, jobs);
        const int rc = ChainsOnDevice(chains, out, &jobs);
        if (rc) return rc;
        BackwardEnd(chains, out);
        ForwardDone(trackers, fstatus, out, cost);
        return PSN_LK_OK;
    }
    // launch 1: backward step 1 of every detection + every forward call
    if (StepAvailable(1)) BackwardJobs(1, chains, out, jobs);
    const size_t nb = jobs.size();
    ForwardJobs(trackers, fstatus, jobs);
    int rc = RunJobs(jobs);
    if (rc) return rc;
    if (nb) BackwardStepDone(chains, out);
    for (int step = 2; nb && StepAvailable(step); step++) {
        jobs.clear();
        BackwardJobs(step, chains, out, jobs);
        if (jobs.empty()) break;
        rc = RunJobs(jobs);
        if (rc) return rc;
        BackwardStepDone(chains, out);
    }
    BackwardEnd(chains, out);
    ForwardDone(trackers, fstatus, out, cost);
    return PSN_LK_OK;
}

}  // namespace psn
