// Tracker2D flow stage (see tracker2d_flow.hpp). Reference lines cited are in
// psn_where/PSNWhere_Tracker2D.cpp unless noted.
#include "tracker2d_flow.hpp"

#include <hip/hip_runtime_api.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
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
    // neighbour counts |v[d] - v[c]| < windowSize of every d. On sorted finite
    // values with windowSize > 0 the neighbours of d are one index range [lo, hi)
    // whose ends never decrease with d (fl(a - b) is monotone in a and b, and
    // |fl(a - b)| = fl(b - a)), so two pointers count exactly what the reference's
    // double loop counts; otherwise (NaN, windowSize <= 0) that loop itself.
    const bool finite = windowSize > 0 &&
                        std::all_of(vecDx.begin(), vecDx.end(), [](double v) { return std::isfinite(v); }) &&
                        std::all_of(vecDy.begin(), vecDy.end(), [](double v) { return std::isfinite(v); });
    auto counts = [&](const std::vector<double> &v, std::vector<size_t> &cnt) {
        cnt.assign(numMoving, 0);
        if (finite) {
            size_t lo = 0, hi = 0;
            for (size_t d = 0; d < numMoving; d++) {
                while (!(v[d] - v[lo] < windowSize)) lo++;  // lo <= d: v[d] - v[d] = 0 < windowSize
                if (hi < d + 1) hi = d + 1;
                while (hi < numMoving && v[hi] - v[d] < windowSize) hi++;
                cnt[d] = hi - lo;
            }
        } else {
            for (size_t d = 0; d < numMoving; d++)
                for (size_t c = 0; c < numMoving; c++)
                    if (std::abs(v[d] - v[c]) < windowSize) cnt[d]++;
        }
    };
    std::vector<size_t> cntX, cntY;
    counts(vecDx, cntX);
    counts(vecDy, cntY);
    for (size_t d = 0; d < numMoving; d++) {
        if (maxX < cntX[d]) {
            est.x = vecDx[d];
            maxX = cntX[d];
        }
        if (maxY < cntY[d]) {
            est.y = vecDy[d];
            maxY = cntY[d];
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
    return InitializeCameras(std::vector<unsigned>{camID}, width, height, device);
}

int Tracker2DFlow::InitializeCameras(const std::vector<unsigned> &camIDs, int width, int height, int device) {
    Finalize();
    if (camIDs.empty() || width <= 0 || height <= 0) return PSN_LK_ERR_ARG;
    width_ = width;
    height_ = height;
    const int nslots = (int)camIDs.size() * kSlotsPerCam;
    // full pyramids of every camera's slots; the reference's default maxLevel 3 needs 4 levels
    const int rc = psn_lk_create(device, width, height, nslots, 3, &lk_);
    if (rc) {
        lk_ = nullptr;
        err_ = "psn_lk_create failed (" + std::to_string(rc) + ")";
        return rc;
    }
    cams_.assign(camIDs.size(), Cam());
    for (size_t c = 0; c < camIDs.size(); c++) {
        cams_[c].camID = camIDs[c];
        for (int i = 0; i < kT2dInterval; i++) cams_[c].ring[i] = (int)c * kSlotsPerCam + i;
        for (int i = 0; i < kT2dStaging; i++) cams_[c].spares[i] = (int)c * kSlotsPerCam + kT2dInterval + i;
        cams_[c].nstaged = 0;
    }
    filled_.assign((size_t)nslots, 0);
    // stream priorities: the backward chains (three dependent launches per frame)
    // are the frame's critical path; the forward calls fill the compute units they
    // leave free instead of taking half of them (the device dispatches waiting
    // workgroups of higher-priority queues first)
    int least = 0, greatest = 0;
    hipStream_t fs = nullptr, cs = nullptr;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&fs, hipStreamNonBlocking, least) != hipSuccess) {
        err_ = "forward stream";
        return PSN_LK_ERR_HIP;
    }
    fwd_stream_ = fs;
    if (hipStreamCreateWithPriority(&fs, hipStreamNonBlocking, least) != hipSuccess) {
        err_ = "forward stream";
        return PSN_LK_ERR_HIP;
    }
    fwd_stream2_ = fs;
    for (int i = 0; i < 2; i++) {
        if (hipStreamCreateWithPriority(&cs, hipStreamNonBlocking, greatest) != hipSuccess) {
            err_ = "chain stream";
            return PSN_LK_ERR_HIP;
        }
        chain_streams_[i] = cs;
    }
    cs = (hipStream_t)chain_streams_[0];
    hipEvent_t e1 = nullptr, e2 = nullptr;
    if (hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e2, hipEventDisableTiming) != hipSuccess) {
        err_ = "result events";
        return PSN_LK_ERR_HIP;
    }
    ev_chain_ = e1;
    ev_fwd_ = e2;
    hipEvent_t e3 = nullptr;
    if (hipEventCreateWithFlags(&e3, hipEventDisableTiming) != hipSuccess) {
        err_ = "gridfast event";
        return PSN_LK_ERR_HIP;
    }
    ev_gf_ = e3;
    gf_rec_ = false;
    for (int p = 0; p < 2; p++) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
            err_ = "forward block events";
            return PSN_LK_ERR_HIP;
        }
        ev_fend_[p] = a;
        ev_fcopied_[p] = b;
    }
    fwd_par_ = 0;
    for (int r = 0; r < kT2dResBlocks; r++) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
            err_ = "result block events";
            return PSN_LK_ERR_HIP;
        }
        ev_set0_[r] = a;
        ev_fread_[r] = b;
        fread_rec_[r] = false;
        chain_info_[r] = ChainInfo();
    }
    next_rb_ = 0;
    last_rb_ = -1;
    trk_rb_ = -1;
    return psn_lk_set_stream(lk_, cs);
}

// Device and pinned-host buffers of a device pass (grown on demand). The
// backward chains and the forward calls have separate arrays: a frame's chains
// may run (launched ahead, RunComplete with a next frame) while its forward
// inputs are staged and, if need be, its forward buffers regrown.
struct Tracker2DFlow::DeviceBuffers {
    size_t nchains = 0, nfwd_pts = 0, nfwd_jobs = 0;
    // chains: inputs, LK outputs, ping-pong point sets, err/status
    // per staging set (a pass and its chain stream): inputs, LK outputs, ping-pong
    // point sets, err/status -- consecutive passes run on the two chain streams at once
    struct Scratch {
        char *d_inblk = nullptr;
        float *d_in = nullptr, *d_out = nullptr, *d_buf[2] = {nullptr, nullptr}, *d_err = nullptr;
        uint8_t *d_status = nullptr;
        double *d_boxes = nullptr;
        int *d_cnt = nullptr, *d_tot = nullptr, *d_last = nullptr;
    } sc[2];
    // forward calls: inputs [counts | (256-B aligned) points], outputs [status | (aligned) points] (one copy each)
    float *d_fin = nullptr, *d_fout[2] = {nullptr, nullptr}, *d_ferr[2] = {nullptr, nullptr};
    uint8_t *d_fstatus[2] = {nullptr, nullptr};
    int *d_fcnt = nullptr;
    char *d_fiblk = nullptr, *d_foblk[2] = {nullptr, nullptr}, *h_fiblk = nullptr, *h_foblk = nullptr;
    size_t fi_off_pts = 0, fo_off_pts = 0;
    // pinned staging of the chain inputs (and GridFAST features), two sets: a
    // pass's set is written by its launch and read back by its completion, and
    // the next frame's chains may be launched in between (RunComplete with next)
    // [boxes f64 x4 | last steps | counts | (256-B aligned) points] per chain, one block per
    // side so that one copy carries a pass's inputs (carve_in)
    struct Stage {
        char *h_inblk = nullptr;
        float *h_in = nullptr;
        double *h_boxes = nullptr;
        int *h_cnt = nullptr, *h_rawcnt = nullptr, *h_last = nullptr;
    } stage[2];
    size_t in_off_last = 0, in_off_cnt = 0, in_off_in = 0, in_bytes = 0;
    void layout_in(size_t K, size_t cap) {
        in_off_last = K * 32;
        in_off_cnt = in_off_last + K * 4;
        in_off_in = (in_off_cnt + K * 4 + 255) & ~(size_t)255;
        in_bytes = in_off_in + K * cap * 8;
    }
    void carve_in(char *base, double *&boxes, int *&last, int *&cnt, float *&in) const {
        boxes = (double *)base;
        last = (int *)(base + in_off_last);
        cnt = (int *)(base + in_off_cnt);
        in = (float *)(base + in_off_in);
    }
    // pinned staging: forward inputs, then results
    float *h_fin = nullptr, *h_fwd_out = nullptr;
    uint8_t *h_fwd_st = nullptr;
    int *h_fcnt = nullptr;
    // the chain's results live in one block per side, [nsteps | set counts | boxes | sets], so that
    // one memset clears the counters and one copy returns every used byte
    // Three result blocks, used by consecutive passes in turn: a pass's block is
    // read by the next frame's forward launch (its set 0: the trackers' features)
    // while the chains of the frame after write theirs.
    static constexpr int kResBlocks = kT2dResBlocks;
    char *d_res[kResBlocks] = {}, *h_res[kResBlocks] = {};
    size_t res_sets_off = 0;
    struct ResView {
        int *nsteps, *setcnt;
        double *obox;
        float *sets;
    };
    ResView view(char *base) const {
        ResView v{};
        carve(base, v.obox, v.sets, v.setcnt, v.nsteps, nchains, PSN_T2D_CHAIN_STEPS);
        return v;
    }
    void carve(char *base, double *&obox, float *&sets, int *&setcnt, int *&nsteps, size_t K, size_t S) const {
        nsteps = (int *)base;
        setcnt = nsteps + K;
        obox = (double *)(base + res_box_off(K, S));
        sets = (float *)(base + res_sets_off);
    }
    static size_t res_box_off(size_t K, size_t S) { return (K * (1 + S) * 4 + 255) & ~(size_t)255; }
    static void free_all(std::initializer_list<void *> dev, std::initializer_list<void *> host) {
        for (void *p : dev)
            if (p) (void)hipFree(p);
        for (void *p : host)
            if (p) (void)hipHostFree(p);
    }
    void release_chains() {
        free_all({d_res[0], d_res[1], d_res[2]}, {h_res[0], h_res[1], h_res[2]});
        for (Scratch &x : sc) {
            free_all({x.d_inblk, x.d_out, x.d_buf[0], x.d_buf[1], x.d_err, x.d_status, x.d_tot}, {});
            x = Scratch();
        }
        for (Stage &g : stage) {
            free_all({}, {g.h_inblk, g.h_rawcnt});
            g = Stage();
        }
        for (int r = 0; r < kResBlocks; r++) d_res[r] = h_res[r] = nullptr;
        nchains = 0;
    }
    void release_forward() {
        free_all({d_fiblk, d_foblk[0], d_foblk[1], d_ferr[0], d_ferr[1]}, {h_fiblk, h_foblk});
        d_fiblk = d_foblk[0] = d_foblk[1] = h_fiblk = h_foblk = nullptr;
        d_fin = d_fout[0] = d_fout[1] = d_ferr[0] = d_ferr[1] = nullptr;
        d_fstatus[0] = d_fstatus[1] = nullptr;
        d_fcnt = nullptr;
        h_fin = h_fwd_out = nullptr;
        h_fwd_st = nullptr;
        h_fcnt = nullptr;
        nfwd_pts = nfwd_jobs = 0;
    }
    void release() {
        release_chains();
        release_forward();
    }
};

void Tracker2DFlow::SyncChains() {
    for (void *cs : chain_streams_)
        if (cs) (void)hipStreamSynchronize((hipStream_t)cs);
}

void Tracker2DFlow::SyncForward() {
    for (void *fs : {fwd_stream_, fwd_stream2_})
        if (fs) (void)hipStreamSynchronize((hipStream_t)fs);
}

void Tracker2DFlow::Finalize() {
    if (dev_) {
        // every stream that may still use the device buffers: the LK context's,
        // both chain streams (a frame launched ahead runs on the other one) and
        // both forward streams
        if (lk_) psn_lk_sync(lk_);
        SyncChains();
        SyncForward();
        dev_->release();
        delete dev_;
        dev_ = nullptr;
    }
    for (void **fs : {&fwd_stream_, &fwd_stream2_})
        if (*fs) {
            (void)hipStreamSynchronize((hipStream_t)*fs);
            (void)hipStreamDestroy((hipStream_t)*fs);
            *fs = nullptr;
        }
    if (lk_) psn_lk_destroy(lk_);
    lk_ = nullptr;
    for (void *&cs : chain_streams_)
        if (cs) {
            (void)hipStreamSynchronize((hipStream_t)cs);
            (void)hipStreamDestroy((hipStream_t)cs);
            cs = nullptr;
        }
    for (void **e : {&ev_chain_, &ev_fwd_, &ev_gf_, &ev_set0_[0], &ev_set0_[1], &ev_set0_[2], &ev_fread_[0], &ev_fread_[1],
                     &ev_fread_[2], &ev_fend_[0], &ev_fend_[1], &ev_fcopied_[0], &ev_fcopied_[1]})
        if (*e) {
            (void)hipEventDestroy((hipEvent_t)*e);
            *e = nullptr;
        }
    wait_chain_ = wait_fwd_ = false;
    cams_.clear();
}

// Buffer capacities grow geometrically (powers of two from `floor`): a regrow
// drains the streams and reallocates pinned memory (milliseconds), so a
// tracker population that creeps up frame by frame regrows O(log n) times.
static size_t grow_cap(size_t need, size_t floor) {
    size_t c = floor;
    while (c < need) c *= 2;
    return c;
}

// Chain buffers for nchains detections: grown only between passes (no chain in
// flight on the chain stream).
int Tracker2DFlow::EnsureChains(size_t nchains) {
    if (!dev_) dev_ = new DeviceBuffers();
    DeviceBuffers &b = *dev_;
    if (b.nchains >= nchains && b.sc[0].d_in) return PSN_LK_OK;
    if (lk_) psn_lk_sync(lk_);
    SyncChains();
    // a forward launch may still read a result block's set 0
    SyncForward();
    b.release_chains();
    for (int r = 0; r < DeviceBuffers::kResBlocks; r++) {
        chain_info_[r].valid = false;
        fread_rec_[r] = false;
    }
    const size_t K = grow_cap(nchains, 16);
    const size_t cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS, npt = K * cap;
    bool ok = true;
    auto dm = [&](void **p, size_t bytes) { ok = ok && hipMalloc(p, bytes) == hipSuccess; };
    auto hm = [&](void **p, size_t bytes) { ok = ok && hipHostMalloc(p, bytes, hipHostMallocCoherent) == hipSuccess; };
    b.layout_in(K, cap);
    for (DeviceBuffers::Scratch &x : b.sc) {
        dm((void **)&x.d_inblk, b.in_bytes);
        dm((void **)&x.d_out, npt * 8);
        dm((void **)&x.d_buf[0], npt * 8);
        dm((void **)&x.d_buf[1], npt * 8);
        dm((void **)&x.d_err, npt * 4);
        dm((void **)&x.d_status, npt);
        dm((void **)&x.d_tot, K * 4);
    }
    b.res_sets_off = DeviceBuffers::res_box_off(K, S) + K * S * 4 * 8;
    const size_t res_bytes = b.res_sets_off + K * S * cap * 8;
    for (int r = 0; r < DeviceBuffers::kResBlocks; r++) dm((void **)&b.d_res[r], res_bytes);
    for (int r = 0; r < DeviceBuffers::kResBlocks; r++) hm((void **)&b.h_res[r], res_bytes);
    for (DeviceBuffers::Stage &g : b.stage) {
        hm((void **)&g.h_inblk, b.in_bytes);
        hm((void **)&g.h_rawcnt, K * 4);
    }
    if (!ok) {
        b.release_chains();
        err_ = "chain buffers: allocation failed";
        return PSN_LK_ERR_NOMEM;
    }
    for (DeviceBuffers::Scratch &x : b.sc) b.carve_in(x.d_inblk, x.d_boxes, x.d_last, x.d_cnt, x.d_in);
    for (DeviceBuffers::Stage &g : b.stage) b.carve_in(g.h_inblk, g.h_boxes, g.h_last, g.h_cnt, g.h_in);
    b.nchains = K;
    return PSN_LK_OK;
}

// Forward buffers for nfwd_pts points in nfwd_jobs calls: the forward stream is
// the only device user, so growing them never waits for a chain in flight.
int Tracker2DFlow::EnsureForward(size_t nfwd_pts, size_t nfwd_jobs) {
    if (!dev_) dev_ = new DeviceBuffers();
    DeviceBuffers &b = *dev_;
    if (b.nfwd_pts >= nfwd_pts && b.nfwd_jobs >= nfwd_jobs && b.d_fin) return PSN_LK_OK;
    SyncForward();
    SyncChains();  // result copies of the forward blocks run on the chain streams
    // results of a pass not unpacked yet (its copy was enqueued) move to the new buffers
    std::vector<uint8_t> keep_st;
    std::vector<float> keep_pts;
    if (b.h_foblk) {
        keep_st.assign(b.h_fwd_st, b.h_fwd_st + b.nfwd_pts);
        keep_pts.assign(b.h_fwd_out, b.h_fwd_out + 2 * b.nfwd_pts);
    }
    b.release_forward();
    const size_t F = grow_cap(nfwd_pts, 1024), J = grow_cap(nfwd_jobs, 16);
    bool ok = true;
    auto dm = [&](void **p, size_t bytes) { ok = ok && hipMalloc(p, bytes) == hipSuccess; };
    auto hm = [&](void **p, size_t bytes) { ok = ok && hipHostMalloc(p, bytes, hipHostMallocCoherent) == hipSuccess; };
    b.fi_off_pts = (J * 4 + 255) & ~(size_t)255;
    b.fo_off_pts = (F + 255) & ~(size_t)255;
    dm((void **)&b.d_fiblk, b.fi_off_pts + F * 8);
    dm((void **)&b.d_foblk[0], b.fo_off_pts + F * 8);
    dm((void **)&b.d_foblk[1], b.fo_off_pts + F * 8);
    dm((void **)&b.d_ferr[0], F * 4);
    dm((void **)&b.d_ferr[1], F * 4);
    hm((void **)&b.h_fiblk, b.fi_off_pts + F * 8);
    hm((void **)&b.h_foblk, b.fo_off_pts + F * 8);
    if (!ok) {
        b.release_forward();
        err_ = "forward buffers: allocation failed";
        return PSN_LK_ERR_NOMEM;
    }
    b.d_fcnt = (int *)b.d_fiblk;
    b.d_fin = (float *)(b.d_fiblk + b.fi_off_pts);
    b.h_fcnt = (int *)b.h_fiblk;
    b.h_fin = (float *)(b.h_fiblk + b.fi_off_pts);
    for (int p = 0; p < 2; p++) {
        b.d_fstatus[p] = (uint8_t *)b.d_foblk[p];
        b.d_fout[p] = (float *)(b.d_foblk[p] + b.fo_off_pts);
    }
    b.h_fwd_st = (uint8_t *)b.h_foblk;
    b.h_fwd_out = (float *)(b.h_foblk + b.fo_off_pts);
    if (!keep_st.empty()) {
        std::memcpy(b.h_fwd_st, keep_st.data(), keep_st.size());
        std::memcpy(b.h_fwd_out, keep_pts.data(), keep_pts.size() * sizeof(float));
    }
    b.nfwd_pts = F;
    b.nfwd_jobs = J;
    return PSN_LK_OK;
}

// Error of a chain whose square window (box width, :782) the LK cannot run:
// CV_Assert(winSize > 2) in the reference, or outside the LK's window limits
// (psn_lk_window_supported: the same predicate psn_lk_track applies).
static int window_error(int win) {
    if (win <= 2) return PSN_LK_ERR_WINSIZE;
    if (!psn_lk_window_supported(win, win)) return PSN_LK_ERR_UNSUPPORTED;
    return PSN_LK_OK;
}

// The same for a forward call's box window (:877).
int Tracker2DFlow::forward_window_error(int w, int h) {
    if (w <= 2 || h <= 2) return PSN_LK_ERR_WINSIZE;
    if (!psn_lk_window_supported(w, h)) return PSN_LK_ERR_UNSUPPORTED;
    return PSN_LK_OK;
}

// Enqueue one device pass over the cameras in pc (everything asynchronous, one
// host sync in PassComplete):
//   1. each detection's features at t: given (host points) or GridFAST on the
//      device straight into the chain inputs (:734-757), detections below the
//      feature minimum (:744) gated to count 0 on the device;
//   2. the backward chains (:763-811): per step ONE counted LK launch over every
//      detection of every camera (capacity PSN_T2D_CHAIN_CAP points each; a
//      stopped chain's count is 0, its workgroups exit at once) and one
//      LocalSearchKLT + inlier-compaction kernel writing the next step's points
//      and counts. A camera whose ring holds fewer past frames ends its chains
//      earlier (per-chain last step); its queries in later steps are empty.
//      The chain stream has the highest priority: its launches are the frame's
//      critical path;
//   3. the forward calls of every camera's trackers (:871-877): one counted LK
//      launch on the (lowest-priority) forward stream, enqueued after the chain
//      so that the chain's first kernels are dispatched before it.
// The device-to-host copies of the results are enqueued by PassComplete: a copy
// waiting for the pass would hold up, on the copy engine, the uploads of the
// next frames (StageFrame) that the caller enqueues in between.
int Tracker2DFlow::PassLaunch(std::vector<PassCam> &pc, bool gridfast, uint32_t seed) {
    const int rc = PassLaunchChains(pc, gridfast, seed);
    return rc ? rc : PassLaunchForward(pc);
}

// 1-2 of the pass: features and the backward chains, on the chain stream.
int Tracker2DFlow::PassLaunchChains(std::vector<PassCam> &pc, bool gridfast, uint32_t seed) {
    const size_t cap = PSN_T2D_CHAIN_CAP;
    size_t K = 0;
    for (PassCam &p : pc) {
        p.k0 = K;
        K += p.dets->size();
    }
    const int si = stage_;  // this pass's staging set
    stage_ ^= 1;
    // this pass's result block: neither the previous pass's (in flight) nor the
    // one the current trackers' set 0 lives in (their next forward call reads it
    // when a frame fails)
    int rb = next_rb_;
    while (rb == last_rb_ || rb == trk_rb_) rb = (rb + 1) % DeviceBuffers::kResBlocks;
    next_rb_ = (rb + 1) % DeviceBuffers::kResBlocks;
    last_rb_ = rb;
    for (PassCam &p : pc) {
        p.set = si;
        p.rb = rb;
    }
    std::vector<char> &win_bad_ = win_bad_sets_[si];
    win_bad_.assign(K, 0);
    // what the next frame's forward launch reads of this pass: per detection the
    // forward window of its box (the tracker it becomes keeps the box, :1087)
    ChainInfo &ci = chain_info_[rb];
    ci.K = K;
    ci.valid = false;
    ci.k0.assign(cams_.size(), 0);
    ci.ndet.assign(cams_.size(), 0);
    ci.win.assign(K, {0, 0});
    for (PassCam &p : pc) {
        ci.k0[p.cam] = p.k0;
        ci.ndet[p.cam] = p.dets->size();
        for (size_t i = 0; i < p.dets->size(); i++) {
            const Rect box = (*p.dets)[i].box.scale(kFlowScale);
            ci.win[p.k0 + i] = {(int)(box.w * kWinSizeRatio), (int)(box.h * kWinSizeRatio)};
        }
    }
    if (K == 0) {
        ci.valid = true;
        return PSN_LK_OK;
    }
    int rc = EnsureChains(K);
    if (rc) return rc;
    DeviceBuffers::Stage &b = dev_->stage[si];
    DeviceBuffers &dall = *dev_;
    DeviceBuffers::Scratch &db = dall.sc[si];
    // the pass's chain stream (consecutive passes alternate: frame t+1's chains run
    // beside frame t's tail); every LK launch of the pass goes to it
    hipStream_t st = (hipStream_t)ChainStream(si);
    rc = psn_lk_set_stream(lk_, st);
    if (rc) return fail(rc, "chain stream");
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            err_ = std::string(what) + ": " + hipGetErrorString(e);
            rc = PSN_LK_ERR_HIP;
        }
    };
    {
        int max_steps = 0;
        for (PassCam &p : pc) {
            const int steps = StepsAvailable(p.cam);
            for (size_t i = 0; i < p.dets->size(); i++) {
                const size_t k = p.k0 + i;
                const Rect box = (*p.dets)[i].box.scale(kFlowScale);
                b.h_boxes[4 * k] = box.x;
                b.h_boxes[4 * k + 1] = box.y;
                b.h_boxes[4 * k + 2] = box.w;
                b.h_boxes[4 * k + 3] = box.h;
                win_bad_[k] = window_error((int)(box.w * kWinSizeRatio)) != 0;
                b.h_last[k] = win_bad_[k] ? 0 : steps;
                if (!win_bad_[k]) max_steps = std::max(max_steps, steps);
            }
        }
        if (gridfast) {
            psn_gridfast_params gp;
            psn_gridfast_default_params(&gp);
            gp.cap = (int)cap;  // kT2dMaxFeatures
            std::vector<int> rois(4 * K), slots, nrois;
            // the detector's cell scratch lives in the LK context: the previous
            // pass's detections (on the other chain stream) are done with it first
            if (gf_rec_) chk(hipStreamWaitEvent(st, (hipEvent_t)ev_gf_, 0), "gridfast scratch");
            // every camera's detections in one detector launch (per camera in the
            // reference: sets of rois at consecutive k, outputs at p.k0)
            for (PassCam &p : pc) {
                const size_t n = p.dets->size();
                if (!n) continue;
                slots.push_back(cams_[p.cam].ring[kT2dInterval - 1]);
                nrois.push_back((int)n);
                for (size_t i = 0; i < n; i++) {
                    // cv::Rect((int)x, (int)y, (int)w, (int)h) of the cropped, scaled box
                    const Rect r = (*p.dets)[i].box.scale(kFlowScale).cropWithSize(width_, height_);
                    const size_t k = p.k0 + i;
                    rois[4 * k] = (int)r.x;
                    rois[4 * k + 1] = (int)r.y;
                    rois[4 * k + 2] = (int)r.w;
                    rois[4 * k + 3] = (int)r.h;
                }
            }
            rc = psn_gridfast_detect_device_sets(lk_, (int)slots.size(), slots.data(), nrois.data(), rois.data(), &gp,
                                                 seed, db.d_in, db.d_cnt, db.d_tot);
            if (rc) return fail(rc, "psn_gridfast_detect_device_sets");
            chk(hipEventRecord((hipEvent_t)ev_gf_, st), "gridfast event");
            gf_rec_ = !rc;
            if (!rc && ((rc = psn_t2d_download_device(b.h_rawcnt, db.d_cnt, K * 4, st)) ||
                        (rc = psn_t2d_download_device(b.h_in, db.d_in, K * cap * 8, st))))
                err_ = "features download";
            // boxes and last steps (GridFAST wrote the counts and points on the device)
            if (!rc && (rc = psn_t2d_upload_device(db.d_inblk, b.h_inblk, dall.in_off_cnt, st)))
                err_ = "chain boxes upload";
        } else {
            for (PassCam &p : pc)
                for (size_t i = 0; i < p.dets->size(); i++) {
                    const size_t k = p.k0 + i;
                    const std::vector<Point2f> &f = (*p.features)[i];
                    const size_t n = std::min(f.size(), kT2dMaxFeatures);  // :753-757
                    if (f.size() >= kT2dMinFeatures && win_bad_[k]) {
                        err_ = "detection " + std::to_string(i) + " window";
                        return window_error((int)(b.h_boxes[4 * k + 2] * kWinSizeRatio));
                    }
                    for (size_t j = 0; j < n; j++) {
                        b.h_in[2 * (k * cap + j)] = f[j].x;
                        b.h_in[2 * (k * cap + j) + 1] = f[j].y;
                    }
                    b.h_cnt[k] = (int)n;
                }
            // boxes, last steps, counts and points in one copy (whole rows: a chain
            // row's unused tail is never read)
            // (a kernel reads the pinned block: psn_t2d_upload_device)
            if (!rc && (rc = psn_t2d_upload_device(db.d_inblk, b.h_inblk, dall.in_off_in + K * cap * 8, st)))
                err_ = "chain inputs upload";
        }
        if (rc) return rc;
        // the result block's last reader (a forward launch three frames back) first
        if (fread_rec_[rb]) chk(hipStreamWaitEvent(st, (hipEvent_t)ev_fread_[rb], 0), "result block reuse");
        const DeviceBuffers::ResView rv = dall.view(dall.d_res[rb]);
        psn_t2d_chain_dev cd{};
        cd.ndet = (int)K;
        cd.cap = (int)cap;
        cd.boxes = db.d_boxes;
        cd.cnt = db.d_cnt;
        cd.cur = db.d_in;
        cd.out_boxes = rv.obox;
        cd.sets = rv.sets;
        cd.set_cnt = rv.setcnt;
        cd.nsteps = rv.nsteps;
        cd.last_step = db.d_last;
        // cleared counters, set 0 = the features at t, the feature-minimum gate: one launch
        if (!rc) rc = psn_t2d_chain_begin_device(&cd, (int)kT2dMinFeatures, st);
        if (rc) return rc;
        for (int step = 1; step <= max_steps; step++) {
            queries_.clear();
            for (PassCam &p : pc) {
                const Cam &cam = cams_[p.cam];
                for (size_t i = 0; i < p.dets->size(); i++) {
                    const size_t k = p.k0 + i;
                    psn_lk_query q;
                    psn_lk_default_params(&q.params);
                    q.first_pt = (int)(k * cap);
                    q.num_pts = (int)cap;
                    if (step <= b.h_last[k]) {  // frame t-s+1 -> t-s with the square box-width window (:776-782)
                        q.prev_slot = cam.ring[kT2dInterval - step];
                        q.next_slot = cam.ring[kT2dInterval - 1 - step];
                        q.params.win_w = q.params.win_h = (int)(b.h_boxes[4 * k + 2] * kWinSizeRatio);
                    } else {  // the chain has ended (count 0 on the device): an empty query
                        q.prev_slot = q.next_slot = cam.ring[kT2dInterval - 1];
                    }
                    queries_.push_back(q);
                }
            }
            const float *in = step == 1 ? db.d_in : db.d_buf[step & 1];
            rc = psn_lk_track_device_counted(lk_, queries_.data(), (int)K, db.d_cnt, in, db.d_out, db.d_status, db.d_err);
            if (rc) return fail(rc, "psn_lk_track_device_counted");
            cd.cur = in;
            cd.nxt = db.d_out;
            cd.next_in = db.d_buf[(step + 1) & 1];
            rc = psn_t2d_chain_step_device(&cd, step, st);
            if (rc) return fail(rc, "psn_t2d_chain_step_device");
            // set 0 is final after step 1: the next frame's forward launch may read it
            if (step == 1) chk(hipEventRecord((hipEvent_t)ev_set0_[rb], st), "set-0 event");
        }
        if (max_steps == 0) chk(hipEventRecord((hipEvent_t)ev_set0_[rb], st), "set-0 event");
        ci.valid = rc == PSN_LK_OK;
    }
    return rc;
}

// The forward calls of frame t+1 (:871-877) straight from frame t's chain pass
// (result block src_rb): every detection of frame t becomes an active tracker
// -- matched ones take the detection's box and its set 0, new ones start from
// them (:1087, :1104, :1112-1147) -- so their LK inputs are on the device before
// the host has matched frame t. One counted launch on the forward stream, after
// the pass's set 0 is final and the frames are built: query k reads set 0 of
// detection k (count = its set-0 count, 0 for a detection that is no tracker)
// with the window of its box; the outputs land at the same index in the forward
// result block. pc: the pass of frame t+1 (its frames adopted).
int Tracker2DFlow::LaunchForwardFromChains(std::vector<PassCam> &pc, int src_rb, bool host_fallback) {
    for (PassCam &p : pc) p.fwd_rb = -1;
    if (src_rb < 0 || !chain_info_[src_rb].valid || chain_info_[src_rb].K == 0 || !dev_ || !dev_->d_res[src_rb]) {
        if (!host_fallback) return PSN_LK_OK;
        // the chain results are gone (the chain buffers grew since): the trackers'
        // set 0 from the host, one call per tracker; a window the LK cannot run is
        // a placeholder (the frame fails at its completion, as from the device)
        for (PassCam &p : pc) {
            Cam &cam = cams_[p.cam];
            cam.fwd.clear();
            ForwardJobs(p.cam, cam.trackers, cam.fstatus, cam.fwd);
            for (Job &jb : cam.fwd)
                if (forward_window_error(jb.win_w, jb.win_h)) jb.win_w = jb.win_h = 3;
            p.fwd = &cam.fwd;
        }
        return PassLaunchForward(pc);
    }
    const ChainInfo &ci = chain_info_[src_rb];
    const size_t cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS, K = ci.K;
    int rc = EnsureForward(K * S * cap, K);
    if (rc) return rc;
    DeviceBuffers &b = *dev_;
    const int par = fwd_par_ ^ 1;  // the block the last-but-one launch wrote: its copy waited for below
    hipStream_t st = (hipStream_t)psn_lk_get_stream(lk_), fs = (hipStream_t)FwdStream(par);
    fwd_queries_.assign(K, psn_lk_query{});
    for (PassCam &p : pc) {
        if (p.cam >= ci.k0.size()) continue;
        const Cam &cam = cams_[p.cam];
        for (size_t i = 0; i < ci.ndet[p.cam]; i++) {
            const size_t k = ci.k0[p.cam] + i;
            psn_lk_query &q = fwd_queries_[k];
            psn_lk_default_params(&q.params);  // maxLevel 3, (COUNT|EPS, 30, 0.01), minEig 1e-4
            q.prev_slot = cam.ring[kT2dInterval - 2];  // frame t -> t+1
            q.next_slot = cam.ring[kT2dInterval - 1];
            q.first_pt = (int)(k * S * cap);
            q.num_pts = (int)cap;
            const int ww = ci.win[k].first, wh = ci.win[k].second;
            // a window the LK cannot run: a placeholder (the frame fails at its
            // completion if that detection became a tracker, as the reference's
            // CV_Assert would)
            const bool ok = forward_window_error(ww, wh) == PSN_LK_OK;
            q.params.win_w = ok ? ww : 3;
            q.params.win_h = ok ? wh : 3;
        }
    }
    const DeviceBuffers::ResView rv = b.view(b.d_res[src_rb]);
    if (hipStreamWaitEvent(fs, (hipEvent_t)ev_set0_[src_rb], 0) != hipSuccess ||
        hipStreamWaitEvent(fs, (hipEvent_t)ev_fcopied_[par], 0) != hipSuccess) {
        err_ = "forward: set-0 / block events";
        return PSN_LK_ERR_HIP;
    }
    rc = psn_lk_set_stream(lk_, fs);
    if (!rc)
        rc = psn_lk_track_device_counted_strided(lk_, fwd_queries_.data(), (int)K, rv.setcnt, (int)S, rv.sets,
                                                 b.d_fout[par], b.d_fstatus[par], b.d_ferr[par]);
    const int rs = psn_lk_set_stream(lk_, st);
    if (rc || rs) return fail(rc ? rc : rs, "forward launch");
    fwd_par_ = par;
    if (hipEventRecord((hipEvent_t)ev_fend_[par], fs) != hipSuccess) {
        err_ = "forward: end event";
        return PSN_LK_ERR_HIP;
    }
    if (hipEventRecord((hipEvent_t)ev_fread_[src_rb], fs) != hipSuccess) {
        err_ = "forward: read event";
        return PSN_LK_ERR_HIP;
    }
    fread_rec_[src_rb] = true;
    for (PassCam &p : pc) {
        p.fwd_rb = src_rb;
        p.fwd_n = K * S * cap;
        p.fwd_par = par;
    }
    return PSN_LK_OK;
}

// 3 of the pass: the forward calls of every camera's trackers, on the forward
// stream, in their own arrays (every LK launch waits for the builds of the
// slots it reads).
int Tracker2DFlow::PassLaunchForward(std::vector<PassCam> &pc) {
    size_t J = 0, F = 0;
    for (PassCam &p : pc) {
        p.j0 = J;
        p.f0 = F;
        if (p.fwd) {
            J += p.fwd->size();
            for (const Job &jb : *p.fwd) F += jb.in->size();
        }
    }
    if (J == 0) return PSN_LK_OK;
    int rc = EnsureForward(F, J);
    if (rc) return rc;
    DeviceBuffers &b = *dev_;
    const int par = fwd_par_ ^ 1;
    hipStream_t st = (hipStream_t)psn_lk_get_stream(lk_), fs = (hipStream_t)FwdStream(par);
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            err_ = std::string(what) + ": " + hipGetErrorString(e);
            rc = PSN_LK_ERR_HIP;
        }
    };
    {
        size_t o = 0;
        fwd_queries_.clear();
        for (PassCam &p : pc) {
            if (!p.fwd) continue;
            for (const Job &jb : *p.fwd) {
                const std::vector<Point2f> &pts = *jb.in;
                psn_lk_query q;
                q.prev_slot = jb.prev_slot;
                q.next_slot = jb.next_slot;
                q.first_pt = (int)o;
                q.num_pts = (int)pts.size();
                psn_lk_default_params(&q.params);  // maxLevel 3, (COUNT|EPS, 30, 0.01), minEig 1e-4
                q.params.win_w = jb.win_w;
                q.params.win_h = jb.win_h;
                b.h_fcnt[fwd_queries_.size()] = (int)pts.size();
                fwd_queries_.push_back(q);
                for (size_t i = 0; i < pts.size(); i++, o++) {
                    b.h_fin[2 * o] = pts[i].x;
                    b.h_fin[2 * o + 1] = pts[i].y;
                }
            }
        }
        // counts and points in one copy
        // (one input block: the other stream's last launch has read it)
        chk(hipStreamWaitEvent(fs, (hipEvent_t)ev_fend_[par ^ 1], 0), "forward input block event");
        chk(hipStreamWaitEvent(fs, (hipEvent_t)ev_fcopied_[par], 0), "forward block event");
        if (!rc && (rc = psn_t2d_upload_device(b.d_fiblk, b.h_fiblk, b.fi_off_pts + F * 8, fs)))
            err_ = "forward inputs upload";
        if (rc) return rc;
        rc = psn_lk_set_stream(lk_, fs);
        if (!rc)
            rc = psn_lk_track_device_counted(lk_, fwd_queries_.data(), (int)J, b.d_fcnt, b.d_fin, b.d_fout[par],
                                             b.d_fstatus[par], b.d_ferr[par]);
        const int rs = psn_lk_set_stream(lk_, st);
        if (rc || rs) return fail(rc ? rc : rs, "forward launch");
        fwd_par_ = par;
        chk(hipEventRecord((hipEvent_t)ev_fend_[par], fs), "forward end event");
        for (PassCam &p : pc) p.fwd_par = par;
    }
    return rc;
}

// Wait for the pass and unpack it: features (GridFAST mode), every valid
// detection's chain (boxes, point sets), the forward outputs.
int Tracker2DFlow::PassComplete(std::vector<PassCam> &pc, bool gridfast) {
    int rc = PassWait(pc);
    if (!rc) rc = PassFeatures(pc, gridfast);
    if (!rc) PassUnpack(pc);
    return rc;
}

// Enqueue the result copies and wait for the pass's device work.
int Tracker2DFlow::PassWait(std::vector<PassCam> &pc) {
    const int rc = PassCopy(pc);
    return rc ? rc : PassSync();
}

int Tracker2DFlow::PassCopy(std::vector<PassCam> &pc) {
    int rc = PSN_LK_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !rc) {
            err_ = std::string(what) + ": " + hipGetErrorString(e);
            rc = PSN_LK_ERR_HIP;
        }
    };
    const size_t cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS;
    DeviceBuffers *bp = dev_;
    size_t K = 0, F = 0;
    for (PassCam &p : pc) {
        K += p.dets->size();
        if (p.fwd)
            for (const Job &jb : *p.fwd) F += jb.in->size();
    }
    hipStream_t st = (hipStream_t)(pc.empty() ? psn_lk_get_stream(lk_) : ChainStream(pc[0].set)),
                fs = (hipStream_t)FwdStream(pc.empty() ? fwd_par_ : pc[0].fwd_par);
    const int rb = pc.empty() ? -1 : pc[0].rb;
    if (K && bp && rb >= 0)
        if (!rc && (rc = psn_t2d_download_device(bp->h_res[rb], bp->d_res[rb], bp->res_sets_off + K * S * cap * 8, st)))
            err_ = "chain results download";
    if (!pc.empty() && pc[0].fwd_rb >= 0) F = pc[0].fwd_n;  // the forward launch from the previous frame's chains
    if (F && bp) {
        // status and points in one copy, on the chain stream after the forward
        // launch (the forward stream goes on with the next frame's launch)
        const int par = pc[0].fwd_par;
        chk(hipStreamWaitEvent(st, (hipEvent_t)ev_fend_[par], 0), "forward end wait");
        if (!rc && (rc = psn_t2d_download_device(bp->h_foblk, bp->d_foblk[par], bp->fo_off_pts + F * 8, st)))
            err_ = "forward results download";
        chk(hipEventRecord((hipEvent_t)ev_fcopied_[par], st), "forward copied event");
    }
    // everything the pass enqueued precedes these records (the forward work of
    // a pass without result copy: the forward stream's record)
    chk(hipEventRecord((hipEvent_t)ev_chain_, st), "chain results event");
    chk(hipEventRecord((hipEvent_t)ev_fwd_, fs), "forward results event");
    wait_chain_ = wait_fwd_ = rc == PSN_LK_OK;
    return rc;
}

// Poll the completion events (a blocking stream sync sleeps and wakes ~0.1 ms
// late; the next frame's work is enqueued right after this returns). Past a
// short spin every poll yields the core: ranks sharing a GPU's CPU allotment
// keep their cores for the host work of their own frames.
int Tracker2DFlow::PassSync() {
    for (int i = 0; i < 2; i++) {
        bool &w = i ? wait_fwd_ : wait_chain_;
        if (!w) continue;
        hipEvent_t e = (hipEvent_t)(i ? ev_fwd_ : ev_chain_);
        hipError_t q;
        for (unsigned n = 0; (q = hipEventQuery(e)) == hipErrorNotReady; n++) {
            if (n < 256)
                __builtin_ia32_pause();
            else
                sched_yield();
        }
        w = false;
        if (q != hipSuccess) {
            err_ = std::string(i ? "forward" : "chain") + " sync: " + hipGetErrorString(q);
            return PSN_LK_ERR_HIP;
        }
    }
    return PSN_LK_OK;
}

// After PassWait: GridFAST features (the pass's staging set) and window errors.
int Tracker2DFlow::PassFeatures(std::vector<PassCam> &pc, bool gridfast) {
    if (!gridfast || pc.empty() || !dev_) return PSN_LK_OK;
    const size_t cap = PSN_T2D_CHAIN_CAP;
    const DeviceBuffers::Stage *bp = &dev_->stage[pc[0].set];
    const std::vector<char> &win_bad_ = win_bad_sets_[pc[0].set];
    for (PassCam &p : pc) {
        const size_t n = p.dets->size();
        p.features->assign(n, {});
        for (size_t i = 0; i < n; i++) {
            const size_t k = p.k0 + i;
            const int m = bp->h_rawcnt[k];
            // a window the LK cannot run fails the frame only if the chain had to run it (:744)
            if (win_bad_[k] && (size_t)m >= kT2dMinFeatures) {
                err_ = "detection " + std::to_string(i) + " window";
                return window_error((int)(bp->h_boxes[4 * k + 2] * kWinSizeRatio));
            }
            const float *xy = bp->h_in + 2 * cap * k;
            (*p.features)[i].resize((size_t)m);
            for (int j = 0; j < m; j++) (*p.features)[i][(size_t)j] = Point2f{xy[2 * j], xy[2 * j + 1]};
        }
    }
    return PSN_LK_OK;
}

// After PassWait: the chains' boxes and point sets (h_res) and the forward
// outputs, which a next pass's chain launch leaves alone (unless it regrows the
// chain buffers: ChainsFit).
void Tracker2DFlow::PassUnpack(std::vector<PassCam> &pc) {
    const size_t cap = PSN_T2D_CHAIN_CAP, S = PSN_T2D_CHAIN_STEPS;
    DeviceBuffers *bp = dev_;
    for (PassCam &p : pc) {
        std::vector<Chain> chains;
        BackwardBegin(*p.dets, *p.features, *p.out, chains);  // valid detections, in order
        const DeviceBuffers::ResView hv = p.out->empty() ? DeviceBuffers::ResView{} : bp->view(bp->h_res[p.rb]);
        for (DetectedObject &ob : *p.out) {
            const size_t k = p.k0 + ob.id;  // the detection index = its device chain
            const int ns = hv.nsteps[k];
            for (int s2 = 1; s2 <= ns; s2++) {
                const double *r = hv.obox + (k * S + s2) * 4;
                ob.boxes.push_back(Rect(r[0], r[1], r[2], r[3]).scale(1.0 / kFlowScale));
            }
            for (int r = 0; ns > 0 && r <= ns; r++) {
                const int m = hv.setcnt[k * S + r];
                const float *pp = hv.sets + (k * S + r) * cap * 2;
                std::vector<Point2f> v((size_t)m);
                for (int i = 0; i < m; i++) v[(size_t)i] = Point2f{pp[2 * i], pp[2 * i + 1]};
                ob.vecvecTrackedFeatures.push_back(std::move(v));
            }
        }
        if (p.fwd_rb >= 0) {  // forward outputs of the camera's trackers, at their source detection's index
            Cam &cam = cams_[p.cam];
            cam.fstatus.assign(cam.trackers.size(), {});
            for (size_t j = 0; j < cam.trackers.size(); j++) {
                Tracker2D *tr = cam.trackers[j];
                const size_t off = (cam.fwd_k0 + (size_t)tr->srcDet) * S * cap, m = tr->featurePoints.size();
                tr->trackedPoints.resize(m);
                cam.fstatus[j].resize(m);
                for (size_t i = 0; i < m; i++) {
                    tr->trackedPoints[i] = Point2f{bp->h_fwd_out[2 * (off + i)], bp->h_fwd_out[2 * (off + i) + 1]};
                    cam.fstatus[j][i] = bp->h_fwd_st[off + i];
                }
            }
            continue;
        }
        if (!p.fwd) continue;
        for (size_t j = 0, off = p.f0; j < p.fwd->size(); j++) {
            Job &jb = (*p.fwd)[j];
            const size_t m = jb.in->size();
            jb.out->resize(m);
            jb.status->resize(m);
            for (size_t i = 0; i < m; i++, off++) {
                (*jb.out)[i] = Point2f{bp->h_fwd_out[2 * off], bp->h_fwd_out[2 * off + 1]};
                (*jb.status)[i] = bp->h_fwd_st[off];
            }
        }
    }
}

bool Tracker2DFlow::ChainsFit(const std::vector<CamFrame> &io) const {
    size_t K = 0;
    for (const CamFrame &f : io) K += f.dets.size();
    return K == 0 || (dev_ && dev_->sc[0].d_in && dev_->nchains >= K);
}

// One camera (0), one pass, synchronous.
int Tracker2DFlow::DevicePass(const std::vector<Detection> &dets, std::vector<std::vector<Point2f>> &features,
                              std::vector<DetectedObject> &out, std::vector<Job> *fwd, bool gridfast, uint32_t seed) {
    std::vector<PassCam> pc(1);
    pc[0].cam = 0;
    pc[0].dets = &dets;
    pc[0].features = &features;
    pc[0].out = &out;
    pc[0].fwd = fwd;
    out.clear();
    int rc = PassLaunch(pc, gridfast, seed);
    if (rc) {  // drain what was enqueued before returning the error
        SyncChains();
        SyncForward();
        return rc;
    }
    return PassComplete(pc, gridfast);
}

int Tracker2DFlow::PushFrame(const uint8_t *frame, int stride, int channels) {
    if (!lk_) return PSN_LK_ERR_ARG;
    const int slot = cams_[0].ring[kT2dInterval - 1];
    const int rc = psn_lk_push_frame(lk_, slot, frame, stride, channels);
    if (rc) return fail(rc, "psn_lk_push_frame");
    filled_[(size_t)slot] = 1;
    return PSN_LK_OK;
}

int Tracker2DFlow::PushFrameDevice(const uint8_t *dev, int stride, int channels) {
    if (!lk_) return PSN_LK_ERR_ARG;
    const int slot = cams_[0].ring[kT2dInterval - 1];
    const int rc = psn_lk_push_frame_device(lk_, slot, dev, stride, channels);
    if (rc) return fail(rc, "psn_lk_push_frame_device");
    filled_[(size_t)slot] = 1;
    return PSN_LK_OK;
}

// The next free staging slot of a camera (frames are adopted in push order).
int Tracker2DFlow::NextStagingSlot(size_t cam, int *slot) {
    Cam &c = cams_[cam];
    if (c.nstaged >= kT2dStaging) {
        err_ = "camera " + std::to_string(cam) + ": " + std::to_string(kT2dStaging) + " frames staged already";
        return PSN_LK_ERR_ARG;
    }
    *slot = c.spares[c.nstaged];
    return PSN_LK_OK;
}

int Tracker2DFlow::StageFrame(size_t cam, const uint8_t *frame, int stride, int channels, bool on_device) {
    if (!lk_ || cam >= cams_.size() || !frame) return PSN_LK_ERR_ARG;
    Cam &c = cams_[cam];
    int slot = -1, rc = NextStagingSlot(cam, &slot);
    if (rc) return rc;
    rc = on_device ? psn_lk_push_frame_device(lk_, slot, frame, stride, channels)
                   : psn_lk_push_frame_async(lk_, slot, frame, stride, channels);
    if (rc) return fail(rc, "stage frame");
    filled_[(size_t)slot] = 1;
    c.nstaged++;
    return PSN_LK_OK;
}

int Tracker2DFlow::StageFrameJpeg(size_t cam, const uint8_t *jpeg, size_t len) {
    if (!lk_ || cam >= cams_.size() || !jpeg) return PSN_LK_ERR_ARG;
    Cam &c = cams_[cam];
    int slot = -1, rc = NextStagingSlot(cam, &slot);
    if (rc) return rc;
    rc = psn_lk_push_frame_jpeg(lk_, slot, jpeg, len);
    if (rc) return fail(rc, "stage JPEG frame");
    filled_[(size_t)slot] = 1;
    c.nstaged++;
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
    const int rc = psn_gridfast_detect(lk_, cams_[0].ring[kT2dInterval - 1], rois.data(), (int)n, &p, seed,
                                       gf_xy_.data(), cnt.data(), tot.data());
    if (rc) return fail(rc, "psn_gridfast_detect");
    for (size_t i = 0; i < n; i++) {
        const float *xy = gf_xy_.data() + 2 * kT2dMaxFeatures * i;
        features[i].resize((size_t)cnt[i]);
        for (int k = 0; k < cnt[i]; k++) features[i][(size_t)k] = Point2f{xy[2 * k], xy[2 * k + 1]};
    }
    return PSN_LK_OK;
}

void Tracker2DFlow::RotateRing() { std::rotate(cams_[0].ring, cams_[0].ring + 1, cams_[0].ring + kT2dInterval); }

// steps s = 1..3 need frame t-s: consecutive filled slots behind the newest
int Tracker2DFlow::StepsAvailable(size_t cam) const {
    int s = 0;
    while (s + 1 < kT2dInterval && filled_[(size_t)cams_[cam].ring[kT2dInterval - 2 - s]]) s++;
    return s;
}

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
        for (int k = 0; k < 3; k++) o.location[k] = dets[i].location[k];
        o.height = dets[i].height;
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

void Tracker2DFlow::BackwardJobs(int step, std::vector<Chain> &chains, const std::vector<DetectedObject> &out,
                                 std::vector<Job> &jobs) {
    for (Chain &c : chains) {
        if (!c.active) continue;
        const Rect box = out[c.obj].detection.box.scale(kFlowScale);
        const int win = (int)(box.w * kWinSizeRatio);  // square window of the box width (:782)
        jobs.push_back(Job{cams_[0].ring[kT2dInterval - step], cams_[0].ring[kT2dInterval - 1 - step], win, win, &c.curr,
                           &c.prev, &c.status});
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

void Tracker2DFlow::BackwardEnd(std::vector<DetectedObject> &out, const std::vector<std::vector<Point2f>> &features) {
    for (DetectedObject &o : out)  // no step kept >= 4 inliers: the features at t (:815-818)
        if (o.vecvecTrackedFeatures.empty()) {
            const std::vector<Point2f> &f = features[o.id];
            o.vecvecTrackedFeatures.emplace_back(f.begin(), f.begin() + (ptrdiff_t)std::min(f.size(), kT2dMaxFeatures));
        }
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
    if (device_chain_) {
        std::vector<std::vector<Point2f>> f = features;
        const int rc = DevicePass(dets, f, out, nullptr, false, 0);
        if (rc) return rc;
        BackwardEnd(out, features);
        return PSN_LK_OK;
    }
    std::vector<Chain> chains;
    BackwardBegin(dets, features, out, chains);
    std::vector<Job> jobs;
    for (int step = 1; StepAvailable(step); step++) {
        jobs.clear();
        BackwardJobs(step, chains, out, jobs);
        if (jobs.empty()) break;
        int rc = RunJobs(jobs);
        if (rc) return rc;
        BackwardStepDone(chains, out);
    }
    BackwardEnd(out, features);
    return PSN_LK_OK;
}

// ---------------------------------------------------------------------------
// Forward tracking + matching score (:851-1025)
// ---------------------------------------------------------------------------

void Tracker2DFlow::ForwardJobs(size_t cam, const std::vector<Tracker2D *> &trackers,
                                std::vector<std::vector<uint8_t>> &status, std::vector<Job> &jobs) {
    status.assign(trackers.size(), {});
    const int *ring = cams_[cam].ring;
    for (size_t t = 0; t < trackers.size(); t++) {
        Tracker2D *tr = trackers[t];
        tr->trackedPoints.clear();
        const Rect cur = tr->boxes.back().scale(kFlowScale);
        jobs.push_back(Job{ring[kT2dInterval - 2], ring[kT2dInterval - 1], (int)(cur.w * kWinSizeRatio),
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
                // after a failed frame a tracker's duration (frame based, :1085) runs
                // past its boxes: the reference reads outside the vector (undefined);
                // here the pair cannot match (as oracle/tracker2d_oracle.py)
                if (tb >= tr->boxes.size()) {
                    boxCost = std::numeric_limits<double>::infinity();
                    break;
                }
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
    ForwardJobs(0, trackers, status, jobs);
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
    std::vector<std::vector<uint8_t>> fstatus;
    std::vector<Job> fwd;
    ForwardJobs(0, trackers, fstatus, fwd);
    const int rc = DevicePass(dets, features, out, &fwd, true, seed);
    if (rc) return rc;
    BackwardEnd(out, features);
    ForwardDone(trackers, fstatus, out, cost);
    return PSN_LK_OK;
}

int Tracker2DFlow::TrackFrame(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                              std::vector<DetectedObject> &out, const std::vector<Tracker2D *> &trackers,
                              std::vector<float> &cost) {
    if (!lk_ || features.size() != dets.size()) return PSN_LK_ERR_ARG;
    if (!trackers.empty() && !StepAvailable(1)) return PSN_LK_ERR_SLOT;
    std::vector<std::vector<uint8_t>> fstatus;
    std::vector<Job> jobs;
    if (device_chain_) {
        ForwardJobs(0, trackers, fstatus, jobs);
        std::vector<std::vector<Point2f>> f = features;
        const int rc = DevicePass(dets, f, out, &jobs, false, 0);
        if (rc) return rc;
        BackwardEnd(out, features);
        ForwardDone(trackers, fstatus, out, cost);
        return PSN_LK_OK;
    }
    std::vector<Chain> chains;
    BackwardBegin(dets, features, out, chains);
    // launch 1: backward step 1 of every detection + every forward call
    if (StepAvailable(1)) BackwardJobs(1, chains, out, jobs);
    const size_t nb = jobs.size();
    ForwardJobs(0, trackers, fstatus, jobs);
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
    BackwardEnd(out, features);
    ForwardDone(trackers, fstatus, out, cost);
    return PSN_LK_OK;
}

// ---------------------------------------------------------------------------
// CPSNWhere_Tracker2D::Run of every camera (:251-373), batched
// ---------------------------------------------------------------------------

// Adopt every camera's staged frame as frame t (the ring advances: the oldest
// slot becomes the next staging slot; Run's buffer circulation, :310-316) and
// set up the pass over io (forward calls not yet attached).
int Tracker2DFlow::AdoptFrames(std::vector<CamFrame> &io, bool gridfast, std::vector<PassCam> &pass) {
    if (io.size() != cams_.size()) return PSN_LK_ERR_ARG;
    for (size_t c = 0; c < cams_.size(); c++) {
        if (cams_[c].nstaged == 0) {
            err_ = "camera " + std::to_string(c) + ": no frame staged";
            return PSN_LK_ERR_SLOT;
        }
        if (!gridfast && io[c].features.size() != io[c].dets.size()) return PSN_LK_ERR_ARG;
    }
    pass.assign(cams_.size(), PassCam());
    for (size_t c = 0; c < cams_.size(); c++) {
        Cam &cam = cams_[c];
        // the first staged frame joins the ring as frame t; the oldest ring slot
        // becomes the last staging slot (a later push into it waits for its readers)
        const int oldest = cam.ring[0];
        std::rotate(cam.ring, cam.ring + 1, cam.ring + kT2dInterval);
        cam.ring[kT2dInterval - 1] = cam.spares[0];
        std::rotate(cam.spares, cam.spares + 1, cam.spares + kT2dStaging);
        cam.spares[kT2dStaging - 1] = oldest;
        cam.nstaged--;
        PassCam &p = pass[c];
        p.cam = c;
        p.dets = &io[c].dets;
        p.features = &io[c].features;
        p.out = &io[c].objects;
        p.fwd = nullptr;
        io[c].objects.clear();
    }
    return PSN_LK_OK;
}

void Tracker2DFlow::UnadoptFrames() {
    for (Cam &cam : cams_) {
        const int newest = cam.ring[kT2dInterval - 1];
        std::rotate(cam.ring, cam.ring + kT2dInterval - 1, cam.ring + kT2dInterval);
        cam.ring[0] = cam.spares[kT2dStaging - 1];
        std::rotate(cam.spares, cam.spares + kT2dStaging - 1, cam.spares + kT2dStaging);
        cam.spares[0] = newest;
        cam.nstaged++;
    }
}

// Enqueue frame t's device work for every camera: one pass over all cameras
// (features, backward chains, forward calls of every active tracker). When
// RunComplete(t-1, next = frame t) has launched frame t already, this only
// confirms it.
int Tracker2DFlow::RunLaunch(unsigned frameIdx, std::vector<CamFrame> &io, bool gridfast, uint32_t seed) {
    if (!lk_ || io.size() != cams_.size()) return PSN_LK_ERR_ARG;
    if (launched_ahead_) {
        if (&io != pre_io_ || frameIdx != run_frame_ || gridfast != run_gridfast_) {
            err_ = "RunLaunch: frame " + std::to_string(frameIdx) + " is not the frame launched ahead (" +
                   std::to_string(run_frame_) + ")";
            return PSN_LK_ERR_ARG;
        }
        launched_ahead_ = false;
        pre_io_ = nullptr;
        return PSN_LK_OK;
    }
    int rc = AdoptFrames(io, gridfast, run_pass_);
    if (rc) return rc;
    run_frame_ = frameIdx;
    run_gridfast_ = gridfast;
    // frame t's forward calls from frame t-1's chain pass (when it left trackers),
    // then frame t's features and chains
    bool any = false;
    for (const Cam &cam : cams_) any = any || !cam.active.empty();
    const int saved_next_rb = next_rb_, saved_last_rb = last_rb_, saved_stage = stage_;
    rc = any ? LaunchForwardFromChains(run_pass_, trk_rb_, true) : PSN_LK_OK;
    if (!rc) rc = PassLaunchChains(run_pass_, gridfast, seed);
    if (rc) {  // nothing of the frame stays in flight; the result blocks as before
        SyncChains();
        SyncForward();
        run_pass_.clear();
        next_rb_ = saved_next_rb;
        last_rb_ = saved_last_rb;
        stage_ = saved_stage;
    }
    return rc;
}


// Wait for the frame's device work, then per camera: overlap flags (:824-835),
// matching costs + majority gate (:906-1022), assignment and tracker update
// (:1038-1164), result packaging (:1099-1101, :1144-1146).
int Tracker2DFlow::RunComplete(std::vector<CamFrame> &io) { return RunComplete(io, nullptr, 0, false, 0); }

// With next: frame t+1 is launched from here. Its features and backward chains
// (its frames staged) are enqueued as soon as frame t's device work is done,
// before the host part of frame t, so the GPU runs them while the host matches
// frame t; its forward calls follow frame t's tracker update. Frame t+1's
// chains read only its detections and the ring, never frame t's trackers, so
// the results are those of RunLaunch(t+1) after RunComplete(t).
int Tracker2DFlow::RunComplete(std::vector<CamFrame> &io, std::vector<CamFrame> *next, unsigned nextFrameIdx,
                               bool nextGridfast, uint32_t nextSeed) {
    if (!lk_ || io.size() != cams_.size() || run_pass_.size() != cams_.size() || launched_ahead_ || &io == next)
        return PSN_LK_ERR_ARG;
    // The next frame's chains are enqueued right behind this frame's result copies
    // (stream order keeps them from overwriting what is copied; their inputs go
    // through the other staging set), then this frame is waited for and
    // unpacked while they run. If they need larger chain buffers, the regrow
    // waits, so this frame is unpacked first.
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    auto stamp = [&](int i) { host_us_[i] += std::chrono::duration<double, std::micro>(clk::now() - t0).count(); };
    frame_completed_ = false;
    const int cur_rb = run_pass_.empty() ? -1 : run_pass_[0].rb;
    std::vector<size_t> cur_k0(cams_.size(), 0);
    for (const PassCam &p : run_pass_) cur_k0[p.cam] = p.k0;
    int rc = PassCopy(run_pass_);
    const bool early = !rc && next && ChainsFit(*next);
    int prc = PSN_LK_OK;
    std::vector<PassCam> pre;
    const int saved_next_rb = next_rb_, saved_last_rb = last_rb_;
    // a next frame that cannot be launched leaves no trace: its work drained, its
    // frames staged again (the rings as before), frame t still completed
    auto abandon_next = [&]() {
        SyncChains();
        SyncForward();
        UnadoptFrames();
        next_rb_ = saved_next_rb;
        last_rb_ = saved_last_rb;
        pre.clear();
    };
    // frame t+1: its forward calls straight from frame t's chains (every detection
    // of frame t becomes a tracker), then its features and chains
    auto prelaunch = [&]() {
        prc = AdoptFrames(*next, nextGridfast, pre);
        if (prc) {
            pre.clear();
            return;
        }
        prc = LaunchForwardFromChains(pre, cur_rb, false);
        if (!prc) prc = PassLaunchChains(pre, nextGridfast, nextSeed);
        if (prc) abandon_next();
    };
    if (early) prelaunch();
    stamp(0);  // copies + next frame's forward + chains enqueued
    if (!rc) rc = PassSync();
    stamp(1);  // device work done
    if (!rc) rc = PassFeatures(run_pass_, run_gridfast_);
    if (rc) {
        run_pass_.clear();
        if (next && early && !prc) abandon_next();  // frame t failed: nothing of t+1 stays in flight
        return rc;
    }
    PassUnpack(run_pass_);
    run_pass_.clear();
    if (next && !early) prelaunch();
    stamp(2);  // unpacked
    // a tracker whose box window the forward LK cannot run (CV_Assert in the
    // reference) fails the frame before any camera is updated
    for (size_t c = 0; c < cams_.size(); c++)
        for (const Tracker2D *tr : cams_[c].trackers) {
            const Rect b = tr->boxes.back().scale(kFlowScale);
            const int we = forward_window_error((int)(b.w * kWinSizeRatio), (int)(b.h * kWinSizeRatio));
            if (we) {
                err_ = "camera " + std::to_string(c) + ": tracker " + std::to_string(tr->id) + " forward window";
                if (next && !prc && !pre.empty()) abandon_next();
                return we;
            }
        }
    for (size_t c = 0; c < cams_.size(); c++) {
        Cam &cam = cams_[c];
        CamFrame &f = io[c];
        clk::time_point p = clk::now();
        auto part = [&](int i) {
            const clk::time_point q = clk::now();
            host_us_[5 + i] += std::chrono::duration<double, std::micro>(q - p).count();
            p = q;
        };
        BackwardEnd(f.objects, f.features);
        part(0);
        ForwardDone(cam.trackers, cam.fstatus, f.objects, f.cost);
        part(1);
        const std::vector<int> match = AssignDetections(f.cost, f.objects.size(), cam.trackers.size());
        part(2);
        MatchingAndUpdating(f.objects, cam.active, cam.storage, match, run_frame_, cam.newTrackerID, f.result);
        part(3);
        f.result.camID = cam.camID;
        // the next frame's forward calls (launched from this frame's chains): these trackers
        cam.trackers.assign(cam.active.begin(), cam.active.end());
        cam.fwd_k0 = cur_k0[c];
    }
    trk_rb_ = cur_rb;  // the trackers' set 0
    stamp(3);  // matched, trackers updated
    host_calls_++;
    frame_completed_ = true;
    if (!next || prc) return prc;
    stamp(4);
    run_pass_ = std::move(pre);
    run_frame_ = nextFrameIdx;
    run_gridfast_ = nextGridfast;
    pre_io_ = next;
    launched_ahead_ = true;
    return PSN_LK_OK;
}

}  // namespace psn
