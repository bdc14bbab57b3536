// Tracker2D flow stage on the MI355X LK path (C++ host above the psn_lk C ABI).
//
// Mirrors, with the same names, argument meaning and results, the parts of
// CPSNWhere_Tracker2D (psn_where/PSNWhere_Tracker2D.{h,cpp}) that drive the
// optical flow: ingest + ring (Run, :251-263, :310-316), the backward feature
// tracking chain (:690-838), forward tracking + matching score (:851-1025),
// LocalSearchKLT (:452-554), BoxMatchingCost (:600-613) and ResultWithTracker
// (:1231-1257). The LK calls of a frame are batched: every detection's chain
// step s is one launch, and step 1 shares its launch with the forward calls.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "psn_lk.h"
#include "psn_types.hpp"

namespace psn {

constexpr int kT2dInterval = 4;          // PSN_2D_BACKTRACKING_INTERVAL (:16)
constexpr size_t kT2dMinFeatures = 4;    // PSN_2D_FEATURE_MIN_NUM_TRACK (:12)
constexpr size_t kT2dMaxFeatures = 100;  // PSN_2D_FEATURE_MAX_NUM_TRACK (:13)
constexpr double kFlowScale = 1.0;       // PSN_2D_OPTICALFLOW_SCALE (:18)
constexpr double kWinSizeRatio = 1.0;    // PSN_2D_FEATURE_WIN_SIZE_RATIO (:15)

Rect LocalSearchKLT(Rect preBox, const std::vector<Point2f> &preFeatures, const std::vector<Point2f> &curFeatures,
                    std::vector<size_t> &inlierFeatureIndex);
double BoxMatchingCost(const Rect &box1, const Rect &box2);
void ResultWithTracker(const Tracker2D &tracker, Object2DInfo &out);

class Tracker2DFlow {
  public:
    Tracker2DFlow() = default;
    ~Tracker2DFlow() { Finalize(); }
    Tracker2DFlow(const Tracker2DFlow &) = delete;
    Tracker2DFlow &operator=(const Tracker2DFlow &) = delete;

    int Initialize(unsigned camID, int width, int height, int device);
    void Finalize();
    // ingest frame t into the newest ring slot (cvtColor(BGR2GRAY) + resize 1.0)
    int PushFrame(const uint8_t *frame, int stride, int channels);
    int PushFrameDevice(const uint8_t *dev, int stride, int channels);  // frame already in device memory
    psn_lk_ctx *LkContext() const { return lk_; }
    // buffer circulation at the end of Run
    void RotateRing();

    // Feature extraction of the backward chain (:734-757) on frame t (the
    // newest ring slot): GridFAST masked by each detection's rectROI
    // (box.cropWithSize(cols, rows).cv(), :736), then the seeded shuffle + cap
    // to PSN_2D_FEATURE_MAX_NUM_TRACK. features[i] may hold < 4 points (the
    // backward step then skips detection i, :744).
    int DetectFeatures(const std::vector<Detection> &dets, uint32_t seed, std::vector<std::vector<Point2f>> &features);

    // Track2D_BackwardFeatureTracking for detections that passed the caller's
    // height gate; features[i] = detection i's points at t after shuffle + cap
    // (GridFAST stays with the caller). out = m_vecDetection2D.
    int BackwardFeatureTracking(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                                std::vector<DetectedObject> &out);
    // Track2D_ForwardTrackingAndGetMatchingScore over the active trackers;
    // cost = matchingCostArray [dets x trackers], +inf where not matched.
    int ForwardTrackingAndGetMatchingScore(const std::vector<Tracker2D *> &trackers,
                                           const std::vector<DetectedObject> &dets, std::vector<float> &cost);
    // both: the forward calls overlap the backward chain (own stream)
    int TrackFrame(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                   std::vector<DetectedObject> &out, const std::vector<Tracker2D *> &trackers, std::vector<float> &cost);

    // DetectFeatures + TrackFrame as one device pass (device chain mode): GridFAST
    // writes the chain inputs on the device, the forward launch runs beside it
    int TrackFrameDetect(const std::vector<Detection> &dets, uint32_t seed,
                         std::vector<std::vector<Point2f>> &features, std::vector<DetectedObject> &out,
                         const std::vector<Tracker2D *> &trackers, std::vector<float> &cost);

    psn_lk_ctx *lk() const { return lk_; }
    // backward chain steps on the device (default) or on the host (PSN_T2D_HOST_CHAIN=1)
    void SetDeviceChain(bool on) { device_chain_ = on; }
    bool DeviceChain() const { return device_chain_; }
    const std::string &last_error() const { return err_; }

  private:
    struct Job {  // one calcOpticalFlowPyrLK call
        int prev_slot, next_slot, win_w, win_h;
        const std::vector<Point2f> *in;
        std::vector<Point2f> *out;
        std::vector<uint8_t> *status;
    };
    int RunJobs(std::vector<Job> &jobs);
    int fail(int rc, const char *what);

    struct Chain {  // one detection's backward chain
        size_t obj;
        std::vector<Point2f> curr, prev;
        std::vector<uint8_t> status;
        bool active;
    };
    void BackwardBegin(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                       std::vector<DetectedObject> &out, std::vector<Chain> &chains);
    void BackwardJobs(int step, std::vector<Chain> &chains, const std::vector<DetectedObject> &out,
                      std::vector<Job> &jobs);
    void BackwardStepDone(std::vector<Chain> &chains, std::vector<DetectedObject> &out);
    void BackwardEnd(std::vector<Chain> &chains, std::vector<DetectedObject> &out);
    bool StepAvailable(int step) const;
    // every chain step (LK launch + LocalSearchKLT kernel) enqueued back to back,
    // one host sync at the end; the forward jobs' launch runs beside them
    int ChainsOnDevice(std::vector<Chain> &chains, std::vector<DetectedObject> &out, std::vector<Job> *fwd);
    int EnsureDevice(size_t nchains, size_t nfwd_pts, size_t nfwd_jobs);
    void ForwardJobs(const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                     std::vector<Job> &jobs);
    void ForwardDone(const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                     const std::vector<DetectedObject> &dets, std::vector<float> &cost);

    psn_lk_ctx *lk_ = nullptr;
    // device chain: the forward queries run on their own stream (a hipStream_t),
    // overlapping the backward chain's launches; ev_in_ orders them after the inputs
    void *fwd_stream_ = nullptr, *ev_in_ = nullptr;
    std::vector<psn_lk_query> fwd_queries_;
    unsigned camID_ = 0;
    int width_ = 0, height_ = 0;
    int ring_[kT2dInterval] = {0, 1, 2, 3};  // slot ids, oldest first; ring_[3] = frame t
    bool filled_[kT2dInterval] = {false, false, false, false};
    std::string err_;
    // batched-call staging
    std::vector<float> xy_in_, xy_out_, err_out_, gf_xy_;
    std::vector<uint8_t> st_out_;
    std::vector<psn_lk_query> queries_;
    bool device_chain_ = true;
    struct DeviceBuffers;
    DeviceBuffers *dev_ = nullptr;
};

}  // namespace psn
