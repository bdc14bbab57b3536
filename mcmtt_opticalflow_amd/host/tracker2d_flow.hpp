// Tracker2D flow stage on the MI355X LK path (C++ host above the psn_lk C ABI).
//
// Mirrors, with the same names, argument meaning and results, the parts of
// CPSNWhere_Tracker2D (psn_where/PSNWhere_Tracker2D.{h,cpp}) that drive the
// optical flow: ingest + ring (Run, :251-263, :310-316), the backward feature
// tracking chain (:690-838), forward tracking + matching score (:851-1025),
// LocalSearchKLT (:452-554), BoxMatchingCost (:600-613), and after the flow
// Track2D_MatchingAndUpdating (:1038-1164) with ResultWithTracker (:1231-1257).
//
// One object serves C cameras (CPSNWhere::TrackPeople's per-camera loop,
// PSNWhere.cpp:257-266): they share one LK context (camera c owns ring slots
// [c*kSlotsPerCam, c*kSlotsPerCam + kSlotsPerCam)), so a chain step of every
// detection of every camera is ONE LK launch, and the forward calls of every
// tracker of every camera are one launch on a second stream beside the chain.
#pragma once

#include <cstdint>
#include <list>
#include <string>
#include <vector>

#include "psn_lk.h"
#include "psn_types.hpp"

namespace psn {

constexpr int kT2dInterval = 4;          // PSN_2D_BACKTRACKING_INTERVAL (:16)
// the ring + two staging slots: frame t+2 uploads (and its pyramid builds) while
// frame t+1 waits staged and frame t runs
constexpr int kT2dStaging = 2;
constexpr int kSlotsPerCam = kT2dInterval + kT2dStaging;
constexpr size_t kT2dMinFeatures = 4;    // PSN_2D_FEATURE_MIN_NUM_TRACK (:12)
constexpr size_t kT2dMaxFeatures = 100;  // PSN_2D_FEATURE_MAX_NUM_TRACK (:13)
constexpr int kT2dResBlocks = 3;         // chain result blocks used in turn by consecutive passes
constexpr double kFlowScale = 1.0;       // PSN_2D_OPTICALFLOW_SCALE (:18)
constexpr double kWinSizeRatio = 1.0;    // PSN_2D_FEATURE_WIN_SIZE_RATIO (:15)

Rect LocalSearchKLT(Rect preBox, const std::vector<Point2f> &preFeatures, const std::vector<Point2f> &curFeatures,
                    std::vector<size_t> &inlierFeatureIndex);
double BoxMatchingCost(const Rect &box1, const Rect &box2);
void ResultWithTracker(const Tracker2D &tracker, Object2DInfo &out);
// tracker2d_match.cpp: the assignment of Track2D_MatchingAndUpdating (inf
// handling + minimum-cost matching, :1040-1064) and the update (:1066-1164)
std::vector<int> AssignDetections(const std::vector<float> &cost, size_t rows, size_t cols);
// CPSNWhere_Hungarian::Match (helpers/PSNWhere_Hungarian.cpp:212-359): matched pairs in row-major order
bool HungarianMatch(const std::vector<float> &cost, size_t rows, size_t cols, std::vector<int> &outRows,
                    std::vector<int> &outCols, std::vector<float> &outCosts);
void MatchingAndUpdating(std::vector<DetectedObject> &dets, std::deque<Tracker2D *> &active,
                         std::list<Tracker2D> &storage, const std::vector<int> &match, unsigned frameIdx,
                         unsigned &newTrackerID, Track2DResult &result);

class Tracker2DFlow {
  public:
    Tracker2DFlow() = default;
    ~Tracker2DFlow() { Finalize(); }
    Tracker2DFlow(const Tracker2DFlow &) = delete;
    Tracker2DFlow &operator=(const Tracker2DFlow &) = delete;

    int Initialize(unsigned camID, int width, int height, int device);  // one camera
    int InitializeCameras(const std::vector<unsigned> &camIDs, int width, int height, int device);
    void Finalize();
    size_t NumCameras() const { return cams_.size(); }
    psn_lk_ctx *LkContext() const { return lk_; }

    // ---- single-camera flow-stage API (camera 0), the reference's call order:
    // PushFrame (frame t into the newest ring slot), the steps, RotateRing ----
    int PushFrame(const uint8_t *frame, int stride, int channels);  // cvtColor(BGR2GRAY) + resize 1.0
    int PushFrameDevice(const uint8_t *dev, int stride, int channels);  // frame already in device memory
    void RotateRing();  // buffer circulation at the end of Run
    // Feature extraction of the backward chain (:734-757) on frame t (the
    // newest ring slot): GridFAST masked by each detection's rectROI
    // (box.cropWithSize(cols, rows).cv(), :736), then the seeded shuffle + cap
    // to PSN_2D_FEATURE_MAX_NUM_TRACK. features[i] may hold < 4 points (the
    // backward step then skips detection i, :744).
    int DetectFeatures(const std::vector<Detection> &dets, uint32_t seed, std::vector<std::vector<Point2f>> &features);
    // Track2D_BackwardFeatureTracking for detections that passed the caller's
    // height gate; features[i] = detection i's points at t after shuffle + cap.
    // out = m_vecDetection2D.
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

    // ---- multi-camera Run (CPSNWhere_Tracker2D::Run of every camera) ----
    // StageFrame: frame t of camera `cam` is uploaded (host frames: async, a copy
    // engine for pinned memory) and its pyramid built on the ingest stream, into
    // the camera's next staging slot; launches adopt staged frames in push order
    // (up to kT2dStaging staged at once). May be called for frame t+1 between
    // RunLaunch(t) and RunComplete(t), and for frame t+2 as well once frame t+1
    // is staged (a pipelined driver uploads two frames ahead).
    int StageFrame(size_t cam, const uint8_t *frame, int stride, int channels, bool on_device);
    int StageFrameJpeg(size_t cam, const uint8_t *jpeg, size_t len);  // a baseline JPEG, decoded on the device
    int NextStagingSlot(size_t cam, int *slot);
    struct CamFrame {  // one camera's inputs and outputs of Run
        std::vector<Detection> dets;                      // height-validated detections of frame t
        std::vector<std::vector<Point2f>> features;       // in (given mode) / out (GridFAST mode)
        std::vector<DetectedObject> objects;              // out: m_vecDetection2D
        std::vector<float> cost;                          // out: matchingCostArray
        Track2DResult result;                             // out: m_stTrack2DResult
    };
    // Enqueue frame t's device work for every camera (features given, or GridFAST
    // on the device with `seed` when gridfast); RunComplete waits and runs the host
    // part: matching, tracker update, result packaging.
    int RunLaunch(unsigned frameIdx, std::vector<CamFrame> &io, bool gridfast, uint32_t seed);
    int RunComplete(std::vector<CamFrame> &io);
    // RunComplete of frame t that launches frame t+1 (next: its io, detections
    // set; its frames staged): its features and backward chains as soon as frame
    // t's device work is done, before the host part of frame t, its forward
    // calls after frame t's tracker update. The RunLaunch(nextFrameIdx, *next,
    // nextGridfast, .) that must follow only confirms it. Same results as
    // RunComplete(t) + RunLaunch(t+1).
    int RunComplete(std::vector<CamFrame> &io, std::vector<CamFrame> *next, unsigned nextFrameIdx, bool nextGridfast,
                    uint32_t nextSeed);
    // After a failed RunComplete: true when frame t itself was completed (its
    // results are in io) and only launching the next frame failed. The next
    // frame's staged images and the rings are then as before the call, so a
    // RunLaunch of that frame (e.g. with corrected detections) may follow.
    bool FrameCompleted() const { return frame_completed_; }
    const std::deque<Tracker2D *> &ActiveTrackers(size_t cam) const { return cams_[cam].active; }
    // diagnostic: accumulated host microseconds from RunComplete's entry to its
    // phases (copies + next chains enqueued, device done, unpacked, matched, next
    // forward enqueued) and the number of RunComplete calls; reset on read
    void HostTimes(double out[6]) {
        for (int i = 0; i < 5; i++) out[i] = host_us_[i], host_us_[i] = 0;
        out[5] = host_calls_;
        host_calls_ = 0;
    }
    // diagnostic: accumulated host microseconds of the matching phase's parts over
    // the cameras (overlap flags, forward matching costs, assignment, tracker
    // update + results); reset on read
    void HostMatchTimes(double out[4]) {
        for (int i = 0; i < 4; i++) out[i] = host_us_[5 + i], host_us_[5 + i] = 0;
    }

    // backward chain steps on the device (default) or on the host (single-camera API)
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
    struct Chain {  // one detection's backward chain (host-chain mode)
        size_t obj;
        std::vector<Point2f> curr, prev;
        std::vector<uint8_t> status;
        bool active;
    };
    struct Cam {  // per-camera state
        unsigned camID = 0;
        int ring[kT2dInterval];  // slot ids, oldest first; ring[kT2dInterval - 1] = frame t
        // slots outside the ring (multi-camera Run), FIFO: spares[0 .. nstaged) hold
        // staged frames in push order, the rest are free
        int spares[kT2dStaging];
        int nstaged = 0;
        // Run state: m_listTracker2D, m_queueActiveTracker2D, m_nNewTrackerID
        std::list<Tracker2D> storage;
        std::deque<Tracker2D *> active;
        unsigned newTrackerID = 0;
        std::vector<Tracker2D *> trackers;               // this frame's forward inputs
        size_t fwd_k0 = 0;  // first chain, in the pass that made them, of the detections they came from
        std::vector<std::vector<uint8_t>> fstatus;
        std::vector<Job> fwd;
    };
    // One device pass over several cameras: GridFAST (optional) + the backward
    // chains of every detection + the forward calls of every tracker.
    struct PassCam {
        size_t cam;
        const std::vector<Detection> *dets;
        std::vector<std::vector<Point2f>> *features;  // in, or out with gridfast
        std::vector<DetectedObject> *out;
        std::vector<Job> *fwd;
        size_t k0, j0, f0;  // first chain / forward job / forward point of this camera in the pass
        int set;            // the pass's staging set of chain inputs
        int rb = -1;        // the pass's result block
        int fwd_rb = -1;    // the result block its forward calls read (LaunchForwardFromChains), or -1
        size_t fwd_n = 0;   // forward outputs to copy back (that launch's index range)
        int fwd_par = 0;    // the forward output block its forward launch wrote
    };
    int PassLaunch(std::vector<PassCam> &pc, bool gridfast, uint32_t seed);  // chains, then forward
    int PassLaunchChains(std::vector<PassCam> &pc, bool gridfast, uint32_t seed);
    int PassLaunchForward(std::vector<PassCam> &pc);
    int LaunchForwardFromChains(std::vector<PassCam> &pc, int src_rb, bool host_fallback);
    static int forward_window_error(int w, int h);
    // what a chain pass leaves for the next frame's forward launch
    struct ChainInfo {
        bool valid = false;
        size_t K = 0;
        std::vector<size_t> k0, ndet;                // per camera
        std::vector<std::pair<int, int>> win;        // per chain: the forward window of the detection's box
    };
    ChainInfo chain_info_[kT2dResBlocks];
    int next_rb_ = 0, last_rb_ = -1;
    int trk_rb_ = -1;  // the result block holding the current trackers' set 0 (their next forward call)
    void *ev_set0_[3] = {nullptr, nullptr, nullptr};   // hipEvent_t: a block's set 0 is final (chain stream)
    void *ev_fread_[3] = {nullptr, nullptr, nullptr};  // hipEvent_t: the forward launch reading a block is done
    // Forward outputs alternate between two device blocks, so that a frame's
    // result copy (on its chain stream) never sits between two forward launches
    // on the forward stream: ev_fend_[p] = forward launch into block p done,
    // ev_fcopied_[p] = block p copied to the host (the next launch into p waits)
    int fwd_par_ = 0;
    void *ev_fend_[2] = {nullptr, nullptr}, *ev_fcopied_[2] = {nullptr, nullptr};
    bool fread_rec_[3] = {false, false, false};
    int PassComplete(std::vector<PassCam> &pc, bool gridfast);  // PassWait + PassFeatures + PassUnpack
    int PassWait(std::vector<PassCam> &pc);  // PassCopy + PassSync
    int PassCopy(std::vector<PassCam> &pc);  // enqueue the result copies, record the completion events
    int PassSync();                          // wait for them
    int PassFeatures(std::vector<PassCam> &pc, bool gridfast);
    void PassUnpack(std::vector<PassCam> &pc);
    bool ChainsFit(const std::vector<CamFrame> &io) const;

    int RunJobs(std::vector<Job> &jobs);
    int fail(int rc, const char *what);
    void BackwardBegin(const std::vector<Detection> &dets, const std::vector<std::vector<Point2f>> &features,
                       std::vector<DetectedObject> &out, std::vector<Chain> &chains);
    void BackwardJobs(int step, std::vector<Chain> &chains, const std::vector<DetectedObject> &out,
                      std::vector<Job> &jobs);
    void BackwardStepDone(std::vector<Chain> &chains, std::vector<DetectedObject> &out);
    void BackwardEnd(std::vector<DetectedObject> &out, const std::vector<std::vector<Point2f>> &features);
    int StepsAvailable(size_t cam) const;  // chain steps the camera's ring holds frames for (0..3)
    bool StepAvailable(int step) const { return step <= StepsAvailable(0); }
    int EnsureChains(size_t nchains);
    int EnsureForward(size_t nfwd_pts, size_t nfwd_jobs);
    void ForwardJobs(size_t cam, const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                     std::vector<Job> &jobs);
    void ForwardDone(const std::vector<Tracker2D *> &trackers, std::vector<std::vector<uint8_t>> &status,
                     const std::vector<DetectedObject> &dets, std::vector<float> &cost);
    int DevicePass(const std::vector<Detection> &dets, std::vector<std::vector<Point2f>> &features,
                   std::vector<DetectedObject> &out, std::vector<Job> *fwd, bool gridfast, uint32_t seed);

    psn_lk_ctx *lk_ = nullptr;
    void *fwd_stream_ = nullptr;    // hipStream_t of the forward launch, beside the chain's launches (lowest priority)
    // consecutive forward launches alternate between fwd_stream_ (output block 0)
    // and fwd_stream2_ (block 1): a frame's forward may start while the last
    // one's slowest workgroups still run
    void *fwd_stream2_ = nullptr;
    void *FwdStream(int par) const { return par ? fwd_stream2_ : fwd_stream_; }
    void SyncForward();
    // the backward chains (highest priority): pass i of the staging set si runs on
    // chain_streams_[si], so the chains of frame t+1 start beside frame t's last steps
    void *ev_gf_ = nullptr;  // after a pass's GridFAST launches (the context's detector scratch)
    bool gf_rec_ = false;
    void *chain_streams_[2] = {nullptr, nullptr};
    void *ChainStream(int si) const { return chain_streams_[si & 1]; }
    void SyncChains();
    std::vector<psn_lk_query> fwd_queries_;
    std::vector<Cam> cams_;
    int width_ = 0, height_ = 0;
    std::vector<char> filled_;  // per LK slot
    std::string err_;
    // batched-call staging
    std::vector<float> xy_in_, xy_out_, err_out_, gf_xy_;
    std::vector<uint8_t> st_out_;
    std::vector<psn_lk_query> queries_;
    // per chain of a pass (per staging set): window the LK cannot run (error only if the chain has points)
    std::vector<char> win_bad_sets_[2];
    int stage_ = 0;  // staging set of the next chain launch
    void *ev_chain_ = nullptr, *ev_fwd_ = nullptr;  // hipEvent_t: a pass's result copies done
    bool wait_chain_ = false, wait_fwd_ = false;
    int AdoptFrames(std::vector<CamFrame> &io, bool gridfast, std::vector<PassCam> &pass);
    void UnadoptFrames();  // AdoptFrames undone: frame t's slot back to staging, the oldest back in the ring
    bool frame_completed_ = false;
    std::vector<PassCam> run_pass_;  // the pass between RunLaunch and RunComplete
    std::vector<CamFrame> *pre_io_ = nullptr;  // the io of a frame RunComplete launched ahead
    bool launched_ahead_ = false;              // run_pass_ is that frame, awaiting its RunLaunch
    double host_us_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    long host_calls_ = 0;
    unsigned run_frame_ = 0;
    bool run_gridfast_ = false;
    bool device_chain_ = true;
    struct DeviceBuffers;
    DeviceBuffers *dev_ = nullptr;
};

}  // namespace psn
