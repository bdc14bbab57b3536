// tests/cpp/psnwhere_tracker2d.cpp -- a compiled C++ caller of the drop-in
// boundary, shaped like the reference's CPSNWhere_Tracker2D
// (psn_where/PSNWhere_Tracker2D.h:135-140) after the INTEGRATION.md edits:
//   Initialize(camID, calib)  -> psn_t2d_group_create (one camera: the ring of
//                                4 pyramids)
//   Run(dets, frame, frameIdx) -> ingest (section 2), GridFAST features (3b),
//                                backward chains + forward LK + matching + tracker
//                                update + ResultWithTracker (3, 3c, 3c', 3c''),
//                                FilePrintResult (PSNWhere_Tracker2D.cpp:370 ->
//                                psn_t2d_write_result_txt, 3d); returns the
//                                member stTrack2DResult by reference, as :373 does
//   Finalize()                -> psn_t2d_group_destroy
// Types follow PSNWhere_Types.h:112-209 (PSN_Rect, stDetection, stObject2DInfo,
// stTrack2DResult); cv::Mat and cv::Point2f are replaced by the fields Run
// reads. The calibration-dependent 3D estimate (EstimateDetectionHeight,
// :711-718) stays with the caller, as the boundary has it: the stand-in
// calibration below gives every detection the estimate the repo's tests and
// bench use.
//
// Test harness only (tests/test_cpp_boundary.py builds and runs it); it
// includes include/psn_tracker2d.h and links libpsn_tracker2d.so like the
// reference would. Usage:
//   psnwhere_tracker2d <in_dir> <out_dir/>
// in_dir/meta.txt:  "width height nframes camID"
// in_dir/dets.txt:  per detection "frame x y w h hx hy hw hh"
// in_dir/frame%04d.bgr: width x height x 3 BGR bytes
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "psn_tracker2d.h"

// ---- PSNWhere_Types.h (the fields the boundary carries) ----
struct PSN_Rect {
    double x = 0, y = 0, w = 0, h = 0;
    PSN_Rect() = default;
    PSN_Rect(double x_, double y_, double w_, double h_) : x(x_), y(y_), w(w_), h(h_) {}
};
struct Point2f {
    float x, y;
};
struct stDetection {
    PSN_Rect box;
    std::vector<PSN_Rect> vecPartBoxes;
};
struct stObject2DInfo {
    unsigned int id;
    PSN_Rect box, head;
    double score;
    std::vector<Point2f> featurePointsPrev, featurePointsCurr;
};
struct stTrack2DResult {
    unsigned int camID = 0, frameIdx = 0;
    std::vector<stObject2DInfo> object2DInfos;
    std::vector<PSN_Rect> vecDetectionRects, vecTrackerRects;
};
// cv::Mat: what Run reads of the frame (BGR, 8UC3)
struct Mat {
    unsigned char *data = nullptr;
    int rows = 0, cols = 0, step = 0;
    int channels() const { return 3; }
};
// stCalibrationInfo: the image size (cCamModel.width() / height(), :118-119) and
// the caller's 3D estimate of a detection (the role of EstimateDetectionHeight)
struct stCalibrationInfo {
    int width, height;
    void estimate(const PSN_Rect &b, double loc[3], double *height_mm) const {
        loc[0] = (b.x + b.w / 2) * 10.0;
        loc[1] = (b.y + b.h) * 10.0;
        loc[2] = 0.0;
        *height_mm = 1700.0;
    }
};

class CPSNWhere_Tracker2D {
  public:
    bool Initialize(unsigned int nCamID, stCalibrationInfo *stCalibInfo) {
        m_nCamID = nCamID;
        m_calib = *stCalibInfo;
        m_stTrack2DResult.camID = nCamID;
        m_objects.resize(kMaxObjects);
        const int rc = psn_t2d_group_create(/*device=*/0, 1, &m_nCamID, m_calib.width, m_calib.height, &m_group);
        if (rc) std::fprintf(stderr, "psn_t2d_group_create: %d\n", rc);
        return rc == 0;
    }
    void Finalize() {
        if (m_group) psn_t2d_group_destroy(m_group);
        m_group = nullptr;
    }
    stTrack2DResult &Run(std::vector<stDetection> curDetectionResult, Mat *curFrame, unsigned int frameIdx) {
        m_rc = 0;
        // ingest (:256-263): BGR -> gray + pyramid on the device
        if ((m_rc = psn_t2d_group_push_frame(m_group, 0, curFrame->data, curFrame->step, curFrame->channels()))) {
            std::fprintf(stderr, "push_frame: %s\n", psn_t2d_group_last_error(m_group));
            return m_stTrack2DResult;
        }
        // the detections with the caller's 3D estimate; features from GridFAST (:734-757)
        m_dets.assign(curDetectionResult.size(), psn_t2d_detection{});
        for (size_t i = 0; i < curDetectionResult.size(); i++) {
            const stDetection &d = curDetectionResult[i];
            psn_t2d_detection &r = m_dets[i];
            r.box = psn_rect{d.box.x, d.box.y, d.box.w, d.box.h};
            const PSN_Rect &hd = d.vecPartBoxes.empty() ? d.box : d.vecPartBoxes.front();
            r.head = psn_rect{hd.x, hd.y, hd.w, hd.h};
            m_calib.estimate(d.box, r.location, &r.height);
        }
        psn_t2d_detection *per_cam[1] = {m_dets.data()};
        const int ndet[1] = {(int)m_dets.size()};
        psn_track2d_result res{};
        res.objects = m_objects.data();
        res.cap_objects = kMaxObjects;
        m_rc = psn_t2d_group_run(m_group, frameIdx, per_cam, ndet, PSN_T2D_FEATURES_GRIDFAST, /*seed=*/frameIdx, &res);
        if (m_rc) {
            std::fprintf(stderr, "group_run: %s\n", psn_t2d_group_last_error(m_group));
            return m_stTrack2DResult;
        }
        // stTrack2DResult (the member Run returns by reference, :373)
        m_stTrack2DResult.camID = res.cam_id;
        m_stTrack2DResult.frameIdx = res.frame_idx;
        m_stTrack2DResult.object2DInfos.clear();
        for (int k = 0; k < res.num_objects; k++) {
            const psn_object2d &o = res.objects[k];
            stObject2DInfo info;
            info.id = o.id;
            info.box = PSN_Rect(o.box.x, o.box.y, o.box.w, o.box.h);
            info.head = PSN_Rect(o.head.x, o.head.y, o.head.w, o.head.h);
            info.score = o.score;
            for (int j = 0; j < o.num_prev; j++) info.featurePointsPrev.push_back(Point2f{o.prev[j][0], o.prev[j][1]});
            for (int j = 0; j < o.num_curr; j++) info.featurePointsCurr.push_back(Point2f{o.curr[j][0], o.curr[j][1]});
            m_stTrack2DResult.object2DInfos.push_back(info);
        }
        m_stTrack2DResult.vecDetectionRects.clear();
        m_stTrack2DResult.vecTrackerRects.clear();
        // FilePrintResult (:370)
        if (!m_out_dir.empty() && (m_rc = psn_t2d_write_result_txt(m_out_dir.c_str(), &res)))
            std::fprintf(stderr, "write_result_txt: %d\n", m_rc);
        return m_stTrack2DResult;
    }
    int last_rc() const { return m_rc; }
    std::string m_out_dir;

  private:
    static constexpr int kMaxObjects = 64;
    unsigned int m_nCamID = 0;
    stCalibrationInfo m_calib{};
    psn_t2d_group *m_group = nullptr;
    std::vector<psn_t2d_detection> m_dets;
    std::vector<psn_object2d> m_objects;
    stTrack2DResult m_stTrack2DResult;
    int m_rc = 0;
};

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <in_dir> <out_dir/>\n", argv[0]);
        return 2;
    }
    const std::string in = argv[1];
    int W = 0, H = 0, T = 0;
    unsigned cam = 0;
    FILE *f = std::fopen((in + "/meta.txt").c_str(), "r");
    if (!f || std::fscanf(f, "%d %d %d %u", &W, &H, &T, &cam) != 4) return 3;
    std::fclose(f);
    std::vector<std::vector<stDetection>> dets(T);
    f = std::fopen((in + "/dets.txt").c_str(), "r");
    if (!f) return 3;
    int t;
    double b[8];
    while (std::fscanf(f, "%d %lf %lf %lf %lf %lf %lf %lf %lf", &t, b, b + 1, b + 2, b + 3, b + 4, b + 5, b + 6, b + 7) == 9) {
        if (t < 0 || t >= T) return 3;
        stDetection d;
        d.box = PSN_Rect(b[0], b[1], b[2], b[3]);
        d.vecPartBoxes.push_back(PSN_Rect(b[4], b[5], b[6], b[7]));
        dets[t].push_back(d);
    }
    std::fclose(f);

    stCalibrationInfo calib{W, H};
    CPSNWhere_Tracker2D tracker;
    tracker.m_out_dir = argv[2];
    if (!tracker.Initialize(cam, &calib)) return 4;
    std::vector<unsigned char> buf((size_t)W * H * 3);
    int rc = 0;
    for (t = 0; t < T && !rc; t++) {
        char name[64];
        std::snprintf(name, sizeof name, "/frame%04d.bgr", t);
        f = std::fopen((in + name).c_str(), "rb");
        if (!f || std::fread(buf.data(), 1, buf.size(), f) != buf.size()) return 3;
        std::fclose(f);
        Mat frame;
        frame.data = buf.data();
        frame.rows = H;
        frame.cols = W;
        frame.step = 3 * W;
        const stTrack2DResult &r = tracker.Run(dets[t], &frame, (unsigned)t);
        rc = tracker.last_rc();
        size_t npts = 0;
        for (const stObject2DInfo &o : r.object2DInfos) npts += o.featurePointsCurr.size();
        std::printf("frame %d cam %u: %zu objects, %zu tracked points\n", r.frameIdx, r.camID, r.object2DInfos.size(), npts);
    }
    tracker.Finalize();
    return rc ? 5 : 0;
}
