// C++ boundary types of the Tracker2D flow stage: the arithmetic of
// PSNWhere_Types.h:18-209 (PSN_Point2D, PSN_Rect, stDetection, stObject2DInfo,
// stTrack2DResult) and the per-instance records of PSNWhere_Tracker2D.h:17-47,
// without OpenCV types (cv::Point2f -> Point2f, cv::Mat cost -> vector).
#pragma once

#include <algorithm>
#include <cmath>
#include <deque>
#include <vector>

namespace psn {

struct Point2f {  // cv::Point2f
    float x = 0.f, y = 0.f;
};

struct Point2D {  // PSN_Point2D (double)
    double x = 0.0, y = 0.0;
    Point2D() = default;
    Point2D(double x_, double y_) : x(x_), y(y_) {}
    explicit Point2D(Point2f p) : x((double)p.x), y((double)p.y) {}
    Point2D operator-(const Point2D &a) const { return Point2D(x - a.x, y - a.y); }
    double norm_L2() const { return std::sqrt(x * x + y * y); }
};

struct Rect {  // PSN_Rect (PSNWhere_Types.h:112-182)
    double x = 0.0, y = 0.0, w = 0.0, h = 0.0;
    Rect() = default;
    Rect(double x_, double y_, double w_, double h_) : x(x_), y(y_), w(w_), h(h_) {}
    // centre uses ceil(w/2) (:131-132)
    Point2D center() const { return Point2D(x + std::ceil(w / 2.0), y + std::ceil(h / 2.0)); }
    Point2D bottomCenter() const { return Point2D(x + std::ceil(w / 2.0), y + h); }
    Rect scale(double s) const { return Rect(x * s, y * s, w * s, h * s); }
    Rect cropWithSize(double width, double height) const {
        const double nx = std::max(0.0, x), ny = std::max(0.0, y);
        return Rect(nx, ny, std::min(width - nx - 1, w), std::min(height - ny - 1, h));
    }
    double area() const { return w * h; }
    bool contain(Point2f a) const {
        return (double)a.x >= x && (double)a.x < x + w && (double)a.y >= y && (double)a.y < y + h;
    }
    // strict '<' (:161-164)
    bool overlap(const Rect &a) const {
        return (std::max(x + w, a.x + a.w) - std::min(x, a.x) < w + a.w) &&
               (std::max(y + h, a.y + a.h) - std::min(y, a.y) < h + a.h);
    }
    // |(cx, cy, w) - (a.cx, a.cy, a.w)| / min(w, a.w) with cx = x + w/2 (:165-170)
    double distance(const Rect &a) const {
        const double dx = (x + w / 2.0) - (a.x + a.w / 2.0), dy = (y + h / 2.0) - (a.y + a.h / 2.0), dz = w - a.w;
        return std::sqrt(dx * dx + dy * dy + dz * dz) / std::min(w, a.w);
    }
    double overlappedArea(const Rect &a) const {
        const double ow = std::min(x + w, a.x + a.w) - std::max(x, a.x);
        if (0.0 >= ow) return 0.0;
        const double oh = std::min(y + h, a.y + a.h) - std::max(y, a.y);
        if (0.0 >= oh) return 0.0;
        return ow * oh;
    }
};

struct Detection {  // stDetection
    Rect box;
    std::vector<Rect> vecPartBoxes;  // .front() = the head box (PETS part boxes)
    // the caller's 3D estimate of the detection (EstimateDetectionHeight with the
    // camera calibration, PSNWhere_Tracker2D.cpp:711-718; calibration is not on
    // the flow path): stDetectedObject::location / height
    double location[3] = {0, 0, 0};
    double height = 0.0;
};

struct DetectedObject {  // stDetectedObject (PSNWhere_Tracker2D.h:17-29)
    unsigned id = 0;
    Detection detection;
    bool bMatchedWithTracker = false;
    bool bOverlapWithOtherDetection = false;
    std::vector<std::vector<Point2f>> vecvecTrackedFeatures;  // current -> past
    std::vector<Rect> boxes;                                  // current -> past
    double location[3] = {0, 0, 0};
    double height = 0.0;
};

struct Tracker2D {  // stTracker2D (.h:31-47)
    unsigned id = 0, timeStart = 0, timeEnd = 0, timeLastUpdate = 0, duration = 0, numStatic = 0;
    double confidence = 0.0;
    std::deque<Rect> boxes, heads;
    std::vector<Point2f> featurePoints, trackedPoints;
    double lastPosition[3] = {0, 0, 0};
    double height = 0.0;
    int srcDet = -1;  // the detection (index in its frame) that last set featurePoints (this build)
};

struct Object2DInfo {  // stObject2DInfo (PSNWhere_Types.h:190-198)
    unsigned id = 0;
    Rect box, head;
    double score = 0.0;
    std::vector<Point2f> featurePointsPrev, featurePointsCurr;
};

struct Track2DResult {  // stTrack2DResult (PSNWhere_Types.h:200-209)
    unsigned camID = 0, frameIdx = 0;
    std::vector<Object2DInfo> object2DInfos;
    std::vector<Rect> vecDetectionRects, vecTrackerRects;
    int costRows = 0, costCols = 0;
    std::vector<float> matMatchingCost;  // costRows x costCols, row-major
};

}  // namespace psn
