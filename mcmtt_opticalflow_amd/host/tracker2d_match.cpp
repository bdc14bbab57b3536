// Tracker2D matching, tracker update and result packaging: the host stage of
// CPSNWhere_Tracker2D::Run after the flow (psn_where/PSNWhere_Tracker2D.cpp
// :1038-1164 Track2D_MatchingAndUpdating, :1231-1257 ResultWithTracker). It
// consumes the matching cost of the forward step and produces the
// stTrack2DResult that feeds CPSNWhere_Associator3D (PSNWhere.cpp:264-269).
#include <algorithm>
#include <cmath>
#include <limits>

#include "tracker2d_flow.hpp"

namespace psn {

namespace {
constexpr unsigned kMaxTrackletLength = 3;       // PSN_2D_MAX_TRACKLET_LENGTH (:10)
constexpr double kMaxDetectionDistance = 600.0;  // PSN_2D_MAX_DETECTION_DISTANCE (:23), mm
constexpr double kMaxHeightDifference = 400.0;   // PSN_2D_MAX_HEIGHT_DIFFERENCE (:24), mm

// Minimum-total-cost assignment of min(n, m) pairs on an n x m matrix of finite
// costs, n <= m (shortest augmenting paths with potentials, double arithmetic).
// Returns the column of every row.
std::vector<int> MinCostRows(const std::vector<double> &a, size_t n, size_t m) {
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<double> u(n + 1, 0.0), v(m + 1, 0.0);
    std::vector<size_t> p(m + 1, 0), way(m + 1, 0);
    for (size_t i = 1; i <= n; i++) {
        p[0] = i;
        size_t j0 = 0;
        std::vector<double> minv(m + 1, inf);
        std::vector<char> used(m + 1, 0);
        do {
            used[j0] = 1;
            const size_t i0 = p[j0];
            double delta = inf;
            size_t j1 = 0;
            for (size_t j = 1; j <= m; j++) {
                if (used[j]) continue;
                const double cur = a[(i0 - 1) * m + (j - 1)] - u[i0] - v[j];
                if (cur < minv[j]) {
                    minv[j] = cur;
                    way[j] = j0;
                }
                if (minv[j] < delta) {
                    delta = minv[j];
                    j1 = j;
                }
            }
            for (size_t j = 0; j <= m; j++) {
                if (used[j]) {
                    u[p[j]] += delta;
                    v[j] -= delta;
                } else {
                    minv[j] -= delta;
                }
            }
            j0 = j1;
        } while (p[j0] != 0);
        do {
            const size_t j1 = way[j0];
            p[j0] = p[j1];
            j0 = j1;
        } while (j0);
    }
    std::vector<int> row(n, -1);
    for (size_t j = 1; j <= m; j++)
        if (p[j]) row[p[j] - 1] = (int)(j - 1);
    return row;
}
}  // namespace

// :1040-1060 + the Hungarian (helpers/PSNWhere_Hungarian.cpp Match): non-finite
// costs become max(finite) + 100 (-900 when none is finite), a minimum-total
// cost assignment of min(rows, cols) pairs is taken over the whole matrix, and
// pairs whose cost is that substitute are dropped (:1064).
std::vector<int> AssignDetections(const std::vector<float> &costIn, size_t rows, size_t cols) {
    std::vector<int> match(rows, -1);
    if (rows == 0 || cols == 0) return match;
    std::vector<float> cost(costIn.begin(), costIn.begin() + (ptrdiff_t)(rows * cols));
    float maxCost = -1000.0f;
    for (float c : cost)
        if (std::isfinite(c) && maxCost < c) maxCost = c;
    maxCost = maxCost + 100.0f;
    for (float &c : cost)
        if (!std::isfinite(c)) c = maxCost;
    const bool tr = rows > cols;  // the solver wants rows <= cols
    const size_t n = tr ? cols : rows, m = tr ? rows : cols;
    std::vector<double> a(n * m);
    for (size_t i = 0; i < n; i++)
        for (size_t j = 0; j < m; j++) a[i * m + j] = (double)(tr ? cost[j * cols + i] : cost[i * cols + j]);
    const std::vector<int> r = MinCostRows(a, n, m);
    for (size_t i = 0; i < n; i++) {
        if (r[i] < 0) continue;
        const size_t d = tr ? (size_t)r[i] : i, t = tr ? i : (size_t)r[i];
        if (maxCost == cost[d * cols + t]) continue;
        match[d] = (int)t;
    }
    return match;
}

// :1062-1164. dets = m_vecDetection2D (after the backward step), active =
// m_queueActiveTracker2D (after the forward step), match[d] = tracker of
// detection d (AssignDetections). Matched trackers take the detection's box and
// head, are packed into the result, then take the detection's features;
// unmatched detections start new trackers (ids from newTrackerID); trackers
// not updated this frame end. active becomes the new queue: matched trackers in
// detection order, then the new ones.
void MatchingAndUpdating(std::vector<DetectedObject> &dets, std::deque<Tracker2D *> &active,
                         std::list<Tracker2D> &storage, const std::vector<int> &match, unsigned frameIdx,
                         unsigned &newTrackerID, Track2DResult &result) {
    result.object2DInfos.clear();
    result.frameIdx = frameIdx;
    std::deque<Tracker2D *> next;
    for (size_t d = 0; d < dets.size(); d++) {
        if (match[d] < 0) continue;
        DetectedObject &det = dets[d];
        Tracker2D *tr = active[(size_t)match[d]];
        const double dx = det.location[0] - tr->lastPosition[0], dy = det.location[1] - tr->lastPosition[1],
                     dz = det.location[2] - tr->lastPosition[2];
        if (std::sqrt(dx * dx + dy * dy + dz * dz) > kMaxDetectionDistance) continue;  // :1074
        if (std::abs(det.height - tr->height) > kMaxHeightDifference) continue;         // :1076
        if (tr->duration > kMaxTrackletLength) continue;                                 // :1080
        det.bMatchedWithTracker = true;
        tr->timeEnd = frameIdx;
        tr->timeLastUpdate = frameIdx;
        tr->duration = tr->timeEnd - tr->timeStart + 1;
        tr->numStatic = 0;
        tr->boxes.back() = det.detection.box;
        tr->heads.back() = det.detection.vecPartBoxes.empty() ? Rect() : det.detection.vecPartBoxes.front();
        tr->confidence = 1.0;
        for (int k = 0; k < 3; k++) tr->lastPosition[k] = det.location[k];
        tr->height = det.height;
        next.push_back(tr);
        Object2DInfo info;
        ResultWithTracker(*tr, info);
        result.object2DInfos.push_back(std::move(info));
        tr->featurePoints = det.vecvecTrackedFeatures.front();
        tr->trackedPoints.clear();
    }
    for (DetectedObject &det : dets) {
        if (det.bMatchedWithTracker) continue;
        Tracker2D nt;
        nt.id = newTrackerID++;
        nt.timeStart = nt.timeEnd = nt.timeLastUpdate = frameIdx;
        nt.duration = 1;
        nt.numStatic = 0;
        nt.boxes.push_back(det.detection.box);
        nt.heads.push_back(det.detection.vecPartBoxes.empty() ? Rect() : det.detection.vecPartBoxes.front());
        nt.featurePoints = det.vecvecTrackedFeatures.front();
        nt.confidence = 1.0;
        for (int k = 0; k < 3; k++) nt.lastPosition[k] = det.location[k];
        nt.height = det.height;
        storage.push_back(std::move(nt));
        next.push_back(&storage.back());
        Object2DInfo info;
        ResultWithTracker(storage.back(), info);
        result.object2DInfos.push_back(std::move(info));
    }
    // terminated trackers (:1152-1164) leave the storage (the reference keeps
    // them with cleared vectors; nothing reads them again)
    for (Tracker2D *t : active)
        if (t->timeLastUpdate != frameIdx)
            for (auto it = storage.begin(); it != storage.end(); ++it)
                if (&*it == t) {
                    storage.erase(it);
                    break;
                }
    active.swap(next);
    // vecDetectionRects / vecTrackerRects are never filled by the reference, so
    // matMatchingCost is D x 0 (:1173)
    result.vecDetectionRects.clear();
    result.vecTrackerRects.clear();
    result.costRows = (int)dets.size();
    result.costCols = 0;
    result.matMatchingCost.clear();
}

}  // namespace psn
