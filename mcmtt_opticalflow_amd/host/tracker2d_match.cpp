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

// Munkres on a square float matrix, in CPSNWhere_Hungarian's own order
// (helpers/PSNWhere_Hungarian.cpp steps :405-675): every scan row-major, exact
// zero tests, float32 updates -- ties resolve as the reference resolves them.
// Marks and covers are small integers/flags here (the reference keeps them as
// floats 0/1/2; only their equality tests are used).
class Munkres {
  public:
    enum : uint8_t { kNone = 0, kStar = 1, kPrime = 2 };

    Munkres(std::vector<float> p, size_t n) : n_(n), p_(std::move(p)), mark_(n * n, kNone), rcov_(n, 0), ccov_(n, 0) {}

    // step 2 (:426-458): star the first zero of each row whose column has no star yet
    void StarZeros() {
        std::vector<char> rs(n_, 0), cs(n_, 0);
        for (size_t r = 0; r < n_; r++)
            for (size_t c = 0; c < n_; c++)
                if (P(r, c) == 0.0f && !rs[r] && !cs[c]) {
                    mark_[r * n_ + c] = kStar;
                    rs[r] = cs[c] = 1;
                }
        ClearCovers();
    }

    // step 3 (:465-480): cover the starred columns; true when all of them are
    bool CoverStarredColumns() {
        size_t covered = 0;
        for (size_t c = 0; c < n_; c++) {
            ccov_[c] = 0;
            for (size_t r = 0; r < n_; r++)
                if (mark_[r * n_ + c] == kStar) ccov_[c] = 1;
            covered += (size_t)ccov_[c];
        }
        return covered == n_;
    }

    // step 4 (:491-544): prime the first uncovered zero (row-major) until one lands
    // in a row without a star (returned through r0/c0: step 5) or none is left
    // (false: step 6). A prime beside a star covers its row, uncovers the star's column.
    bool PrimeZeros(size_t &r0, size_t &c0) {
        for (;;) {
            bool found = false;
            for (size_t r = 0; r < n_ && !found; r++) {
                if (rcov_[r]) continue;
                for (size_t c = 0; c < n_; c++)
                    if (P(r, c) == 0.0f && !ccov_[c]) {
                        r0 = r;
                        c0 = c;
                        found = true;
                        break;
                    }
            }
            if (!found) return false;
            mark_[r0 * n_ + c0] = kPrime;
            bool star = false;
            for (size_t c = 0; c < n_; c++)
                if (mark_[r0 * n_ + c] == kStar) {
                    star = true;
                    ccov_[c] = 0;
                }
            if (!star) return true;
            rcov_[r0] = 1;
        }
    }

    // step 5 (:557-631): alternate star (in the prime's column) / prime (in the
    // star's row) from (r0, c0); flip the path, erase primes, clear covers
    void Augment(size_t r0, size_t c0) {
        std::vector<std::pair<size_t, size_t>> path{{r0, c0}};
        for (;;) {
            const size_t col = path.back().second;
            size_t r = n_;
            for (size_t i = 0; i < n_; i++)
                if (mark_[i * n_ + col] == kStar) {
                    r = i;
                    break;
                }
            if (r == n_) break;
            path.push_back({r, col});
            size_t pc = 0;
            for (size_t c = 0; c < n_; c++)
                if (mark_[r * n_ + c] == kPrime) {
                    pc = c;
                    break;
                }
            path.push_back({r, pc});
        }
        for (const auto &e : path) {
            uint8_t &m = mark_[e.first * n_ + e.second];
            m = m == kStar ? kNone : kStar;
        }
        for (uint8_t &m : mark_)
            if (m == kPrime) m = kNone;
        ClearCovers();
    }

    // step 6 (:639-675): min uncovered value added to covered rows, subtracted from
    // uncovered columns -- one float bias per entry (row bias + column bias)
    void Adjust() {
        float fmin = std::numeric_limits<float>::infinity();
        for (size_t r = 0; r < n_; r++) {
            if (rcov_[r]) continue;
            for (size_t c = 0; c < n_; c++)
                if (!ccov_[c] && P(r, c) < fmin) fmin = P(r, c);
        }
        for (size_t r = 0; r < n_; r++) {
            const float rb = rcov_[r] ? fmin : 0.0f;
            for (size_t c = 0; c < n_; c++) {
                const float cb = ccov_[c] ? 0.0f : -fmin;
                P(r, c) += rb + cb;
            }
        }
    }

    // step 1 (:405-419): rows minus their minimum (rows at 0 or inf left alone)
    void SubtractRowMinima() {
        for (size_t r = 0; r < n_; r++) {
            float m = P(r, 0);
            for (size_t c = 1; c < n_; c++) m = std::min(m, P(r, c));
            if (m == 0.0f || m == std::numeric_limits<float>::infinity()) continue;
            for (size_t c = 0; c < n_; c++) P(r, c) -= m;
        }
    }

    // minLineCover (:677-709): steps 2, 3 and 4 once on an edge matrix; the
    // deficiency = n minus the covered lines
    size_t Deficiency() {
        StarZeros();
        (void)CoverStarredColumns();
        size_t r0, c0;
        (void)PrimeZeros(r0, c0);
        size_t lines = 0;
        for (size_t i = 0; i < n_; i++) lines += (size_t)rcov_[i] + (size_t)ccov_[i];
        return n_ - lines;
    }

    // Match's main loop (:298-330): 1, 2, then 3 -> 4 -> (5 -> 3 | 6 -> 4) until 3
    // covers every column. Each step-6 round creates an uncovered zero (x - x), so
    // it terminates; the bound only guards malformed (inf - inf) inputs.
    bool Solve() {
        SubtractRowMinima();
        StarZeros();
        size_t guard = 0;
        const size_t limit = 64 + 8 * n_ * n_ * n_;
        while (!CoverStarredColumns()) {
            size_t r0, c0;
            while (!PrimeZeros(r0, c0)) {
                Adjust();
                if (++guard > limit) return false;
            }
            Augment(r0, c0);
        }
        return true;
    }

    bool Starred(size_t r, size_t c) const { return mark_[r * n_ + c] == kStar; }

  private:
    float &P(size_t r, size_t c) { return p_[r * n_ + c]; }
    void ClearCovers() {
        std::fill(rcov_.begin(), rcov_.end(), 0);
        std::fill(ccov_.begin(), ccov_.end(), 0);
    }
    size_t n_;
    std::vector<float> p_;
    std::vector<uint8_t> mark_;
    std::vector<char> rcov_, ccov_;
};
}  // namespace

// CPSNWhere_Hungarian Initialize(std::vector<float>, rows, cols) + Match()
// (helpers/PSNWhere_Hungarian.cpp:67-89, :212-359; called at PSNWhere_Tracker2D.cpp:1059): infinity pre-processing
// (:711-735), condensed matrix padded by the minimum line cover of its finite
// entries (:241-289), Munkres, then the starred pairs of the first rows x cols
// entries whose cost is finite after the post-processing (:737-747, :339-354).
// Pairs in row-major order. A NaN cost (:78-81) or an empty matrix matches nothing.
bool HungarianMatch(const std::vector<float> &costIn, size_t rows, size_t cols, std::vector<int> &outRows,
                    std::vector<int> &outCols, std::vector<float> &outCosts) {
    outRows.clear();
    outCols.clear();
    outCosts.clear();
    if (rows * cols == 0) return true;
    std::vector<float> cost(costIn.begin(), costIn.begin() + (ptrdiff_t)(rows * cols));
    for (float v : cost)
        if (std::isnan(v)) return true;
    std::vector<char> fin(rows * cols);
    float finiteSum = 0.0f;
    for (size_t i = 0; i < rows * cols; i++) {
        fin[i] = std::isfinite(cost[i]) ? 1 : 0;
        if (fin[i]) finiteSum += cost[i];
    }
    const float repl = std::numeric_limits<float>::max() - finiteSum;
    for (size_t i = 0; i < rows * cols; i++)
        if (!fin[i]) cost[i] = repl;
    std::vector<size_t> xCon, yCon;
    for (size_t r = 0; r < rows; r++) {
        bool any = false;
        for (size_t c = 0; c < cols; c++) any = any || fin[r * cols + c];
        if (any) xCon.push_back(r);
    }
    for (size_t c = 0; c < cols; c++) {
        bool any = false;
        for (size_t r = 0; r < rows; r++) any = any || fin[r * cols + c];
        if (any) yCon.push_back(c);
    }
    size_t n = std::max(rows, cols);
    // the edge matrix of the zero-padded square: 0 where finite, inf elsewhere
    std::vector<float> edge(n * n, 0.0f);
    float pmax = 0.0f;
    for (size_t r = 0; r < n; r++)
        for (size_t c = 0; c < n; c++) {
            const float v = (r < rows && c < cols) ? cost[r * cols + c] : 0.0f;
            if (std::isfinite(v)) {
                if (v > pmax) pmax = v;
            } else {
                edge[r * n + c] = std::numeric_limits<float>::infinity();
            }
        }
    n += Munkres(std::move(edge), n).Deficiency();
    std::vector<float> p(n * n, pmax);
    for (size_t i = 0; i < xCon.size(); i++)
        for (size_t j = 0; j < yCon.size(); j++) p[i * n + j] = cost[xCon[i] * cols + yCon[j]];
    Munkres m(std::move(p), n);
    if (!m.Solve()) return false;
    for (size_t r = 0; r < rows; r++)
        for (size_t c = 0; c < cols; c++) {
            const float v = cost[r * cols + c] == repl ? std::numeric_limits<float>::infinity() : cost[r * cols + c];
            if (m.Starred(r, c) && std::isfinite(v)) {
                outRows.push_back((int)r);
                outCols.push_back((int)c);
                outCosts.push_back(v);
            }
        }
    return true;
}

// :1040-1064: non-finite costs become max(finite) + 100 (-900 when none is
// finite), the reference's Hungarian matches the D x T matrix, and pairs whose
// cost is that substitute are dropped. match[d] = tracker of detection d or -1.
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
    std::vector<int> r, c;
    std::vector<float> v;
    if (!HungarianMatch(cost, rows, cols, r, c, v)) return match;
    for (size_t i = 0; i < r.size(); i++) {
        if (maxCost == v[i]) continue;
        match[(size_t)r[i]] = c[i];
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
        tr->srcDet = (int)det.id;
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
        nt.srcDet = (int)det.id;
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
