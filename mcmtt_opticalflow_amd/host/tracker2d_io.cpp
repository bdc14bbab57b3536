// stTrack2DResult formats (include/psn_tracker2d.h): the reference's text
// files (CPSNWhere_Tracker2D::FilePrintResult, PSNWhere_Tracker2D.cpp:1268-1334;
// psn::Read2DTrackResultWithTxt, PSNWhere_Utils.cpp:1148-1237) and the exact
// binary slot exchanged between cameras (ranks) each frame.
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>

#include "psn_lk.h"
#include "psn_tracker2d.h"

namespace {

std::string result_path(const char *dir, unsigned cam, unsigned frame) {
    char name[96];
    std::snprintf(name, sizeof name, "track2D_result_cam%d_frame%04d.txt", (int)cam, (int)frame);
    return std::string(dir ? dir : "") + name;
}

void put_points(FILE *fp, const char *tag, const float (*xy)[2], int n) {
    std::fprintf(fp, "\t\t%s:%d,{", tag, n);
    for (int i = 0; i < n; i++) {
        std::fprintf(fp, "(%f,%f)", xy[i][0], xy[i][1]);
        if (n > i + 1) std::fprintf(fp, ",");
    }
    std::fprintf(fp, "}\n");
}

void put_rects(FILE *fp, const char *tag, const psn_rect *r, int n) {
    std::fprintf(fp, "%s:%d,{", tag, n);
    for (int i = 0; i < n; i++) {
        std::fprintf(fp, "(%f,%f,%f,%f)", r[i].x, r[i].y, r[i].w, r[i].h);
        if (n > i + 1) std::fprintf(fp, ",");
    }
    std::fprintf(fp, "}\n");
}

// fscanf of a literal pattern; false when the input does not match
bool lit(FILE *fp, const char *pattern) {
    int n = -1;
    std::string p = std::string(pattern) + "%n";
    if (std::fscanf(fp, p.c_str(), &n) < 0) return false;
    return n >= 0;
}

bool read_rect(FILE *fp, const char *fmt, psn_rect *out) {
    float x, y, w, h;  // the reference parses into float (PSNWhere_Utils.cpp:1160-1161)
    if (std::fscanf(fp, fmt, &x, &y, &w, &h) != 4) return false;
    *out = psn_rect{(double)x, (double)y, (double)w, (double)h};
    return true;
}

int read_points(FILE *fp, const char *head, float (*xy)[2], int *n) {
    int cnt = 0;
    if (std::fscanf(fp, head, &cnt) != 1 || cnt < 0) return PSN_LK_ERR_ARG;
    if (cnt > PSN_T2D_MAX_FEATURES) return PSN_T2D_ERR_CAPACITY;
    for (int i = 0; i < cnt; i++) {
        float x, y;
        if (std::fscanf(fp, "(%f,%f)", &x, &y) != 2) return PSN_LK_ERR_ARG;
        if (cnt > i + 1 && !lit(fp, ",")) return PSN_LK_ERR_ARG;
        xy[i][0] = x;
        xy[i][1] = y;
    }
    *n = cnt;
    return lit(fp, "}\n") ? 0 : PSN_LK_ERR_ARG;
}

int read_rects(FILE *fp, const char *head, psn_rect *r, int cap, int *n) {
    int cnt = 0;
    if (std::fscanf(fp, head, &cnt) != 1 || cnt < 0) return PSN_LK_ERR_ARG;
    if (cnt > cap) return PSN_T2D_ERR_CAPACITY;
    for (int i = 0; i < cnt; i++) {
        if (!read_rect(fp, "(%f,%f,%f,%f)", &r[i])) return PSN_LK_ERR_ARG;
        if (cnt > i + 1 && !lit(fp, ",")) return PSN_LK_ERR_ARG;
    }
    *n = cnt;
    return lit(fp, "}\n") ? 0 : PSN_LK_ERR_ARG;
}

// binary slot
constexpr uint32_t kMagic = 0x52325450u;  // "PT2R"
struct SlotHeader {
    uint32_t magic, version, cam_id, frame_idx, nobj, ndet, ntrk, bytes_used;
};
struct SlotObject {
    uint32_t id, num_prev, num_curr, pad;
    double box[4], head[4], score;
};
size_t align8(size_t n) { return (n + 7) & ~(size_t)7; }
size_t object_bytes(int np, int nc) { return align8(sizeof(SlotObject) + 8 * (size_t)(np + nc)); }

}  // namespace

extern "C" {

int psn_t2d_write_result_txt(const char *dir, const psn_track2d_result *r) {
    if (!r || r->num_objects < 0 || r->num_detection_rects < 0 || r->num_tracker_rects < 0 ||
        (r->num_objects > 0 && !r->objects) || (r->num_detection_rects > 0 && !r->detection_rects) ||
        (r->num_tracker_rects > 0 && !r->tracker_rects))
        return PSN_LK_ERR_ARG;
    FILE *fp = std::fopen(result_path(dir, r->cam_id, r->frame_idx).c_str(), "w");
    if (!fp) return PSN_LK_ERR_ARG;
    std::fprintf(fp, "camIdx:%d\nframeIdx:%d\n", (int)r->cam_id, (int)r->frame_idx);
    std::fprintf(fp, "numObjectInfos:%d{\n", r->num_objects);
    for (int i = 0; i < r->num_objects; i++) {
        const psn_object2d &o = r->objects[i];
        std::fprintf(fp, "\t{\n");
        std::fprintf(fp, "\t\tid:%d\n", (int)o.id);
        std::fprintf(fp, "\t\tbox:(%f,%f,%f,%f)\n", o.box.x, o.box.y, o.box.w, o.box.h);
        std::fprintf(fp, "\t\thead:(%f,%f,%f,%f)\n", o.head.x, o.head.y, o.head.w, o.head.h);
        std::fprintf(fp, "\t\tscore:%f\n", o.score);
        put_points(fp, "featurePointsPrev", o.prev, o.num_prev);
        put_points(fp, "featurePointsCurr", o.curr, o.num_curr);
        std::fprintf(fp, "\t}\n");
    }
    std::fprintf(fp, "}\n");
    put_rects(fp, "detectionRects", r->detection_rects, r->num_detection_rects);
    put_rects(fp, "trackerRects", r->tracker_rects, r->num_tracker_rects);
    std::fclose(fp);
    return 0;
}

int psn_t2d_read_result_txt(const char *dir, unsigned cam_id, unsigned frame_idx, psn_track2d_result *r) {
    if (!r) return PSN_LK_ERR_ARG;
    FILE *fp = std::fopen(result_path(dir, cam_id, frame_idx).c_str(), "r");
    if (!fp) return PSN_LK_ERR_ARG;
    int rc = 0;
    int a = 0, b = 0, nobj = 0;
    r->cam_id = cam_id;  // as the reference: the ids requested, not the ones in the file
    r->frame_idx = frame_idx;
    r->num_objects = r->num_detection_rects = r->num_tracker_rects = 0;
    if (std::fscanf(fp, "camIdx:%d\nframeIdx:%d\n", &a, &b) != 2 || std::fscanf(fp, "numObjectInfos:%d{\n", &nobj) != 1 ||
        nobj < 0)
        rc = PSN_LK_ERR_ARG;
    else if (nobj > r->cap_objects || (nobj > 0 && !r->objects))
        rc = PSN_T2D_ERR_CAPACITY;
    for (int i = 0; rc == 0 && i < nobj; i++) {
        psn_object2d &o = r->objects[i];
        int id = 0;
        float sc = 0.f;
        if (!lit(fp, "\t{\n") || std::fscanf(fp, "\t\tid:%d\n", &id) != 1 ||
            !read_rect(fp, "\t\tbox:(%f,%f,%f,%f)\n", &o.box) || !read_rect(fp, "\t\thead:(%f,%f,%f,%f)\n", &o.head) ||
            std::fscanf(fp, "\t\tscore:%f\n", &sc) != 1) {
            rc = PSN_LK_ERR_ARG;
            break;
        }
        o.id = (unsigned)id;
        o.score = (double)sc;
        rc = read_points(fp, "\t\tfeaturePointsPrev:%d,{", o.prev, &o.num_prev);
        if (rc == 0) rc = read_points(fp, "\t\tfeaturePointsCurr:%d,{", o.curr, &o.num_curr);
        if (rc == 0 && !lit(fp, "\t}\n")) rc = PSN_LK_ERR_ARG;
        if (rc == 0) r->num_objects = i + 1;
    }
    if (rc == 0 && !lit(fp, "}\n")) rc = PSN_LK_ERR_ARG;
    if (rc == 0)
        rc = read_rects(fp, "detectionRects:%d,{", r->detection_rects, r->cap_detection_rects, &r->num_detection_rects);
    if (rc == 0) rc = read_rects(fp, "trackerRects:%d,{", r->tracker_rects, r->cap_tracker_rects, &r->num_tracker_rects);
    std::fclose(fp);
    return rc;
}

size_t psn_t2d_result_slot_bytes(int max_objects, int max_rects) {
    if (max_objects < 0 || max_rects < 0) return 0;
    const size_t n = sizeof(SlotHeader) + (size_t)max_objects * object_bytes(PSN_T2D_MAX_FEATURES, PSN_T2D_MAX_FEATURES) +
                     2 * (size_t)max_rects * 4 * sizeof(double);
    return (n + 63) & ~(size_t)63;
}

int psn_t2d_pack_result(const psn_track2d_result *r, void *slot, size_t slot_bytes) {
    if (!r || !slot || r->num_objects < 0 || r->num_detection_rects < 0 || r->num_tracker_rects < 0) return PSN_LK_ERR_ARG;
    size_t need = sizeof(SlotHeader);
    for (int i = 0; i < r->num_objects; i++) {
        const psn_object2d &o = r->objects[i];
        if (o.num_prev < 0 || o.num_prev > PSN_T2D_MAX_FEATURES || o.num_curr < 0 || o.num_curr > PSN_T2D_MAX_FEATURES)
            return PSN_T2D_ERR_CAPACITY;
        need += object_bytes(o.num_prev, o.num_curr);
    }
    need += 4 * sizeof(double) * (size_t)(r->num_detection_rects + r->num_tracker_rects);
    if (need > slot_bytes) return PSN_T2D_ERR_CAPACITY;
    uint8_t *p = (uint8_t *)slot;
    SlotHeader h{kMagic, 1u, r->cam_id, r->frame_idx, (uint32_t)r->num_objects, (uint32_t)r->num_detection_rects,
                 (uint32_t)r->num_tracker_rects, (uint32_t)need};
    std::memcpy(p, &h, sizeof h);
    size_t off = sizeof h;
    for (int i = 0; i < r->num_objects; i++) {
        const psn_object2d &o = r->objects[i];
        SlotObject so{o.id, (uint32_t)o.num_prev, (uint32_t)o.num_curr, 0u,
                      {o.box.x, o.box.y, o.box.w, o.box.h}, {o.head.x, o.head.y, o.head.w, o.head.h}, o.score};
        std::memcpy(p + off, &so, sizeof so);
        std::memcpy(p + off + sizeof so, o.prev, 8 * (size_t)o.num_prev);
        std::memcpy(p + off + sizeof so + 8 * (size_t)o.num_prev, o.curr, 8 * (size_t)o.num_curr);
        const size_t ob = object_bytes(o.num_prev, o.num_curr);
        std::memset(p + off + sizeof so + 8 * (size_t)(o.num_prev + o.num_curr), 0,
                    ob - sizeof so - 8 * (size_t)(o.num_prev + o.num_curr));
        off += ob;
    }
    for (int i = 0; i < r->num_detection_rects; i++, off += 32) std::memcpy(p + off, &r->detection_rects[i], 32);
    for (int i = 0; i < r->num_tracker_rects; i++, off += 32) std::memcpy(p + off, &r->tracker_rects[i], 32);
    return 0;
}

int psn_t2d_unpack_result(const void *slot, size_t slot_bytes, psn_track2d_result *r) {
    if (!slot || !r || slot_bytes < sizeof(SlotHeader)) return PSN_LK_ERR_ARG;
    const uint8_t *p = (const uint8_t *)slot;
    SlotHeader h;
    std::memcpy(&h, p, sizeof h);
    if (h.magic != kMagic || h.version != 1u || h.bytes_used > slot_bytes) return PSN_LK_ERR_ARG;
    // unsigned comparisons: a corrupt or foreign count >= 2^31 must not pass as negative
    auto cap = [](int c) { return (uint32_t)std::max(c, 0); };
    if (h.nobj > cap(r->cap_objects) || h.ndet > cap(r->cap_detection_rects) || h.ntrk > cap(r->cap_tracker_rects))
        return PSN_T2D_ERR_CAPACITY;
    if ((h.nobj && !r->objects) || (h.ndet && !r->detection_rects) || (h.ntrk && !r->tracker_rects))
        return PSN_LK_ERR_ARG;
    r->cam_id = h.cam_id;
    r->frame_idx = h.frame_idx;
    size_t off = sizeof h;
    for (uint32_t i = 0; i < h.nobj; i++) {
        SlotObject so;
        if (off + sizeof so > h.bytes_used) return PSN_LK_ERR_ARG;
        std::memcpy(&so, p + off, sizeof so);
        if (so.num_prev > PSN_T2D_MAX_FEATURES || so.num_curr > PSN_T2D_MAX_FEATURES ||
            off + object_bytes((int)so.num_prev, (int)so.num_curr) > h.bytes_used)
            return PSN_LK_ERR_ARG;
        psn_object2d &o = r->objects[i];
        o.id = so.id;
        o.box = psn_rect{so.box[0], so.box[1], so.box[2], so.box[3]};
        o.head = psn_rect{so.head[0], so.head[1], so.head[2], so.head[3]};
        o.score = so.score;
        o.num_prev = (int)so.num_prev;
        o.num_curr = (int)so.num_curr;
        std::memcpy(o.prev, p + off + sizeof so, 8 * (size_t)so.num_prev);
        std::memcpy(o.curr, p + off + sizeof so + 8 * (size_t)so.num_prev, 8 * (size_t)so.num_curr);
        off += object_bytes((int)so.num_prev, (int)so.num_curr);
    }
    if (off + 32 * ((size_t)h.ndet + (size_t)h.ntrk) > h.bytes_used) return PSN_LK_ERR_ARG;
    for (uint32_t i = 0; i < h.ndet; i++, off += 32) std::memcpy(&r->detection_rects[i], p + off, 32);
    for (uint32_t i = 0; i < h.ntrk; i++, off += 32) std::memcpy(&r->tracker_rects[i], p + off, 32);
    r->num_objects = (int)h.nobj;
    r->num_detection_rects = (int)h.ndet;
    r->num_tracker_rects = (int)h.ntrk;
    return 0;
}

}  // extern "C"
