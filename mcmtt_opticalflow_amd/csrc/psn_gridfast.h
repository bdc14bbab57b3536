// Internal (non-ABI) declarations of the GridFAST kernels (psn_gridfast.hip).
// Public surface: psn_gridfast_* in include/psn_lk.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psn {

constexpr int kGfMaxRois = 64;      // rois per launch (kernel-argument table)
constexpr int kGfMaxRegionW = 1024; // widest cell detection region (cell width - 6)
constexpr int kGfMaxLds = 96 * 1024; // dynamic LDS of the per-cell kernel
constexpr int kGfMaxTotal = 4096;   // maxTotalKeypoints limit (selection sort in LDS)

struct GridFastArgs {
    int w, h, pitch;     // level 0 of the context's ring slots (every slot alike)
    int nroi;
    int threshold, nonmax, grid_rows, grid_cols, per_cell, cap;
    int rw_max, strip, list_cap;  // LDS plan: widest region of the launch, strip rows, keypoint list entries
    uint32_t seed;
    uint32_t *cell_kp;   // [nroi][ncell][per_cell] packed x | y << 16
    int *cell_cnt;       // [nroi][ncell]
    float *out_xy;       // [nroi][cap][2] (rows of rois[0..nroi))
    int *out_count;      // [nroi] min(total, cap)
    int *out_total;      // [nroi] keypoints before the cap (newKeypoints.size())
    int4 rois[kGfMaxRois];
    const uint8_t *roi_img[kGfMaxRois];  // level 0 of the roi's ring slot (its frame's gray image)
    int roi_key[kGfMaxRois];             // the roi's index in its set (shuffle key)
};

// Dynamic LDS bytes of the per-cell kernel for a plan (rw_max, strip, list_cap).
int gridfast_lds_bytes(int rw_max, int strip, int list_cap);
// Both launches (per-cell detection, per-roi selection) on stream s.
hipError_t launch_gridfast(const GridFastArgs &a, hipStream_t s);
hipError_t gridfast_kernels_init();

}  // namespace psn
