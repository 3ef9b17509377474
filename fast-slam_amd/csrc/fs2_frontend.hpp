// fs2_frontend.hpp -- landmark front-end (fs2_frontend.hip): per-scan geometry,
// workspace and the batched driver called by fs2_api.hip (fs2_frontend()).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fs2 {

constexpr int kFeAngles = 180;       // cv2.HoughLines(img, 1, pi/180, ...): numangle
constexpr int kFeMaxRow = 40000;     // accumulator row (numrho + 2) held in LDS: w + h <= 19998 px
constexpr int kFeMaxLines = 4096;    // Hough lines per scan (rank sort and pair loop in LDS)
constexpr int kFeFusedLds = 65536;   // LDS of one fused vote + maxima workgroup (2 per CU)

enum { kFeOk = 0, kFeEmpty = 1, kFeNonFinite = 2, kFeTooLarge = 3, kFeTooManyLines = 4 };

// Image geometry of one scan (hough_transformation.py:47-61) + its regions in
// the batch's scratch arrays.
struct FeGeom {
    int32_t ox, oy, W, H, numrho, status;
    int64_t pix_off, bm_off, acc_off;
};

struct FeBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
};

// Grow-only device buffers of one device (callers serialise access).
struct FeWorkspace {
    FeBuf offs, taps, tabs, pts, filt, geom, bitmap, pix, npix, acc, cand, ncand, lines, nlines, isect_off, isect,
        nisect, par, lab, centres, corners, counts, pack;
    int cand_cap = 0;
    ~FeWorkspace();
};

struct FeArgs {
    int B = 0;
    const int64_t *offs = nullptr;   // host, B + 1
    const double *points = nullptr;  // [offs[B]][2]
    bool points_on_device = false;
    const double *taps = nullptr;    // host, 2 radius + 1 (LineFilter Gaussian)
    int radius = 0;
    int legacy = 0;                  // 1: numpy 1.x promotion after the back-conversion
    int threshold = 80;              // hough_transformation.py:25
    double eps = 0.5;                // landmark_utils.py:57
    double corner = 0.1;             // landmark_utils.py:64
    int cap = 0;                     // rows per scan of the host outputs
};

struct FeHostOut {
    std::vector<int32_t> status;     // per scan (kFe*)
    std::vector<int32_t> counts;     // [B][4] lines, intersections, clusters, corners
    bool fused = false;              // vote + maxima ran fused in LDS
    float *lines = nullptr;          // [B][cap][2] host, nullable
    double *intersections = nullptr, *clusters = nullptr, *corners = nullptr;   // [B][cap][2] host
};

// OpenCV createTrigTable for theta = pi/180: tabs[0:180] = sin, tabs[180:360] = cos
void fe_trig_table(float *tabs);

hipError_t frontend_run(FeWorkspace &ws, const FeArgs &a, FeHostOut &o, hipStream_t s);

}  // namespace fs2
