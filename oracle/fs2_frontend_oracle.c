/*
 * fs2_frontend_oracle.c -- CPU restatement of the reference's landmark
 * front-end: LandmarkUtils.get_measurements_to_landmarks
 * (fast_slam_2/utils/landmark_utils.py:21-89) with
 * HoughTransformation.detect_line_intersections (algorithms/hough_transformation.py:14-145)
 * and GeometryUtils.cluster_points (utils/geometry_utils.py:26-62) at eps 0.5,
 * min_samples 1.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline); libfs2 never
 * links or calls it.
 *
 * Third-party arithmetic restated here (none of it vendored in the reference):
 *  - cv2.circle(img, c, 2, 255, thickness=-1): OpenCV's integer midpoint
 *    circle (imgproc/drawing.cpp, Circle() with fill) -- for radius 2 a
 *    13-pixel diamond (rows -2..2 of half-widths 0,1,2,1,0).
 *  - cv2.HoughLines(img, 1, pi/180, 80): OpenCV 4.5 HoughLinesStandard
 *    (imgproc/hough.cpp): float trig table built by accumulating the float
 *    step, votes r = cvRound(j*cos + i*sin) (round half even, float
 *    arithmetic without contraction), local maxima (> left/up, >= right/down,
 *    > threshold), sorted by votes descending then accumulator index
 *    ascending, rho = (r - (numrho-1)*0.5f), theta = n * (float)(pi/180).
 *    opencv-python is not installed here: this stage is PARITY UNPINNED
 *    against OpenCV itself; everything after it is pinned against the
 *    reference (tests/golden/gen_frontend.py feeds these lines into the
 *    reference's own code).
 *  - numpy float32 sin/cos (np.cos(np.float32)): numpy's SIMD Cody-Waite
 *    reduction + minimax polynomials with FMA (loops_trigonometric); checked
 *    bit-exact against numpy here (tests/test_frontend_oracle.py).
 *  - numpy scalar `** 2`: glibc pow / powf (called directly here).
 * Promotion rules: `legacy` = 0 follows NEP 50 (numpy >= 2, what this
 * container runs and what the fixtures pin): intersections, cluster centres
 * and corners stay float32.  `legacy` = 1 follows numpy 1.x value-based
 * promotion (the reference's requirements.txt pins numpy~=1.24): the
 * back-conversion `(x - offset) / 100` promotes to float64 and everything
 * after it is float64 (unpinned: numpy 1.x is not installed).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FE_PAD 20      /* hough_transformation.py:10 */
#define FE_SCALE 100   /* hough_transformation.py:11 */

/* ---------------------------------------------- numpy float32 sin / cos -- */

static float np_sincosf(float x, int cos_op)
{
    const float q = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(q, -0x1.921fb0p+00f, x);
    r = fmaf(q, -0x1.5110b4p-22f, r);
    r = fmaf(q, -0x1.846988p-48f, r);
    const float r2 = r * r;
    float c = fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = fmaf(c, r2, 0x1.55553cp-05f);
    c = fmaf(c, r2, -0x1.000000p-01f);
    c = fmaf(c, r2, 1.0f);
    float s = fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = fmaf(s, r2, 0x1.11119ap-07f);
    s = fmaf(s, r2, -0x1.555556p-03f);
    s = fmaf(s, r2, 0.0f);
    s = fmaf(s, r, r);
    int iq = (int)q + (cos_op ? 1 : 0);
    float v = (iq & 1) == 0 ? s : c;
    if ((iq & 2) == 2) v = -v;
    return v;
}

float orc_np_sinf(float x) { return np_sincosf(x, 0); }
float orc_np_cosf(float x) { return np_sincosf(x, 1); }

/* ------------------------------------------------------ Hough image ---- */

/* hough_transformation.py:47-61: g = {offset_x, offset_y, width, height} */
void orc_fe_geom(const double *pts, int n, int64_t g[4])
{
    double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int i = 0; i < n; ++i) {
        const double x = pts[2 * i] * FE_SCALE, y = pts[2 * i + 1] * FE_SCALE;
        if (x < mnx) mnx = x;
        if (y < mny) mny = y;
        if (x > mxx) mxx = x;
        if (y > mxy) mxy = y;
    }
    const int64_t min_x = (int64_t)mnx, min_y = (int64_t)mny;
    const int64_t max_x = (int64_t)mxx, max_y = (int64_t)mxy;
    const int64_t ox = (min_x < 0 ? -min_x : 0) + FE_PAD, oy = (min_y < 0 ? -min_y : 0) + FE_PAD;
    g[0] = ox;
    g[1] = oy;
    g[2] = max_x + ox + FE_PAD;
    g[3] = max_y + oy + FE_PAD;
}

/* hough_transformation.py:63-68 + cv2.circle(radius 2, filled) */
void orc_fe_raster(const double *pts, int n, const int64_t g[4], uint8_t *img)
{
    static const int half[5] = {0, 1, 2, 1, 0};
    const int64_t W = g[2];
    memset(img, 0, (size_t)(g[2] * g[3]));
    for (int i = 0; i < n; ++i) {
        const int64_t cx = (int64_t)(pts[2 * i] * FE_SCALE) + g[0];
        const int64_t cy = (int64_t)(pts[2 * i + 1] * FE_SCALE) + g[1];
        for (int dy = -2; dy <= 2; ++dy)
            for (int dx = -half[dy + 2]; dx <= half[dy + 2]; ++dx) img[(cy + dy) * W + cx + dx] = 255;
    }
}

/* OpenCV createTrigTable: float angle accumulated by the float step */
void orc_fe_trig(int numangle, float theta, float *tsin, float *tcos)
{
    float ang = 0.0f;
    for (int n = 0; n < numangle; ang += theta, ++n) {
        tsin[n] = (float)sin((double)ang);
        tcos[n] = (float)cos((double)ang);
    }
}

/* sort key of HoughLinesStandard: votes descending, index ascending */
static const int32_t *g_acc;
static int hough_cmp(const void *a, const void *b)
{
    const int32_t l1 = *(const int32_t *)a, l2 = *(const int32_t *)b;
    if (g_acc[l1] != g_acc[l2]) return g_acc[l1] > g_acc[l2] ? -1 : 1;
    return (l1 > l2) - (l1 < l2);
}

/* cv2.HoughLines(img, 1, np.pi / 180, threshold) -> lines[K][2] = (rho, theta).
 * Returns K; writes at most cap lines. */
int orc_fe_hough(const uint8_t *img, int width, int height, int threshold, float *lines, int cap)
{
    const float theta = (float)(M_PI / 180.0);
    const int numangle = (int)lrint(M_PI / (double)theta);
    const int numrho = (int)lrint((double)(2 * (width + height) + 1) / 1.0);
    const int stride = numrho + 2;
    int32_t *acc = (int32_t *)calloc((size_t)(numangle + 2) * stride, sizeof(int32_t));
    float *ts = (float *)malloc(sizeof(float) * numangle), *tc = (float *)malloc(sizeof(float) * numangle);
    orc_fe_trig(numangle, theta, ts, tc);
    for (int i = 0; i < height; ++i)
        for (int j = 0; j < width; ++j) {
            if (!img[(size_t)i * width + j]) continue;
            for (int n = 0; n < numangle; ++n) {
                const float a = (float)j * tc[n];
                const float b = (float)i * ts[n];
                int r = (int)lrintf(a + b);
                r += (numrho - 1) / 2;
                acc[(n + 1) * stride + r + 1]++;
            }
        }
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * 1024);
    int nb = 0, capb = 1024;
    for (int r = 0; r < numrho; ++r)
        for (int n = 0; n < numangle; ++n) {
            const int base = (n + 1) * stride + r + 1;
            const int32_t v = acc[base];
            if (v > threshold && v > acc[base - 1] && v >= acc[base + 1] && v > acc[base - stride] &&
                v >= acc[base + stride]) {
                if (nb == capb) buf = (int32_t *)realloc(buf, sizeof(int32_t) * (capb *= 2));
                buf[nb++] = base;
            }
        }
    g_acc = acc;
    qsort(buf, (size_t)nb, sizeof(int32_t), hough_cmp);
    const double scale = 1.0 / stride;
    for (int k = 0; k < nb && k < cap; ++k) {
        const int idx = buf[k];
        const int n = (int)floor(idx * scale) - 1;
        const int r = idx - (n + 1) * stride - 1;
        lines[2 * k] = ((float)r - (float)(numrho - 1) * 0.5f) * 1.0f;
        lines[2 * k + 1] = 0.0f + (float)n * theta;
    }
    free(buf);
    free(acc);
    free(ts);
    free(tc);
    return nb;
}

/* hough_transformation.py:83-123 (NEP 50 float32 scalar arithmetic) */
int orc_fe_intersections(const float *lines, int K, int64_t width, int64_t height, float *out, int cap)
{
    int m = 0;
    const double deg45 = 0.7853981633974483;   /* np.deg2rad(45) */
    for (int i = 0; i < K; ++i)
        for (int j = i + 1; j < K; ++j) {
            const float rho1 = lines[2 * i], th1 = lines[2 * i + 1];
            const float rho2 = lines[2 * j], th2 = lines[2 * j + 1];
            float ad = fabsf(th1 - th2);
            const float alt = (float)M_PI - ad;
            if (alt < ad) ad = alt;
            if ((double)ad < deg45) continue;
            const float a1 = orc_np_cosf(th1), b1 = orc_np_sinf(th1);
            const float a2 = orc_np_cosf(th2), b2 = orc_np_sinf(th2);
            const float p = a1 * b2, q = a2 * b1;
            const float det = p - q;
            if (!(fabsf(det) > 1e-10f)) continue;
            const float xn1 = b2 * rho1, xn2 = b1 * rho2;
            const float yn1 = a1 * rho2, yn2 = a2 * rho1;
            const float x = (xn1 - xn2) / det;
            const float y = (yn1 - yn2) / det;
            if (x >= 0.0f && x < (float)width && y >= 0.0f && y < (float)height) {
                if (m < cap) {
                    out[2 * m] = x;
                    out[2 * m + 1] = y;
                }
                ++m;
            }
        }
    return m;
}

/* hough_transformation.py:125-145 */
void orc_fe_back(const float *isect, int n, int64_t off_x, int64_t off_y, int legacy, double *out)
{
    for (int k = 0; k < n; ++k) {
        if (legacy) {
            out[2 * k] = ((double)isect[2 * k] - (double)off_x) / 100.0;
            out[2 * k + 1] = ((double)isect[2 * k + 1] - (double)off_y) / 100.0;
        } else {
            out[2 * k] = (double)((isect[2 * k] - (float)off_x) / 100.0f);
            out[2 * k + 1] = (double)((isect[2 * k + 1] - (float)off_y) / 100.0f);
        }
    }
}

/* ---------------------------------------------------- DBSCAN, min 1 ---- */

static int uf_find(int *p, int a)
{
    while (p[a] != a) {
        p[a] = p[p[a]];
        a = p[a];
    }
    return a;
}

/* GeometryUtils.cluster_points(points, eps, 1) (geometry_utils.py:26-62):
 * clusters = components of the graph dx*dx + dy*dy <= eps*eps (every point is
 * core), numbered by smallest member; centre = numpy mean(axis=0): index-order
 * sums (float32 for NEP 50 inputs, float64 legacy), divided by the intp count
 * in float64.  Returns the number of clusters. */
int orc_fe_cluster1(const double *pts, int n, double eps, int legacy, double *centres)
{
    int *par = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    int *lab = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) par[i] = i;
    const double e2 = eps * eps;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            const double dx = pts[2 * i] - pts[2 * j], dy = pts[2 * i + 1] - pts[2 * j + 1];
            const double a = dx * dx, b = dy * dy;
            if (a + b <= e2) {
                const int ri = uf_find(par, i), rj = uf_find(par, j);
                if (ri != rj) par[ri < rj ? rj : ri] = ri < rj ? ri : rj;
            }
        }
    int K = 0;
    for (int i = 0; i < n; ++i) {
        const int r = uf_find(par, i);
        lab[i] = (r == i) ? K++ : lab[r];
    }
    for (int c = 0; c < K; ++c) {
        double sx = 0.0, sy = 0.0;
        float fx = 0.0f, fy = 0.0f;
        int64_t cnt = 0;
        for (int i = 0; i < n; ++i) {
            if (lab[i] != c) continue;
            if (legacy) {
                sx += pts[2 * i];
                sy += pts[2 * i + 1];
            } else {
                fx += (float)pts[2 * i];
                fy += (float)pts[2 * i + 1];
            }
            ++cnt;
        }
        if (legacy) {
            centres[2 * c] = sx / (double)cnt;
            centres[2 * c + 1] = sy / (double)cnt;
        } else {
            centres[2 * c] = (double)(float)((double)fx / (double)cnt);
            centres[2 * c + 1] = (double)(float)((double)fy / (double)cnt);
        }
    }
    free(par);
    free(lab);
    return K;
}

/* landmark_utils.py:66-89: centres with a scan point within threshold */
int orc_fe_corners(const double *centres, int C, const double *scan, int P, double threshold,
                   double *corners)
{
    int m = 0;
    for (int c = 0; c < C; ++c)
        for (int k = 0; k < P; ++k) {
            const double d = sqrt(pow(centres[2 * c] - scan[2 * k], 2.0) +
                                  pow(centres[2 * c + 1] - scan[2 * k + 1], 2.0));
            if (d <= threshold) {
                corners[2 * m] = centres[2 * c];
                corners[2 * m + 1] = centres[2 * c + 1];
                ++m;
                break;
            }
        }
    return m;
}

/* landmark_utils.py:31-34 + GeometryUtils.calculate_distance_and_angle
 * (geometry_utils.py:65-74): math.sqrt(x ** 2 + y ** 2), math.atan2(y, x) */
void orc_fe_measure(const double *corners, int C, int legacy, double *meas)
{
    for (int c = 0; c < C; ++c) {
        const double x = corners[2 * c], y = corners[2 * c + 1];
        if (legacy) {
            meas[2 * c] = sqrt(pow(x, 2.0) + pow(y, 2.0));
        } else {
            const float fx = (float)x, fy = (float)y;
            const float s = powf(fx, 2.0f) + powf(fy, 2.0f);
            meas[2 * c] = sqrt((double)s);
        }
        meas[2 * c + 1] = atan2(y, x);
    }
}

void orc_correlate_reflect(const double *in, int64_t n, int64_t stride, const double *wts, int32_t radius,
                           double *out);

/* Whole front-end for one scan (landmark_utils.py:21-64).  counts = {lines,
 * intersections, clusters, corners}.  Returns the number of measurements
 * (corners); at most cap are written.  Returns -1 on an allocation failure. */
int orc_fe_extract(const double *points, int P, const double *taps, int radius, int legacy,
                   double *meas, int cap, int32_t counts[4])
{
    counts[0] = counts[1] = counts[2] = counts[3] = 0;
    if (P <= 0) return 0;
    double *f = (double *)malloc(sizeof(double) * 2 * P);
    orc_correlate_reflect(points, P, 2, taps, radius, f);
    orc_correlate_reflect(points + 1, P, 2, taps, radius, f + 1);
    int64_t g[4];
    orc_fe_geom(f, P, g);
    uint8_t *img = (uint8_t *)malloc((size_t)(g[2] * g[3]));
    if (!img) {
        free(f);
        return -1;
    }
    orc_fe_raster(f, P, g, img);
    int K = orc_fe_hough(img, (int)g[2], (int)g[3], 80, NULL, 0);
    float *lines = (float *)malloc(sizeof(float) * 2 * (K > 0 ? K : 1));
    orc_fe_hough(img, (int)g[2], (int)g[3], 80, lines, K);
    free(img);
    counts[0] = K;
    const int ni = orc_fe_intersections(lines, K, g[2], g[3], NULL, 0);
    float *is = (float *)malloc(sizeof(float) * 2 * (ni > 0 ? ni : 1));
    orc_fe_intersections(lines, K, g[2], g[3], is, ni);
    counts[1] = ni;
    int M = 0;
    if (ni > 0) {
        double *ip = (double *)malloc(sizeof(double) * 2 * ni);
        double *cent = (double *)malloc(sizeof(double) * 2 * ni);
        double *corn = (double *)malloc(sizeof(double) * 2 * ni);
        orc_fe_back(is, ni, g[0], g[1], legacy, ip);
        const int C = orc_fe_cluster1(ip, ni, 0.5, legacy, cent);
        counts[2] = C;
        M = orc_fe_corners(cent, C, f, P, 0.1, corn);
        counts[3] = M;
        double *mm = (double *)malloc(sizeof(double) * 2 * (M > 0 ? M : 1));
        orc_fe_measure(corn, M, legacy, mm);
        memcpy(meas, mm, sizeof(double) * 2 * (M < cap ? M : cap));
        free(mm);
        free(ip);
        free(cent);
        free(corn);
    }
    free(is);
    free(lines);
    free(f);
    return M;
}
