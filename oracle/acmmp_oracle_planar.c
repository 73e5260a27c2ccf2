/* acmmp_oracle_planar.c — CPU restatement of ACMMP's planar-prior
 * construction (rlav440/ACMMP), TEST INFRASTRUCTURE ONLY: the checker for
 * acmmp_amd/csrc/acmmp_planar.hip, loaded by tests/ through oracle/oracle.py.
 *
 * Follows, in the reference's own loop order:
 *   GetSupportPoints            src/ACMMP.cpp:868-894
 *   ProcessProblem raster       src/acmmp_definitions.cpp:332-353
 *   GetPriorPlaneParams         src/ACMMP.cpp:920-953 (+ Get3DPointonRefCam :230-239)
 *   GetDepthFromPlaneParam      src/ACMMP.cpp:955-958
 *   range check                 src/acmmp_definitions.cpp:356-370
 *   CudaPlanarPriorInitialization src/ACMMP.cpp:811-831
 * Pin: cv::SVD::solveZ's unit null vector of the 3x4 system
 * is taken as the cofactor (generalised cross product) vector in double,
 * normalised, rounded to float. Parity against the reference's own outputs
 * is unpinned (no fixture holds them; OpenCV is not in the image).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/acmmp.h"

/* GetSupportPoints: writes (x, y) pairs, returns the count */
int acmmp_oracle_support_points(const float *costs, int width, int height, int32_t *xy) {
    const int step_size = 5;
    int n = 0;
    for (int col = 0; col < width; col += step_size) {
        for (int row = 0; row < height; row += step_size) {
            float min_cost = 2.0f;
            int tx = 0, ty = 0;
            int c_bound = col + step_size < width ? col + step_size : width;
            int r_bound = row + step_size < height ? row + step_size : height;
            for (int c = col; c < c_bound; ++c) {
                for (int r = row; r < r_bound; ++r) {
                    int center = r * width + c;
                    if (costs[center] < 2.0f && min_cost > costs[center]) {
                        tx = c;
                        ty = r;
                        min_cost = costs[center];
                    }
                }
            }
            if (min_cost < 0.1f) {
                xy[2 * n] = tx;
                xy[2 * n + 1] = ty;
                ++n;
            }
        }
    }
    return n;
}

static double det3(double a0, double a1, double a2, double b0, double b1, double b2, double c0, double c1,
                   double c2) {
    return a0 * (b1 * c2 - b2 * c1) - a1 * (b0 * c2 - b2 * c0) + a2 * (b0 * c1 - b1 * c0);
}

/* GetPriorPlaneParams for one triangle (x1 y1 x2 y2 x3 y3) on a row-major depth map */
void acmmp_oracle_prior_plane(const acmmp_camera *cam, const float *depths, int width, const int32_t *tri,
                              float *out4) {
    float P[3][3];
    for (int k = 0; k < 3; ++k) {
        const int x = tri[2 * k], y = tri[2 * k + 1];
        const float depth = depths[y * width + x];
        P[k][0] = depth * (x - cam->K[2]) / cam->K[0];
        P[k][1] = depth * (y - cam->K[5]) / cam->K[4];
        P[k][2] = depth;
    }
    /* rows (X, Y, Z, 1): n = (+det[Y Z 1], -det[X Z 1], +det[X Y 1], -det[X Y Z]) */
    double B[4];
    B[0] = det3(P[0][1], P[0][2], 1.0, P[1][1], P[1][2], 1.0, P[2][1], P[2][2], 1.0);
    B[1] = -det3(P[0][0], P[0][2], 1.0, P[1][0], P[1][2], 1.0, P[2][0], P[2][2], 1.0);
    B[2] = det3(P[0][0], P[0][1], 1.0, P[1][0], P[1][1], 1.0, P[2][0], P[2][1], 1.0);
    B[3] = -det3(P[0][0], P[0][1], P[0][2], P[1][0], P[1][1], P[1][2], P[2][0], P[2][1], P[2][2]);
    const double len = sqrt(B[0] * B[0] + B[1] * B[1] + B[2] * B[2] + B[3] * B[3]);
    float n4[4];
    for (int k = 0; k < 4; ++k) n4[k] = (float)(B[k] / len);
    float norm2 = sqrt(pow(n4[0], 2) + pow(n4[1], 2) + pow(n4[2], 2));
    if (n4[3] < 0) norm2 *= -1;
    for (int k = 0; k < 4; ++k) out4[k] = n4[k] / norm2;
}

/* Raster + plane fit + range check + label expansion for a triangle list
 * (already restricted to triangles inside the image, in output order).
 * mask: W*H labels (0 = none), prior: W*H float4 (zero where unlabelled). */
void acmmp_oracle_planar_prior(const acmmp_camera *cam, const float *depths, int width, int height,
                               float depth_min, float depth_max, const int32_t *tris, int ntris, float *planes4,
                               uint32_t *mask, float *prior4) {
    float *mask_tri = (float *)calloc((size_t)width * height, sizeof(float));
    for (int idx = 0; idx < ntris; ++idx) {
        const int32_t *t = tris + 6 * idx;
        float L01 = sqrt(pow(t[0] - t[2], 2) + pow(t[1] - t[3], 2));
        float L02 = sqrt(pow(t[0] - t[4], 2) + pow(t[1] - t[5], 2));
        float L12 = sqrt(pow(t[2] - t[4], 2) + pow(t[3] - t[5], 2));
        float max_edge_length = L01 > (L02 > L12 ? L02 : L12) ? L01 : (L02 > L12 ? L02 : L12);
        float step = 1.0 / max_edge_length;
        for (float p = 0; p < 1.0; p += step) {
            for (float q = 0; q < 1.0 - p; q += step) {
                int x = p * t[0] + q * t[2] + (1.0 - p - q) * t[4];
                int y = p * t[1] + q * t[3] + (1.0 - p - q) * t[5];
                mask_tri[y * width + x] = idx + 1.0;
            }
        }
        acmmp_oracle_prior_plane(cam, depths, width, t, planes4 + 4 * idx);
    }
    for (int i = 0; i < width; ++i) {
        for (int j = 0; j < height; ++j) {
            const size_t c = (size_t)j * width + i;
            if (mask_tri[c] > 0) {
                const float *pl = planes4 + 4 * ((int)mask_tri[c] - 1);
                float d = -pl[3] * cam->K[0] /
                          ((i - cam->K[2]) * pl[0] + (cam->K[0] / cam->K[4]) * (j - cam->K[5]) * pl[1] +
                           cam->K[0] * pl[2]);
                if (!(d <= depth_max && d >= depth_min)) mask_tri[c] = 0;
            }
            mask[c] = (uint32_t)mask_tri[c];
            if (mask[c] > 0)
                memcpy(prior4 + 4 * c, planes4 + 4 * (mask[c] - 1), 4 * sizeof(float));
            else
                memset(prior4 + 4 * c, 0, 4 * sizeof(float));
        }
    }
    free(mask_tri);
}

/* pSampler::GetPriorPlaneEstimate (src/acmmp_definitions.cpp:99-177) on
 * already-decoded 16-bit maps: depth (dh x dw x dc, interleaved) and normals
 * (nh x nw x 3, BGR as cv::imread returns them). Mat::convertTo(alpha, beta)
 * is src * alpha + beta in float; depth_normal_to_plane (:72-89) keeps
 * normVec3's multiplication by the norm (:34-41). */
void acmmp_oracle_prior_plane_estimate(const uint16_t *depth, int dw, int dh, int dc, const uint16_t *normals,
                                       int nw, const acmmp_camera *cam, int rows, int cols, float *planes4) {
    const float dist = cam->depth_max - cam->depth_min;
    const float range = dist / 65535.0f;
    const float alpha = (float)(2.0 / 65536.0), beta = -1.0f;
    const int scale = dh / rows;
    for (int i = 0; i < rows; i++) {
        for (int j = 0; j < cols; ++j) {
            const int k = i * cols + j;
            const float base_d = (float)depth[(size_t)(i * scale) * dw * dc + (size_t)(j * scale)] * range +
                                 cam->depth_min;
            const uint16_t *nv = normals + ((size_t)(i * scale) * nw + (size_t)(j * scale)) * 3;
            float n[4] = {(float)nv[0] * alpha + beta, (float)nv[1] * alpha + beta, (float)nv[2] * alpha + beta,
                          0.0f};
            /* getViewDirection */
            float X[3];
            X[0] = base_d * (j - cam->K[2]) / cam->K[0];
            X[1] = base_d * (i - cam->K[5]) / cam->K[4];
            X[2] = base_d;
            const float norm = sqrtf(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
            const float vd[3] = {X[0] / norm, X[1] / norm, X[2] / norm};
            const float dot_product = n[0] * vd[0] + n[1] * vd[1] + n[2] * vd[2];
            if (dot_product > 0.0f) {
                n[0] = -n[0];
                n[1] = -n[1];
                n[2] = -n[2];
            }
            /* normVec3 */
            const float normSquared = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
            const float inverse_sqrt = sqrtf(normSquared);
            n[0] *= inverse_sqrt;
            n[1] *= inverse_sqrt;
            n[2] *= inverse_sqrt;
            /* distance_to_origin */
            n[3] = -(n[0] * X[0] + n[1] * X[1] + n[2] * X[2]);
            memcpy(planes4 + 4 * (size_t)k, n, sizeof(n));
        }
    }
}
