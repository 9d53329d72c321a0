/* TEST INFRASTRUCTURE ONLY (see svo_oracle.h). Restates OpenCV 4.x
 * modules/calib3d/src/triangulate.cpp (cv::triangulatePoints: per point the
 * 4x4 DLT system, rows x*P[2]-P[0], y*P[2]-P[1] per view, homogeneous point =
 * right singular vector of the smallest singular value) and
 * modules/calib3d/src/fundam.cpp (convertPointsFromHomogeneous: float divide by
 * w, 1 if w == 0), as called at R:src/tracking.cpp:125-131.
 * The singular vector's sign is fixed to w >= 0 (OpenCV's depends on its SVD
 * and cancels in the division). */
#include <math.h>

#include "oracle_internal.h"
#include "svo_oracle.h"

void svo_oracle_triangulate(const float P1[12], const float P2[12], const float* pts1, const float* pts2,
                            int n, float* xyzw, float* xyz)
{
    for (int i = 0; i < n; i++) {
        double A[16], w[4], vt[16];
        const float* pv[2] = {pts1 + 2 * i, pts2 + 2 * i};
        const float* Pv[2] = {P1, P2};
        for (int j = 0; j < 2; j++) {
            const double x = pv[j][0], y = pv[j][1];
            for (int k = 0; k < 4; k++) {
                A[(2 * j) * 4 + k] = x * Pv[j][8 + k] - Pv[j][k];
                A[(2 * j + 1) * 4 + k] = y * Pv[j][8 + k] - Pv[j][4 + k];
            }
        }
        ora_svd(A, 4, 4, w, 0, vt);
        const double* v = vt + 12; /* smallest singular value's row */
        const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
        const double sg = v[3] < 0 ? -1.0 : 1.0;
        float h[4];
        for (int k = 0; k < 4; k++) h[k] = (float)(sg * v[k] / nrm);
        if (xyzw)
            for (int k = 0; k < 4; k++) xyzw[4 * i + k] = h[k];
        if (xyz) {
            const float sc = h[3] != 0.f ? 1.f / h[3] : 1.f;
            for (int k = 0; k < 3; k++) xyz[3 * i + k] = h[k] * sc;
        }
    }
}
