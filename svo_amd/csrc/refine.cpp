// Reprojection cost C ABI (§8 a11) and the host pose solver it feeds:
// Levenberg-Marquardt over SE(3) (motion-only bundle adjustment, what a Ceres
// problem with one pose block and AutoDiff reprojection residuals would solve;
// the reference never builds one). Every iteration is one batched
// GPU evaluation (reproj.hip) of residuals, J^T J, J^T r and cost for all
// problems; the 6x6 solves run on the host.
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"

using namespace svo;

namespace {

constexpr int kNE = 28;

// T <- exp(xi^) T, xi = (rho, phi)
void se3_left_update(const double xi[6], double T[12]) {
    const double* rho = xi;
    const double* ph = xi + 3;
    const double th2 = ph[0] * ph[0] + ph[1] * ph[1] + ph[2] * ph[2];
    const double th = std::sqrt(th2);
    double A, B, C;  // sin/th, (1-cos)/th^2, (th-sin)/th^3
    if (th < 1e-8) {
        A = 1 - th2 / 6;
        B = 0.5 - th2 / 24;
        C = 1.0 / 6 - th2 / 120;
    } else {
        A = std::sin(th) / th;
        B = (1 - std::cos(th)) / th2;
        C = (th - std::sin(th)) / (th2 * th);
    }
    const double W[9] = {0, -ph[2], ph[1], ph[2], 0, -ph[0], -ph[1], ph[0], 0};
    double W2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) W2[3 * i + j] = W[3 * i] * W[j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
    double R[9], V[9];
    for (int k = 0; k < 9; k++) {
        const double I = (k % 4 == 0);
        R[k] = I + A * W[k] + B * W2[k];
        V[k] = I + B * W[k] + C * W2[k];
    }
    const double tx[3] = {V[0] * rho[0] + V[1] * rho[1] + V[2] * rho[2], V[3] * rho[0] + V[4] * rho[1] + V[5] * rho[2],
                          V[6] * rho[0] + V[7] * rho[1] + V[8] * rho[2]};
    double Rn[9], tn[3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Rn[3 * i + j] = R[3 * i] * T[j] + R[3 * i + 1] * T[3 + j] + R[3 * i + 2] * T[6 + j];
        tn[i] = R[3 * i] * T[9] + R[3 * i + 1] * T[10] + R[3 * i + 2] * T[11] + tx[i];
    }
    std::memcpy(T, Rn, sizeof(Rn));
    std::memcpy(T + 9, tn, sizeof(tn));
}

// Solve (H + lambda diag(H)) x = -g by Cholesky; false if not positive definite.
bool lm_solve(const double* ne, double lambda, double x[6]) {
    double A[36], b[6];
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) {
            A[6 * a + c] = A[6 * c + a] = ne[k];
            k++;
        }
    for (int a = 0; a < 6; a++) {
        A[7 * a] += lambda * (A[7 * a] > 0 ? A[7 * a] : 1e-12);
        b[a] = -ne[21 + a];
    }
    double L[36] = {0};
    for (int i = 0; i < 6; i++)
        for (int j = 0; j <= i; j++) {
            double s = A[6 * i + j];
            for (int q = 0; q < j; q++) s -= L[6 * i + q] * L[6 * j + q];
            if (i == j) {
                if (!(s > 0)) return false;
                L[7 * i] = std::sqrt(s);
            } else {
                L[6 * i + j] = s / L[7 * j];
            }
        }
    double y[6];
    for (int i = 0; i < 6; i++) {
        double s = b[i];
        for (int q = 0; q < i; q++) s -= L[6 * i + q] * y[q];
        y[i] = s / L[7 * i];
    }
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
        for (int q = i + 1; q < 6; q++) s -= L[6 * q + i] * x[q];
        x[i] = s / L[7 * i];
    }
    return true;
}

struct Staged {
    double *obj, *poses, *res, *jac, *partial, *normal;
    float* img;
    int* counts;
};

int stage(svo_ctx* ctx, const double* obj, const float* img, const int* counts, int P, int max_n, bool want_res,
          bool want_jac, Staged& s) {
    const size_t np = (size_t)P * max_n;
    const size_t bytes = sizeof(double) * (3 * np + 12 * (size_t)P + (want_res ? 2 * np : 0) +
                                           (want_jac ? 12 * np : 0) + reproj_partial_doubles(P, max_n) +
                                           kNE * (size_t)P) +
                         sizeof(float) * 2 * np + sizeof(int) * (size_t)P + 2048;
    char* d = (char*)scratch(ctx, 5, bytes);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    auto carve = [&](size_t n) {
        d = (char*)(((uintptr_t)d + 255) & ~(uintptr_t)255);
        char* r = d;
        d += n;
        return r;
    };
    s.obj = (double*)carve(sizeof(double) * 3 * np);
    s.poses = (double*)carve(sizeof(double) * 12 * P);
    s.res = want_res ? (double*)carve(sizeof(double) * 2 * np) : nullptr;
    s.jac = want_jac ? (double*)carve(sizeof(double) * 12 * np) : nullptr;
    s.partial = (double*)carve(sizeof(double) * reproj_partial_doubles(P, max_n));
    s.normal = (double*)carve(sizeof(double) * kNE * P);
    s.img = (float*)carve(sizeof(float) * 2 * np);
    s.counts = counts ? (int*)carve(sizeof(int) * P) : nullptr;
    SVO_HIP(ctx, hipMemcpyAsync(s.obj, obj, sizeof(double) * 3 * np, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(s.img, img, sizeof(float) * 2 * np, hipMemcpyHostToDevice, ctx->stream));
    if (counts) SVO_HIP(ctx, hipMemcpyAsync(s.counts, counts, sizeof(int) * P, hipMemcpyHostToDevice, ctx->stream));
    return SVO_OK;
}

bool bad_args(const double* obj, const float* img, const int* counts, int P, int max_n, const double* K) {
    if (P < 0 || max_n < 0 || !K) return true;
    if (P > 0 && max_n > 0 && (!obj || !img)) return true;
    if (counts)
        for (int b = 0; b < P; b++)
            if (counts[b] < 0 || counts[b] > max_n) return true;
    return false;
}

}  // namespace

extern "C" {

int svo_reprojection_jacobians(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, const int* counts,
                               int n_problems, int max_n, const double* poses, const double K[9],
                               double huber_delta, double* res, double* jac, double* normal) {
    if (!ctx || bad_args(obj_xyz, img_xy, counts, n_problems, max_n, K) || (n_problems > 0 && !poses))
        return set_error(ctx, SVO_ERR_ARG, "svo_reprojection_jacobians: bad arguments");
    if (n_problems == 0) return SVO_OK;
    Staged s;
    int rc = stage(ctx, obj_xyz, img_xy, counts, n_problems, max_n, res != nullptr, jac != nullptr, s);
    if (rc) return rc;
    SVO_HIP(ctx, hipMemcpyAsync(s.poses, poses, sizeof(double) * 12 * n_problems, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, launch_reproj(s.obj, s.img, s.counts, n_problems, max_n, max_n, s.poses, K, huber_delta, s.res, s.jac,
                               s.partial, normal ? s.normal : nullptr, ctx->stream));
    const size_t np = (size_t)n_problems * max_n;
    if (res) SVO_HIP(ctx, hipMemcpyAsync(res, s.res, sizeof(double) * 2 * np, hipMemcpyDeviceToHost, ctx->stream));
    if (jac) SVO_HIP(ctx, hipMemcpyAsync(jac, s.jac, sizeof(double) * 12 * np, hipMemcpyDeviceToHost, ctx->stream));
    if (normal)
        SVO_HIP(ctx, hipMemcpyAsync(normal, s.normal, sizeof(double) * kNE * n_problems, hipMemcpyDeviceToHost,
                                    ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_refine_poses(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, const int* counts, int n_problems,
                     int max_n, const double K[9], double huber_delta, int max_iterations, double* poses,
                     double* costs, int* iterations) {
    if (!ctx || bad_args(obj_xyz, img_xy, counts, n_problems, max_n, K) || (n_problems > 0 && !poses) ||
        max_iterations < 0)
        return set_error(ctx, SVO_ERR_ARG, "svo_refine_poses: bad arguments");
    if (iterations) *iterations = 0;
    if (n_problems == 0) return SVO_OK;
    const int P = n_problems;
    Staged s;
    int rc = stage(ctx, obj_xyz, img_xy, counts, P, max_n, false, false, s);
    if (rc) return rc;
    std::vector<double> cur(poses, poses + 12 * (size_t)P), trial(cur), ne(kNE * (size_t)P), ne_t(ne);
    std::vector<double> lambda((size_t)P, 1e-4);
    std::vector<char> done((size_t)P, 0);
    auto evaluate = [&](const std::vector<double>& T, std::vector<double>& out) -> int {
        SVO_HIP(ctx, hipMemcpyAsync(s.poses, T.data(), sizeof(double) * 12 * P, hipMemcpyHostToDevice, ctx->stream));
        SVO_HIP(ctx, launch_reproj(s.obj, s.img, s.counts, P, max_n, max_n, s.poses, K, huber_delta, nullptr, nullptr,
                                   s.partial, s.normal, ctx->stream));
        SVO_HIP(ctx, hipMemcpyAsync(out.data(), s.normal, sizeof(double) * kNE * P, hipMemcpyDeviceToHost, ctx->stream));
        SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
        return SVO_OK;
    };
    if ((rc = evaluate(cur, ne))) return rc;
    int it = 0;
    for (; it < max_iterations; it++) {
        bool any = false;
        for (int b = 0; b < P; b++) {
            std::memcpy(&trial[12 * (size_t)b], &cur[12 * (size_t)b], sizeof(double) * 12);
            if (done[b]) continue;
            double dx[6];
            bool ok = false;
            while (!ok && lambda[b] < 1e16) {
                ok = lm_solve(&ne[kNE * (size_t)b], lambda[b], dx);
                if (!ok) lambda[b] *= 10;
            }
            if (!ok) {
                done[b] = 1;
                continue;
            }
            double nx = 0, nt = 0;
            for (int k = 0; k < 6; k++) nx += dx[k] * dx[k];
            for (int k = 9; k < 12; k++) nt += cur[12 * (size_t)b + k] * cur[12 * (size_t)b + k];
            if (std::sqrt(nx) < 1e-12 * (1 + std::sqrt(nt))) {
                done[b] = 1;
                continue;
            }
            se3_left_update(dx, &trial[12 * (size_t)b]);
            any = true;
        }
        if (!any) break;
        if ((rc = evaluate(trial, ne_t))) return rc;
        for (int b = 0; b < P; b++) {
            if (done[b]) continue;
            const double c0 = ne[kNE * (size_t)b + 27], c1 = ne_t[kNE * (size_t)b + 27];
            if (c1 <= c0) {
                std::memcpy(&cur[12 * (size_t)b], &trial[12 * (size_t)b], sizeof(double) * 12);
                std::memcpy(&ne[kNE * (size_t)b], &ne_t[kNE * (size_t)b], sizeof(double) * kNE);
                lambda[b] = lambda[b] * 0.1 > 1e-12 ? lambda[b] * 0.1 : 1e-12;
                if (c0 - c1 <= 1e-15 * c0) done[b] = 1;
            } else {
                lambda[b] *= 10;
                if (lambda[b] >= 1e16) done[b] = 1;
            }
        }
    }
    std::memcpy(poses, cur.data(), sizeof(double) * 12 * P);
    if (costs)
        for (int b = 0; b < P; b++) costs[b] = ne[kNE * (size_t)b + 27];
    if (iterations) *iterations = it;
    return SVO_OK;
}

}  // extern "C"
