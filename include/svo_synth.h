/* svo_synth.h -- deterministic synthetic input for the tests and the benchmark
 * (libsvo_synth.so, host code only). NOT part of the product ABI (svo_gpu.h): the
 * reference reads KITTI PNGs (R:include/async_image_loader.h:57-69), which are not
 * available here, so the workloads are rendered from a synthetic scene instead. */
#ifndef SVO_SYNTH_H
#define SVO_SYNTH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Deterministic synthetic KITTI-like frames: a textured canvas
 * of random rectangles, box-blurred, seen through a rotating pinhole camera
 * (pure rotation => the frame-to-frame motion is a homography, any depth is
 * consistent). Host-side generator, used by tests and bench only. */
int svo_synth_canvas(uint64_t seed, int cw, int ch, int n_rect, uint8_t* canvas);
/* frame = canvas seen by camera rotation R (row-major 3x3, world->camera),
 * intrinsics K; canvas pixel (0,0) sits at image offset (-margin_x, -margin_y)
 * of the unrotated view; adds U[-noise, noise] integer noise (seeded). */
int svo_synth_frame(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y,
                    const double R[9], const double K[9], uint64_t noise_seed, int noise,
                    uint8_t* frame, int w, int h);

/* Right view of a rectified stereo pair of the same synthetic scene: the
 * canvas surface sits at depth rho(u, v) = 12 + 5 sin(u/97 + seed) +
 * 4 cos(v/61 - seed/2) (world z) and
 * the right camera is the left one shifted by the baseline (fx * b = bf). */
int svo_synth_frame_right(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y,
                          const double R[9], const double K[9], double bf, int depth_seed,
                          uint64_t noise_seed, int noise, uint8_t* frame, int w, int h);

/* The same depth-field surface seen by a camera with centre C (world) and
 * rotation R (world -> camera: X_c = R (X - C)) -- a translating camera, so the
 * frames carry parallax -- in front of n_occ textured rectangles: occ[5 k ..]
 * = x0, y0, x1, y1, z (the world plane z, x in [x0, x1], y in [y0, y1]), each
 * drawn from the tw x th texture `occ_tex` (the forward sequences' moving
 * occluders: their points move against the static world). Per pixel the first
 * hit along the ray: the surface by a safeguarded Newton solve of X_z =
 * rho(projection of X from the origin), an occluder by a plane intersection. */
int svo_synth_view(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y, const double R[9],
                   const double C[3], const double K[9], int depth_seed, const double* occ, int n_occ,
                   const uint8_t* occ_tex, int tw, int th, uint64_t noise_seed, int noise, uint8_t* frame, int w,
                   int h);

#ifdef __cplusplus
}
#endif
#endif /* SVO_SYNTH_H */
