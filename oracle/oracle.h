/*
 * oracle.h -- CPU restatement of the reference render path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only as the checker / the timed CPU baseline. The product
 * (librt_hip.so, the HIP kernels) never links or calls it.
 *
 * Parity pinning. The reference cannot be compiled in this image: image.h:7
 * includes <tinyexr.h> from the empty third_party/tinyexr submodule, and the
 * task rules forbid stand-in headers. The reference ships no tests, golden
 * images or known-answer vectors. The oracle is therefore pinned only by
 * outputs of the reference recorded in SURVEY.md (the md5 of main()'s
 * "Cornell Box" PPM, rays-per-sample statistics, the RTOW value range), which
 * the glibc-compat mode must reproduce; see tests/test_oracle_pins.py and
 * DESIGN.md §Oracle. Anything those records do not cover is "parity unpinned".
 *
 * Two RNG modes:
 *  - ORC_RNG_COUNTER: the device path's counter RNG keyed by
 *    (seed, pixel, sample, dim) -- see rng dims in DESIGN.md. Parallel.
 *  - ORC_RNG_COMPAT : glibc rand() as random_double() (utility.h:20), draws
 *    sequenced in the order GCC evaluates the reference's expressions.
 *    Serial, like the reference's par_unseq loop is in this image.
 */
#ifndef ORC_ORACLE_H
#define ORC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_RNG_COUNTER = 0, ORC_RNG_COMPAT = 1 };

/* Build the oracle's own object graph from a scene description.
 * Returns NULL on error (message in err). */
void* orc_scene_from_desc(const rt_scene_desc* desc, char* err, int errlen);

/* Build one of the reference's main.cc scenes with the oracle's own code
 * (independent of the product's C++ headers). name: "cornell_box",
 * "cornell_box_with_volume", "rtow" (random_motion_ball, static spheres),
 * "rtow_motion" (random_motion_ball as written), "three_material_ball",
 * "cornell_triangles" (the Cornell box with every quad split in two triangles).
 * image_width / aspect override the scene's camera (aspect <= 0: scene default).
 * Scenes that draw random numbers while being built call srand(1) first, as
 * the reference's main() implicitly does. Fills *cam and the scene's default
 * spp / depth. */
void* orc_builtin(const char* name, int image_width, double aspect, rt_camera_desc* cam, int* spp,
                  int* max_depth);

void orc_scene_free(void* scene);

/* Render tiles (packed like rt_render_tiles, 3 doubles per pixel). Pixel value
 * = mean over samples [first_sample, first_sample + spp). threads <= 0: all
 * hardware threads. ORC_RNG_COMPAT forces one thread and, when seed != 0,
 * calls srand(seed) first (seed == 0 continues the current rand() stream).
 * Returns 0 on success. */
int orc_render(const void* scene, const rt_camera_desc* cam, int spp, int first_sample, int max_depth,
               uint64_t seed, int rng_mode, int threads, const rt_tile* tiles, int ntiles, double* out,
               uint64_t* segments);

/* write_color (color.h:16-36) over a W*H image in render order: P3 text into
 * buf (header included, camera.h:149-151). Returns the byte count needed. */
size_t orc_write_ppm(const double* image, int width, int height, char* buf, size_t cap);

/* The counter RNG: 32-bit draw for (seed, pixel, sample, dim). */
uint32_t orc_rng_u32(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t dim);
/* Development aid: 1 = print every traced segment to stderr (use with threads = 1). */
void orc_set_trace(int on);

/* Scalar building blocks exposed for known-answer tests. out[] sizes noted. */
int orc_kat_sphere_hit(const double c[3], double r, const double o[3], const double d[3], double tmin,
                       double tmax, double out[9]); /* t, p[3], n[3], u, v; returns hit */
int orc_kat_quad_hit(const double q[3], const double u[3], const double v[3], const double o[3],
                     const double d[3], double tmin, double tmax, double out[9]);
int orc_kat_triangle_hit(const double p0[3], const double p1[3], const double p2[3], const double o[3],
                         const double d[3], double tmin, double tmax, double out[7]);
void orc_kat_onb(const double n[3], double out[9]); /* x, y, z */
void orc_kat_refract(const double v[3], const double n[3], double eta, double out[3]);
double orc_kat_reflectance(double cosine, double ri);
int orc_kat_aabb_hit(const double a[3], const double b[3], const double o[3], const double d[3], double tmin,
                     double tmax);
int orc_kat_world_hit(const double* xyzr, int n, int bvh, const double o[3], const double d[3], double tmin,
                      double tmax, double out[7]); /* t, p, normal */
double orc_kat_sphere_pdf(const double c[3], double r, const double o[3], const double dir[3]);
double orc_kat_cosine_pdf(const double n[3], const double dir[3]);
void orc_kat_compat_draws(unsigned seed, int kind, int n, double* out); /* 3n doubles */
void orc_kat_noise(int kind, const double* table, int resolution, const double* pts, int n, double* out,
                   double* out_turb);

#ifdef __cplusplus
}
#endif

#endif
