/*
 * ORACLE TEST INFRASTRUCTURE -- CPU restatement of ReflaxMan's per-pixel trace
 * loop.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this (as the checker / the "port" CPU baseline).  It is never part
 * of the product path: reflaxman_amd fails loudly without its HIP library.
 *
 * Pinning: bit-exact (f32 framebuffer and ARGB8) against golden vectors that
 * oracle/_ref/refharness -- the unmodified reference sources compiled by
 * oracle/Makefile -- produced (tests/golden/, tools/gen_golden.py).
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* event counters (also produced by the GPU stats kernel; tests compare them) */
enum {
  ORC_RAYS = 0, ORC_SEGMENTS,
  ORC_SPH_TESTS, ORC_SPH_B, ORC_SPH_D, ORC_SPH_T,
  ORC_TRI_TESTS, ORC_TRI_Z, ORC_TRI_S, ORC_TRI_T, ORC_TRI_IN, ORC_TRI_D,
  ORC_HIT_SPH, ORC_HIT_TRI,
  ORC_SH_SPH_TESTS, ORC_SH_SPH_B, ORC_SH_SPH_D, ORC_SH_SPH_T,
  ORC_SH_TRI_TESTS, ORC_SH_TRI_Z, ORC_SH_TRI_S, ORC_SH_TRI_T, ORC_SH_TRI_IN,
  ORC_L_EVAL, ORC_L_FACING, ORC_L_LIT, ORC_L_SPEC, ORC_L_POW,
  ORC_DIELECTRIC, ORC_METAL, ORC_CONTINUE, ORC_SKY,
  ORC_TEX_BILINEAR, ORC_TEX_CHECKER, ORC_TEX_OTHER,
  ORC_PLN_TESTS, ORC_PLN_T, ORC_HIT_PLN, ORC_SH_PLN_TESTS, ORC_SH_PLN_T,
  ORC_NCOUNTERS
};

orc_scene *orc_scene_new(float diff_r, float diff_g, float diff_b, float diff_power);
void orc_scene_free(orc_scene *s);
/* texture from ARGB texels (row = file order); w == 0 or argb == NULL -> empty (checker) */
int orc_add_texture(orc_scene *s, uint32_t w, uint32_t h, const uint32_t *argb);
void orc_set_skybox(orc_scene *s, int texture_id); /* -1: none (checker) */
int orc_add_light(orc_scene *s, const float origin[3], float radius, const float rgb[3], float power);
int orc_add_sphere(orc_scene *s, const float center[3], float radius, int dielectric, const float rgb[3], float refl, float transp);
int orc_add_triangle(orc_scene *s, const float v0[3], const float v1[3], const float v2[3], int dielectric,
                     const float rgb[3], float refl, float transp);
int orc_add_plane(orc_scene *s, const float pos[3], const float norm[3], int dielectric, const float rgb[3],
                  float refl, float transp);
int orc_triangle_set_texture(orc_scene *s, int object_id, int texture_id, const float uv[6]);

/* Camera(eye, at, fov) -> view, row-major _11.._33 (Camera.cpp:24-56) */
void orc_camera_view(const float eye[3], const float at[3], float view[9]);

/*
 * One Render::renderBegin + renderNext(W*H) pass (Render.cpp:116-215).
 * image: W*H*3 floats, in/out (additive accumulation, block fill).
 * additive_counter: Render::additiveCounter *after* renderBegin.
 * seeds advance exactly like the reference's two LCG streams.
 * counters: ORC_NCOUNTERS u64 (may be NULL).  nthreads >= 1.
 */
int orc_render(const orc_scene *s, const float eye[3], const float view[9], float fov,
               uint32_t W, uint32_t H, int depth, int ss, int additive, int additive_counter,
               uint32_t *sphere_seed, uint32_t *jitter_seed, float *image, int nthreads, uint64_t *counters);

/* rows [y0, y0+rows) of an ss=1 frame, sphere stream advanced by y0*W traces first */
int orc_render_band(const orc_scene *s, const float eye[3], const float view[9], float fov,
                    uint32_t W, uint32_t H, int depth, uint32_t y0, uint32_t rows,
                    uint32_t sphere_seed, float *rgb_out, uint32_t *argb_out, int nthreads, uint64_t *counters);

/* KATs */
void orc_rand_dirs(uint32_t *seed, uint64_t n, float *out3);
void orc_kat_sphere(const float *rec11, uint64_t n, float *out15);
void orc_kat_triangle(const float *rec21, uint64_t n, uint32_t tw, uint32_t th, const uint32_t *argb, int textured, float *out15);
void orc_kat_plane(const float *rec12, uint64_t n, float *out15);
void orc_kat_skybox(uint32_t tw, uint32_t th, const uint32_t *argb, const float *rays3, uint64_t n, float *out3);
void orc_kat_texture(uint32_t tw, uint32_t th, const uint32_t *argb, const float *uv2, uint64_t n, float *out3);
uint32_t orc_argb(float r, float g, float b);

#ifdef __cplusplus
}
#endif
