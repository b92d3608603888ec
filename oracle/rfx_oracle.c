/*
 * ORACLE TEST INFRASTRUCTURE -- CPU restatement of ReflaxMan's per-pixel trace
 * loop (never shipped; see rfx_oracle.h for who may load it).
 *
 * Every function restates the reference's arithmetic in the reference's exact
 * IEEE operation order; build with -O2 -ffp-contract=off (no FMA contraction,
 * no fast-math), which is how the reference is compiled for parity
 * (SURVEY.md §0.5-0.6).  Citations are /root/reference/src/common/<file>:<line>.
 *
 * Parity pin: tests/test_oracle_golden.py compares this file's output with
 * golden vectors produced by the *unmodified* reference (oracle/_ref).
 */
#include "rfx_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* trace_math.h:17-18 */
#define VSN 1.0842021724855044e-19f /* sqrtf(FLT_MIN) == 2^-63 exactly */
#define DELTA 0.0001f

typedef struct { float x, y, z; } v3;
typedef struct { float r, g, b; } col;
typedef struct { float m11, m12, m13, m21, m22, m23, m31, m32, m33; } m33;

/* ---- Vector3 (Vector3.cpp:36-174) ---------------------------------------- */
static inline v3 V(float x, float y, float z) { v3 v = {x, y, z}; return v; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }          /* :106 */
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }          /* :111 */
static inline v3 vmul(v3 a, float f) { return V(a.x * f, a.y * f, a.z * f); }              /* :116,121 */
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }         /* :126 */
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }                                 /* :166 */
static inline float vsqlen(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }             /* :48 */
static inline float vlen(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }        /* :43 */
static inline v3 vcross(v3 a, v3 b)                                                          /* :138 */
{
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 vdiv(v3 a, float f)                                                         /* :143-151 */
{
  if (fabsf(f) > VSN) return V(a.x / f, a.y / f, a.z / f);
  return a;
}
static inline v3 vnormalized(v3 a)                                                           /* :63-72 */
{
  const float l = vlen(a);
  if (l > VSN) return vdiv(a, l);
  return a;
}
/* Tracemath::normalize (trace_math.cpp:3-12) -- same arithmetic as normalized() */
static inline v3 tm_normalize(v3 a) { return vnormalized(a); }
/* Tracemath::reflect (trace_math.cpp:14-23): v - 2n * ((v.n) / (n.n)) */
static inline v3 tm_reflect(v3 v, v3 n)
{
  const float dn = vdot(n, n);
  if (dn > VSN) return vsub(v, vmul(vmul(n, 2.0f), vdot(v, n) / dn));
  return v;
}
static inline float clampf01(float v, float lo, float hi) { return v < lo ? lo : v > hi ? hi : v; } /* trace_math.h:24 */

/* ---- Matrix33 (Matrix33.cpp) ------------------------------------------- */
static m33 m_cols(v3 u, v3 v, v3 n)                                                           /* :10-15 */
{
  m33 m = {u.x, v.x, n.x, u.y, v.y, n.y, u.z, v.z, n.z};
  return m;
}
static v3 m_mul(const m33 *m, v3 v)                                                           /* :230-235 */
{
  return V(v.x * m->m11 + v.y * m->m12 + v.z * m->m13,
           v.x * m->m21 + v.y * m->m22 + v.z * m->m23,
           v.x * m->m31 + v.y * m->m32 + v.z * m->m33);
}
static void m_invert(m33 *m)                                                                  /* :50-79 */
{
  const float d = m->m11 * (m->m22 * m->m33 - m->m32 * m->m23) +
                  m->m21 * (m->m32 * m->m13 - m->m12 * m->m33) +
                  m->m31 * (m->m12 * m->m23 - m->m13 * m->m22);
  if (fabsf(d) > VSN)
  {
    m33 r = {
      (m->m22 * m->m33 - m->m23 * m->m32) / d, (m->m13 * m->m32 - m->m12 * m->m33) / d, (m->m12 * m->m23 - m->m13 * m->m22) / d,
      (m->m23 * m->m31 - m->m21 * m->m33) / d, (m->m11 * m->m33 - m->m13 * m->m31) / d, (m->m13 * m->m21 - m->m11 * m->m23) / d,
      (m->m21 * m->m32 - m->m22 * m->m31) / d, (m->m12 * m->m31 - m->m11 * m->m32) / d, (m->m11 * m->m22 - m->m12 * m->m21) / d};
    *m = r;
  }
  else
  {
    m33 id = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    *m = id;
  }
}

/* ---- Color (Color.cpp) ---------------------------------------------------- */
static inline col C(float r, float g, float b) { col c = {r, g, b}; return c; }
static inline col cadd(col a, col b) { return C(a.r + b.r, a.g + b.g, a.b + b.b); }         /* :78 */
static inline col cmul(col a, col b) { return C(a.r * b.r, a.g * b.g, a.b * b.b); }         /* :108 */
static inline col cscale(col a, float f) { return C(a.r * f, a.g * f, a.b * f); }           /* :88,93 */
static inline col cclamp(col a)                                                               /* :119-124 */
{
  return C(clampf01(a.r, 0.0f, 1.0f), clampf01(a.g, 0.0f, 1.0f), clampf01(a.b, 0.0f, 1.0f));
}
static inline col from_argb(uint32_t c)                                                       /* :9-14 */
{
  return C((float)((c >> 16) & 0xFF) / 255.0f, (float)((c >> 8) & 0xFF) / 255.0f, (float)(c & 0xFF) / 255.0f);
}
/* float -> unsigned char as g++/x86-64 emits it for MAKEARGB (cvttss2si, low byte) */
static inline uint32_t q8(float f) { return (uint32_t)(uint8_t)(int32_t)f; }
uint32_t orc_argb(float r, float g, float b)                                                  /* :114-117, Color.h:11-15 */
{
  return q8(r * 255.999f) << 16 | q8(g * 255.999f) << 8 | q8(b * 255.999f);
}

/* ---- scene ---------------------------------------------------------------- */
typedef struct { uint32_t w, h; uint32_t *texels; } tex_t;
typedef struct { int dielectric; col color; float refl, transp; } mat_t;
typedef struct { v3 center; float radius, sq_radius; mat_t mat; } sphere_t;
typedef struct {
  v3 v0, norm; m33 ax; m33 tuv; float tu0, tv0; int tex; mat_t mat;
} tri_t;
typedef struct { v3 origin; float radius; col color; float power; } light_t;
typedef struct { v3 pos, norm; mat_t mat; } plane_t;
typedef struct { int kind; int idx; } obj_t; /* kind 0 sphere, 1 triangle, 2 plane */

struct orc_scene {
  col diff_color, env_color;
  float diff_power;
  float half_tile_w, half_tile_h;
  int skybox_tex;
  sphere_t *spheres; int n_spheres;
  tri_t *tris; int n_tris;
  plane_t *planes; int n_planes;
  obj_t *objs; int n_objs;
  light_t *lights; int n_lights;
  tex_t *texs; int n_texs;
};

#define GROW(arr, n) (arr = realloc(arr, sizeof(*(arr)) * ((n) + 1)))

orc_scene *orc_scene_new(float dr, float dg, float db, float dp)             /* Scene.cpp:10-15 */
{
  orc_scene *s = calloc(1, sizeof(*s));
  s->diff_color = C(dr, dg, db);
  s->diff_power = dp;
  s->env_color = cscale(s->diff_color, dp);
  s->skybox_tex = -1;
  s->half_tile_w = 1.0f / 8.0f - FLT_EPSILON;                                 /* Skybox.cpp:5-9 */
  s->half_tile_h = 1.0f / 6.0f - FLT_EPSILON;
  return s;
}

void orc_scene_free(orc_scene *s)
{
  if (!s) return;
  for (int i = 0; i < s->n_texs; ++i) free(s->texs[i].texels);
  free(s->texs); free(s->spheres); free(s->tris); free(s->planes); free(s->objs); free(s->lights);
  free(s);
}

int orc_add_texture(orc_scene *s, uint32_t w, uint32_t h, const uint32_t *argb)
{
  GROW(s->texs, s->n_texs);
  tex_t *t = &s->texs[s->n_texs];
  if (!argb || !w || !h) { t->w = t->h = 0; t->texels = NULL; }           /* failed load -> empty (Texture.cpp:97-104) */
  else
  {
    t->w = w; t->h = h;
    t->texels = malloc((size_t)w * h * 4);
    memcpy(t->texels, argb, (size_t)w * h * 4);
  }
  return s->n_texs++;
}

void orc_set_skybox(orc_scene *s, int texture_id)                            /* Skybox.cpp:21-37 */
{
  s->skybox_tex = texture_id;
  if (texture_id >= 0 && s->texs[texture_id].w)
  {
    s->half_tile_w = 1.0f / 8.0f - 1.0f / (float)s->texs[texture_id].w - FLT_EPSILON;
    s->half_tile_h = 1.0f / 6.0f - 1.0f / (float)s->texs[texture_id].h - FLT_EPSILON;
  }
  else
  {
    s->half_tile_w = 1.0f / 8.0f - FLT_EPSILON;
    s->half_tile_h = 1.0f / 6.0f - FLT_EPSILON;
  }
}

int orc_add_light(orc_scene *s, const float o[3], float radius, const float rgb[3], float power) /* Scene.cpp:48-59 */
{
  if (radius <= VSN) radius = VSN;
  col c = C(rgb[0], rgb[1], rgb[2]);
  s->env_color = cadd(s->env_color, cscale(c, power));                       /* envColor += color * power (unclamped power) */
  GROW(s->lights, s->n_lights);
  light_t *l = &s->lights[s->n_lights];
  l->origin = V(o[0], o[1], o[2]);
  l->radius = radius;
  l->color = c;
  l->power = clampf01(power, 0.0f, 1.0f);                                    /* OmniLight.cpp:8-14 */
  return s->n_lights++;
}

static mat_t make_mat(int dielectric, const float rgb[3], float refl, float transp) /* Material.cpp:8-14 */
{
  mat_t m;
  m.dielectric = dielectric != 0;
  m.color = C(rgb[0], rgb[1], rgb[2]);
  m.refl = clampf01(refl, 0.0f, 1.0f);
  m.transp = clampf01(transp, 0.0f, 1.0f);
  return m;
}

int orc_add_sphere(orc_scene *s, const float c[3], float radius, int diel, const float rgb[3], float refl, float transp)
{                                                                            /* Scene.cpp:29-39, Sphere.cpp:9-20 */
  if (radius <= VSN) radius = VSN;
  GROW(s->spheres, s->n_spheres);
  sphere_t *sp = &s->spheres[s->n_spheres];
  sp->center = V(c[0], c[1], c[2]);
  sp->radius = radius;
  sp->sq_radius = radius * radius;
  sp->mat = make_mat(diel, rgb, refl, transp);
  GROW(s->objs, s->n_objs);
  s->objs[s->n_objs].kind = 0;
  s->objs[s->n_objs].idx = s->n_spheres++;
  return s->n_objs++;
}

int orc_add_triangle(orc_scene *s, const float a[3], const float b[3], const float c[3], int diel,
                     const float rgb[3], float refl, float transp)          /* Triangle.cpp:11-21 */
{
  GROW(s->tris, s->n_tris);
  tri_t *t = &s->tris[s->n_tris];
  v3 v0 = V(a[0], a[1], a[2]), v1 = V(b[0], b[1], b[2]), v2 = V(c[0], c[1], c[2]);
  t->v0 = v0;
  t->mat = make_mat(diel, rgb, refl, transp);
  t->norm = tm_normalize(vcross(vsub(v1, v0), vsub(v2, v0)));
  t->ax = m_cols(vsub(v2, v0), vsub(v1, v0), vneg(t->norm));
  m_invert(&t->ax);
  memset(&t->tuv, 0, sizeof(t->tuv));
  t->tu0 = t->tv0 = 0.0f;
  t->tex = -1;
  GROW(s->objs, s->n_objs);
  s->objs[s->n_objs].kind = 1;
  s->objs[s->n_objs].idx = s->n_tris++;
  return s->n_objs++;
}

int orc_add_plane(orc_scene *s, const float pos[3], const float norm[3], int diel, const float rgb[3], float refl,
                  float transp)                                              /* Plane.cpp:9-14 */
{
  GROW(s->planes, s->n_planes);
  plane_t *p = &s->planes[s->n_planes];
  p->pos = V(pos[0], pos[1], pos[2]);
  p->norm = V(norm[0], norm[1], norm[2]);
  p->mat = make_mat(diel, rgb, refl, transp);
  GROW(s->objs, s->n_objs);
  s->objs[s->n_objs].kind = 2;
  s->objs[s->n_objs].idx = s->n_planes++;
  return s->n_objs++;
}

int orc_triangle_set_texture(orc_scene *s, int obj, int tex, const float uv[6]) /* Triangle.cpp:110-120 */
{
  if (obj < 0 || obj >= s->n_objs || s->objs[obj].kind != 1) return -1;
  tri_t *t = &s->tris[s->objs[obj].idx];
  t->tex = tex;
  t->tu0 = uv[0]; t->tv0 = uv[1];
  v3 p1 = V(uv[0], uv[1], 0), p2 = V(uv[2], uv[3], 0), p3 = V(uv[4], uv[5], 0);
  t->tuv = m_cols(vsub(p3, p1), vsub(p2, p1), V(0, 0, -1));
  return 0;
}

void orc_camera_view(const float e[3], const float a[3], float view[9])     /* Camera.cpp:24-38 */
{
  v3 eye = V(e[0], e[1], e[2]), at = V(a[0], a[1], a[2]);
  v3 up = V(0.0f, 1.0f, 0.0f);
  v3 oz = tm_normalize(vsub(at, eye));
  v3 ox = tm_normalize(vcross(up, oz));
  v3 oy = tm_normalize(vcross(oz, ox));
  m33 m = m_cols(ox, oy, oz);                                                /* setCol(0..2) (Matrix33.cpp:130-135) */
  memcpy(view, &m, 36);
}

/* ---- sampling --------------------------------------------------------------- */
static col texel_xy(const tex_t *t, uint32_t x, uint32_t y)                 /* Texture.cpp:216-229 */
{
  if (x >= t->w || y >= t->h) return C(0, 0, 0);
  if (!t->texels)
    return (((x * 50 / t->w) % 2) ^ ((y * 50 / t->w) % 2)) ? C(0.5f, 0.5f, 0.5f) : C(0.75f, 0.75f, 0.75f);
  return from_argb(t->texels[x + t->w * y]);
}

/* *cat receives the ORC_TEX_* category of the sample (for the event counters) */
static col texel_uv(const tex_t *t, float u, float v, int *cat)             /* Texture.cpp:231-269 */
{
  if (u < 0.0f || u > 1.0f || v < 0.0f || v > 1.0f) { *cat = ORC_TEX_OTHER; return C(0, 0, 0); }
  if (!t || !t->texels)
  {
    *cat = ORC_TEX_CHECKER;
    return (((int)(u * 50) % 2) ^ ((int)(v * 50) % 2)) ? C(0.5f, 0.5f, 0.5f) : C(0.75f, 0.75f, 0.75f);
  }
  const float fx = clampf01(u, 0.0f, 1.0f - FLT_EPSILON) * (float)t->w;
  const float fy = clampf01(v, 0.0f, 1.0f - FLT_EPSILON) * (float)t->h;
  const uint32_t x = (uint32_t)fx, y = (uint32_t)fy;
  if (x < t->w - 1 && y < t->h - 1)
  {
    *cat = ORC_TEX_BILINEAR;
    const col c00 = texel_xy(t, x, y), c01 = texel_xy(t, x, y + 1);
    const col c10 = texel_xy(t, x + 1, y), c11 = texel_xy(t, x + 1, y + 1);
    const float uf = fx - floorf(fx), vf = fy - floorf(fy);
    const float uo = 1 - uf, vo = 1 - vf;
    return cadd(cscale(cadd(cscale(c00, uo), cscale(c10, uf)), vo), cscale(cadd(cscale(c01, uo), cscale(c11, uf)), vf));
  }
  *cat = ORC_TEX_OTHER;
  return texel_xy(t, (uint32_t)fx, (uint32_t)fy);
}

static col skybox_texel(const orc_scene *s, v3 ray, uint64_t *cnt)        /* Skybox.cpp:39-106 */
{
  const float uLeft = 1.0f / 8.0f, vLeft = 3.0f / 6.0f;
  const float uFront = 3.0f / 8.0f, vFront = 3.0f / 6.0f;
  const float uRight = 5.0f / 8.0f, vRight = 3.0f / 6.0f;
  const float uBack = 7.0f / 8.0f, vBack = 3.0f / 6.0f;
  const float uTop = 3.0f / 8.0f, vTop = 5.0f / 6.0f;
  const float uBottom = 3.0f / 8.0f, vBottom = 1.0f / 6.0f;
  const float hw = s->half_tile_w, hh = s->half_tile_h;
  const v3 n = tm_normalize(ray);
  const float x = n.x, y = n.y, z = n.z;
  const float ax = fabsf(x) + VSN, ay = fabsf(y) + VSN, az = fabsf(z) + VSN;
  float u, v;
  if (az >= ax && az >= ay)
  {
    if (z > 0) { u = uFront + x / az * hw; v = vFront + y / az * hh; }
    else { u = uBack - x / az * hw; v = vBack + y / az * hh; }
  }
  else if (ax >= ay && ax >= az)
  {
    if (x > 0) { u = uRight - z / ax * hw; v = vRight + y / ax * hh; }
    else { u = uLeft + z / ax * hw; v = vLeft + y / ax * hh; }
  }
  else
  {
    if (y > 0) { u = uTop + x / ay * hw; v = vTop - z / ay * hh; }
    else { u = uBottom + x / ay * hw; v = vBottom + z / ay * hh; }
  }
  const tex_t *t = s->skybox_tex >= 0 ? &s->texs[s->skybox_tex] : NULL;
  int cat;
  const col c = texel_uv(t, u, v, &cat);
  if (cnt) cnt[cat]++;
  return c;
}

/* ---- primitives ------------------------------------------------------------- */
/* tex_cat: ORC_TEX_* category of a textured triangle's sample, -1 if untextured */
typedef struct { v3 drop, norm, refl; float dist; mat_t mat; int tex_cat; } hit_t;

/* Sphere::trace (Sphere.cpp:44-85); out == NULL -> any-hit query */
static int sphere_trace(const sphere_t *sp, v3 o, v3 ray, hit_t *out, uint64_t *cnt, int shadow)
{
  if (cnt) cnt[shadow ? ORC_SH_SPH_TESTS : ORC_SPH_TESTS]++;
  const v3 vco = vsub(o, sp->center);
  const float a = vsqlen(ray);
  const float b = vdot(vmul(ray, 2.0f), vco);
  const float c = vsqlen(vco) - sp->sq_radius;
  const float d = b * b - 4.0f * a * c;
  /* counters mirror the events of the GPU formulation: B = the test survives the (exact) b > 0 reject */
  if (cnt && !(b > 0.0f)) cnt[shadow ? ORC_SH_SPH_B : ORC_SPH_B]++;
  if (d >= 0.0f && a > VSN)
  {
    if (cnt && !(b > 0.0f)) cnt[shadow ? ORC_SH_SPH_D : ORC_SPH_D]++;
    const float t = (-b - sqrtf(d)) / (2.0f * a);
    if (t > VSN)
    {
      if (cnt) cnt[shadow ? ORC_SH_SPH_T : ORC_SPH_T]++;
      const v3 full = vmul(ray, t);
      const float dist = vlen(full);
      if (dist > DELTA)
      {
        if (out)
        {
          out->tex_cat = -1;
          out->dist = dist;
          out->drop = vadd(o, full);
          out->norm = vsub(out->drop, sp->center);
          out->refl = tm_reflect(full, out->norm);
          out->mat = sp->mat;
        }
        return 1;
      }
    }
  }
  return 0;
}

/* Triangle::trace (Triangle.cpp:53-108) */
static int tri_trace(const orc_scene *s, const tri_t *tr, v3 o, v3 ray, hit_t *out, uint64_t *cnt, int shadow)
{
  if (cnt) cnt[shadow ? ORC_SH_TRI_TESTS : ORC_TRI_TESTS]++;
  const v3 ao = m_mul(&tr->ax, vsub(o, tr->v0));
  const v3 ar = m_mul(&tr->ax, ray);
  if (fabsf(ar.z) > VSN)
  {
    if (cnt) cnt[shadow ? ORC_SH_TRI_Z : ORC_TRI_Z]++;
    /* S = -ao.z and ar.z have equal, non-zero signs (the GPU's exact pre-check before dividing) */
    if (cnt && ((-ao.z > 0.0f && ar.z > 0.0f) || (-ao.z < 0.0f && ar.z < 0.0f))) cnt[shadow ? ORC_SH_TRI_S : ORC_TRI_S]++;
    const float t = -ao.z / ar.z;
    if (t > VSN)
    {
      if (cnt) cnt[shadow ? ORC_SH_TRI_T : ORC_TRI_T]++;
      const float u = ao.x + t * ar.x;
      const float v = ao.y + t * ar.y;
      if (u >= 0.0f && v >= 0.0f && u + v < 1.0f)
      {
        if (cnt) cnt[shadow ? ORC_SH_TRI_IN : ORC_TRI_IN]++;
        const v3 full = vmul(ray, t);
        const float sq = vsqlen(full);
        if (sq > DELTA * DELTA)
        {
          if (out)
          {
            if (cnt) cnt[ORC_TRI_D]++;
            out->drop = vadd(o, full);
            out->norm = tr->norm;
            out->refl = tm_reflect(full, tr->norm);
            out->dist = sqrtf(sq);
            out->mat = tr->mat;
            out->tex_cat = -1;
            if (tr->tex >= 0)
            {
              /* the reference samples the texel for every candidate hit; only the winner's is used,
                 so only the winner's sample is counted (scene_trace) -- the GPU samples the winner only */
              const v3 tv = m_mul(&tr->tuv, V(u, v, 0));
              out->mat.color = texel_uv(&s->texs[tr->tex], tr->tu0 + tv.x, tr->tv0 + tv.y, &out->tex_cat);
            }
          }
          return 1;
        }
      }
    }
  }
  return 0;
}

/* Plane::trace (Plane.cpp:36-73); in a scene through the addPlane extension (the reference's Scene has none) */
static int plane_trace(v3 pos, v3 norm, v3 o, v3 ray, hit_t *out, uint64_t *cnt, int shadow)
{
  if (cnt) cnt[shadow ? ORC_SH_PLN_TESTS : ORC_PLN_TESTS]++;
  const v3 vop = vsub(pos, o);
  const float a = vdot(norm, ray);
  if (fabsf(a) > VSN)
  {
    const float t = vdot(norm, vop) / a;
    if (t > VSN)
    {
      if (cnt) cnt[shadow ? ORC_SH_PLN_T : ORC_PLN_T]++;
      const v3 full = vmul(ray, t);
      const float sq = vsqlen(full);
      if (sq > DELTA * DELTA)
      {
        if (out)
        {
          out->drop = vadd(o, full);
          out->norm = norm;
          out->refl = tm_reflect(full, norm);
          out->dist = sqrtf(sq);
          out->tex_cat = -1;
        }
        return 1;
      }
    }
  }
  return 0;
}

/* ---- Scene::trace (Scene.cpp:73-236) ----------------------------------------- */
static col scene_trace(const orc_scene *s, v3 origin, v3 ray, int depth, v3 randDir, uint64_t *cnt)
{
  col mulColor = C(1.0f, 1.0f, 1.0f);
  col pixel = C(0.0f, 0.0f, 0.0f);
  if (cnt) cnt[ORC_RAYS]++;
  for (int refl = 0; refl < depth; ++refl)
  {
    if (cnt) cnt[ORC_SEGMENTS]++;
    float minDistance = FLT_MAX;
    int hitObj = -1;
    hit_t best, cur;
    for (int i = 0; i < s->n_objs; ++i)                                       /* :86-106, strict '<' keeps the first */
    {
      const obj_t *ob = &s->objs[i];
      int h;
      if (ob->kind == 0) h = sphere_trace(&s->spheres[ob->idx], origin, ray, &cur, cnt, 0);
      else if (ob->kind == 1) h = tri_trace(s, &s->tris[ob->idx], origin, ray, &cur, cnt, 0);
      else
      {
        const plane_t *pl = &s->planes[ob->idx];
        h = plane_trace(pl->pos, pl->norm, origin, ray, &cur, cnt, 0);
        cur.mat = pl->mat;
      }
      if (h && cur.dist < minDistance)
      {
        minDistance = cur.dist;
        best = cur;
        hitObj = i;
      }
    }
    if (hitObj >= 0)
    {
      if (cnt)
      {
        const int k = s->objs[hitObj].kind;
        cnt[k == 0 ? ORC_HIT_SPH : k == 1 ? ORC_HIT_TRI : ORC_HIT_PLN]++;
        if (best.tex_cat >= 0) cnt[best.tex_cat]++;
      }
      const v3 drop = best.drop, norm = best.norm, reflect = best.refl;
      const mat_t *dm = &best.mat;
      const float rayLen = vlen(ray), normLen = vlen(norm), reflectLen = vlen(reflect);
      col sumLight = C(0, 0, 0), sumSpec = C(0, 0, 0);
      for (int li = 0; li < s->n_lights; ++li)                                /* :117-181 */
      {
        const light_t *L = &s->lights[li];
        if (cnt) cnt[ORC_L_EVAL]++;
        const v3 dropToLight = vsub(L->origin, drop);
        if (vdot(dropToLight, norm) > VSN)
        {
          if (cnt) cnt[ORC_L_FACING]++;
          const float lightRadius = L->radius;
          const v3 shadowRay = vadd(dropToLight, vmul(randDir, lightRadius));
          int inShadow = 0;
          for (int i = 0; i < s->n_objs; ++i)
          {
            if (i == hitObj) continue;
            const obj_t *ob = &s->objs[i];
            if (ob->kind == 0 ? sphere_trace(&s->spheres[ob->idx], drop, shadowRay, NULL, cnt, 1)
                : ob->kind == 1 ? tri_trace(s, &s->tris[ob->idx], drop, shadowRay, NULL, cnt, 1)
                                : plane_trace(s->planes[ob->idx].pos, s->planes[ob->idx].norm, drop, shadowRay, NULL, cnt, 1))
            {
              inShadow = 1;
              break;
            }
          }
          if (!inShadow)
          {
            if (cnt) cnt[ORC_L_LIT]++;
            const float dropToLightLen = vlen(dropToLight);
            float a = dropToLightLen * normLen;
            const float lightDropCos = (a > VSN) ? vdot(dropToLight, norm) / a : 0.0f;
            if (L->power > VSN) sumLight = cadd(sumLight, cscale(cscale(L->color, lightDropCos), L->power));
            a = vsqlen(dropToLight);
            const float angSqCos = (a > VSN) ? 1.0f - lightRadius * lightRadius / a : 0.0f;
            if (angSqCos > 0)
            {
              if (cnt) cnt[ORC_L_SPEC]++;
              const v3 dropToLightRand = vadd(vnormalized(dropToLight), vmul(randDir, 1.0f - dm->refl));
              a = vlen(dropToLightRand) * reflectLen;
              float specCos = (a > VSN) ? vdot(dropToLightRand, reflect) / a : 0.0f;
              specCos = clampf01(specCos + (1.0f - sqrtf(angSqCos)), 0.0f, 1.0f);
              if (specCos > VSN && lightRadius > VSN)
              {
                if (cnt) cnt[ORC_L_POW]++;
                const float sp = powf(specCos, 1 + 3 * dm->refl * dropToLightLen / lightRadius) * dm->refl;
                sumSpec = cadd(sumSpec, cscale(L->color, sp));
              }
            }
          }
        }
      }
      const float reflectivity = dm->refl;
      const col color = dm->color;
      sumLight = cadd(cscale(s->diff_color, s->diff_power), sumLight);        /* :186 */
      col fin;
      if (dm->dielectric)                                                      /* :189-201 */
      {
        if (cnt) cnt[ORC_DIELECTRIC]++;
        const float a = rayLen * normLen;
        const float cosA = (a > VSN) ? clampf01(vdot(ray, vneg(norm)) / a, 0.0f, 1.0f) : 0.0f;
        const float r = 0.2f + 0.8f * powf(1.0f - cosA, 3.0f);
        fin = cadd(cmul(cscale(color, 1.0f - r), sumLight), sumSpec);
        fin = cmul(fin, mulColor);
        mulColor = cscale(mulColor, r);
      }
      else                                                                     /* :202-212 */
      {
        if (cnt) cnt[ORC_METAL]++;
        const float r = 0.8f;
        fin = cadd(cmul(cscale(color, 1.0f - r), sumLight), sumSpec);
        fin = cmul(fin, mulColor);
        mulColor = cmul(mulColor, cscale(color, r));
      }
      pixel = cclamp(cadd(pixel, fin));                                        /* :215-216 */
      if (mulColor.r < 0.01f && mulColor.g < 0.01f && mulColor.b < 0.01f) break; /* :219-220 */
      if (cnt) cnt[ORC_CONTINUE]++;
      origin = drop;                                                           /* :223-224 */
      ray = vadd(vnormalized(reflect), vmul(randDir, 1.0f - reflectivity));
    }
    else                                                                       /* :226-231 */
    {
      if (cnt) cnt[ORC_SKY]++;
      pixel = cclamp(cadd(pixel, cmul(cmul(mulColor, skybox_texel(s, ray, cnt)), s->env_color)));
      break;
    }
  }
  return pixel;
}

/* ---- RNG (trace_math.h:34-39, Vector3.cpp:176-188) ----------------------- */
static inline uint32_t lcg(uint32_t *s)
{
  *s = 214013u * *s + 2531011u;
  return (*s >> 16) & 0x7FFF;
}
static inline v3 random_inside_sphere(uint32_t *s)
{
  v3 v;
  do
  {
    v.x = (float)lcg(s) / ((float)0x7FFF / 2) - 1.f;
    v.y = (float)lcg(s) / ((float)0x7FFF / 2) - 1.f;
    v.z = (float)lcg(s) / ((float)0x7FFF / 2) - 1.f;
  } while (vsqlen(v) > 1.f);
  return vmul(v, 1.0f);
}

void orc_rand_dirs(uint32_t *seed, uint64_t n, float *out)
{
  for (uint64_t i = 0; i < n; ++i)
  {
    v3 d = random_inside_sphere(seed);
    out[i * 3] = d.x; out[i * 3 + 1] = d.y; out[i * 3 + 2] = d.z;
  }
}

/* ---- Render::renderNext (Render.cpp:136-215) --------------------------------- */
typedef struct {
  const orc_scene *s;
  v3 eye; m33 view; float rz, wh, hh;
  uint32_t W, H; int depth, ss, accumulate;
  const v3 *rand_dirs;      /* per trace, in the reference's trace order */
  const float *jitter;      /* 2 per pixel (additive) or NULL */
  float *image;
  uint32_t y_begin, y_end, y_step;  /* rows of this worker: y_begin, y_begin + y_step, .. < y_end */
  uint64_t cnt[ORC_NCOUNTERS];
  int counting;
} job_t;

static void *render_rows(void *arg)
{
  job_t *j = (job_t *)arg;
  uint64_t *cnt = j->counting ? j->cnt : NULL;
  const uint32_t W = j->W, H = j->H;
  if (j->ss < 0)
  {
    const uint32_t n = (uint32_t)(-j->ss);
    const uint32_t bw = (W + n - 1) / n;
    for (uint32_t y = j->y_begin; y < j->y_end; ++y)
    {
      if (y % n) continue;
      for (uint32_t x = 0; x < W; x += n)
      {
        const v3 ray = m_mul(&j->view, V((float)x - j->wh, (float)y - j->hh, j->rz));
        const col c = scene_trace(j->s, j->eye, ray, j->depth, j->rand_dirs[(size_t)(y / n) * bw + x / n], cnt);
        const uint32_t ex = x + n < W ? x + n : W, ey = y + n < H ? y + n : H;
        for (uint32_t qx = x; qx < ex; ++qx)
          for (uint32_t qy = y; qy < ey; ++qy)
          {
            float *p = &j->image[((size_t)qx + (size_t)qy * W) * 3];
            p[0] = c.r; p[1] = c.g; p[2] = c.b;
          }
      }
    }
    return NULL;
  }
  const int ss = j->ss;
  const float sq = (float)(ss * ss);
  for (uint32_t y = j->y_begin; y < j->y_end; y += j->y_step)
    for (uint32_t x = 0; x < W; ++x)
    {
      const size_t p = (size_t)y * W + x;
      const float rx = (float)x - j->wh, ry = (float)y - j->hh;
      const float rndx = j->jitter ? j->jitter[p * 2] : 0;
      const float rndy = j->jitter ? j->jitter[p * 2 + 1] : 0;
      col fin = C(0.0f, 0.0f, 0.0f);
      for (int sx = 0; sx < ss; ++sx)
        for (int sy = 0; sy < ss; ++sy)
        {
          v3 ray = V(rx + (float)sx / (float)ss + rndx, ry + (float)sy / (float)ss + rndy, j->rz);
          ray = m_mul(&j->view, ray);
          fin = cadd(fin, scene_trace(j->s, j->eye, ray, j->depth, j->rand_dirs[p * (size_t)(ss * ss) + (size_t)(sx * ss + sy)], cnt));
        }
      if (fabsf(sq) > VSN) fin = C(fin.r / sq, fin.g / sq, fin.b / sq);     /* Color::operator/= (Color.cpp:64-76) */
      float *d = &j->image[p * 3];
      if (j->accumulate) { d[0] += fin.r; d[1] += fin.g; d[2] += fin.b; }
      else { d[0] = fin.r; d[1] = fin.g; d[2] = fin.b; }
    }
  return NULL;
}

static int run_jobs(job_t *proto, uint32_t y0, uint32_t y1, int nthreads, uint64_t *counters)
{
  if (nthreads < 1) nthreads = 1;
  job_t *jobs = calloc((size_t)nthreads, sizeof(job_t));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  const uint32_t rows = y1 - y0;
  uint32_t n_blk = (uint32_t)(-proto->ss > 0 ? -proto->ss : 1);
  for (int t = 0; t < nthreads; ++t)
  {
    jobs[t] = *proto;
    uint32_t a = y0 + (uint32_t)((uint64_t)rows * t / nthreads), b = y0 + (uint32_t)((uint64_t)rows * (t + 1) / nthreads);
    if (proto->ss < 0)
    { /* keep whole n-row blocks together */
      a = (a + n_blk - 1) / n_blk * n_blk; b = (b + n_blk - 1) / n_blk * n_blk;
      if (t == nthreads - 1) b = y1;
    }
    jobs[t].y_begin = a; jobs[t].y_end = b > y1 ? y1 : b; jobs[t].y_step = 1;
    if (proto->ss > 0)
    { /* pixel rows interleaved over the workers (rows differ in cost: sky vs geometry) */
      jobs[t].y_begin = y0 + (uint32_t)t; jobs[t].y_end = y1; jobs[t].y_step = (uint32_t)nthreads;
    }
    memset(jobs[t].cnt, 0, sizeof(jobs[t].cnt));
  }
  if (nthreads == 1) render_rows(&jobs[0]);
  else
  {
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, render_rows, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  if (counters)
    for (int t = 0; t < nthreads; ++t)
      for (int k = 0; k < ORC_NCOUNTERS; ++k) counters[k] += jobs[t].cnt[k];
  free(jobs); free(th);
  return 0;
}

int orc_render(const orc_scene *s, const float eye[3], const float view[9], float fov,
               uint32_t W, uint32_t H, int depth, int ss, int additive, int additive_counter,
               uint32_t *sphere_seed, uint32_t *jitter_seed, float *image, int nthreads, uint64_t *counters)
{
  if (!W || !H || ss == 0 || depth <= 0) return -1;
  job_t j;
  memset(&j, 0, sizeof(j));
  j.s = s;
  j.eye = V(eye[0], eye[1], eye[2]);
  memcpy(&j.view, view, 36);
  j.rz = (float)W / 2.0f / tanf(fov / 2.0f);                                 /* Render.cpp:148 */
  j.wh = W / 2.0f; j.hh = H / 2.0f;
  j.W = W; j.H = H; j.depth = depth; j.ss = ss;
  j.image = image;
  j.counting = counters != NULL;
  size_t traces;
  if (ss < 0) { uint32_t n = (uint32_t)(-ss); traces = (size_t)((W + n - 1) / n) * ((H + n - 1) / n); }
  else traces = (size_t)W * H * (size_t)(ss * ss);
  v3 *dirs = malloc(sizeof(v3) * (traces ? traces : 1));
  float *jit = NULL;
  if (ss > 0)
  {
    j.accumulate = additive_counter > 1;                                     /* :191-194 */
    if (additive)
    { /* Render.cpp's own stream: rndx then rndy, once per pixel, raster order (:177-178) */
      jit = malloc(sizeof(float) * 2 * (size_t)W * H);
      for (size_t p = 0; p < (size_t)W * H; ++p)
      {
        jit[p * 2] = (float)lcg(jitter_seed) / (float)0x7FFF;
        jit[p * 2 + 1] = (float)lcg(jitter_seed) / (float)0x7FFF;
      }
    }
  }
  for (size_t i = 0; i < traces; ++i) dirs[i] = random_inside_sphere(sphere_seed);
  j.rand_dirs = dirs;
  j.jitter = jit;
  run_jobs(&j, 0, H, nthreads, counters);
  free(dirs); free(jit);
  return 0;
}

int orc_render_band(const orc_scene *s, const float eye[3], const float view[9], float fov,
                    uint32_t W, uint32_t H, int depth, uint32_t y0, uint32_t rows,
                    uint32_t seed, float *rgb_out, uint32_t *argb_out, int nthreads, uint64_t *counters)
{
  if (!W || !rows || y0 + rows > H) return -1;
  for (size_t i = 0; i < (size_t)y0 * W; ++i) random_inside_sphere(&seed);
  job_t j;
  memset(&j, 0, sizeof(j));
  j.s = s;
  j.eye = V(eye[0], eye[1], eye[2]);
  memcpy(&j.view, view, 36);
  j.rz = (float)W / 2.0f / tanf(fov / 2.0f);
  j.wh = W / 2.0f; j.hh = H / 2.0f;
  j.W = W; j.H = H; j.depth = depth; j.ss = 1;
  j.counting = counters != NULL;
  /* render into a full-height scratch image, band rows only */
  float *img = calloc((size_t)W * H * 3, sizeof(float));
  v3 *dirs = malloc(sizeof(v3) * (size_t)W * H);
  for (size_t i = (size_t)y0 * W; i < (size_t)(y0 + rows) * W; ++i) dirs[i] = random_inside_sphere(&seed);
  j.rand_dirs = dirs;
  j.image = img;
  run_jobs(&j, y0, y0 + rows, nthreads, counters);
  for (size_t i = 0; i < (size_t)W * rows; ++i)
  {
    const float *p = &img[((size_t)y0 * W + i) * 3];
    if (rgb_out) { rgb_out[i * 3] = p[0]; rgb_out[i * 3 + 1] = p[1]; rgb_out[i * 3 + 2] = p[2]; }
    if (argb_out) argb_out[i] = orc_argb(p[0], p[1], p[2]);
  }
  free(img); free(dirs);
  return 0;
}

/* ---- KAT entry points ----------------------------------------------------- */
static const float KAT_RGB[3] = {0.25f, 0.5f, 0.75f};

static void write_hit(float *w, int hit, const hit_t *h, int any)
{
  memset(w, 0, 15 * sizeof(float));
  w[0] = hit ? 1.0f : 0.0f;
  if (hit)
  {
    w[1] = h->drop.x; w[2] = h->drop.y; w[3] = h->drop.z;
    w[4] = h->norm.x; w[5] = h->norm.y; w[6] = h->norm.z;
    w[7] = h->refl.x; w[8] = h->refl.y; w[9] = h->refl.z;
    w[10] = h->dist;
    w[11] = h->mat.color.r; w[12] = h->mat.color.g; w[13] = h->mat.color.b;
  }
  w[14] = any ? 1.0f : 0.0f;
}

void orc_kat_sphere(const float *f, uint64_t n, float *out)
{
  orc_scene *s = orc_scene_new(0, 0, 0, 0);
  for (uint64_t i = 0; i < n; ++i, f += 11)
  {
    s->n_spheres = 0; s->n_objs = 0;
    orc_add_sphere(s, f + 6, f[9], 0, KAT_RGB, 0.5f, 0.0f);
    hit_t h;
    int hit = sphere_trace(&s->spheres[0], V(f[0], f[1], f[2]), V(f[3], f[4], f[5]), &h, NULL, 0);
    int any = sphere_trace(&s->spheres[0], V(f[0], f[1], f[2]), V(f[3], f[4], f[5]), NULL, NULL, 1);
    write_hit(out + i * 15, hit, &h, any);
  }
  orc_scene_free(s);
}

void orc_kat_triangle(const float *f, uint64_t n, uint32_t tw, uint32_t th, const uint32_t *argb, int textured, float *out)
{
  orc_scene *s = orc_scene_new(0, 0, 0, 0);
  int tex = orc_add_texture(s, tw, th, argb);
  for (uint64_t i = 0; i < n; ++i, f += 21)
  {
    s->n_tris = 0; s->n_objs = 0;
    int obj = orc_add_triangle(s, f + 6, f + 9, f + 12, 0, KAT_RGB, 0.5f, 0.0f);
    if (textured) orc_triangle_set_texture(s, obj, tex, f + 15);
    hit_t h;
    int hit = tri_trace(s, &s->tris[0], V(f[0], f[1], f[2]), V(f[3], f[4], f[5]), &h, NULL, 0);
    int any = tri_trace(s, &s->tris[0], V(f[0], f[1], f[2]), V(f[3], f[4], f[5]), NULL, NULL, 1);
    write_hit(out + i * 15, hit, &h, any);
  }
  orc_scene_free(s);
}

void orc_kat_plane(const float *f, uint64_t n, float *out)
{
  for (uint64_t i = 0; i < n; ++i, f += 12)
  {
    hit_t h;
    memset(&h, 0, sizeof(h));
    v3 pos = V(f[6], f[7], f[8]), nn = V(f[9], f[10], f[11]), o = V(f[0], f[1], f[2]), r = V(f[3], f[4], f[5]);
    int hit = plane_trace(pos, nn, o, r, &h, NULL, 0);
    h.mat.color = C(KAT_RGB[0], KAT_RGB[1], KAT_RGB[2]);
    int any = plane_trace(pos, nn, o, r, NULL, NULL, 1);
    write_hit(out + i * 15, hit, &h, any);
  }
}

void orc_kat_skybox(uint32_t tw, uint32_t th, const uint32_t *argb, const float *rays, uint64_t n, float *out)
{
  orc_scene *s = orc_scene_new(0, 0, 0, 0);
  if (argb && tw && th) orc_set_skybox(s, orc_add_texture(s, tw, th, argb));
  for (uint64_t i = 0; i < n; ++i)
  {
    col c = skybox_texel(s, V(rays[i * 3], rays[i * 3 + 1], rays[i * 3 + 2]), NULL);
    out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
  }
  orc_scene_free(s);
}

void orc_kat_texture(uint32_t tw, uint32_t th, const uint32_t *argb, const float *uv, uint64_t n, float *out)
{
  tex_t t = {argb ? tw : 0, argb ? th : 0, (uint32_t *)argb};
  for (uint64_t i = 0; i < n; ++i)
  {
    int cat;
    col c = texel_uv(&t, uv[i * 2], uv[i * 2 + 1], &cat);
    out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
  }
}
