// Host side of librfx.so: the C-ABI of include/rfx.h.
//
// Scene builder calls restate the reference's constructors (host precompute in
// strict IEEE, shared rfx_math.h), uploads go to SoA device arrays
// (rfx_types.h), and rfx_render_frame enqueues the RNG pre-pass + trace kernel
// on one HIP stream without any host synchronisation.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rfx.h"
#include "rfx_math.h"
#include "rfx_types.h"

#pragma clang fp contract(off)

namespace rfx {
uint64_t rng_blocks_for(uint64_t traces);
void rng_jump_table(uint64_t nblk, uint32_t *out);
hipError_t launch_rng_count(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_blk_cnt, uint64_t blk0,
                            uint64_t nblk_slice, uint16_t *d_masks, hipStream_t st);
hipError_t launch_rng_finish(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed,
                             const uint32_t *d_blk_cnt, const uint16_t *d_masks, uint64_t nblk, uint64_t traces,
                             uint32_t *d_rd_state, int *d_err, uint64_t ss2, uint64_t W, uint32_t row_block,
                             uint32_t rank, uint32_t nranks, hipStream_t st);
hipError_t launch_rng_finish_band(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed,
                                  const uint32_t *d_blk_cnt, const uint16_t *d_masks, uint64_t nblk, uint64_t traces,
                                  uint32_t *d_rd_state, int *d_err, uint64_t lo, uint64_t hi, uint64_t *d_off,
                                  uint32_t *d_range, uint32_t *d_tile_sum, hipStream_t st);
hipError_t launch_rng_fused(const uint32_t *d_seed, const uint32_t *d_jump, uint32_t *d_next_seed, uint64_t nblk,
                            uint64_t traces, uint32_t *d_rd_state, int *d_err, unsigned long long *d_status,
                            unsigned long long *d_ticket, unsigned long long base, uint32_t epoch, hipStream_t st);
hipError_t launch_trace(const DevScene &S, const FrameParams &P, bool stats, hipStream_t st);
hipError_t launch_prim_cull(const DevScene &S, const FrameParams &P, uint64_t *masks, hipStream_t st);
hipError_t launch_queue_sort(const uint32_t *count, const uint32_t *key, uint32_t *hist, uint32_t *order, hipStream_t st);
uint32_t trace_tiles(const FrameParams &P);
bool trace_lanes(const FrameParams &P);
bool trace_chunks(const FrameParams &P);
size_t tile_order_scratch();
hipError_t launch_tile_order(const uint32_t *cost, uint32_t n, uint32_t *order, uint32_t *scratch, hipStream_t st);
void launch_bounce(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st);
hipError_t launch_bounce_lds(int cfg, uint32_t groups, const DevScene &S, const FrameParams &P, hipStream_t st);
hipError_t launch_kat(int what, const DevScene &S, int tex, const void *in, const int32_t *objs, uint32_t n, void *out,
                      hipStream_t st);
hipError_t launch_kat_powf_cube(uint32_t first, uint32_t n, unsigned long long *counts, hipStream_t st);
hipError_t launch_kat_div(uint64_t first, uint32_t n, unsigned long long *counts, hipStream_t st);
hipError_t launch_kat_kernarg(const DevScene &S, const FrameParams &P, int swapped, uint32_t *out, hipStream_t st);
}  // namespace rfx

using namespace rfx;

static thread_local std::string g_last_error;

static int fail(int code, const char *fmt, ...)
{
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(RFX_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

extern "C" int rfx_abi_version(void) { return RFX_ABI_VERSION; }
extern "C" const char *rfx_last_error(void) { return g_last_error.c_str(); }

// ============================================================== scene (host)
// w x h as loaded; no texels = the reference's empty colorBuf (procedural checker).  loaded: the file was read
// (Skybox::loadTexture then derives its half tiles from w and h, Skybox.cpp:21-37).
struct HostTexture { uint32_t w = 0, h = 0; bool loaded = false; std::vector<uint32_t> texels; };
struct HostMat { int dielectric; float r, g, b, refl, transp; };
struct HostSphere { v3 center; float radius, sq_radius; HostMat mat; int obj; };
struct HostTri {
  v3 v0, v1, v2, norm;
  double cond = INFINITY;  // ||M||_F ||M^-1||_F of the basis M = [v2-v0 | v1-v0 | -norm] (cull bound)
  m33 ax, tuv;
  float tu0 = 0, tv0 = 0;
  int tex = -1;
  HostMat mat;
  int obj;
};
struct HostLight { v3 origin; float radius; float r, g, b, power; };
struct HostPlane { v3 pos, norm; HostMat mat; int obj; };

struct rfx_scene {
  col diff, env;
  float diff_power;
  float half_tile_w, half_tile_h;
  int skybox = -1;
  std::vector<HostSphere> spheres;
  std::vector<HostTri> tris;
  std::vector<HostPlane> planes;
  std::vector<int> obj_kind, obj_idx;  // insertion order: kind 0 sphere, 1 triangle, 2 plane
  std::vector<HostLight> lights;
  std::vector<HostTexture> textures;
};

static void default_half_tiles(rfx_scene *s)  // Skybox.cpp:5-9 / failed load :32-33
{
  s->half_tile_w = 1.0f / 8.0f - kFltEpsilon;
  s->half_tile_h = 1.0f / 6.0f - kFltEpsilon;
}

extern "C" rfx_scene *rfx_scene_create(float dr, float dg, float db, float dp)   // Scene.cpp:10-15
{
  rfx_scene *s = new rfx_scene();
  s->diff = mkc(dr, dg, db);
  s->diff_power = dp;
  s->env = cscale(s->diff, dp);
  default_half_tiles(s);
  return s;
}

extern "C" void rfx_scene_destroy(rfx_scene *s) { delete s; }

static HostMat make_mat(int type, const float rgb[3], float refl, float transp)      // Material.cpp:8-14
{
  HostMat m;
  m.dielectric = type == RFX_DIELECTRIC;
  m.r = rgb[0]; m.g = rgb[1]; m.b = rgb[2];
  m.refl = clampf(refl, 0.0f, 1.0f);
  m.transp = clampf(transp, 0.0f, 1.0f);
  return m;
}

extern "C" int rfx_scene_add_sphere(rfx_scene *s, const float c[3], float radius, int type, const float rgb[3],
                                    float refl, float transp)                          // Scene.cpp:29-39
{
  if (!s || !c || !rgb || (type != RFX_METAL && type != RFX_DIELECTRIC)) return fail(RFX_ERR_ARG, "add_sphere: bad args");
  if (radius <= kVerySmall) radius = kVerySmall;
  HostSphere sp;
  sp.center = mk(c[0], c[1], c[2]);
  sp.radius = radius;
  sp.sq_radius = radius * radius;                                                    // Sphere.cpp:19
  sp.mat = make_mat(type, rgb, refl, transp);
  sp.obj = (int)s->obj_kind.size();
  s->obj_kind.push_back(0);
  s->obj_idx.push_back((int)s->spheres.size());
  s->spheres.push_back(sp);
  return sp.obj;
}

extern "C" int rfx_scene_add_triangle(rfx_scene *s, const float a[3], const float b[3], const float c[3], int type,
                                      const float rgb[3], float refl, float transp)    // Triangle.cpp:11-21
{
  if (!s || !a || !b || !c || !rgb || (type != RFX_METAL && type != RFX_DIELECTRIC))
    return fail(RFX_ERR_ARG, "add_triangle: bad args");
  HostTri t;
  const v3 v0 = mk(a[0], a[1], a[2]), v1 = mk(b[0], b[1], b[2]), v2 = mk(c[0], c[1], c[2]);
  t.v0 = v0;
  t.mat = make_mat(type, rgb, refl, transp);
  t.norm = normalized(cross(sub(v1, v0), sub(v2, v0)));
  const m33 basis = from_cols(sub(v2, v0), sub(v1, v0), neg(t.norm));
  t.ax = inverted(basis);
  t.v1 = v1;
  t.v2 = v2;
  {
    const float *a = &basis.m11, *b = &t.ax.m11;
    double na = 0.0, nb = 0.0;
    for (int k = 0; k < 9; ++k) { na += (double)a[k] * a[k]; nb += (double)b[k] * b[k]; }
    const float det = basis.m11 * (basis.m22 * basis.m33 - basis.m32 * basis.m23) +
                      basis.m21 * (basis.m32 * basis.m13 - basis.m12 * basis.m33) +
                      basis.m31 * (basis.m12 * basis.m23 - basis.m13 * basis.m22);
    t.cond = fabsf(det) > kVerySmall ? sqrt(na * nb) : INFINITY;
  }
  memset(&t.tuv, 0, sizeof(t.tuv));
  t.obj = (int)s->obj_kind.size();
  s->obj_kind.push_back(1);
  s->obj_idx.push_back((int)s->tris.size());
  s->tris.push_back(t);
  return t.obj;
}

extern "C" int rfx_scene_add_plane(rfx_scene *s, const float pos[3], const float norm[3], int type, const float rgb[3],
                                   float refl, float transp)                         // Plane.cpp:9-14
{
  if (!s || !pos || !norm || !rgb || (type != RFX_METAL && type != RFX_DIELECTRIC))
    return fail(RFX_ERR_ARG, "add_plane: bad args");
  HostPlane p;
  p.pos = mk(pos[0], pos[1], pos[2]);
  p.norm = mk(norm[0], norm[1], norm[2]);
  p.mat = make_mat(type, rgb, refl, transp);
  p.obj = (int)s->obj_kind.size();
  s->obj_kind.push_back(2);
  s->obj_idx.push_back((int)s->planes.size());
  s->planes.push_back(p);
  return p.obj;
}

extern "C" int rfx_triangle_set_texture(rfx_scene *s, int obj, int tex, const float uv[6])  // Triangle.cpp:110-120
{
  if (!s || !uv || obj < 0 || obj >= (int)s->obj_kind.size() || s->obj_kind[obj] != 1)
    return fail(RFX_ERR_ARG, "set_texture: object %d is not a triangle", obj);
  if (tex < 0 || tex >= (int)s->textures.size()) return fail(RFX_ERR_ARG, "set_texture: bad texture %d", tex);
  HostTri &t = s->tris[s->obj_idx[obj]];
  t.tex = tex;
  t.tu0 = uv[0];
  t.tv0 = uv[1];
  const v3 p1 = mk(uv[0], uv[1], 0), p2 = mk(uv[2], uv[3], 0), p3 = mk(uv[4], uv[5], 0);
  t.tuv = from_cols(sub(p3, p1), sub(p2, p1), mk(0, 0, -1));
  return RFX_OK;
}

extern "C" int rfx_scene_add_light(rfx_scene *s, const float o[3], float radius, const float rgb[3], float power)
{                                                                                     // Scene.cpp:48-59
  if (!s || !o || !rgb) return fail(RFX_ERR_ARG, "add_light: bad args");
  if (radius <= kVerySmall) radius = kVerySmall;
  const col c = mkc(rgb[0], rgb[1], rgb[2]);
  s->env = cadd(s->env, cscale(c, power));
  HostLight l;
  l.origin = mk(o[0], o[1], o[2]);
  l.radius = radius;
  l.r = c.r; l.g = c.g; l.b = c.b;
  l.power = clampf(power, 0.0f, 1.0f);                                                // OmniLight.cpp:13
  s->lights.push_back(l);
  return (int)s->lights.size() - 1;
}

extern "C" int rfx_scene_add_texture_argb(rfx_scene *s, uint32_t w, uint32_t h, const uint32_t *argb)
{
  if (!s) return fail(RFX_ERR_ARG, "add_texture: null scene");
  HostTexture t;
  if (argb && w && h)
  {
    t.w = w; t.h = h;
    t.loaded = true;
    t.texels.assign(argb, argb + (size_t)w * h);
  }
  s->textures.push_back(std::move(t));
  return (int)s->textures.size() - 1;
}

// ---- TGA / BMP (Texture.cpp:34-173, image_headers.h) ----
#pragma pack(push, 1)
struct TgaHeader { int8_t idlen, colmptype, imagetype; int16_t cmorg, cmlen; int8_t cmbits; int16_t xoff, yoff, xsize, ysize; int8_t bpix, imagedesc; };
struct BmpFileHeader { uint16_t bfType; uint32_t bfSize; uint16_t r1, r2; uint32_t bfOffBits; };
struct BmpInfoHeader { uint32_t biSize; int32_t biWidth, biHeight; uint16_t biPlanes, biBitCount; uint32_t biCompression, biSizeImage; int32_t xppm, yppm; uint32_t clrUsed, clrImportant; };
#pragma pack(pop)

// Texture::loadFromTGAFile (Texture.cpp:34-108): type 2, 24/32 bpp, rows in file order (origin bit ignored).
// As in the reference a header with a zero width or height loads successfully as an empty texture (w x h kept,
// no texels).  Negative (int16) sizes, which the reference cannot allocate, fail.
static bool tga_read(const char *path, uint32_t &w, uint32_t &h, std::vector<uint32_t> &out)
{
  w = h = 0;
  out.clear();
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  TgaHeader hd;
  bool ok = false;
  if (fread(&hd, sizeof(hd), 1, f) == 1 && hd.imagetype == 2 && hd.xsize >= 0 && hd.ysize >= 0)
  {
    const uint32_t W = (uint32_t)hd.xsize, H = (uint32_t)hd.ysize;
    const int bpp = hd.bpix;
    const long off = (long)sizeof(hd) + hd.idlen + hd.cmlen * hd.cmbits / 8;
    if (!fseek(f, off, SEEK_SET) && (bpp == 24 || bpp == 32))
    {
      const size_t n = (size_t)W * H, ps = (size_t)bpp / 8;
      std::vector<uint8_t> raw(n * ps);
      if (!n || fread(raw.data(), 1, raw.size(), f) == raw.size())
      {
        out.resize(n);
        for (size_t i = 0; i < n; ++i)
        {
          const uint8_t *p = &raw[i * ps];
          const uint32_t a = bpp == 32 ? p[3] : 0xFFu;
          out[i] = a << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0];
        }
        w = W; h = H;
        ok = true;
      }
    }
  }
  fclose(f);
  if (!ok) out.clear();
  return ok;
}

static bool has_ext(const char *path, const char *ext)
{
  const char *dot = strrchr(path, '.');
  return dot && !strcmp(dot, ext);
}

extern "C" int rfx_tga_load(const char *path, uint32_t *w, uint32_t *h, uint32_t *argb, size_t capacity)
{
  if (!path || !w || !h) return fail(RFX_ERR_ARG, "tga_load: bad args");
  std::vector<uint32_t> px;
  if (!tga_read(path, *w, *h, px)) return fail(RFX_ERR_IO, "tga_load: cannot read %s", path);
  if (argb)
  {
    if (capacity < px.size()) return fail(RFX_ERR_ARG, "tga_load: capacity %zu < %zu", capacity, px.size());
    memcpy(argb, px.data(), px.size() * 4);
  }
  return RFX_OK;
}

extern "C" int rfx_tga_save(const char *path, uint32_t w, uint32_t h, const uint32_t *argb)  // Texture.cpp:110-137
{
  if (!path || !argb || !w || !h) return fail(RFX_ERR_ARG, "tga_save: bad args");
  FILE *f = fopen(path, "wb");
  if (!f) return fail(RFX_ERR_IO, "tga_save: cannot open %s", path);
  TgaHeader hd;
  memset(&hd, 0, sizeof(hd));
  hd.imagetype = 2; hd.xsize = (int16_t)w; hd.ysize = (int16_t)h; hd.bpix = 32;
  bool ok = fwrite(&hd, sizeof(hd), 1, f) == 1 && fwrite(argb, (size_t)w * h * 4, 1, f) == 1;
  fclose(f);
  return ok ? RFX_OK : fail(RFX_ERR_IO, "tga_save: short write");
}

extern "C" int rfx_bmp_save(const char *path, uint32_t w, uint32_t h, const uint32_t *argb)  // Texture.cpp:139-173
{
  if (!path || !argb || !w || !h) return fail(RFX_ERR_ARG, "bmp_save: bad args");
  FILE *f = fopen(path, "wb");
  if (!f) return fail(RFX_ERR_IO, "bmp_save: cannot open %s", path);
  BmpFileHeader fh;
  BmpInfoHeader ih;
  memset(&fh, 0, sizeof(fh));
  memset(&ih, 0, sizeof(ih));
  fh.bfType = ((uint16_t)'M' << 8) | (uint16_t)'B';
  fh.bfSize = (uint32_t)(sizeof(fh) + sizeof(ih) + (size_t)w * h * 4);
  fh.bfOffBits = sizeof(fh) + sizeof(ih);
  ih.biSize = sizeof(ih); ih.biWidth = (int32_t)w; ih.biHeight = (int32_t)h; ih.biPlanes = 1; ih.biBitCount = 32;
  bool ok = fwrite(&fh, sizeof(fh), 1, f) == 1 && fwrite(&ih, sizeof(ih), 1, f) == 1 &&
            fwrite(argb, (size_t)w * h * 4, 1, f) == 1;
  fclose(f);
  return ok ? RFX_OK : fail(RFX_ERR_IO, "bmp_save: short write");
}

extern "C" int rfx_scene_add_texture_file(rfx_scene *s, const char *path, int *loaded)  // Scene.cpp:61-66
{
  if (!s || !path) return fail(RFX_ERR_ARG, "add_texture_file: bad args");
  HostTexture t;
  const bool ok = has_ext(path, ".tga") && tga_read(path, t.w, t.h, t.texels);     // Texture.cpp:175-189
  t.loaded = ok;
  if (loaded) *loaded = ok ? 1 : 0;
  s->textures.push_back(std::move(t));
  return (int)s->textures.size() - 1;
}

static void set_skybox_index(rfx_scene *s, int idx)                                   // Skybox.cpp:21-37
{
  s->skybox = idx;
  const HostTexture &t = s->textures[idx];
  if (t.loaded)
  {
    s->half_tile_w = 1.0f / 8.0f - 1.0f / (float)t.w - kFltEpsilon;
    s->half_tile_h = 1.0f / 6.0f - 1.0f / (float)t.h - kFltEpsilon;
  }
  else
    default_half_tiles(s);
}

extern "C" int rfx_scene_set_skybox_file(rfx_scene *s, const char *path)
{
  if (!s || !path) return fail(RFX_ERR_ARG, "set_skybox_file: bad args");
  int loaded = 0;
  const int idx = rfx_scene_add_texture_file(s, path, &loaded);
  set_skybox_index(s, idx);
  return loaded;
}

extern "C" int rfx_scene_set_skybox_argb(rfx_scene *s, uint32_t w, uint32_t h, const uint32_t *argb)
{
  if (!s) return fail(RFX_ERR_ARG, "set_skybox_argb: null scene");
  const int idx = rfx_scene_add_texture_argb(s, w, h, argb);
  set_skybox_index(s, idx);
  return s->textures[idx].loaded ? 1 : 0;
}

extern "C" int rfx_scene_plane_count(const rfx_scene *s)
{
  if (!s) return fail(RFX_ERR_ARG, "plane_count: null scene");
  return (int)s->planes.size();
}

extern "C" int rfx_scene_counts(const rfx_scene *s, int *ns, int *nt, int *nl, int *nx)
{
  if (!s) return fail(RFX_ERR_ARG, "counts: null scene");
  if (ns) *ns = (int)s->spheres.size();
  if (nt) *nt = (int)s->tris.size();
  if (nl) *nl = (int)s->lights.size();
  if (nx) *nx = (int)s->textures.size();
  return RFX_OK;
}

// ============================================================== camera / images
extern "C" void rfx_camera_view(const float e[3], const float a[3], float view[9])    // Camera.cpp:24-38
{
  const v3 eye = mk(e[0], e[1], e[2]), at = mk(a[0], a[1], a[2]);
  const v3 up = mk(0.0f, 1.0f, 0.0f);
  const v3 oz = normalized(sub(at, eye));
  const v3 ox = normalized(cross(up, oz));
  const v3 oy = normalized(cross(oz, ox));
  const m33 m = from_cols(ox, oy, oz);
  memcpy(view, &m, sizeof(m));
}

extern "C" float rfx_camera_rz(uint32_t width, float fov)                             // Render.cpp:148
{
  return (float)width / 2.0f / tanf(fov / 2.0f);
}

extern "C" void rfx_argb_from_rgb(const float *rgb, size_t n, uint32_t *out)
{
  for (size_t i = 0; i < n; ++i) out[i] = argb(mkc(rgb[i * 3], rgb[i * 3 + 1], rgb[i * 3 + 2]));
}

extern "C" uint32_t rfx_strip_rows(uint32_t H, uint32_t rb, uint32_t rank, uint32_t nranks)
{
  if (nranks <= 1) return H;
  if (!rb || rank >= nranks) return 0;
  const uint32_t full = H / rb, rem = H % rb;
  uint32_t rows = (full / nranks) * rb;
  const uint32_t extra = full % nranks;
  if (rank < extra) rows += rb;
  if (rem && full % nranks == rank) rows += rem;
  return rows;
}

extern "C" uint32_t rfx_strip_row_to_y(uint32_t r, uint32_t rb, uint32_t rank, uint32_t nranks)
{
  if (nranks <= 1) return r;
  return (r / rb * nranks + rank) * rb + r % rb;
}

// ============================================================== renderer
#ifndef RFX_TILE_ORDER_DEFAULT
#define RFX_TILE_ORDER_DEFAULT 1
#endif
#ifndef RFX_TILE_ORDER_MIN_TILES
// 8x8 wave tiles: C3 (3840x2160) has 129,600, C2 (1920x1080) 32,400, a C4 rank's strips at N = 8 65,280 (their
// trace 0.41 ms unsorted vs 0.34 at N = 4 per eighth of the frame, tools/root_overhead.py)
#define RFX_TILE_ORDER_MIN_TILES 49152
#endif
constexpr size_t kPrimWords = 5;        // per wave tile, small scenes (rfx_trace.h kPrimStride)
constexpr size_t kPrimLargeWords = 12;  // per wave tile, large scenes (rfx_trace.h kPrimLargeStride)
// per-view masks of SSAA frames / chunk lists of large scenes: measured slower, compiled out (rfx_trace.h)
#ifndef RFX_PRIM_SSAA
#define RFX_PRIM_SSAA 0
#endif
#ifndef RFX_PRIM_LANES
#define RFX_PRIM_LANES 1  // masks of kModeSsaaLanes frames (the lanes' own small pixel blocks)
#endif
#ifndef RFX_PRIM_CHUNKS
#define RFX_PRIM_CHUNKS 1  // closest-hit masks of kModeSsaaChunks frames (a pixel's sample rectangle), every launch
#endif
#ifndef RFX_PRIM_LARGE
#define RFX_PRIM_LARGE 0
#endif
#ifndef RFX_ONE_LIGHT
#define RFX_ONE_LIGHT 1  // one-light kernel instantiations (rfx_trace.h kCfgOneLight; -DRFX_ONE_LIGHT=0 turns them off)
#endif
#ifndef RFX_BOUNCE_GROUPS_PER_CU
#define RFX_BOUNCE_GROUPS_PER_CU 14
#endif

#ifndef RFX_QUEUE_SORT
// regrouped frames: the bounce kernel takes the parked traces bucket by bucket (1) or in park order (0).  tools/ab.py,
// C5 trace + bounce: park after 3 sorted 3.48 vs 3.40 ms unsorted (+2.3%); after 2: 3.53 vs 3.69 (-4.2%, still
// above park-3 unsorted).  Park order keeps a tile's survivors together, which a coarse cell key cannot beat.
#define RFX_QUEUE_SORT 0
#endif
#ifndef RFX_PARK_AFTER
#define RFX_PARK_AFTER 2  // large-scene plain frames: segments before a live trace is parked for the bounce kernel
#endif
// The tile sort: on the trace launch's own stream (RFX_TILE_SORT_MAIN=0: on a side stream beside the next frame's RNG
// pre-pass, joined by an event pair) every RFX_TILE_SORT_EVERY-th launch.  Trace time against raster order (tools/ab.py,
// C3): every launch -7.5%, every 4th -9.4%, every 16th -9.8%.  The side stream hid the sort but not its events: a kernel
// trace shows ~20 us between two traces on a sorting frame beyond a plain one (fork before the count, join before the
// trace).  Frame ms, interleaved A/B (profiles/r06/ab/*_tile_sort_r6q.jsonl): C3 every 4th beside 0.6556, on the stream
// 0.6526, every 16th beside 0.6513, every 16th on the stream 0.6485 (-1.1%); C2 d4 -0.9%, the 4x4 screenshot -0.4%.
#ifndef RFX_TILE_SORT_MAIN
#define RFX_TILE_SORT_MAIN 1
#endif
#ifndef RFX_TILE_SORT_EVERY
#define RFX_TILE_SORT_EVERY 16
#endif
#ifndef RFX_LAUNCH_TRACES
#define RFX_LAUNCH_TRACES (1ull << 30)  // traces per launch of a split frame (rfx_renderer_set_launch_traces)
#endif
#ifndef RFX_SPLIT_STREAMS
#define RFX_SPLIT_STREAMS 2  // split frames: spans alternate between two streams (1: one stream, no overlap)
#endif
constexpr uint64_t kMaxLaunchTraces = 1ull << 31;  // the band scan's 32-bit offsets (rfx_kernels.hip rng_band_range)
#ifndef RFX_SCAN_EMIT_BLOCKS
// one-device emits of more RNG blocks than this scan the counts first (rng_band_range) instead of summing them per
// block (rng_emit: O(nblk^2) reads); C3 has 4,066 blocks, the 4x4 screenshot frame 16,219.  Re-checked with the
// multi-workgroup tile scan (round 6, profiles/r06/ab/*_scan_emit_threshold_r6x.jsonl): a threshold of 4,096 makes the C4
// and screenshot pre-passes 0.093 -> 0.104 ms, so the per-block sums stay up to 16,384 blocks
#define RFX_SCAN_EMIT_BLOCKS 16384
#endif
struct rfx_renderer {
  int device = 0;
  int cus = 256;  // compute units of the device (the bounce kernel's grid: one resident wave per slot)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // scene on device
  DevScene dev{};
  std::vector<void *> scene_allocs;
  bool has_scene = false;
  // RNG state: d_seed[seed_idx] current; the pre-pass writes the next frame's state to the other word and
  // the host flips seed_idx (no device copy between frames); d_err
  uint32_t *d_seed = nullptr;
  uint32_t seed_idx = 0;
  int *d_err = nullptr;
  uint32_t jitter_seed = 0;
  // workspaces
  uint32_t *d_rd = nullptr; uint64_t rd_cap = 0;  // per-trace LCG states (rng_emit)
  uint32_t *d_rd_alt = nullptr; uint64_t rd_alt_cap = 0;  // emit-ahead: the second randDir buffer
  int emit_pending = -1;  // emit-ahead: buffer (0 d_rd, 1 d_rd_alt) of an emitted, untraced frame, or -1
  int trace_buf = 0;      // buffer the last enqueued trace read
  bool split_alt_busy = false;  // a split frame's odd spans traced from d_rd_alt on split_stream (done at split_ev[2])
  uint64_t emit_key[10] = {};  // the emitted frame's plan (traces, band, geometry): rfx_render_frame_emitted must match it
  // rfx_frame_rng_rewind: the last call was an rfx_render_frame; its start states (the sphere stream's is the other
  // seed word while rewind_flip, or the saved word d_seed[2] while rewind_saved: a frame of several launches) can be
  // restored
  bool rewind_ok = false, rewind_flip = false, rewind_saved = false;
  uint32_t rewind_jitter = 0;
  hipStream_t rewind_stream = nullptr;
  // frames of more traces than launch_traces: consecutive spans alternate between the caller's stream and split_stream
  // (randDirs in d_rd / d_rd_alt); split_ev[k] marks span k's emit (the next span's pre-pass starts from its state)
  uint64_t launch_traces = RFX_LAUNCH_TRACES;
  // bumped whenever the random streams move or are set (emits, set_rng, rewinds): a device group compares it with the
  // value after its own last frame to know whether the members' streams still equal member 0's
  uint64_t state_seq = 0;
  hipStream_t split_stream = nullptr;
  hipEvent_t split_ev[3] = {nullptr, nullptr, nullptr};
  uint32_t *d_blk_cnt = nullptr; uint64_t blk_cap = 0;
  uint64_t *d_blk_off = nullptr;     // band emits: the scanned block offsets ...
  uint32_t *d_rng_range = nullptr;   // ... and the band's first / last / final block
  uint32_t *d_tile_sum = nullptr;    // ... and the multi-workgroup scan's tile totals (one per 4096 blocks)
  // the one-pass pre-pass (rng_fused): per-block status words (blk_cap), the block ticket word (counts up across
  // launches, never reset), the tickets taken so far, the launch's epoch tag
  unsigned long long *d_rng_status = nullptr, *d_rng_ticket = nullptr;
  unsigned long long rng_tickets = 0;
  uint32_t rng_epoch = 0;
  uint16_t *d_rng_masks = nullptr;  // one device's accept flags per pre-pass thread (rng_count -> rng_emit)
  uint32_t *d_jump = nullptr;  // LCG jump table for blk_cap blocks (rng_jump_table)
  // host staging for rfx_render_frame_host
  float *d_img = nullptr; uint32_t *d_argb = nullptr; uint64_t *d_cnt = nullptr; size_t img_cap = 0;
  // tile schedule (rfx_renderer_set_tile_order): a recording trace launch writes per-tile clock costs; a counting
  // sort (lpt_*) turns them into the next launch's order (longest first), on the launch's stream (or, RFX_TILE_SORT_MAIN
  // = 0, on tile_stream while the next frame's RNG pre-pass runs); a launch on another stream waits on tile_join.
  // tile_n: tiles of the launch the order is for.
  int tile_mode = RFX_TILE_ORDER_DEFAULT;
  uint32_t *d_tile_cost = nullptr, *d_tile_order = nullptr, *d_tile_scratch = nullptr;
  uint32_t tile_cap = 0, tile_n = 0;
  uint64_t tile_key = 0;
  hipStream_t tile_stream = nullptr;
  hipEvent_t tile_fork = nullptr, tile_join = nullptr;
  bool tile_pending = false;         // a sort has been launched: its order is valid for (tile_n, tile_key)
  hipStream_t tile_waited = nullptr; // the stream that already waits on the last sort (tile_join)
  uint64_t tile_count = 0;           // scheduled launches (costs are recorded every RFX_TILE_SORT_EVERY-th)
  // ray regrouping of large-scene plain frames (RFX_PARK_AFTER): parked traces, their count and the bounce
  // kernel's claim counter (d_qctr[0], d_qctr[1])
  int park_after = -1;  // rfx_renderer_set_regroup: -1 = default (RFX_PARK_AFTER on large scenes), 0 = off
  // primary-bundle cull masks (small scenes, plain frames): one u64 per wave tile, valid for prim_key
  uint64_t *d_prim_mask = nullptr;
  size_t prim_cap = 0;
  // split frames in the chunk mode: each span's pixel masks, in the buffer of its stream side (render_split)
  uint64_t *d_split_mask[2] = {nullptr, nullptr};
  size_t split_mask_cap[2] = {0, 0};
  std::vector<uint8_t> prim_key;   // the view the masks hold (empty: none)
  std::vector<uint8_t> prim_seen;  // the view of the last plain small-scene launch
  uint64_t scene_gen = 0;  // bumped by every set_scene
  int prim_mode = 1;       // rfx_renderer_set_prim_masks
  int bounce_form = 0;     // the last trace launch's bounce kernel: 0 none, 1 global-memory BVH, 2 LDS-staged BVH
  QRay *d_queue = nullptr;
  uint64_t queue_cap = 0;
  uint32_t *d_qctr = nullptr;   // count, claim counter, then the sort's kQueueBuckets histogram words
  uint32_t *d_qkey = nullptr, *d_qorder = nullptr;  // regroup sort: per entry its bucket; entries in bucket order
  int queue_sort = RFX_QUEUE_SORT;  // rfx_renderer_set_regroup_sort
  // per-phase event timing: triples {start, after pre-pass, after trace} on every timing_every-th frame (the events'
  // own cost stays off the other frames: ~10 us per frame for three records at C1's 640x480)
  bool timing = false, timing_this = false;
  uint32_t timing_every = 1;
  uint64_t timing_seq = 0;
  std::vector<hipEvent_t> events;
  size_t events_used = 0;
};

static uint32_t *seed_cur(rfx_renderer *r) { return r->d_seed + r->seed_idx; }
static uint32_t *seed_next(rfx_renderer *r) { return r->d_seed + (r->seed_idx ^ 1u); }

static int timing_event(rfx_renderer *r, hipStream_t st)
{
  if (!r->timing_this) return RFX_OK;
  if (r->events_used == r->events.size())
  {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    r->events.push_back(e);
  }
  HIP_CHECK(hipEventRecord(r->events[r->events_used++], st));
  return RFX_OK;
}

// the first event of a frame: decides whether this frame is one of the timed ones
static int timing_start(rfx_renderer *r, hipStream_t st)
{
  r->timing_this = r->timing && r->timing_seq++ % r->timing_every == 0;
  return timing_event(r, st);
}

extern "C" int rfx_renderer_set_timing(rfx_renderer *r, int enable)
{
  if (!r || enable < 0) return fail(RFX_ERR_ARG, "set_timing: null renderer or negative period");
  r->timing = enable != 0;
  r->timing_every = enable > 1 ? (uint32_t)enable : 1u;
  r->timing_seq = 0;
  r->timing_this = false;
  r->events_used = 0;
  return RFX_OK;
}

extern "C" int rfx_renderer_get_timing(rfx_renderer *r, double *prepass_ms, double *trace_ms, uint64_t *frames)
{
  if (!r) return fail(RFX_ERR_ARG, "get_timing: null renderer");
  double pre = 0.0, tr = 0.0;
  const size_t n = r->events_used / 3;
  if (n) HIP_CHECK(hipEventSynchronize(r->events[3 * n - 1]));
  for (size_t i = 0; i < n; ++i)
  {
    float a = 0.0f, b = 0.0f;
    HIP_CHECK(hipEventElapsedTime(&a, r->events[3 * i], r->events[3 * i + 1]));
    HIP_CHECK(hipEventElapsedTime(&b, r->events[3 * i + 1], r->events[3 * i + 2]));
    pre += a;
    tr += b;
  }
  r->events_used = 0;
  if (prepass_ms) *prepass_ms = pre;
  if (trace_ms) *trace_ms = tr;
  if (frames) *frames = n;
  return RFX_OK;
}

static int set_dev(rfx_renderer *r)
{
  HIP_CHECK(hipSetDevice(r->device));
  return RFX_OK;
}

extern "C" int rfx_renderer_create(rfx_renderer **out, int device)
{
  if (!out) return fail(RFX_ERR_ARG, "renderer_create: null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RFX_ERR_NODEV, "no HIP device");
  if (device < 0 || device >= n) return fail(RFX_ERR_ARG, "device %d out of range (%d devices)", device, n);
  rfx_renderer *r = new rfx_renderer();
  r->device = device;
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) { delete r; return rc; }
  if (hipStreamCreateWithFlags(&r->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&r->d_seed, 3 * sizeof(uint32_t)) != hipSuccess || hipMalloc(&r->d_err, sizeof(int)) != hipSuccess)
  {
    delete r;
    return fail(RFX_ERR_HIP, "renderer_create: HIP allocation failed");
  }
  r->stream = r->own_stream;
  if (hipDeviceGetAttribute(&r->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || r->cus <= 0)
    r->cus = 256;
  const uint32_t seeds[2] = {1350490027u, 1350490027u};
  if (hipMemcpy(r->d_seed, seeds, sizeof(seeds), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(r->d_err, 0, sizeof(int)) != hipSuccess)
  {
    delete r;
    return fail(RFX_ERR_HIP, "renderer_create: HIP init copy failed");
  }
  *out = r;
  return RFX_OK;
}

static void free_scene(rfx_renderer *r)
{
  for (void *p : r->scene_allocs) (void)hipFree(p);
  r->scene_allocs.clear();
  r->has_scene = false;
}

extern "C" void rfx_renderer_destroy(rfx_renderer *r)
{
  if (!r) return;
  (void)hipSetDevice(r->device);
  (void)hipStreamSynchronize(r->stream);
  free_scene(r);
  (void)hipFree(r->d_seed); (void)hipFree(r->d_err); (void)hipFree(r->d_rd); (void)hipFree(r->d_rd_alt);
  (void)hipFree(r->d_blk_cnt); (void)hipFree(r->d_jump); (void)hipFree(r->d_rng_masks); (void)hipFree(r->d_blk_off);
  (void)hipFree(r->d_tile_sum);
  (void)hipFree(r->d_rng_range);
  (void)hipFree(r->d_rng_status); (void)hipFree(r->d_rng_ticket);
  (void)hipFree(r->d_img); (void)hipFree(r->d_argb); (void)hipFree(r->d_cnt);
  (void)hipFree(r->d_queue); (void)hipFree(r->d_qctr); (void)hipFree(r->d_prim_mask);
  (void)hipFree(r->d_split_mask[0]); (void)hipFree(r->d_split_mask[1]);
  (void)hipFree(r->d_qkey); (void)hipFree(r->d_qorder);
  for (hipEvent_t e : r->events) (void)hipEventDestroy(e);
  if (r->tile_stream) (void)hipStreamSynchronize(r->tile_stream);
  (void)hipFree(r->d_tile_cost); (void)hipFree(r->d_tile_order); (void)hipFree(r->d_tile_scratch);
  if (r->tile_fork) (void)hipEventDestroy(r->tile_fork);
  if (r->tile_join) (void)hipEventDestroy(r->tile_join);
  if (r->tile_stream) (void)hipStreamDestroy(r->tile_stream);
  if (r->split_stream)
  {
    (void)hipStreamSynchronize(r->split_stream);
    (void)hipStreamDestroy(r->split_stream);
  }
  for (hipEvent_t e : r->split_ev)
    if (e) (void)hipEventDestroy(e);
  if (r->own_stream) (void)hipStreamDestroy(r->own_stream);
  delete r;
}

extern "C" int rfx_build_options(void)
{
  return (RFX_PRIM_LARGE ? RFX_BUILD_PRIM_LARGE : 0) | (RFX_PRIM_SSAA ? RFX_BUILD_PRIM_SSAA : 0) |
         (RFX_PRIM_LANES ? RFX_BUILD_PRIM_LANES : 0) | (RFX_ONE_LIGHT ? RFX_BUILD_ONE_LIGHT : 0) |
         (RFX_BVH_LEAF_PAIRS << 8);
}

extern "C" int rfx_renderer_set_launch_traces(rfx_renderer *r, uint64_t max_traces)
{
  if (!r) return fail(RFX_ERR_ARG, "renderer_set_launch_traces: null renderer");
  r->launch_traces = max_traces ? std::min(max_traces, kMaxLaunchTraces) : (uint64_t)RFX_LAUNCH_TRACES;
  return RFX_OK;
}

extern "C" int rfx_renderer_device(const rfx_renderer *r) { return r ? r->device : -1; }

extern "C" int rfx_renderer_set_tile_order(rfx_renderer *r, int mode)
{
  if (!r || mode < 0 || mode > 3) return fail(RFX_ERR_ARG, "renderer_set_tile_order: mode 0, 1, 2 or 3");
  r->tile_mode = mode;
  return RFX_OK;
}

extern "C" int rfx_renderer_set_prim_masks(rfx_renderer *r, int mode)
{
  if (!r || mode < 0 || mode > 2) return fail(RFX_ERR_ARG, "renderer_set_prim_masks: mode 0, 1 or 2");
  r->prim_mode = mode;
  r->prim_key.clear();
  r->prim_seen.clear();
  return RFX_OK;
}

extern "C" int rfx_renderer_bounce_form(const rfx_renderer *r)
{
  if (!r) return fail(RFX_ERR_ARG, "renderer_bounce_form: null renderer");
  return r->bounce_form;
}

extern "C" int rfx_renderer_set_regroup(rfx_renderer *r, int park_after)
{
  if (!r || park_after < -1) return fail(RFX_ERR_ARG, "renderer_set_regroup: -1 (default), 0 (off) or segments >= 1");
  r->park_after = park_after;
  return RFX_OK;
}

extern "C" int rfx_renderer_set_regroup_sort(rfx_renderer *r, int on)
{
  if (!r || on < 0 || on > 1) return fail(RFX_ERR_ARG, "renderer_set_regroup_sort: 0 or 1");
  r->queue_sort = on;
  return RFX_OK;
}

extern "C" int rfx_renderer_set_stream(rfx_renderer *r, void *s)
{
  if (!r) return fail(RFX_ERR_ARG, "set_stream: null renderer");
  r->stream = s ? (hipStream_t)s : r->own_stream;
  return RFX_OK;
}

template <class T>
static int upload(rfx_renderer *r, const std::vector<T> &v, const T **dst)
{
  if (v.empty()) { *dst = nullptr; return RFX_OK; }
  void *p = nullptr;
  HIP_CHECK(hipMalloc(&p, v.size() * sizeof(T)));
  r->scene_allocs.push_back(p);
  HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *dst = (const T *)p;
  return RFX_OK;
}

// Device order of a large scene's spheres: recursive median splits of the centres along their longest axis,
// left parts of even size, so pairs (2j, 2j + 1) are neighbours and every aligned run of 2^k spheres is a
// compact cluster (the 64-sphere chunks of the bundle cull, the leaves of the pair BVH).
static void spatial_order(std::vector<uint32_t> &idx, size_t a, size_t b, const std::vector<HostSphere> &sp)
{
  if (b - a <= 2) return;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (size_t i = a; i < b; ++i)
  {
    const double c[3] = {sp[idx[i]].center.x, sp[idx[i]].center.y, sp[idx[i]].center.z};
    for (int k = 0; k < 3; ++k) { lo[k] = fmin(lo[k], c[k]); hi[k] = fmax(hi[k], c[k]); }
  }
  int axis = 0;
  for (int k = 1; k < 3; ++k)
    if (hi[k] - lo[k] > hi[axis] - lo[axis]) axis = k;
  const size_t mid = a + 2 * ((b - a + 2) / 4);
  auto key = [&](uint32_t i) { return axis == 0 ? sp[i].center.x : axis == 1 ? sp[i].center.y : sp[i].center.z; };
  std::nth_element(idx.begin() + a, idx.begin() + mid, idx.begin() + b,
                   [&](uint32_t x, uint32_t y) { return key(x) < key(y) || (key(x) == key(y) && x < y); });
  spatial_order(idx, a, mid, sp);
  spatial_order(idx, mid, b, sp);
}

// Pair BVH of a large scene: leaves are the device sphere pairs (2j, 2j + 1, neighbours); internal nodes
// split their pairs where the surface-area heuristic is lowest (every position of the pair centres sorted
// along each axis), as long as the split keeps the tree within the kernel's stack depth, else at the
// median of the pair centres along the longest axis (SAH against median splits alone: C5 -0.8%, round 2).  Each
// node stores its two
// children's boxes (spheres grown by their radii); the kernel widens them by its exact-cull margin per ray.
// Returns the node index (or ~pair for a leaf) of range [a, b) of `pairs`; depth: internal levels below.
#ifndef RFX_BVH_STACK
#define RFX_BVH_STACK 16  // the kernel's per-lane traversal stack (rfx_trace.h kBvhStack)
#endif
namespace {
struct PairBox { double lo[3], hi[3], c[3]; };

int build_pair_bvh(std::vector<BvhNode> &nodes, std::vector<uint32_t> &pairs, size_t a, size_t b,
                   const std::vector<PairBox> &box, const double *ref, int level, int &depth)
{
  if (b - a == 1) return ~(int)pairs[a];
  depth = std::max(depth, level + 1);
  const int id = (int)nodes.size();
  nodes.push_back(BvhNode{});
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (size_t i = a; i < b; ++i)
    for (int k = 0; k < 3; ++k) { lo[k] = fmin(lo[k], box[pairs[i]].c[k]); hi[k] = fmax(hi[k], box[pairs[i]].c[k]); }
  int axis = 0;
  for (int k = 1; k < 3; ++k)
    if (hi[k] - lo[k] > hi[axis] - lo[axis]) axis = k;
  size_t mid = a + (b - a) / 2;
  // surface-area heuristic over sorted pair centres (all three axes, every split position), while the depth
  // budget allows an unbalanced split: the subtree of n leaves must still fit RFX_BVH_STACK levels
  const size_t cnt = b - a;
  int need = 0;
  while (((size_t)1 << need) < cnt) ++need;
  if (level + need + 2 <= RFX_BVH_STACK && cnt > 2)
  {
    double best = INFINITY;
    int best_axis = axis;
    size_t best_mid = mid;
    std::vector<uint32_t> tmp(pairs.begin() + a, pairs.begin() + b);
    std::vector<double> right(cnt + 1);
    auto area = [](const double *l, const double *h) {
      const double dx = h[0] - l[0], dy = h[1] - l[1], dz = h[2] - l[2];
      return dx * dy + dy * dz + dz * dx;
    };
    for (int ax = 0; ax < 3; ++ax)
    {
      std::sort(tmp.begin(), tmp.end(), [&](uint32_t x, uint32_t y) {
        return box[x].c[ax] < box[y].c[ax] || (box[x].c[ax] == box[y].c[ax] && x < y);
      });
      double l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (size_t i = cnt; i-- > 0;)
      {
        for (int k = 0; k < 3; ++k) { l[k] = fmin(l[k], box[tmp[i]].lo[k]); h[k] = fmax(h[k], box[tmp[i]].hi[k]); }
        right[i] = area(l, h) * (double)(cnt - i);
      }
      for (int k = 0; k < 3; ++k) { l[k] = INFINITY; h[k] = -INFINITY; }
      // a split leaving at most 2^(budget - 1) leaves on each side keeps the depth bound
      const size_t cap = (size_t)1 << std::min(30, RFX_BVH_STACK - level - 2);
      for (size_t i = 1; i < cnt; ++i)
      {
        for (int k = 0; k < 3; ++k) { l[k] = fmin(l[k], box[tmp[i - 1]].lo[k]); h[k] = fmax(h[k], box[tmp[i - 1]].hi[k]); }
        if (i > cap || cnt - i > cap) continue;
        const double cost = area(l, h) * (double)i + right[i];
        if (cost < best) { best = cost; best_axis = ax; best_mid = a + i; }
      }
    }
    axis = best_axis;
    mid = best_mid;
  }
  std::nth_element(pairs.begin() + a, pairs.begin() + mid, pairs.begin() + b, [&](uint32_t x, uint32_t y) {
    return box[x].c[axis] < box[y].c[axis] || (box[x].c[axis] == box[y].c[axis] && x < y);
  });
  const int kids[2] = {build_pair_bvh(nodes, pairs, a, mid, box, ref, level + 1, depth),
                       build_pair_bvh(nodes, pairs, mid, b, box, ref, level + 1, depth)};
  const size_t range[2][2] = {{a, mid}, {mid, b}};
  BvhNode &n = nodes[id];
  for (int c = 0; c < 2; ++c)
  {
    double l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = range[c][0]; i < range[c][1]; ++i)
      for (int k = 0; k < 3; ++k) { l[k] = fmin(l[k], box[pairs[i]].lo[k]); h[k] = fmax(h[k], box[pairs[i]].hi[k]); }
#if RFX_BVH_PREWIDE
    {
      // the box grown by the node part of the kernel's margin, kCullRel mt[c] (rfx_trace.h kCullRel = 2e-3), from the
      // float mt the kernel would have used, with a relative 1e-6 on top
      double cd = 0.0, hd = 0.0;
      for (int k = 0; k < 3; ++k)
      {
        const double dc = ref[k] - 0.5 * (l[k] + h[k]), dh = 0.5 * (h[k] - l[k]);
        cd += dc * dc;
        hd += dh * dh;
      }
      const double w = 2e-3 * (double)nextafterf((float)((sqrt(cd) + sqrt(hd)) * 1.0001), INFINITY) * (1.0 + 1e-6);
      for (int k = 0; k < 3; ++k) { l[k] -= w; h[k] += w; }
    }
#endif
    // round outwards to float
    n.lx[c] = nextafterf((float)l[0], -INFINITY); n.ly[c] = nextafterf((float)l[1], -INFINITY);
    n.lz[c] = nextafterf((float)l[2], -INFINITY);
    n.hx[c] = nextafterf((float)h[0], INFINITY); n.hy[c] = nextafterf((float)h[1], INFINITY);
    n.hz[c] = nextafterf((float)h[2], INFINITY);
    n.child[c] = kids[c];
    // margin term of the child against the reference point ref (the root box centre), rounded up
    double mt = 0.0;
    {
      // Euclidean: |ref - centre|_2 + the half-diagonal (round 3; the L1 form made C5 2.2% slower)
      double cd = 0.0, hd = 0.0;
      for (int k = 0; k < 3; ++k)
      {
        const double dc = ref[k] - 0.5 * (l[k] + h[k]), dh = 0.5 * (h[k] - l[k]);
        cd += dc * dc;
        hd += dh * dh;
      }
      mt = sqrt(cd) + sqrt(hd);
    }
    n.mt[c] = nextafterf((float)(mt * 1.0001), INFINITY);
  }
  return id;
}
}  // namespace

#ifndef RFX_BVH_STACK
#define RFX_BVH_STACK 16  // the kernel's per-lane traversal stack (rfx_trace.h kBvhStack)
#endif

extern "C" int rfx_renderer_set_scene(rfx_renderer *r, const rfx_scene *s)
{
  if (!r || !s) return fail(RFX_ERR_ARG, "set_scene: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  HIP_CHECK(hipStreamSynchronize(r->stream));
  free_scene(r);
  std::vector<SphereGeo> sg;
  std::vector<MatRec> sm, tm;
  std::vector<int32_t> si;
  // Large scenes (more than 32 spheres): spheres in spatial order (spatial_order: recursive median splits),
  // so each 64-sphere chunk of the device arrays is compact and its bounding sphere can cull it as a whole,
  // and each pair is a BVH leaf.  Every record keeps its object index (sph_info),
  // and the large-scene kernel path compares (distance, object index), so the order changes no result.
  const size_t nsph = s->spheres.size();
  std::vector<uint32_t> order(nsph);
  for (size_t i = 0; i < nsph; ++i) order[i] = (uint32_t)i;
  if (nsph > 32) spatial_order(order, 0, nsph, s->spheres);

  for (uint32_t oi : order)
  {
    const HostSphere &sp = s->spheres[oi];
    sg.push_back({sp.center.x, sp.center.y, sp.center.z, sp.sq_radius});
    sm.push_back({sp.mat.r, sp.mat.g, sp.mat.b, sp.mat.refl});
    si.push_back(sp.obj);
    si.push_back(sp.mat.dielectric);
  }
  // (large scenes: a whole number of BVH leaves of RFX_BVH_LEAF_PAIRS pairs; the padding pairs never hit)
  const size_t npair_dev = sg.size() > 32 ? ((sg.size() + 1) / 2 + RFX_BVH_LEAF_PAIRS - 1) / RFX_BVH_LEAF_PAIRS *
                                                RFX_BVH_LEAF_PAIRS
                                          : (sg.size() + 1) / 2;
  std::vector<SpherePair> sp(npair_dev);
  for (size_t i = 0; i < 2 * sp.size(); ++i)
  {
    SpherePair &p = sp[i / 2];
    const int l = (int)(i & 1);
    const bool real = i < sg.size();
    p.cx[l] = real ? sg[i].cx : 0.0f;
    p.cy[l] = real ? sg[i].cy : 0.0f;
    p.cz[l] = real ? sg[i].cz : 0.0f;
    p.r2[l] = real ? sg[i].sq_radius : -INFINITY;
  }
  std::vector<TriGeo> tg;
  std::vector<TriShade> ts;
  for (const HostTri &t : s->tris)
  {
    TriGeo g{};
    g.v0x = t.v0.x; g.v0y = t.v0.y; g.v0z = t.v0.z;
    g.a11 = t.ax.m11; g.a12 = t.ax.m12; g.a13 = t.ax.m13;
    g.a21 = t.ax.m21; g.a22 = t.ax.m22; g.a23 = t.ax.m23;
    g.a31 = t.ax.m31; g.a32 = t.ax.m32; g.a33 = t.ax.m33;
    tg.push_back(g);
    TriShade h{};
    h.nx = t.norm.x; h.ny = t.norm.y; h.nz = t.norm.z;
    h.tu0 = t.tu0; h.tv0 = t.tv0;
    h.t11 = t.tuv.m11; h.t12 = t.tuv.m12; h.t21 = t.tuv.m21; h.t22 = t.tuv.m22;
    h.tex = t.tex; h.dielectric = t.mat.dielectric; h.obj = t.obj;
    ts.push_back(h);
    tm.push_back({t.mat.r, t.mat.g, t.mat.b, t.mat.refl});
  }
  // bounding spheres for the wave-bundle cull: a sphere's own (radius grown by a relative 1e-5), a
  // triangle's centroid and farthest vertex; a triangle whose axTrans is ill-conditioned (the reference
  // falls back to the identity for a singular basis, Matrix33.cpp:58-79) may report hits far from its
  // vertices, so it gets r = +inf and is never culled
  std::vector<Bound> bd;
  for (uint32_t oi : order)
  {
    const HostSphere &sp = s->spheres[oi];
    bd.push_back({sp.center.x, sp.center.y, sp.center.z, sp.radius * 1.00001f});
  }
  // chunk bounds: 64 consecutive spheres of the device order, centred on their mean centre
  std::vector<Bound> cb;
  for (size_t first = 0; first < nsph; first += 64)
  {
    const size_t last = std::min(nsph, first + 64);
    double m[3] = {0.0, 0.0, 0.0};
    for (size_t i = first; i < last; ++i) { m[0] += bd[i].x; m[1] += bd[i].y; m[2] += bd[i].z; }
    for (double &v : m) v /= (double)(last - first);
    double r = 0.0;
    for (size_t i = first; i < last; ++i)
    {
      const double dx = bd[i].x - m[0], dy = bd[i].y - m[1], dz = bd[i].z - m[2];
      r = fmax(r, sqrt(dx * dx + dy * dy + dz * dz) + (double)bd[i].r);
    }
    cb.push_back({(float)m[0], (float)m[1], (float)m[2], (float)(r * 1.0001 + 1e-6)});
  }
  for (const HostTri &t : s->tris)
  {
    const double cx = ((double)t.v0.x + t.v1.x + t.v2.x) / 3.0, cy = ((double)t.v0.y + t.v1.y + t.v2.y) / 3.0,
                 cz = ((double)t.v0.z + t.v1.z + t.v2.z) / 3.0;
    double r2 = 0.0;
    for (const v3 &q : {t.v0, t.v1, t.v2})
      r2 = fmax(r2, (q.x - cx) * (q.x - cx) + (q.y - cy) * (q.y - cy) + (q.z - cz) * (q.z - cz));
    float r = (float)(sqrt(r2) * 1.0001 + 1e-6);
    if (!(t.cond < 300.0)) r = INFINITY;
    bd.push_back({(float)cx, (float)cy, (float)cz, r});
  }
  // small-scene lane table (rfx_types.h CullRec)
  std::vector<CullRec> cs;
  std::vector<CullTri> ct;
  uint64_t cull_valid = 0;
  const bool small = s->spheres.size() <= 32 && s->tris.size() <= 32;
  if (small)
  {
    cs.assign(64, CullRec{});
    ct.assign(32, CullTri{});
    for (size_t i = 0; i < s->spheres.size(); ++i)
    {
      const int lane = (int)(i & 1u) * 16 + (int)(i >> 1);
      const Bound &b = bd[i];
      CullRec c{};
      c.x = b.x; c.y = b.y; c.z = b.z; c.r = b.r;
      cs[lane] = c;
      cull_valid |= 1ull << lane;
    }
    for (size_t i = 0; i < s->tris.size(); ++i)
    {
      const HostTri &t = s->tris[i];
      const Bound &b = bd[s->spheres.size() + i];
      CullRec c{};
      c.x = b.x; c.y = b.y; c.z = b.z; c.r = b.r;
      if (t.cond < 300.0)
      {
        // plane of the triangle in double: unit normal of (v1 - v0) x (v2 - v0), offset n . v0
        const double ax = (double)t.v1.x - t.v0.x, ay = (double)t.v1.y - t.v0.y, az = (double)t.v1.z - t.v0.z;
        const double bx = (double)t.v2.x - t.v0.x, by = (double)t.v2.y - t.v0.y, bz = (double)t.v2.z - t.v0.z;
        double nx = ay * bz - az * by, ny = az * bx - ax * bz, nz = ax * by - ay * bx;
        const double nl = sqrt(nx * nx + ny * ny + nz * nz);
        if (nl > 0.0)
        {
          nx /= nl; ny /= nl; nz /= nl;
          c.nx = (float)nx; c.ny = (float)ny; c.nz = (float)nz;
          c.d = (float)(nx * t.v0.x + ny * t.v0.y + nz * t.v0.z);
        }
      }
      cs[32 + i] = c;
      cull_valid |= 1ull << (32 + i);
      // footprint record (primary-bundle masks): the dual rows of the basis (A, B, C) = (v2 - v0, v1 - v0, n) in
      // double (the float inverse the reference computes differs by a relative ~cond eps, inside the test's
      // margins); only for well-conditioned triangles (cond < 100)
      CullTri q{};
      q.v0x = t.v0.x; q.v0y = t.v0.y; q.v0z = t.v0.z;
      q.nu = q.nv = q.nuv = INFINITY;
      if (t.cond < 100.0 && c.nx * c.nx + c.ny * c.ny + c.nz * c.nz > 0.5f)
      {
        const double A[3] = {(double)t.v2.x - t.v0.x, (double)t.v2.y - t.v0.y, (double)t.v2.z - t.v0.z};
        const double Bv[3] = {(double)t.v1.x - t.v0.x, (double)t.v1.y - t.v0.y, (double)t.v1.z - t.v0.z};
        const double Cv[3] = {c.nx, c.ny, c.nz};
        auto cross = [](const double *a, const double *b, double *o) {
          o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
        };
        double bc[3], ca[3];
        cross(Bv, Cv, bc);
        cross(Cv, A, ca);
        const double det = A[0] * bc[0] + A[1] * bc[1] + A[2] * bc[2];
        if (fabs(det) > 0.0)
        {
          const double gu[3] = {bc[0] / det, bc[1] / det, bc[2] / det}, gv[3] = {ca[0] / det, ca[1] / det, ca[2] / det};
          q.gux = (float)gu[0]; q.guy = (float)gu[1]; q.guz = (float)gu[2];
          q.gvx = (float)gv[0]; q.gvy = (float)gv[1]; q.gvz = (float)gv[2];
          q.nu = (float)(sqrt(gu[0] * gu[0] + gu[1] * gu[1] + gu[2] * gu[2]) * 1.001);
          q.nv = (float)(sqrt(gv[0] * gv[0] + gv[1] * gv[1] + gv[2] * gv[2]) * 1.001);
          const double s0 = gu[0] + gv[0], s1 = gu[1] + gv[1], s2 = gu[2] + gv[2];
          q.nuv = (float)(sqrt(s0 * s0 + s1 * s1 + s2 * s2) * 1.001);
        }
      }
      ct[i] = q;
    }
  }
  // pair BVH (large scenes; spheres of a pair whose second slot is padding: r2 = -inf, never hit)
  std::vector<BvhNode> bvh;
  int bvh_depth = 0;
  double bvh_ref[3] = {0.0, 0.0, 0.0};
  if (nsph > 32)
  {
    // leaves: groups of RFX_BVH_LEAF_PAIRS consecutive pairs (compact clusters of the median-split order)
    const size_t npairs = ((nsph + 1) / 2 + RFX_BVH_LEAF_PAIRS - 1) / RFX_BVH_LEAF_PAIRS;
    constexpr size_t kLeafSph = 2 * RFX_BVH_LEAF_PAIRS;
    std::vector<PairBox> box(npairs);
    for (size_t j = 0; j < npairs; ++j)
    {
      PairBox &b = box[j];
      for (int k = 0; k < 3; ++k) { b.lo[k] = INFINITY; b.hi[k] = -INFINITY; }
      for (size_t q = kLeafSph * j; q < std::min(nsph, kLeafSph * j + kLeafSph); ++q)
      {
        const double c[3] = {bd[q].x, bd[q].y, bd[q].z}, rr = bd[q].r;
        for (int k = 0; k < 3; ++k) { b.lo[k] = fmin(b.lo[k], c[k] - rr); b.hi[k] = fmax(b.hi[k], c[k] + rr); }
      }
      for (int k = 0; k < 3; ++k) b.c[k] = 0.5 * (b.lo[k] + b.hi[k]);
    }
    std::vector<uint32_t> pairs(npairs);
    for (size_t j = 0; j < npairs; ++j) pairs[j] = (uint32_t)j;
    for (int k = 0; k < 3; ++k)
    {
      double lo = INFINITY, hi = -INFINITY;
      for (const PairBox &pb : box) { lo = fmin(lo, pb.lo[k]); hi = fmax(hi, pb.hi[k]); }
      bvh_ref[k] = (double)(float)(0.5 * (lo + hi));  // the float the kernel measures from
    }
    build_pair_bvh(bvh, pairs, 0, npairs, box, bvh_ref, 0, bvh_depth);
    if (bvh_depth > RFX_BVH_STACK) { bvh.clear(); bvh_depth = 0; }  // deeper than the kernel's stack: chunk loops
    if (bvh.size() > 32767 || npairs > 32768) { bvh.clear(); bvh_depth = 0; }  // int16 stack slots (rfx_trace.h)
  }
  std::vector<PlaneGeo> pg;
  std::vector<MatRec> pm;
  for (const HostPlane &p : s->planes)
  {
    pg.push_back({p.pos.x, p.pos.y, p.pos.z, p.norm.x, p.norm.y, p.norm.z, p.obj, p.mat.dielectric});
    pm.push_back({p.mat.r, p.mat.g, p.mat.b, p.mat.refl});
  }
  // object index -> (kind, index in the device arrays): spheres through their spatial order
  std::vector<int32_t> loc(s->obj_kind.size());
  {
    std::vector<int32_t> sph_dev(nsph);
    for (size_t di = 0; di < nsph; ++di) sph_dev[order[di]] = (int32_t)di;
    for (size_t o = 0; o < loc.size(); ++o)
    {
      const int kind = s->obj_kind[o], idx = s->obj_idx[o];
      loc[o] = kind << 28 | (kind == 0 ? sph_dev[idx] : idx);
    }
  }
  std::vector<LightRec> lr;
  for (const HostLight &l : s->lights) lr.push_back({l.origin.x, l.origin.y, l.origin.z, l.radius, l.r, l.g, l.b, l.power});
  std::vector<TexRec> tr;
  std::vector<uint32_t> pool;
  for (const HostTexture &t : s->textures)
  {
    const bool empty = t.texels.empty();  // the reference's empty colorBuf: checker (Texture.cpp:242-243)
    tr.push_back({(uint32_t)pool.size(), empty ? 0u : t.w, empty ? 0u : t.h, 0});
    pool.insert(pool.end(), t.texels.begin(), t.texels.end());
  }
  DevScene d{};
  if ((rc = upload(r, sg, &d.sph_geo)) || (rc = upload(r, sp, &d.sph_pair)) || (rc = upload(r, sm, &d.sph_mat)) ||
      (rc = upload(r, si, &d.sph_info)) ||
      (rc = upload(r, tg, &d.tri_geo)) || (rc = upload(r, ts, &d.tri_shade)) || (rc = upload(r, tm, &d.tri_mat)) ||
      (rc = upload(r, lr, &d.lights)) || (rc = upload(r, tr, &d.texs)) || (rc = upload(r, pool, &d.texels)) ||
      (rc = upload(r, bd, &d.bound)) || (rc = upload(r, cs, &d.cull_small)) || (rc = upload(r, ct, &d.cull_tri)) || (rc = upload(r, cb, &d.chunk_bound)) ||
      (rc = upload(r, pg, &d.pln_geo)) || (rc = upload(r, pm, &d.pln_mat)) || (rc = upload(r, loc, &d.obj_loc)) ||
      (rc = upload(r, bvh, &d.bvh)))
    return rc;
  {
    // the bounce kernel's LDS copy of the node links and margin terms (rfx_types.h DevScene::bvh_aux): mt rounded up
    // to a multiple of mstep (one step more than the ceiling, so the float decode stays above)
    float mt_max = 0.0f;
    for (const BvhNode &n : bvh) mt_max = fmaxf(mt_max, fmaxf(n.mt[0], n.mt[1]));
    const float mstep = mt_max > 0.0f ? mt_max / 65000.0f : 1.0f;
    std::vector<uint32_t> aux(2 * bvh.size());
    for (size_t i = 0; i < bvh.size(); ++i)
    {
      const BvhNode &n = bvh[i];
      uint32_t q[2];
      for (int c = 0; c < 2; ++c) q[c] = (uint32_t)std::min(65535.0, ceil((double)n.mt[c] / mstep) + 1.0);
      aux[2 * i] = ((uint32_t)(uint16_t)(int16_t)n.child[0]) | ((uint32_t)(uint16_t)(int16_t)n.child[1] << 16);
      aux[2 * i + 1] = q[0] | q[1] << 16;
    }
    if ((rc = upload(r, aux, &d.bvh_aux))) return rc;
    d.bvh_mstep = mstep;
    d.n_bvh = (int32_t)bvh.size();
  }
  d.n_sph = (int32_t)sg.size();
  d.n_tri = (int32_t)tg.size();
  d.n_light = (int32_t)lr.size();
  d.n_chunk = (int32_t)cb.size();
  d.n_pln = (int32_t)pg.size();
  d.n_tex = (int32_t)tr.size();
  d.bvh_depth = bvh_depth;
  d.bvh_rx = (float)bvh_ref[0]; d.bvh_ry = (float)bvh_ref[1]; d.bvh_rz = (float)bvh_ref[2];
  if (!bvh.empty())  // regroup sort keys: 8 origin cells per axis over the root box
  {
    const BvhNode &root = bvh[0];
    const float lo[3] = {fminf(root.lx[0], root.lx[1]), fminf(root.ly[0], root.ly[1]), fminf(root.lz[0], root.lz[1])};
    const float hi[3] = {fmaxf(root.hx[0], root.hx[1]), fmaxf(root.hy[0], root.hy[1]), fmaxf(root.hz[0], root.hz[1])};
    float s[3];
    for (int k = 0; k < 3; ++k) s[k] = hi[k] > lo[k] ? 8.0f / (hi[k] - lo[k]) : 0.0f;
    d.key_lx = lo[0]; d.key_ly = lo[1]; d.key_lz = lo[2];
    d.key_sx = s[0]; d.key_sy = s[1]; d.key_sz = s[2];
  }
  d.n_obj = (int32_t)loc.size();
  d.cull_valid = cull_valid;
  d.skybox_tex = s->skybox;
  const col amb = cscale(s->diff, s->diff_power);                                    // Scene.cpp:186 (first factor)
  d.amb_r = amb.r; d.amb_g = amb.g; d.amb_b = amb.b;
  d.env_r = s->env.r; d.env_g = s->env.g; d.env_b = s->env.b;
  d.half_tile_w = s->half_tile_w;
  d.half_tile_h = s->half_tile_h;
  r->dev = d;
  r->has_scene = true;
  ++r->scene_gen;
  r->prim_key.clear();
  r->prim_seen.clear();
  return RFX_OK;
}

extern "C" int rfx_renderer_set_rng(rfx_renderer *r, uint32_t sphere_seed, uint32_t jitter_seed)
{
  if (!r) return fail(RFX_ERR_ARG, "set_rng: null renderer");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  HIP_CHECK(hipMemcpyAsync(seed_cur(r), &sphere_seed, sizeof(uint32_t), hipMemcpyHostToDevice, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  r->jitter_seed = jitter_seed;
  r->rewind_ok = false;
  ++r->state_seq;
  return RFX_OK;
}

extern "C" int rfx_renderer_get_rng(rfx_renderer *r, uint32_t *sphere_seed, uint32_t *jitter_seed)
{
  if (!r) return fail(RFX_ERR_ARG, "get_rng: null renderer");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  uint32_t s = 0;
  int err = 0;
  HIP_CHECK(hipMemcpyAsync(&s, seed_cur(r), sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
  HIP_CHECK(hipMemcpyAsync(&err, r->d_err, sizeof(int), hipMemcpyDeviceToHost, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  if (err & 1) return fail(RFX_ERR_RNG, "RNG pre-pass ran short of accepted triples");  // (bit 4: an exact fallback)
  if (sphere_seed) *sphere_seed = s;
  if (jitter_seed) *jitter_seed = r->jitter_seed;
  return RFX_OK;
}

// RNG blocks of a frame's traces, split into nslices equal slices (one per rank in the multi-GPU pre-pass)
static uint64_t rng_layout(uint64_t traces, uint32_t nslices, uint64_t *per_slice)
{
  if (!nslices) nslices = 1;
  const uint64_t bps = (rng_blocks_for(traces) + nslices - 1) / nslices;
  if (per_slice) *per_slice = bps;
  return bps * nslices;
}

// the second randDir buffer (emit-ahead frames, the odd spans of a split frame)
static int ensure_rd_alt(rfx_renderer *r, uint64_t traces)
{
  if (r->rd_alt_cap < traces)
  {
    (void)hipFree(r->d_rd_alt);
    r->d_rd_alt = nullptr;
    r->rd_alt_cap = 0;
    HIP_CHECK(hipMalloc(&r->d_rd_alt, traces * sizeof(uint32_t)));
    r->rd_alt_cap = traces;
  }
  return RFX_OK;
}

static int ensure_rng_workspace(rfx_renderer *r, uint64_t traces, uint64_t nblk)
{
  if (traces > r->rd_cap)
  {
    (void)hipFree(r->d_rd);
    r->d_rd = nullptr;
    r->rd_cap = 0;
    HIP_CHECK(hipMalloc(&r->d_rd, traces * sizeof(uint32_t)));
    r->rd_cap = traces;
  }
  if (nblk > r->blk_cap)
  {
    (void)hipFree(r->d_blk_cnt); (void)hipFree(r->d_jump); (void)hipFree(r->d_rng_masks); (void)hipFree(r->d_blk_off);
    (void)hipFree(r->d_rng_status);
    r->d_blk_cnt = nullptr; r->d_jump = nullptr; r->d_rng_masks = nullptr; r->d_blk_off = nullptr; r->blk_cap = 0;
    r->d_rng_status = nullptr;
    HIP_CHECK(hipMalloc(&r->d_blk_cnt, nblk * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&r->d_rng_status, nblk * sizeof(unsigned long long)));
    HIP_CHECK(hipMemset(r->d_rng_status, 0, nblk * sizeof(unsigned long long)));  // epoch 0: no launch's
    r->rng_epoch = 0;
    if (!r->d_rng_ticket)
    {
      HIP_CHECK(hipMalloc(&r->d_rng_ticket, sizeof(unsigned long long)));
      HIP_CHECK(hipMemset(r->d_rng_ticket, 0, sizeof(unsigned long long)));
    }
    HIP_CHECK(hipMalloc(&r->d_blk_off, nblk * sizeof(uint64_t)));
    (void)hipFree(r->d_tile_sum);
    r->d_tile_sum = nullptr;
    HIP_CHECK(hipMalloc(&r->d_tile_sum, (nblk / 4096 + 1) * sizeof(uint32_t)));
    if (!r->d_rng_range) HIP_CHECK(hipMalloc(&r->d_rng_range, 4 * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&r->d_rng_masks, nblk * 256 * sizeof(uint16_t)));
    std::vector<uint32_t> jump(2 * (256 + nblk));
    rng_jump_table(nblk, jump.data());
    HIP_CHECK(hipMalloc(&r->d_jump, jump.size() * sizeof(uint32_t)));
    HIP_CHECK(hipMemcpy(r->d_jump, jump.data(), jump.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    r->blk_cap = nblk;
  }
  return RFX_OK;
}

// Whole pre-pass on one device: every block counted here (the 1-GPU path, and the redundant form of the
// multi-GPU one).  Sphere stream: d_seed[seed_idx] -> pre-pass -> the other word, which becomes current.
static int enqueue_rng(rfx_renderer *r, uint64_t traces, hipStream_t st)
{
  int rc;
  const uint64_t nblk = rng_layout(traces, 1, nullptr);
  if ((rc = ensure_rng_workspace(r, traces, nblk)) != RFX_OK) return rc;
  HIP_CHECK(launch_rng_count(seed_cur(r), r->d_jump, r->d_blk_cnt, 0, nblk, r->d_rng_masks, st));
  HIP_CHECK(launch_rng_finish(seed_cur(r), r->d_jump, seed_next(r), r->d_blk_cnt, r->d_rng_masks, nblk, traces,
                              r->d_rd, r->d_err, 1, 1, 1, 0, 1, st));
  r->seed_idx ^= 1u;
  ++r->state_seq;
  r->rewind_ok = false;
  return RFX_OK;
}

// Validate a frame and build its kernel parameters (everything but the output pointers).
struct FramePlan {
  FrameParams P;
  uint64_t traces = 0;
  hipStream_t st = nullptr;
  // band partition (rfx.h: nranks > 1, row_block 0): the emit writes the randDirs of traces [band_lo, band_hi) only,
  // into a buffer of the band's size (its base pointer offset by band_lo)
  bool band = false;
  uint64_t band_lo = 0, band_hi = UINT64_MAX;
  // one span of a split frame (rfx_render_frame): launches on two streams overlap, so the per-renderer state of
  // single launches (tile schedule, per-view masks, regroup queue) stays out
  bool split = false;
  int split_side = 0;  // the span's stream (0: the caller's, 1: the renderer's second)
  uint64_t rd_traces() const { return band ? band_hi - band_lo : traces; }  // randDir words the plan writes and reads
};

static int plan_frame(rfx_renderer *r, const rfx_frame *f, void *stream, FramePlan &plan);

extern "C" int rfx_frame_rng_blocks(rfx_renderer *r, const rfx_frame *f, uint32_t nslices, uint64_t *per_slice)
{
  FramePlan pl;
  int rc;
  if ((rc = plan_frame(r, f, nullptr, pl)) != RFX_OK) return rc;
  if (!nslices || !per_slice) return fail(RFX_ERR_ARG, "frame_rng_blocks: nslices > 0 and an output required");
  rng_layout(pl.traces, nslices, per_slice);
  return RFX_OK;
}

extern "C" int rfx_frame_rng_count(rfx_renderer *r, const rfx_frame *f, uint32_t slice, uint32_t nslices,
                                   uint32_t *d_blk_counts, void *stream)
{
  FramePlan pl;
  int rc;
  if ((rc = plan_frame(r, f, stream, pl)) != RFX_OK) return rc;
  if (!d_blk_counts || !nslices || slice >= nslices) return fail(RFX_ERR_ARG, "frame_rng_count: bad slice");
  uint64_t bps = 0;
  const uint64_t nblk = rng_layout(pl.traces, nslices, &bps);
  if ((rc = ensure_rng_workspace(r, pl.rd_traces(), nblk)) != RFX_OK) return rc;
  HIP_CHECK(launch_rng_count(seed_cur(r), r->d_jump, d_blk_counts, (uint64_t)slice * bps, bps, nullptr, pl.st));
  return RFX_OK;
}

// Tile schedule of a trace launch: the order sorted from the previous launch's costs when that launch had the
// same grid and mode (key), else the identity; either way this launch records its own costs.
static int tile_schedule(rfx_renderer *r, FrameParams &P, hipStream_t st, uint64_t &key, bool &record)
{
  const uint32_t n = trace_tiles(P);
  key = ((uint64_t)P.W << 40) ^ ((uint64_t)P.grid_rows << 16) ^ ((uint64_t)(uint32_t)P.ss << 4) ^
        (uint64_t)(P.additive * 2 + P.accumulate);
  if (!r->tile_stream)
  {
    HIP_CHECK(hipStreamCreateWithFlags(&r->tile_stream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&r->tile_fork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&r->tile_join, hipEventDisableTiming));
    HIP_CHECK(hipMalloc(&r->d_tile_scratch, tile_order_scratch()));
  }
  if (n > r->tile_cap)
  {
    HIP_CHECK(hipStreamSynchronize(r->tile_stream));  // a pending sort may still read the old buffers
    if (r->tile_pending) HIP_CHECK(hipEventSynchronize(r->tile_join));  // (RFX_TILE_SORT_MAIN: on the launch's stream)
    HIP_CHECK(hipStreamSynchronize(st));
    (void)hipFree(r->d_tile_cost); (void)hipFree(r->d_tile_order);
    r->d_tile_cost = r->d_tile_order = nullptr;
    r->tile_cap = 0;
    r->tile_n = 0;
    r->tile_pending = false;
    HIP_CHECK(hipMalloc(&r->d_tile_cost, (size_t)n * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&r->d_tile_order, (size_t)n * sizeof(uint32_t)));
    r->tile_cap = n;
  }
  // the last sort must have read the costs this launch may overwrite (every workgroup writes its tile's)
  // and written the order it reads
  if (r->tile_pending && r->tile_waited != st)
  {
    HIP_CHECK(hipStreamWaitEvent(st, r->tile_join, 0));
    r->tile_waited = st;
  }
  const bool same = r->tile_pending && r->tile_n == n && r->tile_key == key;
  P.tile_order = (same && r->tile_mode != 2) ? r->d_tile_order : nullptr;
  // record (and re-sort) every RFX_TILE_SORT_EVERY-th launch, and at once after a grid change
  record = !same || r->tile_count % RFX_TILE_SORT_EVERY == 0;
  P.tile_cost = record ? r->d_tile_cost : nullptr;
  ++r->tile_count;
  return RFX_OK;
}

// The randDirs of a planned frame into rd (the scan of the counts and the scatter; the stream state moves past the
// frame), then the caller's event, if any.
static int emit_frame(rfx_renderer *r, FramePlan &pl, const uint32_t *d_counts, const uint16_t *d_masks, uint64_t nblk,
                      uint32_t *rd, hipEvent_t emitted)
{
  const FrameParams &P = pl.P;
  const hipStream_t st = pl.st;
  const uint64_t ss2 = P.ss > 0 ? (uint64_t)(P.ss * P.ss) : 1;
  if (pl.band)  // the band's randDirs into a buffer of the band's size: index trace - band_lo
    HIP_CHECK(launch_rng_finish_band(seed_cur(r), r->d_jump, seed_next(r), d_counts, nullptr, nblk, pl.traces,
                                     rd - pl.band_lo, r->d_err, pl.band_lo, pl.band_hi, r->d_blk_off, r->d_rng_range,
                                     r->d_tile_sum, st));
  else if (P.nranks <= 1 && nblk > RFX_SCAN_EMIT_BLOCKS)
    HIP_CHECK(launch_rng_finish_band(seed_cur(r), r->d_jump, seed_next(r), d_counts, d_masks, nblk, pl.traces, rd,
                                     r->d_err, 0, pl.traces, r->d_blk_off, r->d_rng_range, r->d_tile_sum, st));
  else
    HIP_CHECK(launch_rng_finish(seed_cur(r), r->d_jump, seed_next(r), d_counts, d_masks, nblk, pl.traces, rd,
                                r->d_err, ss2, P.W, P.row_block, P.rank, P.nranks, st));
  r->seed_idx ^= 1u;
  ++r->state_seq;
  // the caller's event: the randDirs are written and the next frame's stream state is known (the next frame's
  // RNG count may start on another stream while this frame traces)
  if (emitted) HIP_CHECK(hipEventRecord(emitted, st));
  return RFX_OK;
}

// The whole pre-pass of a one-device launch in one kernel (rng_fused: count, look-back scan and scatter), with
// emit_frame's bookkeeping.  RFX_RNG_FUSED=0 keeps the two-kernel form (rng_count, then emit_frame).
// Launches of at most RFX_RNG_FUSED_MAX_BLOCKS pre-pass blocks take it.  Its block-order ticket (one atomic per
// workgroup on one word) serialises the launch's start in proportion to the blocks, so it pays only on small launches
// (interleaved A/B, frame ms, one-pass / two-kernel, profiles/r06/ab/prepass_limit_*_r6e.jsonl): 640x480 (166 blocks)
// 0.0552 / 0.0565, 960x540 (269) 0.0657 / 0.0643, 1280x720 (466) 0.0841 / 0.0803, 1920x1080 (1,013) 0.0812 / 0.0679.
#ifndef RFX_RNG_FUSED
#define RFX_RNG_FUSED 1
#endif
#ifndef RFX_RNG_FUSED_MAX_BLOCKS
#define RFX_RNG_FUSED_MAX_BLOCKS 256
#endif
static bool fused_prepass(const FramePlan &pl, uint64_t nblk)
{
  return RFX_RNG_FUSED && !pl.band && pl.P.nranks <= 1 && nblk <= (uint64_t)RFX_RNG_FUSED_MAX_BLOCKS;
}

static int prepass_fused(rfx_renderer *r, FramePlan &pl, uint64_t nblk, uint32_t *rd, hipEvent_t emitted)
{
  // 1 .. 2^28 - 1, a new tag per launch; when the tags wrap, the words earlier launches left are cleared first (a word
  // of a wider launch could otherwise carry the new tag)
  if (r->rng_epoch == (1u << 28) - 1)
  {
    HIP_CHECK(hipMemsetAsync(r->d_rng_status, 0, r->blk_cap * sizeof(unsigned long long), pl.st));
    r->rng_epoch = 0;
  }
  ++r->rng_epoch;
  HIP_CHECK(launch_rng_fused(seed_cur(r), r->d_jump, seed_next(r), nblk, pl.traces, rd, r->d_err, r->d_rng_status,
                             r->d_rng_ticket, r->rng_tickets, r->rng_epoch, pl.st));
  r->rng_tickets += nblk;  // every block of the launch takes one ticket
  r->seed_idx ^= 1u;
  ++r->state_seq;
  if (emitted) HIP_CHECK(hipEventRecord(emitted, pl.st));
  return RFX_OK;
}

static int trace_frame(rfx_renderer *r, FramePlan &pl, const uint32_t *rd, float *d_rgb, uint32_t *d_argb,
                       uint64_t *d_counters);

static int finish_frame(rfx_renderer *r, FramePlan &pl, const uint32_t *d_counts, const uint16_t *d_masks,
                        uint64_t nblk, float *d_rgb, uint32_t *d_argb, uint64_t *d_counters,
                        hipEvent_t emitted = nullptr)
{
  int rc;
  if (r->emit_pending >= 0)
    return fail(RFX_ERR_STATE, "render_frame: an emitted frame awaits rfx_render_frame_emitted (or rfx_frame_rng_discard)");
  if ((rc = emit_frame(r, pl, d_counts, d_masks, nblk, r->d_rd, emitted)) != RFX_OK) return rc;
  r->trace_buf = 0;
  if ((rc = timing_event(r, pl.st)) != RFX_OK) return rc;
  return trace_frame(r, pl, r->d_rd, d_rgb, d_argb, d_counters);
}

// The trace launch(es) of a planned frame whose randDirs are in rd, and the end-of-frame bookkeeping.
static int trace_frame(rfx_renderer *r, FramePlan &pl, const uint32_t *rd, float *d_rgb, uint32_t *d_argb,
                       uint64_t *d_counters)
{
  int rc;
  FrameParams &P = pl.P;
  const hipStream_t st = pl.st;
  P.img = d_rgb;
  P.argb = d_argb;
  // ray regrouping: plain pixels of a large scene park their traces after RFX_PARK_AFTER segments; the bounce
  // kernel resumes them in packed waves (rfx_trace.h bounce_kernel)
  const bool small = r->dev.n_sph <= 32 && r->dev.n_tri <= 32;
  const bool plain = P.ss == 1 && !P.additive && !P.accumulate;
  const int park_after = r->park_after < 0 ? (small ? 0 : RFX_PARK_AFTER) : r->park_after;
  const bool park = park_after > 0 && plain && !d_counters && P.depth > park_after && P.grid_rows && !pl.split;
  const bool sort_queue = park && r->queue_sort;
  if (park)
  {
    if (pl.traces > r->queue_cap)
    {
      (void)hipFree(r->d_queue); (void)hipFree(r->d_qkey); (void)hipFree(r->d_qorder);
      r->d_queue = nullptr;
      r->d_qkey = r->d_qorder = nullptr;
      r->queue_cap = 0;
      HIP_CHECK(hipMalloc(&r->d_queue, pl.traces * sizeof(QRay)));
      HIP_CHECK(hipMalloc(&r->d_qkey, pl.traces * sizeof(uint32_t)));
      HIP_CHECK(hipMalloc(&r->d_qorder, pl.traces * sizeof(uint32_t)));
      r->queue_cap = pl.traces;
    }
    const size_t qwords = 2 + kQueueBuckets;
    if (!r->d_qctr) HIP_CHECK(hipMalloc(&r->d_qctr, qwords * sizeof(uint32_t)));
    HIP_CHECK(hipMemsetAsync(r->d_qctr, 0, (sort_queue ? qwords : 2) * sizeof(uint32_t), st));
    P.queue = r->d_queue;
    P.queue_count = r->d_qctr;
    P.queue_next = r->d_qctr + 1;
    P.park_after = park_after;
    if (sort_queue)
    {
      P.queue_key = r->d_qkey;
      P.queue_order = r->d_qorder;
    }
  }
  P.rd_state = pl.band ? rd - pl.band_lo : rd;  // a band's randDirs are stored from its first trace on (emit_frame)
  P.counters = (unsigned long long *)d_counters;
  // mode 1 schedules only launches of at least RFX_TILE_ORDER_MIN_TILES tiles: on shorter ones the sort's
  // latency (three small launches and a cross-stream wait, ~15 us) is not hidden by the RNG pre-pass
  const bool sched = P.grid_rows && r->tile_mode && !d_counters && P.ss >= 0 && !pl.split &&
                     (r->tile_mode != 1 || trace_tiles(P) >= RFX_TILE_ORDER_MIN_TILES);
  uint64_t key = 0;
  bool record = false;
  if (sched && (rc = tile_schedule(r, P, st, key, record)) != RFX_OK) return rc;
  // primary-bundle cull masks: small scenes, plain and SSAA frames (not block previews), culling launches; large scenes,
  // plain frames: the primary bundles' chunk lists.  Recomputed only when the camera, the frame geometry, the sampling
  // or the scene changed (the bench's frames all reuse one set)
  // The chunk mode (sampleNum > 8: a wave per pixel) takes closest-hit masks only, over each pixel's sample rectangle:
  // one cheap cull per pixel that every chunk of its samples reuses, so they are built for every view and every span
  // of a split frame (into the span's stream side's buffer: the spans of the two streams overlap).
  const bool chunks = RFX_PRIM_CHUNKS && RFX_PRIM_LANES && small && trace_chunks(P);
  if (chunks && pl.split && !d_counters && P.grid_rows && r->prim_mode)
  {
    const int sd = pl.split_side;
    const size_t nwords = (size_t)trace_tiles(P) * kPrimWords;
    if (nwords > r->split_mask_cap[sd])
    {
      (void)hipFree(r->d_split_mask[sd]);
      r->d_split_mask[sd] = nullptr;
      r->split_mask_cap[sd] = 0;
      HIP_CHECK(hipMalloc(&r->d_split_mask[sd], nwords * sizeof(uint64_t)));
      r->split_mask_cap[sd] = nwords;
    }
    HIP_CHECK(launch_prim_cull(r->dev, P, r->d_split_mask[sd], st));
    P.prim_mask = r->d_split_mask[sd];
    P.prim_shadow = 0;
  }
  else if (((small && (plain || (RFX_PRIM_LANES && (trace_lanes(P) || chunks)) || (RFX_PRIM_SSAA && P.ss >= 1)) &&
             !park) ||
            (RFX_PRIM_LARGE && !small && plain)) &&
           !d_counters && P.grid_rows && r->prim_mode && !pl.split)
  {
    struct Key { float cam[15]; uint32_t W, H, grid_rows, row0, row_block, rank, nranks; int32_t depth, ss, additive;
                 uint64_t p_begin, p_end, gen; } k;
    memset(&k, 0, sizeof(k));  // padding bytes too: the key is compared bytewise
    const float cam[15] = {P.eye_x, P.eye_y, P.eye_z, P.v11, P.v12, P.v13, P.v21, P.v22, P.v23,
                           P.v31, P.v32, P.v33, P.rz, P.wh, P.hh};
    memcpy(k.cam, cam, sizeof(cam));
    k.W = P.W; k.H = P.H; k.grid_rows = P.grid_rows; k.row0 = P.row0; k.row_block = P.row_block; k.rank = P.rank;
    k.nranks = P.nranks; k.depth = P.depth > 0 ? 1 : 0; k.p_begin = P.p_begin; k.p_end = P.p_end; k.gen = r->scene_gen;
    k.ss = P.ss; k.additive = P.additive ? 1 : 0;
    const size_t nwords = trace_tiles(P) * (small ? kPrimWords : kPrimLargeWords);
    std::vector<uint8_t> kb((const uint8_t *)&k, (const uint8_t *)&k + sizeof(k));
    if (nwords > r->prim_cap)
    {
      (void)hipFree(r->d_prim_mask);
      r->d_prim_mask = nullptr;
      r->prim_cap = 0;
      HIP_CHECK(hipMalloc(&r->d_prim_mask, nwords * sizeof(uint64_t)));
      r->prim_cap = nwords;
      r->prim_key.clear();
      r->prim_seen.clear();
    }
    // a view seen for the first time renders with per-launch bundles (a camera that moves every frame never pays
    // for masks); the masks are built when the same view comes again, and kept while it stays
    if (r->prim_mode == 2 || kb != r->prim_key)
    {
      const bool repeat = kb == r->prim_seen;
      r->prim_seen = kb;
      r->prim_key.clear();
      if (repeat || r->prim_mode == 2 || chunks)
      {
        HIP_CHECK(launch_prim_cull(r->dev, P, r->d_prim_mask, st));
        r->prim_key = kb;
      }
    }
    if (!r->prim_key.empty())
    {
      P.prim_mask = r->d_prim_mask;
      P.prim_shadow = P.additive || chunks ? 0 : 1;  // jittered frames, chunks: closest-hit masks only (prim_cull_kernel)
    }
  }
  if (P.grid_rows) HIP_CHECK(launch_trace(r->dev, P, d_counters != nullptr, st));
  r->bounce_form = 0;
  if (park)
  {
    // packed waves over the queue, as many as the chip holds at once (RFX_BOUNCE_GROUPS_PER_CU workgroups of two waves
    // per CU: 7 waves per SIMD); a lane whose trace ends takes the next entry, so no wave waits for a slot
    const uint64_t waves = (pl.traces + 63) / 64;
    const uint32_t groups = (uint32_t)std::min<uint64_t>((waves + 1) / 2, (uint64_t)r->cus * RFX_BOUNCE_GROUPS_PER_CU);
    const int cfg = 1 | (r->dev.n_light > 32 ? 2 : 0) | (small ? 4 : 0) | (r->dev.n_pln ? 8 : 0) |  // rfx_trace.h kCfg*
                    (RFX_ONE_LIGHT && r->dev.n_light == 1 ? 32 : 0);  // kCfgOneLight (rfx_trace_plain_park.hip)
    if (sort_queue) HIP_CHECK(launch_queue_sort(r->d_qctr, r->d_qkey, r->d_qctr + 2, r->d_qorder, st));
    // a BVH whose nodes fit the workgroup's LDS (56 B each beside the stacks: up to ~2,100 nodes, i.e. 4,200 spheres):
    // the LDS-staged bounce kernel, one 16-wave workgroup per CU (C5 trace + bounce -4..6%, tools/ab.py); else the
    // two-wave workgroups walking the nodes in global memory
    const uint32_t lgroups = (uint32_t)std::min<uint64_t>((waves + kLdsBvhWaves - 1) / kLdsBvhWaves, (uint64_t)r->cus);
    r->bounce_form = 2;
    if (small || !lds_bvh_fits(r->dev.n_bvh) || launch_bounce_lds(cfg, lgroups, r->dev, P, st) != hipSuccess)
    {
      (void)hipGetLastError();  // an LDS launch the runtime refused: the global-memory form instead
      launch_bounce(cfg, dim3(groups), r->dev, P, st);
      r->bounce_form = 1;  // visible through rfx_renderer_bounce_form, so a silent fall-back shows in the tests
    }
    HIP_CHECK(hipGetLastError());
  }
  if (record)
  {
#if RFX_TILE_SORT_MAIN
    // sort this launch's tile costs into the next launch's order on the launch's own stream: no cross-stream events
    // (tile_join only for a later launch on another stream)
    HIP_CHECK(launch_tile_order(r->d_tile_cost, trace_tiles(P), r->d_tile_order, r->d_tile_scratch, st));
    HIP_CHECK(hipEventRecord(r->tile_join, st));
    r->tile_waited = st;
#else
    // sort this launch's tile costs into the next launch's order beside the next frame's pre-pass
    HIP_CHECK(hipEventRecord(r->tile_fork, st));
    HIP_CHECK(hipStreamWaitEvent(r->tile_stream, r->tile_fork, 0));
    HIP_CHECK(launch_tile_order(r->d_tile_cost, trace_tiles(P), r->d_tile_order, r->d_tile_scratch, r->tile_stream));
    HIP_CHECK(hipEventRecord(r->tile_join, r->tile_stream));
    r->tile_waited = nullptr;
#endif
    r->tile_pending = true;
    r->tile_n = trace_tiles(P);
    r->tile_key = key;
  }
  if ((rc = timing_event(r, st)) != RFX_OK) return rc;
  if (P.additive)                                                                  // 2 draws per pixel, raster order
    r->jitter_seed = lcg_jump(r->jitter_seed, 2ull * (P.p_end - P.p_begin));
  return RFX_OK;
}

extern "C" int rfx_render_frame_counted(rfx_renderer *r, const rfx_frame *f, uint32_t nslices,
                                        const uint32_t *d_blk_counts, float *d_rgb, uint32_t *d_argb,
                                        uint64_t *d_counters, void *stream)
{
  return rfx_render_frame_counted_ev(r, f, nslices, d_blk_counts, d_rgb, d_argb, d_counters, stream, nullptr);
}

extern "C" int rfx_render_frame_counted_ev(rfx_renderer *r, const rfx_frame *f, uint32_t nslices,
                                           const uint32_t *d_blk_counts, float *d_rgb, uint32_t *d_argb,
                                           uint64_t *d_counters, void *stream, void *emitted_event)
{
  FramePlan pl;
  int rc;
  if ((rc = plan_frame(r, f, stream, pl)) != RFX_OK) return rc;
  if (!d_rgb || !d_blk_counts || !nslices) return fail(RFX_ERR_ARG, "render_frame_counted: bad args");
  if (pl.traces == 0) return RFX_OK;
  const uint64_t nblk = rng_layout(pl.traces, nslices, nullptr);
  if ((rc = ensure_rng_workspace(r, pl.rd_traces(), nblk)) != RFX_OK) return rc;
  if ((rc = timing_start(r, pl.st)) != RFX_OK) return rc;
  return finish_frame(r, pl, d_blk_counts, nullptr, nblk, d_rgb, d_argb, d_counters, (hipEvent_t)emitted_event);
}

// What an emitted frame's randDirs depend on: the traces and their band, and the frame geometry that maps pixels to
// trace indices.  rfx_render_frame_emitted refuses a frame whose plan differs (its rows' randDirs were never written).
static void plan_key(const FramePlan &pl, uint64_t key[10])
{
  const FrameParams &P = pl.P;
  key[0] = pl.traces;
  key[1] = pl.band_lo;
  key[2] = pl.band_hi;
  key[3] = ((uint64_t)P.W << 32) | P.H;
  key[4] = ((uint64_t)(uint32_t)P.ss << 32) | P.row_block;
  key[5] = ((uint64_t)P.rank << 32) | P.nranks;
  key[6] = ((uint64_t)P.row0 << 32) | P.grid_rows;
  key[7] = P.p_begin;  // the span and its first trace index in words of their own: no two spans share a key
  key[8] = P.p_end;
  key[9] = P.trace_base;
}

// Emit-ahead (multi-GPU): the emit of frame i + 1 on a side stream while frame i traces.  Two randDir buffers: an emit
// writes the one the last enqueued trace does not read, and the next rfx_render_frame_emitted traces from it.
extern "C" int rfx_frame_rng_emit(rfx_renderer *r, const rfx_frame *f, uint32_t nslices, const uint32_t *d_blk_counts,
                                  void *stream, void *emitted_event)
{
  FramePlan pl;
  int rc;
  if ((rc = plan_frame(r, f, stream, pl)) != RFX_OK) return rc;
  if (!d_blk_counts || !nslices) return fail(RFX_ERR_ARG, "frame_rng_emit: bad args");
  if (r->emit_pending >= 0) return fail(RFX_ERR_STATE, "frame_rng_emit: the last emitted frame has not been traced");
  if (pl.traces == 0) return RFX_OK;
  const uint64_t nblk = rng_layout(pl.traces, nslices, nullptr);
  if ((rc = ensure_rng_workspace(r, pl.rd_traces(), nblk)) != RFX_OK) return rc;
  if ((rc = ensure_rd_alt(r, pl.rd_traces())) != RFX_OK) return rc;
  const int buf = r->trace_buf == 0 ? 1 : 0;  // not the buffer of the last enqueued trace
  // nor one a split frame's spans on the renderer's second stream may still read (the emit may run on a third stream)
  if (buf == 1 && r->split_alt_busy) HIP_CHECK(hipStreamWaitEvent(pl.st, r->split_ev[2], 0));
  r->split_alt_busy = false;
  if ((rc = emit_frame(r, pl, d_blk_counts, nullptr, nblk, buf ? r->d_rd_alt : r->d_rd,
                       (hipEvent_t)emitted_event)) != RFX_OK)
    return rc;
  r->emit_pending = buf;
  plan_key(pl, r->emit_key);
  return RFX_OK;
}

extern "C" int rfx_render_frame_emitted(rfx_renderer *r, const rfx_frame *f, float *d_rgb, uint32_t *d_argb,
                                        uint64_t *d_counters, void *stream)
{
  FramePlan pl;
  int rc;
  if ((rc = plan_frame(r, f, stream, pl)) != RFX_OK) return rc;
  if (!d_rgb) return fail(RFX_ERR_ARG, "render_frame_emitted: null framebuffer");
  if (pl.traces == 0) return RFX_OK;
  if (r->emit_pending < 0) return fail(RFX_ERR_STATE, "render_frame_emitted: no emitted frame (rfx_frame_rng_emit)");
  uint64_t key[10];
  plan_key(pl, key);
  if (memcmp(key, r->emit_key, sizeof(key)) != 0)
    return fail(RFX_ERR_STATE, "render_frame_emitted: the frame differs from the emitted one (band, geometry or traces); "
                               "rfx_frame_rng_discard it first");
  const int buf = r->emit_pending;
  r->emit_pending = -1;
  r->trace_buf = buf;
  if ((rc = timing_start(r, pl.st)) != RFX_OK) return rc;  // (the emit ran on its own stream: no pre-pass time)
  if ((rc = timing_event(r, pl.st)) != RFX_OK) return rc;
  return trace_frame(r, pl, buf ? r->d_rd_alt : r->d_rd, d_rgb, d_argb, d_counters);
}

// Forget an emitted, untraced frame: the stream state returns to before it (the emit read one state word and wrote
// the other, so flipping back restores it).
extern "C" int rfx_frame_rng_discard(rfx_renderer *r)
{
  if (!r) return fail(RFX_ERR_ARG, "frame_rng_discard: null renderer");
  r->rewind_ok = false;
  if (r->emit_pending >= 0)
  {
    r->seed_idx ^= 1u;
    ++r->state_seq;
    r->emit_pending = -1;
  }
  return RFX_OK;
}

extern "C" int rfx_frame_rng_pending(rfx_renderer *r, uint32_t *frame_start)
{
  if (!r || !frame_start) return fail(RFX_ERR_ARG, "frame_rng_pending: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  // an emitted frame read the state word it left behind (emit_frame flipped seed_idx past it)
  const uint32_t *w = r->emit_pending >= 0 ? r->d_seed + (r->seed_idx ^ 1u) : seed_cur(r);
  HIP_CHECK(hipMemcpyAsync(frame_start, w, sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  return r->emit_pending >= 0 ? 1 : 0;
}

static int render_split(rfx_renderer *r, const rfx_frame *f, uint64_t p0, uint64_t p1, float *d_rgb, uint32_t *d_argb,
                        uint64_t *d_counters, void *stream);

extern "C" int rfx_render_frame(rfx_renderer *r, const rfx_frame *f, float *d_rgb, uint32_t *d_argb,
                                uint64_t *d_counters, void *stream)
{
  FramePlan pl;
  int rc;
  if (!d_rgb) return fail(RFX_ERR_ARG, "render_frame: null framebuffer");
  if (r && f && f->sample_num > 0 && f->sample_num <= 256 && f->nranks <= 1 && f->width && f->height)
  {
    // a span of more traces than one launch takes: consecutive pixel spans (Render.cpp:136-215 walks the same cursor)
    const uint64_t npx = (uint64_t)f->width * f->height;
    const uint64_t p0 = f->pixel_begin, p1 = (f->pixel_begin == 0 && f->pixel_end == 0) ? npx : f->pixel_end;
    if (p0 < p1 && p1 <= npx && (p1 - p0) * (uint64_t)(f->sample_num * f->sample_num) > r->launch_traces)
      return render_split(r, f, p0, p1, d_rgb, d_argb, d_counters, stream);
  }
  if ((rc = plan_frame(r, f, stream, pl)) != RFX_OK) return rc;
  const uint32_t jitter0 = r->jitter_seed;
  r->rewind_saved = false;
  if (pl.traces == 0)  // a span with no block corner traces nothing (and draws no randDir)
  {
    r->rewind_ok = true;
    r->rewind_flip = false;
    r->rewind_jitter = jitter0;
    return RFX_OK;
  }
  const uint64_t nblk = rng_layout(pl.traces, 1, nullptr);
  if ((rc = ensure_rng_workspace(r, pl.traces, nblk)) != RFX_OK) return rc;
  if ((rc = timing_start(r, pl.st)) != RFX_OK) return rc;
  if (r->emit_pending >= 0)
    return fail(RFX_ERR_STATE, "render_frame: an emitted frame awaits rfx_render_frame_emitted (or rfx_frame_rng_discard)");
  if (fused_prepass(pl, nblk))
  {
    if ((rc = prepass_fused(r, pl, nblk, r->d_rd, nullptr)) != RFX_OK) return rc;
    r->trace_buf = 0;
    if ((rc = timing_event(r, pl.st)) != RFX_OK) return rc;
    if ((rc = trace_frame(r, pl, r->d_rd, d_rgb, d_argb, d_counters)) != RFX_OK) return rc;
  }
  else
  {
    // one device counts every block, so the emit can take its accept flags instead of regenerating them
    HIP_CHECK(launch_rng_count(seed_cur(r), r->d_jump, r->d_blk_cnt, 0, nblk, r->d_rng_masks, pl.st));
    if ((rc = finish_frame(r, pl, r->d_blk_cnt, r->d_rng_masks, nblk, d_rgb, d_argb, d_counters)) != RFX_OK) return rc;
  }
  r->rewind_ok = true;
  r->rewind_flip = true;
  r->rewind_jitter = jitter0;
  return RFX_OK;
}

// The stream state a frame of several launches starts from, kept in d_seed[2] for rfx_frame_rng_rewind (the seed words
// ping-pong once per launch, so flipping back would restore only the last span's start).
static int save_rewind_state(rfx_renderer *r, hipStream_t st)
{
  HIP_CHECK(hipMemcpyAsync(r->d_seed + 2, seed_cur(r), sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  return RFX_OK;
}

// Pixel spans [p0, p1) of more than r->launch_traces traces: launches of at most that many traces each, whole rows where
// a row fits.  Span k runs on the caller's stream (k even) or the renderer's split stream (k odd) with its randDirs in
// d_rd / d_rd_alt; its pre-pass waits for span k - 1's emit, whose end state it starts from, so span k's trace overlaps
// span k - 1's tail.  Every span is a cursor span of the reference's loop: trace indices and the additive jitter run
// from the span's first pixel (Render.cpp:136-215), so the pixels and both streams equal one launch over [p0, p1).
static int render_split(rfx_renderer *r, const rfx_frame *f, uint64_t p0, uint64_t p1, float *d_rgb, uint32_t *d_argb,
                        uint64_t *d_counters, void *stream)
{
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  if (r->emit_pending >= 0)
    return fail(RFX_ERR_STATE, "render_frame: an emitted frame awaits rfx_render_frame_emitted (or rfx_frame_rng_discard)");
  const uint64_t W = f->width, spp = (uint64_t)(f->sample_num * f->sample_num);
  uint64_t per = std::max<uint64_t>(1, r->launch_traces / spp);  // pixels per launch
  const bool rows = per >= W;
  if (rows) per = per / W * W;
  const uint64_t cap = per * spp;
  const hipStream_t st[2] = {stream ? (hipStream_t)stream : r->stream, nullptr};
  if (!r->split_stream) HIP_CHECK(hipStreamCreateWithFlags(&r->split_stream, hipStreamNonBlocking));
  for (hipEvent_t &e : r->split_ev)
    if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipStream_t s2[2] = {st[0], r->split_stream};
  // workspaces for the largest span before any launch (no re-allocation while spans are in flight)
  if ((rc = ensure_rng_workspace(r, cap, rng_layout(cap, 1, nullptr))) != RFX_OK) return rc;
  if ((rc = ensure_rd_alt(r, cap)) != RFX_OK) return rc;
  const uint32_t jitter0 = r->jitter_seed;
  if ((rc = save_rewind_state(r, s2[0])) != RFX_OK) return rc;
  // the split stream starts after the caller's earlier work (its first span also waits for span 0's emit)
  HIP_CHECK(hipEventRecord(r->split_ev[2], s2[0]));
  HIP_CHECK(hipStreamWaitEvent(s2[1], r->split_ev[2], 0));
  uint64_t k = 0;
  for (uint64_t a = p0; a < p1; ++k)
  {
    const uint64_t b = std::min(p1, rows ? (a / W) * W + per : a + per);
    rfx_frame fk = *f;
    fk.pixel_begin = a;
    fk.pixel_end = b;
    const int side = RFX_SPLIT_STREAMS > 1 ? (int)(k & 1) : 0;
    FramePlan pl;
    if ((rc = plan_frame(r, &fk, s2[side], pl)) != RFX_OK) return rc;
    pl.split = true;
    pl.split_side = side;
    const uint64_t nblk = rng_layout(pl.traces, 1, nullptr);
    if (k > 0) HIP_CHECK(hipStreamWaitEvent(s2[side], r->split_ev[side ^ 1], 0));  // span k - 1's end state
    if ((rc = timing_start(r, pl.st)) != RFX_OK) return rc;
    uint32_t *rd = side ? r->d_rd_alt : r->d_rd;
    if (fused_prepass(pl, nblk))
    {
      if ((rc = prepass_fused(r, pl, nblk, rd, r->split_ev[side])) != RFX_OK) return rc;
    }
    else
    {
      HIP_CHECK(launch_rng_count(seed_cur(r), r->d_jump, r->d_blk_cnt, 0, nblk, r->d_rng_masks, pl.st));
      if ((rc = emit_frame(r, pl, r->d_blk_cnt, r->d_rng_masks, nblk, rd, r->split_ev[side])) != RFX_OK) return rc;
    }
    if ((rc = timing_event(r, pl.st)) != RFX_OK) return rc;
    if ((rc = trace_frame(r, pl, rd, d_rgb, d_argb, d_counters)) != RFX_OK) return rc;
    a = b;
  }
  // the caller's stream continues after every span
  if (k > 1)
  {
    HIP_CHECK(hipEventRecord(r->split_ev[2], s2[1]));
    HIP_CHECK(hipStreamWaitEvent(s2[0], r->split_ev[2], 0));
  }
  r->trace_buf = 0;            // the last span on the caller's stream read d_rd; the odd spans read d_rd_alt until
  r->split_alt_busy = k > 1;   // split_ev[2], which the next emit-ahead into d_rd_alt waits for
  r->rewind_ok = true;
  r->rewind_flip = false;
  r->rewind_saved = true;
  r->rewind_stream = s2[0];
  r->rewind_jitter = jitter0;
  return RFX_OK;
}

// Undo the random-stream advance of the last rfx_render_frame (its pixels stay as written): the pre-pass read the
// frame's start state from one seed word and wrote the end state to the other, so flipping back restores the start
// (a frame of several launches: its start state is copied back from d_seed[2]).
extern "C" int rfx_frame_rng_rewind(rfx_renderer *r)
{
  if (!r) return fail(RFX_ERR_ARG, "frame_rng_rewind: null renderer");
  if (!r->rewind_ok) return fail(RFX_ERR_STATE, "frame_rng_rewind: the last call was not rfx_render_frame");
  if (r->rewind_flip) r->seed_idx ^= 1u;
  ++r->state_seq;
  if (r->rewind_saved)
  {
    int rc;
    if ((rc = set_dev(r)) != RFX_OK) return rc;
    HIP_CHECK(hipMemcpyAsync(seed_cur(r), r->d_seed + 2, sizeof(uint32_t), hipMemcpyDeviceToDevice, r->rewind_stream));
    ++r->state_seq;
  }
  r->jitter_seed = r->rewind_jitter;
  r->rewind_ok = false;
  r->rewind_saved = false;
  return RFX_OK;
}

static int plan_frame(rfx_renderer *r, const rfx_frame *f, void *stream, FramePlan &plan)
{
  if (!r || !f) return fail(RFX_ERR_ARG, "render_frame: bad args");
  if (!r->has_scene) return fail(RFX_ERR_STATE, "render_frame: no scene uploaded");
  r->rewind_ok = false;  // every render path moves on from the last rfx_render_frame
  if (!f->width || !f->height || f->reflect_num <= 0 || f->sample_num == 0)
    return fail(RFX_ERR_ARG, "render_frame: W=%u H=%u reflect_num=%d sample_num=%d", f->width, f->height,
                f->reflect_num, f->sample_num);
  const uint32_t nranks = f->nranks ? f->nranks : 1;
  const bool band = nranks > 1 && !f->row_block;  // band partition: this rank's rows [pixel_begin, pixel_end) / W
  if (nranks > 1 && (f->sample_num < 0 || f->rank >= nranks))
    return fail(RFX_ERR_ARG, "render_frame: a partition needs sample_num > 0, rank < nranks");
  if (f->sample_num > 256 || f->sample_num < -4096) return fail(RFX_ERR_ARG, "render_frame: sample_num out of range");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  hipStream_t st = stream ? (hipStream_t)stream : r->stream;

  const uint32_t W = f->width, H = f->height;
  const uint64_t npx = (uint64_t)W * H;
  uint64_t p0 = f->pixel_begin, p1 = f->pixel_end;
  if (band)
  {
    // the band's rows; the random stream and the trace indices run over the span [span_begin, span_end) of whole rows
    // (the whole W x H frame by default), output rows stay the frame's
    const uint64_t s0 = f->span_begin, s1 = (f->span_begin == 0 && f->span_end == 0) ? npx : f->span_end;
    if (p0 >= p1 || p1 > npx || p0 % W || p1 % W)
      return fail(RFX_ERR_ARG, "render_frame: a band is whole rows [pixel_begin, pixel_end) / W of the frame");
    if (s0 >= s1 || s1 > npx || s0 % W || s1 % W || p0 < s0 || p1 > s1)
      return fail(RFX_ERR_ARG, "render_frame: a band's span is whole rows [span_begin, span_end) / W around the band");
    plan.band = true;
    plan.band_lo = (p0 - s0) * (uint64_t)(f->sample_num * f->sample_num);
    plan.band_hi = (p1 - s0) * (uint64_t)(f->sample_num * f->sample_num);
    p0 = s0;
    p1 = s1;
  }
  if (p0 == 0 && p1 == 0) p1 = npx;
  if (p0 >= p1 || p1 > npx) return fail(RFX_ERR_ARG, "render_frame: pixel span [%llu, %llu) outside frame",
                                        (unsigned long long)p0, (unsigned long long)p1);
  if (nranks > 1 && !band && (p0 != 0 || p1 != npx)) return fail(RFX_ERR_ARG, "render_frame: strips need the whole frame");
  const uint32_t y0 = (uint32_t)(p0 / W), y1 = (uint32_t)((p1 - 1) / W);
  uint64_t traces, trace_base = 0;
  uint32_t grid_rows, row0;
  if (f->sample_num < 0)
  {
    // block preview: corners (x % n == 0 && y % n == 0) inside the span, in raster order (Render.cpp:158-172)
    const uint64_t n = (uint64_t)(-f->sample_num);
    const uint64_t bw = (W + n - 1) / n;
    auto corners_before = [&](uint64_t p) -> uint64_t {
      const uint64_t y = p / W, x = p % W;
      return (y + n - 1) / n * bw + (y % n == 0 ? (x + n - 1) / n : 0);
    };
    trace_base = corners_before(p0);
    traces = corners_before(p1) - trace_base;
    row0 = (uint32_t)(y0 / n);
    grid_rows = (uint32_t)(y1 / n - y0 / n + 1);
  }
  else
  {
    traces = (p1 - p0) * (uint64_t)(f->sample_num * f->sample_num);
    row0 = nranks > 1 ? 0 : y0;
    grid_rows = nranks > 1 ? rfx_strip_rows(H, f->row_block, f->rank, nranks) : y1 - y0 + 1;
    if (band)
    {
      row0 = (uint32_t)(f->pixel_begin / W);
      grid_rows = (uint32_t)((f->pixel_end - f->pixel_begin) / W);
    }
  }
  // one launch (rfx_render_frame splits larger spans before planning them; a band's span must stay within this)
  if (traces > kMaxLaunchTraces)
    return fail(RFX_ERR_ARG, "render_frame: %llu traces in one launch exceed 2^31 (partitions: a smaller span)",
                (unsigned long long)traces);
  plan.traces = traces;
  plan.st = st;
  FrameParams &P = plan.P;
  P = FrameParams{};
  P.eye_x = f->eye[0]; P.eye_y = f->eye[1]; P.eye_z = f->eye[2];
  P.v11 = f->view[0]; P.v12 = f->view[1]; P.v13 = f->view[2];
  P.v21 = f->view[3]; P.v22 = f->view[4]; P.v23 = f->view[5];
  P.v31 = f->view[6]; P.v32 = f->view[7]; P.v33 = f->view[8];
  P.rz = rfx_camera_rz(W, f->fov);
  P.wh = W / 2.0f;
  P.hh = H / 2.0f;
  P.W = W; P.H = H;
  P.depth = f->reflect_num;
  P.ss = f->sample_num;
  P.accumulate = f->sample_num > 0 && f->additive_counter > 1;
  P.additive = f->sample_num > 0 && f->additive;
  P.jitter_seed = r->jitter_seed;
  P.row_block = f->row_block ? f->row_block : 1;
  P.rank = nranks > 1 && !band ? f->rank : 0;
  P.nranks = band ? 1 : nranks;  // a band traces like a 1-GPU span of rows: absolute rows, whole-frame buffers
  P.grid_rows = grid_rows;
  P.row0 = row0;
  P.p_begin = p0;
  P.p_end = p1;
  P.trace_base = trace_base;
  return RFX_OK;
}

extern "C" int rfx_device_alloc(rfx_renderer *r, size_t bytes, void **p)
{
  if (!r || !p) return fail(RFX_ERR_ARG, "device_alloc: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  HIP_CHECK(hipMalloc(p, bytes ? bytes : 1));
  return RFX_OK;
}

extern "C" int rfx_device_free(rfx_renderer *r, void *p)
{
  if (!r) return fail(RFX_ERR_ARG, "device_free: null renderer");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  HIP_CHECK(hipFree(p));
  return RFX_OK;
}

extern "C" int rfx_memcpy_d2h(rfx_renderer *r, void *dst, const void *src, size_t n)
{
  if (!r) return fail(RFX_ERR_ARG, "memcpy: null renderer");
  HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  return RFX_OK;
}

extern "C" int rfx_memcpy_d2d(rfx_renderer *r, void *dst, const void *src, size_t n)
{
  if (!r || (n && (!dst || !src))) return fail(RFX_ERR_ARG, "memcpy_d2d: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  if (n) HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, r->stream));
  return RFX_OK;
}

extern "C" int rfx_memcpy_h2d(rfx_renderer *r, void *dst, const void *src, size_t n)
{
  if (!r) return fail(RFX_ERR_ARG, "memcpy: null renderer");
  HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  return RFX_OK;
}

extern "C" int rfx_synchronize(rfx_renderer *r)
{
  if (!r) return fail(RFX_ERR_ARG, "synchronize: null renderer");
  HIP_CHECK(hipStreamSynchronize(r->stream));
  int err = 0;
  HIP_CHECK(hipMemcpy(&err, r->d_err, sizeof(int), hipMemcpyDeviceToHost));
  if (err & 1) return fail(RFX_ERR_RNG, "RNG pre-pass ran short of accepted triples");  // (bit 4: an exact fallback)
  return RFX_OK;
}

extern "C" int rfx_render_frame_host(rfx_renderer *r, const rfx_frame *f, float *rgb, uint32_t *argb_out,
                                     uint64_t *counters)
{
  if (!r || !f || !rgb) return fail(RFX_ERR_ARG, "render_frame_host: bad args");
  if (f->nranks > 1) return fail(RFX_ERR_ARG, "render_frame_host: whole frames only");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  const size_t px = (size_t)f->width * f->height;
  if (px > r->img_cap)
  {
    (void)hipFree(r->d_img); (void)hipFree(r->d_argb);
    r->d_img = nullptr; r->d_argb = nullptr; r->img_cap = 0;
    HIP_CHECK(hipMalloc(&r->d_img, px * 3 * sizeof(float)));
    HIP_CHECK(hipMalloc(&r->d_argb, px * sizeof(uint32_t)));
    r->img_cap = px;
  }
  if (!r->d_cnt) HIP_CHECK(hipMalloc(&r->d_cnt, RFX_NCOUNTERS * sizeof(uint64_t)));
  HIP_CHECK(hipMemcpyAsync(r->d_img, rgb, px * 3 * sizeof(float), hipMemcpyHostToDevice, r->stream));
  if (counters) HIP_CHECK(hipMemsetAsync(r->d_cnt, 0, RFX_NCOUNTERS * sizeof(uint64_t), r->stream));
  if ((rc = rfx_render_frame(r, f, r->d_img, argb_out ? r->d_argb : nullptr, counters ? r->d_cnt : nullptr, nullptr)))
    return rc;
  HIP_CHECK(hipMemcpyAsync(rgb, r->d_img, px * 3 * sizeof(float), hipMemcpyDeviceToHost, r->stream));
  if (argb_out) HIP_CHECK(hipMemcpyAsync(argb_out, r->d_argb, px * sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
  if (counters)
  {
    uint64_t c[RFX_NCOUNTERS];
    HIP_CHECK(hipMemcpyAsync(c, r->d_cnt, sizeof(c), hipMemcpyDeviceToHost, r->stream));
    HIP_CHECK(hipStreamSynchronize(r->stream));
    for (int k = 0; k < RFX_NCOUNTERS; ++k) counters[k] += c[k];
  }
  return rfx_synchronize(r);
}

extern "C" int rfx_rand_dirs(rfx_renderer *r, uint32_t seed, uint64_t n, float *out3, uint32_t *seed_out)
{
  if (!r || !out3 || !n) return fail(RFX_ERR_ARG, "rand_dirs: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  uint32_t saved = 0;
  HIP_CHECK(hipMemcpyAsync(&saved, seed_cur(r), sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
  HIP_CHECK(hipStreamSynchronize(r->stream));
  HIP_CHECK(hipMemcpyAsync(seed_cur(r), &seed, sizeof(uint32_t), hipMemcpyHostToDevice, r->stream));
  if ((rc = enqueue_rng(r, n, r->stream)) != RFX_OK) return rc;
  std::vector<uint32_t> states(n);
  HIP_CHECK(hipMemcpyAsync(states.data(), r->d_rd, n * sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
  uint32_t after = 0;
  HIP_CHECK(hipMemcpyAsync(&after, seed_cur(r), sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));  // flipped
  HIP_CHECK(hipMemcpyAsync(seed_cur(r), &saved, sizeof(uint32_t), hipMemcpyHostToDevice, r->stream));
  if ((rc = rfx_synchronize(r)) != RFX_OK) return rc;
  for (uint64_t i = 0; i < n; ++i)  // Vector3.cpp:182-184 from each trace's state
  {
    const uint32_t s1 = lcg_step(states[i]), s2 = lcg_step(s1), s3 = lcg_step(s2);
    out3[i * 3] = rand_component(lcg_out(s1));
    out3[i * 3 + 1] = rand_component(lcg_out(s2));
    out3[i * 3 + 2] = rand_component(lcg_out(s3));
  }
  if (seed_out) *seed_out = after;
  return RFX_OK;
}

// ============================================================== device known-answer entry points
// Each runs the trace kernel's own device code (rfx_kernels.hip kat_*) on host arrays, synchronously.
template <class T>
static int kat_buffer(size_t n, const T *src, T **dev)
{
  *dev = nullptr;
  HIP_CHECK(hipMalloc((void **)dev, n ? n * sizeof(T) : sizeof(T)));
  if (src && n) HIP_CHECK(hipMemcpy(*dev, src, n * sizeof(T), hipMemcpyHostToDevice));
  return RFX_OK;
}

static int kat_run(rfx_renderer *r, int what, int tex, const void *in, size_t in_elems, const int32_t *objs,
                   uint64_t n, void *out, size_t out_elems)
{
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  if (n >= (1ull << 31)) return fail(RFX_ERR_ARG, "kat: n too large");
  float *d_in = nullptr, *d_out = nullptr;
  int32_t *d_obj = nullptr;
  rc = kat_buffer(in_elems, (const float *)in, &d_in);
  if (rc == RFX_OK && objs) rc = kat_buffer((size_t)n, objs, &d_obj);
  if (rc == RFX_OK) rc = kat_buffer(out_elems, (const float *)nullptr, &d_out);
  if (rc == RFX_OK)
  {
    hipError_t e = launch_kat(what, r->dev, tex, d_in, d_obj, (uint32_t)n, d_out, r->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d_out, out_elems * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(RFX_ERR_HIP, "kat: %s", hipGetErrorString(e));
  }
  (void)hipFree(d_in); (void)hipFree(d_obj); (void)hipFree(d_out);
  return rc;
}

extern "C" int rfx_kat_objects(rfx_renderer *r, const float *rays, const int32_t *objects, uint64_t n, float *out)
{
  if (!r || (n && (!rays || !objects || !out))) return fail(RFX_ERR_ARG, "kat_objects: bad args");
  if (!r->has_scene) return fail(RFX_ERR_STATE, "kat_objects: no scene uploaded");
  for (uint64_t i = 0; i < n; ++i)
    if (objects[i] < 0 || objects[i] >= r->dev.n_obj) return fail(RFX_ERR_ARG, "kat_objects: object %d", objects[i]);
  return kat_run(r, 0, 0, rays, (size_t)n * 6, objects, n, out, (size_t)n * 15);
}

extern "C" int rfx_kat_texels(rfx_renderer *r, int texture, const float *in, uint64_t n, float *out)
{
  if (!r || (n && (!in || !out))) return fail(RFX_ERR_ARG, "kat_texels: bad args");
  if (!r->has_scene) return fail(RFX_ERR_STATE, "kat_texels: no scene uploaded");
  if (texture >= r->dev.n_tex) return fail(RFX_ERR_ARG, "kat_texels: texture %d", texture);
  return kat_run(r, 1, texture, in, (size_t)n * (texture >= 0 ? 2 : 3), nullptr, n, out, (size_t)n * 3);
}

extern "C" int rfx_kat_powf(rfx_renderer *r, const float *xy, uint64_t n, float *out)
{
  if (!r || (n && (!xy || !out))) return fail(RFX_ERR_ARG, "kat_powf: bad args");
  return kat_run(r, 2, 0, xy, (size_t)n * 2, nullptr, n, out, (size_t)n);
}

extern "C" int rfx_kat_powf_cube(rfx_renderer *r, uint64_t counts[2])
{
  if (!r || !counts) return fail(RFX_ERR_ARG, "kat_powf_cube: bad args");
  unsigned long long *d = nullptr;
  hipError_t e = hipMalloc(&d, 2 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, 2 * sizeof(unsigned long long), r->stream);
  // every float in [0, 1]: bit patterns 0 .. 0x3f800000, in launches of 2^28
  for (uint64_t first = 0; e == hipSuccess && first <= 0x3f800000ull; first += 1ull << 28)
    e = launch_kat_powf_cube((uint32_t)first, (uint32_t)std::min<uint64_t>(1ull << 28, 0x3f800001ull - first), d, r->stream);
  unsigned long long h[2] = {0, 0};
  if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RFX_ERR_HIP, "kat_powf_cube: %s", hipGetErrorString(e));
  counts[0] = h[0];
  counts[1] = h[1];
  return RFX_OK;
}

extern "C" int rfx_kat_div(rfx_renderer *r, uint64_t first, uint64_t n, uint64_t counts[3])
{
  if (!r || !counts) return fail(RFX_ERR_ARG, "kat_div: bad args");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  unsigned long long *d = nullptr;
  hipError_t e = hipMalloc(&d, 3 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemsetAsync(d, 0, 3 * sizeof(unsigned long long), r->stream);
  for (uint64_t k = 0; e == hipSuccess && k < n; k += 1ull << 28)  // launches of up to 2^28 pairs
    e = launch_kat_div(first + k, (uint32_t)std::min<uint64_t>(1ull << 28, n - k), d, r->stream);
  unsigned long long h[3] = {0, 0, 0};
  if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RFX_ERR_HIP, "kat_div: %s", hipGetErrorString(e));
  for (int i = 0; i < 3; ++i) counts[i] = h[i];
  return RFX_OK;
}

extern "C" int rfx_kat_argb(rfx_renderer *r, const float *rgb, uint64_t n, uint32_t *out)
{
  if (!r || (n && (!rgb || !out))) return fail(RFX_ERR_ARG, "kat_argb: bad args");
  return kat_run(r, 3, 0, rgb, (size_t)n * 3, nullptr, n, out, (size_t)n);
}

extern "C" int rfx_kat_kernarg(rfx_renderer *r, int swapped, uint32_t out[3])
{
  if (!r || !out) return fail(RFX_ERR_ARG, "kat_kernarg: bad args");
  if (!r->has_scene) return fail(RFX_ERR_STATE, "kat_kernarg: no scene uploaded");
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  FrameParams P;
  uint32_t *w = (uint32_t *)&P;  // every word distinct, so a shifted read cannot match by accident
  for (size_t i = 0; i < sizeof(P) / 4; ++i) w[i] = 0x9E3779B9u * (uint32_t)(i + 1);
  uint32_t *d = nullptr;
  hipError_t e = hipMalloc(&d, 3 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(d, 0xFF, 3 * sizeof(uint32_t), r->stream);
  if (e == hipSuccess) e = launch_kat_kernarg(r->dev, P, swapped, d, r->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
  if (e == hipSuccess) e = hipMemcpy(out, d, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RFX_ERR_HIP, "kat_kernarg: %s", hipGetErrorString(e));
  return RFX_OK;
}

// ============================================================== internals shared with rfx_group.cpp (rfx_internal.h)
int rfx_detail_fail(int code, const char *msg) { return fail(code, "%s", msg); }
uint32_t *rfx_detail_seed_word(rfx_renderer *r) { return seed_cur(r); }
uint32_t rfx_detail_jitter(const rfx_renderer *r) { return r->jitter_seed; }
void rfx_detail_set_jitter(rfx_renderer *r, uint32_t jitter) { r->jitter_seed = jitter; }
hipStream_t rfx_detail_stream(const rfx_renderer *r) { return r->stream; }
// the last call on r was a counted frame (one pre-pass flip, jitter advanced from jitter0): rfx_frame_rng_rewind
// may undo it, as after rfx_render_frame
void rfx_detail_set_rewindable(rfx_renderer *r, uint32_t jitter0)
{
  r->rewind_ok = true;
  r->rewind_flip = true;
  r->rewind_saved = false;
  r->rewind_jitter = jitter0;
}
int rfx_detail_save_start(rfx_renderer *r, hipStream_t st)
{
  int rc;
  if ((rc = set_dev(r)) != RFX_OK) return rc;
  return save_rewind_state(r, st);
}
void rfx_detail_set_rewindable_saved(rfx_renderer *r, uint32_t jitter0, hipStream_t st)
{
  r->rewind_ok = true;
  r->rewind_flip = false;
  r->rewind_saved = true;
  r->rewind_stream = st;
  r->rewind_jitter = jitter0;
}
uint64_t rfx_detail_launch_traces(const rfx_renderer *r) { return r->launch_traces; }
uint64_t rfx_detail_state_seq(const rfx_renderer *r) { return r->state_seq; }
