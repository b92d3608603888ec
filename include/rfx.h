/*
 * rfx.h -- C-ABI of the MI355X-native ReflaxMan trace loop (librfx.so).
 *
 * The reference has no plugin/FFI layer: its path sits behind the C++ class API
 * of Render (src/common/Render.h:7-42), Scene (Scene.h:28-40), Camera
 * (Camera.h:30-62), Material (Material.h:5-19), OmniLight and Texture.  Each
 * entry point below replaces one of those calls (cited per function) so a
 * host-side shim -- include/reflaxman/ (C++ headers), reflaxman_amd/render.py
 * (Python/ctypes), or the cgo/JNI/ctypes stubs in INTEGRATION.md -- can drop in
 * for the reference's CPU render() call.
 *
 * Conventions: plain pointers and sizes only; status codes (rfx_status) instead
 * of the reference's assert()+silent clamps; colours are float RGB; ARGB texels
 * are uint32 0xAARRGGBB; images are row-major, row 0 = bottom (the reference's
 * ry < 0 looks down, Render.cpp:146-156).  Device pointers are HIP device
 * memory of the renderer's device; `stream` arguments are hipStream_t (NULL =
 * the renderer's stream).
 */
#ifndef RFX_H
#define RFX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RFX_ABI_VERSION 3

typedef enum {
  RFX_OK = 0,
  RFX_ERR_ARG = -1,      /* invalid argument (reference: assert + clamp/fallback) */
  RFX_ERR_HIP = -2,      /* HIP runtime failure; rfx_last_error() has the text */
  RFX_ERR_STATE = -3,    /* call not valid in the current state */
  RFX_ERR_IO = -4,       /* file could not be read/written (reference returns false) */
  RFX_ERR_RNG = -5,      /* RNG pre-pass ran short of accepted triples (never expected) */
  RFX_ERR_NODEV = -6     /* no HIP device */
} rfx_status;

enum { RFX_METAL = 0, RFX_DIELECTRIC = 1 };  /* Material::Type (Material.h:8) */

typedef struct rfx_scene rfx_scene;
typedef struct rfx_renderer rfx_renderer;

int rfx_abi_version(void);
const char *rfx_last_error(void);
/* Compile-time options of this build (A/B variants, tools/ab.py), as bits: per-view chunk lists of large scenes
 * (RFX_PRIM_LARGE, off by default), per-view masks of per-pixel-loop SSAA frames (RFX_PRIM_SSAA, off), of the
 * one-lane-per-sample SSAA modes (RFX_PRIM_LANES, on), one-light kernel instantiations (RFX_ONE_LIGHT, on); bits 8-15:
 * sphere pairs per leaf of the large scenes' BVH. */
enum { RFX_BUILD_PRIM_LARGE = 1, RFX_BUILD_PRIM_SSAA = 2, RFX_BUILD_PRIM_LANES = 4, RFX_BUILD_ONE_LIGHT = 8 };
int rfx_build_options(void);

/* ---------------------------------------------------------------- Scene */
/* Scene(const Color & diffLightColor, float diffLightPower)  -- Scene.cpp:10-15 */
rfx_scene *rfx_scene_create(float diff_r, float diff_g, float diff_b, float diff_power);
void rfx_scene_destroy(rfx_scene *scene);
/* Scene::addSphere(center, radius, Material(type, color, reflectivity, transparency))
 *   -- Scene.cpp:29-39, Sphere.cpp:9-20, Material.cpp:8-14.  Returns the object index (>= 0). */
int rfx_scene_add_sphere(rfx_scene *scene, const float center[3], float radius, int material_type,
                         const float rgb[3], float reflectivity, float transparency);
/* Scene::addTriangle(v1, v2, v3, material) -- Scene.cpp:41-46, Triangle.cpp:11-21.  Returns the object index. */
int rfx_scene_add_triangle(rfx_scene *scene, const float v1[3], const float v2[3], const float v3[3],
                           int material_type, const float rgb[3], float reflectivity, float transparency);
/* Plane(pos, norm, material) -- Plane.cpp:9-14, traced by Plane::trace (Plane.cpp:36-73).  The reference's
 * Scene cannot hold a Plane (no addPlane); this is its natural extension: the plane takes an
 * object index in insertion order like any other object (closest-hit ties, shadow self-skip).  The normal is
 * used as given (the reference never normalises it).  Returns the object index. */
int rfx_scene_add_plane(rfx_scene *scene, const float pos[3], const float norm[3], int material_type,
                        const float rgb[3], float reflectivity, float transparency);
int rfx_scene_plane_count(const rfx_scene *scene);
/* Triangle::setTexture(texture, u1, v1, u2, v2, u3, v3) -- Triangle.cpp:110-120.  uv = {u1,v1,u2,v2,u3,v3}. */
int rfx_triangle_set_texture(rfx_scene *scene, int object_index, int texture_index, const float uv[6]);
/* Scene::addLight(origin, radius, color, power) -- Scene.cpp:48-59, OmniLight.cpp:8-14.  Returns the light index. */
int rfx_scene_add_light(rfx_scene *scene, const float origin[3], float radius, const float rgb[3], float power);
/* Scene::addTexture -- Scene.cpp:61-66, from memory: argb == NULL or w*h == 0 is the reference's failed
 * load (empty texture -> procedural checker, Texture.cpp:242-243).  Returns the texture index. */
int rfx_scene_add_texture_argb(rfx_scene *scene, uint32_t width, uint32_t height, const uint32_t *argb);
/* Scene::addTexture(fileName) -- TGA loader of Texture.cpp:34-108 (type 2, 24/32 bpp).  A file that does
 * not load yields an empty texture, as in the reference; *loaded (optional) reports success. */
int rfx_scene_add_texture_file(rfx_scene *scene, const char *path, int *loaded);
/* Scene::setSkyboxTexture(fileName) -- Scene.cpp:68-71, Skybox.cpp:21-37.  Returns 1 if loaded, 0 if not
 * (checker fallback, as the reference), < 0 on error. */
int rfx_scene_set_skybox_file(rfx_scene *scene, const char *path);
/* same, from memory (NULL -> checker) */
int rfx_scene_set_skybox_argb(rfx_scene *scene, uint32_t width, uint32_t height, const uint32_t *argb);
int rfx_scene_counts(const rfx_scene *scene, int *spheres, int *triangles, int *lights, int *textures);

/* ---------------------------------------------------------------- Camera */
/* Camera(eye, at, fov): view = [ox | oy | oz] columns, row-major _11.._33 -- Camera.cpp:24-38 */
void rfx_camera_view(const float eye[3], const float at[3], float view[9]);
/* rz = W / 2 / tanf(fov / 2) -- Render.cpp:148 (host libm tanf, as the reference) */
float rfx_camera_rz(uint32_t width, float fov);

/* ---------------------------------------------------------------- Images & files */
/* Texture::loadFromTGAFile -- Texture.cpp:34-108.  Call with argb == NULL to query w/h. */
int rfx_tga_load(const char *path, uint32_t *width, uint32_t *height, uint32_t *argb, size_t capacity);
/* Texture::saveToTGAFile / saveToBMPFile -- Texture.cpp:110-173 (32 bpp, rows as stored) */
int rfx_tga_save(const char *path, uint32_t width, uint32_t height, const uint32_t *argb);
int rfx_bmp_save(const char *path, uint32_t width, uint32_t height, const uint32_t *argb);
/* Color::argb over a host float RGB image (Color.cpp:114-117) -- Render::copyImage (Render.cpp:82-101) */
void rfx_argb_from_rgb(const float *rgb, size_t pixels, uint32_t *argb);

/* ---------------------------------------------------------------- Renderer (device) */
int rfx_renderer_create(rfx_renderer **out, int device);
void rfx_renderer_destroy(rfx_renderer *r);
int rfx_renderer_device(const rfx_renderer *r);
/* launches go to this stream (hipStream_t); NULL = a non-blocking stream the renderer owns (so work on the
 * legacy default stream is NOT ordered with it: callers that mix in their own work pass their stream) */
int rfx_renderer_set_stream(rfx_renderer *r, void *hip_stream);
/* upload the scene (host precompute already done by the builder calls) */
int rfx_renderer_set_scene(rfx_renderer *r, const rfx_scene *scene);
/* Trace-launch schedule (no effect on any pixel): 1 (default) = on launches of >= 65536 tiles (8x8 pixels,
 * one wave each; 3840x2160 has 129,600) waves take the tiles longest-first, in the order sorted from an
 * earlier launch's measured per-tile clock costs of the same grid (re-sorted every 4th launch; the first
 * launch, or one after a grid change, runs tiles in raster order); 3 = the same on every launch size;
 * 0 = raster order, no cost recording; 2 = raster order with cost recording (A/B of the sort's overhead).
 * Block-preview frames (sample_num < 0) always run in raster order. */
int rfx_renderer_set_tile_order(rfx_renderer *r, int mode);
/* Ray regrouping of plain one-sample frames (no pixel changes): a trace still alive after park_after bounce
 * segments is parked in an HBM queue and resumed by a second kernel whose lanes each take the next queued trace as
 * soon as theirs ends (lanes whose traces ended no longer idle in their tile's wave).  -1 (default) = after 2
 * segments on scenes with more than 32 spheres or triangles, off on small ones; 0 = off; n >= 1 = after n segments
 * on any scene. */
int rfx_renderer_set_regroup(rfx_renderer *r, int park_after);
/* regrouped frames: 1 = the parked traces are counting-sorted by direction octant and origin cell before the bounce
 * kernel takes them, 0 (default) = taken in park order (a tile's survivors together: faster on C5).
 * Changes the schedule, never a value. */
int rfx_renderer_set_regroup_sort(rfx_renderer *r, int on);
/* Which bounce kernel the last trace launch ran: 0 = none (not regrouped), 1 = the global-memory BVH form, 2 = the
 * LDS-staged BVH form (large scenes whose BVH fits the LDS; 1 when the runtime refused its LDS size). */
int rfx_renderer_bounce_form(const rfx_renderer *r);
/* Primary-bundle cull masks of small-scene plain frames and of SSAA frames run one sample per lane (sampleNum 2, 4,
 * 8, and jittered sampleNum 1) (no pixel changes): the first segment's cull masks of every wave tile, computed by one
 * extra launch for a view (camera, frame geometry, sampling, scene) and reused while the view stays.  1 (default) = built when a view repeats (the second frame of a still camera on), so a camera that
 * moves every frame never pays for them; 2 = built before every launch; 0 = off (per-launch bundles).  SSAA frames of
 * sampleNum > 8 (a wave per pixel) take one closest-hit mask per pixel, built for every view and every launch of a split
 * frame under 1 and 2.  Any call forgets the views seen so far. */
int rfx_renderer_set_prim_masks(rfx_renderer *r, int mode);
/* The reference's two LCG streams (trace_math.h:34-39): Vector3.cpp's (randomInsideSphere) and
 * Render.cpp's (additive jitter).  Both persist across frames exactly as the reference's would. */
int rfx_renderer_set_rng(rfx_renderer *r, uint32_t sphere_seed, uint32_t jitter_seed);
int rfx_renderer_get_rng(rfx_renderer *r, uint32_t *sphere_seed, uint32_t *jitter_seed); /* synchronises */

typedef struct {
  float eye[3];        /* Render::renderCameraEye  (Render.cpp:128) */
  float view[9];       /* Render::renderCameraView (Render.cpp:127), row-major */
  float fov;           /* Camera::fov -> rz = W/2/tanf(fov/2) (Render.cpp:148) */
  uint32_t width, height;
  int32_t reflect_num;      /* renderBegin reflectNum (> 0) */
  int32_t sample_num;       /* renderBegin sampleNum: >0 SSAA n x n, <0 |n| block preview, 0 invalid */
  int32_t additive;         /* renderBegin additive */
  int32_t additive_counter; /* Render::additiveCounter after renderBegin (Render.cpp:130-133) */
  uint32_t row_block;       /* strip partition: rows are dealt in blocks of row_block ...   */
  uint32_t rank, nranks;    /* ... block b belongs to rank b % nranks (nranks == 1: whole frame) */
  uint64_t pixel_begin;     /* raster span [pixel_begin, pixel_end) of this call: the Render::renderNext */
  uint64_t pixel_end;       /* cursor span (Render.cpp:136-215); 0, 0 = the whole frame.  nranks == 1, or a band */
  /* Band partition: nranks > 1 with row_block == 0 -- this rank traces the whole rows [pixel_begin, pixel_end) / W of
   * the W x H frame into whole-frame buffers (d_rgb W*H*3, d_argb W*H; only the band's rows are written), with the
   * frame's random stream sliced nranks ways as for strips (rfx_frame_rng_count / rfx_render_frame_counted).  Rank 0
   * can then receive each band straight into its rows of the frame (reflaxman_amd/dist.py BandFrame). */
  uint64_t span_begin;      /* band partition only: the random stream covers the whole rows [span_begin, span_end) / W */
  uint64_t span_end;        /* of the frame (0, 0 = the whole frame) and the band lies within them -- a frame of 2^32 */
                            /* traces or more is rendered as consecutive row spans (rfx_group_render_frame) */
} rfx_frame;

/* rows of `frame` that `rank` owns under the block-cyclic strip partition */
uint32_t rfx_strip_rows(uint32_t height, uint32_t row_block, uint32_t rank, uint32_t nranks);
/* global row of compact strip row `r` */
uint32_t rfx_strip_row_to_y(uint32_t r, uint32_t row_block, uint32_t rank, uint32_t nranks);

/*
 * One Render::renderBegin + renderNext(W*H) pass on the device (Render.cpp:116-215 + Scene::trace,
 * Scene.cpp:73-236): RNG pre-pass, trace kernel, ARGB epilogue, all stream-ordered, no host sync.
 *   d_rgb  : device float RGB, strip_rows x W x 3 (read-modify-write when additive_counter > 1)
 *   d_argb : device uint32, strip_rows x W, Color::argb of the stored value (copyImage), or NULL
 *   d_counters : device uint64[RFX_NCOUNTERS] accumulated event counters (stats kernel), or NULL
 * Any sample count (Pulse's menu reaches 7680x4320 at 256x256 samples, 2.2e12 traces): a span of more traces than the
 * launch limit (rfx_renderer_set_launch_traces) is rendered as consecutive pixel spans (whole rows where a row fits),
 * each its own pre-pass and trace launch, alternating between two streams so one span's tail overlaps the next span's
 * start; the random streams run on from span to span exactly as the reference's cursor does (Render.cpp:136-215).
 */
#define RFX_NCOUNTERS 40
int rfx_render_frame(rfx_renderer *r, const rfx_frame *frame, float *d_rgb, uint32_t *d_argb,
                     uint64_t *d_counters, void *stream);
/* The most traces one rfx_render_frame launch takes (default 2^30: 4 GB of randDir state per buffer, two buffers);
 * 0 = the default.  Splitting changes no pixel (tests/test_gpu_parity.py forces small limits). */
int rfx_renderer_set_launch_traces(rfx_renderer *r, uint64_t max_traces);

/*
 * Multi-GPU form of the RNG pre-pass, around ONE exchange step.  The trace-ordered
 * random stream is cut into nslices equal slices of LCG blocks; rank r counts the accepted triples of
 * slice r only (rfx_frame_rng_count), the per-block counts are all-gathered (RCCL: nslices *
 * blocks_per_slice uint32 on the device), and rfx_render_frame_counted scans them and emits only the
 * randDirs of this rank's strips before tracing them.  Every rank also carries the stream state past
 * the frame's last trace, so the next frame starts where the reference's would.  rfx_render_frame is
 * the same with nslices = 1 and every block counted locally.
 */
int rfx_frame_rng_blocks(rfx_renderer *r, const rfx_frame *frame, uint32_t nslices, uint64_t *blocks_per_slice);
int rfx_frame_rng_count(rfx_renderer *r, const rfx_frame *frame, uint32_t slice, uint32_t nslices,
                        uint32_t *d_blk_counts, void *stream);
int rfx_render_frame_counted(rfx_renderer *r, const rfx_frame *frame, uint32_t nslices, const uint32_t *d_blk_counts,
                             float *d_rgb, uint32_t *d_argb, uint64_t *d_counters, void *stream);
/* The same, recording the caller's hipEvent_t `emitted_event` on `stream` once the randDirs are emitted, before the
 * trace: from then on the next frame's stream state is on the device, so the next frame's rfx_frame_rng_count and
 * all-gather may run on another stream while this frame traces (reflaxman_amd/dist.py count-ahead).  The renderer's
 * RNG stream must not advance in between (no other render call on this renderer). */
int rfx_render_frame_counted_ev(rfx_renderer *r, const rfx_frame *frame, uint32_t nslices,
                                const uint32_t *d_blk_counts, float *d_rgb, uint32_t *d_argb, uint64_t *d_counters,
                                void *stream, void *emitted_event);

/* Emit-ahead (multi-GPU, reflaxman_amd/dist.py): the counted frame split in two, so the next frame's emit can run on
 * another stream while this frame traces.  rfx_frame_rng_emit scans the all-gathered counts and writes the frame's
 * randDirs into the renderer's second randDir buffer (the one the last enqueued trace does not read; order it after
 * the trace before that), records emitted_event, and moves the stream state past the frame;
 * rfx_render_frame_emitted traces that frame.  One emitted frame at a time; rfx_frame_rng_discard forgets it and
 * restores the stream state.  Other render calls fail while a frame is pending. */
int rfx_frame_rng_emit(rfx_renderer *r, const rfx_frame *frame, uint32_t nslices, const uint32_t *d_blk_counts,
                       void *stream, void *emitted_event);
int rfx_render_frame_emitted(rfx_renderer *r, const rfx_frame *frame, float *d_rgb, uint32_t *d_argb,
                             uint64_t *d_counters, void *stream);
int rfx_frame_rng_discard(rfx_renderer *r);
/* The sphere-stream state the next traced frame starts from: the emitted frame's when one is pending (returns 1),
 * else the current state (returns 0).  Synchronises with the renderer's stream; the emit must have completed (order
 * the renderer's stream after the emit's, or synchronise the device).  A single-GPU renderer seeded with it renders
 * that frame (bench.py's steady-state parity check). */
int rfx_frame_rng_pending(rfx_renderer *r, uint32_t *frame_start);

/* Undo the random-stream advance of the last call, which must be an rfx_render_frame (else RFX_ERR_STATE): both
 * streams return to that frame's start, its pixels stay as written.  The drop-in Render (dropin/Render.h) renders a
 * whole frame at the first renderNext after renderBegin; when the caller leaves that frame early (renderBegin or
 * setImageSize mid-frame, Pulse.cpp:110-124) it rewinds and renders exactly the span the reference's cursor covered,
 * so the streams end where the reference's do (Render.cpp:136-215, trace_math.h:34-39). */
int rfx_frame_rng_rewind(rfx_renderer *r);

/* ---------------------------------------------------------------- Device groups (multi-GPU, one process)
 * A group renders the frame of Render::renderNext (Render.cpp:136-215) on several devices of this process: row bands,
 * one per member, each member counting its slice of the frame's random stream and pushing it to the others (the one
 * exchange step), then emitting and tracing its band; members 1..n-1 copy their band rows into the
 * caller's frame on member 0's device over xGMI (hipMemcpyPeerAsync).  The assembled frame is the single-GPU frame
 * bit for bit.  Bands start equal (8-row multiples) and are re-cut from measured per-member trace times every 8
 * frames (completed measurements only: no frame waits), unless fixed with rfx_group_set_bands.  Member 0's renderer
 * carries the group's random streams: a frame starts every member from member 0's state, so the caller may render
 * other frames (block preview, spans) on member 0 alone in between, and rfx_frame_rng_rewind on member 0 undoes a
 * group frame.  For C/C++ callers without torch.distributed (dropin/Render.h: RFX_DEVICES=0,1,...); the
 * multi-process form is reflaxman_amd/dist.py over RCCL. */
typedef struct rfx_group rfx_group;
int rfx_group_create(rfx_group **out, const int *devices, int n);  /* a device may repeat (one-GPU rehearsal) */
void rfx_group_destroy(rfx_group *g);
int rfx_group_size(const rfx_group *g);
rfx_renderer *rfx_group_renderer(rfx_group *g, int member);       /* per-member settings (tile order, ...) */
int rfx_group_set_scene(rfx_group *g, const rfx_scene *scene);
/* fixed bands: bounds[0] = 0 < bounds[1] < ... < bounds[n] = height rows; bounds NULL = automatic (default) */
int rfx_group_set_bands(rfx_group *g, uint32_t height, const uint32_t *bounds);
int rfx_group_get_bands(const rfx_group *g, uint32_t *bounds);     /* the bands of the last frame (n + 1 rows) */
/* One whole frame (sample_num > 0; SSAA, additive and accumulation included; the partition fields of `frame` must be
 * rank 0 of 1 and the span the whole frame) into d_rgb / d_argb (W*H*3 floats / W*H words, or NULL) on member 0's
 * device, ordered after and before the caller's work on `stream` (member 0's stream; NULL = its renderer's).
 * d_rgb NULL (d_argb given, no accumulation): an ARGB8-only frame -- the members copy 4 B/px to member 0 instead of
 * 16 B/px, for a display that never reads the float image. */
int rfx_group_render_frame(rfx_group *g, const rfx_frame *frame, float *d_rgb, uint32_t *d_argb, void *stream);

/* Optional per-phase timing of rfx_render_frame with HIP events recorded on the launch stream:
 * enable, render, then read the summed device time (ms) of the RNG pre-pass and of the trace kernel
 * over the timed frames since the last read, and their number (synchronises; resets the sums).  enable = 1 times
 * every frame, n > 1 every n-th frame (three event records per timed frame cost ~10 us of a 640x480 frame's ~50). */
int rfx_renderer_set_timing(rfx_renderer *r, int enable);
int rfx_renderer_get_timing(rfx_renderer *r, double *prepass_ms, double *trace_ms, uint64_t *frames);

/* host-buffer convenience for callers without device memory of their own (PCIe-inclusive):
 * rgb: host W*H*3 (in/out), argb: host W*H or NULL.  Partitioning fields must be rank 0 of 1. */
int rfx_render_frame_host(rfx_renderer *r, const rfx_frame *frame, float *rgb, uint32_t *argb,
                          uint64_t *counters);

/* device memory helpers for C/C++ hosts that have no allocator of their own */
int rfx_device_alloc(rfx_renderer *r, size_t bytes, void **dptr);
int rfx_device_free(rfx_renderer *r, void *dptr);
int rfx_memcpy_d2h(rfx_renderer *r, void *dst, const void *src, size_t bytes);
int rfx_memcpy_h2d(rfx_renderer *r, void *dst, const void *src, size_t bytes);
/* device-to-device copy on the renderer's stream (asynchronous) */
int rfx_memcpy_d2d(rfx_renderer *r, void *dst, const void *src, size_t bytes);
int rfx_synchronize(rfx_renderer *r);

/* Sample the RNG stream: the first n randomInsideSphere draws from `seed` (Vector3.cpp:176-188),
 * computed by the device pre-pass, n x 3 floats to host.  *seed_out = state after them. */
int rfx_rand_dirs(rfx_renderer *r, uint32_t seed, uint64_t n, float *out3, uint32_t *seed_out);

/*
 * Device known-answer entry points (validation).  Each runs the trace kernel's own device code on host
 * arrays and returns host results, synchronously, on the scene last uploaded by rfx_renderer_set_scene:
 *   rfx_kat_objects: ray i = rays[6i..6i+5] (origin, direction) against object objects[i] alone ->
 *       out[15i..]: hit, drop3, normal3, reflected ray3, distance, material colour3 (texel of a textured
 *       triangle), any-hit -- SceneObject::trace with and without out-parameters (Sphere.cpp:44-85,
 *       Triangle.cpp:53-108, Plane.cpp:36-73);
 *   rfx_kat_texels: texture >= 0: Texture::getTexelColor(u, v) (in n x 2, Texture.cpp:231-269) of that scene
 *       texture; texture < 0: Skybox::getTexelColor(ray) (in n x 3, Skybox.cpp:39-106) -> out n x 3;
 *   rfx_kat_powf: powf(x, y) as Scene.cpp:175,196 evaluate it (in n x 2 -> out n);
 *   rfx_kat_argb: Color::argb (Color.cpp:114-117) (in n x 3 -> out n);
 *   rfx_kat_powf_cube: the Fresnel site's powf(x, 3) (Scene.cpp:196) as the bounce loop evaluates it (the double
 *       cube where it provably rounds like glibc, rfx_powf.h powf_cube_fast) against glibc's algorithm on the device,
 *       for every float x in [0, 1]: counts[0] = mismatches (0 expected), counts[1] = inputs that took glibc's
 *       algorithm;
 *   rfx_kat_div: the trace loop's division fast paths (rfx_math.h div_rn, normalized's shared reciprocal and the
 *       skybox's div_fast_unit) against IEEE '/' on the operand pairs first .. first + n - 1 of a fixed hash (every
 *       float class, both edges of the fast path's divisor and quotient bounds): counts[0] = quotients whose bits
 *       differ (0 expected), counts[1] = pairs that took div_rn's fast path, counts[2] = quotients checked (5 per
 *       pair).
 */
int rfx_kat_objects(rfx_renderer *r, const float *rays, const int32_t *objects, uint64_t n, float *out);
int rfx_kat_texels(rfx_renderer *r, int texture, const float *in, uint64_t n, float *out);
int rfx_kat_powf(rfx_renderer *r, const float *xy, uint64_t n, float *out);
int rfx_kat_argb(rfx_renderer *r, const float *rgb, uint64_t n, uint32_t *out);
int rfx_kat_powf_cube(rfx_renderer *r, uint64_t counts[2]);
int rfx_kat_div(rfx_renderer *r, uint64_t first, uint64_t n, uint64_t counts[3]);
/* The kernel-argument layout the bounce loops rely on (rfx_trace.h launder_scene / kernarg_params: DevScene at kernarg
 * offset 0, FrameParams after it): a one-lane kernel of the trace kernels' signature compares the records read through
 * the kernarg segment pointer with its by-value arguments.  out[0] / out[1] = differing words of the scene record / the
 * frame parameters (0 expected), out[2] = 1 if the build reads the scene record that way.  swapped = 1 runs the same
 * check in a kernel declared (FrameParams, DevScene): the check must report differences there. */
int rfx_kat_kernarg(rfx_renderer *r, int swapped, uint32_t out[3]);

#ifdef __cplusplus
}
#endif
#endif /* RFX_H */
