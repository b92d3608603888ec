// POD layouts shared by the host C-ABI (rfx_host.cpp) and the gfx950 kernels
// (rfx_trace.h, rfx_kernels.hip).  All device arrays are structure-of-arrays, 16-B aligned,
// and walked in wave-uniform order by the trace kernel, so the compiler serves
// them through the scalar cache (s_load_dwordx4) rather than per-lane loads.
#pragma once
#include <stdint.h>

namespace rfx {

// per-frame event counters (same order as oracle/rfx_oracle.h ORC_*)
enum Counter {
  C_RAYS = 0, C_SEGMENTS,
  C_SPH_TESTS, C_SPH_B, C_SPH_D, C_SPH_T,
  C_TRI_TESTS, C_TRI_Z, C_TRI_S, C_TRI_T, C_TRI_IN, C_TRI_D,
  C_HIT_SPH, C_HIT_TRI,
  C_SH_SPH_TESTS, C_SH_SPH_B, C_SH_SPH_D, C_SH_SPH_T,
  C_SH_TRI_TESTS, C_SH_TRI_Z, C_SH_TRI_S, C_SH_TRI_T, C_SH_TRI_IN,
  C_L_EVAL, C_L_FACING, C_L_LIT, C_L_SPEC, C_L_POW,
  C_DIELECTRIC, C_METAL, C_CONTINUE, C_SKY,
  C_TEX_BILINEAR, C_TEX_CHECKER, C_TEX_OTHER,
  C_PLN_TESTS, C_PLN_T, C_HIT_PLN, C_SH_PLN_TESTS, C_SH_PLN_T,
  C_COUNT
};

struct alignas(16) SphereGeo { float cx, cy, cz, sq_radius; };      // Sphere.cpp:9-20
// Spheres 2j and 2j+1 side by side, so one packed-f32 (v_pk_*) instruction runs the same step of both
// miss tests.  An odd count is padded with sq_radius = -inf: c = +inf, d = -inf or NaN, never a hit.
struct alignas(32) SpherePair { float cx[2], cy[2], cz[2], r2[2]; };
struct alignas(16) MatRec { float r, g, b, refl; };                 // Material.h:9-11 (transparency unused)
// Triangle.cpp:11-21: v0 and axTrans (inverted) -- z row first (every test needs it), then the x and
// y rows interleaved, (a11,a21), (a12,a22), (a13,a23), so (u, v) come out of one v_pk_* chain.
struct alignas(16) TriGeo {
  float v0x, v0y, v0z, a31, a32, a33;
  float a11, a21, a12, a22, a13, a23;
  float pad[4];
};
struct alignas(16) TriShade {                                        // Triangle.cpp:110-120
  float nx, ny, nz, tu0;
  float t11, t12, t21, t22;   // tuvTrans _11 _12 _21 _22 (_13 = _23 = 0 by construction)
  float tv0; int32_t tex; int32_t dielectric; int32_t obj;
};
// Bounding sphere of an object for the wave-bundle cull (rfx_trace.h): spheres first, then triangles.
// r = +inf marks an object that is never culled (an ill-conditioned triangle, see rfx_host.cpp).
struct alignas(16) Bound { float x, y, z, r; };
// Small scenes (<= 32 spheres, <= 32 triangles): one cull record per lane of a wave.  Lanes 0-15 hold
// spheres 0, 2, .., 30, lanes 16-31 spheres 1, 3, .., 31 (so a ballot folds into the pair mask with one
// shift), lanes 32-63 triangles 0-31.  A triangle record also carries its plane (unit normal n, n . v0);
// a sphere's or an empty lane's plane is zero.
struct alignas(16) CullRec { float x, y, z, r, nx, ny, nz, d; };
// Footprint record of small-scene triangle i (for the primary-bundle masks, prim_cull_kernel): vertex v0 and the
// rows gu, gv of the inverse of the reference's basis [v2 - v0 | v1 - v0 | -norm] (Triangle.cpp:17-18), so that
// u = gu . (P - v0) and v = gv . (P - v0) for P in the plane; nu = |gu|, nv = |gv|, nuv = |gu + gv| (+inf: the
// footprint test must not touch the triangle -- ill-conditioned or degenerate).
struct alignas(16) CullTri { float v0x, v0y, v0z, nu, gux, guy, guz, nv, gvx, gvy, gvz, nuv; };
// Bounding-volume hierarchy over the sphere pairs of a large scene (rfx_host.cpp build_pair_bvh): an internal
// node holds its two children's boxes (the spheres grown by their radii) and their indices: c >= 0 an internal
// node, c < 0 the leaf pair ~c (spheres 2(~c), 2(~c) + 1 of the device arrays, which are in spatial order).
// mt[c]: |ref - centre of child c|_2 + its half-diagonal (ref: DevScene::bvh_ref), so that kCullRel (|o - ref|_2 + mt[c])
// bounds the kernel's per-ray box margin from above with one add per child (triangle inequality)
// RFX_BVH_PREWIDE (round 4, kept: C5 trace + bounce -4.0%): the host stores each child box already grown by kCullRel
// mt[c] (rounded outward), so the kernel adds only the per-ray part of the margin, folded into per-ray slab constants.
#ifndef RFX_BVH_PREWIDE
#define RFX_BVH_PREWIDE 1
#endif
struct alignas(16) BvhNode { float lx[2], ly[2], lz[2], hx[2], hy[2], hz[2]; int32_t child[2]; float mt[2]; };
// Sphere pairs per BVH leaf (rfx_host.cpp build_pair_bvh, rfx_trace.h leaf tests): leaf ~g holds the pairs
// [RFX_BVH_LEAF_PAIRS g, RFX_BVH_LEAF_PAIRS (g + 1)) of the device order (sph_pair padded with never-hit pairs)
#ifndef RFX_BVH_LEAF_PAIRS
#define RFX_BVH_LEAF_PAIRS 4
#endif
// Plane(pos, norm, material) (Plane.h:6-14): the normal as given (the reference never normalises it)
struct alignas(16) PlaneGeo { float px, py, pz, nx, ny, nz; int32_t obj, dielectric; };
struct alignas(16) LightRec { float ox, oy, oz, radius, r, g, b, power; }; // OmniLight.h
struct alignas(16) TexRec { uint32_t offset, w, h, pad; };

struct DevScene {
  const SphereGeo *sph_geo;   // n_sph
  const SpherePair *sph_pair; // (n_sph + 1) / 2
  const MatRec *sph_mat;      // n_sph
  const int32_t *sph_info;    // n_sph x2: {object index, dielectric}
  const TriGeo *tri_geo;      // n_tri
  const TriShade *tri_shade;  // n_tri
  const MatRec *tri_mat;      // n_tri
  const LightRec *lights;     // n_light
  const TexRec *texs;         // n_tex
  const uint32_t *texels;     // texel pool, ARGB
  const Bound *bound;         // n_sph + n_tri bounding spheres
  const Bound *chunk_bound;   // n_chunk bounding spheres of 64-sphere chunks (large scenes: spatial order)
  const BvhNode *bvh;         // large scenes: pair BVH, root 0 (null: the chunk loops)
  const CullRec *cull_small;  // 64 lane records (small scenes only, else null)
  const CullTri *cull_tri;    // 32 triangle footprint records (small scenes only, else null)
  const PlaneGeo *pln_geo;    // n_pln (tested by every ray, never culled)
  const MatRec *pln_mat;      // n_pln
  const int32_t *obj_loc;     // n_obj: object index -> kind << 28 | index within its kind's device arrays
  uint64_t cull_valid;        // lanes of cull_small that hold an object
  int32_t n_sph, n_tri, n_light, skybox_tex;
  int32_t n_pln, n_obj, n_tex;
  int32_t bvh_depth;          // internal levels of the BVH (<= kBvhStack)
  float bvh_rx, bvh_ry, bvh_rz;  // the BVH's margin reference point (its root box centre)
  float key_lx, key_ly, key_lz;  // regroup sort keys: origin cell = (o - key_l) * key_s in [0, 8) per axis (the BVH
  float key_sx, key_sy, key_sz;  // root box; 0 scale without a BVH: one cell)
  int32_t n_chunk;            // (n_sph + 63) / 64
  const uint32_t *bvh_aux;    // per node: child indices as two int16 (lo, hi), margin terms as two uint16 * bvh_mstep
  float bvh_mstep;            //   (rounded up) -- the 8-B record the LDS-staged bounce kernel keeps beside the boxes
  int32_t n_bvh;              // nodes of the BVH
  float amb_r, amb_g, amb_b;  // diffLightColor * diffLightPower (Scene.cpp:186, host-folded)
  float env_r, env_g, env_b;  // envColor (Scene.cpp:12,55)
  float half_tile_w, half_tile_h;  // Skybox.cpp:21-37
};

// The bounce kernel with the BVH staged in LDS (rfx_trace.h bounce_kernel_lds): one workgroup of kLdsBvhWaves waves
// per CU; its dynamic LDS holds the node boxes (48 B each), DevScene::bvh_aux (8 B each), the lanes' traversal stacks
// (kLdsBvhStackSlots int16 each) and one output slot (u32) per lane.
constexpr int kLdsBvhWaves = 16, kLdsBvhStackSlots = 16;
constexpr size_t lds_bvh_bytes(int n_bvh)
{
  return (size_t)n_bvh * 56 + sizeof(int16_t) * kLdsBvhStackSlots * 64 * kLdsBvhWaves + 4 * 64 * kLdsBvhWaves;
}
// whether a BVH of n_bvh nodes fits beside the kernel's static LDS (the colour table and powf's tables, < 4 KB)
constexpr bool lds_bvh_fits(int n_bvh) { return n_bvh > 0 && lds_bvh_bytes(n_bvh) + 4096 <= 160 * 1024; }

// A trace parked between bounce segments (large scenes, plain pixels): the state Scene::trace carries from
// one segment to the next (Scene.cpp:80-234: origin, ray, mulColor, pixelColor, refl), the trace index of its
// randDir and the output pixel.  64 B: one lane stores / loads it with four 16-B accesses.
constexpr uint32_t kQueueBuckets = 4096;  // regroup sort buckets (rfx_trace.h queue_key)
struct alignas(16) QRay {
  float ox, oy, oz, dx;
  float dy, dz, mr, mg;
  float mb, pr, pg, pb;
  uint32_t trace, out, refl, pad;
};

struct FrameParams {
  float eye_x, eye_y, eye_z;
  float v11, v12, v13, v21, v22, v23, v31, v32, v33;  // Render::renderCameraView
  float rz, wh, hh;             // Render.cpp:148-150
  uint32_t W, H;
  int32_t depth, ss;            // reflectNum, sampleNum
  int32_t accumulate;           // additiveCounter > 1 (Render.cpp:191)
  int32_t additive;             // jitter on (Render.cpp:177-178)
  uint32_t jitter_seed;         // Render.cpp stream state at frame start
  uint32_t row_block, rank, nranks;  // block-cyclic row strips (nranks == 1: whole frame)
  uint32_t grid_rows;           // rows (ss > 0) or corner rows (ss < 0) covered by the grid
  uint32_t row0;                // first frame row (ss > 0) / corner row (ss < 0) of the grid (nranks == 1)
  uint64_t p_begin, p_end;      // raster pixel range of this call (Render::renderNext cursor span)
  uint64_t trace_base;          // trace index of the first trace in the range (block mode: corner count)
  float *img;                   // W x H x 3 frame (nranks == 1) or strip_rows x W x 3 (in/out when accumulate)
  uint32_t *argb;               // same shape, or null
  const uint32_t *rd_state;     // per trace: LCG state before its accepted randomInsideSphere triple
  unsigned long long *counters; // C_COUNT u64, stats build only
  const uint32_t *tile_order;   // workgroup i renders tile tile_order[i] (previous frame's LPT order), or null: tile i
  uint32_t *tile_cost;          // per tile: its clock cycles this frame (the next frame's order), or null
  uint32_t tiles_x;             // schedule tiles per grid row (set by launch_trace)
  // ray regrouping (plain pixels, large scenes): a trace still alive after park_after segments is appended to
  // queue (queue_count: entries) instead of continuing; the bounce kernel then runs the queue in packed waves whose
  // idle lanes claim the next entries from queue_next.  park_after <= 0: no parking.
  QRay *queue;
  uint32_t *queue_count, *queue_next;
  int32_t park_after;
  // regroup sort (RFX_QUEUE_SORT): queue_key[i] is entry i's bucket (direction octant, origin cell), written at park
  // time; queue_order lists the entries bucket by bucket, and the bounce kernel claims them in that order
  uint32_t *queue_key;
  const uint32_t *queue_order;
  // small scenes, plain and SSAA pixels: per wave tile, the cull mask of its primary bundle and of its primary hits'
  // shadow rays (prim_cull_kernel), or null; prim_shadow: the shadow masks hold (not for jittered additive frames,
  // whose primary hits are not known ahead)
  const uint64_t *prim_mask;
  int32_t prim_shadow;
};

}  // namespace rfx
