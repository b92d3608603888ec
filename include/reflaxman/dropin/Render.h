// reflaxman/dropin/Render.h -- drop-in replacement for the reference's src/common/Render.h.
//
// The reference's Render class (Render.h:7-42) with the same members and semantics, rendering on the MI355X
// through the C-ABI (../../rfx.h) instead of the CPU loop of Render.cpp:136-215:
//   * public camera (the caller's own Camera, Camera.h -- proceedControl/inMotion keep working), scene
//     (./Scene.h), imageWidth, imageHeight, additiveCounter, inProgress;
//   * renderBegin snapshots camera.view / camera.eye (Render.cpp:116-134); renderAll keeps the reference's
//     behaviour (imageHeight *pixels*, Render.cpp:217-221);
//   * renderNext(pixels) -- policy "frame" (default): the first call after renderBegin renders the
//     whole rest of the frame on the device into a second framebuffer, and every call only advances the cursor;
//     the frame becomes the image when the cursor reaches its end.  A caller that leaves a frame early --
//     renderBegin or setImageSize mid-frame (Pulse.cpp:110-124), a scene or fov change, or an imagePixel /
//     copyImage read before the end -- gets exactly the reference's state: the random streams are rewound
//     (rfx_frame_rng_rewind) and exactly the span the cursor covered is rendered into the image, as the reference
//     would have.  Policy "span" (RFX_DROPIN_POLICY=span, or setRenderPolicy) renders each call's span as it
//     comes.  Any chunk pattern gives the reference's images and random streams under either policy;
//   * several GPUs of this process (RFX_DEVICES=0,1,... in the environment): frames rendered ahead with
//     sampleNum > 0 (still frames, screenshots), and frames rendered by one renderNext(W*H) call under either policy,
//     are cut into row bands over the devices (rfx_group_render_frame); block previews and partial spans stay on
//     the first device, which carries the random streams.  Groups of distinct devices are unverified on hardware
//     so far (every group test ran its members on one GPU; tests/test_gpu_group.py skips the multi-device test
//     when only one device is visible);
//   * the float framebuffer (std::vector<Color> image, Render.h:10) lives in HBM and is read back on demand;
//     imagePixel / copyImage then apply the caller's own Color::operator/ and Color::argb, as the reference.
// Random streams: the reference seeds its two per-TU LCG streams from rand() at static init (trace_math.h:34),
// so their values depend on link order; here they default to the harness link order's values and can be set
// with RFX_SPHERE_SEED / RFX_JITTER_SEED in the environment (parity tests replay a given reference build).
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "rfx.h"  // -I <repo>/include
#include "Camera.h"
#include "Scene.h"
#include "Texture.h"

class Render {
 private:
  std::vector<Color> image;  // host copy of the device framebuffer (read back on demand)

  // staged render settings (Render.h:12-19)
  unsigned int curx;
  unsigned int cury;
  int renderReflectNum;
  int renderSampleNum;
  bool renderAdditive;
  Matrix33 renderCameraView;
  Vector3 renderCameraEye;

  rfx_renderer *r = nullptr;
  rfx_group *group = nullptr;  // RFX_DEVICES with two or more devices: r is its member 0
  void *d_image = nullptr;
  void *d_spec = nullptr;  // policy "frame": the frame being rendered ahead of the cursor
  size_t d_capacity = 0;
  unsigned long long uploaded = ~0ull;
  mutable bool host_valid = false;
  bool whole_frame = true;                // policy "frame"
  bool spec_active = false;               // d_spec holds this frame's pixels [spec_begin, W*H) ahead of the cursor
  uint64_t spec_begin = 0;
  float spec_fov = 0.0f;
  unsigned long long spec_revision = 0;

  static bool policy_env()
  {
    const char *v = getenv("RFX_DROPIN_POLICY");
    return !(v && !strcmp(v, "span"));
  }
  rfx_frame frame_of(uint64_t p0, uint64_t p1) const
  {
    rfx_frame f;
    memset(&f, 0, sizeof(f));
    f.eye[0] = renderCameraEye.x; f.eye[1] = renderCameraEye.y; f.eye[2] = renderCameraEye.z;
    memcpy(f.view, &renderCameraView.m[0][0], sizeof(f.view));
    f.fov = camera.fov;  // rz = W/2/tanf(camera.fov/2): the live camera's fov, as Render.cpp:148
    f.width = imageWidth;
    f.height = imageHeight;
    f.reflect_num = renderReflectNum;
    f.sample_num = renderSampleNum;
    f.additive = renderAdditive;
    f.additive_counter = additiveCounter;
    f.nranks = 1;
    f.pixel_begin = p0;
    f.pixel_end = p1;
    return f;
  }
  void upload_scene()
  {
    if (uploaded != scene.revision())
    {
      rfx_dropin::check(group ? rfx_group_set_scene(group, scene.handle()) : rfx_renderer_set_scene(r, scene.handle()),
                        "rfx_renderer_set_scene");
      uploaded = scene.revision();
    }
  }
  // Leave the frame rendered ahead at the cursor: rewind the random streams to its start and render exactly the span
  // [spec_begin, cursor) into the image, as the reference's renderNext calls had (the rest keeps its old pixels).
  void settle(bool keep_pixels = true)
  {
    if (!spec_active) return;
    spec_active = false;
    rfx_dropin::check(rfx_frame_rng_rewind(r), "Render: rewind");
    const uint64_t c = (uint64_t)cury * imageWidth + curx;
    if (c > spec_begin)
    {
      const float fov = camera.fov;
      camera.fov = spec_fov;  // the span as it was rendered ahead
      const rfx_frame f = frame_of(spec_begin, c);
      camera.fov = fov;
      rfx_dropin::check(rfx_render_frame(r, &f, (float *)(keep_pixels ? d_image : d_spec), nullptr, nullptr, nullptr),
                        "Render: settle");
    }
    host_valid = false;
  }

  static uint32_t seed_env(const char *name, uint32_t dflt)
  {
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, nullptr, 0) : dflt;
  }
  void sync_host() const
  {
    if (host_valid) return;
    Render *self = const_cast<Render *>(this);
    self->settle();  // a read mid-frame sees the reference's image: the span rendered so far, old pixels after it
    const size_t n = (size_t)imageWidth * imageHeight;
    if (self->image.size() < n) self->image.resize(n);
    if (n) rfx_dropin::check(rfx_memcpy_d2h(r, &self->image.front(), d_image, n * sizeof(float) * 3), "Render: read back");
    host_valid = true;
  }

 public:
  Camera camera;
  Scene scene;
  unsigned int imageWidth;
  unsigned int imageHeight;
  int additiveCounter;
  bool inProgress;

  Render(const char *exePath)  // Render.cpp:5-18
      : curx(0), cury(0), renderReflectNum(0), renderSampleNum(0), renderAdditive(false), imageWidth(0), imageHeight(0),
        additiveCounter(0), inProgress(false)
  {
    static_assert(sizeof(Color) == 3 * sizeof(float), "Color must be three floats (Color.h)");
    std::vector<int> devs;
    if (const char *v = getenv("RFX_DEVICES"))
      for (const char *p = v; *p;)
      {
        char *e = nullptr;
        const long d = strtol(p, &e, 10);
        if (e == p) break;
        devs.push_back((int)d);
        p = *e ? e + 1 : e;
      }
    if (devs.size() >= 2)
    {
      rfx_dropin::check(rfx_group_create(&group, &devs.front(), (int)devs.size()), "rfx_group_create");
      r = rfx_group_renderer(group, 0);
    }
    else
      rfx_dropin::check(rfx_renderer_create(&r, devs.empty() ? 0 : devs[0]), "rfx_renderer_create");
    rfx_dropin::check(rfx_renderer_set_rng(r, seed_env("RFX_SPHERE_SEED", 1350490027u), seed_env("RFX_JITTER_SEED", 424238335u)),
                      "rfx_renderer_set_rng");
    whole_frame = policy_env();
    loadScene(exePath);
  }
  ~Render()
  {
    if (d_image) rfx_device_free(r, d_image);
    if (d_spec) rfx_device_free(r, d_spec);
    if (group)
      rfx_group_destroy(group);
    else
      rfx_renderer_destroy(r);
  }
  Render(const Render &) = delete;
  Render &operator=(const Render &) = delete;

  void loadScene(const char *exePath)  // Render.cpp:25-55
  {
    const std::string skyboxTextureFileName = std::string(exePath) + "./textures/skybox.tga";
    const std::string planeTextureFileName = std::string(exePath) + "./textures/himiya.tga";
    camera = Camera(Vector3(7.427f, 3.494f, -3.773f), Vector3(6.5981f, 3.127f, -3.352f), 1.05f);
    scene = Scene(Color(0.95f, 0.95f, 1.0f), 0.15f);
    scene.setSkyboxTexture(skyboxTextureFileName.c_str());
    scene.addLight(Vector3(11.8e9f, 4.26e9f, 3.08e9f), 3.48e8f, Color(1.0f, 1.0f, 0.95f), 0.85f);
    scene.addSphere(Vector3(-1.25f, 1.5f, -0.25f), 1.5f, Material(Material::mtMetal, Color(1.0f, 1.0f, 1.0f), 1.0f, 0.0f));
    scene.addSphere(Vector3(0.15f, 1.0f, 1.75f), 1.0f, Material(Material::mtMetal, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    scene.addSphere(Vector3(-3.0f, 0.6f, -3.0f), 0.6f, Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.0f, 0.0f));
    scene.addSphere(Vector3(-0.5f, 0.5f, -2.5f), 0.5f, Material(Material::mtDielectric, Color(0.5f, 1.0f, 0.15f), 0.75f, 0.0f));
    scene.addSphere(Vector3(1.0f, 0.4f, -1.5f), 0.4f, Material(Material::mtDielectric, Color(0.0f, 0.5f, 1.0f), 1.0f, 0.0f));
    scene.addSphere(Vector3(1.8f, 0.4f, 0.1f), 0.4f, Material(Material::mtMetal, Color(1.0f, 0.65f, 0.45f), 1.0f, 0.0f));
    scene.addSphere(Vector3(1.7f, 0.5f, 1.9f), 0.5f, Material(Material::mtMetal, Color(1.0f, 0.90f, 0.60f), 0.75f, 0.0f));
    scene.addSphere(Vector3(0.6f, 0.6f, 4.2f), 0.6f, Material(Material::mtMetal, Color(0.9f, 0.9f, 0.9f), 0.0f, 0.0f));
    Texture *planeTexture = scene.addTexture(planeTextureFileName.c_str());
    Triangle *tr1 = scene.addTriangle(Vector3(-14.0f, 0.0f, -10.0f), Vector3(-14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, -10.0f),
                                      Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    tr1->setTexture(planeTexture, 0.0f, 0.0f, 0.0f, 1.0f, 1.0f, 0.0f);
    Triangle *tr2 = scene.addTriangle(Vector3(-14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, -10.0f),
                                      Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    tr2->setTexture(planeTexture, 0.0f, 1.0f, 1.0f, 1.0f, 1.0f, 0.0f);
  }

  void setImageSize(unsigned int width, unsigned int height)  // Render.cpp:57-80
  {
    if (width > 0 && height > 0)
    {
      settle(false);  // a frame left mid-way: the random streams as far as the cursor got (Render.cpp:57-80)
      const size_t bytes = (size_t)width * height * sizeof(float) * 3;
      if (bytes > d_capacity)
      {
        if (d_image) rfx_device_free(r, d_image);
        d_image = nullptr;
        rfx_dropin::check(rfx_device_alloc(r, bytes, &d_image), "Render::setImageSize");
        if (d_spec) rfx_device_free(r, d_spec);
        d_spec = nullptr;
        if (whole_frame) rfx_dropin::check(rfx_device_alloc(r, bytes, &d_spec), "Render::setImageSize");
        d_capacity = bytes;
      }
      std::vector<float> zero((size_t)width * height * 3, 0.0f);
      rfx_dropin::check(rfx_memcpy_h2d(r, d_image, &zero.front(), bytes), "Render::setImageSize");
      imageWidth = width;
      imageHeight = height;
      additiveCounter = 0;
      inProgress = false;
      curx = 0;
      cury = 0;
      host_valid = false;
    }
  }

  void copyImage(Texture &texture) const  // Render.cpp:82-101
  {
    if (imageWidth == texture.getWidth() && imageHeight == texture.getHeight())
    {
      sync_host();
      const Color *imagePixel = &image.front();
      ARGB *texPixel = texture.getColorBuffer();
      const ARGB *endTexPixel = texPixel + imageWidth * imageHeight;
      while (texPixel < endTexPixel) *texPixel++ = (imagePixel++)->argb();
    }
    else
      texture.clear(0);
  }

  Color imagePixel(int x, int y) const  // Render.cpp:103-114
  {
    if (x >= 0 && y >= 0)
    {
      sync_host();
      return additiveCounter > 1 ? image[x + y * imageWidth] / float(additiveCounter) : image[x + y * imageWidth];
    }
    return Color(0, 0, 0);
  }

  void renderBegin(int reflectNum, int sampleNum, bool additive)  // Render.cpp:116-134
  {
    settle();  // the last frame left mid-way keeps what the reference's cursor rendered
    renderReflectNum = reflectNum;
    renderSampleNum = sampleNum;
    renderAdditive = additive;
    inProgress = true;
    curx = 0;
    cury = 0;
    renderCameraView = camera.view;
    renderCameraEye = camera.eye;
    if (additive)
      additiveCounter++;
    else
      additiveCounter = 0;
  }

  bool renderNext(unsigned int pixels)  // Render.cpp:136-215, the cursor's span rendered on the device
  {
    if (!pixels || !inProgress || curx >= imageWidth || cury >= imageHeight || renderReflectNum <= 0 || !renderSampleNum)
      return false;
    const uint64_t total = (uint64_t)imageWidth * imageHeight;
    const uint64_t p0 = (uint64_t)cury * imageWidth + curx;
    const uint64_t p1 = p0 + pixels < total ? p0 + pixels : total;
    if (spec_active && (scene.revision() != spec_revision || camera.fov != spec_fov))
      settle();  // what was rendered ahead no longer holds for the rest of the frame
    upload_scene();
    if (whole_frame && d_spec && !spec_active && p1 < total)
    {
      // render the rest of the frame [p0, total) ahead into d_spec; it starts as the image (old pixels that an
      // additive frame accumulates onto, block-preview fills of corners before p0)
      if (p0 > 0 || (renderSampleNum > 0 && additiveCounter > 1))
        rfx_dropin::check(rfx_memcpy_d2d(r, d_spec, d_image, (size_t)total * sizeof(float) * 3), "Render::renderNext");
      const rfx_frame f = frame_of(p0, total);
      if (group && p0 == 0 && renderSampleNum > 0)  // the whole frame in row bands over the group's devices
        rfx_dropin::check(rfx_group_render_frame(group, &f, (float *)d_spec, nullptr, nullptr), "Render::renderNext");
      else
        rfx_dropin::check(rfx_render_frame(r, &f, (float *)d_spec, nullptr, nullptr, nullptr), "Render::renderNext");
      spec_active = true;
      spec_begin = p0;
      spec_fov = camera.fov;
      spec_revision = scene.revision();
    }
    else if (!spec_active)
    {
      const rfx_frame f = frame_of(p0, p1);
      if (group && p0 == 0 && p1 == total && renderSampleNum > 0)  // one call for the whole frame (renderNext(W*H))
        rfx_dropin::check(rfx_group_render_frame(group, &f, (float *)d_image, nullptr, nullptr), "Render::renderNext");
      else
        rfx_dropin::check(rfx_render_frame(r, &f, (float *)d_image, nullptr, nullptr, nullptr), "Render::renderNext");
    }
    host_valid = false;  // the reference's image has changed (a read mid-frame settles the frame rendered ahead)
    curx = (unsigned int)(p1 % imageWidth);
    cury = (unsigned int)(p1 / imageWidth);
    if (p1 == total)
    {
      inProgress = false;
      if (spec_active)  // the frame rendered ahead is complete: it is the image
      {
        void *t = d_image;
        d_image = d_spec;
        d_spec = t;
        spec_active = false;
      }
    }
    return inProgress;
  }

  void renderAll(int reflectNum, int sampleNum, bool additive)  // Render.cpp:217-221, as shipped
  {
    renderBegin(reflectNum, sampleNum, additive);
    renderNext(imageHeight);
  }

  float getRenderProgress() const  // Render.cpp:223-226
  {
    return float(curx + cury * imageWidth) * 100.0f / imageWidth / imageHeight;
  }

  rfx_renderer *renderer() const { return r; }
  // "frame" (true, default): render the rest of the frame at the first renderNext after renderBegin; "span" (false):
  // render each renderNext's span as it comes (Render.cpp:136-215 chunk by chunk)
  void setRenderPolicy(bool wholeFrame)
  {
    settle();
    whole_frame = wholeFrame;
    if (whole_frame && !d_spec && d_capacity) rfx_dropin::check(rfx_device_alloc(r, d_capacity, &d_spec), "Render");
  }
};
