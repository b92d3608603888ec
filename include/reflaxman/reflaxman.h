// reflaxman/reflaxman.h -- header-only C++ host shim over the C-ABI (../rfx.h), for hosts that do NOT
// keep the reference's sources.  (A host that does -- the reference's own Pulse app -- uses the drop-in
// headers reflaxman/dropin/{Render,Scene}.h instead, with its own Camera/Color/Texture/...; INTEGRATION.md.)
//
// Mirrors the reference's class API so host code written against
// src/common/{Render,Scene,Camera,Material,Color,Vector3,Texture}.h recompiles
// against this header (namespace reflaxman; `using namespace reflaxman;`)
// and renders on the MI355X instead of the CPU:
//
//   Render (Render.h:7-42)   public camera/scene/imageWidth/imageHeight/additiveCounter/inProgress,
//                            setImageSize, renderBegin, renderNext, renderAll, copyImage,
//                            imagePixel, getRenderProgress, loadScene
//   Scene (Scene.h:28-40)    ctor(Color, float), addSphere -> Sphere*, addTriangle -> Triangle*,
//                            addLight -> OmniLight*, addTexture -> Texture*, setSkyboxTexture
//   Triangle::setTexture (Triangle.h:16), Camera(eye, at, fov) (Camera.h:55), Material (Material.h),
//   Texture (Texture.h): W x H ARGB buffer, Texture(fileName) (TGA), saveToFile (.bmp / .tga), clear
//
// Differences that are not visible to a well-behaved caller: Scene/Render are
// non-copyable (the reference's implicit shallow copies double-free), and
// errors surface as rfx_status / std::runtime_error instead of assert().
// Link: -lrfx (reflaxman_amd/lib/librfx.so).
#pragma once
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../rfx.h"

namespace reflaxman {

inline void rfx_check(int rc, const char *what)
{
  if (rc < 0) throw std::runtime_error(std::string(what) + ": " + rfx_last_error());
}

struct Vector3 {
  float x, y, z;
  Vector3() : x(0), y(0), z(0) {}
  Vector3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};

typedef uint32_t ARGB;

struct Color {
  float r, g, b;
  Color() : r(0), g(0), b(0) {}
  Color(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
  ARGB argb() const  // Color.cpp:114-117
  {
    ARGB out;
    const float c[3] = {r, g, b};
    rfx_argb_from_rgb(c, 1, &out);
    return out;
  }
};

struct Material {  // Material.h:5-19 (clamping is applied by the library, Material.cpp:8-14)
  enum Type { mtMetal = RFX_METAL, mtDielectric = RFX_DIELECTRIC };
  Type type;
  Color color;
  float reflectivity, transparency;
  Material() : type(mtMetal), reflectivity(0), transparency(0) {}
  Material(Type t, const Color &c, float refl, float transp) : type(t), color(c), reflectivity(refl), transparency(transp) {}
};

struct Camera {  // Camera.h:30-62 (rendering fields)
  float fov;
  Vector3 eye;
  float view[9];  // Matrix33 row-major _11.._33
  Camera() : fov(0) { for (float &v : view) v = 0; }
  Camera(const Vector3 &eye_, const Vector3 &at, float fov_) : fov(fov_), eye(eye_)
  {
    const float e[3] = {eye_.x, eye_.y, eye_.z}, a[3] = {at.x, at.y, at.z};
    rfx_camera_view(e, a, view);
  }
};

class Texture {  // Texture.h:4-34 (image side: W x H ARGB, TGA load, BMP/TGA save)
 public:
  Texture() : width(0), height(0) {}
  Texture(unsigned w, unsigned h) : width(w), height(h), buf((size_t)w * h, 0) {}
  explicit Texture(const char *fileName) : width(0), height(0) { loadFromFile(fileName); }
  bool loadFromFile(const char *fileName)  // Texture.cpp:175-189 (.tga only), Texture.cpp:34-108
  {
    const std::string f = fileName;
    const size_t dot = f.find_last_of('.');
    width = height = 0;
    buf.clear();
    if (dot == std::string::npos || f.substr(dot) != ".tga") return false;
    uint32_t w = 0, h = 0;
    if (rfx_tga_load(fileName, &w, &h, nullptr, 0) != RFX_OK) return false;
    buf.assign((size_t)w * h, 0);
    if ((size_t)w * h && rfx_tga_load(fileName, &w, &h, buf.data(), buf.size()) != RFX_OK) { buf.clear(); return false; }
    width = w;
    height = h;
    return true;
  }
  void clear(ARGB bkColor) { for (ARGB &c : buf) c = bkColor; }  // Texture.cpp:278-283
  unsigned getWidth() const { return width; }
  unsigned getHeight() const { return height; }
  ARGB *getColorBuffer() { return buf.data(); }
  const ARGB *getColorBuffer() const { return buf.data(); }
  bool saveToFile(const char *fileName) const  // Texture.cpp:195-207
  {
    const std::string f = fileName;
    const size_t dot = f.find_last_of('.');
    if (dot == std::string::npos) return false;
    const std::string ext = f.substr(dot);
    if (ext == ".tga") return rfx_tga_save(fileName, width, height, buf.data()) == RFX_OK;
    if (ext == ".bmp") return rfx_bmp_save(fileName, width, height, buf.data()) == RFX_OK;
    return false;
  }

 private:
  unsigned width, height;
  std::vector<ARGB> buf;
};

class Scene;

class Sphere {  // Scene::addSphere's Sphere*: a handle of the object index
 public:
  Sphere(Scene *s, int obj) : scene(s), object(obj) {}
  int objectIndex() const { return object; }

 private:
  Scene *scene;
  int object;
};

struct OmniLight {  // Scene::addLight's OmniLight* (OmniLight.h): the light as recorded (radius/power clamped)
  Vector3 origin;
  float radius;
  Color color;
  float power;
};

class Triangle {  // Scene::addTriangle's Triangle*
 public:
  Triangle(Scene *s, int obj) : scene(s), object(obj) {}
  inline void setTexture(const Texture *texture, float u1, float v1, float u2, float v2, float u3, float v3);
  int objectIndex() const { return object; }

 private:
  Scene *scene;
  int object;
};

class Scene {
 public:
  Scene() : h(rfx_scene_create(0, 0, 0, 0)) {}
  Scene(const Color &diffLightColor, float diffLightPower)
      : h(rfx_scene_create(diffLightColor.r, diffLightColor.g, diffLightColor.b, diffLightPower)) {}
  ~Scene() { rfx_scene_destroy(h); }
  Scene(const Scene &) = delete;
  Scene &operator=(const Scene &) = delete;
  Scene &operator=(Scene &&o) noexcept
  {
    std::swap(h, o.h);
    std::swap(spheres, o.spheres);
    std::swap(tris, o.tris);
    std::swap(lights, o.lights);
    std::swap(texs, o.texs);
    std::swap(tex_index, o.tex_index);
    ++version;
    return *this;
  }

  Sphere *addSphere(const Vector3 &c, float radius, const Material &m)  // Scene.cpp:29-39
  {
    const float cc[3] = {c.x, c.y, c.z}, rgb[3] = {m.color.r, m.color.g, m.color.b};
    const int obj = rfx_scene_add_sphere(h, cc, radius, m.type, rgb, m.reflectivity, m.transparency);
    rfx_check(obj, "Scene::addSphere");
    ++version;
    spheres.emplace_back(new Sphere(this, obj));
    return spheres.back().get();
  }
  Triangle *addTriangle(const Vector3 &v1, const Vector3 &v2, const Vector3 &v3, const Material &m)
  {
    const float a[3] = {v1.x, v1.y, v1.z}, b[3] = {v2.x, v2.y, v2.z}, c[3] = {v3.x, v3.y, v3.z};
    const float rgb[3] = {m.color.r, m.color.g, m.color.b};
    const int obj = rfx_scene_add_triangle(h, a, b, c, m.type, rgb, m.reflectivity, m.transparency);
    rfx_check(obj, "Scene::addTriangle");
    ++version;
    tris.emplace_back(new Triangle(this, obj));
    return tris.back().get();
  }
  OmniLight *addLight(const Vector3 &o, float radius, const Color &c, float power)  // Scene.cpp:48-59
  {
    const float oo[3] = {o.x, o.y, o.z}, rgb[3] = {c.r, c.g, c.b};
    const int idx = rfx_scene_add_light(h, oo, radius, rgb, power);
    rfx_check(idx, "Scene::addLight");
    ++version;
    if (radius <= 1.0842021724855044e-19f) radius = 1.0842021724855044e-19f;  // Scene.cpp:50-53
    const float p = power < 0.0f ? 0.0f : power > 1.0f ? 1.0f : power;     // OmniLight.cpp:13
    lights.emplace_back(new OmniLight{o, radius, c, p});
    return lights.back().get();
  }
  Texture *addTexture(const char *fileName)  // Scene.cpp:61-66: failed loads give the checker texture
  {
    const int idx = rfx_scene_add_texture_file(h, fileName, nullptr);
    rfx_check(idx, "Scene::addTexture");
    ++version;
    texs.emplace_back(new Texture(fileName));
    tex_index.emplace_back(texs.back().get(), idx);
    return texs.back().get();
  }
  int textureIndex(const Texture *t) const
  {
    for (const auto &e : tex_index)
      if (e.first == t) return e.second;
    return -1;
  }
  bool setSkyboxTexture(const char *fileName)
  {
    const int ok = rfx_scene_set_skybox_file(h, fileName);
    rfx_check(ok, "Scene::setSkyboxTexture");
    ++version;
    return ok == 1;
  }
  rfx_scene *handle() const { return h; }
  unsigned long long revision() const { return version; }
  void touch() { ++version; }

 private:
  rfx_scene *h;
  std::vector<std::unique_ptr<Sphere>> spheres;
  std::vector<std::unique_ptr<Triangle>> tris;
  std::vector<std::unique_ptr<OmniLight>> lights;
  std::vector<std::unique_ptr<Texture>> texs;
  std::vector<std::pair<const Texture *, int>> tex_index;
  unsigned long long version = 0;
};

inline void Triangle::setTexture(const Texture *t, float u1, float v1, float u2, float v2, float u3, float v3)
{
  const float uv[6] = {u1, v1, u2, v2, u3, v3};
  rfx_check(rfx_triangle_set_texture(scene->handle(), object, scene->textureIndex(t), uv), "Triangle::setTexture");
  scene->touch();
}

class Render {  // Render.h:7-42
 public:
  Camera camera;
  Scene scene;
  unsigned imageWidth = 0, imageHeight = 0;
  int additiveCounter = 0;
  bool inProgress = false;

  explicit Render(const char *exePath, int device = 0, uint32_t sphereSeed = 1350490027u, uint32_t jitterSeed = 424238335u)
  {
    rfx_check(rfx_renderer_create(&r, device), "rfx_renderer_create");
    rfx_check(rfx_renderer_set_rng(r, sphereSeed, jitterSeed), "rfx_renderer_set_rng");
    loadScene(exePath);
  }
  ~Render()
  {
    if (d_img) rfx_device_free(r, d_img);
    rfx_renderer_destroy(r);
  }
  Render(const Render &) = delete;
  Render &operator=(const Render &) = delete;

  void loadScene(const char *exePath)  // Render.cpp:25-55
  {
    const std::string sky = std::string(exePath) + "./textures/skybox.tga";
    const std::string plane = std::string(exePath) + "./textures/himiya.tga";
    camera = Camera(Vector3(7.427f, 3.494f, -3.773f), Vector3(6.5981f, 3.127f, -3.352f), 1.05f);
    scene = Scene(Color(0.95f, 0.95f, 1.0f), 0.15f);
    scene.setSkyboxTexture(sky.c_str());
    scene.addLight(Vector3(11.8e9f, 4.26e9f, 3.08e9f), 3.48e8f, Color(1.0f, 1.0f, 0.95f), 0.85f);
    scene.addSphere(Vector3(-1.25f, 1.5f, -0.25f), 1.5f, Material(Material::mtMetal, Color(1.0f, 1.0f, 1.0f), 1.0f, 0.0f));
    scene.addSphere(Vector3(0.15f, 1.0f, 1.75f), 1.0f, Material(Material::mtMetal, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    scene.addSphere(Vector3(-3.0f, 0.6f, -3.0f), 0.6f, Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.0f, 0.0f));
    scene.addSphere(Vector3(-0.5f, 0.5f, -2.5f), 0.5f, Material(Material::mtDielectric, Color(0.5f, 1.0f, 0.15f), 0.75f, 0.0f));
    scene.addSphere(Vector3(1.0f, 0.4f, -1.5f), 0.4f, Material(Material::mtDielectric, Color(0.0f, 0.5f, 1.0f), 1.0f, 0.0f));
    scene.addSphere(Vector3(1.8f, 0.4f, 0.1f), 0.4f, Material(Material::mtMetal, Color(1.0f, 0.65f, 0.45f), 1.0f, 0.0f));
    scene.addSphere(Vector3(1.7f, 0.5f, 1.9f), 0.5f, Material(Material::mtMetal, Color(1.0f, 0.90f, 0.60f), 0.75f, 0.0f));
    scene.addSphere(Vector3(0.6f, 0.6f, 4.2f), 0.6f, Material(Material::mtMetal, Color(0.9f, 0.9f, 0.9f), 0.0f, 0.0f));
    Texture *planeTexture = scene.addTexture(plane.c_str());
    Triangle *tr1 = scene.addTriangle(Vector3(-14.0f, 0.0f, -10.0f), Vector3(-14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, -10.0f),
                                      Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    tr1->setTexture(planeTexture, 0.0f, 0.0f, 0.0f, 1.0f, 1.0f, 0.0f);
    Triangle *tr2 = scene.addTriangle(Vector3(-14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, 10.0f), Vector3(14.0f, 0.0f, -10.0f),
                                      Material(Material::mtDielectric, Color(1.0f, 1.0f, 1.0f), 0.95f, 0.0f));
    tr2->setTexture(planeTexture, 0.0f, 1.0f, 1.0f, 1.0f, 1.0f, 0.0f);
  }

  void setImageSize(unsigned width, unsigned height)  // Render.cpp:57-80
  {
    if (!width || !height) return;
    const size_t bytes = (size_t)width * height * 12;
    if (bytes > cap)
    {
      if (d_img) rfx_device_free(r, d_img);
      d_img = nullptr;
      rfx_check(rfx_device_alloc(r, bytes, &d_img), "setImageSize");
      cap = bytes;
    }
    std::vector<float> zero((size_t)width * height * 3, 0.0f);
    rfx_check(rfx_memcpy_h2d(r, d_img, zero.data(), bytes), "setImageSize");
    imageWidth = width;
    imageHeight = height;
    additiveCounter = 0;
    inProgress = false;
    curx = cury = 0;
    host_valid = false;
  }

  void renderBegin(int reflectNum, int sampleNum, bool additive)  // Render.cpp:116-134
  {
    refl = reflectNum;
    ss = sampleNum;
    add = additive;
    inProgress = true;
    curx = cury = 0;
    staged = camera;
    additiveCounter = additive ? additiveCounter + 1 : 0;
  }

  bool renderNext(unsigned pixels)  // Render.cpp:136-215: renders exactly the cursor's span on the GPU
  {
    if (!pixels || !inProgress || curx >= imageWidth || cury >= imageHeight) return false;
    const uint64_t total = (uint64_t)imageWidth * imageHeight;
    const uint64_t p0 = (uint64_t)cury * imageWidth + curx;
    const uint64_t p1 = p0 + pixels < total ? p0 + pixels : total;
    if (uploaded != scene.revision())
    {
      rfx_check(rfx_renderer_set_scene(r, scene.handle()), "rfx_renderer_set_scene");
      uploaded = scene.revision();
    }
    rfx_frame f = {};
    for (int i = 0; i < 3; ++i) f.eye[i] = (&staged.eye.x)[i];
    for (int i = 0; i < 9; ++i) f.view[i] = staged.view[i];
    f.fov = camera.fov;  // rz uses the live camera's fov (Render.cpp:148)
    f.width = imageWidth;
    f.height = imageHeight;
    f.reflect_num = refl;
    f.sample_num = ss;
    f.additive = add;
    f.additive_counter = additiveCounter;
    f.nranks = 1;
    f.pixel_begin = p0;
    f.pixel_end = p1;
    rfx_check(rfx_render_frame(r, &f, (float *)d_img, nullptr, nullptr, nullptr), "renderNext");
    host_valid = false;
    curx = (unsigned)(p1 % imageWidth);
    cury = (unsigned)(p1 / imageWidth);
    if (p1 == total) inProgress = false;
    return inProgress;
  }

  void renderAll(int reflectNum, int sampleNum, bool additive)  // Render.cpp:217-221, as shipped
  {
    renderBegin(reflectNum, sampleNum, additive);
    renderNext(imageHeight);
  }

  Color imagePixel(int x, int y) const  // Render.cpp:103-114
  {
    if (x < 0 || y < 0) return Color(0, 0, 0);
    const float *c = &host()[((size_t)y * imageWidth + x) * 3];
    if (additiveCounter > 1)
    {
      const float k = float(additiveCounter);
      return Color(c[0] / k, c[1] / k, c[2] / k);
    }
    return Color(c[0], c[1], c[2]);
  }

  void copyImage(Texture &texture) const  // Render.cpp:82-101
  {
    if (texture.getWidth() != imageWidth || texture.getHeight() != imageHeight)
    {
      texture.clear(0);
      return;
    }
    rfx_argb_from_rgb(host().data(), (size_t)imageWidth * imageHeight, texture.getColorBuffer());
  }

  float getRenderProgress() const  // Render.cpp:223-226
  {
    return float(curx + cury * imageWidth) * 100.0f / imageWidth / imageHeight;
  }

  rfx_renderer *handle() const { return r; }

 private:
  const std::vector<float> &host() const
  {
    if (!host_valid)
    {
      image.resize((size_t)imageWidth * imageHeight * 3);
      rfx_check(rfx_memcpy_d2h(r, image.data(), d_img, image.size() * 4), "image readback");
      host_valid = true;
    }
    return image;
  }

  rfx_renderer *r = nullptr;
  void *d_img = nullptr;
  size_t cap = 0;
  unsigned curx = 0, cury = 0;
  int refl = 0, ss = 0;
  bool add = false;
  Camera staged;
  unsigned long long uploaded = ~0ull;
  mutable std::vector<float> image;
  mutable bool host_valid = false;
};

}  // namespace reflaxman
