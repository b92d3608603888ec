// reflaxman/dropin/Scene.h -- drop-in replacement for the reference's src/common/Scene.h.
//
// Same class name and public API as the reference (Scene.h:28-40): Scene(), Scene(diffLightColor,
// diffLightPower), addSphere -> Sphere*, addTriangle -> Triangle*, addLight -> OmniLight*, addTexture ->
// Texture*, setSkyboxTexture -> bool.  The scene is recorded through the C-ABI (../../rfx.h), which runs the
// reference's host precompute (Sphere.cpp:9-20, Triangle.cpp:11-21/110-120, OmniLight.cpp:8-14,
// Material.cpp:8-14, Skybox.cpp:21-37) and uploads it; the trace itself runs in the MI355X kernels.
//
// The caller keeps compiling the reference's value types from its own sources -- Vector3, Matrix33,
// Color, Material, OmniLight, Texture, Camera -- and includes them from its own tree; Sphere, Triangle,
// SceneObject, Skybox, Plane and Scene::trace are not needed (their .cpp files leave the build).  See
// INTEGRATION.md ("Drop-in for the reference's own caller").
//
// Differences a well-behaved caller cannot see: Scene is movable, not copyable (the reference's implicit
// copy double-deletes, so its callers only ever assign a fresh temporary: Render.cpp:32); Sphere and
// Triangle are handles (the caller never calls trace() on them: Scene::trace is the renderer's).
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rfx.h"  // -I <repo>/include
#include "Color.h"
#include "Material.h"
#include "OmniLight.h"
#include "Texture.h"
#include "Vector3.h"

namespace rfx_dropin {
inline void check(int rc, const char *what)
{
  if (rc < 0) throw std::runtime_error(std::string(what) + ": " + rfx_last_error());
}
inline void rgb(const Color &c, float out[3]) { out[0] = c.r; out[1] = c.g; out[2] = c.b; }
inline void xyz(const Vector3 &v, float out[3]) { out[0] = v.x; out[1] = v.y; out[2] = v.z; }
}  // namespace rfx_dropin

class Scene;

// Scene::addSphere's Sphere* (Sphere.h): a handle of the sphere's object index.
class Sphere {
 public:
  Sphere(Scene *s, int obj) : scene(s), object(obj) {}
  int objectIndex() const { return object; }

 private:
  friend class Scene;
  Scene *scene;
  int object;
};

// Scene::addTriangle's Triangle* (Triangle.h): setTexture as Triangle.cpp:110-120.
class Triangle {
 public:
  Triangle(Scene *s, int obj) : scene(s), object(obj) {}
  inline void setTexture(const Texture *texture, const float u1, const float v1, const float u2, const float v2,
                         const float u3, const float v3);
  int objectIndex() const { return object; }

 private:
  friend class Scene;
  Scene *scene;
  int object;
};

class Scene {
 public:
  Scene() : h(rfx_scene_create(0.0f, 0.0f, 0.0f, 0.0f)) { bump(); }
  Scene(const Color &diffLightColor, float diffLightPower)
      : h(rfx_scene_create(diffLightColor.r, diffLightColor.g, diffLightColor.b, diffLightPower)) { bump(); }
  ~Scene() { release(); }
  Scene(const Scene &) = delete;
  Scene &operator=(const Scene &) = delete;
  Scene(Scene &&o) noexcept { take(o); }
  Scene &operator=(Scene &&o) noexcept
  {
    if (this != &o)
    {
      release();
      take(o);
    }
    return *this;
  }

  Sphere *addSphere(const Vector3 &center, float radius, const Material &material)  // Scene.cpp:29-39
  {
    float c[3], col[3];
    rfx_dropin::xyz(center, c);
    rfx_dropin::rgb(material.color, col);
    const int obj = rfx_scene_add_sphere(h, c, radius, material.type == Material::mtDielectric ? RFX_DIELECTRIC : RFX_METAL,
                                         col, material.reflectivity, material.transparency);
    rfx_dropin::check(obj, "Scene::addSphere");
    bump();
    spheres.emplace_back(new Sphere(this, obj));
    return spheres.back().get();
  }

  Triangle *addTriangle(const Vector3 &v1, const Vector3 &v2, const Vector3 &v3, const Material &material)
  {                                                                                     // Scene.cpp:41-46
    float a[3], b[3], c[3], col[3];
    rfx_dropin::xyz(v1, a);
    rfx_dropin::xyz(v2, b);
    rfx_dropin::xyz(v3, c);
    rfx_dropin::rgb(material.color, col);
    const int obj = rfx_scene_add_triangle(h, a, b, c, material.type == Material::mtDielectric ? RFX_DIELECTRIC : RFX_METAL,
                                           col, material.reflectivity, material.transparency);
    rfx_dropin::check(obj, "Scene::addTriangle");
    bump();
    triangles.emplace_back(new Triangle(this, obj));
    return triangles.back().get();
  }

  OmniLight *addLight(const Vector3 &origin, float radius, const Color &color, float power)  // Scene.cpp:48-59
  {
    float o[3], col[3];
    rfx_dropin::xyz(origin, o);
    rfx_dropin::rgb(color, col);
    rfx_dropin::check(rfx_scene_add_light(h, o, radius, col, power), "Scene::addLight");
    bump();
    if (radius <= 1.0842021724855044e-19f) radius = 1.0842021724855044e-19f;  // VERY_SMALL_NUMBER clamp, Scene.cpp:50-53
    lights.emplace_back(new OmniLight(origin, radius, color, power));  // the caller's record, as the reference returns
    return lights.back().get();
  }

  // Scene.cpp:61-66: the texture is read by the library's TGA reader (Texture.cpp:34-108 semantics; a failed
  // load is the checker texture) and the caller's own Texture(fileName) is returned as the handle, exactly
  // the object the reference would have returned.
  Texture *addTexture(const char *fileName)
  {
    const int idx = rfx_scene_add_texture_file(h, fileName, nullptr);
    rfx_dropin::check(idx, "Scene::addTexture");
    bump();
    textures.emplace_back(new Texture(fileName));
    texture_index[textures.back().get()] = idx;
    return textures.back().get();
  }

  bool setSkyboxTexture(const char *fileName)  // Scene.cpp:68-71
  {
    const int ok = rfx_scene_set_skybox_file(h, fileName);
    rfx_dropin::check(ok, "Scene::setSkyboxTexture");
    bump();
    return ok == 1;
  }

  // renderer side
  rfx_scene *handle() const { return h; }
  unsigned long long revision() const { return version; }
  void touch() { bump(); }
  int textureIndex(const Texture *t) const
  {
    const std::map<const Texture *, int>::const_iterator it = texture_index.find(t);
    return it == texture_index.end() ? -1 : it->second;
  }

 private:
  void release()
  {
    if (h) rfx_scene_destroy(h);
    h = nullptr;
    spheres.clear();
    triangles.clear();
    lights.clear();
    textures.clear();
    texture_index.clear();
  }
  void take(Scene &o)
  {
    h = o.h;
    o.h = nullptr;
    spheres = std::move(o.spheres);
    triangles = std::move(o.triangles);
    lights = std::move(o.lights);
    textures = std::move(o.textures);
    texture_index = std::move(o.texture_index);
    for (auto &sp : spheres) sp->scene = this;  // the handles belong to this scene now
    for (auto &tr : triangles) tr->scene = this;
    bump();
  }
  // Revisions come from one process-wide counter, so no two states of any Scene object share one: Render::renderNext
  // re-uploads whenever the revision differs from the uploaded one (a freshly assigned Scene included).
  void bump()
  {
    static std::atomic<unsigned long long> counter(0);
    version = ++counter;
  }

  rfx_scene *h = nullptr;
  std::vector<std::unique_ptr<Sphere>> spheres;
  std::vector<std::unique_ptr<Triangle>> triangles;
  std::vector<std::unique_ptr<OmniLight>> lights;
  std::vector<std::unique_ptr<Texture>> textures;
  std::map<const Texture *, int> texture_index;
  unsigned long long version = 0;
};

inline void Triangle::setTexture(const Texture *texture, const float u1, const float v1, const float u2, const float v2,
                                 const float u3, const float v3)
{
  const float uv[6] = {u1, v1, u2, v2, u3, v3};
  rfx_dropin::check(rfx_triangle_set_texture(scene->handle(), object, scene->textureIndex(texture), uv),
                    "Triangle::setTexture");
  scene->touch();
}
