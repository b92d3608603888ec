/*
 * ORACLE TEST INFRASTRUCTURE -- never shipped, never linked into the product.
 *
 * Headless driver for the *unmodified* ReflaxMan reference sources
 * (/root/reference/src/common/*.cpp), compiled by oracle/Makefile into
 * oracle/_ref/refharness.  It only calls the reference's public API:
 *   Render ctor / setImageSize / renderBegin / renderNext / imagePixel / copyImage
 *       (src/common/Render.cpp:5-226)
 *   Scene ctor / addSphere / addTriangle / addLight / addTexture / setSkyboxTexture
 *       (src/common/Scene.cpp:10-71), Triangle::setTexture (Triangle.cpp:110-120)
 *   Sphere/Triangle/Plane::trace, Skybox::getTexelColor, Texture::getTexelColor,
 *   Color::argb, Vector3::randomInsideSphere, Camera ctor  (KAT modes)
 *   Texture(fileName) / loadFromFile, Texture(w, h) + saveToFile (file-format modes)
 * Scene has no addPlane; a scene file's "plane" line puts a reference Plane (Plane.cpp) into the Scene's
 * object list through a pointer to that private member (formed by the explicit-instantiation rule of
 * [temp.explicit], no source change), so the reference's own Scene::trace renders it.
 * Used to generate tests/golden/* and, on the GPU box, as the timed
 * "reference" CPU baseline of bench.py.
 *
 * Scene files are the repo's plain-text scene description (see
 * reflaxman_amd/scenes.py); floats are C99 hex literals so both sides read the
 * exact same bits.
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "trace_math.h"
#include "Render.h"
#include "Plane.h"
#include "Skybox.h"

// Scene::sceneObjects (Scene.h:15-19) is private and Scene has no addPlane: a pointer to the member, formed in
// an explicit template instantiation (where access checking does not apply), lets the harness append a Plane.
typedef std::vector<SceneObject *> Scene::*SceneObjectsPtr;
template <SceneObjectsPtr M>
struct SceneObjectsAccess {
  friend SceneObjectsPtr scene_objects_member() { return M; }
};
SceneObjectsPtr scene_objects_member();
template struct SceneObjectsAccess<&Scene::sceneObjects>;

static void die(const char *msg) { fprintf(stderr, "refharness: %s\n", msg); exit(2); }

static std::vector<char> read_file(const char *path)
{
  FILE *f = fopen(path, "rb");
  if (!f) die("cannot open input");
  std::vector<char> buf;
  char tmp[1 << 16];
  size_t n;
  while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
  fclose(f);
  return buf;
}

static void write_file(const std::string &path, const void *data, size_t bytes)
{
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) die("cannot open output");
  if (bytes && fwrite(data, bytes, 1, f) != 1) die("short write");
  fclose(f);
}

static std::string dir_of(const std::string &p)
{
  size_t s = p.find_last_of('/');
  return s == std::string::npos ? std::string("./") : p.substr(0, s + 1);
}

static std::string tex_path(const std::string &dir, const char *tok)
{
  if (!strcmp(tok, "-")) return "/nonexistent/absent.tga";  // -> checker fallback (Texture.cpp:242-243)
  if (tok[0] == '/') return tok;
  return dir + tok;
}

// Build r.scene / r.camera from a scene file (or keep Render::loadScene's default scene).
static void load_scene(Render &r, const char *scene_arg)
{
  if (!strcmp(scene_arg, "default")) return;  // Render ctor already ran loadScene (Render.cpp:25-55)
  std::vector<char> text = read_file(scene_arg);
  text.push_back('\0');
  const std::string dir = dir_of(scene_arg);
  std::vector<Triangle *> objects_tri;  // object index -> Triangle* (NULL for spheres)
  std::vector<Texture *> textures;
  char *save = NULL;
  for (char *line = strtok_r(&text[0], "\n", &save); line; line = strtok_r(NULL, "\n", &save))
  {
    char kw[32];
    if (sscanf(line, "%31s", kw) != 1 || kw[0] == '#') continue;
    const char *p = line + strlen(kw);
    std::vector<float> f;
    char tok[1024] = {0};
    if (!strcmp(kw, "skybox") || !strcmp(kw, "texture"))
    {
      if (sscanf(p, "%1023s", tok) != 1) die("bad texture line");
    }
    else
    {
      char *end;
      for (;;)
      {
        float v = strtof(p, &end);
        if (end == p) break;
        f.push_back(v);
        p = end;
      }
    }
    if (!strcmp(kw, "diffuse")) { if (f.size() != 4) die("diffuse"); r.scene = Scene(Color(f[0], f[1], f[2]), f[3]); }
    else if (!strcmp(kw, "camera")) { if (f.size() != 7) die("camera"); r.camera = Camera(Vector3(f[0], f[1], f[2]), Vector3(f[3], f[4], f[5]), f[6]); }
    else if (!strcmp(kw, "skybox")) { r.scene.setSkyboxTexture(tex_path(dir, tok).c_str()); }
    else if (!strcmp(kw, "texture")) { textures.push_back(r.scene.addTexture(tex_path(dir, tok).c_str())); }
    else if (!strcmp(kw, "light")) { if (f.size() != 8) die("light"); r.scene.addLight(Vector3(f[0], f[1], f[2]), f[3], Color(f[4], f[5], f[6]), f[7]); }
    else if (!strcmp(kw, "sphere"))
    {
      if (f.size() != 10) die("sphere");
      r.scene.addSphere(Vector3(f[0], f[1], f[2]), f[3],
                        Material(f[4] != 0.0f ? Material::mtDielectric : Material::mtMetal, Color(f[5], f[6], f[7]), f[8], f[9]));
      objects_tri.push_back(NULL);
    }
    else if (!strcmp(kw, "triangle"))
    {
      if (f.size() != 15) die("triangle");
      objects_tri.push_back(r.scene.addTriangle(Vector3(f[0], f[1], f[2]), Vector3(f[3], f[4], f[5]), Vector3(f[6], f[7], f[8]),
                        Material(f[9] != 0.0f ? Material::mtDielectric : Material::mtMetal, Color(f[10], f[11], f[12]), f[13], f[14])));
    }
    else if (!strcmp(kw, "plane"))
    {
      if (f.size() != 12) die("plane");
      Plane *pl = new Plane(Vector3(f[0], f[1], f[2]), Vector3(f[3], f[4], f[5]),
                            Material(f[6] != 0.0f ? Material::mtDielectric : Material::mtMetal, Color(f[7], f[8], f[9]), f[10], f[11]));
      (r.scene.*scene_objects_member()).push_back(pl);  // owned and deleted by ~Scene (Scene.cpp:17-27)
      objects_tri.push_back(NULL);
    }
    else if (!strcmp(kw, "settex"))
    {
      if (f.size() != 8) die("settex");
      size_t oi = (size_t)f[0], ti = (size_t)f[1];
      if (oi >= objects_tri.size() || !objects_tri[oi] || ti >= textures.size()) die("settex index");
      objects_tri[oi]->setTexture(textures[ti], f[2], f[3], f[4], f[5], f[6], f[7]);
    }
    else die("unknown scene keyword");
  }
}

static void dump_image(Render &r, unsigned W, unsigned H, const std::string &out)
{
  std::vector<float> rgb((size_t)W * H * 3);
  for (unsigned y = 0; y < H; ++y)
    for (unsigned x = 0; x < W; ++x)
    {
      Color c = r.imagePixel(x, y);
      float *d = &rgb[((size_t)y * W + x) * 3];
      d[0] = c.r; d[1] = c.g; d[2] = c.b;
    }
  write_file(out + ".f32", &rgb[0], rgb.size() * 4);
  Texture t(W, H);
  r.copyImage(t);
  write_file(out + ".argb", t.getColorBuffer(), (size_t)W * H * 4);
}

static Material kat_material(float type, float cr, float cg, float cb, float refl)
{
  return Material(type != 0.0f ? Material::mtDielectric : Material::mtMetal, Color(cr, cg, cb), refl, 0.0f);
}

int main(int argc, char **argv)
{
  if (argc < 2) die("usage: refharness <mode> ...");
  const std::string mode = argv[1];
  Render r("/nonexistent/");  // textures absent -> procedural checker (Texture.cpp:242-243)

  if (mode == "render")
  {
    // render SCENE W H DEPTH SS ADDITIVE FRAMES OUT
    if (argc != 10) die("render SCENE W H DEPTH SS ADDITIVE FRAMES OUT");
    load_scene(r, argv[2]);
    unsigned W = atoi(argv[3]), H = atoi(argv[4]);
    int depth = atoi(argv[5]), ss = atoi(argv[6]);
    bool additive = atoi(argv[7]) != 0;
    int frames = atoi(argv[8]);
    r.setImageSize(W, H);
    for (int fr = 0; fr < frames; ++fr)
    {
      r.renderBegin(depth, ss, additive);
      while (r.renderNext(W * H)) {}
    }
    dump_image(r, W, H, argv[9]);
    return 0;
  }
  if (mode == "band")
  {
    // band SCENE W H DEPTH Y0 ROWS OUT : rows [Y0, Y0+ROWS) of a ss=1 frame, stream advanced to the band start.
    if (argc != 9) die("band SCENE W H DEPTH Y0 ROWS OUT");
    load_scene(r, argv[2]);
    unsigned W = atoi(argv[3]), H = atoi(argv[4]);
    int depth = atoi(argv[5]);
    unsigned y0 = atoi(argv[6]), rows = atoi(argv[7]);
    for (size_t i = 0; i < (size_t)y0 * W; ++i) Vector3::randomInsideSphere(1.0f);
    // ray construction exactly as Render::renderNext (Render.cpp:146-156,164-165, ss=1)
    const float rz = float(W) / 2.0f / tanf(r.camera.fov / 2.0f);
    const float wh = W / 2.0f, hh = H / 2.0f;
    std::vector<float> rgb((size_t)W * rows * 3);
    std::vector<ARGB> argb((size_t)W * rows);
    for (unsigned y = y0; y < y0 + rows; ++y)
      for (unsigned x = 0; x < W; ++x)
      {
        Vector3 ray(float(x) - wh, float(y) - hh, rz);
        ray = r.camera.view * ray;
        Color c = r.scene.trace(r.camera.eye, ray, depth);
        size_t i = (size_t)(y - y0) * W + x;
        rgb[i * 3 + 0] = c.r; rgb[i * 3 + 1] = c.g; rgb[i * 3 + 2] = c.b;
        argb[i] = c.argb();
      }
    write_file(std::string(argv[8]) + ".f32", &rgb[0], rgb.size() * 4);
    write_file(std::string(argv[8]) + ".argb", &argb[0], argb.size() * 4);
    return 0;
  }
  if (mode == "bandss")
  {
    // bandss SCENE W H DEPTH SS FRAME Y0 ROWS OUT : rows [Y0, Y0+ROWS) of frame FRAME (0-based) of a sequence of
    // non-additive frames with SS x SS samples per pixel (SS >= 1), the stream advanced over every draw before the
    // band: FRAME whole frames and Y0 rows, SS*SS draws per pixel (one Scene::trace per sample, Scene.cpp:75).
    // Each pixel is computed exactly as Render::renderNext's renderSampleNum > 0 branch (Render.cpp:146-194) with
    // renderAdditive false: the reference's own Vector3/Matrix33/Color operators, in its order.  Bands of one frame
    // rendered by separate processes concatenate to the frame Render::renderNext produces (tools/gen_golden.py).
    if (argc != 11) die("bandss SCENE W H DEPTH SS FRAME Y0 ROWS OUT");
    load_scene(r, argv[2]);
    const unsigned W = atoi(argv[3]), H = atoi(argv[4]);
    const int depth = atoi(argv[5]), ss = atoi(argv[6]);
    const unsigned frame = atoi(argv[7]), y0 = atoi(argv[8]), rows = atoi(argv[9]);
    if (ss < 1 || y0 + (size_t)rows > H) die("bandss: bad ss or rows");
    const size_t spp = (size_t)ss * ss;
    const size_t skip = ((size_t)frame * W * H + (size_t)y0 * W) * spp;
    for (size_t i = 0; i < skip; ++i) Vector3::randomInsideSphere(1.0f);
    const Vector3 origin = r.camera.eye;
    const Matrix33 view = r.camera.view;
    const float sqRenderSampleNum = float(ss * ss);
    const float rz = float(W) / 2.0f / tanf(r.camera.fov / 2.0f);
    const float wh = W / 2.0f, hh = H / 2.0f;
    const float rndx = 0, rndy = 0;
    std::vector<float> rgb((size_t)W * rows * 3);
    std::vector<ARGB> argb((size_t)W * rows);
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (unsigned y = y0; y < y0 + rows; ++y)
      for (unsigned x = 0; x < W; ++x)
      {
        const float rx = float(x) - wh;
        const float ry = float(y) - hh;
        Color finColor = Color(0.0f, 0.0f, 0.0f);
        for (int ssx = 0; ssx < ss; ssx++)
          for (int ssy = 0; ssy < ss; ssy++)
          {
            Vector3 ray = Vector3(rx + float(ssx) / ss + rndx, ry + float(ssy) / ss + rndy, rz);
            ray = view * ray;
            finColor += r.scene.trace(origin, ray, depth);
          }
        finColor /= sqRenderSampleNum;
        const size_t i = (size_t)(y - y0) * W + x;
        rgb[i * 3 + 0] = finColor.r; rgb[i * 3 + 1] = finColor.g; rgb[i * 3 + 2] = finColor.b;
        argb[i] = finColor.argb();
      }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    write_file(std::string(argv[10]) + ".f32", &rgb[0], rgb.size() * 4);
    write_file(std::string(argv[10]) + ".argb", &argb[0], argb.size() * 4);
    // the band's trace time (the stream advance before it excluded): the timed CPU baseline of SSAA configs
    printf("{\"traced_samples\": %llu, \"trace_seconds\": %.6f}\n", (unsigned long long)W * rows * spp,
           (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec));
    return 0;
  }
  if (mode == "rows")
  {
    // rows SCENE W H DEPTH Y0 STRIDE COUNT OUT : rows Y0, Y0+STRIDE, ... of an ss=1 frame (bounded,
    // representative sample for the timed CPU baseline).  The stream is advanced over the skipped rows
    // outside the timed region; stdout reports the trace time of the sampled rows only.
    if (argc != 10) die("rows SCENE W H DEPTH Y0 STRIDE COUNT OUT");
    load_scene(r, argv[2]);
    unsigned W = atoi(argv[3]), H = atoi(argv[4]);
    int depth = atoi(argv[5]);
    unsigned y0 = atoi(argv[6]), stride = atoi(argv[7]), count = atoi(argv[8]);
    if (!stride || y0 + (size_t)(count - 1) * stride >= H) die("rows out of frame");
    const float rz = float(W) / 2.0f / tanf(r.camera.fov / 2.0f);
    const float wh = W / 2.0f, hh = H / 2.0f;
    std::vector<float> rgb((size_t)W * count * 3);
    std::vector<ARGB> argb((size_t)W * count);
    double traced = 0.0;
    unsigned next = 0;  // next row whose randDirs have not been drawn
    for (unsigned k = 0; k < count; ++k)
    {
      const unsigned y = y0 + k * stride;
      for (size_t i = (size_t)next * W; i < (size_t)y * W; ++i) Vector3::randomInsideSphere(1.0f);
      timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      for (unsigned x = 0; x < W; ++x)
      {
        Vector3 ray(float(x) - wh, float(y) - hh, rz);
        ray = r.camera.view * ray;
        Color c = r.scene.trace(r.camera.eye, ray, depth);
        size_t i = (size_t)k * W + x;
        rgb[i * 3 + 0] = c.r; rgb[i * 3 + 1] = c.g; rgb[i * 3 + 2] = c.b;
        argb[i] = c.argb();
      }
      clock_gettime(CLOCK_MONOTONIC, &t1);
      traced += (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
      next = y + 1;
    }
    write_file(std::string(argv[9]) + ".f32", &rgb[0], rgb.size() * 4);
    write_file(std::string(argv[9]) + ".argb", &argb[0], argb.size() * 4);
    printf("{\"traced_pixels\": %llu, \"trace_seconds\": %.6f}\n", (unsigned long long)W * count, traced);
    return 0;
  }
  if (mode == "rand")
  {
    // rand N OUT : the first N randDir draws of the Vector3.cpp stream
    if (argc != 4) die("rand N OUT");
    size_t n = strtoull(argv[2], NULL, 10);
    std::vector<float> v(n * 3);
    for (size_t i = 0; i < n; ++i)
    {
      Vector3 d = Vector3::randomInsideSphere(1.0f);
      v[i * 3] = d.x; v[i * 3 + 1] = d.y; v[i * 3 + 2] = d.z;
    }
    write_file(argv[3], &v[0], v.size() * 4);
    return 0;
  }
  if (mode == "kat_sphere" || mode == "kat_triangle" || mode == "kat_plane")
  {
    // kat_* IN OUT [TEX]: one object per record, full trace outputs.
    // sphere  record (11 f32): origin3 ray3 center3 radius pad
    // triangle record (21 f32): origin3 ray3 v0 3 v1 3 v2 3 uv6
    // plane   record (12 f32): origin3 ray3 pos3 norm3
    // out record (15 f32): hit(0/1) drop3 norm3 refl3 dist color3 any_hit(0/1)
    if (argc < 4) die("kat_* IN OUT [TEX]");
    std::vector<char> in = read_file(argv[2]);
    const float *f = (const float *)&in[0];
    size_t rec = mode == "kat_sphere" ? 11 : mode == "kat_triangle" ? 21 : 12;
    size_t n = in.size() / 4 / rec;
    Texture *tex = NULL;
    if (mode == "kat_triangle" && argc > 4) tex = new Texture(tex_path("", argv[4]).c_str());
    std::vector<float> out(n * 15, 0.0f);
    const Material mat = kat_material(0.0f, 0.25f, 0.5f, 0.75f, 0.5f);
    for (size_t i = 0; i < n; ++i, f += rec)
    {
      Vector3 o(f[0], f[1], f[2]), d(f[3], f[4], f[5]);
      Vector3 drop(0, 0, 0), norm(0, 0, 0), refl(0, 0, 0);
      float dist = 0;
      Material m = mat;
      bool hit, any;
      if (mode == "kat_sphere")
      {
        Sphere s(Vector3(f[6], f[7], f[8]), f[9], mat);
        hit = s.trace(o, d, &drop, &norm, &refl, &dist, &m);
        any = s.trace(o, d, NULL, NULL, NULL, NULL, NULL);
      }
      else if (mode == "kat_triangle")
      {
        Triangle t(Vector3(f[6], f[7], f[8]), Vector3(f[9], f[10], f[11]), Vector3(f[12], f[13], f[14]), mat);
        if (tex) t.setTexture(tex, f[15], f[16], f[17], f[18], f[19], f[20]);
        hit = t.trace(o, d, &drop, &norm, &refl, &dist, &m);
        any = t.trace(o, d, NULL, NULL, NULL, NULL, NULL);
      }
      else
      {
        Plane p(Vector3(f[6], f[7], f[8]), Vector3(f[9], f[10], f[11]), mat);
        hit = p.trace(o, d, &drop, &norm, &refl, &dist, &m);
        any = p.trace(o, d, NULL, NULL, NULL, NULL, NULL);
      }
      float *w = &out[i * 15];
      w[0] = hit ? 1.0f : 0.0f;
      if (hit)
      {
        w[1] = drop.x; w[2] = drop.y; w[3] = drop.z;
        w[4] = norm.x; w[5] = norm.y; w[6] = norm.z;
        w[7] = refl.x; w[8] = refl.y; w[9] = refl.z;
        w[10] = dist;
        w[11] = m.color.r; w[12] = m.color.g; w[13] = m.color.b;
      }
      w[14] = any ? 1.0f : 0.0f;
    }
    write_file(argv[3], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "kat_skybox")
  {
    // kat_skybox TEX IN OUT : ray3 -> color3
    if (argc != 5) die("kat_skybox TEX IN OUT");
    Skybox sky;
    sky.loadTexture(tex_path("", argv[2]).c_str());
    std::vector<char> in = read_file(argv[3]);
    const float *f = (const float *)&in[0];
    size_t n = in.size() / 12;
    std::vector<float> out(n * 3);
    for (size_t i = 0; i < n; ++i)
    {
      Color c = sky.getTexelColor(Vector3(f[i * 3], f[i * 3 + 1], f[i * 3 + 2]));
      out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
    }
    write_file(argv[4], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "kat_texture")
  {
    // kat_texture TEX IN OUT : (u, v) -> color3
    if (argc != 5) die("kat_texture TEX IN OUT");
    Texture *tex = strcmp(argv[2], "-") ? new Texture(tex_path("", argv[2]).c_str()) : new Texture();
    std::vector<char> in = read_file(argv[3]);
    const float *f = (const float *)&in[0];
    size_t n = in.size() / 8;
    std::vector<float> out(n * 3);
    for (size_t i = 0; i < n; ++i)
    {
      Color c = tex->getTexelColor(f[i * 2], f[i * 2 + 1]);
      out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
    }
    write_file(argv[4], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "kat_argb")
  {
    // kat_argb IN OUT : color3 -> Color::argb()
    if (argc != 4) die("kat_argb IN OUT");
    std::vector<char> in = read_file(argv[2]);
    const float *f = (const float *)&in[0];
    size_t n = in.size() / 12;
    std::vector<ARGB> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = Color(f[i * 3], f[i * 3 + 1], f[i * 3 + 2]).argb();
    write_file(argv[3], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "kat_camera")
  {
    // kat_camera IN OUT : eye3 at3 fov -> view (row-major _11.._33) + rz for W=1
    if (argc != 4) die("kat_camera IN OUT");
    std::vector<char> in = read_file(argv[2]);
    const float *f = (const float *)&in[0];
    size_t n = in.size() / 28;
    std::vector<float> out(n * 9);
    for (size_t i = 0; i < n; ++i)
    {
      Camera c(Vector3(f[i * 7], f[i * 7 + 1], f[i * 7 + 2]), Vector3(f[i * 7 + 3], f[i * 7 + 4], f[i * 7 + 5]), f[i * 7 + 6]);
      memcpy(&out[i * 9], c.view.m, 36);
    }
    write_file(argv[3], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "kat_pow")
  {
    // kat_pow IN OUT : (x, y) -> pow(float, float) exactly as Scene.cpp:175/196 calls it
    if (argc != 4) die("kat_pow IN OUT");
    std::vector<char> in = read_file(argv[2]);
    const float *f = (const float *)&in[0];
    size_t n = in.size() / 8;
    std::vector<float> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = pow(f[i * 2], f[i * 2 + 1]);
    write_file(argv[3], n ? &out[0] : NULL, out.size() * 4);
    return 0;
  }
  if (mode == "savetex")
  {
    // savetex W H IN OUT : Texture(W, H) filled with IN's W*H ARGB words, saveToFile(OUT) (.bmp / .tga)
    if (argc != 6) die("savetex W H IN OUT");
    unsigned W = atoi(argv[2]), H = atoi(argv[3]);
    std::vector<char> in = read_file(argv[4]);
    if (in.size() != (size_t)W * H * 4) die("savetex: input size");
    Texture t(W, H);
    memcpy(t.getColorBuffer(), &in[0], in.size());
    printf("%d\n", t.saveToFile(argv[5]) ? 1 : 0);
    return 0;
  }
  if (mode == "loadtex")
  {
    // loadtex IN OUT : Texture::loadFromFile(IN) (what Scene::addTexture does) -> OUT: ok, w, h, texels
    if (argc != 4) die("loadtex IN OUT");
    Texture t;
    const bool ok = t.loadFromFile(argv[2]);
    std::vector<uint32_t> out;
    out.push_back(ok ? 1u : 0u);
    out.push_back(t.getWidth());
    out.push_back(t.getHeight());
    if ((size_t)t.getWidth() * t.getHeight())
    {
      const ARGB *p = t.getColorBuffer();
      out.insert(out.end(), p, p + (size_t)t.getWidth() * t.getHeight());
    }
    write_file(argv[3], &out[0], out.size() * 4);
    return 0;
  }
  die("unknown mode");
  return 2;
}
