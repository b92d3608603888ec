// The drop-in Scene's revision (include/reflaxman/dropin/Scene.h), which Render::renderNext compares with the scene it
// uploaded last: no two states of any Scene share a revision -- a freshly assigned Scene with the same number of
// mutations as an earlier one included (Render.cpp:32's `scene = Scene(...)` followed by adds) -- and the handles a
// moved Scene returns keep working on the Scene they now belong to.  Host calls only (no GPU).
#include <stdio.h>

#include <set>

#include "Scene.h"

static int fails = 0;
#define CHECK(c)                                             \
  do {                                                       \
    if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

int main()
{
  std::set<unsigned long long> seen;
  Scene a(Color(0.95f, 0.95f, 1.0f), 0.15f);
  CHECK(seen.insert(a.revision()).second);
  const Material m(Material::mtMetal, Color(1.0f, 1.0f, 1.0f), 0.5f, 0.0f);
  for (int i = 0; i < 15; ++i)
  {
    a.addSphere(Vector3(float(i), 1.0f, 0.0f), 0.5f, m);
    CHECK(seen.insert(a.revision()).second);
  }
  const unsigned long long ra = a.revision();
  // the reference's re-initialisation: assign an empty temporary, then add in place
  a = Scene(Color(0.5f, 0.5f, 0.5f), 0.2f);
  CHECK(a.revision() != ra);
  CHECK(seen.insert(a.revision()).second);
  for (int i = 0; i < 15; ++i)
  {
    a.addSphere(Vector3(float(i), 2.0f, 0.0f), 0.5f, m);
    CHECK(seen.insert(a.revision()).second);  // never the revision the first scene had after 15 adds
  }
  // a Scene built elsewhere and moved in: its triangle handle now works on `a`
  Scene b(Color(0.1f, 0.1f, 0.1f), 0.1f);
  Texture *t = b.addTexture("no-such-file.tga");
  Triangle *tr = b.addTriangle(Vector3(0.0f, 0.0f, 0.0f), Vector3(1.0f, 0.0f, 0.0f), Vector3(0.0f, 1.0f, 0.0f), m);
  a = std::move(b);
  const unsigned long long before = a.revision();
  CHECK(seen.insert(before).second);
  tr->setTexture(t, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 1.0f);  // through a's handle (was: the moved-from b's null handle)
  CHECK(a.revision() != before);
  int ns = -1, nt = -1, nl = -1, nx = -1;
  rfx_scene_counts(a.handle(), &ns, &nt, &nl, &nx);
  CHECK(ns == 0 && nt == 1 && nx == 1);
  printf(fails ? "FAILED %d\n" : "ok\n", fails);
  return fails ? 1 : 0;
}
