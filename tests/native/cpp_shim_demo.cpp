// A host program written against the reference's class API (Render / Scene / Camera), compiled
// against include/reflaxman/reflaxman.h + librfx.so instead of src/common/*.cpp.
//   cpp_shim_demo W H DEPTH SS ADDITIVE FRAMES CHUNK OUT   -> OUT.f32 (imagePixel), OUT.argb (copyImage)
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "reflaxman/reflaxman.h"

using namespace reflaxman;

int main(int argc, char **argv)
{
  if (argc != 9) { fprintf(stderr, "usage: W H DEPTH SS ADDITIVE FRAMES CHUNK OUT\n"); return 2; }
  const unsigned W = atoi(argv[1]), H = atoi(argv[2]), chunk = atoi(argv[7]);
  const int depth = atoi(argv[3]), ss = atoi(argv[4]), frames = atoi(argv[6]);
  const bool additive = atoi(argv[5]) != 0;
  try
  {
    Render render("/nonexistent/", 0, 1350490027u, 987654321u);  // textures absent -> checker, as Render.cpp:25-55
    render.setImageSize(W, H);
    for (int f = 0; f < frames; ++f)
    {
      render.renderBegin(depth, ss, additive);
      while (render.renderNext(chunk)) {}
    }
    std::vector<float> rgb((size_t)W * H * 3);
    for (unsigned y = 0; y < H; ++y)
      for (unsigned x = 0; x < W; ++x)
      {
        Color c = render.imagePixel(x, y);
        float *d = &rgb[((size_t)y * W + x) * 3];
        d[0] = c.r; d[1] = c.g; d[2] = c.b;
      }
    Texture t(W, H);
    render.copyImage(t);
    const std::string out = argv[8];
    FILE *f = fopen((out + ".f32").c_str(), "wb");
    fwrite(rgb.data(), 4, rgb.size(), f);
    fclose(f);
    f = fopen((out + ".argb").c_str(), "wb");
    fwrite(t.getColorBuffer(), 4, (size_t)W * H, f);
    fclose(f);
    if (!t.saveToFile((out + ".bmp").c_str())) return 3;
    printf("progress %.1f%%\n", render.getRenderProgress());
  }
  catch (const std::exception &e)
  {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
