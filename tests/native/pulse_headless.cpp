// Headless platform for the reference's own application controller (src/common/Pulse.cpp, unmodified):
// a BasePlatformInterface with a fake clock drives Pulse.  Built twice by tools/pulse_build.py:
//   * against the reference's Render.cpp / Scene.cpp ... (the CPU renderer): the goldens;
//   * against include/reflaxman/dropin/{Render,Scene}.h + librfx.so: the same Pulse on the MI355X.
//
// Usage:
//   pulse_headless OUTDIR/ RES_KEY(1-9) SS_KEY(1-9) [WIN_W WIN_H]
//       the screenshot flow -- F2, a resolution key, an SSAA key, then exec() until the BMP is written
//       (Pulse.cpp:156-209, 346-438) -- prints the file name;
//   pulse_headless OUTDIR/ session WIN_W WIN_H TICK_US [nohash]
//       an interactive session (Pulse::renderImage, Pulse.cpp:102-154): still frames (depth 15, additive), keys
//       pressed in the middle of a frame (the frame is abandoned: Pulse.cpp:110), motion frames with the keys held
//       (block preview, depth 4, sampleNum adapted from the frame time: Pulse.cpp:112-118), keys released (the
//       camera decelerates, Camera.cpp:110-239, then still frames accumulate again).  Every completed frame is read
//       back the way the window does it (getRenderImagePixel over the client area, linux/main.cpp:53-88) and
//       hashed; one line per frame: "frame I execs N ms T hash H read R".  T is the wall time of the frame's exec()
//       calls, R that of the window's first pixel read (which waits for the frame and copies it to the host).
//       The fake clock advances TICK_US per reading, so Pulse's chunk doubling and sample adaptation are the same
//       in both builds.
//   pulse_headless OUT frames W H DEPTH SS ADDITIVE N
//       no Pulse: N frames of Render's default scene, each rendered by one renderNext(W*H) call; writes OUT.f32
//       (imagePixel) and OUT.argb (copyImage).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <chrono>
#include <string>

#include "Pulse.h"

class HeadlessPlatform : public BasePlatformInterface {
 public:
  HeadlessPlatform(const std::string &dir, unsigned w, unsigned h, uint64_t tick)
      : dir_(dir), w_(w), h_(h), t_(1), tick_(tick) {}
  std::string getExePath() { return dir_; }
  uint64_t getPerformanceCounter() { return t_ += tick_; }
  uint64_t getPerformanceFrequency() { return 1000000; }
  uint64_t getSystemTime() { return 0x0123456789ABCDEFull; }
  void getMainWindowClientSize(unsigned int *const width, unsigned int *const height) { *width = w_; *height = h_; }
  void invalidateMainWindow() {}
  void sleep(unsigned int) {}

 private:
  std::string dir_;
  unsigned w_, h_;
  uint64_t t_, tick_;
};

static const KEY_CODE kDigit[9] = {KEY_1, KEY_2, KEY_3, KEY_4, KEY_5, KEY_6, KEY_7, KEY_8, KEY_9};

static int screenshot(const std::string &dir, int res, int ss, unsigned ww, unsigned wh)
{
  HeadlessPlatform plat(dir, ww, wh, 1000);  // 1 ms per reading: chunks double every call
  Pulse pulse(&plat);
  pulse.onResize(ww, wh);                 // stInit -> stCameraControl, Render::setImageSize
  pulse.onKeyEvent(KEY_F2, true);         // -> resolution menu
  pulse.onKeyEvent(kDigit[res - 1], true);
  pulse.onKeyEvent(kDigit[ss - 1], true); // -> stScreenshotRenderBegin
  char name[256];
  snprintf(name, sizeof(name), "%sscrnshoot_%08X%08X.bmp", dir.c_str(), 0x01234567u, 0x89ABCDEFu);
  struct stat st;
  for (long i = 0; i < 100000000L; ++i)
  {
    pulse.exec();
    if (stat(name, &st) == 0)
    {
      pulse.exec();  // stScreenshotRenderEnd: back to the window size
      printf("%s\n", name);
      return 0;
    }
  }
  fprintf(stderr, "no screenshot written\n");
  return 1;
}

// FNV-1a 64 over the window's pixels as linux/main.cpp:82-84 reads them (x fastest, y from 0)
static uint64_t frame_hash(Pulse &pulse, unsigned w, unsigned h)
{
  uint64_t x = 1469598103934665603ull;
  for (unsigned y = 0; y < h; ++y)
    for (unsigned i = 0; i < w; ++i)
    {
      const uint32_t p = pulse.getRenderImagePixel(i, y);
      for (int b = 0; b < 4; ++b)
      {
        x ^= (p >> (8 * b)) & 0xFFu;
        x *= 1099511628211ull;
      }
    }
  return x;
}

static int session(const std::string &dir, unsigned w, unsigned h, uint64_t tick, bool hash)
{
  HeadlessPlatform plat(dir, w, h, tick);
  Pulse pulse(&plat);
  pulse.onResize(w, h);
  typedef std::chrono::steady_clock clk;
  int frame = 0;
  long execs = 0;
  double ms = 0.0;
  // run exec() until the next frame completes (or `limit` calls), timing the calls
  auto run = [&](long limit) -> bool {
    for (long i = 0; i < limit; ++i)
    {
      const clk::time_point t0 = clk::now();
      pulse.exec();
      ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
      ++execs;
      if (pulse.imageReady)
      {
        // the window's first pixel read waits for the frame on the device and copies it back (Render::imagePixel)
        const clk::time_point t1 = clk::now();
        (void)pulse.getRenderImagePixel(0, 0);
        const double read_ms = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
        const uint64_t hv = hash ? frame_hash(pulse, w, h) : 0;
        printf("frame %d execs %ld ms %.4f hash %016llx read %.4f\n", frame++, execs, ms, (unsigned long long)hv,
               read_ms);
        fflush(stdout);
        execs = 0;
        ms = 0.0;
        pulse.imageReady = false;  // the window drew it (linux/main.cpp:87)
        return true;
      }
    }
    return false;
  };
  const long kMax = 100000000L;
  for (int i = 0; i < 2; ++i) run(kMax);      // still frames: depth 15, additive
  run(7);                                     // seven chunks into the third still frame ...
  pulse.onKeyEvent(KEY_RIGHT, true);          // ... keys go down: the frame is abandoned for a motion frame
  pulse.onKeyEvent(KEY_W, true);
  for (int i = 0; i < 6; ++i) run(kMax);      // motion frames: block preview, depth 4
  pulse.onKeyEvent(KEY_RIGHT, false);
  pulse.onKeyEvent(KEY_W, false);
  for (int i = 0; i < 8; ++i) run(kMax);      // the camera decelerates, then still frames accumulate again
  return 0;
}

// A caller that renders each frame in one call, as Render::renderNext(W*H) allows (Render.cpp:136-215): N frames of
// the default scene (Render's own loadScene), then the image read back as imagePixel (OUT.f32, row 0 first) and
// copyImage (OUT.argb).  No Pulse: this is any non-interactive program's use of the renderer.
static int frames(const std::string &out, unsigned w, unsigned h, int depth, int ss, bool additive, int n)
{
  Render render((out + ".").c_str());  // textures absent -> the checker fallback, as the goldens
  render.setImageSize(w, h);
  for (int i = 0; i < n; ++i)
  {
    render.renderBegin(depth, ss, additive);
    if (render.renderNext(w * h)) return 3;  // one call covers the frame
  }
  FILE *f = fopen((out + ".f32").c_str(), "wb");
  if (!f) return 4;
  for (unsigned y = 0; y < h; ++y)
    for (unsigned x = 0; x < w; ++x)
    {
      const Color c = render.imagePixel(x, y);
      fwrite(&c.r, 4, 1, f);
      fwrite(&c.g, 4, 1, f);
      fwrite(&c.b, 4, 1, f);
    }
  fclose(f);
  Texture t(w, h);
  render.copyImage(t);
  f = fopen((out + ".argb").c_str(), "wb");
  if (!f) return 4;
  fwrite(t.getColorBuffer(), 4, (size_t)w * h, f);
  fclose(f);
  printf("ok\n");
  return 0;
}

int main(int argc, char **argv)
{
  if (argc == 9 && !strcmp(argv[2], "frames"))
    return frames(argv[1], (unsigned)atoi(argv[3]), (unsigned)atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                  atoi(argv[7]) != 0, atoi(argv[8]));
  if (argc >= 6 && !strcmp(argv[2], "session"))
    return session(argv[1], (unsigned)atoi(argv[3]), (unsigned)atoi(argv[4]), (uint64_t)strtoull(argv[5], nullptr, 0),
                   !(argc > 6 && !strcmp(argv[6], "nohash")));
  if (argc < 4)
  {
    fprintf(stderr, "usage: pulse_headless OUTDIR/ RES_KEY SS_KEY [WIN_W WIN_H] | OUTDIR/ session W H TICK_US [nohash]\n");
    return 2;
  }
  const std::string dir = argv[1];
  const int res = atoi(argv[2]), ss = atoi(argv[3]);
  const unsigned ww = argc > 5 ? (unsigned)atoi(argv[4]) : 320, wh = argc > 5 ? (unsigned)atoi(argv[5]) : 240;
  if (res < 1 || res > 9 || ss < 1 || ss > 9) return 2;
  return screenshot(dir, res, ss, ww, wh);
}
