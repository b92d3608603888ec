// Headless platform for the reference's own application controller (src/common/Pulse.cpp, unmodified):
// a BasePlatformInterface with a fake clock drives Pulse through its screenshot flow -- F2, a resolution
// key, an SSAA key, then exec() until the BMP is written (Pulse.cpp:156-209, 346-438) -- and prints the
// file name.  Built twice by tests/test_dropin_pulse.py:
//   * against the reference's Render.cpp / Scene.cpp ... (the CPU renderer): the golden screenshot;
//   * against include/reflaxman/dropin/{Render,Scene}.h + librfx.so: the same Pulse on the MI355X.
// Usage: pulse_headless OUTDIR/ RES_KEY(1-9) SS_KEY(1-9) [WIN_W WIN_H]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <string>

#include "Pulse.h"

class HeadlessPlatform : public BasePlatformInterface {
 public:
  HeadlessPlatform(const std::string &dir, unsigned w, unsigned h) : dir_(dir), w_(w), h_(h), t_(1) {}
  std::string getExePath() { return dir_; }
  uint64_t getPerformanceCounter() { return t_ += 1000; }  // 1 ms per reading: chunks double every call
  uint64_t getPerformanceFrequency() { return 1000000; }
  uint64_t getSystemTime() { return 0x0123456789ABCDEFull; }
  void getMainWindowClientSize(unsigned int *const width, unsigned int *const height) { *width = w_; *height = h_; }
  void invalidateMainWindow() {}
  void sleep(unsigned int) {}

 private:
  std::string dir_;
  unsigned w_, h_;
  uint64_t t_;
};

static const KEY_CODE kDigit[9] = {KEY_1, KEY_2, KEY_3, KEY_4, KEY_5, KEY_6, KEY_7, KEY_8, KEY_9};

int main(int argc, char **argv)
{
  if (argc < 4) { fprintf(stderr, "usage: pulse_headless OUTDIR/ RES_KEY SS_KEY [WIN_W WIN_H]\n"); return 2; }
  const std::string dir = argv[1];
  const int res = atoi(argv[2]), ss = atoi(argv[3]);
  const unsigned ww = argc > 5 ? (unsigned)atoi(argv[4]) : 320, wh = argc > 5 ? (unsigned)atoi(argv[5]) : 240;
  if (res < 1 || res > 9 || ss < 1 || ss > 9) return 2;
  HeadlessPlatform plat(dir, ww, wh);
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
