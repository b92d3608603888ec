// One trace_kernel family of librfx.so: mode kModePlain, render --
// its own TU so the families compile in parallel (reflaxman_amd/_build.py).
#include "rfx_trace.h"

namespace rfx {

void launch_trace_plain_fast(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<false, kModePlain>(cfg, grid, S, P, st);
}

}  // namespace rfx

#ifdef RFX_DEBUG_PROF
extern "C" int rfx_debug_cull_read(unsigned long long *out, int reset)
{
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rfx::g_cull), sizeof(rfx::g_cull)) != hipSuccess) return -1;
  if (reset)
  {
    static const unsigned long long zero[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rfx::g_cull), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 32;
}

extern "C" int rfx_debug_prof_read(unsigned long long *out, int reset)
{
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rfx::g_prof), sizeof(rfx::g_prof)) != hipSuccess) return -1;
  if (reset)
  {
    static const unsigned long long zero[2 * rfx::P_COUNT] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rfx::g_prof), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 2 * rfx::P_COUNT;
}
#endif

#ifdef RFX_DEBUG_WAVES
// each wave tile's (start, end) s_memrealtime of the last plain launch, tiles [0, n); returns the tiles read
extern "C" int rfx_debug_wave_time_read(unsigned long long *out, int n)
{
  if (n < 0 || (uint32_t)n > rfx::kWaveTimeMax) n = (int)rfx::kWaveTimeMax;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rfx::g_wave_time), 2 * (size_t)n * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return n;
}
#endif
