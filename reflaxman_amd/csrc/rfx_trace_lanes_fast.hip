// One trace_kernel family of librfx.so: mode kModeSsaaLanes (SSAA frames, one lane per sample), render --
// its own TU so the families compile in parallel (reflaxman_amd/_build.py).
// RFX_LANES_WAVES_PER_EU: this family's own occupancy target (default: the trace kernels' RFX_WAVES_PER_EU)
#if !defined(RFX_WAVES_PER_EU) && defined(RFX_LANES_WAVES_PER_EU)
#define RFX_WAVES_PER_EU RFX_LANES_WAVES_PER_EU
#endif
#include "rfx_trace.h"

namespace rfx {

void launch_trace_lanes_fast(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<false, kModeSsaaLanes>(cfg, grid, S, P, st);
}

}  // namespace rfx
