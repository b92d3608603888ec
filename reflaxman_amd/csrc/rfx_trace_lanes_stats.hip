// One trace_kernel family of librfx.so: mode kModeSsaaLanes (SSAA frames, one lane per sample), stats (event
// counters, no culling) --
// its own TU so the families compile in parallel (reflaxman_amd/_build.py).
#include "rfx_trace.h"

namespace rfx {

void launch_trace_lanes_stats(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<true, kModeSsaaLanes>(cfg, grid, S, P, st);
}

}  // namespace rfx
