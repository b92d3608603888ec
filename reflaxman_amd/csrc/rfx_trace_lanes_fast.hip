// One trace_kernel family of librfx.so: mode kModeSsaaLanes (SSAA frames, one lane per sample), render --
// its own TU so the families compile in parallel (reflaxman_amd/_build.py).
#include "rfx_trace.h"

namespace rfx {

void launch_trace_lanes_fast(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<false, kModeSsaaLanes>(cfg, grid, S, P, st);
}

}  // namespace rfx
