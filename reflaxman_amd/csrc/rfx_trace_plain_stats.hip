// One trace_kernel family of librfx.so: mode kModePlain, stats (event counters, no culling) --
// its own TU so the families compile in parallel (reflaxman_amd/_build.py).
#include "rfx_trace.h"

namespace rfx {

void launch_trace_plain_stats(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<true, kModePlain>(cfg, grid, S, P, st);
}

}  // namespace rfx
