// One trace_kernel family of librfx.so: mode kModeSsaaChunks (SSAA frames of sampleNum > 8, one pixel per wave, its
// samples 64 at a time), stats (event counters, no culling) -- its own TU so the families compile in parallel (reflaxman_amd/_build.py).
#include "rfx_trace.h"

namespace rfx {

void launch_trace_chunks_stats(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  launch_cfg<true, kModeSsaaChunks>(cfg, grid, S, P, st);
}

}  // namespace rfx
