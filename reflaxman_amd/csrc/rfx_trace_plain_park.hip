// The ray-regrouping family of librfx.so: plain-pixel trace kernels that park their live traces after
// FrameParams::park_after segments (kCfgPark) and the bounce kernel that resumes the parked traces in packed
// waves -- its own TU so it compiles in parallel with the other families (reflaxman_amd/_build.py).
#include "rfx_trace.h"

#include <atomic>

namespace rfx {

constexpr int kLdsLimitDevices = 64;  // devices whose LDS-limit attribute is cached (others: set at every launch)

template <int CFG>
static void launch_park_one(dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  hipLaunchKernelGGL((trace_kernel<false, kModePlain, CFG | kCfgPark>), grid, dim3(kWgThreads), 0, st, S, P);
}

void launch_trace_plain_park(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  switch (cfg & ~kCfgPark)
  {
    case 1 | kCfgOneLight: launch_park_one<1 | kCfgOneLight>(grid, S, P, st); break;
    case 5 | kCfgOneLight: launch_park_one<5 | kCfgOneLight>(grid, S, P, st); break;
    case 1: launch_park_one<1>(grid, S, P, st); break;
    case 3: launch_park_one<3>(grid, S, P, st); break;
    case 5: launch_park_one<5>(grid, S, P, st); break;
    case 7: launch_park_one<7>(grid, S, P, st); break;
    case 9: launch_park_one<9>(grid, S, P, st); break;
    case 11: launch_park_one<11>(grid, S, P, st); break;
    case 13: launch_park_one<13>(grid, S, P, st); break;
    case 15: launch_park_one<15>(grid, S, P, st); break;
    default:  // one light, other configurations: the general kernels
      if (cfg & kCfgOneLight) launch_trace_plain_park(cfg & ~kCfgOneLight, grid, S, P, st);
      break;
  }
}

// the bounce kernel of the parked traces (rfx_trace.h bounce_kernel)
template <int CFG>
static void launch_bounce_one(dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  hipLaunchKernelGGL((bounce_kernel<CFG>), grid, dim3(kWgThreads), 0, st, S, P);
}

// the LDS-staged bounce kernel (large scenes, rfx_trace.h bounce_kernel_lds): one workgroup per CU
template <int CFG>
static hipError_t launch_bounce_lds_one(uint32_t groups, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  // the kernel may take the whole CU's LDS: raise its dynamic limit (every size lds_bvh_fits accepts) once per device
  // -- the attribute belongs to the current device, and a device group drives several from one process
  static std::atomic<int> limit_set[kLdsLimitDevices];  // 0 not yet, 1 raised, 2 refused
  int dev = 0;
  const bool cached = hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kLdsLimitDevices;
  int state = cached ? limit_set[dev].load(std::memory_order_relaxed) : 0;
  if (state == 0)
  {
    state = hipFuncSetAttribute(reinterpret_cast<const void *>(&bounce_kernel_lds<CFG>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096) == hipSuccess ? 1 : 2;
    if (cached) limit_set[dev].store(state, std::memory_order_relaxed);
  }
  if (state != 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL((bounce_kernel_lds<CFG>), dim3(groups), dim3(kLdsBvhThreads), lds_bvh_bytes(S.n_bvh), st, S, P);
  return hipGetLastError();
}

hipError_t launch_bounce_lds(int cfg, uint32_t groups, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  switch (cfg)
  {
    case 1 | kCfgOneLight: return launch_bounce_lds_one<1 | kCfgOneLight>(groups, S, P, st);
    case 9 | kCfgOneLight: return launch_bounce_lds_one<9 | kCfgOneLight>(groups, S, P, st);
    case 1: return launch_bounce_lds_one<1>(groups, S, P, st);
    case 3: return launch_bounce_lds_one<3>(groups, S, P, st);
    case 9: return launch_bounce_lds_one<9>(groups, S, P, st);
    case 11: return launch_bounce_lds_one<11>(groups, S, P, st);
    default:  // one light, other configurations: the general kernels
      return (cfg & kCfgOneLight) ? launch_bounce_lds(cfg & ~kCfgOneLight, groups, S, P, st) : hipErrorInvalidValue;
  }
}

void launch_bounce(int cfg, dim3 grid, const DevScene &S, const FrameParams &P, hipStream_t st)
{
  switch (cfg)
  {
    case 1 | kCfgOneLight: launch_bounce_one<1 | kCfgOneLight>(grid, S, P, st); break;
    case 5 | kCfgOneLight: launch_bounce_one<5 | kCfgOneLight>(grid, S, P, st); break;
    case 1: launch_bounce_one<1>(grid, S, P, st); break;
    case 3: launch_bounce_one<3>(grid, S, P, st); break;
    case 5: launch_bounce_one<5>(grid, S, P, st); break;
    case 7: launch_bounce_one<7>(grid, S, P, st); break;
    case 9: launch_bounce_one<9>(grid, S, P, st); break;
    case 11: launch_bounce_one<11>(grid, S, P, st); break;
    case 13: launch_bounce_one<13>(grid, S, P, st); break;
    case 15: launch_bounce_one<15>(grid, S, P, st); break;
    default:  // one light, other configurations: the general kernels
      if (cfg & kCfgOneLight) launch_bounce(cfg & ~kCfgOneLight, grid, S, P, st);
      break;
  }
}

}  // namespace rfx

#ifdef RFX_DEBUG_WAVES
// this translation unit's copy of the wave timeline (the parking trace kernels and the bounce kernel; the others are
// read by rfx_debug_wave_time_read in rfx_trace_plain_fast.hip)
extern "C" int rfx_debug_wave_time_read_park(unsigned long long *out, int n)
{
  if (n < 0 || (uint32_t)n > rfx::kWaveTimeMax) n = (int)rfx::kWaveTimeMax;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rfx::g_wave_time), 2 * (size_t)n * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return n;
}
#endif
