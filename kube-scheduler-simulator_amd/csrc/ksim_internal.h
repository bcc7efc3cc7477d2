// ksim_internal.h — launcher interface between the host runtime
// (ksim_engine.cpp) and the kernels (ksim_kernels.hip).
#pragma once

#include "ksim_device.h"

namespace ksim {

struct LaunchArgs {
  DevCluster c;
  DevPods P;
  ksim_profile prof;
  DevState* st;
  DevScratch s;
  DevEvalOut o;
  int32_t* chosen;   // [n_pods] device, may be null
};

// One scheduling cycle for the pod at st->cursor (no-op once cursor >= end).
void launch_cycle(const LaunchArgs& a, hipStream_t stream, bool compat);
void launch_assume(const DevCluster& c, const ksim_pod& p, int32_t node, int sign, hipStream_t stream);

}  // namespace ksim
