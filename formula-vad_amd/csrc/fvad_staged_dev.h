// Device helpers shared by the staged kernels' translation units
// (fvad_staged.hip, fvad_wave.hip).
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_internal.h"
#include "fvad_staged.h"

namespace fvad {
constexpr int kHist = kPitchBuf - kFrame;  // 1248
constexpr float kScale960 = 1.f / 960;
__device__ __forceinline__ int ticks_of(const StagedArgs &a, int s) {
  return a.ticks_valid ? a.ticks_valid[s] : a.n_ticks;
}

// Dynamic group scheduling of the persistent kernels: a workgroup takes the
// index of its next group from one of 8 queues (queue x serves groups x,
// x + 8, x + 16, ... and the workgroups with blockIdx % 8 == x, i.e. one XCD's
// under round-robin dispatch, which keeps each counter's atomics local and
// few).  A workgroup that starts late -- beside another kernel's waves --
// just takes fewer groups instead of stretching the launch with a tail.
// The counters a.work[slot][8] are zeroed on the stream before every launch.
constexpr int kQueues = 8;
enum WorkSlot { kWorkFftA = 0, kWorkPlpc, kWorkPcorr, kWorkPspec, kWorkSynth, kWorkFftB, kWorkSlots };
__device__ __forceinline__ long long take_group(const StagedArgs &a, int slot) {
  const int x = blockIdx.x % kQueues;
  return x + (long long)kQueues * atomicAdd(&a.work[slot * kQueues + x], 1u);
}

// Per-wave variant: lane 0 of the wave takes the next unit of its
// workgroup's queue (blockIdx % 8), broadcast to the wave.  A grid must have
// at least min(units, kQueues) workgroups so that every queue with units is
// served.
__device__ __forceinline__ long long wave_take(const StagedArgs &a, int slot, int lane) {
  const int x = blockIdx.x % kQueues;
  unsigned v = 0;
  if (lane == 0) v = atomicAdd(&a.work[slot * kQueues + x], 1u);
  v = __shfl(v, 0);
  return x + (long long)kQueues * v;
}

// analysis / synthesis window value for index i of the 960-sample window
__device__ __forceinline__ float win960(const float *__restrict__ hw, int i) {
  return (i < kFrame) ? hw[i] : hw[kWin - 1 - i];
}

__device__ __forceinline__ const float *frame_pb(const StagedArgs &a, int f) {
  const int s = f / a.V, v = f - s * a.V;
  return a.xs + (size_t)s * a.L + (size_t)v * kFrame;
}
// frame index of slot fr of group g, or -1 (same rule as group_frames)
__device__ __forceinline__ int frame_of(const StagedArgs &a, long long g, int F, int fr) {
  const long long f = g * F + fr;
  if (f >= (long long)a.n_streams * a.V) return -1;
  const int s = (int)(f / a.V), v = (int)(f - (long long)s * a.V);
  return v < ticks_of(a, s) * a.n_channels ? (int)f : -1;
}

}  // namespace fvad
