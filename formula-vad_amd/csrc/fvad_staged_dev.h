// Device helpers shared by the staged kernels' translation units
// (fvad_staged.hip, fvad_wave.hip, fvad_pitch.hip).
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "fvad_device.h"
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
// x_lp row of frame f: its x_lp[n] (n >= 1) is frame_xlp(a, f)[n]
constexpr int kXlpHist = kHist / 2;  // 624
__device__ __forceinline__ float *frame_xlp(const StagedArgs &a, int f) {
  const int s = f / a.V, v = f - s * a.V;
  return a.xlp + (size_t)s * a.LX + (size_t)v * (kFrame / 2);
}
// pitch_downsample's x_lp value from pitch-buffer samples x[2n-1], x[2n], x[2n+1] (n >= 1)
__device__ __forceinline__ float xlp_value(float xm, float x0, float xp) { return .5f * (.5f * (xm + xp) + x0); }
// frame index of slot fr of group g, or -1 (same rule as group_frames)
__device__ __forceinline__ int frame_of(const StagedArgs &a, long long g, int F, int fr) {
  const long long f = g * F + fr;
  if (f >= (long long)a.n_streams * a.V) return -1;
  const int s = (int)(f / a.V), v = (int)(f - (long long)s * a.V);
  return v < ticks_of(a, s) * a.n_channels ? (int)f : -1;
}

// Workgroup barrier for LDS traffic only: __syncthreads() also waits for the
// wave's outstanding global stores (vmcnt(0)), so a wave that stores results
// late in a phase holds every wave at the barrier for the stores' round trip.
// Use only where no thread of the workgroup reads back, in the same kernel,
// global data another thread wrote before the barrier.
#ifndef FVAD_FULL_SYNC
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#else
__device__ __forceinline__ void lds_sync() { __syncthreads(); }
#endif

// Diagnostic build only (-DFVAD_STAMPS): per-phase s_memtime totals of
// thread 0 (it joins every barrier, so a phase's stamp is its critical path),
// accumulated into a.stamps[base + id]; no other code reads them.
#ifdef FVAD_STAMPS
#define STAMP_INIT()                \
  unsigned long long st_acc[16] = {}; \
  unsigned long long st_last = __builtin_amdgcn_s_memtime()
#define RSTAMP(id)                                                \
  do {                                                            \
    if (tid == 0) {                                               \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      st_acc[id] += t_ - st_last;                                 \
      st_last = t_;                                               \
    }                                                             \
  } while (0)
#define STAMP_FLUSH(base, n)                                                  \
  do {                                                                        \
    if (tid == 0 && a.stamps)                                                 \
      for (int i_ = 0; i_ < (n); i_++) atomicAdd(&a.stamps[(base) + i_], st_acc[i_]); \
  } while (0)
#else
#define STAMP_INIT() \
  do {               \
  } while (0)
#define RSTAMP(id) \
  do {             \
  } while (0)
#define STAMP_FLUSH(base, n) \
  do {                       \
  } while (0)
#endif

// remove_doubling's candidate loop that does not depend on the previous
// frame, so k_select's serial part is compares only.
//   T0, candidate count, g0 = pitch_gain(xcorr(T0), xx, yy[T0]), xcorr(T0),
//   yy[T0], the pseudo-interpolation offset of T0; then per k = 2..15:
//   T1, g1 = pitch_gain(xy, xx, yy), xy = (xcorr(T1) + xcorr(T1b)) / 2,
//   yy = (yy[T1] + yy[T1b]) / 2, the offset of T1.
namespace rec {
constexpr int kT0 = 0, kNValid = 1, kG0 = 2, kXy0 = 3, kYy0 = 4, kOff0 = 5;
constexpr int kK = 8, kKStride = 5;  // T1, g1, xy, yy, offset
constexpr int kSize = 80;
}  // namespace rec
static_assert(rec::kSize == kPitchRecord, "pitch record size");
static_assert(rec::kK + 14 * rec::kKStride <= rec::kSize && rec::kSize % 4 == 0, "pitch record layout");

// remove_doubling's final pseudo-interpolation from the xcorr at T-1, T, T+1
__device__ __forceinline__ int pitch_offset(float x0, float x1, float x2) {
  if ((x2 - x0) > .7f * (x1 - x0)) return 1;
  if ((x0 - x2) > .7f * (x1 - x2)) return -1;
  return 0;
}

__device__ __forceinline__ int rd_T1(int T0, int k) { return (int)((unsigned)(2 * T0 + k) / (unsigned)(2 * k)); }
__device__ __forceinline__ int rd_T1b(int T0, int T1, int k) {
  if (k == 2) return (T1 + T0 > 384) ? T0 : T0 + T1;
  return (int)((unsigned)(2 * second_check(k) * T0 + k) / (unsigned)(2 * k));
}

}  // namespace fvad
