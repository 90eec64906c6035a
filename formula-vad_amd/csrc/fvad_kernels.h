// Kernel argument blocks and launch wrappers (fvad_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "fvad_internal.h"

namespace fvad {

struct PrepArgs {
  int n_streams, n_channels, n_ticks;
  const int *ticks_valid;  // nullable
  const float *pcm;        // [t][s][c][480] normalised input
  float *xbuf;             // [t][s][c][480] high-passed, s16 scale
  float *ratio;            // [t][s]
  float *state;            // [s][st::kWords]
  int raw_s16;             // rnnoise compat: input already s16-scaled
};

struct FrameArgs {
  int n_streams, n_channels, n_ticks;
  const int *ticks_valid;  // nullable
  const float *xbuf;
  const float *ratio;
  float *state;
  float *ring;  // [s][c][ring_len] denoised re-block ring
  int ring_len;
  const Plan *plan;
  const DevModel *model;  // device-resident layer descriptors
  int n_bands;
  int band_lo[kMaxBandCfg], band_hi[kMaxBandCfg];
  int bin_lo_all, bin_hi_all;
  float *out_vad, *out_win_ratio, *out_win_vad, *out_band, *out_den;
  int *out_win_flag;
  int raw_s16;  // rnnoise compat: emit s16-scaled output (no 1/32767)
  unsigned long long *stamps;  // diagnostic build only (FVAD_STAMPS)
};

size_t frame_lds_bytes();
hipError_t launch_prep(const PrepArgs &a, hipStream_t stream);
hipError_t launch_frame(const FrameArgs &a, hipStream_t stream);
hipError_t launch_kiss_fftr(int ncfft, const int *fac, int nf, const float *twb, const float *sup, const int *perm,
                            const float *in, float *out, float *work, hipStream_t stream);

}  // namespace fvad
