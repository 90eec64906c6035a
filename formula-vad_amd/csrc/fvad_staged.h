// Argument block and launcher of the staged (time-parallel) pipeline
// (fvad_staged.hip).  Frame f = s * V + v, v = tick * C + channel: the
// channels of a stream are one interleaved virtual rnnoise stream
// (VAD.zig:274-296), so frame order within a stream is tick-major.
#pragma once
#include <hip/hip_runtime.h>

#include "fvad_internal.h"

namespace fvad {

constexpr int kStagedKernels = 11;
constexpr int kWorkCounters = 64;  // persistent-kernel queues (fvad_staged.hip: take_group)
constexpr int kPitchRecord = 80;  // floats per frame of the pitch record (k_pcorr -> k_select)

// Pitch tile buffer (k_plpc -> k_pcorr): a tile is 64 streams at one frame
// position; each quarter (16 streams) is one contiguous block of kRows rows of
// 16 floats (the yy_lookup region is laid out frame-major instead).  xf (x_lp
// after celt_fir5) is not stored: k_pcorr rebuilds it from the x_lp rows and
// the frame's FIR coefficients (5.2 -> 1.8 KB written per frame).
namespace ptile {
constexpr int kTile = 64, kQuarter = 16;
constexpr int kFir = 0;             // celt_fir5 coefficients lpc2[0..4], then x_lp[0] (the frame's edge value)
constexpr int kSc = 8;              // Syy before step i of the coarse find_best_pitch, i < 147
constexpr int kSf = kSc + 147;      // Syy before step 8k of the fine find_best_pitch, k < 37 (k_pcorr
                                    //   walks the recurrence from there to the <= 10 lags it needs)
constexpr int kSfCk = 37;
constexpr int kXx = kSf + kSfCk;    // xx
constexpr int kRows = kXx + 1;
}  // namespace ptile

// Device VADMachine (VADMachine.zig:126-230), one lane per stream.
struct VadmConst {
  int n_lt, n_st, n_r, slot;           // RollingAverage lengths, engine band slot
  long long lt_off, st_off, r_off;     // buffer offsets (floats): long-term [stream][lt_pitch] (a stream's
  int lt_pitch;                        //   fold walks its own row), short-term and ratio [i][stream]
  unsigned long long min_open, max_gap, rec_pad;
  float thr_factor, ratio_thr, min_dur, sr;
  int has_init;
  double init;
};
struct VadmState {
  unsigned long long speech_start, speech_end, windows_done;
  double lt_last, st_last, r_last, lt_pre;  // lt_pre: cached prefix (see ra_push_long)
  // lt_nw: entries pushed; lt_defer: long pushes since lt_last was last folded
  // exactly (k_vadm_hbm's deferred fold: lt_last is then stale, and lt_approx /
  // lt_amax / lt_fpre carry the walk's estimate, its bound's magnitude and the
  // exact fold through the last pushed index; every sync point resolves it)
  unsigned lt_widx, lt_count, st_widx, st_count, r_widx, r_count, lt_nw, lt_defer;
  // lt_neg: long pushes until every negative (or NaN) entry has left the
  // long-term buffer; the lazy walk's bound needs nonnegative terms, so the
  // machine folds at every push until then (band energies are >= 0 and a
  // window's min is at most 999, so this stays 0 on every pipeline output)
  int lt_has, st_has, r_has, state, lt_pre_ok, lt_neg;
  float rnn_vad, vol_ratio;
  unsigned rnn_vad_count, vol_ratio_count, n_segs, pad;
  double lt_approx, lt_amax, lt_fpre;
};
struct VadmSeg {
  unsigned long long sample_from, sample_to;
  float debug_rnn_vad, debug_avg_speech_vol_ratio;
};
struct VadmArgs {
  int n;  // machines (0: k_vadm not launched)
  VadmConst c[kMaxBandCfg];
  VadmState *st;  // [m][stream]
  float *buf;     // rolling-average data (f32: each entry is a pushed f32)
  VadmSeg *seg;   // [m][stream][seg_cap]
  int seg_cap;
  unsigned defer_max;  // test hook (FVAD_DEBUG_VADM_DEFER_MAX): fold once this many long pushes are owed; 0 = kLtDeferMax
  int vfinal;  // this launch is a sync point's: every machine's long-term average folded exactly at the end
  int par_serial_every;  // test hook (FVAD_DEBUG_VADM_PAR_SERIAL_EVERY): k_vadm_par hands stream s to its
                         //   in-kernel serial walk when s % par_serial_every == 0; 0 = never
  double bound_scale;    // test hook (FVAD_DEBUG_VADM_BOUND_SCALE): the lazy test's bound E times this
                         //   (1 in production; +inf: every test the estimate would settle folds instead)
  unsigned long long *count;  // test hook (FVAD_DEBUG_VADM_COUNT): null, or [kVadmCounts] device counters
  long long negate_at;   // test hook (FVAD_DEBUG_VADM_NEGATE_AT): window number whose band minimum enters
                         //   the machine negated (lt_neg's path); -1 = none
};
// the lazy long-term walk's counters (FVAD_DEBUG_VADM_COUNT): long-term tests
// decided from an exact average, from the estimate, left open by the bound (an
// exact fold), and the folds at the end of a push (sync point or defer limit)
enum { kVcExact = 0, kVcSettled = 1, kVcOpen = 2, kVcEndFold = 3, kVadmCounts = 4 };

struct StagedArgs {
  int n_streams, n_channels, n_ticks;
  int V;                   // frame-row stride per stream (= max_ticks * C)
  int L;                   // xs row length (= 1248 + V * 480)
  const int *ticks_valid;  // nullable
  const int *tail;         // nullable: real samples (1..480) in each stream's last valid tick (use_denoiser = 0)
  const float *pcm;        // [t][s][c][480] normalised input
  const int16_t *pcm16;    // nullable: the same as 16-bit samples k (k / 32768), read by k_prep3 instead of pcm
  float *xs;               // [s][L] high-passed s16-scale samples, 1248 history first
  float *xlp;              // [s][LX] pitch_downsample's x_lp over xs (x_lp[m] from xs[2m-1..2m+1]),
  int LX;                  //   624 history first (= 624 + V * 240); m = 0 unused
  float *ratio;            // [t][s] per-tick volume ratio
  float *state;            // [s][st::kWords]
  float2 *X;               // [f][481] analysis spectrum, then filtered/gained spectrum
  float2 *P;               // [f][481] pitch spectrum
  float *Ex, *Ep, *Exp;    // [f][22]
  float *Lyf;              // [f][22] DCT(Ly) features 0..21 (before deltas)
  float *f34;              // [f][8] features 34..40
  int *silence;            // [f]
  float *rec;              // [f][kPitchRecord]
  float *ptile;            // [tile][quarter][ptile::kRows][16]
  int *pitch;              // [f] selected pitch index
  float *vadf;             // [f] per-frame vad probability
  float *gr, *gs;          // [f][22] GRU gains g and smoothed gains max(g, .6*lastg)
  const int8_t *rnn_img;   // rnnimg image (fvad_internal.h), device
  const void *gru16_frags;   // FVAD_MODE_FP16: MFMA A fragments (fvad_gru16.hip), null otherwise
  const float *gru16_bias;   //   and the gate biases per tile row
  int fuse16;                // FVAD_MODE_FP16_FUSED: the pitch spectrum runs inside the GRU kernel (k_fused16)
  int rnn_act[rnnimg::kMats];  // activation of each image matrix
  float *ys;               // [f][960] windowed synthesis output
  float *ring;             // [s][c][ring_len]
  int ring_len;
  int *win_tick;           // [s][wmax] output slot of window j: tick * wpt + (its rank in the tick); -1: none
  long long *win_start;    // [s][wmax] absolute sample index of window j
  int wmax;
  int wpt;                 // window slots per (tick, stream) of the outputs: windows_per_tick(fft_size)
  // FFT B's tables (the Plan's up to kMaxFftB, separate device arrays above)
  // and, when a transform does not fit in LDS, k_fftb's device scratch:
  // fb_work_blocks workgroups, fb_work_stride float2 each
  const float2 *fb_tw, *fb_sup;
  const int *fb_perm;
  const float *fb_hann;
  float2 *fb_work;
  int fb_work_blocks;
  long long fb_work_stride;
  const Plan *plan;
  const DevModel *model;
  int n_bands;
  int nfft_b;                  // FFT B size (fft_size)
  int use_denoiser;            // 0: raw fft_size frames straight to FFT B (launch_nodenoise)
  int band_lo[kMaxBandCfg], band_hi[kMaxBandCfg];
  int bin_lo_all, bin_hi_all;
  // per (tick, stream): out_vad, out_win_flag (windows completed in the tick,
  // 0..wpt); per window slot [t][s][wpt]: out_win_ratio, out_win_vad, and
  // out_band [t][s][wpt][c][band]
  float *out_vad, *out_win_ratio, *out_win_vad, *out_band, *out_den;
  int *out_win_flag;
  int raw_s16;
  VadmArgs vadm;
  unsigned *work;          // [kWorkCounters] dynamic group counters of the persistent kernels
  unsigned long long *stamps;  // diagnostic build only (FVAD_STAMPS): per-phase cycles of k_rnn3
};

// Timing events: kernel i runs between ev[kStagedTime[i][0]] and
// ev[kStagedTime[i][1]]; ev[0] and ev[kStagedLast] bracket the launch.
constexpr int kStagedEvents = 15, kStagedLast = 13;
constexpr int kStagedTime[kStagedKernels][2] = {{0, 1}, {2, 3},   {14, 4},  {4, 5},   {5, 6},  {7, 8},
                                                {8, 9}, {9, 10}, {10, 11}, {11, 12}, {12, 13}};
// k_prep3 on `stream` (ev[0], ev[1] around it); the engine runs it one push
// ahead on its own stream (double-buffered xs / ratio / ticks).
hipError_t launch_prep(const StagedArgs &a, hipStream_t stream, hipEvent_t *ev);
// Launch the other 10 kernels; when ev != nullptr their timing events are
// recorded.
// fft_a_done (optional): recorded right after k_fftAw (the next push's
// k_prep3 waits for it).  fa_stream (optional, with fft_a_done): k_fftAw runs
// there instead, after fa_after (the previous push's synth_done: the last
// reader of X / Ex / Lyf / silence), so it overlaps the previous push's tail
// on `stream`; `stream` waits for it before k_plpc.  synth_done (optional):
// recorded on `stream` after k_synthw.
hipError_t launch_staged(const StagedArgs &a, int n_cu, hipStream_t stream, hipEvent_t *ev,
                         hipEvent_t fft_a_done = nullptr, hipStream_t fa_stream = nullptr,
                         hipEvent_t fa_after = nullptr, hipEvent_t synth_done = nullptr);
// k_pcorr over `tiles` pitch tiles (fvad_pitch.hip)
hipError_t launch_pcorr(const StagedArgs &a, long long tiles, int n_cu, hipStream_t stream);
const char *staged_kernel_name(int i);
// true when launch_staged runs k_olafb in place of k_ola, k_winmeta, k_fftbw
bool olafb_fused(const StagedArgs &a);
// The wave-per-frame FFT kernels (fvad_wave.hip), persistent grids; kWaveFftB
// needs fft_size 2048 (a 1024-point complex transform); kWaveOlaFb (k_ola +
// k_winmeta + k_fftbw fused) needs fft_size 2048 and n_channels <= 4.
enum WaveKernel { kWaveFftA, kWavePspec, kWaveSynth, kWaveFftB, kWaveOlaFb };
hipError_t launch_wave(WaveKernel which, const StagedArgs &a, int n_cu, hipStream_t stream);
// Device VADMachines over the window outputs a.out_* of one push: overlap =
// the light HBM variant meant to co-run with the next push on a side stream.
// fast: k_vadm_par (a burst of 16 lanes per stream, for a GPU with nothing
// else queued) where it applies, else k_vadm_hbm (32 waves, overlaps quietly);
// *ran_par (nullable): which of the two was launched
hipError_t launch_vadm(const StagedArgs &a, hipStream_t stream, bool fast = false, bool *ran_par = nullptr);
// use_denoiser = 0 (VAD.zig:206-212,239-249): k_ndring, k_ndmeta, FFT B
hipError_t launch_nodenoise(const StagedArgs &a, int n_cu, hipStream_t stream);
// k_fftb's scratch need: 0 when a transform fits in LDS, else float2 per workgroup
long long fftb_work_stride(int nfft_b, int bin_lo_all, int bin_hi_all, int generic);
bool fftb_generic(int nc);  // kf_factor(nc) has a radix > 5
// 16-bit ingest: dst[i] = src[i] / 32768.0f (exact), n a multiple of 8
hipError_t launch_pcm16(const int16_t *src, float *dst, size_t n, hipStream_t stream);
// fp16 / MFMA recurrence (fvad_gru16.hip), run in k_rnn3's place when a.gru16_frags is set;
// with a.fuse16 it is k_fused16, which also does k_pspecw's work
hipError_t launch_gru16(const StagedArgs &a, hipStream_t stream);
int gru16_frag_count();   // A fragments of 64 lanes x 8 f16
int gru16_bias_rows();
void gru16_build(const int8_t *rnn_img, uint16_t *frags, float *bias);

}  // namespace fvad
