/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, scalar, CPU restatement of Formula-VAD's per-frame hot path, used
 * exclusively as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing in the product (formula-vad_amd/) links,
 * loads or calls this code.
 *
 * What it restates (see DESIGN.md §Oracle for the full citation map):
 *   - rnnoise classic per-frame algorithm (xiph/rnnoise, pre-0.2 layout; the
 *     submodule lib/rnnoise is EMPTY in /root/reference, so this follows the
 *     published algorithm as recalled — SURVEY.md Appendix A), called from
 *     /root/reference/src/Denoiser.zig:45-66;
 *   - celt/opus mixed-radix kiss_fft used inside rnnoise (FFT A, 960 points);
 *   - mborgerding kissfft real FFT (FFT B) as wrapped by src/FFT.zig:70-98;
 *   - src/audio_utils/window_fn.zig, src/audio_utils.zig:14-24;
 *   - src/AudioPipeline.zig:86-157, src/AudioPipeline/VAD.zig:214-381,
 *     SegmentWriter.zig:40-108, PipelineFFT.zig:88-112, VADMachine.zig:126-310,
 *     structures/RollingAverage.zig, structures/MultiRingBuffer.zig;
 *   - src/Evaluator.zig:90-156, src/Evaluator/{statistics,formats,SpeechSegment}.zig.
 *
 * PARITY STATUS: "parity unpinned" against the true rnnoise/kissfft numerics
 * (their sources and the rnnoise weights are absent, the Zig toolchain is absent,
 * there is no network).  The oracle IS pinned against every known-answer vector
 * the reference's own tests hold (SegmentWriter.zig:124-175,
 * MultiRingBuffer.zig:203-249, statistics.zig:286-360) and against derived KATs
 * (FFT.zig normalisation, rnnoise analysis/synthesis perfect reconstruction,
 * silence gate, tansig/DCT tables) — see tests/test_oracle_*.py.
 *
 * Floating point: compiled with -ffp-contract=off, C promotion rules of the
 * recalled sources reproduced literally (double literals promote).
 */
#ifndef FVAD_ORACLE_H
#define FVAD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- rnnoise model ---------------- */
#define ORA_ACT_TANH 0
#define ORA_ACT_SIGMOID 1
#define ORA_ACT_RELU 2

typedef struct {
  int nb_inputs, nb_neurons, activation;
  int8_t *input_weights; /* [nb_inputs][nb_neurons] */
  int8_t *bias;          /* [nb_neurons] */
} ora_dense;

typedef struct {
  int nb_inputs, nb_neurons, activation;
  int8_t *input_weights;     /* [nb_inputs][3*nb_neurons] */
  int8_t *recurrent_weights; /* [nb_neurons][3*nb_neurons] */
  int8_t *bias;              /* [3*nb_neurons] */
} ora_gru;

typedef struct {
  ora_dense input_dense;
  ora_gru vad_gru, noise_gru, denoise_gru;
  ora_dense denoise_output, vad_output;
} ora_model;

ora_model *ora_model_synthetic(uint64_t seed);
ora_model *ora_model_from_text(const char *path);
void ora_model_free(ora_model *m);
/* Flatten all int8 arrays in text-file order; returns count (blob may be NULL). */
size_t ora_model_blob(const ora_model *m, int8_t *blob);

/* ---------------- rnnoise state ---------------- */
typedef struct ora_denoise ora_denoise;
ora_denoise *ora_rnnoise_create(const ora_model *m);
void ora_rnnoise_destroy(ora_denoise *st);
int ora_rnnoise_get_frame_size(void);
/* in/out: 480 floats in s16 scale. returns vad probability. */
float ora_rnnoise_process_frame(ora_denoise *st, float *out, const float *in);
/* test hook: 1 = force gains to 1 and skip the RNN / pitch filter (weight-free KAT) */
void ora_rnnoise_set_bypass(ora_denoise *st, int bypass);
/* instrumented work counts, added into counts[4]: frames, silent frames (E < 0.04:
 * no GRU, pitch filter or gains), fine-search lags computed, remove_doubling
 * candidates evaluated (the loop's break at T1 < minperiod) */
void ora_rnnoise_counts(const ora_denoise *st, uint64_t *counts);
/* debug: last frame's pitch index and gain, silence flag, features */
void ora_rnnoise_debug(const ora_denoise *st, int *pitch, float *gain, int *silence, float *features);

/* tables for KATs */
void ora_tables(float *half_window480, float *dct22x22, float *tansig201);
/* FFT A (celt kiss_fft, forward, scaled 1/n) on 960 complex points */
void ora_fft960(const float *in_ri, float *out_ri);

/* ---------------- kissfft real FFT (FFT B) ---------------- */
/* Same lenmem protocol as mborgerding kiss_fftr_alloc. */
void *ora_kiss_fftr_alloc(int nfft, int inverse, void *mem, size_t *lenmem);
void ora_kiss_fftr(void *cfg, const float *timedata, float *freqdata_ri);

/* ---------------- FFT.zig / window_fn.zig ---------------- */
void ora_hann_periodic(float *w, int n);
float ora_window_norm_factor(const float *w, int n);
/* FFT.fft: magnitude spectrum (n/2+1 bins) of samples*window, normalised */
int ora_fftzig(int nfft, const float *samples, const float *window, float *mag);
float ora_rms_volume(const float *x, int n);
int ora_recording_channel(const float *const *ch, int n_channels, int n); /* Recorder.zig:95-110 */

/* ---------------- reference unit-test restatements ---------------- */
/* SegmentWriter.write on a 1-channel segment with (first, second) split source */
typedef struct { float *buf; size_t len; size_t write_index; uint64_t index; } ora_segwriter;
size_t ora_segwriter_write(ora_segwriter *w, const float *first, size_t n_first,
                           const float *second, size_t n_second, size_t offset,
                           long max_write /* <0 = null */);
/* MultiRingBuffer(int32) write of one channel */
typedef struct { int32_t *buf; size_t capacity; uint64_t total_write_count; } ora_ring_i32;
size_t ora_ring_write(ora_ring_i32 *r, const int32_t *src, size_t src_len,
                      size_t src_read_offset, size_t max_write_count);

/* ---------------- VAD pipeline (AudioPipeline + VAD + VADMachine) ---------------- */
typedef struct {
  float speech_min_freq, speech_max_freq;
  float long_term_speech_avg_sec;
  int has_initial_long_term_avg;
  double initial_long_term_avg;
  float short_term_speech_avg_sec;
  float speech_threshold_factor;
  float channel_vol_ratio_avg_sec;
  float channel_vol_ratio_threshold;
  float min_consecutive_sec_to_open;
  float max_speech_gap_sec;
  float min_vad_duration_sec;
} ora_vadm_config;
void ora_vadm_config_default(ora_vadm_config *c);

typedef struct {
  uint64_t sample_from, sample_to;
  float debug_rnn_vad, debug_avg_speech_vol_ratio;
} ora_segment;

typedef struct ora_pipeline ora_pipeline;
/* fft_size: VAD.Config.fft_size; use_denoiser: VAD.Config.use_denoiser. buffer_length 0 = 10 s. */
ora_pipeline *ora_pipeline_create(int n_channels, int sample_rate, size_t buffer_length,
                                  int fft_size, int use_denoiser, const ora_model *model,
                                  const ora_vadm_config *main_cfg, const ora_vadm_config *alt_cfgs,
                                  int n_alt);
void ora_pipeline_destroy(ora_pipeline *p);
/* planar channel pointers, n samples each. returns first sample index. */
uint64_t ora_pipeline_push(ora_pipeline *p, const float *const *channel_pcm, size_t n);
/* main VADMachine segments (alt_idx<0) or alternative machine alt_idx */
size_t ora_pipeline_segments(const ora_pipeline *p, int alt_idx, ora_segment *out, size_t cap);
/* the machine's whole state (VADMachine.zig:65-125; RollingAverage.zig:5-14 for
 * long_term [0], short_term [1], ratio [2]); field layout of fvad.h's
 * fvad_vadm_snapshot, so the checker compares the two field by field */
typedef struct {
  int speech_state;
  uint64_t speech_start, speech_end, windows;
  double avg[3];
  uint64_t write_idx[3], written[3];
  float speech_rnn_vad, speech_vol_ratio;
  uint64_t speech_rnn_vad_count, speech_vol_ratio_count, n_segments;
} ora_vadm_snapshot;
void ora_pipeline_vadm_snapshot(const ora_pipeline *p, int alt_idx, ora_vadm_snapshot *out);
/* RollingAverage.data (which: 0 long_term, 1 short_term, 2 ratio); returns its length */
size_t ora_pipeline_vadm_rolling(const ora_pipeline *p, int alt_idx, int which, double *out, size_t cap);

/* per-frame trace of the hot path (filled when tracing is enabled) */
typedef struct {
  uint64_t frame_index; /* absolute sample index of the frame start */
  float vad_low;        /* min over channels of rnnoise vad */
  float vol_ratio;      /* preAnalyzeSegment ratio */
} ora_frame_trace;
typedef struct {
  uint64_t index;       /* absolute sample index of the window start */
  float band[8];        /* per channel band sum (main machine's band) */
  float vol_ratio;      /* share-weighted window ratio */
  float vad;            /* last contributing frame's vad (or -1 if no denoiser) */
} ora_window_trace;
void ora_pipeline_enable_trace(ora_pipeline *p, ora_frame_trace *frames, size_t frames_cap,
                               ora_window_trace *windows, size_t windows_cap, float *denoised,
                               size_t denoised_cap_samples_per_channel);
void ora_pipeline_trace_counts(const ora_pipeline *p, size_t *n_frames, size_t *n_windows);

/* ---------------- Evaluator ---------------- */
typedef struct {
  float ignore_shorter_than_sec, extrude_start, extrude_end, fill_gaps;
} ora_stat_config;
typedef struct {
  float total_positives_sec, true_positives_sec, false_positives_sec, false_negatives_sec;
  float true_positive_rate, false_negative_rate, false_discovery_rate, precision;
  float fm_index, f_score, f_score_beta;
} ora_single_stats;
typedef struct { float overall, min, max, avg; } ora_agg_stat;
typedef struct {
  float total_positives_sec, true_positives_sec, false_positives_sec, false_negatives_sec;
  ora_agg_stat true_positive_rate, false_negative_rate, false_discovery_rate, precision;
  float fm_index, f_score, f_score_beta;
} ora_aggregate_stats;

/* segments given as (from_sec, to_sec) pairs */
int ora_evaluate(const float *vad_from_to, size_t n_vad, const float *ref_from_to, size_t n_ref,
                 const ora_stat_config *cfg, ora_single_stats *out);
void ora_aggregate(const ora_single_stats *stats, size_t n, ora_aggregate_stats *out);
/* statistics.calcFalsePositiveSec on one vad segment against explicit matched refs */
float ora_calc_false_positive_sec(float vad_from, float vad_to, const float *ref_from_to,
                                  size_t n_ref, const ora_stat_config *cfg);
/* formats.parseAudacitySegments: returns count, writes up to cap (from,to) pairs */
long ora_parse_audacity(const char *txt, size_t len, float *from_to, size_t cap);

/* ---------------- CPU baseline timing ---------------- */
/* Run n_streams independent stereo/mono denoisers over n_frames frames of the given
 * interleaved pcm [frame][stream][ch][480] (s16 scale) using n_threads threads.
 * Returns seconds elapsed. */
double ora_bench_denoise(const ora_model *m, const float *pcm, int n_streams, int n_channels,
                         int n_frames, int n_threads, float *vad_out);
/* The whole per-stream path the GPU bench times: AudioPipeline.pushSamples ->
 * VAD (rnnoise, re-block, FFT B band sums) -> VADMachine (default config), one
 * pipeline per stream, pushed in chunks of `chunk` samples per channel.
 * pcm: planar [stream][ch][n_samples] in [-1, 1].  Pipelines are created
 * before and destroyed after the timed region; n_threads workers take
 * contiguous stream ranges (simulator.zig:217-228 runs a thread per
 * instance).  Returns seconds of the timed region; counts (nullable, [4]) as
 * ora_rnnoise_counts summed over the streams. */
double ora_bench_pipeline(const ora_model *m, const float *pcm, int n_streams, int n_channels,
                          size_t n_samples, size_t chunk, int n_threads, uint64_t *counts);
/* the rnnoise state of a pipeline (NULL without the denoiser) */
const ora_denoise *ora_pipeline_denoiser(const ora_pipeline *p);

#ifdef __cplusplus
}
#endif
#endif
