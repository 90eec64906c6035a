/*
 * fvad.h — C ABI of the MI355X-native Formula-VAD hot path (libfvad.so).
 *
 * Plain C types only (pointers, sizes, ints, floats): a Zig host can
 * @cImport this header exactly as the reference @cImports rnnoise.h and
 * kiss_fftr.h today (src/Denoiser.zig:12-14, src/FFT.zig:5-9).
 *
 * Three layers:
 *   1. compatibility shims with the signatures and semantics the reference
 *      binds today (rnnoise_*, kiss_fftr*) — batch-of-1 calls into the HIP
 *      kernels;
 *   2. the batched engine (fvad_engine_*): thousands of concurrent 48 kHz
 *      streams per GPU, one tick = 480 samples per channel per stream;
 *   3. the host mirror of the reference pipeline / evaluator API
 *      (fvad_pipeline_*, fvad_vadm_*, fvad_eval_*), C++ above this ABI.
 *
 * Every entry point returns an int status (FVAD_OK = 0, negative = error)
 * unless noted; fvad_last_error() gives the message of the last failure on the
 * calling thread.  Ownership: the library owns device buffers and handles; the
 * caller owns every host array it passes.
 */
#ifndef FVAD_H
#define FVAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FVAD_OK 0
#define FVAD_EINVAL (-1)   /* invalid argument / size (Denoiser.zig:48-54, FFT.zig:29-31,71-81) */
#define FVAD_EDEVICE (-2)  /* HIP runtime / device error, or no device */
#define FVAD_ENOMEM (-3)   /* host or device allocation failed */
#define FVAD_EIO (-4)      /* file could not be opened */
#define FVAD_EFORMAT (-5)  /* malformed model / plan / label file */
#define FVAD_ERATE (-6)    /* sample rate != 48000 (VAD.zig:101-104) */

const char *fvad_last_error(void);
const char *fvad_version(void);

/* ------------------------------------------------------------------ */
/* 1a. rnnoise compatibility (replaces lib/rnnoise as bound by          */
/*     src/Denoiser.zig:12-14,23,36,60,69)                              */
/* ------------------------------------------------------------------ */
typedef struct fvad_model fvad_model;
typedef struct DenoiseState DenoiseState;
typedef struct fvad_model RNNModel;

/* rnnoise_create(RNNModel *model) — Denoiser.zig:23.  model == NULL selects
 * the process-wide default model (fvad_set_default_model, else the synthetic
 * model with seed 0, since rnn_data.c is not available).  Returns NULL on
 * failure (as upstream; Denoiser.zig:46 checks for it). */
DenoiseState *rnnoise_create(RNNModel *model);
/* rnnoise_destroy — Denoiser.zig:36 */
void rnnoise_destroy(DenoiseState *st);
/* rnnoise_process_frame — Denoiser.zig:60.  in/out: 480 floats in s16 scale;
 * returns the VAD probability.  Runs the HIP frame kernel (batch of 1). */
float rnnoise_process_frame(DenoiseState *st, float *out, const float *in);
/* rnnoise_get_frame_size — Denoiser.zig:69 (returns 480) */
int rnnoise_get_frame_size(void);
void fvad_set_default_model(const fvad_model *model);

/* ------------------------------------------------------------------ */
/* 1b. kissfft compatibility (replaces lib/kissfft as bound by           */
/*     src/FFT.zig:5-9,90,179-208)                                       */
/* ------------------------------------------------------------------ */
typedef struct { float r; float i; } kiss_fft_cpx;
typedef struct kiss_fftr_state *kiss_fftr_cfg;
/* kiss_fftr_alloc — FFT.zig:183,199.  Same lenmem protocol: with mem == NULL
 * or *lenmem too small it returns NULL and writes the required size into
 * *lenmem; otherwise the config lives in the caller's memory.  Forward only;
 * nfft must be even (kissfft's mixed radix: factors 4, 2, 3, 5 and generic
 * primes, as kf_factor picks them; the reference uses 2048). */
kiss_fftr_cfg kiss_fftr_alloc(int nfft, int inverse_fft, void *mem, size_t *lenmem);
/* kiss_fftr — FFT.zig:90.  timedata: nfft floats; freqdata: nfft/2+1 bins. */
void kiss_fftr(kiss_fftr_cfg cfg, const float *timedata, kiss_fft_cpx *freqdata);

/* ------------------------------------------------------------------ */
/* Models (rnn_data.c / rnn_reader.c replacement)                       */
/* ------------------------------------------------------------------ */
int fvad_model_synthetic(uint64_t seed, fvad_model **out);
int fvad_model_load_text(const char *path, fvad_model **out);
void fvad_model_free(fvad_model *m);
/* all int8 arrays in text-file order; returns the count (blob may be NULL) */
size_t fvad_model_blob(const fvad_model *m, int8_t *blob);

/* ------------------------------------------------------------------ */
/* 2. Batched engine — the hot path                                     */
/*    One engine = one GPU = a partition of streams.  A tick is 480      */
/*    samples of every channel of every stream (VAD.zig:214-251 frame    */
/*    loop, Denoiser per channel on one shared state VAD.zig:274-296,    */
/*    480 -> fft_size re-blocking VAD.zig:298-348, FFT B + band sum      */
/*    PipelineFFT.zig:88-112).                                            */
/* ------------------------------------------------------------------ */
typedef struct fvad_engine fvad_engine;

#define FVAD_MAX_CHANNELS 8
#define FVAD_MAX_BANDS 4

typedef struct {
  int n_streams;        /* streams in this engine's partition */
  int n_channels;       /* channels per stream (2 = onboard stereo) */
  int device;           /* HIP device ordinal */
  int sample_rate;      /* must be 48000 */
  int fft_size;         /* VAD.Config.fft_size: even, 2..4194304 (FFT.zig:29-31; fused mode: 480..2048,
                         * radices 2..5).  Below 480 one tick completes several windows (VAD.zig:307-347):
                         * see fvad_engine_windows_per_tick */
  int max_ticks;        /* largest n_ticks per push */
  int n_bands;          /* band sums to report per window, 1..4 */
  int band_lo[FVAD_MAX_BANDS]; /* inclusive FFT-B bin ranges (FFT.freqToBin) */
  int band_hi[FVAD_MAX_BANDS];
  int want_denoised;    /* keep denoised PCM (VAD.zig temp_denoiser_segment) */
  int mode;             /* FVAD_MODE_STAGED (default), FVAD_MODE_FUSED, FVAD_MODE_FP16 or FVAD_MODE_FP16_FUSED */
  int use_denoiser;     /* VAD.Config.use_denoiser (default 1).  0: fft_size frames of raw input go
                         * straight to FFT B (VAD.zig:206-212,239-249); per-tick vad / ratio are -1,
                         * the window ratio is preAnalyzeSegment's over the frame, window vad -1 */
  /* ABI note (r5): the trailing `unsigned cu_mask[8]` of earlier builds was removed; a binding
   * compiled against them must drop it (fvad_engine_config_default fills every field) */
} fvad_engine_config;

/* staged: time-parallel frame kernels + a thin per-stream recurrence kernel;
 * fused: one workgroup runs every frame of a stream (lower memory); staged
 * and fused give identical results (bit-exact with the CPU reference).
 * fp16: BASELINE configs[4] -- the staged pipeline with the GRU stack on the
 * matrix cores (int8 weights as f16, f16 inputs, f32 accumulation): within
 * the stated tolerance (vad |d| <= 2e-2), not bit-exact.
 * fp16_fused: configs[4]'s fused FFT -> feature -> GRU kernel -- fp16 with
 * the pitch-spectrum FFT and its features computed inside the GRU kernel
 * (k_fused16 replaces k_pspecw + k_gru16); results identical to fp16's. */
#define FVAD_MODE_STAGED 0
#define FVAD_MODE_FUSED 1
#define FVAD_MODE_FP16 2
#define FVAD_MODE_FP16_FUSED 3
#define FVAD_MAX_TIMES 16

void fvad_engine_config_default(fvad_engine_config *cfg, int n_streams, int n_channels);

int fvad_engine_create(const fvad_engine_config *cfg, const fvad_model *model, fvad_engine **out);
void fvad_engine_destroy(fvad_engine *e);
/* reset every stream to a freshly created rnnoise / VAD state */
int fvad_engine_reset(fvad_engine *e);

/* Per-tick outputs, host arrays owned by the caller, indexed [tick][stream]...
 * Any pointer may be NULL to skip that output.  The window outputs have W =
 * fvad_engine_windows_per_tick(e) slots per (tick, stream): W = 1 for fft_size
 * >= 480 (the layout is then [ticks][streams]...), more below 480, where one
 * 480-sample frame fills several FFT buffers (VAD.zig:307-347); slot w < the
 * tick's win_flag holds the tick's w-th completed window, in sample order. */
typedef struct {
  float *vad;          /* [ticks][streams]  min over channels of rnnoise vad (VAD.zig:284-293) */
  float *ratio;        /* [ticks][streams]  preAnalyzeSegment volume ratio (VAD.zig:253-272) */
  int32_t *win_flag;   /* [ticks][streams]  FFT-B windows completed in this tick (0..W; 0 or 1 when W = 1) */
  float *win_ratio;    /* [ticks][streams][W]  share-weighted window volume ratio (VAD.zig:319-325) */
  float *win_vad;      /* [ticks][streams][W]  window vad = last frame's vad (VAD.zig:330) */
  float *band;         /* [ticks][streams][W][channels][n_bands] band sums (PipelineFFT.zig:99-112); 0 in
                        * slots without a window */
  float *denoised;     /* [ticks][streams][channels][480] normalised denoised PCM (want_denoised) */
} fvad_outputs;

/* W, the window slots per (tick, stream) of fvad_outputs: 1 for fft_size >=
 * 480, else floor((fft_size - 1 + 480) / fft_size) -- the most windows one
 * tick can complete */
int fvad_engine_windows_per_tick(const fvad_engine *e);

/* pcm: host [ticks][streams][channels][480] normalised f32.  ticks_valid
 * (nullable): stream s only consumes its first ticks_valid[s] ticks (ragged
 * end of file; the rest of its slots are ignored).  Synchronous. */
int fvad_engine_push(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                     fvad_outputs *out);
/* The same with last_tick_samples (nullable): stream s's last valid tick holds
 * only last_tick_samples[s] (1..480) real samples, the rest of its slot is
 * ignored.  Only use_denoiser = 0 engines accept a partial tick: that path
 * reads fft_size frames (VAD.zig:206-220) and counts samples, so a window
 * completes as soon as its last sample is in, whatever the push sizes; with
 * the denoiser a frame needs all 480 samples (FVAD_EINVAL otherwise). */
int fvad_engine_push_ex(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                        const int32_t *last_tick_samples, fvad_outputs *out);

/* Streaming ingest (the simulator's read loop, SimulationInstance.zig:194-203,
 * reads the next chunk while the pipeline works on the last one).  Up to
 * FVAD_MAX_IN_FLIGHT pushes may be in flight: submit copies the input into a
 * pinned slot (or takes it in place when pcm is the pointer
 * fvad_engine_input_slot returned), queues the H2D copy on its own stream --
 * overlapping the earlier pushes' kernels; it waits only until the device
 * input buffer it fills has been read by the k_prep3 of the push two before --
 * then the kernels and the output copies into pinned memory, and returns
 * without waiting.  collect returns the outputs of the oldest submitted push
 * (blocking until they are on the host; out may be NULL, *n_ticks its tick
 * count).  submit fails with FVAD_EINVAL while FVAD_MAX_IN_FLIGHT pushes are
 * uncollected. */
#define FVAD_MAX_IN_FLIGHT 3
/* the pinned [max_ticks][streams][channels][480] slot the next submit reads;
 * blocks until that slot's previous copy to the device finished; NULL on error */
float *fvad_engine_input_slot(fvad_engine *e);
int fvad_engine_submit(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid);
int fvad_engine_submit_ex(fvad_engine *e, const float *pcm, int n_ticks, const int32_t *ticks_valid,
                          const int32_t *last_tick_samples);
int fvad_engine_collect(fvad_engine *e, fvad_outputs *out, int *n_ticks);
/* 16-bit PCM ingest (onboard WAV audio is 16-bit): the same push as
 * fvad_engine_submit_ex on the samples k / 32768.0f (libsndfile's short ->
 * float normalisation, as the reference's sf_read_float gives
 * AudioPipeline.pushSamples, src/AudioPipeline.zig:86-120; exact in f32), so
 * the outputs are bit-identical to a float submit of those samples.  Half the
 * host-to-device bytes; the conversion runs on the device: staged engines
 * with the denoiser read the 16-bit samples in k_prep3 itself, the others
 * convert on the copy stream (k_pcm16).  The slot and the submit/collect
 * rules are fvad_engine_input_slot's and fvad_engine_submit's. */
int16_t *fvad_engine_input_slot_i16(fvad_engine *e);
int fvad_engine_submit_i16(fvad_engine *e, const int16_t *pcm, int n_ticks, const int32_t *ticks_valid,
                           const int32_t *last_tick_samples);

/* Device-resident variants for benchmarking / zero-copy producers. */
/* allocate a device input of n_ticks and fill it with the synthetic generator */
int fvad_engine_load_synthetic(fvad_engine *e, int n_ticks, uint32_t stream_id_base);
/* n_pushes distinct pushes of n_ticks resident in HBM: stream s's first
 * n_pushes * n_ticks ticks of fvad_synth_stream(stream_id_base + s) (generated
 * at that length); run_resident cycles through them, starting at push 0 */
int fvad_engine_load_synthetic_ex(fvad_engine *e, int n_ticks, int n_pushes, uint32_t stream_id_base);
/* the resident push the next run_resident reads */
int fvad_engine_resident_seek(fvad_engine *e, int push);
/* run one push over the resident device input (the next one of the cycle),
 * async on the engine stream */
int fvad_engine_run_resident(fvad_engine *e, int n_ticks);
int fvad_engine_sync(fvad_engine *e);
/* average per-launch kernel durations (ms) of the timed resident runs,
 * measured with HIP events on the engine's stream.  ms_avg holds
 * FVAD_MAX_TIMES doubles: [0] whole push (GPU time from its first to its last
 * kernel; staged kernels may overlap), [1 + i] kernel i (names below).  With
 * device VADMachines the last two names are k_vadm_hbm (a push's machine run
 * beside the next push) and k_vadm_par (the push whose machine ran at a sync
 * point, nothing queued behind it), each averaged over its own runs. */
int fvad_engine_kernel_times(fvad_engine *e, double *ms_avg, int *n_runs);
/* name of kernel i of this engine's mode, NULL past the last one */
const char *fvad_engine_kernel_name(const fvad_engine *e, int i);
int fvad_engine_clear_times(fvad_engine *e);
/* copy outputs of the last resident run to host */
int fvad_engine_fetch(fvad_engine *e, int n_ticks, fvad_outputs *out);

/* ------------------------------------------------------------------ */
/* 3. Host mirror of the reference API (C++ above this ABI)             */
/* ------------------------------------------------------------------ */
/* VADMachine.Config (VADMachine.zig:18-39) */
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
} fvad_vadm_config;
void fvad_vadm_config_default(fvad_vadm_config *c);

/* VAD.VADSpeechSegment (VAD.zig:25-30) */
typedef struct {
  uint64_t sample_from, sample_to;
  float debug_rnn_vad, debug_avg_speech_vol_ratio;
} fvad_segment;

/* VADMachine (VADMachine.zig:65-310) on its own: feed it one FFT-B window at a
 * time (absolute sample index of the window start, the per-channel band sums
 * of its speech band, the window's vad and volume ratio). */
typedef struct fvad_vadm fvad_vadm;
int fvad_vadm_create(const fvad_vadm_config *cfg, int sample_rate, int fft_size, int n_channels, fvad_vadm **out);
void fvad_vadm_destroy(fvad_vadm *v);
/* speech band as FFT-B bins (FFT.freqToBin of speech_min/max_freq) */
void fvad_vadm_bins(const fvad_vadm *v, int *lo, int *hi);
int fvad_vadm_run(fvad_vadm *v, uint64_t index, const float *band_per_channel, float vad, float vol_ratio);
size_t fvad_vadm_segments(const fvad_vadm *v, fvad_segment *out, size_t cap);

/* Device VADMachines (VADMachine.zig:126-230 run on the GPU, one lane per
 * stream, after FFT B of every push).  Staged engines only.
 * Each config's speech band (FFT.freqToBin of speech_min/max_freq) must be one
 * of the engine's bands.  Up to FVAD_MAX_BANDS machines; segments accumulate
 * on the device, seg_capacity per (stream, machine); a reset clears them.
 * A push's machines are enqueued when the next push is launched (beside it, on
 * a side stream) or at the next sync point (fvad_engine_sync, _segments,
 * _vadm_state, _vadm_snapshot, _kernel_times), so after submit / collect the
 * last collected push's windows are not in the machine state yet; every
 * reader above flushes them first.  A reset or destroy drops them. */
int fvad_engine_attach_vadm(fvad_engine *e, const fvad_vadm_config *cfgs, int n, int seg_capacity);
/* total segments of (stream, machine) so far; copies min(total, capacity, cap) */
size_t fvad_engine_segments(fvad_engine *e, int stream, int machine, fvad_segment *out, size_t cap);
/* the same from segment index `first` on (returns the total count) */
size_t fvad_engine_segments_range(fvad_engine *e, int stream, int machine, size_t first, fvad_segment *out,
                                  size_t cap);
/* speech state of an attached machine (VADMachine.zig:11-16: 0 closed, 1 opening,
 * 2 open, 3 closing) and its current speech start / end sample indices */
int fvad_engine_vadm_state(fvad_engine *e, int stream, int machine, int *speech_state, uint64_t *speech_start,
                           uint64_t *speech_end);
/* The whole state of an attached machine in the reference's terms
 * (VADMachine.zig:65-125 fields; RollingAverage.zig:5-14 for long_term [0],
 * short_term [1] and the channel volume ratio [2]), after every queued push:
 * what a checker compares with a CPU VADMachine fed the same windows. */
typedef struct {
  int speech_state;                 /* 0 closed, 1 opening, 2 open, 3 closing */
  uint64_t speech_start, speech_end;  /* speech_start_index, speech_end_index */
  uint64_t windows;                 /* windows the machine has run */
  double avg[3];                    /* RollingAverage.last_avg (0 before the first avg) */
  uint64_t write_idx[3];            /* RollingAverage.write_idx */
  uint64_t written[3];              /* RollingAverage.written_count */
  float speech_rnn_vad, speech_vol_ratio;  /* the current speech's tracked sums */
  uint64_t speech_rnn_vad_count, speech_vol_ratio_count;
  uint64_t n_segments;              /* segments emitted so far (also past seg_capacity) */
} fvad_vadm_snapshot;
int fvad_engine_vadm_snapshot(fvad_engine *e, int stream, int machine, fvad_vadm_snapshot *out);
/* RollingAverage.data of (stream, machine), which = 0 long-term, 1 short-term,
 * 2 volume ratio, as doubles: copies min(len, cap) entries, returns len (< 0:
 * error code) */
long fvad_engine_vadm_rolling(fvad_engine *e, int stream, int machine, int which, double *out, size_t cap);

/* Several engines on one GPU (e.g. a GPU's streams split into sub-partitions
 * that push concurrently): e runs its k_prep3 (FVAD_SHARE_PREP) and / or its
 * device VADMachine kernels (FVAD_SHARE_SIDE, both engines with machines
 * attached) on other's streams from now on, so the engines' side work queues
 * in order instead of taking a hardware queue each (a process gets
 * GPU_MAX_HW_QUEUES of them, 4 by default, shared round-robin once they run
 * out: a main stream sharing one with another engine's k_prep3 waits for it).
 * Synchronises both engines; results are unchanged (dependencies are events).
 * Only k_prep3 moves: an engine alone on its prep stream also runs k_fftAw
 * there (beside its previous push's tail), one whose prep stream is shared
 * runs k_fftAw on its own engine stream, so the main pipelines stay
 * uncoupled.  The last engine using a stream destroys it. */
#define FVAD_SHARE_PREP 1
#define FVAD_SHARE_SIDE 2
int fvad_engine_share_streams(fvad_engine *e, fvad_engine *other, int which);

/* Test hooks: knobs and a recorder the parity tests use; no product path sets
 * them.  fvad_engine_set_debug keys:
 *   FVAD_DEBUG_VADM_PAR_SERIAL_EVERY  value k > 0: k_vadm_par hands every
 *     stream s with s % k == 0 to its in-kernel serial walk (the fallback for a
 *     machine outside the window-parallel case); 0: never (default)
 *   FVAD_DEBUG_VADM_ALWAYS_PAR  value 1: every push's VADMachine runs as
 *     k_vadm_par, not only the one flushed at a sync point
 *   FVAD_DEBUG_VADM_LT_FULL  value 1: the machines restart (as by a reset)
 *     with every long-term entry counted as pushed, holding (float)init: the
 *     long-term walk of a stream past its first long_term_speech_avg_sec, for
 *     timing (tools/vadm_steady.py); the values then differ from the reference
 *   FVAD_DEBUG_VADM_DEFER_MAX  value k > 0: between sync points k_vadm_hbm
 *     folds a machine's long-term average once k long pushes are owed (1: at
 *     the end of every push); 0: the default bound (4096).  Results are the
 *     same for every k: a sync point resolves every owed fold
 *   FVAD_DEBUG_VADM_BOUND_SCALE  value k > 0: the lazy long-term walk's error
 *     bound E (fvad_exact.h lt_bound) times k; -1: infinite, so every test the
 *     estimate would decide takes the exact fold instead; 0: back to 1.
 *     Results are the same for every k >= 1
 *   FVAD_DEBUG_VADM_COUNT  value 1: count the long-term tests by how they were
 *     decided (fvad_engine_debug_counts), from zero; 0: stop counting
 *   FVAD_DEBUG_VADM_NEGATE_AT  value k >= 0: window k of every stream enters
 *     every machine with its band minimum negated (a value the pipeline never
 *     produces: the path that folds exactly until that entry has left the
 *     long-term buffer); -1: off (default) */
#define FVAD_DEBUG_VADM_PAR_SERIAL_EVERY 1
#define FVAD_DEBUG_VADM_ALWAYS_PAR 2
#define FVAD_DEBUG_VADM_LT_FULL 3
#define FVAD_DEBUG_VADM_DEFER_MAX 4
#define FVAD_DEBUG_VADM_BOUND_SCALE 5
#define FVAD_DEBUG_VADM_COUNT 6
#define FVAD_DEBUG_VADM_NEGATE_AT 7
int fvad_engine_set_debug(fvad_engine *e, int key, int value);
/* FVAD_DEBUG_VADM_COUNT's counters, out[0..min(n, 4)): long-term tests decided
 * from an exact average, tests the bound settled from the estimate, tests it
 * left open (an exact fold), folds at the end of a push.  Returns the count
 * written (synchronises the engine). */
int fvad_engine_debug_counts(fvad_engine *e, unsigned long long *out, int n);
/* Output log: the per-tick outputs (fvad_outputs without denoised) of the next
 * n_pushes pushes are copied into device memory on the engine stream as each
 * push's kernels end -- no host synchronisation, so a run of asynchronous
 * pushes (run_resident, submit) keeps its schedule; read them back after the
 * pushes with fvad_engine_output_log_read (push = 0 .. n_pushes - 1 in launch
 * order).  n_pushes = 0 frees the log.  Staged / fp16 engines with the denoiser. */
int fvad_engine_output_log(fvad_engine *e, int n_pushes);
int fvad_engine_output_log_read(fvad_engine *e, int push, fvad_outputs *out, int *n_ticks);

/* VAD.Config (VAD.zig:17-23) */
typedef struct {
  int fft_size;                                     /* even, 2..4194304 (FFT.zig:28-31) */
  int use_denoiser;                                 /* 0: fft_size frames of raw input to FFT B */
  fvad_vadm_config vad_machine_config;              /* main machine */
  const fvad_vadm_config *alt_vad_machine_configs;  /* alternative machines (training), nullable */
  int n_alt;                                        /* <= FVAD_MAX_BANDS - 1 */
} fvad_vad_config;
void fvad_vad_config_default(fvad_vad_config *c);

/* AudioPipeline (AudioPipeline.zig:20-26,39-120) for one stream, backed by a
 * 1-stream engine.  n_alt alternative VADMachine configs (VAD.zig:20-23). */
typedef struct fvad_pipeline fvad_pipeline;
int fvad_pipeline_create(int sample_rate, int n_channels, const fvad_model *model, int device,
                         const fvad_vadm_config *main_cfg, const fvad_vadm_config *alt_cfgs, int n_alt,
                         fvad_pipeline **out);
/* the same with a whole VAD.Config (fft_size, use_denoiser, machines) */
int fvad_pipeline_create_ex(int sample_rate, int n_channels, const fvad_model *model, int device,
                            const fvad_vad_config *vad_config, fvad_pipeline **out);
void fvad_pipeline_destroy(fvad_pipeline *p);
/* pushSamples: planar channel pointers, n samples each; *first_index receives
 * the absolute index of the first pushed sample (AudioPipeline.zig:86-120) */
int fvad_pipeline_push(fvad_pipeline *p, const float *const *channel_pcm, size_t n, uint64_t *first_index);
/* vad_segments of the main (alt < 0) or an alternative machine */
size_t fvad_pipeline_segments(const fvad_pipeline *p, int alt, fvad_segment *out, size_t cap);

/* Recorder (Recorder.zig:95-110 findBestChannel): the channel with the lowest
 * rmsVolume (audio_utils.zig:14-24) over n samples; the first one on ties. */
int fvad_recording_channel(const float *const *channel_pcm, int n_channels, size_t n);
/* on_recording (AudioPipeline.zig:15-18, :134-195, Recorder.zig:52-146): called
 * from fvad_pipeline_push once per completed main-machine segment with the raw
 * pushed input of [sample_from, sample_to) on its lowest-RMS channel
 * (AudioBuffer: one channel, global_start_frame_number = start_sample).
 * fn = NULL detaches; only segments completed after attaching are recorded. */
typedef void (*fvad_recording_fn)(void *ctx, const float *pcm, size_t n, uint64_t start_sample, int channel);
int fvad_pipeline_set_recorder(fvad_pipeline *p, fvad_recording_fn fn, void *ctx);

/* Multi-stream simulator core (simulator.zig:217-228 runs one thread per
 * instance): streams grouped by channel count, each group partitioned
 * contiguously over the devices, one engine + host thread per part, lock-step
 * pushes of ticks_per_push ticks.  pcm[s] points to planar [channels][len[s]]
 * audio of stream s (fvad_multi_run), or a reader pulls it push by push
 * (fvad_multi_run_stream: the simulator's streaming read loop,
 * SimulationInstance.zig:171-203). */
typedef struct fvad_multi fvad_multi;
int fvad_multi_create(int n_streams, int n_channels, const fvad_model *model, const int *devices,
                      int n_devices, const fvad_vadm_config *cfg, int ticks_per_push, fvad_multi **out);
/* per-stream channel counts and a whole VAD.Config */
int fvad_multi_create_ex(int n_streams, const int *n_channels, const fvad_model *model, const int *devices,
                         int n_devices, const fvad_vad_config *vad_config, int ticks_per_push, fvad_multi **out);
void fvad_multi_destroy(fvad_multi *m);
int fvad_multi_run(fvad_multi *m, const float *const *pcm, const size_t *len);
/* reader: write up to max_frames frames of stream `stream` planar into
 * channel_dst[c][0..), return the count (0 = end of stream).  Called from the
 * part threads; a stream is always read by the same thread, in order. */
typedef size_t (*fvad_read_fn)(void *ctx, int stream, float *const *channel_dst, size_t max_frames);
int fvad_multi_run_stream(fvad_multi *m, fvad_read_fn read, void *ctx);
/* segments of the main machine (machine 0) or alternative machine i (machine i + 1) */
size_t fvad_multi_segments_alt(const fvad_multi *m, int stream, int machine, fvad_segment *out, size_t cap);
size_t fvad_multi_segments(const fvad_multi *m, int stream, fvad_segment *out, size_t cap);

/* Evaluator / statistics (Evaluator.zig:90-156, statistics.zig:85-284) */
typedef struct {
  float ignore_shorter_than_sec, extrude_start, extrude_end, fill_gaps;
} fvad_stat_config;
typedef struct {
  float total_positives_sec, true_positives_sec, false_positives_sec, false_negatives_sec;
  float true_positive_rate, false_negative_rate, false_discovery_rate, precision;
  float fm_index, f_score, f_score_beta;
} fvad_single_stats;
typedef struct { float overall, min, max, avg; } fvad_agg_stat;
typedef struct {
  float total_positives_sec, true_positives_sec, false_positives_sec, false_negatives_sec;
  fvad_agg_stat true_positive_rate, false_negative_rate, false_discovery_rate, precision;
  float fm_index, f_score, f_score_beta;
} fvad_aggregate_stats;
/* segments as (from_sec, to_sec) pairs */
int fvad_eval_stats(const float *vad_from_to, size_t n_vad, const float *ref_from_to, size_t n_ref,
                    const fvad_stat_config *cfg, fvad_single_stats *out);
void fvad_eval_aggregate(const fvad_single_stats *stats, size_t n, fvad_aggregate_stats *out);
/* formats.parseAudacitySegments (formats.zig:7-36): returns count or <0 */
long fvad_parse_audacity(const char *txt, size_t len, float *from_to, size_t cap);

/* Synthetic 48 kHz onboard audio; returns label count */
long fvad_synth_stream(uint32_t stream_id, size_t n, int n_channels, float *out, float *labels,
                       size_t label_cap);

/* The same streams in the engine's push layout: ticks [tick0, tick0 + n_ticks)
 * of streams base .. base + n_streams - 1, each generated at total_ticks * 480
 * samples, into out[t][s][c][480].  The last whole block is cached in host
 * memory (fvad_synth_cache_clear frees it). */
int fvad_synth_ticks(uint32_t stream_id_base, int n_streams, int n_channels, int total_ticks, int tick0,
                     int n_ticks, float *out);
void fvad_synth_cache_clear(void);

/* simulator -i plan.json (simulator.zig:74-139) — returns process exit code */
int fvad_simulator_main(int argc, char **argv);

#ifdef __cplusplus
}
#endif
#endif
