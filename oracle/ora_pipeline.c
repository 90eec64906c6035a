/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar restatement of the reference's frame dispatch and decision logic:
 *   MultiRingBuffer.writeAssumeCapacity / readSlice  (structures/MultiRingBuffer.zig:73-194)
 *   SegmentWriter.write / reset                      (AudioPipeline/SegmentWriter.zig:40-108)
 *   AudioPipeline.pushSamples                        (AudioPipeline.zig:86-120)
 *   VAD.collectInputStep / preAnalyzeSegment / denoiserStep / fftBufferStep / fftStep
 *                                                    (AudioPipeline/VAD.zig:214-381)
 *   Denoiser.denoise scaling                         (Denoiser.zig:45-94)
 *   PipelineFFT.fft / averageVolumeInBand            (AudioPipeline/PipelineFFT.zig:88-112)
 *   FFT.freqToBin                                    (FFT.zig:120-131)
 *   VADMachine.init / run / onSpeechEnd / margins    (AudioPipeline/VADMachine.zig:65-310)
 *   RollingAverage                                   (structures/RollingAverage.zig:1-56)
 * The Recorder side effect (AudioPipeline.zig:134-195, Recorder.zig) does not
 * influence any VAD decision and is not restated.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define MAXCH 8

/* ---------------- SegmentWriter (1 channel view used by the KAT) ---------------- */
size_t ora_segwriter_write(ora_segwriter *w, const float *first, size_t n_first,
                           const float *second, size_t n_second, size_t offset, long max_write) {
  const size_t capacity = w->len;
  const size_t remaining = (w->write_index < capacity) ? capacity - w->write_index : 0;
  const size_t other_len = n_first + n_second;
  size_t other_rem, to_write, nf;
  if (remaining == 0) return 0;
  other_rem = other_len - offset;
  if (max_write >= 0 && (size_t)max_write < other_rem) other_rem = (size_t)max_write;
  to_write = remaining < other_rem ? remaining : other_rem;
  nf = (n_first > offset) ? ((to_write < n_first - offset) ? to_write : n_first - offset) : 0;
  if (nf > 0) memcpy(w->buf + w->write_index, first + offset, nf * sizeof(float));
  if (nf < to_write) {
    const size_t rem = to_write - nf;
    const size_t src_from = (offset >= n_first) ? offset - n_first : 0;
    memcpy(w->buf + w->write_index + nf, second + src_from, rem * sizeof(float));
  }
  w->write_index += to_write;
  return to_write;
}

/* ---------------- MultiRingBuffer (single channel i32, KAT) ---------------- */
static size_t ring_write_assume(ora_ring_i32 *r, const int32_t *src, size_t n_total, size_t off,
                                size_t maxw) {
  const size_t dst = (size_t)(r->total_write_count % r->capacity);
  const size_t to_end = r->capacity - dst;
  const size_t src_rem = (n_total < off) ? 0 : n_total - off;
  const size_t n = src_rem < maxw ? src_rem : maxw;
  const size_t n1 = to_end < n ? to_end : n;
  const size_t n2 = n - n1;
  if (n == 0) return 0;
  memcpy(r->buf + dst, src + off, n1 * sizeof(int32_t));
  if (n2 > 0) memcpy(r->buf, src + off + n1, n2 * sizeof(int32_t));
  r->total_write_count += n;
  return n;
}

size_t ora_ring_write(ora_ring_i32 *r, const int32_t *src, size_t src_len, size_t off, size_t maxw) {
  /* MultiRingBuffer.write: split into capacity-sized steps (MultiRingBuffer.zig:51-71) */
  const size_t max_src = off + maxw;
  size_t written = 0;
  for (;;) {
    const size_t step_off = off + written;
    size_t step_max = max_src - step_off;
    size_t n;
    if (r->capacity < step_max) step_max = r->capacity;
    n = ring_write_assume(r, src, src_len, step_off, step_max);
    written += n;
    if (n < r->capacity) break;
  }
  return written;
}

/* ---------------- RollingAverage ---------------- */
typedef struct {
  double *data;
  size_t len, write_idx, written_count;
  int has_last;
  double last_avg;
} rolling;

static double rolling_avg(rolling *r) {
  double avg = 0.0;
  const double scalar = 1.0 / (double)r->written_count;
  size_t i;
  for (i = 0; i < r->written_count; i++) avg += r->data[i] * scalar;
  r->last_avg = avg;
  r->has_last = 1;
  return avg;
}

static void rolling_init(rolling *r, size_t count, int has_init, double init) {
  size_t i;
  memset(r, 0, sizeof(*r));
  r->len = count;
  r->data = (double *)calloc(count ? count : 1, sizeof(double));
  if (has_init) {
    for (i = 0; i < count; i++) r->data[i] = init;
    r->written_count = count;
    rolling_avg(r);
  }
}

static double rolling_push(rolling *r, float sample) {
  r->data[r->write_idx] = (double)sample;
  r->write_idx = (r->write_idx + 1) % r->len;
  if (r->written_count < r->len) r->written_count++;
  return rolling_avg(r);
}

/* ---------------- VADMachine ---------------- */
void ora_vadm_config_default(ora_vadm_config *c) {
  c->speech_min_freq = 100;
  c->speech_max_freq = 1500;
  c->long_term_speech_avg_sec = 180;
  c->has_initial_long_term_avg = 1;
  c->initial_long_term_avg = 0.005;
  c->short_term_speech_avg_sec = 0.2f;
  c->speech_threshold_factor = 18;
  c->channel_vol_ratio_avg_sec = 0.5f;
  c->channel_vol_ratio_threshold = 0.5f;
  c->min_consecutive_sec_to_open = 0.2f;
  c->max_speech_gap_sec = 2;
  c->min_vad_duration_sec = 0.7f;
}

enum { ST_CLOSED = 0, ST_OPENING, ST_OPEN, ST_CLOSING };

typedef struct {
  ora_vadm_config cfg;
  int sample_rate, n_channels, fft_size;
  int state;
  rolling long_term, short_term, ratio;
  uint64_t speech_start_index, speech_end_index;
  float speech_rnn_vad;
  size_t speech_rnn_vad_count;
  float speech_vol_ratio;
  size_t speech_vol_ratio_count;
  ora_segment *segs;
  size_t n_segs, cap_segs;
  size_t min_bin, max_bin;
  uint64_t n_runs; /* windows run (checker bookkeeping, not a reference field) */
} vadm;

static size_t freq_to_bin(int sample_rate, int nfft, float freq) {
  const float bin_width = (float)sample_rate / (float)nfft;
  return (size_t)roundf(freq / bin_width); /* Zig @round: half away from zero == roundf */
}

static void vadm_init(vadm *m, const ora_vadm_config *cfg, int sample_rate, int n_channels, int fft_size) {
  const float eval_per_sec = (float)sample_rate / (float)fft_size;
  const size_t lt = (size_t)(eval_per_sec * cfg->long_term_speech_avg_sec);
  const size_t st = (size_t)(eval_per_sec * cfg->short_term_speech_avg_sec);
  const size_t cr = (size_t)(eval_per_sec * cfg->channel_vol_ratio_avg_sec);
  memset(m, 0, sizeof(*m));
  m->cfg = *cfg;
  m->sample_rate = sample_rate;
  m->n_channels = n_channels;
  m->fft_size = fft_size;
  rolling_init(&m->long_term, lt > 1 ? lt : 1, cfg->has_initial_long_term_avg, cfg->initial_long_term_avg);
  rolling_init(&m->short_term, st > 1 ? st : 1, 0, 0);
  rolling_init(&m->ratio, cr, 0, 0);
  m->cap_segs = 100;
  m->segs = (ora_segment *)malloc(sizeof(ora_segment) * m->cap_segs);
  m->min_bin = freq_to_bin(sample_rate, fft_size, cfg->speech_min_freq);
  m->max_bin = freq_to_bin(sample_rate, fft_size, cfg->speech_max_freq);
}

static void vadm_free(vadm *m) {
  free(m->long_term.data);
  free(m->short_term.data);
  free(m->ratio.data);
  free(m->segs);
}

static uint64_t rec_start(const vadm *m, uint64_t from) {
  const uint64_t sb = (uint64_t)((float)m->sample_rate * 2);
  return (sb > from) ? 0 : from - sb;
}
static uint64_t rec_end(const vadm *m, uint64_t to) { return to + (uint64_t)((float)m->sample_rate * 2); }

static void track(vadm *m, int has_vad, float vad, float ratio, int from, int to) {
  if (from == ST_CLOSED && to == ST_OPENING) {
    m->speech_rnn_vad = has_vad ? vad : 0;
    m->speech_rnn_vad_count = 1;
    m->speech_vol_ratio = ratio;
    m->speech_vol_ratio_count = 1;
  } else if (from == ST_OPENING || from == ST_OPEN) {
    m->speech_rnn_vad += has_vad ? vad : 0;
    m->speech_rnn_vad_count += 1;
    m->speech_vol_ratio += ratio;
    m->speech_vol_ratio_count += 1;
  }
}

static void on_speech_end(vadm *m) {
  const uint64_t from = m->speech_start_index, to = m->speech_end_index;
  const uint64_t len = to - from;
  const float sr = (float)m->sample_rate;
  const float len_rt = (float)len / sr;
  if (len_rt >= m->cfg.min_vad_duration_sec) {
    ora_segment s;
    s.sample_from = rec_start(m, from);
    s.sample_to = rec_end(m, to);
    s.debug_rnn_vad = m->speech_rnn_vad / (float)m->speech_rnn_vad_count;
    s.debug_avg_speech_vol_ratio = m->speech_vol_ratio / (float)m->speech_vol_ratio_count;
    if (m->n_segs == m->cap_segs) {
      m->cap_segs *= 2;
      m->segs = (ora_segment *)realloc(m->segs, sizeof(ora_segment) * m->cap_segs);
    }
    m->segs[m->n_segs++] = s;
  }
}

/* VADMachine.run: bins = [n_channels][n_bins] magnitude spectra of the window */
static void vadm_run(vadm *m, uint64_t index, const float *const *bins, int has_vad, float vad,
                     float vol_ratio, float *band_out) {
  const ora_vadm_config *c = &m->cfg;
  const float sr = (float)m->sample_rate;
  float vols[MAXCH];
  float min_v = 999, max_v = 0;
  int ch;
  size_t i;
  size_t min_open, max_gap;
  double short_term, ratio_avg, threshold_base, threshold;
  int met;
  m->n_runs++;
  for (ch = 0; ch < m->n_channels; ch++) {
    vols[ch] = 0.0f;
    for (i = m->min_bin; i <= m->max_bin; i++) vols[ch] += bins[ch][i];
    if (band_out) band_out[ch] = vols[ch];
  }
  for (ch = 0; ch < m->n_channels; ch++) {
    if (vols[ch] < min_v) min_v = vols[ch];
    if (vols[ch] > max_v) max_v = vols[ch];
  }
  (void)max_v;
  min_open = (size_t)(sr * c->min_consecutive_sec_to_open);
  max_gap = (size_t)(sr * c->max_speech_gap_sec);
  short_term = rolling_push(&m->short_term, min_v);
  ratio_avg = rolling_push(&m->ratio, vol_ratio);
  if (m->long_term.has_last)
    threshold_base = m->long_term.last_avg;
  else if (c->has_initial_long_term_avg)
    threshold_base = c->initial_long_term_avg;
  else
    threshold_base = short_term;
  threshold = threshold_base * (double)c->speech_threshold_factor;
  met = (short_term > threshold) && (ratio_avg > (double)c->channel_vol_ratio_threshold);
  if (!met) rolling_push(&m->long_term, min_v);
  switch (m->state) {
    case ST_CLOSED:
      if (met) {
        m->state = ST_OPENING;
        m->speech_start_index = index;
      }
      track(m, has_vad, vad, vol_ratio, ST_CLOSED, m->state);
      break;
    case ST_OPENING: {
      const uint64_t since = index - m->speech_start_index;
      if (met && since >= min_open)
        m->state = ST_OPEN;
      else if (!met)
        m->state = ST_CLOSED;
      track(m, has_vad, vad, vol_ratio, ST_OPENING, m->state);
      break;
    }
    case ST_OPEN:
      if (!met) {
        m->state = ST_CLOSING;
        m->speech_end_index = index;
      }
      track(m, has_vad, vad, vol_ratio, ST_OPEN, m->state);
      break;
    case ST_CLOSING: {
      const uint64_t since = index - m->speech_end_index;
      if (met)
        m->state = ST_OPEN;
      else if (since >= max_gap) {
        m->state = ST_CLOSED;
        on_speech_end(m);
      }
      track(m, has_vad, vad, vol_ratio, ST_CLOSING, m->state);
      break;
    }
  }
}

/* ---------------- AudioPipeline + VAD ---------------- */
struct ora_pipeline {
  int n_channels, sample_rate, fft_size, use_denoiser;
  size_t capacity;
  float *ring[MAXCH];
  uint64_t total_write_count, read_count;
  ora_denoise *den;
  float *fft_buf[MAXCH];
  size_t fft_write_index;
  uint64_t fft_index;
  float rnn_vad_acc, vol_ratio_acc;
  float *window;
  float *bins[MAXCH];
  vadm main;
  vadm *alts;
  int n_alt;
  /* trace */
  ora_frame_trace *tf;
  size_t tf_cap, tf_n;
  ora_window_trace *tw;
  size_t tw_cap, tw_n;
  float *tden;
  size_t tden_cap, tden_n;
};

ora_pipeline *ora_pipeline_create(int n_channels, int sample_rate, size_t buffer_length, int fft_size,
                                  int use_denoiser, const ora_model *model,
                                  const ora_vadm_config *main_cfg, const ora_vadm_config *alt_cfgs,
                                  int n_alt) {
  ora_pipeline *p;
  int ch, i;
  ora_vadm_config def;
  if (sample_rate != 48000 || n_channels < 1 || n_channels > MAXCH) return NULL; /* VAD.zig:101-104 */
  if (fft_size == 0 || (fft_size % 2) != 0) return NULL;                       /* FFT.zig:29-31 */
  p = (ora_pipeline *)calloc(1, sizeof(ora_pipeline));
  p->n_channels = n_channels;
  p->sample_rate = sample_rate;
  p->fft_size = fft_size;
  p->use_denoiser = use_denoiser;
  p->capacity = buffer_length ? buffer_length : (size_t)sample_rate * 10; /* AudioPipeline.zig:45 */
  for (ch = 0; ch < n_channels; ch++) {
    p->ring[ch] = (float *)calloc(p->capacity, sizeof(float));
    p->fft_buf[ch] = (float *)calloc(fft_size, sizeof(float));
    p->bins[ch] = (float *)calloc(fft_size / 2 + 1, sizeof(float));
  }
  p->den = ora_rnnoise_create(model);
  p->window = (float *)malloc(sizeof(float) * fft_size);
  ora_hann_periodic(p->window, fft_size);
  if (!main_cfg) {
    ora_vadm_config_default(&def);
    main_cfg = &def;
  }
  vadm_init(&p->main, main_cfg, sample_rate, n_channels, fft_size);
  p->n_alt = n_alt;
  if (n_alt > 0) {
    p->alts = (vadm *)calloc(n_alt, sizeof(vadm));
    for (i = 0; i < n_alt; i++) vadm_init(&p->alts[i], &alt_cfgs[i], sample_rate, n_channels, fft_size);
  }
  return p;
}

void ora_pipeline_destroy(ora_pipeline *p) {
  int ch, i;
  if (!p) return;
  for (ch = 0; ch < p->n_channels; ch++) {
    free(p->ring[ch]);
    free(p->fft_buf[ch]);
    free(p->bins[ch]);
  }
  ora_rnnoise_destroy(p->den);
  free(p->window);
  vadm_free(&p->main);
  for (i = 0; i < p->n_alt; i++) vadm_free(&p->alts[i]);
  free(p->alts);
  free(p);
}

void ora_pipeline_enable_trace(ora_pipeline *p, ora_frame_trace *frames, size_t frames_cap,
                               ora_window_trace *windows, size_t windows_cap, float *denoised,
                               size_t den_cap) {
  p->tf = frames;
  p->tf_cap = frames_cap;
  p->tw = windows;
  p->tw_cap = windows_cap;
  p->tden = denoised;
  p->tden_cap = den_cap;
}

void ora_pipeline_trace_counts(const ora_pipeline *p, size_t *nf, size_t *nw) {
  if (nf) *nf = p->tf_n;
  if (nw) *nw = p->tw_n;
}

/* copy [from, to) of channel ch out of the ring (readSlice + SplitSlice iteration) */
static void ring_read(const ora_pipeline *p, int ch, uint64_t from, size_t n, float *dst) {
  size_t i;
  for (i = 0; i < n; i++) dst[i] = p->ring[ch][(from + i) % p->capacity];
}

static void fft_step(ora_pipeline *p, uint64_t index, const float *const *seg, int has_vad, float vad,
                     float vol_ratio) {
  int ch, i;
  float band[MAXCH];
  for (ch = 0; ch < p->n_channels; ch++) ora_fftzig(p->fft_size, seg[ch], p->window, p->bins[ch]);
  vadm_run(&p->main, index, (const float *const *)p->bins, has_vad, vad, vol_ratio, band);
  for (i = 0; i < p->n_alt; i++)
    vadm_run(&p->alts[i], index, (const float *const *)p->bins, has_vad, vad, vol_ratio, NULL);
  if (p->tw && p->tw_n < p->tw_cap) {
    ora_window_trace *t = &p->tw[p->tw_n++];
    memset(t, 0, sizeof(*t));
    t->index = index;
    for (ch = 0; ch < p->n_channels; ch++) t->band[ch] = band[ch];
    t->vol_ratio = vol_ratio;
    t->vad = has_vad ? vad : -1.0f;
  }
}

static void collect_input(ora_pipeline *p) {
  const size_t frame = p->use_denoiser ? 480 : (size_t)p->fft_size;
  float *in[MAXCH], *den[MAXCH];
  float scaled[480], out[480];
  int ch;
  for (ch = 0; ch < p->n_channels; ch++) {
    in[ch] = (float *)malloc(sizeof(float) * frame);
    den[ch] = (float *)malloc(sizeof(float) * frame);
  }
  while (p->total_write_count - p->read_count >= frame) {
    const uint64_t from = p->read_count;
    float vmin = 1, vmax = 0, ratio;
    p->read_count = from + frame;
    for (ch = 0; ch < p->n_channels; ch++) ring_read(p, ch, from, frame, in[ch]);
    /* preAnalyzeSegment (VAD.zig:253-272) */
    for (ch = 0; ch < p->n_channels; ch++) {
      const float v = ora_rms_volume(in[ch], (int)frame);
      if (v < vmin) vmin = v;
      if (v > vmax) vmax = v;
    }
    ratio = (vmax == 0) ? 0 : vmin / vmax;
    if (p->use_denoiser) {
      /* denoiserStep (VAD.zig:274-296): one shared rnnoise state, channels in order */
      const float scalar = (float)32767;        /* maxInt(i16) as f32, Denoiser.zig:72 */
      const float inv = 1.0f / (float)32767;    /* Denoiser.zig:73 */
      float vad_low = 1;
      size_t off = 0;
      int i;
      for (ch = 0; ch < p->n_channels; ch++) {
        float vad;
        for (i = 0; i < 480; i++) scaled[i] = in[ch][i] * scalar;
        vad = ora_rnnoise_process_frame(p->den, out, scaled);
        for (i = 0; i < 480; i++) den[ch][i] = out[i] * inv;
        if (vad < vad_low) vad_low = vad;
      }
      if (p->tf && p->tf_n < p->tf_cap) {
        ora_frame_trace *t = &p->tf[p->tf_n++];
        t->frame_index = from;
        t->vad_low = vad_low;
        t->vol_ratio = ratio;
      }
      if (p->tden && p->tden_n + 480 <= p->tden_cap) {
        for (ch = 0; ch < p->n_channels; ch++)
          memcpy(p->tden + (size_t)ch * p->tden_cap + p->tden_n, den[ch], 480 * sizeof(float));
        p->tden_n += 480;
      }
      /* fftBufferStep (VAD.zig:298-348) */
      for (;;) {
        const size_t cap = (size_t)p->fft_size;
        const size_t rem = cap - p->fft_write_index;
        const size_t left = 480 - off;
        const size_t written = rem < left ? rem : left;
        const float share = (float)written / (float)cap;
        int full;
        for (ch = 0; ch < p->n_channels; ch++)
          memcpy(p->fft_buf[ch] + p->fft_write_index, den[ch] + off, written * sizeof(float));
        p->fft_write_index += written;
        off += written;
        full = p->fft_write_index == cap;
        p->rnn_vad_acc += vad_low * share;
        p->vol_ratio_acc += ratio * share;
        if (full) {
          fft_step(p, p->fft_index, (const float *const *)p->fft_buf, 1, vad_low, p->vol_ratio_acc);
          p->fft_index += cap;
          p->fft_write_index = 0;
          p->rnn_vad_acc = 0;
          p->vol_ratio_acc = 0;
        }
        if (off == 480) break;
      }
    } else {
      fft_step(p, from, (const float *const *)in, 0, 0, ratio);
    }
  }
  for (ch = 0; ch < p->n_channels; ch++) {
    free(in[ch]);
    free(den[ch]);
  }
}

uint64_t ora_pipeline_push(ora_pipeline *p, const float *const *pcm, size_t n) {
  const uint64_t first = p->total_write_count;
  const size_t chunk = p->capacity / 2; /* AudioPipeline.zig:92 */
  size_t read_offset = 0;
  for (;;) {
    /* writeAssumeCapacity */
    const size_t dst = (size_t)(p->total_write_count % p->capacity);
    const size_t to_end = p->capacity - dst;
    const size_t src_rem = n - read_offset;
    const size_t nw = src_rem < chunk ? src_rem : chunk;
    const size_t n1 = to_end < nw ? to_end : nw;
    int ch;
    for (ch = 0; ch < p->n_channels; ch++) {
      memcpy(p->ring[ch] + dst, pcm[ch] + read_offset, n1 * sizeof(float));
      if (nw > n1) memcpy(p->ring[ch], pcm[ch] + read_offset + n1, (nw - n1) * sizeof(float));
    }
    p->total_write_count += nw;
    read_offset += nw;
    collect_input(p);
    if (nw < chunk) break;
  }
  return first;
}

size_t ora_pipeline_segments(const ora_pipeline *p, int alt_idx, ora_segment *out, size_t cap) {
  const vadm *m = (alt_idx < 0) ? &p->main : &p->alts[alt_idx];
  size_t i;
  for (i = 0; i < m->n_segs && i < cap; i++) out[i] = m->segs[i];
  return m->n_segs;
}

const ora_denoise *ora_pipeline_denoiser(const ora_pipeline *p) { return p->use_denoiser ? p->den : NULL; }

/* the whole machine state (VADMachine.zig:65-125, RollingAverage.zig:5-14) for
 * the checker's comparison with the device machine; alt_idx < 0: the main one */
static const vadm *machine_of(const ora_pipeline *p, int alt_idx) {
  return (alt_idx < 0) ? &p->main : &p->alts[alt_idx];
}

void ora_pipeline_vadm_snapshot(const ora_pipeline *p, int alt_idx, ora_vadm_snapshot *out) {
  const vadm *m = machine_of(p, alt_idx);
  const rolling *r[3] = {&m->long_term, &m->short_term, &m->ratio};
  int k;
  memset(out, 0, sizeof(*out));
  out->speech_state = m->state;
  out->speech_start = m->speech_start_index;
  out->speech_end = m->speech_end_index;
  out->windows = m->n_runs;
  for (k = 0; k < 3; k++) {
    out->avg[k] = r[k]->last_avg;
    out->write_idx[k] = r[k]->write_idx;
    out->written[k] = r[k]->written_count;
  }
  out->speech_rnn_vad = m->speech_rnn_vad;
  out->speech_vol_ratio = m->speech_vol_ratio;
  out->speech_rnn_vad_count = m->speech_rnn_vad_count;
  out->speech_vol_ratio_count = m->speech_vol_ratio_count;
  out->n_segments = m->n_segs;
}

size_t ora_pipeline_vadm_rolling(const ora_pipeline *p, int alt_idx, int which, double *out, size_t cap) {
  const vadm *m = machine_of(p, alt_idx);
  const rolling *r = which == 0 ? &m->long_term : which == 1 ? &m->short_term : &m->ratio;
  size_t i;
  for (i = 0; i < r->len && i < cap; i++) out[i] = r->data[i];
  return r->len;
}
