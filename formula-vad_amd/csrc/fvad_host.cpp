// Host mirror of the reference's pipeline-side API, above the C ABI:
//   RollingAverage            (structures/RollingAverage.zig:1-56)
//   VADMachine                (AudioPipeline/VADMachine.zig:18-310)
//   AudioPipeline.pushSamples (AudioPipeline.zig:86-120) + VAD frame dispatch
//                             (VAD.zig:214-251) on a 1-stream engine
//   multi-stream simulator core (replaces simulator.zig:217-228's thread per
//                             instance with a lock-step tick loop per GPU)
//   Evaluator / statistics / formats (Evaluator.zig:90-156,
//                             Evaluator/statistics.zig:85-284, formats.zig:7-36)
// The per-frame DSP runs on the GPU (fvad_engine_*); what stays here is the
// per-window decision logic (cheap: 23.4 windows/s/stream) and the judge.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fvad.h"
#include "fvad_internal.h"

namespace {

constexpr int kPipelineSegCap = 1 << 16;  // device segment slots per machine (one stream)
constexpr int kMultiSegCap = 1024;        // per stream and machine in the multi-stream core

// ---------------- RollingAverage ----------------
struct RollingAverage {
  std::vector<double> data;
  bool has_last = false;
  double last_avg = 0;
  size_t write_idx = 0, written_count = 0;
  RollingAverage(size_t count, bool has_init, double init) : data(count, 0.0) {
    if (has_init) {
      for (size_t i = 0; i < count; i++) data[i] = init;
      written_count = count;
      avg();
    }
  }
  double avg() {
    double a = 0.0;
    const double scalar = 1.0 / (double)written_count;
    for (size_t i = 0; i < written_count; i++) a += data[i] * scalar;
    last_avg = a;
    has_last = true;
    return a;
  }
  double push(float sample) {
    data[write_idx] = (double)sample;
    write_idx = (write_idx + 1) % data.size();
    if (written_count < data.size()) written_count++;
    return avg();
  }
};

size_t freq_to_bin(int sample_rate, int nfft, float freq) {
  const float bin_width = (float)sample_rate / (float)nfft;
  return (size_t)std::round(freq / bin_width);  // Zig @round: half away from zero
}

// ---------------- VADMachine ----------------
struct VADMachine {
  enum State { kClosed, kOpening, kOpen, kClosing };
  fvad_vadm_config cfg;
  int sample_rate, fft_size;
  State state = kClosed;
  RollingAverage long_term, short_term, ratio;
  uint64_t speech_start = 0, speech_end = 0;
  float rnn_vad = 0;
  size_t rnn_vad_count = 0;
  float vol_ratio = 0;
  size_t vol_ratio_count = 0;
  std::vector<fvad_segment> segments;
  int band_slot = 0;  // which engine band this machine reads
  size_t min_bin, max_bin;

  static size_t len_of(float eval_per_sec, float sec) { return (size_t)(eval_per_sec * sec); }
  VADMachine(const fvad_vadm_config &c, int sr, int fft)
      : cfg(c),
        sample_rate(sr),
        fft_size(fft),
        long_term(std::max<size_t>(1, len_of((float)sr / (float)fft, c.long_term_speech_avg_sec)),
                  c.has_initial_long_term_avg != 0, c.initial_long_term_avg),
        short_term(std::max<size_t>(1, len_of((float)sr / (float)fft, c.short_term_speech_avg_sec)), false, 0),
        ratio(std::max<size_t>(1, len_of((float)sr / (float)fft, c.channel_vol_ratio_avg_sec)), false, 0) {
    segments.reserve(100);
    min_bin = freq_to_bin(sr, fft, c.speech_min_freq);
    max_bin = freq_to_bin(sr, fft, c.speech_max_freq);
  }
  uint64_t rec_start(uint64_t from) const {
    const uint64_t sb = (uint64_t)((float)sample_rate * 2);
    return sb > from ? 0 : from - sb;
  }
  uint64_t rec_end(uint64_t to) const { return to + (uint64_t)((float)sample_rate * 2); }
  void track(float vad, float vr, State from, State to) {
    if (from == kClosed && to == kOpening) {
      rnn_vad = vad;
      rnn_vad_count = 1;
      vol_ratio = vr;
      vol_ratio_count = 1;
    } else if (from == kOpening || from == kOpen) {
      rnn_vad += vad;
      rnn_vad_count += 1;
      vol_ratio += vr;
      vol_ratio_count += 1;
    }
  }
  void on_speech_end() {
    const uint64_t len = speech_end - speech_start;
    const float len_rt = (float)len / (float)sample_rate;
    if (len_rt >= cfg.min_vad_duration_sec) {
      fvad_segment s;
      s.sample_from = rec_start(speech_start);
      s.sample_to = rec_end(speech_end);
      s.debug_rnn_vad = rnn_vad / (float)rnn_vad_count;
      s.debug_avg_speech_vol_ratio = vol_ratio / (float)vol_ratio_count;
      segments.push_back(s);
    }
  }
  // VADMachine.run: channel band sums of this window, window vad (has_vad) and ratio
  void run(uint64_t index, const float *band_per_channel, int n_ch, int band_stride, float vad, float vr) {
    float min_v = 999, max_v = 0;
    for (int c = 0; c < n_ch; c++) {
      const float v = band_per_channel[c * band_stride];
      if (v < min_v) min_v = v;
      if (v > max_v) max_v = v;
    }
    const float sr = (float)sample_rate;
    const size_t min_open = (size_t)(sr * cfg.min_consecutive_sec_to_open);
    const size_t max_gap = (size_t)(sr * cfg.max_speech_gap_sec);
    const double st_avg = short_term.push(min_v);
    const double r_avg = ratio.push(vr);
    double base;
    if (long_term.has_last)
      base = long_term.last_avg;
    else if (cfg.has_initial_long_term_avg)
      base = cfg.initial_long_term_avg;
    else
      base = st_avg;
    const double threshold = base * (double)cfg.speech_threshold_factor;
    const bool met = st_avg > threshold && r_avg > (double)cfg.channel_vol_ratio_threshold;
    if (!met) long_term.push(min_v);
    switch (state) {
      case kClosed:
        if (met) {
          state = kOpening;
          speech_start = index;
        }
        track(vad, vr, kClosed, state);
        break;
      case kOpening:
        if (met && index - speech_start >= min_open)
          state = kOpen;
        else if (!met)
          state = kClosed;
        track(vad, vr, kOpening, state);
        break;
      case kOpen:
        if (!met) {
          state = kClosing;
          speech_end = index;
        }
        track(vad, vr, kOpen, state);
        break;
      case kClosing:
        if (met)
          state = kOpen;
        else if (index - speech_end >= max_gap) {
          state = kClosed;
          on_speech_end();
        }
        track(vad, vr, kClosing, state);
        break;
    }
  }
};

// Engine band slots for a set of machine configs (unique bin ranges).
int assign_bands(std::vector<VADMachine> &ms, fvad_engine_config &ec) {
  ec.n_bands = 0;
  for (auto &m : ms) {
    int slot = -1;
    for (int b = 0; b < ec.n_bands; b++)
      if (ec.band_lo[b] == (int)m.min_bin && ec.band_hi[b] == (int)m.max_bin) slot = b;
    if (slot < 0) {
      if (ec.n_bands == FVAD_MAX_BANDS) return FVAD_EINVAL;
      slot = ec.n_bands++;
      ec.band_lo[slot] = (int)m.min_bin;
      ec.band_hi[slot] = (int)m.max_bin;
    }
    m.band_slot = slot;
  }
  return FVAD_OK;
}

}  // namespace

extern "C" void fvad_vadm_config_default(fvad_vadm_config *c) {
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

// ---------------------------------------------------------------------------
// Standalone VADMachine (host decision logic; testable without a GPU)
// ---------------------------------------------------------------------------
struct fvad_vadm {
  VADMachine m;
  int n_channels;
  fvad_vadm(const fvad_vadm_config &c, int sr, int fft, int ch) : m(c, sr, fft), n_channels(ch) {}
};

extern "C" int fvad_vadm_create(const fvad_vadm_config *cfg, int sample_rate, int fft_size, int n_channels,
                                fvad_vadm **out) {
  if (!out || n_channels < 1 || fft_size <= 0 || sample_rate <= 0) return FVAD_EINVAL;
  fvad_vadm_config def;
  fvad_vadm_config_default(&def);
  *out = new fvad_vadm(cfg ? *cfg : def, sample_rate, fft_size, n_channels);
  return FVAD_OK;
}

extern "C" void fvad_vadm_destroy(fvad_vadm *v) { delete v; }

extern "C" void fvad_vadm_bins(const fvad_vadm *v, int *lo, int *hi) {
  if (lo) *lo = (int)v->m.min_bin;
  if (hi) *hi = (int)v->m.max_bin;
}

extern "C" int fvad_vadm_run(fvad_vadm *v, uint64_t index, const float *band_per_channel, float vad,
                             float vol_ratio) {
  if (!v || !band_per_channel) return FVAD_EINVAL;
  v->m.run(index, band_per_channel, v->n_channels, 1, vad, vol_ratio);
  return FVAD_OK;
}

extern "C" size_t fvad_vadm_segments(const fvad_vadm *v, fvad_segment *out, size_t cap) {
  const auto &segs = v->m.segments;
  for (size_t i = 0; i < segs.size() && i < cap; i++) out[i] = segs[i];
  return segs.size();
}

namespace {
struct StreamMachines {
  std::vector<VADMachine> machines;  // [0] = main; they run on the device (k_vadm_hbm)
};
}  // namespace

// ---------------------------------------------------------------------------
// AudioPipeline (single stream)
// ---------------------------------------------------------------------------
struct fvad_pipeline {
  int n_channels;
  fvad_engine *engine = nullptr;
  fvad_engine_config ec;
  StreamMachines sm;
  std::vector<std::vector<float>> pending;  // samples not yet forming a full 480 frame
  uint64_t total_write_count = 0;
  std::vector<float> pcm;
  // Recorder: raw input history [hist0, total_write_count) per channel, kept
  // from the earliest sample a capture that may still complete can start at
  std::vector<std::vector<float>> hist;
  uint64_t hist0 = 0;
  fvad_recording_fn rec_fn = nullptr;
  void *rec_ctx = nullptr;
  size_t rec_done = 0;  // main-machine segments already handed to rec_fn
};

namespace {
// AudioPipeline's ring holds 10 s (AudioPipeline.zig:45); a capture starts
// 2 s before its speech start (VADMachine.getOffsetRecordingStart), and a
// closed machine's next speech start lies within the last window's latency
constexpr uint64_t kRecKeep = 48000 * 10;
constexpr uint64_t kRecMargin = 48000 * 2;
}  // namespace

extern "C" int fvad_recording_channel(const float *const *pcm, int n_channels, size_t n) {
  if (!pcm || n_channels < 1) return FVAD_EINVAL;
  int best = 0;
  float best_vol = 9999;
  for (int c = 0; c < n_channels; c++) {
    float sum = 0.0f;
    for (size_t i = 0; i < n; i++) sum += pcm[c][i] * pcm[c][i];
    const float mean = sum / (float)n;
    const float vol = std::sqrt(mean);
    if (vol < best_vol) {
      best = c;
      best_vol = vol;
    }
  }
  return best;
}

extern "C" void fvad_vad_config_default(fvad_vad_config *c) {
  std::memset(c, 0, sizeof(*c));
  c->fft_size = 2048;
  c->use_denoiser = 1;
  fvad_vadm_config_default(&c->vad_machine_config);
}

extern "C" int fvad_pipeline_create_ex(int sample_rate, int n_channels, const fvad_model *model, int device,
                                       const fvad_vad_config *vc, fvad_pipeline **out) {
  if (!model || !out || !vc || n_channels < 1 || n_channels > FVAD_MAX_CHANNELS || vc->n_alt < 0 ||
      (vc->n_alt > 0 && !vc->alt_vad_machine_configs))
    return FVAD_EINVAL;
  if (sample_rate != 48000) return FVAD_ERATE;
  fvad_pipeline *p = new fvad_pipeline();
  p->n_channels = n_channels;
  p->sm.machines.emplace_back(vc->vad_machine_config, sample_rate, vc->fft_size);
  for (int i = 0; i < vc->n_alt; i++) p->sm.machines.emplace_back(vc->alt_vad_machine_configs[i], sample_rate, vc->fft_size);
  fvad_engine_config_default(&p->ec, 1, n_channels);
  p->ec.device = device;
  p->ec.max_ticks = 100;
  p->ec.fft_size = vc->fft_size;
  p->ec.use_denoiser = vc->use_denoiser;
  int rc = assign_bands(p->sm.machines, p->ec);
  if (!rc) rc = fvad_engine_create(&p->ec, model, &p->engine);
  if (!rc) {
    // the machines run on the device after every push (k_vadm_hbm)
    std::vector<fvad_vadm_config> cfgs;
    for (auto &m : p->sm.machines) cfgs.push_back(m.cfg);
    rc = fvad_engine_attach_vadm(p->engine, cfgs.data(), (int)cfgs.size(), kPipelineSegCap);
  }
  if (rc) {
    if (p->engine) fvad_engine_destroy(p->engine);
    delete p;
    return rc;
  }
  p->pending.assign(n_channels, {});
  p->pcm.resize((size_t)p->ec.max_ticks * n_channels * fvad::kFrame);
  *out = p;
  return FVAD_OK;
}

extern "C" int fvad_pipeline_create(int sample_rate, int n_channels, const fvad_model *model, int device,
                                    const fvad_vadm_config *main_cfg, const fvad_vadm_config *alt_cfgs, int n_alt,
                                    fvad_pipeline **out) {
  fvad_vad_config vc;
  fvad_vad_config_default(&vc);
  if (main_cfg) vc.vad_machine_config = *main_cfg;
  vc.alt_vad_machine_configs = alt_cfgs;
  vc.n_alt = n_alt;
  return fvad_pipeline_create_ex(sample_rate, n_channels, model, device, &vc, out);
}

extern "C" void fvad_pipeline_destroy(fvad_pipeline *p) {
  if (!p) return;
  fvad_engine_destroy(p->engine);
  delete p;
}

namespace {
// Recordings of the main machine's newly completed segments, then trim the
// history (AudioPipeline.maybeRecordBuffer / Recorder.finalize, keep = true)
int record_segments(fvad_pipeline *p) {
  const int C = p->n_channels;
  const size_t total = fvad_engine_segments_range(p->engine, 0, 0, p->rec_done, nullptr, 0);
  if (total > p->rec_done) {
    std::vector<fvad_segment> segs(total - p->rec_done);
    const size_t k = std::min(segs.size(), (size_t)kPipelineSegCap > p->rec_done ? (size_t)kPipelineSegCap - p->rec_done : 0);
    fvad_engine_segments_range(p->engine, 0, 0, p->rec_done, segs.data(), k);
    std::vector<const float *> ch(C);
    for (size_t i = 0; i < k; i++) {
      const uint64_t from = segs[i].sample_from, to = segs[i].sample_to;
      if (from < p->hist0 || to > p->hist0 + p->hist[0].size() || to <= from) continue;  // not retained
      for (int c = 0; c < C; c++) ch[c] = p->hist[c].data() + (from - p->hist0);
      const size_t len = (size_t)(to - from);
      const int best = fvad_recording_channel(ch.data(), C, len);
      p->rec_fn(p->rec_ctx, ch[best], len, from, best);
    }
    p->rec_done = total;
  }
  int state = 0;
  uint64_t speech_start = 0;
  int rc = fvad_engine_vadm_state(p->engine, 0, 0, &state, &speech_start, nullptr);
  if (rc) return rc;
  uint64_t keep_from = p->total_write_count > kRecKeep ? p->total_write_count - kRecKeep : 0;
  if (state != 0) keep_from = std::min(keep_from, speech_start > kRecMargin ? speech_start - kRecMargin : 0);
  if (keep_from > p->hist0) {
    const size_t drop = (size_t)std::min<uint64_t>(keep_from - p->hist0, p->hist[0].size());
    for (int c = 0; c < C; c++) p->hist[c].erase(p->hist[c].begin(), p->hist[c].begin() + drop);
    p->hist0 += drop;
  }
  return FVAD_OK;
}
}  // namespace

extern "C" int fvad_pipeline_set_recorder(fvad_pipeline *p, fvad_recording_fn fn, void *ctx) {
  if (!p) return FVAD_EINVAL;
  p->rec_fn = fn;
  p->rec_ctx = ctx;
  p->hist.assign(p->n_channels, {});
  p->hist0 = p->total_write_count;
  p->rec_done = fn ? fvad_engine_segments_range(p->engine, 0, 0, 0, nullptr, 0) : 0;
  return FVAD_OK;
}

extern "C" int fvad_pipeline_push(fvad_pipeline *p, const float *const *pcm, size_t n, uint64_t *first_index) {
  if (!p || (!pcm && n)) return FVAD_EINVAL;
  if (first_index) *first_index = p->total_write_count;
  const int C = p->n_channels;
  for (int c = 0; c < C; c++) p->pending[c].insert(p->pending[c].end(), pcm[c], pcm[c] + n);
  if (p->rec_fn)
    for (int c = 0; c < C; c++) p->hist[c].insert(p->hist[c].end(), pcm[c], pcm[c] + n);
  p->total_write_count += n;
  // with the denoiser the VAD loop takes whole 480-sample frames and keeps
  // the rest for the next push (VAD.zig:219-220); without it every sample
  // goes in at once (the engine counts samples and completes each fft_size
  // window as soon as its last sample is in, VAD.zig:206-212), the last tick
  // partial
  const size_t have = p->pending[0].size();
  const bool nd = !p->ec.use_denoiser;
  size_t left = nd ? have : have / fvad::kFrame * fvad::kFrame;
  size_t consumed = 0;
  while (left > 0) {
    const size_t take = std::min<size_t>(left, (size_t)p->ec.max_ticks * fvad::kFrame);
    const int nt = (int)((take + fvad::kFrame - 1) / fvad::kFrame);
    const int32_t last = (int32_t)(take - (size_t)(nt - 1) * fvad::kFrame);
    for (int t = 0; t < nt; t++)
      for (int c = 0; c < C; c++) {
        const size_t k = t + 1 < nt ? fvad::kFrame : (size_t)last;
        float *dst = &p->pcm[((size_t)t * C + c) * fvad::kFrame];
        std::memcpy(dst, &p->pending[c][consumed + (size_t)t * fvad::kFrame], k * sizeof(float));
        if (k < (size_t)fvad::kFrame) std::memset(dst + k, 0, (fvad::kFrame - k) * sizeof(float));
      }
    int rc = last == fvad::kFrame ? fvad_engine_push(p->engine, p->pcm.data(), nt, nullptr, nullptr)
                                  : fvad_engine_push_ex(p->engine, p->pcm.data(), nt, nullptr, &last, nullptr);
    if (rc) return rc;
    consumed += take;
    left -= take;
  }
  for (int c = 0; c < C; c++) p->pending[c].erase(p->pending[c].begin(), p->pending[c].begin() + consumed);
  return p->rec_fn ? record_segments(p) : FVAD_OK;
}

extern "C" size_t fvad_pipeline_segments(const fvad_pipeline *p, int alt, fvad_segment *out, size_t cap) {
  const size_t idx = alt < 0 ? 0 : (size_t)alt + 1;
  if (!p || idx >= p->sm.machines.size()) return 0;
  return fvad_engine_segments(p->engine, 0, (int)idx, out, cap);
}

// ---------------------------------------------------------------------------
// Multi-stream simulator core (simulator.zig:217-228 runs a thread per
// instance): streams grouped by channel count, each group partitioned
// contiguously over the devices; one engine and one host thread per (group,
// device) part, lock-step pushes, no collectives.  Input is pulled from a
// reader per push (the simulator's 48 000-frame read loop,
// SimulationInstance.zig:171-203) straight into the engine's pinned slot,
// with FVAD_MAX_IN_FLIGHT pushes in flight.
// ---------------------------------------------------------------------------
struct fvad_multi {
  int n_streams, ticks_per_push, n_machines;
  std::vector<int> channels;  // [stream]
  struct Part {
    int device, n_channels;
    std::vector<int> streams;  // global stream ids, in order
    fvad_engine *engine = nullptr;
    fvad_engine_config ec;
  };
  std::vector<Part> parts;
  std::vector<std::pair<int, int>> where;  // stream -> (part, index in part)
};

extern "C" int fvad_multi_create_ex(int n_streams, const int *n_channels, const fvad_model *model, const int *devices,
                                    int n_devices, const fvad_vad_config *vc, int ticks_per_push, fvad_multi **out) {
  if (!model || !out || !vc || n_streams < 1 || n_devices < 1 || !devices || !n_channels || ticks_per_push < 1 ||
      vc->n_alt < 0 || (vc->n_alt > 0 && !vc->alt_vad_machine_configs))
    return FVAD_EINVAL;
  for (int s = 0; s < n_streams; s++)
    if (n_channels[s] < 1 || n_channels[s] > FVAD_MAX_CHANNELS) return FVAD_EINVAL;
  fvad_multi *m = new fvad_multi();
  m->n_streams = n_streams;
  m->ticks_per_push = ticks_per_push;
  m->n_machines = 1 + vc->n_alt;
  m->channels.assign(n_channels, n_channels + n_streams);
  m->where.assign(n_streams, {-1, -1});
  std::vector<VADMachine> ms;
  ms.emplace_back(vc->vad_machine_config, 48000, vc->fft_size);
  for (int i = 0; i < vc->n_alt; i++) ms.emplace_back(vc->alt_vad_machine_configs[i], 48000, vc->fft_size);
  std::vector<fvad_vadm_config> cfgs;
  for (auto &x : ms) cfgs.push_back(x.cfg);
  std::vector<int> groups(m->channels);
  std::sort(groups.begin(), groups.end());
  groups.erase(std::unique(groups.begin(), groups.end()), groups.end());
  for (int C : groups) {
    std::vector<int> ids;
    for (int s = 0; s < n_streams; s++)
      if (m->channels[s] == C) ids.push_back(s);
    const int nd = std::min<int>(n_devices, (int)ids.size());
    for (int d = 0; d < nd; d++) {
      fvad_multi::Part p;
      p.device = devices[d];
      p.n_channels = C;
      const size_t i0 = ids.size() * d / nd, i1 = ids.size() * (d + 1) / nd;
      p.streams.assign(ids.begin() + i0, ids.begin() + i1);
      fvad_engine_config_default(&p.ec, (int)p.streams.size(), C);
      p.ec.device = p.device;
      p.ec.max_ticks = ticks_per_push;
      p.ec.fft_size = vc->fft_size;
      p.ec.use_denoiser = vc->use_denoiser;
      int rc = assign_bands(ms, p.ec);
      if (!rc) rc = fvad_engine_create(&p.ec, model, &p.engine);
      if (!rc) rc = fvad_engine_attach_vadm(p.engine, cfgs.data(), (int)cfgs.size(), kMultiSegCap);
      if (rc) {
        if (p.engine) fvad_engine_destroy(p.engine);
        fvad_multi_destroy(m);
        return rc;
      }
      for (size_t k = 0; k < p.streams.size(); k++) m->where[p.streams[k]] = {(int)m->parts.size(), (int)k};
      m->parts.push_back(std::move(p));
    }
  }
  *out = m;
  return FVAD_OK;
}

extern "C" int fvad_multi_create(int n_streams, int n_channels, const fvad_model *model, const int *devices,
                                 int n_devices, const fvad_vadm_config *cfg, int ticks_per_push, fvad_multi **out) {
  if (n_streams < 1) return FVAD_EINVAL;
  fvad_vad_config vc;
  fvad_vad_config_default(&vc);
  if (cfg) vc.vad_machine_config = *cfg;
  std::vector<int> ch(n_streams, n_channels);
  return fvad_multi_create_ex(n_streams, ch.data(), model, devices, n_devices, &vc, ticks_per_push, out);
}

extern "C" void fvad_multi_destroy(fvad_multi *m) {
  if (!m) return;
  for (auto &p : m->parts) fvad_engine_destroy(p.engine);
  delete m;
}

extern "C" int fvad_multi_run_stream(fvad_multi *m, fvad_read_fn read, void *ctx) {
  if (!m || !read) return FVAD_EINVAL;
  std::vector<int> rcs(m->parts.size(), FVAD_OK);
  std::vector<std::thread> th;
  for (size_t pi = 0; pi < m->parts.size(); pi++) {
    th.emplace_back([&, pi]() {
      fvad_multi::Part &p = m->parts[pi];
      const int B = (int)p.streams.size(), T = p.ec.max_ticks, C = p.n_channels;
      const size_t cap = (size_t)T * fvad::kFrame;
      std::vector<float> tmp((size_t)C * cap);
      std::vector<float *> dst(C);
      for (int c = 0; c < C; c++) dst[c] = tmp.data() + (size_t)c * cap;
      std::vector<int32_t> valid(B), last(B);
      std::vector<char> done(B, 0);
      // no denoiser: a stream's final partial tick goes in too (its samples
      // can complete an fft_size window, VAD.zig:206-220); with the denoiser a
      // tail shorter than a frame is never processed (VAD.zig:219)
      const bool nd = !p.ec.use_denoiser;
      int in_flight = 0, rc = FVAD_OK, live = B;
      while (live > 0 && !rc) {
        float *buf = fvad_engine_input_slot(p.engine);
        if (!buf) {
          rc = FVAD_EDEVICE;
          break;
        }
        int nt = 0;
        bool partial = false;
        for (int b = 0; b < B; b++) {
          valid[b] = 0;
          last[b] = fvad::kFrame;
          if (done[b]) continue;
          size_t got = 0;
          while (got < cap) {
            std::vector<float *> d(C);
            for (int c = 0; c < C; c++) d[c] = dst[c] + got;
            const size_t r = read(ctx, p.streams[b], d.data(), cap - got);
            if (r == 0) break;
            got += r;
          }
          if (got < cap) {
            done[b] = 1;
            live--;
          }
          valid[b] = (int)(got / fvad::kFrame);
          if (nd && got % fvad::kFrame) {
            last[b] = (int32_t)(got % fvad::kFrame);
            valid[b]++;
            partial = true;
          }
          nt = std::max(nt, valid[b]);
          for (int t = 0; t < valid[b]; t++)
            for (int c = 0; c < C; c++) {
              const size_t k = t + 1 < valid[b] ? fvad::kFrame : (size_t)last[b];
              float *d = &buf[(((size_t)t * B + b) * C + c) * fvad::kFrame];
              std::memcpy(d, dst[c] + (size_t)t * fvad::kFrame, k * sizeof(float));
              if (k < (size_t)fvad::kFrame) std::memset(d + k, 0, (fvad::kFrame - k) * sizeof(float));
            }
        }
        if (nt == 0) break;
        if (in_flight == FVAD_MAX_IN_FLIGHT && !(rc = fvad_engine_collect(p.engine, nullptr, nullptr))) in_flight--;
        if (!rc && !(rc = fvad_engine_submit_ex(p.engine, buf, nt, valid.data(), partial ? last.data() : nullptr)))
          in_flight++;
      }
      while (in_flight > 0) {
        const int r2 = fvad_engine_collect(p.engine, nullptr, nullptr);
        if (!rc) rc = r2;
        in_flight--;
      }
      rcs[pi] = rc;
    });
  }
  for (auto &t : th) t.join();
  for (int rc : rcs)
    if (rc) return rc;
  return FVAD_OK;
}

namespace {
struct MemReader {
  const float *const *pcm;
  const size_t *len;
  const std::vector<int> *channels;
  std::vector<size_t> pos;
};
size_t mem_read(void *ctx, int s, float *const *dst, size_t max_frames) {
  MemReader *r = static_cast<MemReader *>(ctx);
  const size_t n = std::min(max_frames, r->len[s] - r->pos[s]);
  for (int c = 0; c < (*r->channels)[s]; c++)
    std::memcpy(dst[c], r->pcm[s] + (size_t)c * r->len[s] + r->pos[s], n * sizeof(float));
  r->pos[s] += n;
  return n;
}
}  // namespace

extern "C" int fvad_multi_run(fvad_multi *m, const float *const *pcm, const size_t *len) {
  if (!m || !pcm || !len) return FVAD_EINVAL;
  MemReader r{pcm, len, &m->channels, std::vector<size_t>(m->n_streams, 0)};
  return fvad_multi_run_stream(m, mem_read, &r);
}

extern "C" size_t fvad_multi_segments_alt(const fvad_multi *m, int stream, int machine, fvad_segment *out,
                                          size_t cap) {
  if (!m || stream < 0 || stream >= m->n_streams || machine < 0 || machine >= m->n_machines) return 0;
  const auto &w = m->where[stream];
  return fvad_engine_segments(m->parts[w.first].engine, w.second, machine, out, cap);
}

extern "C" size_t fvad_multi_segments(const fvad_multi *m, int stream, fvad_segment *out, size_t cap) {
  return fvad_multi_segments_alt(m, stream, 0, out, cap);
}

// ---------------------------------------------------------------------------
// Evaluator / statistics / formats
// ---------------------------------------------------------------------------
namespace {
struct Seg {
  float from, to;
  std::vector<size_t> opp;
};
float overlap_with(float af, float at, float bf, float bt) {
  const float max_from = af > bf ? af : bf;
  const float min_to = at < bt ? at : bt;
  return min_to - max_from;
}
void sort_by_start(std::vector<Seg> &v) {
  std::stable_sort(v.begin(), v.end(), [](const Seg &a, const Seg &b) { return a.from < b.from; });
}
float false_positive(const Seg &v, const std::vector<Seg> &refs, const fvad_stat_config &c) {
  // extrudeSegments (statistics.zig:191-218) + calcOverlapMany
  const size_t n = v.opp.size();
  std::vector<float> f(n), t(n);
  for (size_t i = 0; i < n; i++) {
    f[i] = refs[v.opp[i]].from;
    t[i] = refs[v.opp[i]].to;
  }
  if (n > 0) {
    f[0] -= c.extrude_start;
    t[n - 1] += c.extrude_end;
    for (size_t i = 0; i + 1 < n; i++)
      if (f[i + 1] - t[i] <= c.fill_gaps) t[i] = f[i + 1];
  }
  float ov = 0.0f;
  for (size_t i = 0; i < n; i++) {
    const float o = overlap_with(v.from, v.to, f[i], t[i]);
    ov += 0.0f > o ? 0.0f : o;
  }
  return (v.to - v.from) - ov;
}
float f_score(float beta, float p, float r) {
  const float b2 = beta * beta;  // std.math.pow(f32, beta, 2)
  return (1 + b2) * (p * r) / (b2 * p + r);
}
}  // namespace

extern "C" int fvad_eval_stats(const float *vad, size_t nv, const float *ref, size_t nr, const fvad_stat_config *cfg,
                               fvad_single_stats *out) {
  if ((!vad && nv) || (!ref && nr) || !cfg || !out) return FVAD_EINVAL;
  std::vector<Seg> vs(nv), rs(nr);
  for (size_t i = 0; i < nv; i++) vs[i] = {vad[2 * i], vad[2 * i + 1], {}};
  for (size_t i = 0; i < nr; i++) rs[i] = {ref[2 * i], ref[2 * i + 1], {}};
  sort_by_start(vs);
  sort_by_start(rs);
  for (auto &v : vs)
    for (size_t j = 0; j < rs.size(); j++)
      if (overlap_with(v.from, v.to, rs[j].from, rs[j].to) > 0.0f) v.opp.push_back(j);
  for (auto &r : rs)
    for (size_t j = 0; j < vs.size(); j++)
      if (overlap_with(r.from, r.to, vs[j].from, vs[j].to) > 0.0f) r.opp.push_back(j);
  fvad_single_stats s;
  std::memset(&s, 0, sizeof(s));
  for (const auto &v : vs) {
    s.false_positives_sec += false_positive(v, rs, *cfg);
    const float tp = (v.to - v.from) - false_positive(v, rs, *cfg);
    s.true_positives_sec += tp;
    s.total_positives_sec += tp;
  }
  for (const auto &r : rs) {
    if ((r.to - r.from) < cfg->ignore_shorter_than_sec) continue;
    float ov = 0.0f;
    for (size_t j : r.opp) {
      const float o = overlap_with(r.from, r.to, vs[j].from, vs[j].to);
      ov += 0.0f > o ? 0.0f : o;
    }
    const float fn = (r.to - r.from) - ov;
    s.false_negatives_sec += fn;
    s.total_positives_sec += fn;
  }
  s.true_positive_rate = s.true_positives_sec / s.total_positives_sec;
  s.false_negative_rate = s.false_negatives_sec / s.total_positives_sec;
  s.false_discovery_rate = s.false_positives_sec / (s.false_positives_sec + s.true_positives_sec);
  s.precision = s.true_positives_sec / (s.true_positives_sec + s.false_positives_sec);
  s.f_score_beta = 0.7f;
  s.f_score = f_score(s.f_score_beta, s.precision, s.true_positive_rate);
  s.fm_index = std::sqrt(s.precision * s.true_positive_rate);
  *out = s;
  return FVAD_OK;
}

extern "C" void fvad_eval_aggregate(const fvad_single_stats *st, size_t n, fvad_aggregate_stats *a) {
  std::memset(a, 0, sizeof(*a));
  fvad_agg_stat *aggs[4] = {&a->true_positive_rate, &a->false_negative_rate, &a->false_discovery_rate, &a->precision};
  for (auto *x : aggs) {
    x->min = 2;
    x->max = -2;
  }
  float sums[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < n; i++) {
    const fvad_single_stats &s = st[i];
    a->total_positives_sec += s.total_positives_sec;
    a->true_positives_sec += s.true_positives_sec;
    a->false_positives_sec += s.false_positives_sec;
    a->false_negatives_sec += s.false_negatives_sec;
    const float vals[4] = {s.true_positive_rate, s.false_negative_rate, s.false_discovery_rate, s.precision};
    for (int k = 0; k < 4; k++) {
      sums[k] += vals[k];
      if (vals[k] < aggs[k]->min) aggs[k]->min = vals[k];
      if (vals[k] > aggs[k]->max) aggs[k]->max = vals[k];
    }
  }
  const float nf = (float)n;
  a->true_positive_rate.overall = a->true_positives_sec / a->total_positives_sec;
  a->false_negative_rate.overall = a->false_negatives_sec / a->total_positives_sec;
  a->false_discovery_rate.overall = a->false_positives_sec / (a->false_positives_sec + a->true_positives_sec);
  a->precision.overall = a->true_positives_sec / (a->true_positives_sec + a->false_positives_sec);
  for (int k = 0; k < 4; k++) aggs[k]->avg = sums[k] / nf;
  a->f_score_beta = 0.7f;
  a->f_score = f_score(a->f_score_beta, a->precision.overall, a->true_positive_rate.overall);
  a->fm_index = std::sqrt(a->precision.overall * a->true_positive_rate.overall);
}

extern "C" long fvad_parse_audacity(const char *txt, size_t len, float *out, size_t cap) {
  // formats.parseAudacitySegments: split the raw text on '\n' (CRs are NOT
  // stripped, formats.zig:11-14), each line on '\t'; lines with < 2 fields are
  // skipped, an unparsable from/to field is an error.
  long n = 0;
  size_t pos = 0;
  while (pos <= len) {
    size_t e = pos;
    while (e < len && txt[e] != '\n') e++;
    size_t t1 = pos;
    while (t1 < e && txt[t1] != '\t') t1++;
    if (t1 < e) {
      size_t t2 = t1 + 1;
      while (t2 < e && txt[t2] != '\t') t2++;
      const std::string a(txt + pos, t1 - pos), b(txt + t1 + 1, t2 - t1 - 1);
      if (a.empty() || b.empty()) return FVAD_EFORMAT;
      char *end = nullptr;
      const float from = std::strtof(a.c_str(), &end);
      if (*end) return FVAD_EFORMAT;
      const float to = std::strtof(b.c_str(), &end);
      if (*end) return FVAD_EFORMAT;
      if ((size_t)n < cap && out) {
        out[2 * n] = from;
        out[2 * n + 1] = to;
      }
      n++;
    }
    pos = e + 1;
  }
  return n;
}
