// Synthetic onboard-audio generator (SURVEY.md §8(d) "Synthetic inputs").
//
// Deterministic per stream: seed = 0xF1AD0000 ^ stream_id.  48 kHz, f32 in
// [-1, 1], planar channels.  Content:
//   * engine: 8-harmonic series, f0 sweeping inside [150, 600] Hz, amplitude
//     0.01-0.03 (kept below the speech band trigger so the VADMachine sees
//     speech bursts), same in every channel;
//   * pink noise (Paul Kellet filter) at about -40 dBFS, independent per channel;
//   * speech-like bursts: glottal pulse train (90-250 Hz, slow vibrato) through
//     three formant resonators, 0.7-6 s on / 1-20 s off, amplitude 0.15-0.5,
//     louder in one channel (L/R gain ratio 0.6-1.0); burst intervals are the
//     ground-truth labels (Audacity txt, seconds);
//   * every 20th stream has 1 s of digital silence (exact zeros) at t = 5 s.
// This is workload data for tests and bench; it is not part of the hot path.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fvad.h"
#include "fvad_internal.h"

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double range(double a, double b) { return a + (b - a) * uni(); }
  double gauss() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

struct Resonator {  // 2-pole resonator, unity-ish peak gain
  double a1 = 0, a2 = 0, g = 0, y1 = 0, y2 = 0;
  void set(double f, double bw, double fs) {
    const double r = std::exp(-M_PI * bw / fs);
    a1 = 2 * r * std::cos(2 * M_PI * f / fs);
    a2 = -r * r;
    g = 1 - r;
  }
  double step(double x) {
    const double y = g * x + a1 * y1 + a2 * y2;
    y2 = y1;
    y1 = y;
    return y;
  }
};

}  // namespace

// Writes n samples of each of n_ch channels (planar, out[ch*n + i]).  Labels
// (from_sec, to_sec pairs) up to label_cap are written to labels; returns the
// number of labels.
extern "C" long fvad_synth_stream(uint32_t stream_id, size_t n, int n_ch, float *out, float *labels,
                                  size_t label_cap) {
  const double fs = 48000.0;
  Rng rng{0xF1AD0000ull ^ (uint64_t)stream_id};
  // stream-level parameters
  const double eng_amp = rng.range(0.01, 0.03);
  const double f0_lo = rng.range(150, 300), f0_hi = rng.range(350, 600);
  const double sweep_hz = rng.range(0.05, 0.3);
  double harm_amp[8];
  for (int h = 0; h < 8; h++) harm_amp[h] = rng.range(0.3, 1.0) / (1 + 0.3 * h);
  const bool has_silence = (stream_id % 20) == 19;
  std::vector<double> pink_b(7 * (size_t)n_ch, 0.0);
  // burst schedule
  struct Burst {
    size_t a, b;
    double amp, f0, louder_gain;
    int louder_ch;
    double f1, f2, f3;
  };
  std::vector<Burst> bursts;
  {
    double t = rng.range(1.0, 8.0);
    while (t < (double)n / fs) {
      Burst B;
      const double on = rng.range(0.7, 6.0);
      B.a = (size_t)(t * fs);
      B.b = (size_t)std::fmin((t + on) * fs, (double)n);
      B.amp = rng.range(0.15, 0.5);
      B.f0 = rng.range(90, 250);
      B.louder_ch = (int)(rng.next() % (uint64_t)(n_ch > 0 ? n_ch : 1));
      B.louder_gain = rng.range(0.6, 1.0);
      B.f1 = rng.range(500, 800);
      B.f2 = rng.range(1000, 1800);
      B.f3 = rng.range(2200, 3000);
      bursts.push_back(B);
      t += on + rng.range(1.0, 20.0);
    }
  }
  long n_labels = 0;
  for (const Burst &B : bursts) {
    if (B.b <= B.a) continue;
    if ((size_t)n_labels < label_cap && labels) {
      labels[2 * n_labels] = (float)((double)B.a / fs);
      labels[2 * n_labels + 1] = (float)((double)B.b / fs);
    }
    n_labels++;
  }
  // render
  double eng_phase[8] = {0};
  double glot_phase = 0;
  size_t bi = 0;
  Resonator r1, r2, r3;
  std::vector<double> chn(n_ch);
  for (size_t i = 0; i < n; i++) {
    const double t = (double)i / fs;
    const double f0 = f0_lo + (f0_hi - f0_lo) * 0.5 * (1 + std::sin(2 * M_PI * sweep_hz * t));
    double eng = 0;
    for (int h = 0; h < 8; h++) {
      eng_phase[h] += 2 * M_PI * f0 * (h + 1) / fs;
      if (eng_phase[h] > 2 * M_PI) eng_phase[h] -= 2 * M_PI;
      eng += harm_amp[h] * std::sin(eng_phase[h]);
    }
    eng *= eng_amp * 0.5;
    while (bi < bursts.size() && i >= bursts[bi].b) bi++;
    double speech = 0;
    int louder = -1;
    double lg = 1;
    if (bi < bursts.size() && i >= bursts[bi].a) {
      const Burst &B = bursts[bi];
      if (i == B.a) {
        r1.set(B.f1, 90, fs);
        r2.set(B.f2, 120, fs);
        r3.set(B.f3, 160, fs);
        glot_phase = 0;
      }
      const double vib = 1 + 0.05 * std::sin(2 * M_PI * 5 * t);
      glot_phase += B.f0 * vib / fs;
      double pulse = 0;
      if (glot_phase >= 1) {
        glot_phase -= 1;
        pulse = 1;
      }
      const double src = pulse - 0.02 * rng.gauss() * 0.1;
      const double env_t = (double)(i - B.a) / fs, env_r = (double)(B.b - i) / fs;
      const double env = std::fmin(1.0, std::fmin(env_t / 0.05, env_r / 0.05));
      speech = B.amp * env * (0.9 * r1.step(src) + 0.6 * r2.step(src) + 0.3 * r3.step(src)) * 8.0;
      louder = B.louder_ch;
      lg = B.louder_gain;
    }
    for (int c = 0; c < n_ch; c++) {
      double *b = &pink_b[7 * (size_t)c];
      const double w = rng.gauss() * 0.0035;
      b[0] = 0.99886 * b[0] + w * 0.0555179;
      b[1] = 0.99332 * b[1] + w * 0.0750759;
      b[2] = 0.96900 * b[2] + w * 0.1538520;
      b[3] = 0.86650 * b[3] + w * 0.3104856;
      b[4] = 0.55000 * b[4] + w * 0.5329522;
      b[5] = -0.7616 * b[5] - w * 0.0168980;
      const double pink = b[0] + b[1] + b[2] + b[3] + b[4] + b[5] + b[6] + w * 0.5362;
      b[6] = w * 0.115926;
      double v = eng + pink;
      if (louder >= 0) v += speech * ((c == louder) ? 1.0 : lg);
      if (has_silence && t >= 5.0 && t < 6.0) v = 0;
      if (v > 1) v = 1;
      if (v < -1) v = -1;
      out[(size_t)c * n + i] = (float)v;
    }
  }
  return n_labels;
}

// The same streams in the engine's push layout: ticks [tick0, tick0 + n_ticks)
// of streams base .. base + n_streams - 1, each generated with length
// total_ticks * 480 (the generator's output depends on the length), written
// as out[t][s][c][480].  Nothing is cached (a rank of an 8-GPU run would
// otherwise hold its whole 7.9 GB synthetic block for the job): streams are
// generated in groups on up to 16 host threads, each thread holding one
// stream at a time.
namespace {
unsigned synth_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }
}  // namespace

int fvad_synth_group(uint32_t base, int s0, int ns, int n_channels, int total_ticks, int tick0, int n_ticks,
                     float *out, size_t out_streams) {
  constexpr size_t F = fvad::kFrame;
  const size_t C = (size_t)n_channels, n = (size_t)total_ticks * F;
  const unsigned nthr = std::min<unsigned>(synth_threads(), (unsigned)ns);
  std::vector<std::thread> pool;
  bool oom = false;
  std::mutex mu;
  for (unsigned w = 0; w < nthr; w++) {
    pool.emplace_back([&, w]() {
      std::vector<float> one;
      try {
        one.resize(C * n);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        oom = true;
        return;
      }
      for (int s = (int)w; s < ns; s += (int)nthr) {
        fvad_synth_stream(base + (uint32_t)(s0 + s), n, (int)C, one.data(), nullptr, 0);
        for (size_t t = 0; t < (size_t)n_ticks; t++)
          for (size_t ch = 0; ch < C; ch++)
            std::memcpy(out + ((t * out_streams + (size_t)s) * C + ch) * F, one.data() + ch * n + (tick0 + t) * F,
                        F * sizeof(float));
      }
    });
  }
  for (auto &th : pool) th.join();
  return oom ? FVAD_ENOMEM : FVAD_OK;
}

extern "C" int fvad_synth_ticks(uint32_t base, int n_streams, int n_channels, int total_ticks, int tick0,
                                int n_ticks, float *out) {
  if (n_streams < 1 || n_channels < 1 || total_ticks < 1 || tick0 < 0 || n_ticks < 0 ||
      tick0 + n_ticks > total_ticks || (!out && n_ticks))
    return FVAD_EINVAL;
  if (!n_ticks) return FVAD_OK;
  return fvad_synth_group(base, 0, n_streams, n_channels, total_ticks, tick0, n_ticks, out, (size_t)n_streams);
}

// (kept for the ABI: nothing is cached since r5)
extern "C" void fvad_synth_cache_clear(void) {}
