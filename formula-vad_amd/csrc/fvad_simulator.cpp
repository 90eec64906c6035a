// `fvad-simulator -i plan.json` — the reference's simulator entry point
// (src/simulator.zig:74-139) on the batched GPU engine.
//
//   plan.json schema (simulator.zig:37-72, unknown fields ignored):
//     {"instances": [{"name", "audio_path", "ref_path"}],
//      "config": {"vad_config": {"fft_size", "use_denoiser", "vad_machine_config": {...},
//                 "alt_vad_machine_configs": [...]},
//                 "output_dir", "preload_audio", "audio_read_frame_count"}}
//   Paths are relative to the plan file (simulator.zig:142,
//   SimulationInstance.zig:91-95).  Audio: WAV (PCM 16/24/32-bit or float32,
//   48 kHz) — libsndfile/ogg are not available, see DESIGN.md.
//   Instances run in lock-step on the GPU(s) (simulator.zig:217-228 spawns one
//   thread per instance instead), streamed from their files push by push
//   (preload_audio: read whole first); any even fft_size (FFT.zig:29-31),
//   use_denoiser, alternative machines (run on the device; like the
//   reference, only the main machine's segments are reported); instances may
//   differ in channel count.  audio_read_frame_count does not change results
//   (the pipeline is chunking-invariant) and is not used.  Statistics use
//   {ignore_shorter_than = min_vad_duration_sec, extrude 5/10, fill gaps 5}
//   (simulator.zig:123-128); the report follows report_generator.zig:29-116.
#include <algorithm>
#include <cctype>
#include <cstdarg>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <memory>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/fvad.h"

namespace {

// ---------------- minimal JSON ----------------
struct Json {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<Json> a;
  std::map<std::string, Json> o;
  const Json *get(const std::string &k) const {
    if (kind != Obj) return nullptr;
    auto it = o.find(k);
    return it == o.end() ? nullptr : &it->second;
  }
};

struct Parser {
  const char *p, *e;
  bool ok = true;
  void ws() {
    while (p < e && std::isspace((unsigned char)*p)) p++;
  }
  bool lit(const char *w) {
    size_t n = std::strlen(w);
    if ((size_t)(e - p) >= n && std::strncmp(p, w, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  Json parse() {
    Json j;
    ws();
    if (p >= e) {
      ok = false;
      return j;
    }
    if (*p == '{') {
      j.kind = Json::Obj;
      p++;
      ws();
      if (p < e && *p == '}') {
        p++;
        return j;
      }
      while (ok) {
        ws();
        Json k = parse();
        if (k.kind != Json::Str) {
          ok = false;
          break;
        }
        ws();
        if (p >= e || *p != ':') {
          ok = false;
          break;
        }
        p++;
        j.o[k.s] = parse();
        ws();
        if (p < e && *p == ',') {
          p++;
          continue;
        }
        if (p < e && *p == '}') {
          p++;
          break;
        }
        ok = false;
      }
    } else if (*p == '[') {
      j.kind = Json::Arr;
      p++;
      ws();
      if (p < e && *p == ']') {
        p++;
        return j;
      }
      while (ok) {
        j.a.push_back(parse());
        ws();
        if (p < e && *p == ',') {
          p++;
          continue;
        }
        if (p < e && *p == ']') {
          p++;
          break;
        }
        ok = false;
      }
    } else if (*p == '"') {
      j.kind = Json::Str;
      p++;
      while (p < e && *p != '"') {
        if (*p == '\\' && p + 1 < e) {
          p++;
          const char c = *p;
          j.s += c == 'n' ? '\n' : c == 't' ? '\t' : c == 'r' ? '\r' : c;
        } else {
          j.s += *p;
        }
        p++;
      }
      if (p >= e) ok = false;
      p++;
    } else if (lit("true")) {
      j.kind = Json::Bool;
      j.b = true;
    } else if (lit("false")) {
      j.kind = Json::Bool;
    } else if (lit("null")) {
      j.kind = Json::Null;
    } else {
      char *end = nullptr;
      j.kind = Json::Num;
      j.n = std::strtod(p, &end);
      if (end == p) ok = false;
      p = end;
    }
    return j;
  }
};

bool read_file(const std::string &path, std::string &out) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  std::fclose(f);
  return true;
}

bool write_file(const std::string &path, const std::string &data) {
  FILE *f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
  return true;
}

std::string dirname_of(const std::string &p) {
  const size_t k = p.find_last_of('/');
  return k == std::string::npos ? "." : (k == 0 ? "/" : p.substr(0, k));
}
std::string join(const std::string &a, const std::string &b) {
  if (!b.empty() && b[0] == '/') return b;
  return a + "/" + b;
}
void make_path(const std::string &p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); i++) {
    cur += p[i];
    if (p[i] == '/' || i + 1 == p.size()) mkdir(cur.c_str(), 0755);
  }
}

// Mono 32-bit float WAV (AudioBuffer.Format.wav = SF_FORMAT_WAV | SF_FORMAT_FLOAT,
// AudioBuffer.zig:11-13): the recordings' container here (the reference saves
// them as ogg/vorbis, which is out of scope)
bool write_wav_f32(const std::string &path, const float *x, size_t n, int sample_rate) {
  std::string h;
  auto u32 = [&](uint32_t v) { h.append(reinterpret_cast<const char *>(&v), 4); };
  auto u16 = [&](uint16_t v) { h.append(reinterpret_cast<const char *>(&v), 2); };
  const uint32_t data_bytes = (uint32_t)(n * 4);
  h += "RIFF";
  u32(4 + (8 + 16) + (8 + 4) + (8 + data_bytes));
  h += "WAVEfmt ";
  u32(16);
  u16(3);  // WAVE_FORMAT_IEEE_FLOAT
  u16(1);
  u32((uint32_t)sample_rate);
  u32((uint32_t)sample_rate * 4);
  u16(4);
  u16(32);
  h += "fact";
  u32(4);
  u32((uint32_t)n);
  h += "data";
  u32(data_bytes);
  h.append(reinterpret_cast<const char *>(x), n * 4);
  return write_file(path, h);
}

// ---------------- WAV ingest (AudioFileStream replacement) ----------------
// Streams frames from the file (AudioFileStream.zig:56-98 over libsndfile):
// the header is parsed once, read() converts the next frames to planar f32,
// read_at() re-reads a range (the Recorder's capture of a segment).
// preload_audio (simulator.zig:41-42) reads the whole file into memory first.
struct WavStream {
  FILE *f = nullptr;
  int channels = 0, sample_rate = 0, fmt = 0, bits = 0, bps = 0;
  long long data_off = 0;
  size_t n = 0, pos = 0;        // frames in the file, next frame to read
  std::vector<float> pre;       // preloaded planar [ch][n] (preload_audio)
  std::vector<unsigned char> raw;

  ~WavStream() {
    if (f) std::fclose(f);
  }
  bool open(const std::string &path, std::string &err) {
    f = std::fopen(path.c_str(), "rb");
    if (!f) {
      err = "cannot open " + path;
      return false;
    }
    unsigned char h[12];
    if (std::fread(h, 1, 12, f) != 12 || std::memcmp(h, "RIFF", 4) || std::memcmp(h + 8, "WAVE", 4)) {
      err = path + ": not a RIFF/WAVE file (only WAV is supported without libsndfile)";
      return false;
    }
    long long data_len = -1;
    unsigned char ck[8];
    while (std::fread(ck, 1, 8, f) == 8) {
      const uint32_t len = le32(ck + 4);
      const long long body = std::ftell(f);
      if (!std::memcmp(ck, "fmt ", 4)) {
        unsigned char fm[40] = {};
        if (std::fread(fm, 1, std::min<uint32_t>(len, 40), f) < 16) break;
        fmt = (int)le16(fm);
        channels = (int)le16(fm + 2);
        sample_rate = (int)le32(fm + 4);
        bits = (int)le16(fm + 14);
        if (fmt == 0xFFFE && len >= 40) fmt = (int)le16(fm + 24);  // WAVE_FORMAT_EXTENSIBLE subformat
      } else if (!std::memcmp(ck, "data", 4)) {
        data_off = body;
        data_len = len;
        break;
      }
      std::fseek(f, body + len + (len & 1), SEEK_SET);
    }
    if (data_len < 0 || channels < 1) {
      err = path + ": missing fmt/data chunk";
      return false;
    }
    if (!((fmt == 1 && (bits == 16 || bits == 24 || bits == 32)) || (fmt == 3 && bits == 32))) {
      err = path + ": unsupported WAV encoding";
      return false;
    }
    bps = bits / 8;
    std::fseek(f, 0, SEEK_END);
    const long long avail = std::ftell(f) - data_off;
    n = (size_t)(std::min(data_len, avail) / ((long long)bps * channels));
    std::fseek(f, data_off, SEEK_SET);
    return true;
  }
  static uint32_t le16(const unsigned char *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
  static uint32_t le32(const unsigned char *p) { return le16(p) | le16(p + 2) << 16; }
  float sample(const unsigned char *o) const {
    float v;
    if (fmt == 3) {
      uint32_t u = le32(o);
      std::memcpy(&v, &u, 4);
    } else if (bits == 16) {
      v = (float)(int16_t)le16(o) / 32768.0f;  // libsndfile short->float normalisation
    } else if (bits == 24) {
      const int32_t x = (int32_t)(le16(o) | (uint32_t)o[2] << 16) << 8;
      v = (float)((double)x / 2147483648.0);
    } else {
      v = (float)((double)(int32_t)le32(o) / 2147483648.0);
    }
    return v;
  }
  // frames [from, from + k) into dst[c][0..k)
  size_t read_at(size_t from, float *const *dst, size_t k) {
    if (from >= n) return 0;
    k = std::min(k, n - from);
    if (!pre.empty()) {
      for (int c = 0; c < channels; c++) std::memcpy(dst[c], pre.data() + (size_t)c * n + from, k * sizeof(float));
      return k;
    }
    raw.resize(k * bps * channels);
    std::fseek(f, data_off + (long long)from * bps * channels, SEEK_SET);
    k = std::fread(raw.data(), (size_t)bps * channels, k, f);
    for (size_t i = 0; i < k; i++)
      for (int c = 0; c < channels; c++) dst[c][i] = sample(raw.data() + (i * channels + c) * bps);
    return k;
  }
  size_t read(float *const *dst, size_t k) {
    const size_t r = read_at(pos, dst, k);
    pos += r;
    return r;
  }
  void preload() {
    std::vector<float> buf((size_t)channels * n, 0.0f);
    std::vector<float *> d(channels);
    for (int c = 0; c < channels; c++) d[c] = buf.data() + (size_t)c * n;
    (void)read_at(0, d.data(), n);  // from the file (pre is still empty)
    pre.swap(buf);
  }
};

float num(const Json *j, float def) { return (j && j->kind == Json::Num) ? (float)j->n : def; }

void vadm_from_json(const Json *j, fvad_vadm_config &c) {
  fvad_vadm_config_default(&c);
  if (!j) return;
  c.speech_min_freq = num(j->get("speech_min_freq"), c.speech_min_freq);
  c.speech_max_freq = num(j->get("speech_max_freq"), c.speech_max_freq);
  c.long_term_speech_avg_sec = num(j->get("long_term_speech_avg_sec"), c.long_term_speech_avg_sec);
  if (const Json *v = j->get("initial_long_term_avg")) {
    if (v->kind == Json::Null) {
      c.has_initial_long_term_avg = 0;
    } else if (v->kind == Json::Num) {
      c.has_initial_long_term_avg = 1;
      c.initial_long_term_avg = v->n;
    }
  }
  c.short_term_speech_avg_sec = num(j->get("short_term_speech_avg_sec"), c.short_term_speech_avg_sec);
  c.speech_threshold_factor = num(j->get("speech_threshold_factor"), c.speech_threshold_factor);
  c.channel_vol_ratio_avg_sec = num(j->get("channel_vol_ratio_avg_sec"), c.channel_vol_ratio_avg_sec);
  c.channel_vol_ratio_threshold = num(j->get("channel_vol_ratio_threshold"), c.channel_vol_ratio_threshold);
  c.min_consecutive_sec_to_open = num(j->get("min_consecutive_sec_to_open"), c.min_consecutive_sec_to_open);
  c.max_speech_gap_sec = num(j->get("max_speech_gap_sec"), c.max_speech_gap_sec);
  c.min_vad_duration_sec = num(j->get("min_vad_duration_sec"), c.min_vad_duration_sec);
}

std::string fmt(const char *f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char *f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

const char *kDefinitions =
    "P   (Positives):                            Total duration of real speech segments (from reference labels)\n"
    "TP  (True positives):                       Duration of correctly detected speech segments\n"
    "FP  (False positives):                      Duration of incorrectly detected speech segments\n"
    "FN  (False negatives):                      Duration of missed speech segments\n"
    "TPR (True positive rate, sensitivity):      Probability that VAD detects a real speech segment. = TP / P \n"
    "FNR (False negative rate, miss rate):       Probability that VAD misses a speech segment.       = FN / P \n"
    "PPV (Precision, Positive predictive value): Probability that detected speech segment is true.   = TP / (TP + FP) \n"
    "FDR (False discovery rate):                 Probability that detected speech segment is false.  = FP / (TP + FP) ";

void usage() {
  std::printf("    -h, --help             Display this help and exit\n"
              "    -i, --input <str>      Simulation plan (path to JSON)\n"
              "    -d, --devices <list>   GPU ordinals, comma separated (default 0)\n"
              "    -m, --model <str>      rnnoise text model (default: synthetic seed 1)\n");
}

}  // namespace



extern "C" int fvad_simulator_main(int argc, char **argv) {
  std::string plan_path, model_path;
  std::vector<int> devices{0};
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if ((a == "-i" || a == "--input") && i + 1 < argc) {
      plan_path = argv[++i];
    } else if ((a == "-d" || a == "--devices") && i + 1 < argc) {
      devices.clear();
      std::string s = argv[++i];
      size_t p = 0;
      while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        if (q > p) devices.push_back(std::atoi(s.substr(p, q - p).c_str()));
        p = q + 1;
      }
    } else if ((a == "-m" || a == "--model") && i + 1 < argc) {
      model_path = argv[++i];
    } else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else {
      usage();
      return 1;
    }
  }
  if (plan_path.empty()) {
    usage();
    return 0;
  }
  std::string plan_txt;
  if (!read_file(plan_path, plan_txt)) {
    std::printf("Failed to initialize simulation: error.FileNotFound\n");
    return 1;
  }
  Parser ps{plan_txt.data(), plan_txt.data() + plan_txt.size()};
  Json plan = ps.parse();
  const Json *insts = plan.get("instances");
  if (!ps.ok || !insts || insts->kind != Json::Arr) {
    std::printf("Failed to initialize simulation: error.InvalidPlan\n");
    return 1;
  }
  const std::string base = dirname_of(plan_path);
  const Json *cfg = plan.get("config");
  const Json *vcfg = cfg ? cfg->get("vad_config") : nullptr;
  // VAD.Config (VAD.zig:17-23) and the simulator's own options (simulator.zig:37-45)
  fvad_vad_config vc;
  fvad_vad_config_default(&vc);
  fvad_vadm_config &mcfg = vc.vad_machine_config;
  vadm_from_json(vcfg ? vcfg->get("vad_machine_config") : nullptr, mcfg);
  std::vector<fvad_vadm_config> alts;
  bool preload = false;
  if (vcfg) {
    const Json *fs = vcfg->get("fft_size");
    const Json *ud = vcfg->get("use_denoiser");
    const Json *al = vcfg->get("alt_vad_machine_configs");
    if (fs && fs->kind == Json::Num) vc.fft_size = (int)fs->n;
    if (ud && ud->kind == Json::Bool) vc.use_denoiser = ud->b ? 1 : 0;
    if (al && al->kind == Json::Arr)
      for (const Json &aj : al->a) {
        fvad_vadm_config c;
        vadm_from_json(&aj, c);
        alts.push_back(c);
      }
  }
  vc.alt_vad_machine_configs = alts.empty() ? nullptr : alts.data();
  vc.n_alt = (int)alts.size();
  if (cfg) {
    const Json *pl = cfg->get("preload_audio");
    if (pl && pl->kind == Json::Bool) preload = pl->b;
  }
  // output directory <base>/<output_dir>/<unix ts>/ (simulator.zig:153-172)
  std::string out_dir;
  if (cfg) {
    const Json *od = cfg->get("output_dir");
    if (od && od->kind == Json::Str) {
      out_dir = join(join(base, od->s), std::to_string((long long)std::time(nullptr)));
      make_path(out_dir);
      write_file(join(out_dir, "plan.json"), plan_txt);
    }
  }
  struct Inst {
    std::string name;
    WavStream audio;
    std::vector<float> refs;
    std::vector<fvad_segment> segs;
  };
  std::vector<Inst> inst(insts->a.size());
  for (size_t k = 0; k < insts->a.size(); k++) {
    const Json &ij = insts->a[k];
    const Json *nm = ij.get("name"), *ap = ij.get("audio_path"), *rp = ij.get("ref_path");
    if (!nm || !ap || !rp) {
      std::printf("Failed to initialize simulation: error.MissingField\n");
      return 1;
    }
    inst[k].name = nm->s;
    std::string err;
    if (!inst[k].audio.open(join(base, ap->s), err)) {
      std::printf("Failed to initialize simulation: %s\n", err.c_str());
      return 1;
    }
    if (inst[k].audio.sample_rate != 48000) {
      std::printf("Failed to initialize simulation: error.InvalidSampleRate\n");
      return 1;
    }
    if (preload) inst[k].audio.preload();
    std::string ref_txt;
    if (!read_file(join(base, rp->s), ref_txt)) {
      std::printf("Failed to initialize simulation: error.FileNotFound (%s)\n", rp->s.c_str());
      return 1;
    }
    const long n = fvad_parse_audacity(ref_txt.data(), ref_txt.size(), nullptr, 0);
    if (n < 0) {
      std::printf("Failed to initialize simulation: error.InvalidCharacter (%s)\n", rp->s.c_str());
      return 1;
    }
    inst[k].refs.resize(2 * (size_t)n);
    fvad_parse_audacity(ref_txt.data(), ref_txt.size(), inst[k].refs.data(), (size_t)n);
  }
  fvad_model *model = nullptr;
  int rc = model_path.empty() ? fvad_model_synthetic(1, &model) : fvad_model_load_text(model_path.c_str(), &model);
  if (rc) {
    std::printf("Failed to initialize simulation: model: %s\n", fvad_last_error());
    return 1;
  }
  if (!inst.empty()) {
    fvad_multi *multi = nullptr;
    std::vector<int> chans(inst.size());
    for (size_t k = 0; k < inst.size(); k++) chans[k] = inst[k].audio.channels;
    rc = fvad_multi_create_ex((int)inst.size(), chans.data(), model, devices.data(), (int)devices.size(), &vc, 100,
                              &multi);
    if (rc) {
      std::printf("simulation failed: %s\n", fvad_last_error());
      fvad_model_free(model);
      return 1;
    }
    for (auto &I : inst)
      std::fprintf(stderr, "info(sim_instance): %s: Streaming %.2fs from audio file. Running...\n", I.name.c_str(),
                   (double)I.audio.n / 48000.0);
    // the read loop: each part thread pulls its instances' next frames
    auto reader = [](void *ctx, int s, float *const *dst, size_t max_frames) -> size_t {
      return (*static_cast<std::vector<Inst> *>(ctx))[s].audio.read(dst, max_frames);
    };
    rc = fvad_multi_run_stream(multi, reader, &inst);
    if (rc) {
      std::printf("simulation failed: %s\n", fvad_last_error());
      fvad_multi_destroy(multi);
      fvad_model_free(model);
      return 1;
    }
    for (size_t k = 0; k < inst.size(); k++) {
      const size_t n = fvad_multi_segments(multi, (int)k, nullptr, 0);
      inst[k].segs.resize(n);
      fvad_multi_segments(multi, (int)k, inst[k].segs.data(), n);
    }
    fvad_multi_destroy(multi);
    // on_recording (SimulationInstance.zig:28-58): the Recorder's capture of
    // every completed segment -- raw input of [sample_from, sample_to) on the
    // lowest-RMS channel (Recorder.zig:95-146) -- saved as NNN-<name>.wav
    if (!out_dir.empty()) {
      for (auto &I : inst) {
        size_t count = 0;
        const int channels = I.audio.channels;
        std::vector<float> buf;
        std::vector<float *> dst(channels);
        std::vector<const float *> ch(channels);
        for (auto &sg : I.segs) {
          if (sg.sample_to > I.audio.n || sg.sample_to <= sg.sample_from) continue;
          const size_t len = (size_t)(sg.sample_to - sg.sample_from);
          buf.assign((size_t)channels * len, 0.0f);
          for (int c = 0; c < channels; c++) ch[c] = dst[c] = buf.data() + (size_t)c * len;
          if (I.audio.read_at(sg.sample_from, dst.data(), len) != len) continue;
          const int best = fvad_recording_channel(ch.data(), channels, len);
          char nm[32];
          std::snprintf(nm, sizeof nm, "%03zu-", count++);
          if (!write_wav_f32(join(out_dir, std::string(nm) + I.name + ".wav"), ch[best], len, 48000))
            std::fprintf(stderr, "error(sim_instance): Failed to save recording %s%s.wav\n", nm, I.name.c_str());
        }
      }
    }
  }
  fvad_model_free(model);

  // statistics + report (report_generator.zig:29-116)
  fvad_stat_config sc{mcfg.min_vad_duration_sec, 5, 10, 5};
  std::string rep;
  rep += "\n\n=> Definitions\n\n";
  rep += kDefinitions;
  rep += "\n\n=> Performance Report\n\n";
  rep += fmt("| %30s | %4s | %4s | %4s | %4s | %6s | %6s | %6s | %8s |\n", "Name", "P", "TP", "FP", "FN", "TPR", "FNR",
             "PPV", "FDR (!)");
  rep += "| ------------------------------ | ---- | ---- | ---- | ---- | ------ | ------ | ------ | -------- |\n";
  std::vector<fvad_single_stats> all;
  for (auto &I : inst) {
    std::vector<float> vs;
    for (auto &s : I.segs) {
      vs.push_back((float)s.sample_from / 48000.0f);
      vs.push_back((float)s.sample_to / 48000.0f);
    }
    fvad_single_stats st;
    fvad_eval_stats(vs.data(), vs.size() / 2, I.refs.data(), I.refs.size() / 2, &sc, &st);
    all.push_back(st);
    rep += fmt("| %30s | %4.0f | %4.0f | %4.0f | %4.0f | %5.1f%% | %5.1f%% | %5.1f%% | %7.1f%% |\n", I.name.c_str(),
               st.total_positives_sec, st.true_positives_sec, st.false_positives_sec, st.false_negatives_sec,
               st.true_positive_rate * 100, st.false_negative_rate * 100, st.precision * 100,
               st.false_discovery_rate * 100);
    if (!out_dir.empty()) {
      // serializeEvaluatorToAudacityTxt (formats.zig:38-56): vad segments then unmatched refs
      std::string txt;
      std::vector<char> matched_ref(I.refs.size() / 2, 0);
      for (size_t v = 0; v < I.segs.size(); v++) {
        const float f = vs[2 * v], t = vs[2 * v + 1];
        bool any = false;
        for (size_t r = 0; r < I.refs.size() / 2; r++) {
          const float mf = std::max(f, I.refs[2 * r]), mt = std::min(t, I.refs[2 * r + 1]);
          if (mt - mf > 0.0f) {
            any = true;
            matched_ref[r] = 1;
          }
        }
        const std::string dbg = fmt("rnn:%.2f%% vr:%.2f", I.segs[v].debug_rnn_vad * 100,
                                    I.segs[v].debug_avg_speech_vol_ratio);
        txt += fmt("%.4f\t%.4f\t%s%s\n", f, t, any ? "" : "UNMATCHED ", dbg.c_str());
      }
      for (size_t r = 0; r < I.refs.size() / 2; r++)
        if (!matched_ref[r]) txt += fmt("%.4f\t%.4f\tmissed\n", I.refs[2 * r], I.refs[2 * r + 1]);
      write_file(join(out_dir, I.name + "-audacity.txt"), txt);
    }
  }
  fvad_aggregate_stats ag;
  fvad_eval_aggregate(all.data(), all.size(), &ag);
  rep += "\n=> Aggregate stats \n\n";
  rep += fmt("Total speech duration  (P): %7.1f sec\n", ag.total_positives_sec);
  rep += fmt("True positives        (TP): %7.1f sec\n", ag.true_positives_sec);
  rep += fmt("False positives       (FP): %7.1f sec\n", ag.false_positives_sec);
  rep += fmt("False negatives       (FN): %7.1f sec", ag.false_negatives_sec);
  rep += "    Min.    Avg.    Max. \n";
  const fvad_agg_stat *rows[4] = {&ag.true_positive_rate, &ag.false_negative_rate, &ag.precision,
                                  &ag.false_discovery_rate};
  const char *labels[4] = {"True positive rate   (TPR)", "False negative rate  (FNR)", "Precision            (PPV)",
                           "False discovery rate (FDR)"};
  for (int r = 0; r < 4; r++)
    rep += fmt("%s:   %5.1f%%  |  %5.1f%% /%5.1f%% /%5.1f%% \n", labels[r], rows[r]->overall * 100, rows[r]->min * 100,
               rows[r]->avg * 100, rows[r]->max * 100);
  rep += fmt("F-Score (\xce\xb2 = %5.2f)       :   %5.1f%% \n", ag.f_score_beta, ag.f_score * 100);
  rep += fmt("Fowlkes-Mallows index     :   %5.1f%% \n", ag.fm_index * 100);
  std::fputs(rep.c_str(), stdout);
  if (!out_dir.empty()) write_file(join(out_dir, "report.txt"), rep);
  // machine-readable per-instance summary for tests
  if (const char *js = std::getenv("FVAD_SIM_JSON")) {
    std::string j = "{\"instances\": [";
    for (size_t k = 0; k < inst.size(); k++) {
      j += fmt("%s{\"name\": \"%s\", \"tp\": %.9g, \"fp\": %.9g, \"fn\": %.9g, \"segments\": [", k ? ", " : "",
               inst[k].name.c_str(), all[k].true_positives_sec, all[k].false_positives_sec,
               all[k].false_negatives_sec);
      for (size_t s = 0; s < inst[k].segs.size(); s++)
        j += fmt("%s[%llu, %llu]", s ? ", " : "", (unsigned long long)inst[k].segs[s].sample_from,
                 (unsigned long long)inst[k].segs[s].sample_to);
      j += "]}";
    }
    j += "]}\n";
    write_file(js, j);
  }
  return 0;
}
