// Compatibility shims with the exact C signatures the reference binds today:
//   rnnoise_create / rnnoise_destroy / rnnoise_process_frame /
//   rnnoise_get_frame_size           (src/Denoiser.zig:12-14,23,36,60,69)
//   kiss_fftr_alloc / kiss_fftr      (src/FFT.zig:5-9,90,179-208)
// Both route every call to the HIP kernels (batch of one).  There is no CPU
// fallback: without a usable GPU rnnoise_create returns NULL and kiss_fftr
// aborts with a diagnostic, so a missing device fails loudly.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/fvad.h"
#include "fvad_internal.h"
#include "fvad_kernels.h"

void fvad_engine_set_raw_s16(fvad_engine *e, int raw);

namespace {
std::mutex g_mu;
const fvad_model *g_default_model = nullptr;
fvad_model *g_synth_default = nullptr;
}  // namespace

struct DenoiseState {
  fvad_engine *engine;
};

extern "C" void fvad_set_default_model(const fvad_model *model) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_default_model = model;
}

extern "C" DenoiseState *rnnoise_create(RNNModel *model) {
  const fvad_model *m = model;
  if (!m) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_default_model) {
      if (!g_synth_default && fvad_model_synthetic(0, &g_synth_default) != FVAD_OK) return nullptr;
      m = g_synth_default;
    } else {
      m = g_default_model;
    }
  }
  fvad_engine_config cfg;
  fvad_engine_config_default(&cfg, 1, 1);
  cfg.max_ticks = 1;
  cfg.want_denoised = 1;
  cfg.mode = FVAD_MODE_FUSED;  // one frame per call: nothing to parallelise over time
  fvad_engine *e = nullptr;
  if (fvad_engine_create(&cfg, m, &e) != FVAD_OK) return nullptr;
  fvad_engine_set_raw_s16(e, 1);
  DenoiseState *st = new DenoiseState{e};
  return st;
}

extern "C" void rnnoise_destroy(DenoiseState *st) {
  if (!st) return;
  fvad_engine_destroy(st->engine);
  delete st;
}

extern "C" int rnnoise_get_frame_size(void) { return fvad::kFrame; }

extern "C" float rnnoise_process_frame(DenoiseState *st, float *out, const float *in) {
  if (!st || !out || !in) return 0.0f;
  float vad = 0.0f;
  fvad_outputs o;
  std::memset(&o, 0, sizeof(o));
  o.vad = &vad;
  o.denoised = out;
  if (fvad_engine_push(st->engine, in, 1, nullptr, &o) != FVAD_OK) {
    std::fprintf(stderr, "rnnoise_process_frame: %s\n", fvad_last_error());
    std::abort();
  }
  return vad;
}

// ---------------------------------------------------------------------------
// kiss_fftr: the cfg lives in caller memory (FFT.zig:36-40 allocates it).
// Layout: header | twiddles[ncfft] | super[ncfft/2] | perm[ncfft].
// ---------------------------------------------------------------------------
struct kiss_fftr_state {
  int nfft, ncfft, stages, inverse;
  uint64_t magic;
};

namespace {
constexpr uint64_t kMagic = 0x4656414446465452ull;  // "FVADFFTR"

size_t cfg_bytes(int ncfft) {
  return sizeof(kiss_fftr_state) + sizeof(float) * 2 * ncfft + sizeof(float) * 2 * (ncfft / 2) +
         sizeof(int) * ncfft;
}

void leaf_perm(int *perm, int out_base, int in_base, int fstride, int n) {
  // kf_work leaf placement for radix-4-only factorisations
  const int m = n / 4;
  if (m == 1) {
    for (int j = 0; j < 4; j++) perm[out_base + j] = in_base + j * fstride;
  } else {
    for (int j = 0; j < 4; j++) leaf_perm(perm, out_base + j * m, in_base + j * fstride, fstride * 4, m);
  }
}

struct DevScratch {
  int dev = -1;
  size_t cap = 0;
  float *buf = nullptr;
  hipStream_t stream = nullptr;
} g_fft;

}  // namespace

extern "C" kiss_fftr_cfg kiss_fftr_alloc(int nfft, int inverse_fft, void *mem, size_t *lenmem) {
  if (nfft <= 0 || (nfft & 1)) return nullptr;
  const int ncfft = nfft / 2;
  int stages = 0, n = ncfft;
  while (n > 1 && n % 4 == 0) {
    n /= 4;
    stages++;
  }
  if (n != 1 || stages < 1 || ncfft > 4096) {  // LDS holds ncfft complex (<= 32 KiB)
    if (lenmem) *lenmem = 0;
    return nullptr;  // device path: nfft/2 must be a power of 4
  }
  const size_t need = cfg_bytes(ncfft);
  kiss_fftr_state *st = nullptr;
  if (lenmem == nullptr) {
    st = (kiss_fftr_state *)std::malloc(need);
  } else {
    if (*lenmem >= need) st = (kiss_fftr_state *)mem;
    *lenmem = need;
  }
  if (!st) return nullptr;
  st->nfft = nfft;
  st->ncfft = ncfft;
  st->stages = stages;
  st->inverse = inverse_fft;
  st->magic = kMagic;
  float *tw = reinterpret_cast<float *>(st + 1);
  float *sup = tw + 2 * ncfft;
  int *perm = reinterpret_cast<int *>(sup + 2 * (ncfft / 2));
  for (int i = 0; i < ncfft; i++) {
    const double pi = 3.141592653589793238462643383279502884197169399375105820974944;
    double phase = -2 * pi * i / ncfft;
    if (inverse_fft) phase *= -1;
    tw[2 * i] = (float)std::cos(phase);
    tw[2 * i + 1] = (float)std::sin(phase);
  }
  for (int i = 0; i < ncfft / 2; i++) {
    double phase = -3.14159265358979323846264338327 * ((double)(i + 1) / ncfft + .5);
    if (inverse_fft) phase *= -1;
    sup[2 * i] = (float)std::cos(phase);
    sup[2 * i + 1] = (float)std::sin(phase);
  }
  leaf_perm(perm, 0, 0, 1, ncfft);
  return st;
}

extern "C" void kiss_fftr(kiss_fftr_cfg cfg, const float *timedata, kiss_fft_cpx *freqdata) {
  if (!cfg || cfg->magic != kMagic || cfg->inverse) {
    std::fprintf(stderr, "kiss fft usage error: improper alloc\n");
    return;
  }
  const int nc = cfg->ncfft;
  const float *tw = reinterpret_cast<const float *>(cfg + 1);
  const size_t tab_floats = 2 * (size_t)nc + 2 * (size_t)(nc / 2) + (size_t)nc;
  const size_t need = tab_floats + 2 * (size_t)nc + 2 * (size_t)(nc + 1);
  std::lock_guard<std::mutex> lk(g_mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    std::fprintf(stderr, "kiss_fftr: no HIP device\n");
    std::abort();
  }
  if (g_fft.dev != dev || g_fft.cap < need) {
    if (g_fft.buf) (void)hipFree(g_fft.buf);
    if (!g_fft.stream && hipStreamCreate(&g_fft.stream) != hipSuccess) std::abort();
    if (hipMalloc(&g_fft.buf, need * sizeof(float)) != hipSuccess) {
      std::fprintf(stderr, "kiss_fftr: device allocation failed\n");
      std::abort();
    }
    g_fft.cap = need;
    g_fft.dev = dev;
  }
  float *d_tab = g_fft.buf;
  float *d_in = d_tab + tab_floats;
  float *d_out = d_in + 2 * (size_t)nc;
  hipStream_t s = g_fft.stream;
  bool ok = hipMemcpyAsync(d_tab, tw, tab_floats * sizeof(float), hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemcpyAsync(d_in, timedata, 2 * (size_t)nc * sizeof(float), hipMemcpyHostToDevice, s) == hipSuccess &&
            fvad::launch_kiss_fftr(nc, cfg->stages, d_tab, d_tab + 2 * nc,
                                   reinterpret_cast<const int *>(d_tab + 2 * nc + 2 * (nc / 2)), d_in, d_out,
                                   s) == hipSuccess &&
            hipMemcpyAsync(freqdata, d_out, 2 * (size_t)(nc + 1) * sizeof(float), hipMemcpyDeviceToHost, s) ==
                hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  if (!ok) {
    std::fprintf(stderr, "kiss_fftr: HIP failure\n");
    std::abort();
  }
}
