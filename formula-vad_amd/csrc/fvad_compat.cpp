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
  int nfft, ncfft, nf, inverse;
  uint64_t magic;
  int fac[2 * fvad::kMaxFactors];  // kf_factor(ncfft): (p, m) pairs
};

namespace {
constexpr uint64_t kMagic = 0x4656414446465452ull;  // "FVADFFTR"

// cfg memory: header, twiddles [ncfft], super twiddles [ncfft/2], leaf
// permutation [ncfft] -- the device tables are uploaded from it per call
size_t tab_floats(int ncfft) { return 2 * (size_t)ncfft + 2 * (size_t)(ncfft / 2) + (size_t)ncfft; }
size_t cfg_bytes(int ncfft) { return sizeof(kiss_fftr_state) + sizeof(float) * tab_floats(ncfft); }

// kf_factor (kissfft): powers of 4, then 2, then odd primes
int factor(int n, int *fac) {
  int p = 4, k = 0;
  const double floor_sqrt = std::floor(std::sqrt((double)n));
  do {
    while (n % p) {
      switch (p) {
        case 4: p = 2; break;
        case 2: p = 3; break;
        default: p += 2; break;
      }
      if (p > floor_sqrt) p = n;
    }
    n /= p;
    fac[2 * k] = p;
    fac[2 * k + 1] = n;
    k++;
  } while (n > 1);
  return k;
}

// kf_work's leaf placement: Fout position -> input index
void leaf_perm(int *perm, int out_base, int in_base, int fstride, const int *fac) {
  const int p = fac[0], m = fac[1];
  if (m == 1) {
    for (int j = 0; j < p; j++) perm[out_base + j] = in_base + j * fstride;
  } else {
    for (int j = 0; j < p; j++) leaf_perm(perm, out_base + j * m, in_base + j * fstride, fstride * p, fac + 2);
  }
}

struct DevScratch {
  int dev = -1;
  size_t cap = 0;
  float *buf = nullptr;
  hipStream_t stream = nullptr;
} g_fft;

}  // namespace

// Same protocol as mborgerding kiss_fftr_alloc (FFT.zig:179-208): with
// lenmem != NULL the required size is written to *lenmem and the cfg is built
// in mem only when *lenmem was large enough (mem = NULL, *lenmem = 1 is the
// size probe: returns NULL).  Any even nfft; forward transforms only.
extern "C" kiss_fftr_cfg kiss_fftr_alloc(int nfft, int inverse_fft, void *mem, size_t *lenmem) {
  if (nfft <= 0 || (nfft & 1)) return nullptr;
  const int ncfft = nfft / 2;
  const size_t need = cfg_bytes(ncfft);
  kiss_fftr_state *st = nullptr;
  if (lenmem == nullptr) {
    st = (kiss_fftr_state *)std::malloc(need);
  } else {
    if (mem != nullptr && *lenmem >= need) st = (kiss_fftr_state *)mem;
    *lenmem = need;
  }
  if (!st) return nullptr;
  st->nfft = nfft;
  st->ncfft = ncfft;
  st->inverse = inverse_fft;
  st->magic = kMagic;
  st->nf = factor(ncfft, st->fac);
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
  leaf_perm(perm, 0, 0, 1, st->fac);
  return st;
}

extern "C" void kiss_fftr(kiss_fftr_cfg cfg, const float *timedata, kiss_fft_cpx *freqdata) {
  if (!cfg || cfg->magic != kMagic || cfg->inverse) {
    std::fprintf(stderr, "kiss fft usage error: improper alloc\n");
    return;
  }
  const int nc = cfg->ncfft;
  const float *tw = reinterpret_cast<const float *>(cfg + 1);
  const size_t tf = tab_floats(nc);
  // device: tables, factors, input, output, work arrays W + S (used when
  // they do not fit the kernel's LDS)
  const size_t fac_floats = 2 * fvad::kMaxFactors;
  const size_t need = tf + fac_floats + 2 * (size_t)nc + 2 * (size_t)(nc + 1) + 4 * (size_t)nc;
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
  int *d_fac = reinterpret_cast<int *>(d_tab + tf);
  float *d_in = d_tab + tf + fac_floats;
  float *d_out = d_in + 2 * (size_t)nc;
  float *d_work = d_out + 2 * (size_t)(nc + 1);
  hipStream_t s = g_fft.stream;
  bool ok = hipMemcpyAsync(d_tab, tw, tf * sizeof(float), hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemcpyAsync(d_fac, cfg->fac, sizeof(cfg->fac), hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemcpyAsync(d_in, timedata, 2 * (size_t)nc * sizeof(float), hipMemcpyHostToDevice, s) == hipSuccess &&
            fvad::launch_kiss_fftr(nc, d_fac, cfg->nf, d_tab, d_tab + 2 * nc,
                                   reinterpret_cast<const int *>(d_tab + 2 * nc + 2 * (nc / 2)), d_in, d_out, d_work,
                                   s) == hipSuccess &&
            hipMemcpyAsync(freqdata, d_out, 2 * (size_t)(nc + 1) * sizeof(float), hipMemcpyDeviceToHost, s) ==
                hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  if (!ok) {
    std::fprintf(stderr, "kiss_fftr: HIP failure\n");
    std::abort();
  }
}
