// rnnoise model handling for the MI355X engine.
//
// rnnoise_create(NULL) (Denoiser.zig:23) uses the weights compiled into
// rnn_data.c, which is absent from /root/reference.  The engine therefore takes
// an explicit model:
//   * fvad_model_load_text: the rnnoise text model format (rnn_reader.c,
//     [upstream, recalled]) - "rnnoise-nu model file version 1" followed by six
//     layers (input_dense, vad_gru, noise_gru, denoise_gru, denoise_output,
//     vad_output), each "nb_inputs nb_neurons activation" then its int8 arrays;
//   * fvad_model_synthetic: deterministic int8 weights for
//     parity fixtures and benchmarks.
// Layout on the device: every int8 array converted to f32 (exact) so the
// kernels' multiply is the same f32 product the C code forms after integer
// promotion.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "fvad_internal.h"
#include "../../include/fvad.h"

using fvad::HostLayer;
using fvad::HostModel;

struct fvad_model {
  HostModel m;
};

namespace {

struct LayerSpec {
  int nin, nout, act;
  bool gru;
  int sw, sr, sb;  // synthetic scales for input weights, recurrent weights, bias
};

// text-file layer order; activations of the upstream model (tanh, relu x3, sigmoid x2)
const LayerSpec kSpec[6] = {
    {42, 24, fvad::kActTanh, false, 64, 0, 16},     // input_dense
    {24, 24, fvad::kActRelu, true, 64, 40, 16},     // vad_gru
    {90, 48, fvad::kActRelu, true, 40, 24, 16},     // noise_gru
    {114, 96, fvad::kActRelu, true, 40, 20, 16},    // denoise_gru
    {96, 22, fvad::kActSigmoid, false, 48, 0, 16},  // denoise_output
    {24, 1, fvad::kActSigmoid, false, 64, 0, 16},   // vad_output
};

size_t layout(HostModel &hm) {
  size_t off = 0;
  for (int l = 0; l < 6; l++) {
    HostLayer &L = hm.layers[l];
    const size_t g = L.gru ? 3 : 1;
    L.off_w = off;
    off += (size_t)L.nin * L.nout * g;
    if (L.gru) {
      L.off_r = off;
      off += (size_t)L.nout * L.nout * 3;
    }
    L.off_b = off;
    off += (size_t)L.nout * g;
  }
  return off;
}

uint64_t mix(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

bool check_shapes(const HostModel &hm) {
  // connectivity required by compute_rnn (rnn.c): input 42 features
  const HostLayer *L = hm.layers;
  if (L[0].nin != fvad::kFeat) return false;
  if (L[1].nin != L[0].nout) return false;
  if (L[2].nin != L[0].nout + L[1].nout + fvad::kFeat) return false;
  if (L[3].nin != L[1].nout + L[2].nout + fvad::kFeat) return false;
  if (L[4].nin != L[3].nout || L[4].nout != fvad::kBands) return false;
  if (L[5].nin != L[1].nout || L[5].nout != 1) return false;
  for (int i = 0; i < 6; i++)
    if (L[i].nout > fvad::kMaxNeurons || L[i].nout < 1) return false;
  return true;
}

}  // namespace

extern "C" int fvad_model_synthetic(uint64_t seed, fvad_model **out) {
  if (!out) return FVAD_EINVAL;
  fvad_model *m = new fvad_model();
  for (int l = 0; l < 6; l++) {
    m->m.layers[l].nin = kSpec[l].nin;
    m->m.layers[l].nout = kSpec[l].nout;
    m->m.layers[l].act = kSpec[l].act;
    m->m.layers[l].gru = kSpec[l].gru;
  }
  m->m.blob_size = layout(m->m);
  m->m.blob = (int8_t *)std::calloc(m->m.blob_size, 1);
  uint64_t s = seed;
  for (int l = 0; l < 6; l++) {
    const HostLayer &L = m->m.layers[l];
    const LayerSpec &S = kSpec[l];
    const size_t g = L.gru ? 3 : 1;
    auto fill = [&](size_t off, size_t n, int scale) {
      for (size_t i = 0; i < n; i++)
        m->m.blob[off + i] = (int8_t)((int)(mix(s) % (uint64_t)(2 * scale + 1)) - scale);
    };
    fill(L.off_w, (size_t)L.nin * L.nout * g, S.sw);
    if (L.gru) fill(L.off_r, (size_t)L.nout * L.nout * 3, S.sr);
    fill(L.off_b, (size_t)L.nout * g, S.sb);
  }
  *out = m;
  return FVAD_OK;
}

extern "C" int fvad_model_load_text(const char *path, fvad_model **out) {
  if (!path || !out) return FVAD_EINVAL;
  FILE *f = std::fopen(path, "r");
  if (!f) return FVAD_EIO;
  int ver = 0;
  if (std::fscanf(f, "rnnoise-nu model file version %d\n", &ver) != 1 || ver != 1) {
    std::fclose(f);
    return FVAD_EFORMAT;
  }
  fvad_model *m = new fvad_model();
  // first pass: read headers and arrays into a temporary blob
  std::string err;
  size_t cap = 1 << 20, used = 0;
  int8_t *blob = (int8_t *)std::malloc(cap);
  auto rd = [&](int *v) { return std::fscanf(f, "%d", v) == 1; };
  bool ok = true;
  for (int l = 0; l < 6 && ok; l++) {
    HostLayer &L = m->m.layers[l];
    int nin, nout, act;
    if (!rd(&nin) || !rd(&nout) || !rd(&act) || nin < 0 || nin > 128 || nout < 0 || nout > 128 || act < 0 ||
        act > 128) {
      ok = false;
      break;
    }
    L.nin = nin;
    L.nout = nout;
    L.act = act == 1 ? fvad::kActSigmoid : act == 2 ? fvad::kActRelu : fvad::kActTanh;
    L.gru = kSpec[l].gru;
    const size_t g = L.gru ? 3 : 1;
    size_t counts[3] = {(size_t)nin * nout * g, L.gru ? (size_t)nout * nout * 3 : 0, (size_t)nout * g};
    size_t *offs[3] = {&L.off_w, &L.off_r, &L.off_b};
    for (int a = 0; a < 3 && ok; a++) {
      *offs[a] = used;
      for (size_t i = 0; i < counts[a]; i++) {
        int v;
        if (!rd(&v)) {
          ok = false;
          break;
        }
        if (used == cap) {
          cap *= 2;
          blob = (int8_t *)std::realloc(blob, cap);
        }
        blob[used++] = (int8_t)v;
      }
    }
  }
  std::fclose(f);
  if (!ok || !check_shapes(m->m)) {
    std::free(blob);
    delete m;
    return FVAD_EFORMAT;
  }
  m->m.blob = blob;
  m->m.blob_size = used;
  *out = m;
  return FVAD_OK;
}

extern "C" void fvad_model_free(fvad_model *m) {
  if (!m) return;
  std::free(m->m.blob);
  delete m;
}

extern "C" size_t fvad_model_blob(const fvad_model *m, int8_t *blob) {
  if (!m) return 0;
  if (blob) std::memcpy(blob, m->m.blob, m->m.blob_size);
  return m->m.blob_size;
}

const HostModel *fvad_model_host(const fvad_model *m) { return &m->m; }
