/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * rnnoise model container.  rnn_data.c (the built-in weights used by
 * rnnoise_create(NULL), Denoiser.zig:23) is absent from /root/reference, so
 * parity runs on (a) a deterministic synthetic int8 model whose generator is
 * specified in DESIGN.md §Model and implemented independently by the product,
 * or (b) a model file in the rnnoise text format [upstream rnn_reader.c,
 * recalled]: header "rnnoise-nu model file version 1", then for each layer in
 * the order input_dense, vad_gru, noise_gru, denoise_gru, denoise_output,
 * vad_output: nb_inputs nb_neurons activation(0 tanh,1 sigmoid,2 relu) and the
 * int8 arrays (dense: weights, bias; gru: input weights, recurrent weights, bias).
 * Also used by the CPU baseline (ora_bench_denoise, pthreads).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "oracle.h"

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void fill(int8_t *p, size_t n, int scale, uint64_t *s) {
  size_t i;
  for (i = 0; i < n; i++) p[i] = (int8_t)((int)(splitmix64(s) % (uint64_t)(2 * scale + 1)) - scale);
}

static void dense_alloc(ora_dense *d, int in, int out, int act) {
  d->nb_inputs = in;
  d->nb_neurons = out;
  d->activation = act;
  d->input_weights = (int8_t *)calloc((size_t)in * out, 1);
  d->bias = (int8_t *)calloc((size_t)out, 1);
}

static void gru_alloc(ora_gru *g, int in, int out, int act) {
  g->nb_inputs = in;
  g->nb_neurons = out;
  g->activation = act;
  g->input_weights = (int8_t *)calloc((size_t)in * out * 3, 1);
  g->recurrent_weights = (int8_t *)calloc((size_t)out * out * 3, 1);
  g->bias = (int8_t *)calloc((size_t)out * 3, 1);
}

ora_model *ora_model_synthetic(uint64_t seed) {
  ora_model *m = (ora_model *)calloc(1, sizeof(ora_model));
  uint64_t s = seed;
  dense_alloc(&m->input_dense, 42, 24, ORA_ACT_TANH);
  gru_alloc(&m->vad_gru, 24, 24, ORA_ACT_RELU);
  gru_alloc(&m->noise_gru, 90, 48, ORA_ACT_RELU);
  gru_alloc(&m->denoise_gru, 114, 96, ORA_ACT_RELU);
  dense_alloc(&m->denoise_output, 96, 22, ORA_ACT_SIGMOID);
  dense_alloc(&m->vad_output, 24, 1, ORA_ACT_SIGMOID);
  /* generation order == text-file order; scales from DESIGN.md §Model */
  fill(m->input_dense.input_weights, 42 * 24, 64, &s);
  fill(m->input_dense.bias, 24, 16, &s);
  fill(m->vad_gru.input_weights, 24 * 72, 64, &s);
  fill(m->vad_gru.recurrent_weights, 24 * 72, 40, &s);
  fill(m->vad_gru.bias, 72, 16, &s);
  fill(m->noise_gru.input_weights, 90 * 144, 40, &s);
  fill(m->noise_gru.recurrent_weights, 48 * 144, 24, &s);
  fill(m->noise_gru.bias, 144, 16, &s);
  fill(m->denoise_gru.input_weights, 114 * 288, 40, &s);
  fill(m->denoise_gru.recurrent_weights, 96 * 288, 20, &s);
  fill(m->denoise_gru.bias, 288, 16, &s);
  fill(m->denoise_output.input_weights, 96 * 22, 48, &s);
  fill(m->denoise_output.bias, 22, 16, &s);
  fill(m->vad_output.input_weights, 24, 64, &s);
  fill(m->vad_output.bias, 1, 16, &s);
  return m;
}

static int read_int(FILE *f, int *v) { return fscanf(f, "%d", v) == 1; }

static int read_arr(FILE *f, int8_t *p, size_t n) {
  size_t i;
  int v;
  for (i = 0; i < n; i++) {
    if (!read_int(f, &v)) return 0;
    p[i] = (int8_t)v;
  }
  return 1;
}

static int read_hdr(FILE *f, int *in, int *out, int *act) {
  int a;
  if (!read_int(f, in) || *in < 0 || *in > 128) return 0;
  if (!read_int(f, out) || *out < 0 || *out > 128) return 0;
  if (!read_int(f, &a) || a < 0 || a > 128) return 0;
  *act = (a == 1) ? ORA_ACT_SIGMOID : (a == 2) ? ORA_ACT_RELU : ORA_ACT_TANH;
  return 1;
}

static int read_dense(FILE *f, ora_dense *d) {
  int in, out, act;
  if (!read_hdr(f, &in, &out, &act)) return 0;
  dense_alloc(d, in, out, act);
  return read_arr(f, d->input_weights, (size_t)in * out) && read_arr(f, d->bias, (size_t)out);
}

static int read_gru(FILE *f, ora_gru *g) {
  int in, out, act;
  if (!read_hdr(f, &in, &out, &act)) return 0;
  gru_alloc(g, in, out, act);
  return read_arr(f, g->input_weights, (size_t)in * out * 3) &&
         read_arr(f, g->recurrent_weights, (size_t)out * out * 3) && read_arr(f, g->bias, (size_t)out * 3);
}

ora_model *ora_model_from_text(const char *path) {
  FILE *f = fopen(path, "r");
  ora_model *m;
  int ver;
  if (!f) return NULL;
  if (fscanf(f, "rnnoise-nu model file version %d\n", &ver) != 1 || ver != 1) {
    fclose(f);
    return NULL;
  }
  m = (ora_model *)calloc(1, sizeof(ora_model));
  if (!read_dense(f, &m->input_dense) || !read_gru(f, &m->vad_gru) || !read_gru(f, &m->noise_gru) ||
      !read_gru(f, &m->denoise_gru) || !read_dense(f, &m->denoise_output) || !read_dense(f, &m->vad_output)) {
    fclose(f);
    ora_model_free(m);
    return NULL;
  }
  fclose(f);
  return m;
}

void ora_model_free(ora_model *m) {
  if (!m) return;
  free(m->input_dense.input_weights);
  free(m->input_dense.bias);
  free(m->vad_gru.input_weights);
  free(m->vad_gru.recurrent_weights);
  free(m->vad_gru.bias);
  free(m->noise_gru.input_weights);
  free(m->noise_gru.recurrent_weights);
  free(m->noise_gru.bias);
  free(m->denoise_gru.input_weights);
  free(m->denoise_gru.recurrent_weights);
  free(m->denoise_gru.bias);
  free(m->denoise_output.input_weights);
  free(m->denoise_output.bias);
  free(m->vad_output.input_weights);
  free(m->vad_output.bias);
  free(m);
}

static size_t put(int8_t *blob, size_t off, const int8_t *p, size_t n) {
  if (blob) memcpy(blob + off, p, n);
  return off + n;
}

size_t ora_model_blob(const ora_model *m, int8_t *blob) {
  size_t o = 0;
  const ora_dense *d[3] = {&m->input_dense, &m->denoise_output, &m->vad_output};
  const ora_gru *g[3] = {&m->vad_gru, &m->noise_gru, &m->denoise_gru};
  int i;
  o = put(blob, o, d[0]->input_weights, (size_t)d[0]->nb_inputs * d[0]->nb_neurons);
  o = put(blob, o, d[0]->bias, (size_t)d[0]->nb_neurons);
  for (i = 0; i < 3; i++) {
    const size_t in = g[i]->nb_inputs, n = g[i]->nb_neurons;
    o = put(blob, o, g[i]->input_weights, in * n * 3);
    o = put(blob, o, g[i]->recurrent_weights, n * n * 3);
    o = put(blob, o, g[i]->bias, n * 3);
  }
  for (i = 1; i < 3; i++) {
    o = put(blob, o, d[i]->input_weights, (size_t)d[i]->nb_inputs * d[i]->nb_neurons);
    o = put(blob, o, d[i]->bias, (size_t)d[i]->nb_neurons);
  }
  return o;
}

/* ---------------- CPU baseline (bench.py cpu_baseline leg) ---------------- */
typedef struct {
  const ora_model *m;
  const float *pcm;
  int s0, s1, n_streams, n_channels, n_frames;
  float *vad_out;
} bench_job;

static void *bench_worker(void *arg) {
  bench_job *j = (bench_job *)arg;
  float out[480];
  int s, t, c;
  for (s = j->s0; s < j->s1; s++) {
    ora_denoise *st = ora_rnnoise_create(j->m);
    for (t = 0; t < j->n_frames; t++) {
      float vad_low = 1;
      for (c = 0; c < j->n_channels; c++) {
        const float *in = j->pcm + (((size_t)t * j->n_streams + s) * j->n_channels + c) * 480;
        const float v = ora_rnnoise_process_frame(st, out, in);
        if (v < vad_low) vad_low = v;
      }
      if (j->vad_out) j->vad_out[(size_t)t * j->n_streams + s] = vad_low;
    }
    ora_rnnoise_destroy(st);
  }
  return NULL;
}

double ora_bench_denoise(const ora_model *m, const float *pcm, int n_streams, int n_channels,
                         int n_frames, int n_threads, float *vad_out) {
  pthread_t th[256];
  bench_job jobs[256];
  struct timespec a, b;
  int i;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  if (n_threads > n_streams) n_threads = n_streams;
  ora_tables(NULL, NULL, NULL); /* initialise the lazily built global tables before threading */
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (i = 0; i < n_threads; i++) {
    jobs[i].m = m;
    jobs[i].pcm = pcm;
    jobs[i].s0 = (int)((long)n_streams * i / n_threads);
    jobs[i].s1 = (int)((long)n_streams * (i + 1) / n_threads);
    jobs[i].n_streams = n_streams;
    jobs[i].n_channels = n_channels;
    jobs[i].n_frames = n_frames;
    jobs[i].vad_out = vad_out;
    pthread_create(&th[i], NULL, bench_worker, &jobs[i]);
  }
  for (i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

typedef struct {
  ora_pipeline **pipes;
  const float *pcm;
  int s0, s1, n_channels;
  size_t n_samples, chunk;
} pipe_job;

static void *pipe_worker(void *arg) {
  const pipe_job *j = (const pipe_job *)arg;
  const float *ch[16];
  size_t off, n;
  int s, c;
  for (s = j->s0; s < j->s1; s++) {
    for (off = 0; off < j->n_samples; off += n) {
      n = j->n_samples - off < j->chunk ? j->n_samples - off : j->chunk;
      for (c = 0; c < j->n_channels; c++) ch[c] = j->pcm + ((size_t)s * j->n_channels + c) * j->n_samples + off;
      ora_pipeline_push(j->pipes[s], ch, n);
    }
  }
  return NULL;
}

double ora_bench_pipeline(const ora_model *m, const float *pcm, int n_streams, int n_channels,
                          size_t n_samples, size_t chunk, int n_threads, uint64_t *counts) {
  pthread_t th[256];
  pipe_job jobs[256];
  struct timespec a, b;
  ora_pipeline **pipes;
  ora_vadm_config cfg;
  int i;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  if (n_threads > n_streams) n_threads = n_streams;
  if (n_channels < 1 || n_channels > 16 || chunk == 0) return -1.0;
  ora_tables(NULL, NULL, NULL);
  ora_vadm_config_default(&cfg);
  pipes = (ora_pipeline **)calloc((size_t)n_streams, sizeof(*pipes));
  for (i = 0; i < n_streams; i++) pipes[i] = ora_pipeline_create(n_channels, 48000, 0, 2048, 1, m, &cfg, NULL, 0);
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (i = 0; i < n_threads; i++) {
    jobs[i].pipes = pipes;
    jobs[i].pcm = pcm;
    jobs[i].s0 = (int)((long)n_streams * i / n_threads);
    jobs[i].s1 = (int)((long)n_streams * (i + 1) / n_threads);
    jobs[i].n_channels = n_channels;
    jobs[i].n_samples = n_samples;
    jobs[i].chunk = chunk;
    pthread_create(&th[i], NULL, pipe_worker, &jobs[i]);
  }
  for (i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  for (i = 0; i < n_streams; i++) {
    if (counts && ora_pipeline_denoiser(pipes[i])) ora_rnnoise_counts(ora_pipeline_denoiser(pipes[i]), counts);
    ora_pipeline_destroy(pipes[i]);
  }
  free(pipes);
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
