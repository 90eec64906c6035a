/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of the Evaluator (segment matching + duration statistics):
 *   Evaluator.initAndRun            (src/Evaluator.zig:90-156)
 *   SpeechSegment overlap / sort    (src/Evaluator/SpeechSegment.zig:14-56)
 *   statistics.fromEvaluator etc.   (src/Evaluator/statistics.zig:85-284)
 *   formats.parseAudacitySegments   (src/Evaluator/formats.zig:7-36)
 * All arithmetic is f32 as in the reference.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

typedef struct {
  float from, to;
  size_t *opp; /* indices into the opposite list */
  size_t n_opp;
} seg;

static float overlap_with(float af, float at, float bf, float bt) {
  const float max_from = af > bf ? af : bf;
  const float min_to = at < bt ? at : bt;
  return min_to - max_from;
}

/* stable insertion sort by from_sec (SpeechSegment.sortByStart, std.mem.sort) */
static void sort_by_start(seg *s, size_t n) {
  size_t i, j;
  for (i = 1; i < n; i++) {
    seg t = s[i];
    j = i;
    while (j > 0 && s[j - 1].from > t.from) {
      s[j] = s[j - 1];
      j--;
    }
    s[j] = t;
  }
}

static void find_overlapping(seg *target, const seg *others, size_t n_others) {
  size_t i, k = 0;
  target->opp = (size_t *)malloc(sizeof(size_t) * (n_others ? n_others : 1));
  for (i = 0; i < n_others; i++)
    if (overlap_with(target->from, target->to, others[i].from, others[i].to) > 0.0f) target->opp[k++] = i;
  target->n_opp = k;
}

static float calc_fp(float vf, float vt, const float *rf, const float *rt, size_t n,
                     const ora_stat_config *cfg) {
  /* extrudeSegments (statistics.zig:191-218) then calcOverlapMany */
  float *f = (float *)malloc(sizeof(float) * (n ? n : 1));
  float *t = (float *)malloc(sizeof(float) * (n ? n : 1));
  float overlap = 0.0f;
  size_t i;
  for (i = 0; i < n; i++) {
    f[i] = rf[i];
    t[i] = rt[i];
  }
  if (n > 0) {
    f[0] -= cfg->extrude_start;
    t[n - 1] += cfg->extrude_end;
    for (i = 0; i + 1 < n; i++)
      if (f[i + 1] - t[i] <= cfg->fill_gaps) t[i] = f[i + 1];
  }
  for (i = 0; i < n; i++) {
    const float o = overlap_with(vf, vt, f[i], t[i]);
    overlap += (0.0f > o) ? 0.0f : o;
  }
  free(f);
  free(t);
  return (vt - vf) - overlap;
}

float ora_calc_false_positive_sec(float vf, float vt, const float *ref, size_t n,
                                  const ora_stat_config *cfg) {
  float *rf = (float *)malloc(sizeof(float) * (n ? n : 1));
  float *rt = (float *)malloc(sizeof(float) * (n ? n : 1));
  float r;
  size_t i;
  for (i = 0; i < n; i++) {
    rf[i] = ref[2 * i];
    rt[i] = ref[2 * i + 1];
  }
  r = calc_fp(vf, vt, rf, rt, n, cfg);
  free(rf);
  free(rt);
  return r;
}

static float f_score(float beta, float precision, float recall) {
  const float b2 = beta * beta;
  return (1 + b2) * (precision * recall) / (b2 * precision + recall);
}

int ora_evaluate(const float *vad, size_t nv, const float *ref, size_t nr, const ora_stat_config *cfg,
                 ora_single_stats *out) {
  seg *vs = (seg *)calloc(nv ? nv : 1, sizeof(seg));
  seg *rs = (seg *)calloc(nr ? nr : 1, sizeof(seg));
  size_t i, k;
  ora_single_stats s;
  memset(&s, 0, sizeof(s));
  for (i = 0; i < nv; i++) {
    vs[i].from = vad[2 * i];
    vs[i].to = vad[2 * i + 1];
  }
  for (i = 0; i < nr; i++) {
    rs[i].from = ref[2 * i];
    rs[i].to = ref[2 * i + 1];
  }
  sort_by_start(vs, nv);
  sort_by_start(rs, nr);
  for (i = 0; i < nv; i++) find_overlapping(&vs[i], rs, nr);
  for (i = 0; i < nr; i++) find_overlapping(&rs[i], vs, nv);
  for (i = 0; i < nv; i++) {
    float *rf = (float *)malloc(sizeof(float) * (vs[i].n_opp ? vs[i].n_opp : 1));
    float *rt = (float *)malloc(sizeof(float) * (vs[i].n_opp ? vs[i].n_opp : 1));
    float fp, tp;
    for (k = 0; k < vs[i].n_opp; k++) {
      rf[k] = rs[vs[i].opp[k]].from;
      rt[k] = rs[vs[i].opp[k]].to;
    }
    fp = calc_fp(vs[i].from, vs[i].to, rf, rt, vs[i].n_opp, cfg);
    s.false_positives_sec += fp;
    tp = (vs[i].to - vs[i].from) - calc_fp(vs[i].from, vs[i].to, rf, rt, vs[i].n_opp, cfg);
    s.true_positives_sec += tp;
    s.total_positives_sec += tp;
    free(rf);
    free(rt);
  }
  for (i = 0; i < nr; i++) {
    float ov = 0.0f, fn;
    if ((rs[i].to - rs[i].from) < cfg->ignore_shorter_than_sec) continue;
    for (k = 0; k < rs[i].n_opp; k++) {
      const float o = overlap_with(rs[i].from, rs[i].to, vs[rs[i].opp[k]].from, vs[rs[i].opp[k]].to);
      ov += (0.0f > o) ? 0.0f : o;
    }
    fn = (rs[i].to - rs[i].from) - ov;
    s.false_negatives_sec += fn;
    s.total_positives_sec += fn;
  }
  s.true_positive_rate = s.true_positives_sec / s.total_positives_sec;
  s.false_negative_rate = s.false_negatives_sec / s.total_positives_sec;
  s.false_discovery_rate = s.false_positives_sec / (s.false_positives_sec + s.true_positives_sec);
  s.precision = s.true_positives_sec / (s.true_positives_sec + s.false_positives_sec);
  s.f_score_beta = 0.7f;
  s.f_score = f_score(s.f_score_beta, s.precision, s.true_positive_rate);
  s.fm_index = sqrtf(s.precision * s.true_positive_rate);
  *out = s;
  for (i = 0; i < nv; i++) free(vs[i].opp);
  for (i = 0; i < nr; i++) free(rs[i].opp);
  free(vs);
  free(rs);
  return 0;
}

void ora_aggregate(const ora_single_stats *st, size_t n, ora_aggregate_stats *a) {
  float s_tpr = 0, s_fnr = 0, s_fdr = 0, s_p = 0;
  size_t i;
  const float nf = (float)n;
  memset(a, 0, sizeof(*a));
  a->true_positive_rate.min = a->false_negative_rate.min = a->false_discovery_rate.min = a->precision.min = 2;
  a->true_positive_rate.max = a->false_negative_rate.max = a->false_discovery_rate.max = a->precision.max = -2;
  for (i = 0; i < n; i++) {
    const ora_single_stats *s = &st[i];
    a->total_positives_sec += s->total_positives_sec;
    a->true_positives_sec += s->true_positives_sec;
    a->false_positives_sec += s->false_positives_sec;
    a->false_negatives_sec += s->false_negatives_sec;
    s_tpr += s->true_positive_rate;
    if (s->true_positive_rate < a->true_positive_rate.min) a->true_positive_rate.min = s->true_positive_rate;
    if (s->true_positive_rate > a->true_positive_rate.max) a->true_positive_rate.max = s->true_positive_rate;
    s_fnr += s->false_negative_rate;
    if (s->false_negative_rate < a->false_negative_rate.min) a->false_negative_rate.min = s->false_negative_rate;
    if (s->false_negative_rate > a->false_negative_rate.max) a->false_negative_rate.max = s->false_negative_rate;
    s_fdr += s->false_discovery_rate;
    if (s->false_discovery_rate < a->false_discovery_rate.min) a->false_discovery_rate.min = s->false_discovery_rate;
    if (s->false_discovery_rate > a->false_discovery_rate.max) a->false_discovery_rate.max = s->false_discovery_rate;
    s_p += s->precision;
    if (s->precision < a->precision.min) a->precision.min = s->precision;
    if (s->precision > a->precision.max) a->precision.max = s->precision;
  }
  a->true_positive_rate.overall = a->true_positives_sec / a->total_positives_sec;
  a->false_negative_rate.overall = a->false_negatives_sec / a->total_positives_sec;
  a->false_discovery_rate.overall = a->false_positives_sec / (a->false_positives_sec + a->true_positives_sec);
  a->precision.overall = a->true_positives_sec / (a->true_positives_sec + a->false_positives_sec);
  a->true_positive_rate.avg = s_tpr / nf;
  a->false_negative_rate.avg = s_fnr / nf;
  a->false_discovery_rate.avg = s_fdr / nf;
  a->precision.avg = s_p / nf;
  a->f_score_beta = 0.7f;
  a->f_score = f_score(a->f_score_beta, a->precision.overall, a->true_positive_rate.overall);
  a->fm_index = sqrtf(a->precision.overall * a->true_positive_rate.overall);
}

long ora_parse_audacity(const char *txt, size_t len, float *out, size_t cap) {
  size_t pos = 0;
  long n = 0;
  while (pos <= len) {
    size_t e = pos, tab1, tab2;
    char buf[128];
    char *endp;
    float from, to;
    while (e < len && txt[e] != '\n') e++;
    /* fields split on '\t' of the (un-CR-stripped) line [pos, e) */
    tab1 = pos;
    while (tab1 < e && txt[tab1] != '\t') tab1++;
    if (tab1 < e) {
      size_t l1 = tab1 - pos, l2;
      tab2 = tab1 + 1;
      while (tab2 < e && txt[tab2] != '\t') tab2++;
      l2 = tab2 - (tab1 + 1);
      if (l1 >= sizeof(buf) || l2 >= sizeof(buf)) return -1;
      memcpy(buf, txt + pos, l1);
      buf[l1] = 0;
      from = strtof(buf, &endp);
      if (l1 == 0 || *endp) return -1; /* std.fmt.parseFloat error */
      memcpy(buf, txt + tab1 + 1, l2);
      buf[l2] = 0;
      to = strtof(buf, &endp);
      if (l2 == 0 || *endp) return -1;
      if ((size_t)n < cap) {
        out[2 * n] = from;
        out[2 * n + 1] = to;
      }
      n++;
    }
    pos = e + 1;
  }
  return n;
}
