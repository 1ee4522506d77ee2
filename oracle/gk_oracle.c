/*
 * gk_oracle.c -- C restatement of the reference GKArray, batched over streams.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the MI355X engine and the
 * "port" CPU baseline of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * It follows /root/reference/gkarray/gkarray.py ("gk:N" = line N) with raw
 * values treated as Entry(val, 1, 0), exactly like
 * oracle/gk_oracle.py, and is itself pinned against the golden vectors made
 * from the reference (tests/test_oracle_golden.py).  Streams are independent;
 * they are processed in parallel with OpenMP, each stream strictly in its own
 * insertion order.  Build: make -C oracle  (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  double v;
  int64_t g;
  int64_t d;
} rec_t;

typedef struct {
  int64_t n;
  double mn, mx, sum, avg;
  rec_t* tab;
  int64_t E, cap;
  double* pend;
  int64_t p, pcap;
} stream_t;

typedef struct {
  int64_t S;
  double eps;
  int64_t P;
  stream_t* st;
} gko_set;

static void* xrealloc(void* p, size_t n) {
  void* q = realloc(p, n ? n : 1);
  if (!q) abort();
  return q;
}

gko_set* gko_create(int64_t S, double eps) {
  gko_set* h = (gko_set*)calloc(1, sizeof(gko_set));
  h->S = S;
  h->eps = eps;
  h->P = (int64_t)(1.0 / eps) + 1; /* gk:60 */
  h->st = (stream_t*)calloc((size_t)(S ? S : 1), sizeof(stream_t));
  for (int64_t s = 0; s < S; ++s) {
    h->st[s].mn = INFINITY; /* gk:25 */
    h->st[s].mx = -INFINITY;
  }
  return h;
}

void gko_destroy(gko_set* h) {
  if (!h) return;
  for (int64_t s = 0; s < h->S; ++s) {
    free(h->st[s].tab);
    free(h->st[s].pend);
  }
  free(h->st);
  free(h);
}

/* stable merge sort of records by value (Python's sorted(), gk:72) */
static void msort(rec_t* a, rec_t* tmp, int64_t n) {
  if (n < 2) return;
  const int64_t h = n / 2;
  msort(a, tmp, h);
  msort(a + h, tmp, n - h);
  int64_t i = 0, j = h, k = 0;
  while (i < h && j < n) {
    if (a[j].v < a[i].v) tmp[k++] = a[j++];
    else tmp[k++] = a[i++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, (size_t)n * sizeof(rec_t));
}

/* merge_compress(extra) (gk:63-109) */
static void flush_stream(const gko_set* h, stream_t* s, const rec_t* extra, int64_t nextra) {
  const double T = floor((2.0 * h->eps) * (double)(s->n - 1)); /* gk:70 */
  const int64_t M = s->p + nextra;
  rec_t* inc = (rec_t*)malloc((size_t)(M ? M : 1) * sizeof(rec_t));
  rec_t* tmp = (rec_t*)malloc((size_t)(M ? M : 1) * sizeof(rec_t));
  for (int64_t i = 0; i < s->p; ++i) {
    inc[i].v = s->pend[i];
    inc[i].g = 1;
    inc[i].d = 0;
  }
  for (int64_t i = 0; i < nextra; ++i) inc[s->p + i] = extra[i]; /* gk:71 */
  msort(inc, tmp, M);
  rec_t* E = s->tab;
  const int64_t NE = s->E;
  rec_t* out = (rec_t*)malloc((size_t)(M + NE + 1) * sizeof(rec_t));
  int64_t no = 0, i = 0, j = 0;
  while (i < M || j < NE) {
    if (i == M) { /* gk:77-84 */
      if (j + 1 < NE && (double)(E[j].g + E[j + 1].g + E[j + 1].d) <= T) E[j + 1].g += E[j].g;
      else out[no++] = E[j];
      ++j;
    } else if (j == NE) { /* gk:85-92 */
      if (i + 1 < M && (double)(inc[i].g + inc[i + 1].g + inc[i + 1].d) <= T) inc[i + 1].g += inc[i].g;
      else out[no++] = inc[i];
      ++i;
    } else if (inc[i].v < E[j].v) { /* gk:93-99 */
      if ((double)(inc[i].g + E[j].g + E[j].d) <= T) {
        E[j].g += inc[i].g;
      } else {
        inc[i].d = E[j].g + E[j].d - inc[i].g;
        out[no++] = inc[i];
      }
      ++i;
    } else { /* gk:100-106 */
      if (j + 1 < NE && (double)(E[j].g + E[j + 1].g + E[j + 1].d) <= T) E[j + 1].g += E[j].g;
      else out[no++] = E[j];
      ++j;
    }
  }
  free(s->tab);
  s->tab = out;
  s->E = no;
  s->cap = M + NE + 1;
  s->p = 0;
  free(inc);
  free(tmp);
}

static void add_value(const gko_set* h, stream_t* s, double v) {
  s->n += 1;                                   /* gk:52 */
  s->sum = s->sum + v;                         /* gk:53 */
  s->avg = s->avg + (v - s->avg) * (1.0 / (double)s->n); /* gk:54 */
  if (s->p == s->pcap) {
    s->pcap = s->pcap ? 2 * s->pcap : (h->P + 1);
    s->pend = (double*)xrealloc(s->pend, (size_t)s->pcap * sizeof(double));
  }
  s->pend[s->p++] = v;                         /* gk:55 */
  if (v < s->mn) s->mn = v;                    /* gk:56-57 */
  if (v > s->mx) s->mx = v;                    /* gk:58-59 */
  if (s->n % h->P == 0) flush_stream(h, s, NULL, 0); /* gk:60-61 */
}

int gko_ingest(gko_set* h, const double* values, const int64_t* offs, int nthreads) {
  int64_t s;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (s = 0; s < h->S; ++s) {
    stream_t* st = &h->st[s];
    for (int64_t i = offs[s]; i < offs[s + 1]; ++i) add_value(h, st, values[i]);
  }
  (void)nthreads;
  return 0;
}

/* force 1: merge_compress() if values are pending; force 2: unconditional */
int gko_flush(gko_set* h, int force, int nthreads) {
  int64_t s;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (s = 0; s < h->S; ++s) {
    stream_t* st = &h->st[s];
    if ((force == 1 && st->p > 0) || force == 2) flush_stream(h, st, NULL, 0);
  }
  (void)nthreads;
  return 0;
}

static double percentile_linear(const rec_t* t, int64_t E, double q) {
  /* numpy 2.2.6 percentile, linear method (see oracle/gk_oracle.py) */
  const double qq = (q * 100.0) / 100.0;
  const double vi = (double)(E - 1) * qq;
  double prev, a, b;
  if (vi >= (double)(E - 1)) {
    prev = -1.0;
    a = b = t[E - 1].v;
  } else if (vi < 0.0) {
    prev = 0.0;
    a = b = t[0].v;
  } else {
    prev = floor(vi);
    a = t[(int64_t)prev].v;
    b = t[(int64_t)prev + 1].v;
  }
  const double gamma = vi - prev;
  const double diff = b - a;
  if (gamma >= 0.5) return b - diff * (1.0 - gamma);
  return a + diff * gamma;
}

/* quantiles (gk:187-232).  mode 0: list semantics with sorted qs (leftover ->
 * _max); mode 1: quantile(q) per q (leftover -> entries[-1].val).  The caller
 * flushes first (force 1) as the reference does. */
int gko_quantiles(gko_set* h, const double* qs, int nq, double* out, int mode, int nthreads) {
  int64_t s;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
  for (s = 0; s < h->S; ++s) {
    const stream_t* st = &h->st[s];
    for (int k = 0; k < nq; ++k) {
      const double q = qs[k];
      double r;
      if (st->n == 0 || !(q >= 0.0 && q <= 1.0)) {
        r = NAN;
      } else if ((double)st->n < 1.0 / h->eps) {
        r = percentile_linear(st->tab, st->E, q);
      } else {
        const int64_t rank = (int64_t)(q * (double)(st->n - 1) + 1.0); /* gk:173 */
        const int64_t spread = (int64_t)(h->eps * (double)(st->n - 1)); /* gk:174 */
        int64_t acc = 0, i = 0;
        for (; i < st->E; ++i) {
          acc += st->tab[i].g;
          if (acc + st->tab[i].d - 1 > rank + spread) break;
        }
        if (i == 0) r = st->mn;
        else if (i < st->E) r = st->tab[i - 1].v;
        else r = (mode == 0) ? st->mx : st->tab[st->E - 1].v;
      }
      out[s * nq + k] = r;
    }
  }
  (void)nthreads;
  return 0;
}

/* dst.merge(src) stream by stream (gk:111-154); src is flushed (mutated) */
int gko_merge(gko_set* dst, gko_set* src, int nthreads) {
  if (dst->eps != src->eps) return -2; /* gk:118-119 */
  if (dst->S != src->S) return -1;
  int64_t s;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (s = 0; s < dst->S; ++s) {
    stream_t* a = &dst->st[s];
    stream_t* b = &src->st[s];
    if (b->n == 0) { /* gk:121-123 */
      flush_stream(dst, a, NULL, 0);
      continue;
    }
    if (a->n == 0) { /* gk:125-133 */
      flush_stream(src, b, NULL, 0);
      free(a->tab);
      a->tab = (rec_t*)malloc((size_t)(b->E ? b->E : 1) * sizeof(rec_t));
      memcpy(a->tab, b->tab, (size_t)b->E * sizeof(rec_t));
      a->E = b->E;
      a->cap = b->E;
      a->mn = b->mn;
      a->mx = b->mx;
      a->n = b->n;
      a->sum = b->sum;
      a->avg = b->avg;
      continue;
    }
    const int64_t spread = (int64_t)(src->eps * (double)(b->n - 1)); /* gk:136 */
    flush_stream(src, b, NULL, 0);                                  /* gk:137 */
    const int64_t L = b->E;
    rec_t* conv = (rec_t*)malloc((size_t)(L + 1) * sizeof(rec_t));
    int64_t nc = 0;
    int64_t gv = b->tab[0].g + b->tab[0].d - spread - 1; /* gk:138-140 */
    if (gv > 0) {
      conv[nc].v = b->mn; conv[nc].g = gv; conv[nc].d = 0; ++nc;
    }
    for (int64_t i = 0; i + 1 < L; ++i) { /* gk:141-144 */
      gv = b->tab[i + 1].g + b->tab[i + 1].d - b->tab[i].d;
      if (gv > 0) {
        conv[nc].v = b->tab[i].v; conv[nc].g = gv; conv[nc].d = 0; ++nc;
      }
    }
    gv = spread + 1 - b->tab[L - 1].d; /* gk:145-147 */
    if (gv > 0) {
      conv[nc].v = b->tab[L - 1].v; conv[nc].g = gv; conv[nc].d = 0; ++nc;
    }
    a->n += b->n; /* gk:149 */
    if (b->mn < a->mn) a->mn = b->mn; /* gk:151 */
    if (b->mx > a->mx) a->mx = b->mx; /* gk:152 */
    flush_stream(dst, a, conv, nc); /* gk:154 */
    free(conv);
  }
  (void)nthreads;
  return 0;
}

void gko_stats(const gko_set* h, int64_t* n, double* mn, double* mx, double* sum, double* avg,
               int32_t* E, int32_t* p) {
  for (int64_t s = 0; s < h->S; ++s) {
    const stream_t* st = &h->st[s];
    if (n) n[s] = st->n;
    if (mn) mn[s] = st->mn;
    if (mx) mx[s] = st->mx;
    if (sum) sum[s] = st->sum;
    if (avg) avg[s] = st->avg;
    if (E) E[s] = (int32_t)st->E;
    if (p) p[s] = (int32_t)st->p;
  }
}

/* tables in CSR: offs[S+1] must be the exclusive scan of E (gko_stats) */
void gko_export(const gko_set* h, const int64_t* offs, double* v, int64_t* g, int64_t* d) {
  for (int64_t s = 0; s < h->S; ++s) {
    const stream_t* st = &h->st[s];
    for (int64_t j = 0; j < st->E; ++j) {
      v[offs[s] + j] = st->tab[j].v;
      g[offs[s] + j] = st->tab[j].g;
      d[offs[s] + j] = st->tab[j].d;
    }
  }
}

void gko_export_pending(const gko_set* h, const int64_t* offs, double* v) {
  for (int64_t s = 0; s < h->S; ++s) {
    const stream_t* st = &h->st[s];
    for (int64_t j = 0; j < st->p; ++j) v[offs[s] + j] = st->pend[j];
  }
}

int gko_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
