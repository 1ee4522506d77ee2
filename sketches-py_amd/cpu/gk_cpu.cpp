// gk_cpu.cpp -- the host (CPU) engine of the batched GKArray: every entry
// point of include/gk_capi.h on host memory (include/gk_cpu.h), streams in
// parallel on host threads, each stream strictly in insertion order.
//
// Reference: githomin/sketches-py gkarray/gkarray.py ("gk:N" = line N).  It is
// an independent implementation (not the test oracle): the add-driven flush
// uses the closed form of the four-rule walk (SURVEY.md 3.2 -- gap counts
// against the old table, one integer carry per entry), merges use the
// general walk (gk:76-106).  Built with -ffp-contract=off, no fast-math: the
// reference's float64 expressions (gk:54, gk:70, numpy's linear percentile)
// are evaluated exactly as written.
#include <math.h>
#include <sched.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <limits>
#include <string>
#include <thread>

#include "gk_host_stats.h"
#include <vector>

#include "gk_cpu.h"
#include "gk_format.h"
#include "gk_pack.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// one (v, g, delta) tuple of a table (gk:8-16)
struct Rec {
  double v;
  int64_t g;
  int64_t d;
};

struct Stream {
  int64_t n = 0;                                        // _n (gk:27)
  double mn = std::numeric_limits<double>::infinity();  // _min (gk:25)
  double mx = -std::numeric_limits<double>::infinity(); // _max (gk:26)
  double sum = 0.0, avg = 0.0;                          // _sum, _avg (gk:28-29)
  std::vector<Rec> tab;                                 // entries (gk:23)
  std::vector<double> pend;                             // incoming (gk:24)
};

int default_threads() {
  if (const char* e = getenv("GK_CPU_THREADS")) {
    const int t = atoi(e);
    if (t > 0) return t;
  }
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) {
    const int n = CPU_COUNT(&cs);
    if (n > 0) return n;
  }
  const unsigned hc = std::thread::hardware_concurrency();
  return hc ? (int)hc : 1;
}

// Run fn(s) for s in [0, S): dynamic chunks of streams over `threads` threads.
template <typename F>
void parallel_for(int64_t S, int threads, F&& fn) {
  constexpr int64_t kChunk = 64;
  const int64_t chunks = (S + kChunk - 1) / kChunk;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, chunks));
  if (T <= 1) {
    for (int64_t s = 0; s < S; ++s) fn(s);
    return;
  }
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      const int64_t c = next.fetch_add(1, std::memory_order_relaxed);
      if (c >= chunks) break;
      const int64_t e = std::min(S, (c + 1) * kChunk);
      for (int64_t s = c * kChunk; s < e; ++s) fn(s);
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(T - 1);
  for (int t = 1; t < T; ++t) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
}

}  // namespace

struct gk_set {
  int64_t S = 0;
  double eps = 0;
  int64_t P = 0;  // int(1.0/eps) + 1 (gk:60)
  int threads = 1;
  std::vector<Stream> st;
  bool timing = false;
  double ingest_ms = 0;
  int64_t launches = 0;
  gk_set* fold_scratch = nullptr;  // gk_fold_packed (made on first use)
};

namespace {

// ---- float64 control arithmetic, exactly the reference's expressions -------
int64_t threshold(const gk_set* h, int64_t n) {
  return (int64_t)floor(2.0 * h->eps * (double)(n - 1));  // gk:70: (2.0*eps)*(n-1)
}

// gk:52-59 for one value
inline void add_stats(Stream& s, double v) { gk_host_stat_step(s.n, s.sum, s.avg, s.mn, s.mx, v); }

// Stable order of the pending values by value (gk:71-72: Python's sorted();
// -0.0 == +0.0, so equal keys keep insertion order): sorted by (value,
// insertion index), which is the stable order, with no allocation.
struct Keyed {
  double v;
  uint32_t i;
};
inline bool keyed_less(const Keyed& a, const Keyed& b) { return a.v < b.v || (!(b.v < a.v) && a.i < b.i); }

void sorted_pending(const std::vector<double>& pend, std::vector<Keyed>& key, std::vector<double>& out) {
  const size_t n = pend.size();
  out.resize(n);
  if (n <= 24) {  // insertion sort is stable
    for (size_t i = 0; i < n; ++i) {
      const double x = pend[i];
      size_t j = i;
      while (j > 0 && x < out[j - 1]) {
        out[j] = out[j - 1];
        --j;
      }
      out[j] = x;
    }
    return;
  }
  key.resize(n);
  for (size_t i = 0; i < n; ++i) key[i] = Keyed{pend[i], (uint32_t)i};
  std::sort(key.begin(), key.end(), keyed_less);
  for (size_t i = 0; i < n; ++i) out[i] = key[i].v;
}

// merge_compress() of an add-driven flush (gk:63-109 with every incoming record
// (x, 1, 0)), in closed form: entry j, with carry c from a removed
// predecessor, absorbs the k = clamp(T - d_j - (g_j + c), 0, m_j) smallest of
// the m_j values of its gap [v_{j-1}, v_j) (gk:93-95); the others are kept as
// (x, 1, G + d_j - 1), G = g_j + c + k (gk:96-98); entry j is removed into j+1
// iff G + g_{j+1} + d_{j+1} <= T (gk:100-103), else kept as (v_j, G, d_j).  The
// values past the last entry chain in runs of max(T, 1) (gk:85-92).
void flush_add(Stream& s, int64_t T, std::vector<Keyed>& key, std::vector<double>& xs, std::vector<Rec>& out) {
  sorted_pending(s.pend, key, xs);
  const std::vector<Rec>& E = s.tab;
  const size_t ne = E.size(), nx = xs.size();
  out.clear();
  out.reserve(ne + nx);
  size_t i = 0;
  int64_t carry = 0;
  for (size_t j = 0; j < ne; ++j) {
    const double vj = E[j].v;
    size_t m = 0;
    while (i + m < nx && xs[i + m] < vj) ++m;  // gk:93: strict, ties go after the entry
    const int64_t Gp = E[j].g + carry;
    const int64_t k = std::min<int64_t>((int64_t)m, std::max<int64_t>(0, T - E[j].d - Gp));
    const int64_t G = Gp + k;
    for (size_t t = i + (size_t)k; t < i + m; ++t) out.push_back(Rec{xs[t], 1, G + E[j].d - 1});
    i += m;
    if (j + 1 < ne && G + E[j + 1].g + E[j + 1].d <= T) {
      carry = G;
    } else {
      out.push_back(Rec{vj, G, E[j].d});
      carry = 0;
    }
  }
  int64_t c = 0;
  for (; i < nx; ++i) {
    c += 1;
    if (i + 1 == nx || c + 1 > T) {
      out.push_back(Rec{xs[i], c, 0});
      c = 0;
    }
  }
  s.tab.swap(out);
  s.pend.clear();
}

// merge_compress(entries) with explicit records (gk:63-109): the general
// four-rule walk over the stable order of incoming (pending values as
// (x, 1, 0), then the records, gk:71) and the table.
void flush_general(Stream& s, int64_t T, const Rec* recs, size_t nrec, std::vector<Keyed>& key, std::vector<Rec>& inc,
                   std::vector<Rec>& out) {
  // incoming = pending (x, 1, 0) + records, in that order (gk:71), stably sorted
  const size_t np = s.pend.size(), ntot = np + nrec;
  key.resize(ntot);
  for (size_t i = 0; i < ntot; ++i) key[i] = Keyed{i < np ? s.pend[i] : recs[i - np].v, (uint32_t)i};
  std::sort(key.begin(), key.end(), keyed_less);
  inc.resize(ntot);
  for (size_t k = 0; k < ntot; ++k) {
    const uint32_t i = key[k].i;
    inc[k] = i < np ? Rec{s.pend[i], 1, 0} : recs[i - np];
  }
  std::vector<Rec>& E = s.tab;
  const size_t ni = inc.size(), ne = E.size();
  out.clear();
  out.reserve(ni + ne);
  size_t i = 0, j = 0;
  while (i < ni || j < ne) {
    if (i == ni || (j < ne && !(inc[i].v < E[j].v))) {  // gk:77-84, gk:100-106
      if (j + 1 < ne && E[j].g + E[j + 1].g + E[j + 1].d <= T) E[j + 1].g += E[j].g;
      else out.push_back(E[j]);
      ++j;
    } else if (j == ne) {  // gk:85-92
      if (i + 1 < ni && inc[i].g + inc[i + 1].g + inc[i + 1].d <= T) inc[i + 1].g += inc[i].g;
      else out.push_back(inc[i]);
      ++i;
    } else {  // gk:93-99: inc[i].v < E[j].v
      if (inc[i].g + E[j].g + E[j].d <= T) {
        E[j].g += inc[i].g;
      } else {
        Rec r = inc[i];
        r.d = E[j].g + E[j].d - r.g;
        out.push_back(r);
      }
      ++i;
    }
  }
  s.tab.swap(out);
  s.pend.clear();
}

struct Scratch {
  std::vector<Keyed> key;
  std::vector<double> xs;
  std::vector<Rec> out, inc;
};
thread_local Scratch tl_scratch;

// GKArray.add for a run of values (gk:49-61): a flush whenever n reaches a
// multiple of P (counted down instead of a modulo per value).
void ingest_stream(const gk_set* h, Stream& s, const double* x, int64_t L) {
  Scratch& sc = tl_scratch;
  int64_t k = 0;
  while (k < L) {
    const int64_t need = h->P - s.n % h->P;  // adds until the next flush point (gk:60)
    const int64_t take = std::min(need, L - k);
    for (int64_t t = 0; t < take; ++t) {
      const double v = x[k + t];
      add_stats(s, v);
      s.pend.push_back(v);
    }
    k += take;
    if (take == need) flush_add(s, threshold(h, s.n), sc.key, sc.xs, sc.out);
  }
}

// merge_compress() where values are pending (size/quantile, gk:45-46, 166, 197)
void flush_if_pending(const gk_set* h, Stream& s) {
  if (!s.pend.empty()) flush_add(s, threshold(h, s.n), tl_scratch.key, tl_scratch.xs, tl_scratch.out);
}

// numpy 2.2.6 percentile(values, q*100), method 'linear' (gk:171, gk:202):
// q/100 (np:4257), virtual index (n-1)*q (np:107), bounds (np:4748-4750),
// gamma (np:4632), _lerp with its gamma >= 0.5 branch (np:4653-4657)
double percentile_linear(const std::vector<Rec>& E, double q) {
  const int64_t n = (int64_t)E.size();
  const double qq = (q * 100.0) / 100.0;
  const double vi = (double)(n - 1) * qq;
  double prev, a, b;
  if (vi >= (double)(n - 1)) {
    prev = -1.0;
    a = b = E[n - 1].v;
  } else if (vi < 0.0) {
    prev = 0.0;
    a = b = E[0].v;
  } else {
    prev = floor(vi);
    const int64_t pi = (int64_t)prev;
    a = E[pi].v;
    b = E[pi + 1].v;
  }
  const double gamma = vi - prev;
  const double diff = b - a;
  if (gamma >= 0.5) return b - diff * (1.0 - gamma);
  return a + diff * gamma;
}

double nan_value() { return std::numeric_limits<double>::quiet_NaN(); }

// GKArray.quantile(q) (gk:156-185) after the flush
double quantile_one(const gk_set* h, const Stream& s, double q) {
  if (q < 0 || q > 1 || s.n == 0) return nan_value();
  if ((double)s.n < 1.0 / h->eps) return percentile_linear(s.tab, q);
  const int64_t rank = (int64_t)(q * (double)(s.n - 1) + 1);  // gk:173
  const int64_t spread = (int64_t)(h->eps * (double)(s.n - 1));  // gk:174
  double g_sum = 0.0;
  size_t i = 0;
  for (; i < s.tab.size(); ++i) {
    g_sum += (double)s.tab[i].g;
    if (g_sum + (double)s.tab[i].d - 1 > (double)(rank + spread)) break;
  }
  if (i == 0) return s.mn;
  return s.tab[i - 1].v;
}

// GKArray.quantiles(qs) (gk:187-232) after the flush, qs sorted
void quantiles_list(const gk_set* h, const Stream& s, const double* qs, int nq, double* out) {
  if (s.n == 0) {
    for (int k = 0; k < nq; ++k) out[k] = nan_value();
    return;
  }
  if ((double)s.n < 1.0 / h->eps) {  // gk:200-202
    for (int k = 0; k < nq; ++k) out[k] = (qs[k] >= 0 && qs[k] <= 1) ? percentile_linear(s.tab, qs[k]) : nan_value();
    return;
  }
  const int64_t spread = (int64_t)(h->eps * (double)(s.n - 1));  // gk:210
  double g_sum = 0.0;
  size_t i = 0;
  int j = 0;
  while (i < s.tab.size() && j < nq) {  // gk:213-224
    g_sum += (double)s.tab[i].g;
    while (j < nq) {
      if (qs[j] < 0 || qs[j] > 1) {
        out[j++] = nan_value();
      } else if (g_sum + (double)s.tab[i].d - 1 > (double)((int64_t)(qs[j] * (double)(s.n - 1) + 1) + spread)) {
        out[j++] = i == 0 ? s.mn : s.tab[i - 1].v;
      } else {
        break;
      }
    }
    ++i;
  }
  for (; j < nq; ++j) out[j] = (qs[j] < 0 || qs[j] > 1) ? nan_value() : s.mx;  // gk:225-230
}

int check_set(const gk_set* h) {
  if (!h) return fail(GK_E_ARG, "null set");
  return GK_OK;
}

int check_query(const double* qs, int nq, double* out, int mode) {
  if (nq < 0 || (nq > 0 && (!qs || !out))) return fail(GK_E_ARG, "bad quantile arguments");
  if (mode != GK_Q_LIST && mode != GK_Q_SINGLE) return fail(GK_E_ARG, "bad mode %d", mode);
  for (int i = 0; i < nq; ++i)
    if (std::isnan(qs[i])) return fail(GK_E_ARG, "cannot convert float NaN to integer");
  return GK_OK;
}

// gk:205: an unsorted list is answered q by q with quantile()
int effective_mode(const double* qs, int nq, int mode) {
  if (mode == GK_Q_LIST)
    for (int i = 1; i < nq; ++i)
      if (qs[i] < qs[i - 1]) return GK_Q_SINGLE;
  return mode;
}

void answer(const gk_set* h, const Stream& s, const double* qs, int nq, int mode, double* out) {
  if (mode == GK_Q_SINGLE) {
    for (int k = 0; k < nq; ++k) out[k] = quantile_one(h, s, qs[k]);
  } else {
    quantiles_list(h, s, qs, nq, out);
  }
}

int ingest_impl(gk_set* h, const double* values, const int64_t* offsets, const double* qs, int nq, double* out,
                int mode) {
  if (!offsets) return fail(GK_E_ARG, "offsets is null");
  if (!values) return fail(GK_E_ARG, "values is null");
  for (int64_t s = 0; s < h->S; ++s)
    if (offsets[s + 1] < offsets[s]) return fail(GK_E_ARG, "offsets must be non-decreasing");
  const auto t0 = std::chrono::steady_clock::now();
  parallel_for(h->S, h->threads, [&](int64_t s) {
    Stream& st = h->st[s];
    ingest_stream(h, st, values + offsets[s], offsets[s + 1] - offsets[s]);
    if (qs) {
      if (nq > 0 && st.n > 0) flush_if_pending(h, st);  // gk:166-167 / gk:197-198
      answer(h, st, qs, nq, mode, out + s * (int64_t)nq);
    }
  });
  if (h->timing) {
    h->ingest_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    h->launches += 1;
  }
  return GK_OK;
}

// GKArray.merge(other) (gk:111-154) for one stream
void merge_stream(const gk_set* h, Stream& a, Stream& b, std::vector<Rec>& conv) {
  Scratch& sc = tl_scratch;
  if (b.n == 0) {  // gk:121-123: unconditional flush of self
    flush_general(a, threshold(h, a.n), nullptr, 0, sc.key, sc.inc, sc.out);
    return;
  }
  if (a.n == 0) {  // gk:125-133: other flushed, self takes a copy of its state
    flush_general(b, threshold(h, b.n), nullptr, 0, sc.key, sc.inc, sc.out);
    a.tab = b.tab;
    a.mn = b.mn;
    a.mx = b.mx;
    a.n = b.n;
    a.sum = b.sum;
    a.avg = b.avg;
    return;
  }
  const int64_t spread = (int64_t)(h->eps * (double)(b.n - 1));  // gk:136 (before the flush)
  flush_general(b, threshold(h, b.n), nullptr, 0, sc.key, sc.inc, sc.out);  // gk:137
  conv.clear();
  const std::vector<Rec>& E = b.tab;
  const size_t L = E.size();
  int64_t g = E[0].g + E[0].d - spread - 1;  // gk:138-140
  if (g > 0) conv.push_back(Rec{b.mn, g, 0});
  for (size_t i = 0; i + 1 < L; ++i) {  // gk:141-144
    g = E[i + 1].g + E[i + 1].d - E[i].d;
    if (g > 0) conv.push_back(Rec{E[i].v, g, 0});
  }
  g = spread + 1 - E[L - 1].d;  // gk:145-147
  if (g > 0) conv.push_back(Rec{E[L - 1].v, g, 0});
  a.n += b.n;                    // gk:149 (_sum/_avg are not merged)
  if (b.mn < a.mn) a.mn = b.mn;  // gk:151: Python min() keeps the first on ties
  if (b.mx > a.mx) a.mx = b.mx;  // gk:152
  flush_general(a, threshold(h, a.n), conv.data(), conv.size(), sc.key, sc.inc, sc.out);  // gk:154
}

}  // namespace

extern "C" {

int gk_version(void) { return 100; }

const char* gk_last_error(void) { return g_err.c_str(); }

int gk_create(int64_t num_streams, double eps, int64_t cap_hint, int device, gk_set** out) {
  (void)cap_hint;
  (void)device;
  if (!out) return fail(GK_E_ARG, "out is null");
  *out = nullptr;
  if (num_streams < 0 || num_streams > INT32_MAX) return fail(GK_E_ARG, "num_streams out of range");
  // any finite eps > 0, as the reference (gk:21); eps > 1 gives P = 1 (gk:60)
  if (!std::isfinite(eps) || !(eps > 0.0)) return fail(GK_E_ARG, "eps must be finite and > 0");
  const double inv = 1.0 / eps;
  if (inv >= 9.0e18) return fail(GK_E_UNSUPPORTED, "eps=%g: flush period beyond int64", eps);
  gk_set* h = new (std::nothrow) gk_set();
  if (!h) return fail(GK_E_NOMEM, "set allocation failed");
  h->S = num_streams;
  h->eps = eps;
  h->P = (int64_t)inv + 1;  // gk:60
  h->threads = default_threads();
  try {
    h->st.resize((size_t)num_streams);
  } catch (...) {
    delete h;
    return fail(GK_E_NOMEM, "state for %lld streams failed", (long long)num_streams);
  }
  *out = h;
  return GK_OK;
}

int gk_destroy(gk_set* h) {
  if (h && h->fold_scratch) gk_destroy(h->fold_scratch);
  delete h;
  return GK_OK;
}

int gk_cpu_set_threads(gk_set* h, int threads) {
  int rc = check_set(h);
  if (rc) return rc;
  if (threads < 0) return fail(GK_E_ARG, "threads must be >= 0");
  h->threads = threads ? threads : default_threads();
  return GK_OK;
}

int gk_cpu_threads(const gk_set* h) { return h ? h->threads : -1; }

int gk_reset(gk_set* h, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  parallel_for(h->S, h->threads, [&](int64_t s) { h->st[s] = Stream(); });
  return GK_OK;
}

int gk_ingest(gk_set* h, const double* values, const int64_t* offsets, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  return ingest_impl(h, values, offsets, nullptr, 0, nullptr, GK_Q_LIST);
}

int gk_flush(gk_set* h, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  parallel_for(h->S, h->threads, [&](int64_t s) { flush_if_pending(h, h->st[s]); });
  return GK_OK;
}

int gk_sync(gk_set* h, void* stream) {
  (void)stream;
  return check_set(h);
}

int gk_quantiles(gk_set* h, const double* qs, int nq, double* out, int mode, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (!rc) rc = check_query(qs, nq, out, mode);
  if (rc) return rc;
  if (nq == 0) return GK_OK;
  mode = effective_mode(qs, nq, mode);
  parallel_for(h->S, h->threads, [&](int64_t s) {
    Stream& st = h->st[s];
    if (st.n > 0) flush_if_pending(h, st);
    answer(h, st, qs, nq, mode, out + s * (int64_t)nq);
  });
  return GK_OK;
}

int gk_ingest_quantiles(gk_set* h, const double* values, const int64_t* offsets, const double* qs, int nq,
                        double* out, int mode, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (!rc) rc = check_query(qs, nq, out, mode);
  if (rc) return rc;
  if (nq == 0) return ingest_impl(h, values, offsets, nullptr, 0, nullptr, mode);
  return ingest_impl(h, values, offsets, qs, nq, out, effective_mode(qs, nq, mode));
}

int gk_stats(gk_set* h, int64_t* n, double* mn, double* mx, double* sum, double* avg, int32_t* table_size,
             int32_t* pending, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  for (int64_t s = 0; s < h->S; ++s) {
    const Stream& st = h->st[s];
    if (n) n[s] = st.n;
    if (mn) mn[s] = st.mn;
    if (mx) mx[s] = st.mx;
    if (sum) sum[s] = st.sum;
    if (avg) avg[s] = st.avg;
    if (table_size) table_size[s] = (int32_t)st.tab.size();
    if (pending) pending[s] = (int32_t)st.pend.size();
  }
  return GK_OK;
}

int gk_merge(gk_set* dst, gk_set* const* srcs, int nsrcs, void* stream) {
  (void)stream;
  int rc = check_set(dst);
  if (rc) return rc;
  if (nsrcs < 0 || (nsrcs > 0 && !srcs)) return fail(GK_E_ARG, "bad source list");
  for (int k = 0; k < nsrcs; ++k) {
    if (!srcs[k]) return fail(GK_E_ARG, "null source %d", k);
    if (srcs[k]->eps != dst->eps)  // gk:118-119
      return fail(GK_E_EPS_MISMATCH, "Cannot merge two GKArrays with different epsilon values");
    if (srcs[k]->S != dst->S)
      return fail(GK_E_ARG, "stream counts differ (%lld vs %lld)", (long long)srcs[k]->S, (long long)dst->S);
  }
  // the fold runs per stream: dst.merge(srcs[0]); dst.merge(srcs[1]); ...
  // A source may be dst itself (gk:111-154 accepts other is self: the flush
  // of gk:137 empties dst's own incoming, the conversion reads the flushed
  // table into `conv` before gk:154 rewrites it, gk:149 doubles n) or repeat
  // (flushed again at each merge, as the reference does).
  parallel_for(dst->S, dst->threads, [&](int64_t s) {
    std::vector<Rec> conv;
    for (int k = 0; k < nsrcs; ++k) merge_stream(dst, dst->st[s], srcs[k]->st[s], conv);
  });
  return GK_OK;
}

int gk_merge_compress(gk_set* h, const double* v, const int32_t* g, const int32_t* d, const int64_t* eoffs,
                      void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!eoffs || !v || !g || !d) return fail(GK_E_ARG, "null record arrays");
  parallel_for(h->S, h->threads, [&](int64_t s) {
    std::vector<Rec> recs;
    for (int64_t k = eoffs[s]; k < eoffs[s + 1]; ++k) recs.push_back(Rec{v[k], g[k], d[k]});
    Stream& st = h->st[s];
    flush_general(st, threshold(h, st.n), recs.data(), recs.size(), tl_scratch.key, tl_scratch.inc, tl_scratch.out);
  });
  return GK_OK;
}

int gk_export_sizes(gk_set* h, int32_t* sizes, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  for (int64_t s = 0; s < h->S; ++s) sizes[s] = (int32_t)h->st[s].tab.size();
  return GK_OK;
}

int gk_export(gk_set* h, const int64_t* offs, double* v, int32_t* g, int32_t* d, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!offs) return fail(GK_E_ARG, "offs is null");
  parallel_for(h->S, h->threads, [&](int64_t s) {
    const std::vector<Rec>& t = h->st[s].tab;
    const int64_t o = offs[s];
    for (size_t j = 0; j < t.size(); ++j) {
      if (v) v[o + j] = t[j].v;
      if (g) g[o + j] = (int32_t)t[j].g;
      if (d) d[o + j] = (int32_t)t[j].d;
    }
  });
  return GK_OK;
}

int gk_export_pending_sizes(gk_set* h, int32_t* sizes, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  for (int64_t s = 0; s < h->S; ++s) sizes[s] = (int32_t)h->st[s].pend.size();
  return GK_OK;
}

int gk_export_pending(gk_set* h, const int64_t* poffs, double* pv, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!poffs || !pv) return fail(GK_E_ARG, "null pointer");
  for (int64_t s = 0; s < h->S; ++s) std::copy(h->st[s].pend.begin(), h->st[s].pend.end(), pv + poffs[s]);
  return GK_OK;
}

int gk_import(gk_set* h, const int64_t* offs, const double* v, const int32_t* g, const int32_t* d,
              const int64_t* poffs, const double* pv, const int64_t* n, const double* mn, const double* mx,
              const double* sum, const double* avg, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!offs || !poffs || !n || !mn || !mx || !sum || !avg) return fail(GK_E_ARG, "null pointer");
  for (int64_t s = 0; s < h->S; ++s)
    if (offs[s + 1] < offs[s] || poffs[s + 1] < poffs[s] || n[s] < 0 || poffs[s + 1] - poffs[s] > n[s] % h->P)
      return fail(GK_E_ARG, "stream %lld: bad table / pending sizes (pending <= n %% %d)", (long long)s, h->P);
  parallel_for(h->S, h->threads, [&](int64_t s) {
    Stream& st = h->st[s];
    st.n = n[s];
    st.mn = mn[s];
    st.mx = mx[s];
    st.sum = sum[s];
    st.avg = avg[s];
    st.tab.clear();
    for (int64_t k = offs[s]; k < offs[s + 1]; ++k) st.tab.push_back(Rec{v[k], g[k], d[k]});
    st.pend.assign(pv + poffs[s], pv + poffs[s + 1]);
  });
  return GK_OK;
}

// ---- versioned state files (gk_format.h) ------------------------------------
static int fmt_error(int rc, const char* path) {
  switch (rc) {
    case gkfmt::E_IO: return fail(GK_E_IO, "cannot read/write state file %s", path);
    case gkfmt::E_VERSION: return fail(GK_E_FORMAT, "%s: unsupported state format version", path);
    case gkfmt::E_CHECKSUM: return fail(GK_E_FORMAT, "%s: checksum mismatch (corrupt state file)", path);
    default: return fail(GK_E_FORMAT, "%s: not a GKSTATE file or truncated", path);
  }
}

int gk_save(gk_set* h, const char* path, void* stream) {
  (void)stream;
  int rc = check_set(h);
  if (rc) return rc;
  if (!path) return fail(GK_E_ARG, "path is null");
  gkfmt::State f;
  f.eps = h->eps;
  f.resize_streams(h->S);
  for (int64_t s = 0; s < h->S; ++s) {
    const Stream& st = h->st[s];
    f.sizes[s] = (int32_t)st.tab.size();
    f.psizes[s] = (int32_t)st.pend.size();
    f.n[s] = st.n;
    f.mn[s] = st.mn;
    f.mx[s] = st.mx;
    f.sum[s] = st.sum;
    f.avg[s] = st.avg;
    for (const Rec& r : st.tab) {
      f.v.push_back(r.v);
      f.g.push_back((int32_t)r.g);
      f.d.push_back((int32_t)r.d);
    }
    f.pv.insert(f.pv.end(), st.pend.begin(), st.pend.end());
  }
  rc = gkfmt::write(path, f);
  return rc ? fmt_error(rc, path) : GK_OK;
}

int gk_peek(const char* path, double* eps, int64_t* num_streams) {
  if (!path) return fail(GK_E_ARG, "path is null");
  gkfmt::Header hd;
  const int rc = gkfmt::peek(path, &hd);
  if (rc) return fmt_error(rc, path);
  if (eps) *eps = hd.eps;
  if (num_streams) *num_streams = hd.S;
  return GK_OK;
}

int gk_load(gk_set* h, const char* path, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!path) return fail(GK_E_ARG, "path is null");
  gkfmt::State f;
  rc = gkfmt::read(path, &f);
  if (rc) return fmt_error(rc, path);
  if (f.S != h->S)
    return fail(GK_E_ARG, "%s holds %lld streams, the set has %lld", path, (long long)f.S, (long long)h->S);
  if (f.eps != h->eps)
    return fail(GK_E_EPS_MISMATCH, "%s was saved with eps=%.17g, the set has eps=%.17g", path, f.eps, h->eps);
  std::vector<int64_t> offs(f.S + 1, 0), poffs(f.S + 1, 0);
  for (int64_t s = 0; s < f.S; ++s) {
    offs[s + 1] = offs[s] + f.sizes[s];
    poffs[s + 1] = poffs[s] + f.psizes[s];
  }
  return gk_import(h, offs.data(), f.v.data(), f.g.data(), f.d.data(), poffs.data(), f.pv.data(), f.n.data(),
                   f.mn.data(), f.mx.data(), f.sum.data(), f.avg.data(), stream);
}

int64_t gk_num_streams(const gk_set* h) { return h ? h->S : -1; }
double gk_eps(const gk_set* h) { return h ? h->eps : 0.0; }
// ---- packed state (gk_pack.h): host buffers --------------------------------
namespace {
struct HostMem {
  static int to_host(void* host, const void* src, size_t n, void*) {
    memcpy(host, src, n);
    return GK_OK;
  }
  static int from_host(void* dst, const void* host, size_t n, void*) {
    memcpy(dst, host, n);
    return GK_OK;
  }
};
}  // namespace

int gk_pack_bytes(gk_set* h, int64_t* bytes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!bytes) return fail(GK_E_ARG, "bytes is null");
  std::vector<int32_t> e(std::max<int64_t>(h->S, 1)), p(std::max<int64_t>(h->S, 1));
  return gkpack::pack_bytes<HostMem>(h, e.data(), p.data(), bytes, stream);
}

int gk_pack(gk_set* h, void* buf, int64_t bytes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!buf) return fail(GK_E_ARG, "buf is null");
  std::vector<int32_t> e(std::max<int64_t>(h->S, 1)), p(std::max<int64_t>(h->S, 1));
  std::string err;
  rc = gkpack::pack<HostMem>(h, e.data(), p.data(), buf, bytes, stream, err);
  return (rc && !err.empty()) ? fail(rc, "%s", err.c_str()) : rc;
}

int gk_fold_packed(gk_set* dst, const void* const* bufs, int nbufs, void* stream) {
  int rc = check_set(dst);
  if (rc) return rc;
  std::string err;
  auto make = [&](gk_set** out) {
    const int r = gk_create(dst->S, dst->eps, 0, 0, out);
    if (!r) (*out)->threads = dst->threads;
    return r;
  };
  rc = gkpack::fold<HostMem>(dst, bufs, nbufs, &dst->fold_scratch, make, stream, err);
  return (rc && !err.empty()) ? fail(rc, "%s", err.c_str()) : rc;
}

int gk_flush_period(const gk_set* h) { return h ? (int)std::min<int64_t>(h->P, INT32_MAX) : -1; }
int gk_capacity(const gk_set* h, int cls) { return (h && cls == 0) ? INT32_MAX : -1; }  // unbounded, one class
int64_t gk_num_promoted(const gk_set* h) { return h ? 0 : -1; }
int64_t gk_host_chains_taken(gk_set* h) { return h ? 0 : -1; }  // the host engine walks every chain itself

int gk_timing_enable(gk_set* h, int on) {
  int rc = check_set(h);
  if (rc) return rc;
  h->timing = on != 0;
  return GK_OK;
}

int gk_timing_read(gk_set* h, double* flush_ms, double* stats_ms, int64_t* launches) {
  int rc = check_set(h);
  if (rc) return rc;
  if (flush_ms) *flush_ms = h->ingest_ms;
  if (stats_ms) *stats_ms = 0;
  if (launches) *launches = h->launches;
  h->ingest_ms = 0;
  h->launches = 0;
  return GK_OK;
}

}  // extern "C"
