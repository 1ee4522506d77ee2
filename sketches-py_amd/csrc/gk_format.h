// gk_format.h -- versioned on-disk / in-memory format of a set's full state
// (checkpoint, interchange between the HIP and CPU engines, RCCL-free
// hand-off between processes).  Header-only; shared by gk_capi.cpp (HIP) and
// gk_cpu.cpp (CPU engine).
//
// The reference keeps state only in Python objects (gkarray.py gk:21-29:
// entries, incoming, _n, _min, _max, _sum, _avg; Entry.__repr__ gk:15-16 is its
// only textual surface) and has no serialization, so this format is new.  It
// stores exactly that state per stream, with no flush: a loaded set behaves
// like the saved one for every later call.
//
// Layout, version 1 (little-endian; every array 8-byte aligned):
//   off  size  field
//   0    8     magic "GKSTATE\0"
//   8    4     u32 version (1)
//   12   4     u32 header bytes (80)
//   16   8     f64 eps
//   24   8     i64 S                 streams
//   32   8     i64 E_total           sum of table sizes
//   40   8     i64 P_total           sum of pending counts
//   48   8     u64 sum_a             sum of the payload's 64-bit words (mod 2^64)
//   56   8     u64 sum_b             sum of (i+1) * word_i (mod 2^64)
//   64   4     u32 flags (0)
//   68  12     reserved (0)
//   80   ...   payload:
//              i32 sizes[S]  i32 pending[S]          (entries / incoming lengths)
//              i64 n[S]  f64 min[S] max[S] sum[S] avg[S]
//              f64 v[E_total]  i32 g[E_total]  i32 d[E_total]   (tables, stream order)
//              f64 pv[P_total]                        (incoming, insertion order)
//              zero padding of the last array to 8 bytes
// Tables and pending values are concatenated in stream order; stream s's
// records start at the exclusive prefix sum of sizes.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

namespace gkfmt {

constexpr char kMagic[8] = {'G', 'K', 'S', 'T', 'A', 'T', 'E', '\0'};
constexpr uint32_t kVersion = 1;
constexpr uint32_t kHeaderBytes = 80;

struct Header {
  char magic[8];
  uint32_t version;
  uint32_t header_bytes;
  double eps;
  int64_t S;
  int64_t E_total;
  int64_t P_total;
  uint64_t sum_a;
  uint64_t sum_b;
  uint32_t flags;
  uint32_t reserved0;
  uint64_t reserved1;
};
static_assert(sizeof(Header) == kHeaderBytes, "header layout");

// Host-side copy of a set's state (what gk_export + gk_export_pending + gk_stats return).
struct State {
  double eps = 0;
  int64_t S = 0;
  std::vector<int32_t> sizes, psizes;
  std::vector<int64_t> n;
  std::vector<double> mn, mx, sum, avg;
  std::vector<double> v, pv;
  std::vector<int32_t> g, d;

  void resize_streams(int64_t s) {
    S = s;
    sizes.assign(s, 0);
    psizes.assign(s, 0);
    n.assign(s, 0);
    mn.assign(s, 0);
    mx.assign(s, 0);
    sum.assign(s, 0);
    avg.assign(s, 0);
  }
  int64_t e_total() const {
    int64_t t = 0;
    for (int32_t x : sizes) t += x;
    return t;
  }
  int64_t p_total() const {
    int64_t t = 0;
    for (int32_t x : psizes) t += x;
    return t;
  }
};

// running checksum over 64-bit words (the payload is a whole number of words)
struct Sum {
  uint64_t a = 0, b = 0, i = 0;
  void add(const void* p, size_t bytes) {
    const unsigned char* c = (const unsigned char*)p;
    size_t k = 0;
    for (; k + 8 <= bytes; k += 8) {
      uint64_t w;
      memcpy(&w, c + k, 8);
      a += w;
      b += (++i) * w;
    }
    if (k < bytes) {  // last partial word, zero padded
      uint64_t w = 0;
      memcpy(&w, c + k, bytes - k);
      a += w;
      b += (++i) * w;
    }
  }
};

inline size_t pad8(size_t b) { return (b + 7) & ~(size_t)7; }

// error codes returned by write/read (mapped to GK_E_* by the callers)
enum { OK = 0, E_IO = 1, E_FORMAT = 2, E_VERSION = 3, E_CHECKSUM = 4 };

inline int write_chunk(FILE* f, Sum& s, const void* p, size_t bytes) {
  if (bytes && fwrite(p, 1, bytes, f) != bytes) return E_IO;
  s.add(p, bytes);
  const size_t pad = pad8(bytes) - bytes;
  if (pad) {
    const unsigned char z[8] = {0};
    if (fwrite(z, 1, pad, f) != pad) return E_IO;
  }
  return OK;
}

inline int write(const char* path, const State& st) {
  FILE* f = fopen(path, "wb");
  if (!f) return E_IO;
  Header h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, kMagic, 8);
  h.version = kVersion;
  h.header_bytes = kHeaderBytes;
  h.eps = st.eps;
  h.S = st.S;
  h.E_total = (int64_t)st.v.size();
  h.P_total = (int64_t)st.pv.size();
  int rc = fwrite(&h, 1, sizeof(h), f) == sizeof(h) ? OK : E_IO;
  Sum s;
  const size_t S = (size_t)st.S, E = st.v.size(), P = st.pv.size();
  // sizes and pending are adjacent i32 arrays: written as one 8-byte-aligned run
  std::vector<int32_t> sp(2 * S);
  if (S) {
    memcpy(sp.data(), st.sizes.data(), 4 * S);
    memcpy(sp.data() + S, st.psizes.data(), 4 * S);
  }
  if (!rc) rc = write_chunk(f, s, sp.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.n.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.mn.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.mx.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.sum.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.avg.data(), 8 * S);
  if (!rc) rc = write_chunk(f, s, st.v.data(), 8 * E);
  std::vector<int32_t> gd(2 * E);
  if (E) {
    memcpy(gd.data(), st.g.data(), 4 * E);
    memcpy(gd.data() + E, st.d.data(), 4 * E);
  }
  if (!rc) rc = write_chunk(f, s, gd.data(), 8 * E);
  if (!rc) rc = write_chunk(f, s, st.pv.data(), 8 * P);
  if (!rc) {
    h.sum_a = s.a;
    h.sum_b = s.b;
    if (fseek(f, 0, SEEK_SET) != 0 || fwrite(&h, 1, sizeof(h), f) != sizeof(h)) rc = E_IO;
  }
  if (fclose(f) != 0 && !rc) rc = E_IO;
  return rc;
}

inline int read_header(FILE* f, Header* h) {
  if (fread(h, 1, sizeof(*h), f) != sizeof(*h)) return E_FORMAT;
  if (memcmp(h->magic, kMagic, 8) != 0) return E_FORMAT;
  if (h->version != kVersion) return E_VERSION;
  if (h->header_bytes != kHeaderBytes || h->S < 0 || h->E_total < 0 || h->P_total < 0) return E_FORMAT;
  return OK;
}

inline int peek(const char* path, Header* h) {
  FILE* f = fopen(path, "rb");
  if (!f) return E_IO;
  const int rc = read_header(f, h);
  fclose(f);
  return rc;
}

inline int read_chunk(FILE* f, Sum& s, void* p, size_t bytes) {
  if (bytes && fread(p, 1, bytes, f) != bytes) return E_FORMAT;
  s.add(p, bytes);
  const size_t pad = pad8(bytes) - bytes;
  unsigned char z[8];
  if (pad && fread(z, 1, pad, f) != pad) return E_FORMAT;
  return OK;
}

inline int read(const char* path, State* st) {
  FILE* f = fopen(path, "rb");
  if (!f) return E_IO;
  Header h;
  int rc = read_header(f, &h);
  if (rc) {
    fclose(f);
    return rc;
  }
  st->eps = h.eps;
  st->resize_streams(h.S);
  const size_t S = (size_t)h.S, E = (size_t)h.E_total, P = (size_t)h.P_total;
  Sum s;
  std::vector<int32_t> sp(2 * S);
  rc = read_chunk(f, s, sp.data(), 8 * S);
  if (!rc && S) {
    memcpy(st->sizes.data(), sp.data(), 4 * S);
    memcpy(st->psizes.data(), sp.data() + S, 4 * S);
  }
  if (!rc) rc = read_chunk(f, s, st->n.data(), 8 * S);
  if (!rc) rc = read_chunk(f, s, st->mn.data(), 8 * S);
  if (!rc) rc = read_chunk(f, s, st->mx.data(), 8 * S);
  if (!rc) rc = read_chunk(f, s, st->sum.data(), 8 * S);
  if (!rc) rc = read_chunk(f, s, st->avg.data(), 8 * S);
  st->v.resize(E);
  st->g.resize(E);
  st->d.resize(E);
  st->pv.resize(P);
  if (!rc) rc = read_chunk(f, s, st->v.data(), 8 * E);
  std::vector<int32_t> gd(2 * E);
  if (!rc) rc = read_chunk(f, s, gd.data(), 8 * E);
  if (!rc && E) {
    memcpy(st->g.data(), gd.data(), 4 * E);
    memcpy(st->d.data(), gd.data() + E, 4 * E);
  }
  if (!rc) rc = read_chunk(f, s, st->pv.data(), 8 * P);
  fclose(f);
  if (rc) return rc;
  if (s.a != h.sum_a || s.b != h.sum_b) return E_CHECKSUM;
  // the size arrays must describe the stored records
  int64_t et = 0, pt = 0;
  for (size_t k = 0; k < S; ++k) {
    if (st->sizes[k] < 0 || st->psizes[k] < 0) return E_FORMAT;
    et += st->sizes[k];
    pt += st->psizes[k];
  }
  if (et != h.E_total || pt != h.P_total) return E_FORMAT;
  return OK;
}

}  // namespace gkfmt
