// gk_pack.h -- packed state: a set's whole state (header words, tables,
// pending values) as ONE contiguous, self-describing buffer, the unit of the
// row-shard exchange.  Any transport moves it as bytes
// (rcclAllGather / MPI_Allgather on device buffers, a socket, a file); the
// rank-ordered fold of packed states is the reference's left fold
// sk0.merge(sk1)...merge(sk_{k-1}) (gkarray.py gk:111-154) for every stream.
//
// Header-only and written against the public C ABI (gk_capi.h) only, so the
// HIP engine (gk_capi.cpp, device buffers) and the CPU engine (gk_cpu.cpp,
// host buffers) share it; `Mem` supplies the engine's copies.
//
// Layout, version 1 (little-endian; every section starts on a 256-byte
// boundary so that the device-side copies are coalesced):
//   header (64 B): u64 magic "GKPACK01", u32 version, u32 header bytes,
//                  f64 eps, i64 S, i64 E_total, i64 P_total, i64 total bytes,
//                  u64 reserved
//   i64 n[S]  f64 min[S] max[S] sum[S] avg[S]          (gk:21-29 header words)
//   i64 eoffs[S+1]  i64 poffs[S+1]                     (exclusive prefix sums)
//   f64 v[E_total]  i32 g[E_total]  i32 d[E_total]     (entries, stream order)
//   f64 pv[P_total]                                    (incoming, insertion order)
// The sections are exactly gk_import's arguments, so unpacking is one import.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "gk_capi.h"

namespace gkpack {

constexpr uint64_t kMagic = 0x31304B4341504B47ull;  // "GKPACK01"
constexpr uint32_t kVersion = 1;

struct Header {
  uint64_t magic;
  uint32_t version;
  uint32_t header_bytes;
  double eps;
  int64_t S;
  int64_t E;
  int64_t P;
  int64_t bytes;
  uint64_t reserved;
};
static_assert(sizeof(Header) == 64, "packed header");

struct Layout {
  int64_t S = 0, E = 0, P = 0;
  size_t n = 0, mn = 0, mx = 0, sum = 0, avg = 0, eoffs = 0, poffs = 0, v = 0, g = 0, d = 0, pv = 0, total = 0;
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline Layout layout(int64_t S, int64_t E, int64_t P) {
  Layout L;
  L.S = S;
  L.E = E;
  L.P = P;
  size_t o = align256(sizeof(Header));
  auto put = [&](size_t& field, size_t bytes) {
    field = o;
    o = align256(o + bytes);
  };
  put(L.n, 8 * (size_t)S);
  put(L.mn, 8 * (size_t)S);
  put(L.mx, 8 * (size_t)S);
  put(L.sum, 8 * (size_t)S);
  put(L.avg, 8 * (size_t)S);
  put(L.eoffs, 8 * ((size_t)S + 1));
  put(L.poffs, 8 * ((size_t)S + 1));
  put(L.v, 8 * (size_t)E);
  put(L.g, 4 * (size_t)E);
  put(L.d, 4 * (size_t)E);
  put(L.pv, 8 * (size_t)P);
  L.total = o;
  return L;
}

template <typename T>
inline T* at(void* base, size_t off) {
  return (T*)((char*)base + off);
}
template <typename T>
inline const T* at(const void* base, size_t off) {
  return (const T*)((const char*)base + off);
}

// Mem (engine memory):
//   static int to_host(void* host, const void* src, size_t n, void* stream);   // completes before returning
//   static int from_host(void* dst, const void* host, size_t n, void* stream);  // completes before returning
// `esz` / `psz`: engine buffers of S int32 each (table / pending sizes).
template <class Mem>
int sizes(gk_set* set, int64_t S, int32_t* esz, int32_t* psz, std::vector<int64_t>& eo, std::vector<int64_t>& po,
          void* stream) {
  std::vector<int32_t> e(S), p(S);
  int rc = gk_export_sizes(set, esz, stream);
  if (!rc) rc = gk_export_pending_sizes(set, psz, stream);
  if (!rc && S) rc = Mem::to_host(e.data(), esz, 4 * (size_t)S, stream);
  if (!rc && S) rc = Mem::to_host(p.data(), psz, 4 * (size_t)S, stream);
  if (rc) return rc;
  eo.assign(S + 1, 0);
  po.assign(S + 1, 0);
  for (int64_t s = 0; s < S; ++s) {
    eo[s + 1] = eo[s] + e[s];
    po[s + 1] = po[s] + p[s];
  }
  return GK_OK;
}

template <class Mem>
int pack_bytes(gk_set* set, int32_t* esz, int32_t* psz, int64_t* bytes, void* stream) {
  const int64_t S = gk_num_streams(set);
  std::vector<int64_t> eo, po;
  int rc = sizes<Mem>(set, S, esz, psz, eo, po, stream);
  if (rc) return rc;
  *bytes = (int64_t)layout(S, eo[S], po[S]).total;
  return GK_OK;
}

// Returns GK_OK, an engine status, or GK_E_ARG with `err` set (buffer too small).
template <class Mem>
int pack(gk_set* set, int32_t* esz, int32_t* psz, void* buf, int64_t bytes, void* stream, std::string& err) {
  const int64_t S = gk_num_streams(set);
  std::vector<int64_t> eo, po;
  int rc = sizes<Mem>(set, S, esz, psz, eo, po, stream);
  if (rc) return rc;
  const Layout L = layout(S, eo[S], po[S]);
  if (bytes < (int64_t)L.total) {
    err = "packed state needs " + std::to_string(L.total) + " bytes, the buffer has " + std::to_string(bytes);
    return GK_E_ARG;
  }
  Header h{};
  h.magic = kMagic;
  h.version = kVersion;
  h.header_bytes = sizeof(Header);
  h.eps = gk_eps(set);
  h.S = S;
  h.E = eo[S];
  h.P = po[S];
  h.bytes = (int64_t)L.total;
  rc = Mem::from_host(buf, &h, sizeof(h), stream);
  if (!rc) rc = Mem::from_host(at<int64_t>(buf, L.eoffs), eo.data(), 8 * (size_t)(S + 1), stream);
  if (!rc) rc = Mem::from_host(at<int64_t>(buf, L.poffs), po.data(), 8 * (size_t)(S + 1), stream);
  if (rc) return rc;
  if (S == 0) return GK_OK;
  rc = gk_stats(set, at<int64_t>(buf, L.n), at<double>(buf, L.mn), at<double>(buf, L.mx), at<double>(buf, L.sum),
                at<double>(buf, L.avg), nullptr, nullptr, stream);
  if (!rc) rc = gk_export(set, at<int64_t>(buf, L.eoffs), at<double>(buf, L.v), at<int32_t>(buf, L.g),
                          at<int32_t>(buf, L.d), stream);
  if (!rc && L.P) rc = gk_export_pending(set, at<int64_t>(buf, L.poffs), at<double>(buf, L.pv), stream);
  if (!rc) rc = gk_sync(set, stream);
  return rc;
}

// Header of a packed buffer, validated against `dst`.
template <class Mem>
int read_header(gk_set* dst, const void* buf, Header* h, void* stream, std::string& err) {
  int rc = Mem::to_host(h, buf, sizeof(Header), stream);
  if (rc) return rc;
  if (h->magic != kMagic || h->header_bytes != sizeof(Header)) {
    err = "not a packed GK state";
    return GK_E_FORMAT;
  }
  if (h->version != kVersion) {
    err = "packed GK state version " + std::to_string(h->version) + " is not supported";
    return GK_E_FORMAT;
  }
  if (h->eps != gk_eps(dst)) {  // gk:118-119
    err = "Cannot merge two GKArrays with different epsilon values";
    return GK_E_EPS_MISMATCH;
  }
  if (h->S != gk_num_streams(dst)) {
    err = "packed state holds " + std::to_string(h->S) + " streams, the set has " +
          std::to_string(gk_num_streams(dst));
    return GK_E_ARG;
  }
  // sizes and offsets must be internally consistent before gk_import copies
  // anything (a corrupt header or offset table is refused).  The buffer's
  // own length is not known here (gk_fold_packed takes bare pointers): the
  // caller guarantees each buffer holds the header's `bytes` (gk_capi.h) --
  // a buffer truncated after an intact header and offset table is not caught
  if (h->E < 0 || h->P < 0 || h->E > ((int64_t)1 << 40) || h->P > ((int64_t)1 << 40) ||
      h->bytes != (int64_t)layout(h->S, h->E, h->P).total) {
    err = "packed state header is inconsistent (sizes / byte count)";
    return GK_E_FORMAT;
  }
  const Layout L = layout(h->S, h->E, h->P);
  std::vector<int64_t> eo(h->S + 1), po(h->S + 1);
  rc = Mem::to_host(eo.data(), at<int64_t>(buf, L.eoffs), 8 * (size_t)(h->S + 1), stream);
  if (!rc) rc = Mem::to_host(po.data(), at<int64_t>(buf, L.poffs), 8 * (size_t)(h->S + 1), stream);
  if (rc) return rc;
  bool ok = eo[0] == 0 && po[0] == 0 && eo[h->S] == h->E && po[h->S] == h->P;
  for (int64_t s = 0; ok && s < h->S; ++s) ok = eo[s + 1] >= eo[s] && po[s + 1] >= po[s];
  if (!ok) {
    err = "packed state offsets are not monotone from 0 to the header's totals";
    return GK_E_FORMAT;
  }
  return GK_OK;
}

template <class Mem>
int import_packed(gk_set* set, const void* buf, const Header& h, void* stream) {
  const Layout L = layout(h.S, h.E, h.P);
  return gk_import(set, at<int64_t>(buf, L.eoffs), at<double>(buf, L.v), at<int32_t>(buf, L.g),
                   at<int32_t>(buf, L.d), at<int64_t>(buf, L.poffs), at<double>(buf, L.pv), at<int64_t>(buf, L.n),
                   at<double>(buf, L.mn), at<double>(buf, L.mx), at<double>(buf, L.sum), at<double>(buf, L.avg),
                   stream);
}

// dst := bufs[0]; dst.merge(bufs[r]) for r = 1 .. nbufs-1, in that order
// (gk:111-154: each merge flushes `other` first).  `scratch`: a set of dst's
// shape (S, eps) that receives bufs[r] before each merge; made on first use
// by `make_scratch` and kept by the caller.
template <class Mem, class MakeScratch>
int fold(gk_set* dst, const void* const* bufs, int nbufs, gk_set** scratch, MakeScratch&& make_scratch, void* stream,
         std::string& err) {
  if (nbufs < 1 || !bufs) {
    err = "at least one packed state is needed";
    return GK_E_ARG;
  }
  std::vector<Header> hs(nbufs);
  for (int r = 0; r < nbufs; ++r) {
    if (!bufs[r]) {
      err = "packed state " + std::to_string(r) + " is null";
      return GK_E_ARG;
    }
    int rc = read_header<Mem>(dst, bufs[r], &hs[r], stream, err);
    if (rc) return rc;
  }
  int rc = import_packed<Mem>(dst, bufs[0], hs[0], stream);
  if (rc) return rc;
  for (int r = 1; r < nbufs; ++r) {
    if (!*scratch) {
      rc = make_scratch(scratch);
      if (rc) return rc;
    }
    rc = import_packed<Mem>(*scratch, bufs[r], hs[r], stream);
    if (!rc) rc = gk_merge(dst, scratch, 1, stream);
    if (rc) return rc;
  }
  return gk_sync(dst, stream);
}

}  // namespace gkpack
