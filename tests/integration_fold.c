/* INTEGRATION.md section 4 ("Row-shard fold from C over RCCL"), compiled and
 * run against the host engine (libgkarray_cpu.so: the same include/gk_capi.h
 * on host memory).  N ranks live in this one process; the two collectives of
 * that sequence are replaced by stand-ins that do what RCCL does to the bytes:
 *   ncclAllReduce(max) of the packed sizes -> the maximum over the ranks' sizes
 *   ncclAllGather of the packed buffers    -> memcpy of every rank's buffer
 *                                             into slot r of one `all` buffer
 * Every other call is the section's code unchanged (gk_pack_bytes, gk_pack,
 * gk_fold_packed).  Each rank folds into its own dst set; the program checks
 * that all ranks' folds are byte-identical (gk_pack of each dst) and writes
 * rank 0's folded state for tests/test_integration_c.py, which compares it
 * with the oracle's rank-ordered left fold (gk:111-154).
 *
 * Input  (argv[1]): int64 S, double eps, int32 nranks, then per rank int64
 *                   offsets[S+1] and float64 values[offsets[S]].
 * Output (argv[2]): the folded state of rank 0: int32 sizes[S], int32
 *                   pending[S], int64 n[S], float64 min/max/sum/avg[S], then
 *                   the tables (float64 v, int32 g, int32 d; CSR by sizes) and
 *                   the pending values (CSR by pending).
 * Build: gcc -O2 -Iinclude tests/integration_fold.c -Lsketches-py_amd/gkarray_amd -lgkarray_cpu
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gk_capi.h"

#define MAXR 64

static void die(const char* what, int rc) {
  fprintf(stderr, "integration_fold: %s failed (%d): %s\n", what, rc, gk_last_error());
  exit(1);
}

/* the stand-in collectives: in-process "ranks" */
static void allreduce_max_i64(int64_t* per_rank, int nranks) {
  int64_t m = per_rank[0];
  for (int r = 1; r < nranks; ++r)
    if (per_rank[r] > m) m = per_rank[r];
  for (int r = 0; r < nranks; ++r) per_rank[r] = m;
}
static void allgather_bytes(void* const* mine, void* all, int64_t bytes, int nranks) {
  for (int r = 0; r < nranks; ++r) memcpy((char*)all + (size_t)r * bytes, mine[r], (size_t)bytes);
}

/* INTEGRATION.md section 4, for all ranks at once (the collectives are the
 * synchronisation points, so each step runs for every rank before the next) */
static void fold_row_shards(gk_set** set, gk_set** dst, int nranks) {
  int64_t mine[MAXR], bytes[MAXR];
  int rc;
  for (int r = 0; r < nranks; ++r)
    if ((rc = gk_pack_bytes(set[r], &mine[r], NULL))) die("gk_pack_bytes", rc);
  memcpy(bytes, mine, sizeof(int64_t) * nranks);
  allreduce_max_i64(bytes, nranks); /* ncclAllReduce(d_n, d_n, 1, ncclInt64, ncclMax) */
  void* mine_buf[MAXR];
  void* all[MAXR];
  for (int r = 0; r < nranks; ++r) {
    mine_buf[r] = malloc((size_t)bytes[r]);
    all[r] = malloc((size_t)bytes[r] * nranks);
    memset(mine_buf[r], 0xA5, (size_t)bytes[r]); /* trailing bytes unused */
    if ((rc = gk_pack(set[r], mine_buf[r], bytes[r], NULL))) die("gk_pack", rc);
  }
  for (int r = 0; r < nranks; ++r) allgather_bytes(mine_buf, all[r], bytes[r], nranks); /* ncclAllGather */
  for (int r = 0; r < nranks; ++r) {
    const void* bufs[MAXR];
    for (int k = 0; k < nranks; ++k) bufs[k] = (const char*)all[r] + (size_t)k * bytes[r];
    if ((rc = gk_fold_packed(dst[r], bufs, nranks, NULL))) die("gk_fold_packed", rc);
  }
  for (int r = 0; r < nranks; ++r) {
    free(all[r]);
    free(mine_buf[r]);
  }
}

static void* read_all(FILE* f, size_t n) {
  void* p = malloc(n ? n : 1);
  if (n && fread(p, 1, n, f) != n) {
    fprintf(stderr, "integration_fold: short input\n");
    exit(1);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: integration_fold IN OUT\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t S;
  double eps;
  int32_t nranks;
  if (fread(&S, 8, 1, f) != 1 || fread(&eps, 8, 1, f) != 1 || fread(&nranks, 4, 1, f) != 1) return 2;
  if (nranks < 1 || nranks > MAXR || S < 0) return 2;
  gk_set* set[MAXR];
  gk_set* dst[MAXR];
  int rc;
  for (int r = 0; r < nranks; ++r) {
    int64_t* offs = (int64_t*)read_all(f, sizeof(int64_t) * (size_t)(S + 1));
    double* v = (double*)read_all(f, sizeof(double) * (size_t)offs[S]);
    if ((rc = gk_create(S, eps, 0, 0, &set[r]))) die("gk_create", rc);
    if ((rc = gk_create(S, eps, 0, 0, &dst[r]))) die("gk_create", rc);
    if ((rc = gk_ingest(set[r], v, offs, NULL))) die("gk_ingest", rc);
    if ((rc = gk_sync(set[r], NULL))) die("gk_sync", rc);
    free(offs);
    free(v);
  }
  fclose(f);
  fold_row_shards(set, dst, nranks);

  /* every rank holds the same fold: compare the packed bytes */
  int64_t b0 = 0;
  if ((rc = gk_pack_bytes(dst[0], &b0, NULL))) die("gk_pack_bytes", rc);
  void* p0 = calloc(1, (size_t)b0); /* (pack leaves the alignment gaps untouched) */
  if ((rc = gk_pack(dst[0], p0, b0, NULL))) die("gk_pack", rc);
  for (int r = 1; r < nranks; ++r) {
    int64_t b = 0;
    if ((rc = gk_pack_bytes(dst[r], &b, NULL))) die("gk_pack_bytes", rc);
    void* p = calloc(1, (size_t)b);
    if ((rc = gk_pack(dst[r], p, b, NULL))) die("gk_pack", rc);
    if (b != b0 || memcmp(p, p0, (size_t)b)) {
      fprintf(stderr, "integration_fold: rank %d's fold differs from rank 0's\n", r);
      return 1;
    }
    free(p);
  }
  free(p0);

  /* rank 0's folded state */
  const size_t s1 = (size_t)(S ? S : 1);
  int32_t* sizes = (int32_t*)malloc(4 * s1);
  int32_t* pend = (int32_t*)malloc(4 * s1);
  int64_t* n = (int64_t*)malloc(8 * s1);
  double *mn = (double*)malloc(8 * s1), *mx = (double*)malloc(8 * s1);
  double *sm = (double*)malloc(8 * s1), *av = (double*)malloc(8 * s1);
  if ((rc = gk_stats(dst[0], n, mn, mx, sm, av, sizes, pend, NULL))) die("gk_stats", rc);
  int64_t* offs = (int64_t*)calloc(s1 + 1, 8);
  int64_t* poffs = (int64_t*)calloc(s1 + 1, 8);
  for (int64_t s = 0; s < S; ++s) {
    offs[s + 1] = offs[s] + sizes[s];
    poffs[s + 1] = poffs[s] + pend[s];
  }
  const size_t E = (size_t)offs[S], Pn = (size_t)poffs[S];
  double* v = (double*)malloc(8 * (E ? E : 1));
  int32_t* g = (int32_t*)malloc(4 * (E ? E : 1));
  int32_t* d = (int32_t*)malloc(4 * (E ? E : 1));
  double* pv = (double*)malloc(8 * (Pn ? Pn : 1));
  if ((rc = gk_export(dst[0], offs, v, g, d, NULL))) die("gk_export", rc);
  if ((rc = gk_export_pending(dst[0], poffs, pv, NULL))) die("gk_export_pending", rc);
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  fwrite(sizes, 4, (size_t)S, o);
  fwrite(pend, 4, (size_t)S, o);
  fwrite(n, 8, (size_t)S, o);
  double* hdr[4] = {mn, mx, sm, av};
  for (int k = 0; k < 4; ++k) fwrite(hdr[k], 8, (size_t)S, o);
  fwrite(v, 8, E, o);
  fwrite(g, 4, E, o);
  fwrite(d, 4, E, o);
  fwrite(pv, 8, Pn, o);
  fclose(o);
  for (int r = 0; r < nranks; ++r) {
    gk_destroy(set[r]);
    gk_destroy(dst[r]);
  }
  printf("integration_fold: %d ranks, %lld streams folded, %zu entries\n", nranks, (long long)S, E);
  return 0;
}
