// Host-side graph build for libmirec.so (runs once per graph) and the
// library's status helpers.
//
// The reference materialises the symmetric edge list [2, 2E] int64
// (model/lgcn.py:53-61) and PyG's gcn_norm recomputes degrees and per-edge
// weights on every LGConv call.  Here the edge list is turned once into a
// destination-major CSR (int64 rowptr, int32 col) by a stable counting sort
// (rows keep the reference's edge order, multi-edges are kept) plus
// dinv = deg^-1/2, which is all the propagation kernel needs.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "mirec.h"

namespace mirec {
thread_local int g_last_hip_error = 0;
}

extern "C" const char *mirec_strerror(int code) {
  switch (code) {
    case MIREC_OK: return "ok";
    case MIREC_ERR_ARG: return "invalid argument";
    case MIREC_ERR_DIM: return "unsupported embedding dim (need 4,8,16,32,64,128 or 256)";
    case MIREC_ERR_HIP: return "HIP runtime error";
    case MIREC_ERR_WORKSPACE: return "workspace too small";
    case MIREC_ERR_RANGE: return "index out of range";
  }
  return "unknown mirec status";
}

extern "C" int mirec_abi_version(void) { return MIREC_ABI_VERSION; }

extern "C" int mirec_last_hip_error(void) { return mirec::g_last_hip_error; }

extern "C" int mirec_struct_sizes(size_t *csr, size_t *prop, size_t *adam_hparams) {
  if (csr == nullptr || prop == nullptr || adam_hparams == nullptr) return MIREC_ERR_ARG;
  *csr = sizeof(mirec_csr_t);
  *prop = sizeof(mirec_prop_t);
  *adam_hparams = sizeof(mirec_adam_hparams_t);
  return MIREC_OK;
}

static void fill_dinv(const int64_t *rowptr, int64_t n, float *dinv) {
  for (int64_t v = 0; v < n; ++v) {
    const int64_t d = rowptr[v + 1] - rowptr[v];
    dinv[v] = d > 0 ? (float)(1.0 / std::sqrt((double)d)) : 0.f;
  }
}

extern "C" int mirec_csr_bipartite(const int64_t *train_user, const int64_t *train_item,
                                   int64_t n_edges, int64_t n_users, int64_t m_items,
                                   int64_t *rowptr, int32_t *col, float *dinv) {
  if (n_edges < 0 || n_users <= 0 || m_items <= 0 || rowptr == nullptr) return MIREC_ERR_ARG;
  if (n_edges > 0 && (train_user == nullptr || train_item == nullptr || col == nullptr))
    return MIREC_ERR_ARG;
  const int64_t n = n_users + m_items;
  if (n >= INT32_MAX) return MIREC_ERR_RANGE;
  std::memset(rowptr, 0, sizeof(int64_t) * (n + 1));
  for (int64_t e = 0; e < n_edges; ++e) {
    const int64_t u = train_user[e], i = train_item[e];
    if (u < 0 || u >= n_users || i < 0 || i >= m_items) return MIREC_ERR_RANGE;
    ++rowptr[u + 1];
    ++rowptr[n_users + i + 1];
  }
  for (int64_t v = 0; v < n; ++v) rowptr[v + 1] += rowptr[v];
  std::vector<int64_t> cur(rowptr, rowptr + n);
  // Destination n_users+i receives from the first half of the reference
  // edge list (user -> item), destination u from the second half
  // (item -> user); both in edge order.
  for (int64_t e = 0; e < n_edges; ++e) {
    const int64_t u = train_user[e], it = n_users + train_item[e];
    col[cur[it]++] = (int32_t)u;
    col[cur[u]++] = (int32_t)it;
  }
  if (dinv != nullptr) fill_dinv(rowptr, n, dinv);
  return MIREC_OK;
}

extern "C" int mirec_csr_from_coo(const int64_t *src, const int64_t *dst, int64_t nnz,
                                  int64_t n_nodes, int64_t *rowptr, int32_t *col, float *dinv) {
  if (nnz < 0 || n_nodes <= 0 || rowptr == nullptr) return MIREC_ERR_ARG;
  if (nnz > 0 && (src == nullptr || dst == nullptr || col == nullptr)) return MIREC_ERR_ARG;
  if (n_nodes >= INT32_MAX) return MIREC_ERR_RANGE;
  std::memset(rowptr, 0, sizeof(int64_t) * (n_nodes + 1));
  for (int64_t e = 0; e < nnz; ++e) {
    if (src[e] < 0 || src[e] >= n_nodes || dst[e] < 0 || dst[e] >= n_nodes)
      return MIREC_ERR_RANGE;
    ++rowptr[dst[e] + 1];
  }
  for (int64_t v = 0; v < n_nodes; ++v) rowptr[v + 1] += rowptr[v];
  std::vector<int64_t> cur(rowptr, rowptr + n_nodes);
  for (int64_t e = 0; e < nnz; ++e) col[cur[dst[e]]++] = (int32_t)src[e];
  if (dinv != nullptr) fill_dinv(rowptr, n_nodes, dinv);
  return MIREC_OK;
}

extern "C" int mirec_csr_long_rows(const int64_t *rowptr, int64_t n_rows, int32_t split,
                                   int64_t *n_long, int64_t *n_seg, int32_t *long_rows,
                                   int64_t *long_segptr, int32_t *seg_row, int64_t *seg_beg) {
  if (rowptr == nullptr || n_rows < 0 || split <= 0 || n_long == nullptr || n_seg == nullptr)
    return MIREC_ERR_ARG;
  const bool fill = long_rows != nullptr;
  if (fill && (long_segptr == nullptr || seg_row == nullptr || seg_beg == nullptr))
    return MIREC_ERR_ARG;
  int64_t nl = 0, ns = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t beg = rowptr[r], deg = rowptr[r + 1] - beg;
    if (deg <= split) continue;
    const int64_t k = (deg + split - 1) / split;
    if (fill) {
      long_rows[nl] = (int32_t)r;
      long_segptr[nl] = ns;
      for (int64_t s = 0; s < k; ++s) {
        seg_row[ns + s] = (int32_t)r;
        seg_beg[ns + s] = beg + s * split;
      }
    }
    ++nl;
    ns += k;
  }
  if (fill) long_segptr[nl] = ns;
  *n_long = nl;
  *n_seg = ns;
  return MIREC_OK;
}

// Rows [0, n_rows) of the CSR with each row's entries sorted ascending (a
// copy: the propagation keeps the reference's edge order).  The samplers test
// "negative item in the user's positives" (negative_sample.py:121-126) by
// binary search in these rows instead of a scan.  Rows are split over up to
// 16 threads by entry count.
extern "C" int mirec_csr_sort_rows(const int64_t *rowptr, const int32_t *col, int64_t n_rows,
                                   int32_t *col_sorted) {
  if (rowptr == nullptr || n_rows < 0 || (rowptr[n_rows] > 0 && (col == nullptr ||
                                                                col_sorted == nullptr)))
    return MIREC_ERR_ARG;
  const int64_t total = rowptr[n_rows] - rowptr[0];
  if (total == 0) return MIREC_OK;
  const int n_thr = (int)std::max<int64_t>(
      1, std::min<int64_t>(16, std::min<int64_t>((int64_t)std::thread::hardware_concurrency(),
                                                 total / (1 << 16) + 1)));
  std::vector<int64_t> cut(n_thr + 1, n_rows);
  cut[0] = 0;
  for (int t = 1; t < n_thr; ++t) {  // first row whose start passes t/n_thr of the entries
    const int64_t want = rowptr[0] + total * t / n_thr;
    cut[t] = std::lower_bound(rowptr, rowptr + n_rows, want) - rowptr;
  }
  auto work = [&](int t) {
    for (int64_t r = cut[t]; r < cut[t + 1]; ++r) {
      const int64_t a = rowptr[r] - rowptr[0], b = rowptr[r + 1] - rowptr[0];
      std::copy(col + rowptr[r], col + rowptr[r + 1], col_sorted + a);
      std::sort(col_sorted + a, col_sorted + b);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_thr; ++t) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  return MIREC_OK;
}

// Per-user positive CDF for the weighted samplers (the sample_pow option,
// negative_sample.py:53-56): probs[e - rowptr[0]] = the probability of entry
// e of its user row (rows 0 .. n_users - 1, the allPos order), each row's
// probabilities non-negative with a positive sum; cdf[e - rowptr[0]] = the
// inclusive cumulative sum in float64 divided by the row total (numpy's
// choice normalises the same way), kept in float64 — an entry of
// probability 1e-12 after a row mass of 0.5 stays its own CDF step (a float
// CDF would merge it into its neighbour) — the row's last entry exactly 1.
// Empty rows are skipped.
extern "C" int mirec_pos_cdf_build(const int64_t *rowptr, int64_t n_users, const double *probs,
                                   double *cdf) {
  if (rowptr == nullptr || n_users < 0) return MIREC_ERR_ARG;
  const int64_t base = rowptr[0], total = rowptr[n_users] - base;
  if (total > 0 && (probs == nullptr || cdf == nullptr)) return MIREC_ERR_ARG;
  for (int64_t u = 0; u < n_users; ++u) {
    const int64_t a = rowptr[u] - base, b = rowptr[u + 1] - base;
    if (b < a) return MIREC_ERR_ARG;
    if (a == b) continue;
    double s = 0.0;
    for (int64_t e = a; e < b; ++e) {
      if (!(probs[e] >= 0.0) || !std::isfinite(probs[e])) return MIREC_ERR_ARG;
      s += probs[e];
    }
    if (!(s > 0.0)) return MIREC_ERR_ARG;
    double c = 0.0, prev = 0.0;
    for (int64_t e = a; e < b; ++e) {
      c += probs[e];
      double v = c / s;
      v = v < prev ? prev : (v > 1.0 ? 1.0 : v);
      cdf[e] = v;
      prev = v;
    }
    cdf[b - 1] = 1.0;
  }
  return MIREC_OK;
}
