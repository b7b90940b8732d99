// Sanitizer driver for the host C++ of libmirec (csrc/graph.cpp,
// csrc/ingest.cpp): built with -fsanitize=address,undefined by
// tests/test_host.py::test_host_code_under_asan_ubsan and run on random and
// malformed inputs; exits non-zero on a failed check (the sanitizers abort on
// any memory or UB error).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "mirec.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      return 1;                                                    \
    }                                                              \
  } while (0)

static int check_bipartite(std::mt19937_64 &rng, int64_t nu, int64_t mi, int64_t ne) {
  std::vector<int64_t> u(ne), it(ne);
  for (int64_t e = 0; e < ne; ++e) {
    u[e] = (int64_t)(rng() % nu);
    it[e] = (int64_t)(rng() % mi);
  }
  const int64_t n = nu + mi;
  std::vector<int64_t> rowptr(n + 1);
  std::vector<int32_t> col(2 * ne + 1);
  std::vector<float> dinv(n);
  CHECK(mirec_csr_bipartite(u.data(), it.data(), ne, nu, mi, rowptr.data(), col.data(),
                            dinv.data()) == MIREC_OK);
  CHECK(rowptr[0] == 0 && rowptr[n] == 2 * ne);
  for (int64_t r = 0; r < n; ++r) {
    CHECK(rowptr[r + 1] >= rowptr[r]);
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    CHECK(deg == 0 ? dinv[r] == 0.f : dinv[r] > 0.f);
    for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k)
      CHECK(r < nu ? (col[k] >= nu && col[k] < n) : (col[k] >= 0 && col[k] < nu));
  }
  // sorted user rows (the samplers' binary-search copy)
  std::vector<int32_t> srt(rowptr[nu] + 1);
  CHECK(mirec_csr_sort_rows(rowptr.data(), col.data(), nu, srt.data()) == MIREC_OK);
  for (int64_t r = 0; r < nu; ++r)
    for (int64_t k = rowptr[r] + 1; k < rowptr[r + 1]; ++k) CHECK(srt[k - 1] <= srt[k]);
  // long-row schedule, both passes
  int64_t nl = 0, ns = 0;
  CHECK(mirec_csr_long_rows(rowptr.data(), n, 7, &nl, &ns, nullptr, nullptr, nullptr,
                            nullptr) == MIREC_OK);
  std::vector<int32_t> lr(nl + 1), sr(ns + 1);
  std::vector<int64_t> lsp(nl + 1), sb(ns + 1);
  CHECK(mirec_csr_long_rows(rowptr.data(), n, 7, &nl, &ns, lr.data(), lsp.data(), sr.data(),
                            sb.data()) == MIREC_OK);
  CHECK(lsp[nl] == ns);
  // generic COO form on the same edges
  std::vector<int64_t> src(2 * ne), dst(2 * ne);
  for (int64_t e = 0; e < ne; ++e) {
    src[e] = u[e];
    dst[e] = nu + it[e];
    src[ne + e] = nu + it[e];
    dst[ne + e] = u[e];
  }
  std::vector<int64_t> rp2(n + 1);
  std::vector<int32_t> c2(2 * ne + 1);
  std::vector<float> d2(n);
  CHECK(mirec_csr_from_coo(src.data(), dst.data(), 2 * ne, n, rp2.data(), c2.data(),
                           d2.data()) == MIREC_OK);
  for (int64_t r = 0; r <= n; ++r) CHECK(rp2[r] == rowptr[r]);
  return 0;
}

static int check_ingest(std::mt19937_64 &rng) {
  std::string txt;
  const int lines = 2000;
  for (int l = 0; l < lines; ++l) {
    txt += std::to_string(l);
    const int k = (int)(rng() % 12);
    for (int j = 0; j < k; ++j) txt += ((rng() & 1) ? " " : "\t") + std::to_string(rng() % 999);
    if (rng() % 7 == 0) txt += "  ";
    txt += (rng() % 11 == 0) ? "\n\n" : "\n";
  }
  for (int threads : {1, 4}) {
    int64_t nl = 0, ni = 0, mu = 0, mx = 0;
    CHECK(mirec_parse_interactions(txt.data(), (int64_t)txt.size(), -1, threads, &nl, &ni, &mu,
                                   &mx, nullptr, nullptr, nullptr) == MIREC_OK);
    CHECK(nl == lines && mu == lines - 1);
    std::vector<int64_t> lu(nl), lo(nl + 1), items(ni + 1);
    CHECK(mirec_parse_interactions(txt.data(), (int64_t)txt.size(), -1, threads, &nl, &ni, &mu,
                                   &mx, lu.data(), lo.data(), items.data()) == MIREC_OK);
    for (int64_t k = 0; k < nl; ++k) CHECK(lu[k] == k && lo[k + 1] >= lo[k]);
  }
  const char *bad[] = {"0 1 2\n1 3x 4\n", "x\n", "0 -\n", "0 1\n2 99999999999999999999999\n"};
  for (const char *b : bad) {
    int64_t nl = 0, ni = 0, mu = 0, mx = 0;
    const int rc = mirec_parse_interactions(b, (int64_t)std::string(b).size(), -1, 1, &nl, &ni,
                                            &mu, &mx, nullptr, nullptr, nullptr);
    CHECK(rc != MIREC_OK);
  }
  return 0;
}

int main() {
  std::mt19937_64 rng(7);
  CHECK(check_bipartite(rng, 500, 80, 6000) == 0);
  CHECK(check_bipartite(rng, 1, 1, 1) == 0);
  CHECK(check_bipartite(rng, 3000, 5, 40000) == 0);
  CHECK(check_ingest(rng) == 0);
  // argument checks
  CHECK(mirec_csr_bipartite(nullptr, nullptr, 1, 1, 1, nullptr, nullptr, nullptr) != MIREC_OK);
  CHECK(mirec_csr_sort_rows(nullptr, nullptr, 1, nullptr) != MIREC_OK);
  std::puts("host_check ok");
  return 0;
}
