// Native ingest of the reference's interaction files (dataloader.py:93-150:
// one line per user, "uid i1 i2 ..." separated by spaces).  The reference
// parses them in a Python loop (~1e5 lines/s); here the
// buffer is cut into per-thread chunks at line boundaries, every thread
// counts its lines / items, a prefix sum places each chunk, and a second
// pass writes uid, per-line item offsets and the items.  Output order is
// file order, so allPos stays line-indexed exactly like the reference's.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "mirec.h"

namespace {

struct Chunk {
  const char *beg, *end;
  int64_t lines = 0, items = 0, max_uid = -1, max_item = -1;
  bool stop = false;   // this chunk holds the stop line
  int64_t line0 = 0, item0 = 0;
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// Parses one line [p, e).  Returns false for an empty line (no uid).
// Integers: optional '-', decimal digits; any other byte ends a token.
template <class F>
inline bool parse_line(const char *p, const char *e, int64_t &uid, F &&on_item, bool &bad) {
  bool have_uid = false;
  while (p < e) {
    while (p < e && is_space(*p)) ++p;
    if (p >= e) break;
    bool neg = false;
    if (*p == '-') {
      neg = true;
      ++p;
    }
    if (p >= e || *p < '0' || *p > '9') {
      bad = true;
      return have_uid;
    }
    int64_t v = 0;
    while (p < e && *p >= '0' && *p <= '9') {
      const int d = *p++ - '0';
      if (v > (INT64_MAX - d) / 10) {  // an id that does not fit int64: malformed
        bad = true;
        return have_uid;
      }
      v = v * 10 + d;
    }
    if (p < e && !is_space(*p)) {
      bad = true;
      return have_uid;
    }
    if (neg) v = -v;
    if (!have_uid) {
      uid = v;
      have_uid = true;
    } else {
      on_item(v);
    }
  }
  return have_uid;
}

template <class F>
void scan(Chunk &c, int64_t stop_uid, bool &bad, F &&on_line) {
  const char *p = c.beg;
  while (p < c.end) {
    const char *nl = static_cast<const char *>(memchr(p, '\n', c.end - p));
    const char *e = nl ? nl : c.end;
    int64_t uid = -1;
    on_line(p, e, uid);
    p = nl ? nl + 1 : c.end;
    if (uid >= 0 && stop_uid >= 0 && uid == stop_uid) {
      c.stop = true;
      return;
    }
  }
}

}  // namespace

extern "C" int mirec_parse_interactions(const char *buf, int64_t len, int64_t stop_uid,
                                        int32_t n_threads, int64_t *n_lines, int64_t *n_items,
                                        int64_t *max_uid, int64_t *max_item, int64_t *line_uid,
                                        int64_t *line_off, int64_t *items) {
  if ((buf == nullptr && len > 0) || len < 0 || !n_lines || !n_items || !max_uid || !max_item)
    return MIREC_ERR_ARG;
  const bool fill = line_uid != nullptr;
  if (fill && (line_off == nullptr || items == nullptr)) return MIREC_ERR_ARG;
  int T = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 1, 64));
  if (len < (int64_t)1 << 20) T = 1;
  // chunk boundaries at line starts
  std::vector<Chunk> ch(T);
  const char *end = buf + len;
  const char *p = buf;
  for (int t = 0; t < T; ++t) {
    ch[t].beg = p;
    const char *q = t == T - 1 ? end : buf + len * (t + 1) / T;
    if (q < p) q = p;
    if (t < T - 1 && q < end) {
      const char *nl = static_cast<const char *>(memchr(q, '\n', end - q));
      q = nl ? nl + 1 : end;
    }
    ch[t].end = q;
    p = q;
  }
  std::vector<char> bad(T, 0);
  // pass 1: counts
  auto count = [&](int t) {
    Chunk c = ch[t];  // thread-local copy: no false sharing on the counters
    bool b = false;
    scan(c, stop_uid, b, [&](const char *s, const char *e, int64_t &uid) {
      int64_t k = 0, mx = c.max_item;
      if (parse_line(s, e, uid, [&](int64_t v) { ++k; mx = std::max(mx, v); }, b)) {
        ++c.lines;
        c.items += k;
        c.max_item = mx;
        c.max_uid = std::max(c.max_uid, uid);
      } else {
        uid = -1;
      }
    });
    ch[t] = c;
    bad[t] = b;
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(count, t);
    count(0);
    for (auto &x : th) x.join();
  }
  // the stop line ends the file: later chunks are dropped
  int last = T - 1;
  for (int t = 0; t < T; ++t)
    if (ch[t].stop) {
      last = t;
      break;
    }
  int64_t L = 0, I = 0, mu = -1, mi = -1;
  for (int t = 0; t <= last; ++t) {
    if (bad[t]) return MIREC_ERR_ARG;
    ch[t].line0 = L;
    ch[t].item0 = I;
    L += ch[t].lines;
    I += ch[t].items;
    mu = std::max(mu, ch[t].max_uid);
    mi = std::max(mi, ch[t].max_item);
  }
  *n_lines = L;
  *n_items = I;
  *max_uid = mu;
  *max_item = mi;
  if (!fill) return MIREC_OK;
  // pass 2: fill
  auto write = [&](int t) {
    Chunk c = ch[t];
    int64_t li = c.line0, ii = c.item0;
    bool b = false;
    c.stop = false;
    scan(c, stop_uid, b, [&](const char *s, const char *e, int64_t &uid) {
      const int64_t i0 = ii;
      if (parse_line(s, e, uid, [&](int64_t v) { items[ii++] = v; }, b)) {
        line_uid[li] = uid;
        line_off[li] = i0;
        ++li;
      } else {
        uid = -1;
      }
    });
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t <= last; ++t) th.emplace_back(write, t);
    write(0);
    for (auto &x : th) x.join();
  }
  line_off[L] = I;
  return MIREC_OK;
}
