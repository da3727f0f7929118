// gen.cpp -- synthetic edit histories (see gen.h).  Input generation only.
#include "gen.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t mix(uint64_t x) { return splitmix64(x); }

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { return splitmix64(s); }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
};

uint32_t bits_for(uint64_t v) {
  uint32_t b = 0;
  while (v >> b) b++;
  return b;
}

// A pool with O(1) random pick, insert and removal by value.
struct Pool {
  std::vector<uint32_t> items, where;
  void reset(size_t n) {
    items.clear();
    where.assign(n, UINT32_MAX);
  }
  bool has(uint32_t v) const { return where[v] != UINT32_MAX; }
  void add(uint32_t v) {
    where[v] = (uint32_t)items.size();
    items.push_back(v);
  }
  void del(uint32_t v) {
    uint32_t i = where[v], last = items.back();
    items[i] = last;
    where[last] = i;
    items.pop_back();
    where[v] = UINT32_MAX;
  }
};

enum { K_NORMAL = 0, K_HIDE = 1, K_HHIDE = 2, K_HSHOW = 3, K_ROOT = 4 };

struct DocGen {
  std::vector<uint32_t> ts, site, cause, next, order;
  std::vector<uint8_t> kind;
  std::vector<uint32_t> nonspecial;  // every non-special node (root included)
  Pool visible, hidden;

  void run(const cwg_params &p, uint64_t d, uint32_t site_bits, uint64_t *idk, uint64_t *ck,
           uint8_t *kd) {
    const uint32_t n = p.nodes_per_doc + 1;
    ts.assign(n, 0);
    site.assign(n, 0);
    cause.assign(n, 0);
    kind.assign(n, 0);
    next.assign(n, UINT32_MAX);
    nonspecial.clear();
    visible.reset(n);
    hidden.reset(n);
    Rng rng(mix(p.seed ^ d));
    std::vector<uint32_t> clock(p.n_sites + 1, 0), last(p.n_sites + 1, UINT32_MAX);
    kind[0] = K_ROOT;
    nonspecial.push_back(0);
    uint32_t tail = 0;  // last node of the weave (F4 insertion keeps it exactly)
    for (uint32_t m = 1; m < n; m++) {
      const uint32_t s = 1 + rng.below(p.n_sites);
      const double u = rng.uni();
      uint32_t c;
      uint8_t k;
      if (u < p.p_hide && !visible.items.empty()) {
        k = K_HIDE;
        c = visible.items[rng.below((uint32_t)visible.items.size())];
        visible.del(c);
        hidden.add(c);
      } else if (u < p.p_hide + p.p_show && !hidden.items.empty()) {
        k = K_HSHOW;
        c = hidden.items[rng.below((uint32_t)hidden.items.size())];
        hidden.del(c);
        visible.add(c);
      } else {
        k = K_NORMAL;
        const double q = rng.uni();
        if (q < p.p_conj) c = tail;
        else if (q < p.p_conj + p.p_chain && last[s] != UINT32_MAX) c = last[s];
        else c = nonspecial[rng.below((uint32_t)nonspecial.size())];
      }
      const uint32_t t = std::max(clock[s], ts[c]) + 1;
      clock[s] = t;
      ts[m] = t;
      site[m] = s;
      cause[m] = c;
      kind[m] = k;
      if (k == K_NORMAL) {
        nonspecial.push_back(m);
        visible.add(m);
        last[s] = m;
      }
      // keep the weave's tail for conj-style causes (SURVEY F4 insertion)
      uint32_t at = c;
      if (k == K_NORMAL)
        while (next[at] != UINT32_MAX && kind[next[at]] != K_NORMAL && kind[next[at]] != K_ROOT)
          at = next[at];
      next[m] = next[at];
      next[at] = m;
      if (at == tail) tail = m;
      if (p.sync_every && m % p.sync_every == 0) {
        uint32_t mx = 0;
        for (uint32_t x : clock) mx = std::max(mx, x);
        std::fill(clock.begin(), clock.end(), mx);
      }
    }
    order.resize(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    if (p.shuffle)
      for (uint32_t i = n - 1; i > 0; i--) std::swap(order[i], order[rng.below(i + 1)]);
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t i = order[j];
      idk[j] = ((uint64_t)ts[i] << site_bits) | site[i];
      ck[j] = i == 0 ? UINT64_MAX : (((uint64_t)ts[cause[i]] << site_bits) | site[cause[i]]);
      kd[j] = kind[i];
    }
  }
};

}  // namespace

extern "C" {

void cwg_layout(const cwg_params *p, uint32_t *ts_bits, uint32_t *site_bits) {
  *ts_bits = bits_for(p->nodes_per_doc);  // ts <= number of non-root nodes
  *site_bits = bits_for(p->n_sites);
}

int cwg_generate(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, uint64_t *id_key,
                 uint64_t *cause_key, uint8_t *kind, int nthreads) {
  if (!p || doc_end < doc_begin || p->n_sites == 0) return -1;
  uint32_t tsb, sb;
  cwg_layout(p, &tsb, &sb);
  const uint64_t n = (uint64_t)p->nodes_per_doc + 1;
  std::atomic<uint64_t> next{doc_begin};
  auto work = [&]() {
    DocGen g;
    for (;;) {
      const uint64_t d = next.fetch_add(1);
      if (d >= doc_end) break;
      const uint64_t o = (d - doc_begin) * n;
      g.run(*p, d, sb, id_key + o, cause_key + o, kind + o);
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; t++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  return 0;
}

}  // extern "C"
