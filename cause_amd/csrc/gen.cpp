// gen.cpp -- synthetic edit histories (see gen.h).  Input generation only.
#include "gen.h"

#include <algorithm>
#include <atomic>
#include <cmath>
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

  // K = uint64_t (K64 keys, nil = all ones) or uint32_t (K32 keys, nil = CW_NIL32)
  template <typename K>
  void run(const cwg_params &p, uint64_t d, uint32_t site_bits, K *idk, K *ck, uint8_t *kd) {
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
      idk[j] = (K)(((uint64_t)ts[i] << site_bits) | site[i]);
      ck[j] = i == 0 ? (K)~(K)0 : (K)(((uint64_t)ts[cause[i]] << site_bits) | site[cause[i]]);
      kd[j] = kind[i];
    }
  }
};

struct MapGen {
  std::vector<uint32_t> ts, site, order, values, idcaused, cnode;
  std::vector<uint64_t> token;
  std::vector<uint8_t> cis, kind;

  void run(const cwg_map_params &p, const std::vector<double> &cdf, uint64_t d, uint32_t site_bits,
           uint64_t *idk, uint64_t *ck, uint8_t *ci, uint8_t *kd) {
    const uint32_t n = p.nodes_per_coll;
    ts.assign(n, 0);
    site.assign(n, 0);
    cnode.assign(n, 0);
    token.assign(n, 0);
    cis.assign(n, 0);
    kind.assign(n, 0);
    values.clear();
    idcaused.clear();
    Rng rng(mix(p.seed ^ (d * 0x2545F4914F6CDD1Dull)));
    std::vector<uint32_t> clock(p.n_sites + 1, 0);
    auto pick_key = [&]() {
      const double u = rng.uni() * cdf.back();
      return (uint64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    };
    const double q_id = p.p_hhide + p.p_hshow, q_bad = q_id + p.p_bad, q_hide = q_bad + p.p_hide;
    for (uint32_t m = 0; m < n; m++) {
      const uint32_t s = 1 + rng.below(p.n_sites);
      const double u = rng.uni();
      uint32_t cts = 0;
      if (u < q_id && !values.empty()) {
        const uint32_t c = values[rng.below((uint32_t)values.size())];
        kind[m] = u < p.p_hhide ? K_HHIDE : K_HSHOW;
        cis[m] = 1;
        cnode[m] = c;
        cts = ts[c];
        idcaused.push_back(m);
      } else if (u >= q_id && u < q_bad && !idcaused.empty()) {
        const uint32_t c = idcaused[rng.below((uint32_t)idcaused.size())];
        kind[m] = K_HHIDE;
        cis[m] = 1;
        cnode[m] = c;
        cts = ts[c];
      } else {
        kind[m] = (u >= q_bad && u < q_hide) ? K_HIDE : K_NORMAL;
        token[m] = pick_key();
        if (kind[m] == K_NORMAL) values.push_back(m);
      }
      const uint32_t t = std::max(clock[s], cts) + 1;
      clock[s] = t;
      ts[m] = t;
      site[m] = s;
      if (p.sync_every && (m + 1) % p.sync_every == 0) {
        uint32_t mx = 0;
        for (uint32_t x : clock) mx = std::max(mx, x);
        std::fill(clock.begin(), clock.end(), mx);
      }
    }
    order.resize(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    if (p.shuffle && n > 1)
      for (uint32_t i = n - 1; i > 0; i--) std::swap(order[i], order[rng.below(i + 1)]);
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t i = order[j];
      idk[j] = ((uint64_t)ts[i] << site_bits) | site[i];
      ck[j] = cis[i] ? (((uint64_t)ts[cnode[i]] << site_bits) | site[cnode[i]]) : token[i];
      ci[j] = cis[i];
      kd[j] = kind[i];
    }
  }
};

}  // namespace

extern "C" {

void cwg_map_layout(const cwg_map_params *p, uint32_t *ts_bits, uint32_t *site_bits,
                    uint32_t *token_bits) {
  *ts_bits = bits_for(p->nodes_per_coll);
  *site_bits = bits_for(p->n_sites);
  *token_bits = std::max<uint32_t>(1, bits_for(p->n_keys ? p->n_keys - 1 : 0));
}

int cwg_map_generate(const cwg_map_params *p, uint64_t coll_begin, uint64_t coll_end,
                     uint64_t *id_key, uint64_t *cause, uint8_t *cause_is_id, uint8_t *kind,
                     int nthreads) {
  if (!p || coll_end < coll_begin || p->n_sites == 0 || p->n_keys == 0) return -1;
  uint32_t tsb, sb, tb;
  cwg_map_layout(p, &tsb, &sb, &tb);
  std::vector<double> cdf(p->n_keys);
  double acc = 0;
  for (uint32_t k = 0; k < p->n_keys; k++) {
    acc += 1.0 / std::pow((double)(k + 1), p->zipf_s);
    cdf[k] = acc;
  }
  const uint64_t n = p->nodes_per_coll;
  std::atomic<uint64_t> next{coll_begin};
  auto work = [&]() {
    MapGen g;
    for (;;) {
      const uint64_t d = next.fetch_add(1);
      if (d >= coll_end) break;
      const uint64_t o = (d - coll_begin) * n;
      g.run(*p, cdf, d, sb, id_key + o, cause + o, cause_is_id + o, kind + o);
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; t++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  return 0;
}


void cwg_layout(const cwg_params *p, uint32_t *ts_bits, uint32_t *site_bits) {
  *ts_bits = bits_for(p->nodes_per_doc);  // ts <= number of non-root nodes
  *site_bits = bits_for(p->n_sites);
}

}  // extern "C"

template <typename K>
static int gen_docs(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, K *id_key,
                    K *cause_key, uint8_t *kind, int nthreads) {
  if (!p || doc_end < doc_begin || p->n_sites == 0) return -1;
  uint32_t tsb, sb;
  cwg_layout(p, &tsb, &sb);
  if (sizeof(K) == 4 && tsb + sb > 31) return -1;  // K32: every key below CW_K32_RESERVED
  const uint64_t n = (uint64_t)p->nodes_per_doc + 1;
  std::atomic<uint64_t> next{doc_begin};
  auto work = [&]() {
    DocGen g;
    for (;;) {
      const uint64_t d = next.fetch_add(1);
      if (d >= doc_end) break;
      const uint64_t o = (d - doc_begin) * n;
      g.run<K>(*p, d, sb, id_key + o, cause_key + o, kind + o);
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; t++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  return 0;
}

extern "C" {

int cwg_generate(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, uint64_t *id_key,
                 uint64_t *cause_key, uint8_t *kind, int nthreads) {
  return gen_docs<uint64_t>(p, doc_begin, doc_end, id_key, cause_key, kind, nthreads);
}

int cwg_generate32(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, uint32_t *id_key,
                   uint32_t *cause_key, uint8_t *kind, int nthreads) {
  return gen_docs<uint32_t>(p, doc_begin, doc_end, id_key, cause_key, kind, nthreads);
}

}  // extern "C"
