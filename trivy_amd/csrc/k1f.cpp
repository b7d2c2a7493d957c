// K1F tables (k1f.hpp): each literal's window, the 16 buckets, the per-byte entries and the
// verification image; and a CPU emulation of k1f_kernel for the tests.
#include "k1f.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

namespace tsg {

namespace {

const uint32_t kBigram[] = {
#include "bigram.inc"
};

uint8_t fold(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

// First-order Markov model of source text over ASCII-lowercased bytes (bigram.inc): the
// expected number of windows per byte of text that a bucket's four position sets accept.
struct TextModel {
  std::vector<double> pi;     // [256]
  std::vector<double> trans;  // [256 * 256] P(b | a)
  TextModel() : pi(256, 0), trans(256 * 256, 0) {
    std::vector<double> cnt(256 * 256, 0.01);  // smoothing: every bigram is possible
    for (uint32_t e : kBigram) cnt[(e & 0xFF) * 256 + ((e >> 8) & 0xFF)] += std::exp2((double)(e >> 16) / 16.0) - 1.0;
    double tot = 0;
    for (int a = 0; a < 256; a++) {
      double row = 0;
      for (int b = 0; b < 256; b++) row += cnt[a * 256 + b];
      for (int b = 0; b < 256; b++) trans[a * 256 + b] = cnt[a * 256 + b] / row;
      pi[a] = row;
      tot += row;
    }
    for (double& x : pi) x /= tot;
  }
};

const TextModel& model() {
  static const TextModel m;
  return m;
}

// Position sets of a window (lowercased bytes; an empty set = "any").
struct Win {
  std::vector<uint8_t> s[4];
};

Win win_union(const Win& a, const Win& b) {
  Win u;
  for (int j = 0; j < 4; j++) {
    if (a.s[j].empty() || b.s[j].empty()) continue;  // "any" absorbs
    u.s[j] = a.s[j];
    u.s[j].insert(u.s[j].end(), b.s[j].begin(), b.s[j].end());
    std::sort(u.s[j].begin(), u.s[j].end());
    u.s[j].erase(std::unique(u.s[j].begin(), u.s[j].end()), u.s[j].end());
  }
  return u;
}

double win_cost(const Win& w) {
  const TextModel& m = model();
  double v[256], nv[256];
  for (int b = 0; b < 256; b++) v[b] = w.s[0].empty() ? m.pi[b] : 0.0;
  for (uint8_t b : w.s[0]) v[b] = m.pi[b];
  for (int j = 1; j < 4; j++) {
    std::fill(nv, nv + 256, 0.0);
    std::vector<int> src;
    for (int a = 0; a < 256; a++)
      if (v[a] > 0) src.push_back(a);
    auto step = [&](int b) {
      double s = 0;
      for (int a : src) s += v[a] * m.trans[a * 256 + b];
      nv[b] = s;
    };
    if (w.s[j].empty())
      for (int b = 0; b < 256; b++) step(b);
    else
      for (uint8_t b : w.s[j]) step(b);
    std::copy(nv, nv + 256, v);
  }
  double s = 0;
  for (int b = 0; b < 256; b++) s += v[b];
  return s;
}

// Exact n-gram counts of a sample of the data (ASCII lowercased): what a bucket's position
// sets accept there, for the adaptation's rebuild.  A window's "any" positions are always a
// prefix (a short literal's window ends at its last byte), so a bucket with a of them is
// priced by the (4 - a)-grams of its other positions.
struct Grams {
  // open addressing, u32 key -> count (count 0 = empty)
  struct Map {
    std::vector<uint32_t> key, cnt;
    uint32_t mask = 0;
    void init(size_t n) {
      size_t cap = 1024;
      while (cap < 2 * n) cap *= 2;
      key.assign(cap, 0);
      cnt.assign(cap, 0);
      mask = (uint32_t)cap - 1;
    }
    uint32_t slot(uint32_t k) const {
      uint32_t h = (k * 0x9E3779B1u) & mask;
      while (cnt[h] && key[h] != k) h = (h + 1) & mask;
      return h;
    }
    void add(uint32_t k) {
      const uint32_t h = slot(k);
      key[h] = k;
      cnt[h]++;
    }
    uint32_t get(uint32_t k) const { return cnt[slot(k)]; }
  };
  std::vector<uint32_t> h1, h2;  // [256], [65536]
  Map h3, h4;
  uint64_t n = 0;
  Grams(const uint8_t* d, size_t len) : h1(256, 0), h2(65536, 0) {
    std::vector<uint8_t> l(len);
    for (size_t i = 0; i < len; i++) l[i] = fold(d[i]);
    n = len;
    h3.init(len);
    h4.init(len);
    for (size_t i = 0; i < len; i++) {
      h1[l[i]]++;
      if (i >= 1) h2[l[i - 1] | l[i] << 8]++;
      if (i >= 2) h3.add(l[i - 2] | l[i - 1] << 8 | (uint32_t)l[i] << 16);
      if (i >= 3) h4.add(l[i - 3] | l[i - 2] << 8 | (uint32_t)l[i - 1] << 16 | (uint32_t)l[i] << 24);
    }
  }
  // windows of the sample that the position sets accept; < 0 when there are too many
  // combinations to enumerate
  double count(const Win& w) const {
    int a = 0;
    while (a < 4 && w.s[a].empty()) a++;
    if (a == 4) return (double)n;
    double combos = 1;
    for (int j = a; j < 4; j++) combos *= (double)w.s[j].size();
    if (combos > 65536) return -1;
    double tot = 0;
    uint32_t idx[4] = {0, 0, 0, 0};
    for (;;) {
      uint32_t key = 0;
      for (int j = a; j < 4; j++) key |= (uint32_t)w.s[j][idx[j]] << (8 * (j - a));
      tot += a == 0 ? h4.get(key) : a == 1 ? h3.get(key) : a == 2 ? h2[key] : h1[key];
      int j = 3;
      while (j >= a && ++idx[j] == w.s[j].size()) idx[j--] = 0;
      if (j < a) break;
    }
    return tot;
  }
};

Win lit_window(const std::string& l, int j0) {
  Win w;
  for (int j = 0; j < 4; j++)
    if (j0 + j >= 0) w.s[j].push_back(fold((uint8_t)l[j0 + j]));
  return w;
}

}  // namespace

bool k1f_build(const Plan& p, const std::vector<uint8_t>& quiet, K1FTables* t, std::string* why,
               const uint8_t* sample, size_t sample_len) {
  auto no = [&](const char* r) {
    if (why) *why = r;
    return false;
  };
  const int n = p.n_lit;
  if (!p.kw_dfa || (int)p.k1_lits.size() != n) return no("no K1 literal list");
  if (p.run_k[0] != kFRunU || p.run_k[1] != kFRunD) return no("run lengths other than 32 / 12");
  std::vector<int> act;
  for (int i = 0; i < n; i++) {
    if (p.k1_lits[i].empty()) return no("an empty literal");
    if (p.k1_lits[i].size() > 0xFFFF) return no("a literal longer than 65535 bytes");
    if ((quiet.empty() || !quiet[i]) && p.k1_lits[i] != never_literal()) act.push_back(i);
  }
  if (act.size() > 400) return no("more than 400 literals");
  // The price of a bucket: its expected windows per byte under the text model, or with a
  // sample of the data its exact count there plus a tenth of the model's expectation (which
  // orders the windows the sample never holds)
  std::unique_ptr<Grams> grams;
  if (sample && sample_len >= 4096) grams = std::make_unique<Grams>(sample, sample_len);
  auto win_price = [&](const Win& w) {
    const double m = win_cost(w);
    if (!grams) return m;
    const double c = grams->count(w);
    return (c < 0 ? m * (double)grams->n : c) + 0.1 * m * (double)grams->n;
  };
  // each literal's window: the cheapest
  t->j0.assign(n, 0);
  t->bucket_of.assign(n, -1);
  std::vector<Win> win(act.size());
  for (size_t a = 0; a < act.size(); a++) {
    const std::string& l = p.k1_lits[act[a]];
    const int len = (int)l.size();
    int best = len < 4 ? len - 4 : 0;
    double bc = win_price(lit_window(l, best));
    for (int j0 = best + 1; len >= 4 && j0 <= len - 4; j0++) {
      const double c = win_price(lit_window(l, j0));
      if (c < bc) {
        bc = c;
        best = j0;
      }
    }
    t->j0[act[a]] = best;
    win[a] = lit_window(l, best);
  }
  // buckets: agglomerative, merging the two groups whose union adds the least expected cost
  std::vector<std::vector<int>> grp;
  std::vector<Win> gw;
  std::vector<double> gc;
  for (size_t a = 0; a < act.size(); a++) {
    grp.push_back({(int)a});
    gw.push_back(win[a]);
    gc.push_back(win_price(win[a]));
  }
  const size_t G0 = grp.size();
  std::vector<double> pc(G0 * G0, 0);  // merge cost of (x, y), x < y, by slot
  auto pair_cost = [&](size_t x, size_t y) { return win_price(win_union(gw[x], gw[y])) - gc[x] - gc[y]; };
  pool_for(G0, 16, [&](size_t x) {
    for (size_t y = x + 1; y < G0; y++) pc[x * G0 + y] = pair_cost(x, y);
  }, 1);
  std::vector<char> alive(G0, 1);
  size_t ngroups = G0;
  while (ngroups > (size_t)kFBuckets) {
    double best = 0;
    size_t bx = 0, by = 0;
    bool have = false;
    for (size_t x = 0; x < G0; x++) {
      if (!alive[x]) continue;
      for (size_t y = x + 1; y < G0; y++)
        if (alive[y] && (!have || pc[x * G0 + y] < best)) {
          best = pc[x * G0 + y];
          bx = x;
          by = y;
          have = true;
        }
    }
    grp[bx].insert(grp[bx].end(), grp[by].begin(), grp[by].end());
    gw[bx] = win_union(gw[bx], gw[by]);
    gc[bx] = win_price(gw[bx]);
    alive[by] = 0;
    ngroups--;
    pool_for(G0, 16, [&](size_t z) {
      if (alive[z] && z != bx) pc[std::min(z, bx) * G0 + std::max(z, bx)] = pair_cost(std::min(z, bx), std::max(z, bx));
    }, 8);
  }
  std::vector<std::vector<int>> buckets;  // literal slots (into act) per bucket
  for (size_t x = 0; x < G0; x++)
    if (alive[x]) buckets.push_back(grp[x]);
  // entries
  t->ent.assign(256 * 4, 0);
  for (int b = 0; b < 256; b++) {
    const uint8_t fb = fold((uint8_t)b);
    const bool u = p.run_cls[b] & 1, d = (p.run_cls[b] & 2) != 0;
    for (int j = 0; j < 4; j++) {
      uint32_t lo = 0;
      for (size_t k = 0; k < buckets.size(); k++) {
        bool acc = false;
        for (int a : buckets[k]) {
          const Win& w = win[a];
          acc |= w.s[j].empty() || w.s[j][0] == fb;
        }
        if (acc) lo |= 1u << k;
      }
      const uint32_t hi = (0xFFFFu & ~(0x11u << j)) | (u ? 1u << j : 0u) | (d ? 0x10u << j : 0u);
      t->ent[b * 4 + j] = lo | hi << 16;
    }
  }
  // verification image: bucket starts | records (bucket order) | literal bytes
  std::vector<K1FLit> recs;
  std::vector<uint16_t> bstart;
  std::vector<uint8_t> bytes;
  for (size_t k = 0; k < buckets.size(); k++) {
    bstart.push_back((uint16_t)recs.size());
    for (int a : buckets[k]) {
      const int id = act[a];
      const std::string& l = p.k1_lits[id];
      K1FLit r{};
      const int j0 = t->j0[id];
      for (int j = 0; j < 4; j++)
        if (j0 + j >= 0) {
          r.wkey |= (uint32_t)fold((uint8_t)l[j0 + j]) << (8 * j);
          r.wmask |= 0xFFu << (8 * j);
        }
      r.wend = (uint16_t)(j0 + 3);
      r.len = (uint16_t)l.size();
      r.boff = (uint32_t)bytes.size();
      for (char c : l) bytes.push_back(fold((uint8_t)c));
      bytes.resize((bytes.size() + 3) / 4 * 4, 0);
      r.kw = id < p.n_kw ? id : -1;
      r.ev = p.lit_event[id];
      r.id = (uint32_t)id;
      recs.push_back(r);
      t->bucket_of[id] = (int)k;
    }
  }
  while (bstart.size() <= (size_t)kFBuckets) bstart.push_back((uint16_t)recs.size());
  const uint32_t o_bytes = kFImgLits + (uint32_t)recs.size() * (uint32_t)sizeof(K1FLit);
  t->img.assign(o_bytes + bytes.size(), 0);
  std::memcpy(t->img.data(), bstart.data(), bstart.size() * 2);
  for (auto& r : recs) r.boff += o_bytes;
  if (!recs.empty()) std::memcpy(t->img.data() + kFImgLits, recs.data(), recs.size() * sizeof(K1FLit));
  if (!bytes.empty()) std::memcpy(t->img.data() + o_bytes, bytes.data(), bytes.size());
  t->img.resize((t->img.size() + 15) / 16 * 16, 0);
  if (t->img.size() > kFImgMax) return no("verification image larger than its LDS budget");
  t->nlit = (uint32_t)recs.size();
  return true;
}

// ------------------------------------------------------------------ CPU emulation
void k1f_emulate(const Plan& p, const K1FTables& t, const BatchView& bv, uint32_t chunk,
                 std::vector<uint32_t>* kw, std::vector<uint32_t>* ev, uint64_t stats[2]) {
  const uint32_t F = bv.nfiles;
  const uint64_t total = bv.offsets[F];
  const int W = p.kw_words;
  kw->assign((size_t)F * W, 0);
  ev->assign((total + chunk - 1) / chunk, 0);
  stats[0] = stats[1] = 0;
  auto byte = [&](int64_t q) -> uint8_t { return (q < 0 || (uint64_t)q >= total) ? 0 : bv.data[q]; };
  auto d = [&](uint8_t b, int j) { return t.ent[b * 4 + j]; };
  auto R = [&](int64_t q) {
    return k1f_and3(d(byte(q - 3), 0), d(byte(q - 2), 1), d(byte(q - 1), 2)) & d(byte(q), 3);
  };
  const uint16_t* bstart = (const uint16_t*)t.img.data();
  const K1FLit* recs = (const K1FLit*)(t.img.data() + kFImgLits);
  auto load4 = [&](int64_t q) {  // bytes q..q+3
    return (uint32_t)byte(q) | (uint32_t)byte(q + 1) << 8 | (uint32_t)byte(q + 2) << 16 | (uint32_t)byte(q + 3) << 24;
  };
  // verification of the window ending at q (bucket mask bm), as the kernel does it
  auto verify = [&](uint64_t q, uint32_t bm) {
    const uint32_t w = k1f_lower4(load4((int64_t)q - 3));
    for (; bm; bm &= bm - 1) {
      const uint32_t k = k1f_ctz(bm);
      for (uint32_t i = bstart[k]; i < bstart[k + 1]; i++) {
        const K1FLit& L = recs[i];
        if ((w & L.wmask) != L.wkey || q < L.wend) continue;
        const uint64_t s = q - L.wend, e = s + L.len - 1;
        if (e >= total) continue;
        bool ok = true;
        for (uint32_t o = 0; o < L.len && ok; o += 4) {
          uint32_t lv;
          std::memcpy(&lv, t.img.data() + L.boff + o, 4);
          const uint32_t m = L.len - o >= 4 ? 0xFFFFFFFFu : (1u << (8 * (L.len - o))) - 1;
          ok = ((k1f_lower4(load4((int64_t)(s + o))) & m) == lv);
        }
        if (!ok) continue;
        stats[1]++;
        (*ev)[e / chunk] |= L.ev;
        if (L.kw >= 0) {
          const uint32_t f = (uint32_t)(std::upper_bound(bv.offsets, bv.offsets + F + 1, e) - bv.offsets) - 1;
          if (s >= bv.offsets[f]) (*kw)[(size_t)f * W + L.kw / 32] |= 1u << (L.kw % 32);
        }
      }
    }
  };
  uint32_t m1 = 0, m2 = 0;  // flags of the previous two words (zero bytes before the batch)
  for (uint64_t P = 0; P < total; P += 16) {
    uint32_t r[16];
    for (int k = 0; k < 16; k++) r[k] = R((int64_t)(P + k));
    // the kernel ORs four windows per group and lists the word with the group mask and
    // the union of their buckets; the verification recomputes each window of a listed group
    uint32_t any = 0;
    for (int g = 0; g < 4; g++) {
      const uint32_t gr = r[4 * g] | r[4 * g + 1] | r[4 * g + 2] | r[4 * g + 3];
      if (!(gr & 0xFFFFu)) continue;
      stats[0]++;
      any |= gr;
      for (int k = 4 * g; k < 4 * g + 4; k++)
        if (P + k < total && (r[k] & 0xFFFFu)) verify(P + k, r[k] & 0xFFFFu);
    }
    (void)any;
    const uint32_t m = k1f_flags(r[3], r[7], r[11], r[15]);
    const uint32_t rb = k1f_runs(m, m1, m2);
    if (rb) (*ev)[P / chunk] |= rb;
    m2 = m1;
    m1 = m;
  }
}

}  // namespace tsg
