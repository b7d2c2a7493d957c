// Subset construction for the secret-scan DFAs.  See dfa.hpp for the semantics.
#include "dfa.hpp"

#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <unordered_map>

namespace tsg {

namespace {

struct ByteEdge {
  uint8_t lo, hi;
  uint32_t to;
};

struct NNode {
  std::vector<uint32_t> eps;
  std::vector<std::pair<uint32_t, uint32_t>> asserts;  // (EmptyOp, target)
  std::vector<ByteEdge> bytes;
  int match = -1;
};

struct NFA {
  std::vector<NNode> n;
  uint32_t start = 0;
  bool need_word = false, need_nl = false, need_bot = false, any_assert = false;
  int nregex = 0;

  uint32_t add() {
    n.emplace_back();
    return (uint32_t)n.size() - 1;
  }
};

// ---- UTF-8 range splitting (rune range -> sequences of byte ranges)
void encode(int32_t r, uint8_t* b, int* len) {
  if (r < 0x80) {
    b[0] = (uint8_t)r;
    *len = 1;
  } else if (r < 0x800) {
    b[0] = 0xC0 | (r >> 6);
    b[1] = 0x80 | (r & 0x3F);
    *len = 2;
  } else if (r < 0x10000) {
    b[0] = 0xE0 | (r >> 12);
    b[1] = 0x80 | ((r >> 6) & 0x3F);
    b[2] = 0x80 | (r & 0x3F);
    *len = 3;
  } else {
    b[0] = 0xF0 | (r >> 18);
    b[1] = 0x80 | ((r >> 12) & 0x3F);
    b[2] = 0x80 | ((r >> 6) & 0x3F);
    b[3] = 0x80 | (r & 0x3F);
    *len = 4;
  }
}

using Seq = std::vector<std::pair<uint8_t, uint8_t>>;

void split_same_len(int32_t lo, int32_t hi, std::vector<Seq>* out) {
  uint8_t a[4], b[4];
  int la, lb;
  encode(lo, a, &la);
  encode(hi, b, &lb);
  for (int i = 1; i < la; i++) {
    int32_t m = (1 << (6 * i)) - 1;
    if ((lo & ~m) != (hi & ~m)) {
      if ((lo & m) != 0) {
        split_same_len(lo, lo | m, out);
        split_same_len((lo | m) + 1, hi, out);
        return;
      }
      if ((hi & m) != m) {
        split_same_len(lo, (hi & ~m) - 1, out);
        split_same_len(hi & ~m, hi, out);
        return;
      }
    }
  }
  Seq s;
  for (int k = 0; k < la; k++) s.push_back({a[k], b[k]});
  out->push_back(s);
}

void split_range(int32_t lo, int32_t hi, std::vector<Seq>* out) {
  const int32_t bounds[][2] = {{0, 0x7F}, {0x80, 0x7FF}, {0x800, 0xD7FF},
                               {0xE000, 0xFFFF}, {0x10000, 0x10FFFF}};
  for (auto& bd : bounds) {
    int32_t a = std::max(lo, bd[0]), b = std::min(hi, bd[1]);
    if (a <= b) split_same_len(a, b, out);
  }
}

bool ranges_contain(const Ranges& r, int32_t c) {
  for (auto& p : r)
    if (p.first <= c && c <= p.second) return true;
  return false;
}

void add_rune_edges(NFA& nfa, uint32_t from, uint32_t to, const Ranges& r) {
  if (r.size() == 1 && r[0].first == kHighByteRune) {  // relaxed program: any byte >= 0x80
    nfa.n[from].bytes.push_back({0x80, 0xFF, to});
    return;
  }
  std::vector<Seq> seqs;
  for (auto& p : r) split_range(p.first, p.second, &seqs);
  for (auto& s : seqs) {
    uint32_t cur = from;
    for (size_t k = 0; k < s.size(); k++) {
      uint32_t nx = (k + 1 == s.size()) ? to : nfa.add();
      nfa.n[cur].bytes.push_back({s[k].first, s[k].second, nx});
      cur = nx;
    }
  }
  // an invalid byte decodes to one U+FFFD rune of width 1
  if (ranges_contain(r, kRuneError)) nfa.n[from].bytes.push_back({0x80, 0xFF, to});
}

void add_prog(NFA& nfa, const Prog& p, int id, uint32_t union_start) {
  uint32_t base = (uint32_t)nfa.n.size();
  for (size_t k = 0; k < p.inst.size(); k++) nfa.add();
  for (size_t k = 0; k < p.inst.size(); k++) {
    const Inst& in = p.inst[k];
    uint32_t me = base + (uint32_t)k;
    switch (in.op) {
      case Op::Fail:
        break;
      case Op::Alt:
        nfa.n[me].eps.push_back(base + in.out);
        nfa.n[me].eps.push_back(base + in.arg);
        break;
      case Op::Cap:
      case Op::Nop:
        nfa.n[me].eps.push_back(base + in.out);
        break;
      case Op::Empty:
        nfa.n[me].asserts.push_back({in.arg, base + in.out});
        nfa.any_assert = true;
        if (in.arg & kBeginLine) nfa.need_nl = true;
        if (in.arg & kBeginText) nfa.need_bot = true;
        if (in.arg & (kWordBoundary | kNoWordBoundary)) nfa.need_word = true;
        break;
      case Op::Match:
        nfa.n[me].match = id;
        break;
      case Op::Rune:
        add_rune_edges(nfa, me, base + in.out, p.runes[in.arg]);
        break;
    }
  }
  nfa.n[union_start].eps.push_back(base + p.start);
}

int64_t longest_match(const NFA& nfa) {
  std::vector<int8_t> color(nfa.n.size(), 0);
  std::vector<int64_t> memo(nfa.n.size(), -2);
  bool unbounded = false;
  std::function<int64_t(uint32_t)> go = [&](uint32_t u) -> int64_t {
    if (color[u] == 2) return memo[u];
    if (color[u] == 1) {
      unbounded = true;
      return 0;
    }
    color[u] = 1;
    int64_t best = nfa.n[u].match >= 0 ? 0 : -1;
    for (uint32_t t : nfa.n[u].eps) {
      int64_t v = go(t);
      if (v >= 0) best = std::max(best, v);
    }
    for (auto& a : nfa.n[u].asserts) {
      int64_t v = go(a.second);
      if (v >= 0) best = std::max(best, v);
    }
    for (auto& e : nfa.n[u].bytes) {
      int64_t v = go(e.to);
      if (v >= 0) best = std::max(best, v + 1);
    }
    color[u] = 2;
    memo[u] = best;
    return best;
  };
  int64_t r = go(nfa.start);
  return unbounded ? -1 : r;
}

struct KeyHash {
  size_t operator()(const std::vector<uint32_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t x : v) {
      h ^= x;
      h *= 1099511628211ull;
    }
    return (size_t)h;
  }
};

class Builder {
 public:
  Builder(NFA& nfa, const DFAOptions& opt) : nfa_(nfa), opt_(opt), mark_(nfa.n.size(), 0) {}

  std::unique_ptr<DFA> run(std::string* err) {
    auto d = std::make_unique<DFA>();
    d_ = d.get();
    d->nregex = nfa_.nregex;
    d->mask_words = std::max(1, (nfa_.nregex + 63) / 64);
    d->need_word = nfa_.need_word;
    d->need_nl = nfa_.need_nl;
    d->need_bot = nfa_.need_bot;
    d->masks.push_back(std::vector<uint64_t>(d->mask_words, 0));
    make_classes();
    for (int c = 0; c < 4; c++) d->start[c] = get_state({}, norm((Ctx)c), false);
    if (opt_.anchored) d->anchored = get_state({nfa_.start}, norm(kCtxOther), true);
    for (size_t s = 0; s < keys_.size(); s++) {
      if ((int)keys_.size() > opt_.max_states) {
        if (err) *err = "DFA state cap exceeded (" + std::to_string(opt_.max_states) + ")";
        return nullptr;
      }
      expand((uint32_t)s);
    }
    if ((int)keys_.size() > opt_.max_states) {
      if (err) *err = "DFA state cap exceeded (" + std::to_string(opt_.max_states) + ")";
      return nullptr;
    }
    d->nstates = (int)keys_.size();
    d->max_len = longest_match(nfa_);
    merge_equal_classes(d.get());
    mark_immortal(d.get());
    return d;
  }

 private:
  struct Key {
    std::vector<uint32_t> k;
    uint8_t ctx;
    bool noinject;
  };
  NFA& nfa_;
  DFAOptions opt_;
  DFA* d_ = nullptr;
  std::vector<Key> keys_;
  std::unordered_map<std::vector<uint32_t>, uint32_t, KeyHash> index_;
  std::vector<uint32_t> mark_;
  uint32_t stamp_ = 0;
  std::vector<int> rep_;  // class -> representative byte
  std::map<std::vector<uint64_t>, uint32_t> mask_index_;

  Ctx norm(Ctx c) const {
    if (c == kCtxBOT && !nfa_.need_bot) c = nfa_.need_nl ? kCtxNL : kCtxOther;
    if (c == kCtxNL && !nfa_.need_nl) c = kCtxOther;
    if (c == kCtxWord && !nfa_.need_word) c = kCtxOther;
    return c;
  }
  Ctx ctx_of_byte(uint8_t c) const {
    if (c == '\n') return norm(kCtxNL);
    if (is_word_byte(c)) return norm(kCtxWord);
    return norm(kCtxOther);
  }
  static int32_t rep_of_ctx(uint8_t c) {
    switch (c) {
      case kCtxBOT: return kEOT;
      case kCtxNL: return '\n';
      case kCtxWord: return 'a';
      default: return ' ';
    }
  }

  void make_classes() {
    // signature of a byte = the byte edges containing it (+ assertion-relevant bits)
    std::vector<const ByteEdge*> edges;
    for (auto& nd : nfa_.n)
      for (auto& e : nd.bytes) edges.push_back(&e);
    size_t words = (edges.size() + 63) / 64 + 1;
    std::vector<std::vector<uint64_t>> sig(256, std::vector<uint64_t>(words, 0));
    for (size_t k = 0; k < edges.size(); k++)
      for (int b = edges[k]->lo; b <= edges[k]->hi; b++) sig[b][k / 64] |= 1ull << (k % 64);
    for (int b = 0; b < 256; b++) {
      uint64_t extra = 0;
      if (nfa_.any_assert) {
        extra |= (b == '\n') ? 1 : 0;
        extra |= is_word_byte(b) ? 2 : 0;
      }
      sig[b][words - 1] = extra;
    }
    std::map<std::vector<uint64_t>, int> cls;
    for (int b = 0; b < 256; b++) {
      auto it = cls.find(sig[b]);
      int c;
      if (it == cls.end()) {
        c = (int)cls.size();
        cls[sig[b]] = c;
        rep_.push_back(b);
      } else {
        c = it->second;
      }
      d_->cls[b] = (uint8_t)c;
    }
    d_->nclasses = (int)rep_.size();
  }

  uint32_t get_state(std::vector<uint32_t> k, Ctx ctx, bool noinject) {
    std::vector<uint32_t> key = k;
    key.push_back(0x80000000u | ((uint32_t)ctx << 1) | (noinject ? 1u : 0u));
    auto it = index_.find(key);
    if (it != index_.end()) return it->second;
    uint32_t id = (uint32_t)keys_.size();
    index_.emplace(std::move(key), id);
    keys_.push_back(Key{std::move(k), (uint8_t)ctx, noinject});
    return id;
  }

  uint32_t intern_mask(const std::vector<uint64_t>& m) {
    bool any = false;
    for (uint64_t w : m) any |= w != 0;
    if (!any) return 0;
    auto it = mask_index_.find(m);
    if (it != mask_index_.end()) return it->second;
    uint32_t id = (uint32_t)d_->masks.size();
    d_->masks.push_back(m);
    mask_index_[m] = id;
    return id;
  }

  // closure of kernel (+ injected start) under assertions evaluated at (r1, r2)
  void closure(const Key& key, int32_t r1, int32_t r2, std::vector<uint32_t>* byte_states,
               std::vector<uint64_t>* mm) {
    ++stamp_;
    std::vector<uint32_t> stack(key.k.begin(), key.k.end());
    if (!key.noinject) stack.push_back(nfa_.start);
    mm->assign(d_->mask_words, 0);
    byte_states->clear();
    while (!stack.empty()) {
      uint32_t u = stack.back();
      stack.pop_back();
      if (mark_[u] == stamp_) continue;
      mark_[u] = stamp_;
      const NNode& nd = nfa_.n[u];
      if (nd.match >= 0) (*mm)[nd.match / 64] |= 1ull << (nd.match % 64);
      if (!nd.bytes.empty()) byte_states->push_back(u);
      for (uint32_t t : nd.eps) stack.push_back(t);
      for (auto& a : nd.asserts)
        if (empty_ok(a.first, r1, r2)) stack.push_back(a.second);
    }
  }

  void expand(uint32_t s) {
    const int nc = d_->nclasses;
    if (d_->next.size() < (size_t)(s + 1) * nc) {
      d_->next.resize((size_t)(s + 1) * nc);
      d_->acc.resize((size_t)(s + 1) * nc);
      d_->eot_acc.resize(s + 1);
      d_->to_noinject.resize(s + 1);
      d_->dead.resize(s + 1);
      d_->noinject.resize(s + 1);
    }
    Key key = keys_[s];  // copy: keys_ may grow
    int32_t r1 = rep_of_ctx(key.ctx);
    std::vector<uint32_t> bs, nxt;
    std::vector<uint64_t> mm;
    for (int c = 0; c < nc; c++) {
      uint8_t b = (uint8_t)rep_[c];
      closure(key, r1, b, &bs, &mm);
      nxt.clear();
      for (uint32_t u : bs)
        for (auto& e : nfa_.n[u].bytes)
          if (e.lo <= b && b <= e.hi) nxt.push_back(e.to);
      std::sort(nxt.begin(), nxt.end());
      nxt.erase(std::unique(nxt.begin(), nxt.end()), nxt.end());
      uint32_t t = get_state(nxt, ctx_of_byte(b), key.noinject);
      d_->next[(size_t)s * nc + c] = t;
      d_->acc[(size_t)s * nc + c] = intern_mask(mm);
    }
    closure(key, r1, kEOT, &bs, &mm);
    d_->eot_acc[s] = intern_mask(mm);
    d_->noinject[s] = key.noinject ? 1 : 0;
    d_->dead[s] = (key.noinject && key.k.empty()) ? 1 : 0;
    d_->to_noinject[s] = (key.noinject || !opt_.with_noinject) ? s : get_state(key.k, (Ctx)key.ctx, true);
  }
};

}  // namespace

// Byte classes come from the NFA's edge ranges, so bytes that every state treats alike
// can still sit in different classes (the keyword automaton's 'A' and 'a' edges are two
// ranges).  Classes whose columns are equal in every state (next state and accept mask)
// are merged, in order of first appearance: the tables shrink (the builtin keyword
// automaton 68 -> 42 classes) and nothing else changes (DFA::ctx_of reads bytes, and the
// next state already encodes each byte's context).
void merge_equal_classes(DFA* d) {
  const size_t ns = (size_t)d->nstates, nc = (size_t)d->nclasses;
  if (nc < 2 || d->next.size() < ns * nc) return;
  std::map<std::vector<uint32_t>, uint32_t> seen;
  std::vector<uint32_t> newc(nc), keep;
  std::vector<uint32_t> col(2 * ns);
  for (size_t c = 0; c < nc; c++) {
    for (size_t st = 0; st < ns; st++) {
      col[2 * st] = d->next[st * nc + c];
      col[2 * st + 1] = d->acc[st * nc + c];
    }
    auto it = seen.find(col);
    if (it == seen.end()) {
      it = seen.emplace(col, (uint32_t)keep.size()).first;
      keep.push_back((uint32_t)c);
    }
    newc[c] = it->second;
  }
  const size_t m = keep.size();
  if (m == nc) return;
  std::vector<uint32_t> next(ns * m), acc(ns * m);
  for (size_t st = 0; st < ns; st++)
    for (size_t k = 0; k < m; k++) {
      next[st * m + k] = d->next[st * nc + keep[k]];
      acc[st * m + k] = d->acc[st * nc + keep[k]];
    }
  d->next.swap(next);
  d->acc.swap(acc);
  for (int b = 0; b < 256; b++) d->cls[b] = (uint8_t)newc[d->cls[b]];
  d->nclasses = (int)m;
}

// immortal = noinject and unable to reach a dead state (backward search from the dead
// states over the transitions; noinject states only lead to noinject states)
void mark_immortal(DFA* d) {
  const size_t ns = (size_t)d->nstates, nc = (size_t)d->nclasses;
  std::vector<std::vector<uint32_t>> pred(ns);
  for (size_t s = 0; s < ns; s++)
    if (d->noinject[s])
      for (size_t c = 0; c < nc; c++) pred[d->next[s * nc + c]].push_back((uint32_t)s);
  std::vector<uint8_t> mortal(ns, 0);
  std::vector<uint32_t> st;
  for (size_t s = 0; s < ns; s++)
    if (d->dead[s]) {
      mortal[s] = 1;
      st.push_back((uint32_t)s);
    }
  while (!st.empty()) {
    const uint32_t t = st.back();
    st.pop_back();
    for (uint32_t s : pred[t])
      if (!mortal[s]) {
        mortal[s] = 1;
        st.push_back(s);
      }
  }
  d->immortal.assign(ns, 0);
  for (size_t s = 0; s < ns; s++) d->immortal[s] = d->noinject[s] && !mortal[s];
}

Ctx DFA::ctx_of(uint8_t c, const DFA& d) {
  Ctx x = kCtxOther;
  if (c == '\n') x = kCtxNL;
  else if (is_word_byte(c)) x = kCtxWord;
  if (x == kCtxNL && !d.need_nl) x = kCtxOther;
  if (x == kCtxWord && !d.need_word) x = kCtxOther;
  return x;
}

void DFA::match_any(const uint8_t* b, size_t n, std::vector<uint64_t>* out) const {
  out->assign(mask_words, 0);
  uint32_t s = start[kCtxBOT];
  for (size_t i = 0; i < n; i++) {
    size_t e = (size_t)s * nclasses + cls[b[i]];
    uint32_t a = acc[e];
    if (a)
      for (int w = 0; w < mask_words; w++) (*out)[w] |= masks[a][w];
    s = next[e];
  }
  uint32_t a = eot_acc[s];
  if (a)
    for (int w = 0; w < mask_words; w++) (*out)[w] |= masks[a][w];
}

std::unique_ptr<DFA> build_dfa(const std::vector<const Prog*>& progs, const DFAOptions& opt,
                               std::string* err) {
  NFA nfa;
  nfa.start = nfa.add();
  nfa.nregex = (int)progs.size();
  for (size_t i = 0; i < progs.size(); i++) add_prog(nfa, *progs[i], (int)i, nfa.start);
  Builder b(nfa, opt);
  return b.run(err);
}

std::unique_ptr<DFA> build_reverse_dfa(const Prog& prog, const DFAOptions& opt, std::string* err) {
  NFA fwd;
  fwd.start = fwd.add();
  fwd.nregex = 1;
  add_prog(fwd, prog, 0, fwd.start);
  NFA rev;
  rev.n.resize(fwd.n.size());
  rev.nregex = 1;
  for (uint32_t u = 0; u < fwd.n.size(); u++) {
    const NNode& nd = fwd.n[u];
    for (uint32_t t : nd.eps) rev.n[t].eps.push_back(u);
    for (auto& a : nd.asserts) rev.n[a.second].eps.push_back(u);
    for (auto& e : nd.bytes) rev.n[e.to].bytes.push_back({e.lo, e.hi, u});
  }
  rev.start = rev.add();
  for (uint32_t u = 0; u < fwd.n.size(); u++)
    if (fwd.n[u].match >= 0) rev.n[rev.start].eps.push_back(u);
  rev.n[fwd.start].match = 0;
  DFAOptions o = opt;
  o.with_noinject = false;
  o.anchored = true;
  Builder b(rev, o);
  return b.run(err);
}

void DFA::pack() {
  packed.assign(next.size(), 0);
  for (size_t i = 0; i < next.size(); i++)
    packed[i] = next[i] * (uint32_t)nclasses | (acc[i] ? 1u << 31 : 0u) | (dead[next[i]] ? 1u << 30 : 0u);
}

int64_t reverse_match_start(const DFA& d, const uint8_t* b, int64_t e) {
  const int nc = d.nclasses;
  if (!d.packed.empty()) {  // one load per byte: row, accept and dead flags together
    uint32_t row = d.anchored * (uint32_t)nc;
    int64_t best = -1;
    for (int64_t q = e; q > 0; q--) {
      const uint32_t x = d.packed[row + d.cls[b[q - 1]]];
      if (x >> 31) best = q;
      row = x & 0x3FFFFFFFu;
      if (x & (1u << 30)) return best;
    }
    if (d.eot_acc[row / (uint32_t)nc]) best = 0;
    return best;
  }
  uint32_t s = d.anchored;
  int64_t best = -1;
  int64_t q = e;
  for (; q > 0; q--) {
    const size_t i = (size_t)s * nc + d.cls[b[q - 1]];
    if (d.acc[i]) best = q;
    s = d.next[i];
    if (d.dead[s]) return best;
  }
  if (d.eot_acc[s]) best = 0;
  return best;
}

int64_t max_match_len(const Prog& prog) {
  NFA nfa;
  nfa.start = nfa.add();
  nfa.nregex = 1;
  add_prog(nfa, prog, 0, nfa.start);
  return longest_match(nfa);
}

std::unique_ptr<DFA> build_keyword_dfa(const std::vector<std::string>& kws, const DFAOptions& opt,
                                       std::string* err) {
  NFA nfa;
  nfa.start = nfa.add();
  nfa.nregex = (int)kws.size();
  for (size_t i = 0; i < kws.size(); i++) {
    const std::string& k = kws[i];
    if (k.empty()) {
      nfa.n[nfa.start].match = (int)i;  // "" is contained in everything
      continue;
    }
    if (k == never_literal()) continue;
    uint32_t cur = nfa.start;
    for (size_t j = 0; j < k.size(); j++) {
      uint8_t c = (uint8_t)k[j];
      if (c >= 'A' && c <= 'Z') c += 32;  // every literal ASCII case-folded (see above)
      uint32_t nx = nfa.add();
      nfa.n[cur].bytes.push_back({c, c, nx});
      if (c >= 'a' && c <= 'z') nfa.n[cur].bytes.push_back({(uint8_t)(c - 32), (uint8_t)(c - 32), nx});
      cur = nx;
    }
    nfa.n[cur].match = (int)i;
  }
  Builder b(nfa, opt);
  return b.run(err);
}

}  // namespace tsg
