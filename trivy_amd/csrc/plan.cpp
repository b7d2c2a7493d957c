// GPU plan construction, host resolver, CPU batch path and kernel emulation.
#include "plan.hpp"
#include "internal.hpp"
#include <deque>
#include <condition_variable>
#include <mutex>
#include <functional>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <set>
#include <thread>
#include <x86intrin.h>

namespace tsg {

static std::string ascii_lower(std::string s) {
  for (char& c : s)
    if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
  return s;
}

static bool is_ascii(const std::string& s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

// 4-byte strings frequent in source text (common4.inc): a K1X window on one of them costs a
// verify record per occurrence
static const std::unordered_set<uint32_t>& common4() {
  static const std::unordered_set<uint32_t> set = [] {
    static const char kCommon4[][5] = {
#include "common4.inc"
    };
    std::unordered_set<uint32_t> s;
    for (const auto& g : kCommon4) s.insert(x_prefix4((const uint8_t*)g));
    return s;
  }();
  return set;
}

// K1X windows of every literal of the plan: per literal the offset j0 whose windows hold
// the fewest common 4-grams, then are shared by the fewest other literals (a window shared
// by k literals costs k verifications per hit: 100 `begin_<name>` anchors all starting
// "begi" made every "-----BEGIN" line of a batch check 100 literals).
static void x_place_windows(Plan* p, int step) {
  std::unordered_map<uint32_t, uint32_t> mult;
  for (const auto& l : p->x_lits) {
    std::unordered_set<uint32_t> mine;
    for (size_t j = 0; j + 4 <= l.size(); j++) mine.insert(x_prefix4((const uint8_t*)l.data() + j));
    for (uint32_t g : mine) mult[g]++;
  }
  p->x_j0.assign(p->x_lits.size(), 0);
  for (size_t i = 0; i < p->x_lits.size(); i++) {
    const std::string& l = p->x_lits[i];
    const size_t last = std::min(l.size() - 3 - (size_t)step, (size_t)256 - (size_t)step);
    uint64_t best = UINT64_MAX;
    for (size_t j = 0; j <= last; j++) {
      uint64_t c = 0;
      for (size_t t = j; t < j + (size_t)step; t++) {
        const uint32_t g = x_prefix4((const uint8_t*)l.data() + t);
        c += (common4().count(g) ? 1000000u : 0u) + mult[g];
      }
      if (c < best) {
        best = c;
        p->x_j0[i] = (uint8_t)j;
      }
    }
  }
}

// K1X windows of a lowercased literal at step `step`: the first offset j0 whose windows
// j0 .. j0 + step - 1 hold the fewest common 4-grams.  Returns that count (0: a quiet
// literal), -1 when the literal is too short for the step.
static int x_pick(const std::string& l, int step, uint32_t* j0) {
  if (l.size() < (size_t)step + 3) return -1;
  const size_t last = std::min(l.size() - 3 - (size_t)step, (size_t)256 - (size_t)step);
  int best = -1;
  for (size_t j = 0; j <= last && best != 0; j++) {
    int c = 0;
    for (size_t t = j; t < j + (size_t)step; t++) c += common4().count(x_prefix4((const uint8_t*)l.data() + t)) ? 1 : 0;
    if (best < 0 || c < best) {
      best = c;
      *j0 = (uint32_t)j;
    }
  }
  return best;
}

namespace {

bool in_set(const uint64_t* set, const uint8_t* cls, int bit) {
  for (int c = 0; c < 128; c++)
    if (((set[c >> 6] >> (c & 63)) & 1) && !((cls[c] >> bit) & 1)) return false;
  return true;
}

struct Anchor {
  uint32_t kind = kEvAlways;  // kEvRunU, kEvRunD, kEvLit0 (literal), kEvAlways
  std::string lit;
  int first_atom = 0;
  int64_t evdist = 0;
  std::string desc = "none";
};

// The event every match of a rule must contain, preferring long class runs (the secret
// part of nearly every rule) over literals: the keyword gate already handles rare
// literals, and common ones ("key", "sk", "-----") would put events everywhere.  A rule
// without keywords (every file gated) takes a long literal first when it has one (score
// >= 6, e.g. a 5-byte name): token runs are common, its literal is not.
Anchor choose_anchor(const Regexp& re, const Plan& p, bool literal_first) {
  const std::vector<AtomInfo> at = re.Atoms();
  const int n = (int)at.size();
  std::vector<int64_t> B(n + 1, 0);
  for (int i = 0; i < n; i++)
    B[i + 1] = (B[i] < 0 || at[i].max_bytes < 0) ? -1 : B[i] + at[i].max_bytes;
  Anchor best;
  auto take = [&](uint32_t kind, int t, int64_t len, const std::string& lit, const char* what) {
    Anchor a;
    a.kind = kind;
    a.lit = lit;
    if (B[t] >= 0) {
      a.first_atom = 0;
      a.evdist = B[t] + len - 1;
    } else {
      a.first_atom = t;  // unbounded prefix: the GPU program is the suffix from the anchor
      a.evdist = len - 1;
    }
    a.desc = std::string(what) + (lit.empty() ? "" : " '" + lit + "'") + " at atom " +
             std::to_string(t) + (a.first_atom ? " (suffix)" : "");
    return a;
  };
  double best_score = 0;
  auto best_literal = [&]() {
    for (int i = 0; i < n;) {
      if (at[i].lit < 0) {
        i++;
        continue;
      }
      int j = i;
      std::string s;
      double score = 0;
      while (j < n && at[j].lit >= 0) {
        int c = at[j].lit;
        if (s.size() < 24) {
          s.push_back((char)c);
          score += (c >= 'a' && c <= 'z') ? 1.0 : (c >= '0' && c <= '9') ? 1.3 : 1.6;
        }
        j++;
      }
      if (score >= 3.0 && score > best_score) {
        best_score = score;
        best = take(1u << kEvLit0, i, (int64_t)s.size(), s, "literal");
      }
      i = j;
    }
  };
  if (literal_first) {
    best_literal();
    if (best_score >= 6.0) return best;
    best = Anchor();
    best_score = 0;
  }
  for (int bit = 0; bit < 2; bit++) {
    const int k = p.run_k[bit];
    for (int i = 0; i < n;) {
      if (!(at[i].ascii_only && in_set(at[i].set, p.run_cls, bit))) {
        i++;
        continue;
      }
      int j = i;
      int64_t run = 0;
      while (j < n && at[j].ascii_only && in_set(at[j].set, p.run_cls, bit)) run += at[j++].min_bytes;
      if (run >= k) return take(bit == 0 ? kEvRunU : kEvRunD, i, k, "", bit == 0 ? "run U" : "run D");
      i = j;
    }
  }
  best_literal();
  return best;
}

// Inject-mode states of the union of two DFAs' searches, counted as the reachable pairs
// of their product (each union state is a pair of component states), up to `cap`.  A
// lower bound on the states a subset construction of the merged programs builds, so
// "> cap" rejects a merge without building it.
size_t product_states(const DFA& a, const DFA& b, size_t cap) {
  std::vector<uint8_t> seen((size_t)a.nstates * b.nstates, 0);
  std::vector<std::pair<uint32_t, uint32_t>> stack;
  uint16_t pcls[256][2];
  int np = 0;
  {
    std::map<std::pair<int, int>, int> idx;
    for (int c = 0; c < 256; c++) {
      auto k = std::make_pair((int)a.cls[c], (int)b.cls[c]);
      if (!idx.count(k)) idx[k] = np++;
      pcls[c][0] = (uint16_t)a.cls[c];
      pcls[c][1] = (uint16_t)b.cls[c];
    }
  }
  std::vector<int> rep;  // one byte per joint class
  {
    std::set<std::pair<int, int>> done;
    for (int c = 0; c < 256; c++)
      if (done.insert({pcls[c][0], pcls[c][1]}).second) rep.push_back(c);
  }
  size_t n = 0;
  auto push = [&](uint32_t x, uint32_t y) {
    uint8_t& v = seen[(size_t)x * b.nstates + y];
    if (v) return;
    v = 1;
    n++;
    stack.push_back({x, y});
  };
  for (int c = 0; c < 4; c++) push(a.start[c], b.start[c]);
  while (!stack.empty() && n <= cap) {
    auto [x, y] = stack.back();
    stack.pop_back();
    for (int c : rep) push(a.next[(size_t)x * a.nclasses + pcls[c][0]], b.next[(size_t)y * b.nclasses + pcls[c][1]]);
  }
  return n;
}

}  // namespace

std::unique_ptr<Plan> build_plan(const Ruleset& rs, const PlanOptions& opt, std::string* err) {
  auto p = std::make_unique<Plan>();
  const size_t R = rs.rules.size();
  p->rule_kw_mode.assign(R, kKwAlways);
  p->rule_kws.assign(R, {});
  p->rule_group.assign(R, -1);
  p->rule_hostonly.assign(R, 0);
  p->rule_maxlen.assign(R, -1);
  p->rule_event.assign(R, kEvAlways);
  p->rule_evdist.assign(R, 0);
  p->rule_first_atom.assign(R, 0);
  p->rule_anchor.assign(R, "none");
  // run classes: U = [A-Za-z0-9+/=_.-] (secrets, tokens, base64), D = [0-9-]
  for (int c = 0; c < 256; c++) {
    bool u = (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') ||
             c == '+' || c == '/' || c == '=' || c == '_' || c == '.' || c == '-';
    bool d = (c >= '0' && c <= '9') || c == '-';
    p->run_cls[c] = (uint8_t)((u ? 1 : 0) | (d ? 2 : 0));
  }

  // ---- keywords (Rule.MatchKeywords, scanner.go:164-176)
  std::map<std::string, uint32_t> kwid;
  std::vector<std::string> kws;
  for (size_t r = 0; r < R; r++) {
    const RuleC& rule = rs.rules[r];
    if (rule.kw_lower.empty()) continue;
    bool ascii = true;
    for (const auto& k : rule.kw_lower) ascii &= is_ascii(k);
    if (!ascii) {
      p->rule_kw_mode[r] = kKwUnknown;
      continue;
    }
    p->rule_kw_mode[r] = kKwBits;
    for (const auto& k : rule.kw_lower) {
      auto it = kwid.find(k);
      uint32_t id;
      if (it == kwid.end()) {
        id = (uint32_t)kws.size();
        kwid[k] = id;
        kws.push_back(k);
      } else {
        id = it->second;
      }
      p->rule_kws[r].push_back(id);
    }
  }
  p->fb_kw0 = (int)kws.size();
  kws.push_back("\xc4\xb0");      // U+0130, bytes.ToLower -> "i"
  kws.push_back("\xe2\x84\xaa");  // U+212A, bytes.ToLower -> "k"; (?i)k folds to it
  kws.push_back("\xc5\xbf");      // U+017F, (?i)s folds to it
  p->n_kw = (int)kws.size();
  p->kw_words = (p->n_kw + 31) / 32;
  for (const auto& k : kws) p->kw_len.push_back((uint16_t)std::min<size_t>(k.size(), 0xFFFF));

  // ---- per rule: anchor event and GPU program
  DFAOptions one;
  one.max_states = opt.max_group_states;
  auto fits = [&](const DFA& d, size_t nrules) {
    return d.nstates <= opt.max_group_states &&
           (size_t)d.nstates * d.nclasses * 2 <= (size_t)opt.max_group_table_bytes &&
           (int)nrules <= opt.max_rules_per_group;
  };
  p->rule_relax.assign(R, -1);
  p->rule_atoms.assign(R, -1);
  p->rule_winback.assign(R, -1);
  p->rule_prog.assign(R, Prog{});
  std::vector<std::unique_ptr<DFA>> single(R);
  const auto t_rules0 = std::chrono::steady_clock::now();
  std::vector<Anchor> anchor(R);
  // rules are independent here: build their programs on the shared pool
  const int plan_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  pool_for(R, plan_threads, [&](size_t r) {
    const RuleC& rule = rs.rules[r];
    if (!rule.regex) return;
    p->rule_maxlen[r] = max_match_len(rule.regex->prog());
    if (opt.anchors) anchor[r] = choose_anchor(*rule.regex, *p, rule.kw_lower.empty());
    const int fa = anchor[r].first_atom;
    // exact program first, then ever stronger relaxations of counted repetitions, then
    // ever shorter prefixes of the top-level concatenation
    for (int k : {-1, 32, 16, 8, 4, 2, 1, 0}) {
      Prog pr = (k < 0 && fa == 0) ? rule.regex->prog() : rule.regex->RelaxedProg(k, -1, fa);
      std::string e;
      auto d = build_dfa({&pr}, one, &e);
      if (d && fits(*d, 1)) {
        single[r] = std::move(d);
        p->rule_relax[r] = k;
        p->rule_prog[r] = std::move(pr);
        break;
      }
    }
    for (int t = rule.regex->NumAtoms() - fa - 1; !single[r] && t >= 1; t--) {
      for (int k : {8, 2, 0}) {
        Prog pr = rule.regex->RelaxedProg(k, t, fa);
        std::string e;
        auto d = build_dfa({&pr}, one, &e);
        if (d && fits(*d, 1)) {
          single[r] = std::move(d);
          p->rule_relax[r] = k;
          p->rule_atoms[r] = t;
          p->rule_prog[r] = std::move(pr);
          break;
        }
      }
    }
    if (!single[r]) {
      p->rule_hostonly[r] = 1;
      return;
    }
    // where a GPU end offset e lets the exact match start
    if (fa > 0) {
      p->rule_winback[r] = -1;
    } else if (p->rule_atoms[r] >= 0) {
      p->rule_winback[r] = max_match_len(rule.regex->RelaxedProg(-1, p->rule_atoms[r]));
    } else {
      p->rule_winback[r] = p->rule_maxlen[r];
    }
    p->rule_event[r] = anchor[r].kind;
    p->rule_evdist[r] = anchor[r].evdist;
    p->rule_first_atom[r] = fa;
    p->rule_anchor[r] = anchor[r].desc;
  }, 1);

  const bool tprof = getenv("TSG_PROF") != nullptr;
  auto tnow = [] { return std::chrono::steady_clock::now(); };
  auto tms = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  auto tp = tnow();
  if (tprof) fprintf(stderr, "plan: per-rule DFAs %.1f ms\n", tms(t_rules0));
  // ---- K2 rule groups: greedy packing under the state / table caps, among rules with
  // the same kind of event (their windows coincide)
  auto group_kwmask = [&](GroupPlan& g) {
    g.kwmask.assign(p->kw_words, 0);
    for (uint32_t r : g.rules) {
      if (p->rule_kw_mode[r] != kKwBits) {
        g.always = true;
        continue;
      }
      for (uint32_t k : p->rule_kws[r]) g.kwmask[k / 32] |= 1u << (k % 32);
    }
    // (the folding-rune pseudo keywords gate nothing here: a file holding one is always
    // resolved on the host, which scans its uncertain-keyword rules whole and adds windows
    // before the runes that (?i) folds, whatever K2 found)
  };
  for (uint32_t kind : {kEvRunU, kEvRunD, 1u << kEvLit0, kEvAlways}) {
    std::vector<uint32_t> cur;
    std::unique_ptr<DFA> cur_dfa;
    auto flush = [&]() {
      if (cur.empty()) return;
      GroupPlan g;
      g.dfa = std::move(cur_dfa);
      g.rules = cur;
      group_kwmask(g);
      g.events = kind;
      g.evdist = 0;
      for (uint32_t r : cur) {
        p->rule_group[r] = (int)p->groups.size();
        g.evdist = std::max(g.evdist, p->rule_evdist[r]);
      }
      p->groups.push_back(std::move(g));
      cur.clear();
    };
    for (size_t r = 0; r < R; r++) {
      if (!single[r] || p->rule_event[r] != kind) continue;
      if (cur.empty()) {
        cur.push_back((uint32_t)r);
        cur_dfa = std::move(single[r]);
        continue;
      }
      // two programs whose DFAs together exceed the cap have not merged under it on any
      // rule set measured (unanchored searches share few states): skip the construction
      if (cur_dfa->nstates + single[r]->nstates > opt.max_group_states ||
          product_states(*cur_dfa, *single[r], opt.max_group_states) > (size_t)opt.max_group_states) {
        flush();
        cur.push_back((uint32_t)r);
        cur_dfa = std::move(single[r]);
        continue;
      }
      std::vector<const Prog*> progs;
      for (uint32_t q : cur) progs.push_back(&p->rule_prog[q]);
      progs.push_back(&p->rule_prog[r]);
      std::string e;
      auto merged = build_dfa(progs, one, &e);
      if (getenv("TSG_PROF2"))
        fprintf(stderr, "merge %d+%d (nc %d,%d) -> %d %s\n", cur_dfa->nstates, single[r]->nstates,
                cur_dfa->nclasses, single[r]->nclasses, merged ? merged->nstates : -1,
                merged && fits(*merged, cur.size() + 1) ? "ok" : "FAIL");
      if (merged && fits(*merged, cur.size() + 1)) {
        cur.push_back((uint32_t)r);
        cur_dfa = std::move(merged);
      } else {
        flush();
        cur.push_back((uint32_t)r);
        cur_dfa = std::move(single[r]);
      }
    }
    flush();
  }

  if (tprof) {
    fprintf(stderr, "plan: grouping %.1f ms (%zu groups)\n", tms(tp), p->groups.size());
    for (size_t g = 0; g < p->groups.size(); g++)
      fprintf(stderr, "plan: group %zu: %zu rules, %d states x %d classes (%zu table bytes), events %#x\n", g,
              p->groups[g].rules.size(), p->groups[g].dfa->nstates, p->groups[g].dfa->nclasses,
              (size_t)p->groups[g].dfa->nstates * p->groups[g].dfa->nclasses * 2, p->groups[g].events);
  }
  tp = tnow();
  // ---- K1 automaton: keywords + anchor literals; literal groups share event bits
  std::vector<char> litg(p->groups.size(), 0);
  for (size_t g = 0; g < p->groups.size(); g++) litg[g] = p->groups[g].events == (1u << kEvLit0);
  // keywords left out of K1 (table budget): a literal no ASCII text contains holds their id
  std::vector<char> kw_dropped(kws.size(), 0);
  // hashed mode (K1X): the keywords and anchors that leave the automaton
  std::vector<char> kw_hashed(kws.size(), 0), anchor_hashed(R, 0);
  auto build_k1 = [&](bool with_anchors) -> bool {
    std::vector<std::string> lits = kws;
    for (size_t k = 0; k < lits.size(); k++)
      if (kw_dropped[k] || kw_hashed[k]) lits[k] = never_literal();
    std::map<std::string, std::pair<int32_t, uint32_t>> xl;  // K1X literal -> keyword id, events
    for (size_t k = 0; k < kws.size(); k++)
      if (kw_hashed[k]) xl[ascii_lower(kws[k])] = {(int32_t)k, 0u};
    std::vector<uint32_t> lit_event(lits.size(), 0);
    std::map<std::string, uint32_t> lid;
    for (size_t i = 0; i < lits.size(); i++) lid.emplace(lits[i], (uint32_t)i);
    int nlitgroups = 0;
    for (size_t gi = 0; gi < p->groups.size(); gi++) {
      GroupPlan& g = p->groups[gi];
      if (!litg[gi]) continue;
      if (!with_anchors) {
        g.events = kEvAlways;
        for (uint32_t r : g.rules) p->rule_event[r] = kEvAlways;
        continue;
      }
      const uint32_t bit = 1u << (kEvLit0 + (nlitgroups++ % kEvLitBits));
      g.events = bit;
      for (uint32_t r : g.rules) {
        p->rule_event[r] = bit;
        const std::string& s = anchor[r].lit;
        if (anchor_hashed[r]) {
          auto xi = xl.find(ascii_lower(s));
          if (xi == xl.end()) xl[ascii_lower(s)] = {-1, bit};
          else xi->second.second |= bit;
          continue;
        }
        auto it = lid.find(s);
        uint32_t id;
        if (it == lid.end()) {
          id = (uint32_t)lits.size();
          lid.emplace(s, id);
          lits.push_back(s);
          lit_event.push_back(0);
        } else {
          id = it->second;
        }
        lit_event[id] |= bit;
      }
    }
    DFAOptions o;
    o.max_states = 32767;
    o.with_noinject = false;
    std::string e;
    auto d = build_keyword_dfa(lits, o, &e);
    if (!d) return false;
    if ((size_t)d->nstates * d->nclasses * 2 > (size_t)opt.max_kw_table_bytes) return false;
    p->n_lit = (int)lits.size();
    p->lit_event = lit_event;
    p->k1_lits = lits;
    p->kw_mask_events.assign(d->masks.size(), 0);
    for (size_t m = 0; m < d->masks.size(); m++)
      for (int id = 0; id < p->n_lit; id++)
        if ((d->masks[m][id / 64] >> (id % 64)) & 1) p->kw_mask_events[m] |= lit_event[id];
    size_t longest = 0;
    for (const auto& s : lits) longest = std::max(longest, s.size());
    int w = (int)std::max<size_t>(longest, (size_t)std::max(p->run_k[0], p->run_k[1]));
    p->warm = (w - 1 + 15) / 16 * 16;
    p->kw_dfa = std::move(d);
    p->x_lits.clear();
    p->x_kw.clear();
    p->x_event.clear();
    p->x_j0.clear();
    for (const auto& kv : xl) {
      p->x_lits.push_back(kv.first);
      p->x_kw.push_back(kv.second.first);
      p->x_event.push_back(kv.second.second);
    }
    return true;
  };
  // table bytes of an automaton over the keywords (and anchors): its states are the
  // literals' distinct prefixes, its classes at most the distinct bytes + 1
  auto k1_estimate = [&](bool with_anchors) {
    std::set<std::string> pre;
    bool bytes[256] = {false};
    auto add = [&](const std::string& s) {
      for (size_t i = 1; i <= s.size(); i++) pre.insert(s.substr(0, i));
      for (unsigned char ch : s) bytes[ch] = true;
    };
    for (size_t k = 0; k < kws.size(); k++)
      if (!kw_dropped[k] && !kw_hashed[k]) add(kws[k]);
    if (with_anchors)
      for (size_t r = 0; r < R; r++)
        if (!anchor[r].lit.empty() && !anchor_hashed[r]) add(anchor[r].lit);
    size_t ncls = 1;
    for (int c = 0; c < 256; c++) ncls += bytes[c];
    return (pre.size() + 1) * ncls * 2;
  };
  // (an estimate far over the budget skips the exact build)
  auto try_k1 = [&](bool with_anchors) {
    return k1_estimate(with_anchors) <= 4 * (size_t)opt.max_kw_table_bytes && build_k1(with_anchors);
  };
  bool k1_ok = (opt.anchors && try_k1(true)) || try_k1(false);
  if (!k1_ok && !knobs().no_k1x.load()) {
    // Too many literal bytes for an LDS-resident automaton (large user rule sets).  K1X
    // samples one 4-byte window every x_step bytes, so it takes literals of x_step + 3 bytes
    // or more; the shorter ones stay in the automaton, and the others fill what is left of a
    // packed table (k1_packed_fits) in rule order -- the builtin rules' first
    // (scanner.go:302-311), whose keywords are the ones common in real text -- the rest are
    // hashed.  Keyword bits stay exact, anchors keep their events.
    // the widest step whose automaton fits the packed table, else the widest that builds
    // (the x_step test knob forces one)
    const int forced = knobs().x_step.load();
    for (int attempt = 0; attempt < 6 && !k1_ok; attempt++) {
      const int step = (attempt % 3 == 0) ? 4 : (attempt % 3 == 1) ? 2 : 1;
      const bool need_packed = attempt < 3;
      if (forced && step != forced) continue;
      const size_t xmin = (size_t)step + 3;
      std::set<std::string> pre;
      bool bytes[256] = {false};
      size_t nbytes = 0;
      // table bytes with literal s added: rows x (classes padded to 2 mod 4) x 2, an upper
      // bound of the exact automaton's (k1_estimate)
      auto cost = [&](const std::string& s) {
        const std::string l = ascii_lower(s);
        size_t npre = 0, nb = 0;
        bool seen[256] = {false};
        for (size_t i = 1; i <= l.size(); i++) npre += pre.count(l.substr(0, i)) ? 0 : 1;
        for (unsigned char ch : l) {
          if (!bytes[ch] && !seen[ch]) nb++;
          seen[ch] = true;
        }
        return (pre.size() + npre + 1) * (nbytes + nb + 1 + 3) * 2;
      };
      auto take = [&](const std::string& s) {
        const std::string l = ascii_lower(s);
        for (size_t i = 1; i <= l.size(); i++) pre.insert(l.substr(0, i));
        for (unsigned char ch : l) {
          if (!bytes[ch]) nbytes++;
          bytes[ch] = true;
        }
      };
      std::fill(kw_hashed.begin(), kw_hashed.end(), 0);
      std::fill(anchor_hashed.begin(), anchor_hashed.end(), 0);
      for (size_t k = 0; k < kws.size(); k++)
        if (!kw_dropped[k] && kws[k].size() < xmin) take(kws[k]);
      for (size_t r = 0; r < R; r++)
        if (!anchor[r].lit.empty() && anchor[r].lit.size() < xmin) take(anchor[r].lit);
      // two passes in rule order: literals whose every K1X window choice holds a 4-gram
      // common in text first, then the quiet ones
      for (int pass = 0; pass < 2; pass++) {
        std::vector<char> kw_seen(kws.size(), 0);
        auto place = [&](const std::string& s, char* hashed) {
          uint32_t j0 = 0;
          const int c = x_pick(ascii_lower(s), step, &j0);
          if (c < 0 || (pass == 0) != (c > 0)) return;  // too short (kept above), or the other pass
          if (cost(s) <= 65536) take(s);
          else *hashed = 1;
        };
        for (size_t r = 0; r < R; r++) {
          for (uint32_t k : p->rule_kws[r])
            if ((int)k < p->fb_kw0 && !kw_dropped[k] && !kw_seen[k]) {
              kw_seen[k] = 1;
              place(kws[k], &kw_hashed[k]);
            }
          if (!anchor[r].lit.empty()) place(anchor[r].lit, &anchor_hashed[r]);
        }
        for (int k = 0; k < p->fb_kw0; k++)  // keywords no rule lists (none today)
          if (!kw_seen[k] && !kw_dropped[k]) place(kws[k], &kw_hashed[k]);
      }
      k1_ok = (opt.anchors && try_k1(true)) || try_k1(false);
      if (k1_ok && need_packed && !forced &&
          (size_t)p->kw_dfa->nstates * p->kw_dfa->nclasses * 2 > 65536)
        k1_ok = false;
      if (k1_ok) {
        p->x_step = step;
        x_place_windows(&*p, step);
      }
    }
    if (!k1_ok) {
      std::fill(kw_hashed.begin(), kw_hashed.end(), 0);
      std::fill(anchor_hashed.begin(), anchor_hashed.end(), 0);
    }
  }
  if (!k1_ok) {
    // Too many keyword bytes for an LDS-resident automaton (large user rule sets): leave
    // keywords out, longest first (they cost the most states), until it fits.  Their rules
    // get the exact keyword gate on the host, and their groups are scanned on every file.
    std::vector<int> order;
    for (int k = 0; k < p->fb_kw0; k++) order.push_back(k);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return kws[a].size() > kws[b].size(); });
    // Estimate first, so the exact build runs once or twice.
    size_t next = 0;
    while (next < order.size() && k1_estimate(false) > (size_t)opt.max_kw_table_bytes) {
      const size_t m = std::max<size_t>(1, (order.size() - next) / 8);
      for (size_t k = 0; k < m && next < order.size(); k++) kw_dropped[order[next++]] = 1;
    }
    bool ok = (opt.anchors && try_k1(true)) || build_k1(false);
    while (next < order.size() && !ok) {
      for (size_t m = std::max<size_t>(1, order.size() / 32); m > 0 && next < order.size(); m--)
        kw_dropped[order[next++]] = 1;
      ok = build_k1(opt.anchors) || build_k1(false);
    }
    if (!ok) {
      if (err) *err = "keyword automaton exceeds the K1 table budget";
      return nullptr;
    }
    for (size_t r = 0; r < R; r++) {
      if (p->rule_kw_mode[r] != kKwBits) continue;
      for (uint32_t k : p->rule_kws[r])
        if (kw_dropped[k]) p->rule_kw_mode[r] = kKwUnknown;
    }
    for (auto& g : p->groups) group_kwmask(g);
  }

  if (tprof) fprintf(stderr, "plan: K1 %.1f ms\n", tms(tp));
  tp = tnow();
  // ---- host resolver: fold-rune DFAs of the unbounded relaxed rules
  p->rule_fold_dfa.resize(R);
  std::vector<Prog> fold_prog(R);
  pool_for(R, plan_threads, [&](size_t r) {
    const RuleC& rule = rs.rules[r];
    if (!rule.regex || p->rule_relax[r] < 0 || p->rule_maxlen[r] >= 0 || p->rule_group[r] < 0) return;
    DFAOptions o;
    o.max_states = 4096;
    for (int k : {p->rule_relax[r], 8, 2, 0}) {
      Prog pr = rule.regex->RelaxedProg(k, -1, 0, true);
      std::string e;
      auto d = build_dfa({&pr}, o, &e);
      if (d) {
        p->rule_fold_dfa[r] = std::move(d);
        fold_prog[r] = std::move(pr);
        break;
      }
    }
  }, 1);
  {  // all unbounded rules' fold programs in one DFA (resolve_batch: one pass per file)
    std::vector<const Prog*> progs;
    for (size_t r = 0; r < R; r++) {
      if (!rs.rules[r].regex || p->rule_maxlen[r] >= 0) continue;
      if (p->rule_fold_dfa[r]) {
        progs.push_back(&fold_prog[r]);
      } else if (p->rule_group[r] >= 0 && p->rule_relax[r] < 0) {
        progs.push_back(&p->rule_prog[r]);
      } else {
        continue;
      }
      p->fold_rules.push_back((uint32_t)r);
    }
    if (progs.size() > 1) {
      DFAOptions o;
      o.max_states = 16384;
      std::string e;
      p->fold_all_dfa = build_dfa(progs, o, &e);
      if (p->fold_all_dfa) p->fold_all_dfa->pack();
    }
  }
  // ---- host resolver: reverse DFAs of the exact programs
  p->rule_rev.resize(R);
  // (only where the forward bound is loose: unbounded or long windows; the subset
  // construction of the counted generic rules would cost more than it saves)
  for (size_t r = 0; r < R; r++) {
    if (!rs.rules[r].regex || (p->rule_winback[r] >= 0 && p->rule_winback[r] <= 1024)) continue;
    DFAOptions o;
    o.max_states = 2048;
    std::string e;
    auto t0 = std::chrono::steady_clock::now();
    p->rule_rev[r] = build_reverse_dfa(rs.rules[r].regex->prog(), o, &e);
    if (p->rule_rev[r]) p->rule_rev[r]->pack();
    if (getenv("TSG_PROF"))
      fprintf(stderr, "rev %s: %d states %.1f ms\n", rs.rules[r].id.c_str(),
              p->rule_rev[r] ? p->rule_rev[r]->nstates : -1,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }

  if (tprof) fprintf(stderr, "plan: reverse DFAs %.1f ms\n", tms(tp));
  // ---- Global.AllowPath automaton (exact on ASCII paths)
  std::vector<const Prog*> paths;
  for (const auto& a : rs.allow)
    if (a.path) paths.push_back(&a.path->prog());
  if (!paths.empty()) {
    DFAOptions o;
    o.max_states = 1 << 16;
    std::string e;
    p->allow_path_dfa = build_dfa(paths, o, &e);  // may be null: exact VM is used then
  }
  return p;
}

// ------------------------------------------------------------------ threading
// One process-wide pool of worker threads shared by every parallel_for, so concurrent
// batch resolutions (tsg_batch_submit pipelines them) never run more than the pool's
// threads plus their callers, and per-thread caches (the backtracker's visited rows)
// survive from one batch to the next.
namespace {

struct PJob {
  std::function<void(size_t)> body;
  size_t n = 0, grain = 64;
  std::atomic<size_t> next{0};
  int pending = 0;  // queued or running helper tasks (under m)
  std::mutex m;
  std::condition_variable cv;
  void work() {
    for (;;) {
      const size_t s = next.fetch_add(grain);
      if (s >= n) break;
      const size_t e = std::min(n, s + grain);
      for (size_t i = s; i < e; i++) body(i);
    }
  }
};

class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool;  // never destroyed: workers may still wait at exit
    return *p;
  }
  // runs j on the caller and up to `helpers` pool threads; returns when all are done
  // at least n worker threads (more concurrent jobs can then run side by side)
  void reserve(int n) { grow(std::min(n, 256)); }
  void run(PJob& j, int helpers) {
    grow(helpers);
    {
      std::lock_guard<std::mutex> g(m_);
      j.pending = helpers;
      for (int h = 0; h < helpers; h++) q_.push_back(&j);
    }
    cv_.notify_all();
    j.work();
    {  // helpers that have not started are not needed any more
      std::lock_guard<std::mutex> g(m_);
      int removed = 0;
      for (auto it = q_.begin(); it != q_.end();)
        if (*it == &j) {
          it = q_.erase(it);
          removed++;
        } else {
          ++it;
        }
      std::lock_guard<std::mutex> g2(j.m);
      j.pending -= removed;
    }
    std::unique_lock<std::mutex> lk(j.m);
    j.cv.wait(lk, [&] { return j.pending == 0; });
  }

 private:
  void grow(int want) {
    std::lock_guard<std::mutex> g(m_);
    while ((int)th_.size() < want) {
      th_.emplace_back([this] { worker(); });
      th_.back().detach();
    }
  }
  void worker() {
    for (;;) {
      PJob* j;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        j = q_.front();
        q_.pop_front();
      }
      j->work();
      std::lock_guard<std::mutex> g(j->m);
      if (--j->pending == 0) j->cv.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<PJob*> q_;
  std::vector<std::thread> th_;
};

}  // namespace

template <class F>
static void parallel_for(size_t n, int nthreads, F f, size_t grain = 64) {
  if (nthreads <= 1 || n < 2 * grain) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  PJob j;
  j.body = [&f](size_t i) { f(i); };
  j.n = n;
  j.grain = grain;
  Pool::get().run(j, std::min(nthreads, 256) - 1);
}

void pool_reserve(int threads) { Pool::get().reserve(threads); }

void pool_for(size_t n, int nthreads, const std::function<void(size_t)>& f, size_t grain) {
  parallel_for(n, nthreads, f, grain);
}

bool path_allowed(const Ruleset& rs, const Plan* plan, const char* p, size_t n) {
  if (plan && plan->allow_path_dfa) {
    bool ascii = true;
    for (size_t i = 0; i < n && ascii; i++) ascii = (uint8_t)p[i] < 0x80;
    if (ascii) {  // any accept (a non-empty mask) = some allow path regexp matches
      const DFA& d = *plan->allow_path_dfa;
      uint32_t s = d.start[kCtxBOT];
      for (size_t i = 0; i < n; i++) {
        const size_t e = (size_t)s * d.nclasses + d.cls[(uint8_t)p[i]];
        if (d.acc[e]) return true;
        s = d.next[e];
      }
      return d.eot_acc[s] != 0;
    }
  }
  return rs.AllowPath(std::string(p, n));
}

void scan_batch_cpu(const Ruleset& rs, const BatchView& b, int nthreads,
                    std::vector<FileResult>* out) {
  out->assign(b.nfiles, FileResult{});
  parallel_for(b.nfiles, nthreads, [&](size_t i) {
    std::string path(b.paths + b.path_offsets[i], b.path_offsets[i + 1] - b.path_offsets[i]);
    scan_file(rs, path, b.data + b.offsets[i], b.offsets[i + 1] - b.offsets[i], nullptr,
              &(*out)[i]);
  });
}

// rune boundary at or before p in the canonical (from-0) UTF-8 segmentation
static int64_t align_rune(const uint8_t* d, int64_t n, int64_t p) {
  if (p <= 0) return 0;
  if (p >= n) return n;
  if ((d[p] & 0xC0) != 0x80) return p;
  for (int k = 1; k <= 3 && p - k >= 0; k++) {
    int64_t q = p - k;
    if ((d[q] & 0xC0) != 0x80) {
      int w;
      decode_rune(d, (size_t)n, (size_t)q, &w);
      return (q + w > p) ? q : p;
    }
  }
  return p;
}

namespace {

// One lane's work on one file segment [a, b) of file [fs, fe): inject mode over the
// segment, then (if the file continues) noinject mode until every thread started in
// the segment has died.  on_acc(mask_index, position_in_file).
template <class OnAcc>
bool run_segment(const DFA& d, const uint8_t* data, uint64_t fs, uint64_t fe, uint64_t a,
                 uint64_t b, uint32_t ext_cap, OnAcc on_acc) {
  const int nc = d.nclasses;
  uint32_t s = (a == fs) ? d.start[kCtxBOT] : d.start[DFA::ctx_of(data[a - 1], d)];
  if (!d.packed.empty()) {  // one load per byte: next row | accept | next dead (DFA::pack)
    uint32_t row = s * (uint32_t)nc;
    for (uint64_t p = a; p < b; p++) {
      const uint32_t e = row + d.cls[data[p]];
      const uint32_t x = d.packed[e];
      if (x >> 31) on_acc(d.acc[e], p - fs);
      row = x & 0x3FFFFFFFu;
    }
    s = row / (uint32_t)nc;
  }
  for (uint64_t p = d.packed.empty() ? a : b; p < b; p++) {
    size_t e = (size_t)s * nc + d.cls[data[p]];
    if (d.acc[e]) on_acc(d.acc[e], p - fs);
    s = d.next[e];
  }
  if (b >= fe) {
    if (d.eot_acc[s]) on_acc(d.eot_acc[s], fe - fs);
    return false;
  }
  s = d.to_noinject[s];
  uint64_t p = b;
  while (p < fe && !d.dead[s]) {
    // at the kernels' 16-byte word boundaries: past ext_cap, or in a state whose threads
    // never die (the tail would run to the end of the file) -> the host resolves the
    // file whole
    if ((p == b || (p & 15) == 0) && (p - b >= ext_cap || d.immortal[s])) return true;
    size_t e = (size_t)s * nc + d.cls[data[p]];
    if (d.acc[e]) on_acc(d.acc[e], p - fs);
    s = d.next[e];
    p++;
  }
  if (p == fe && !d.dead[s] && d.eot_acc[s]) on_acc(d.eot_acc[s], fe - fs);
  return false;
}

}  // namespace

void resolve_batch(const Ruleset& rs, const Plan& plan, const BatchView& b,
                   const KernelOutputView& ko, int nthreads, BatchResult* out) {
  const uint32_t F = b.nfiles;
  const size_t R = rs.rules.size();
  const uint64_t t_ser0 = __rdtsc();
  // K2 transition records (kCandTrans) -> one candidate per rule of their accept mask
  std::vector<Candidate> expanded;
  const Candidate* kc = ko.cand;
  size_t nkc = ko.ncand;
  const bool words = plan.groups.size() <= 0x3FFF;  // kCandWord records (kernels.hip accept_word)
  {
    size_t ntrans = 0;
    for (size_t i = 0; i < nkc; i++) ntrans += (kc[i].rule & kCandTrans) && kc[i].end != kCandWhole;
    if (ntrans) {
      // one record's candidates into `out` (a word record replays its word from the batch)
      auto expand = [&](const Candidate& c, std::vector<Candidate>& out) {
        if (!(c.rule & kCandTrans) || c.end == kCandWhole) {
          out.push_back(c);
          return;
        }
        const bool word = words && (c.rule & kCandWord);
        const uint32_t g = (c.rule >> 16) & (words ? 0x3FFFu : 0x7FFFu), ix = c.rule & 0xFFFFu;
        if (g >= plan.groups.size()) return;
        const GroupPlan& gp = plan.groups[g];
        const DFA& d = *gp.dfa;
        const uint32_t ncd = (uint32_t)std::max(2, d.nclasses);  // the device's row width
        if (word) {  // kCandWord: replay the word from row ix at byte `end` to the word's end
          size_t st = ix / ncd;
          if (st >= (size_t)d.nstates || c.file >= F) return;
          const uint64_t f0 = b.offsets[c.file], flen = b.offsets[c.file + 1] - f0;
          const uint64_t pend = std::min<uint64_t>(flen, (((f0 + c.end) | 15) + 1) - f0);
          for (uint64_t p = c.end; p < pend; p++) {
            const size_t e = st * d.nclasses + d.cls[b.data[f0 + p]];
            if (d.acc[e]) {
              const auto& m = d.masks[d.acc[e]];
              for (size_t k = 0; k < gp.rules.size(); k++)
                if ((m[k / 64] >> (k % 64)) & 1) out.push_back({c.file, gp.rules[k], (uint32_t)p});
            }
            st = d.next[e];
          }
          return;
        }
        const size_t st = ix / ncd, cl = std::min<size_t>(ix % ncd, (size_t)d.nclasses - 1);
        if (st >= (size_t)d.nstates) return;
        const auto& m = d.masks[d.acc[st * d.nclasses + cl]];
        for (size_t k = 0; k < gp.rules.size(); k++)
          if ((m[k / 64] >> (k % 64)) & 1) out.push_back({c.file, gp.rules[k], c.end});
      };
      // In parallel, in record order: each word record's replay reads the batch at its own
      // place (a cache and TLB miss in a pinned multi-GiB slot), and serially that was half
      // of a layer piece's resolution (12-15 of ~28 Mcyc per 256 MiB piece, TSG_PROF).
      constexpr size_t kRecBlk = 2048;
      const size_t nrb = (nkc + kRecBlk - 1) / kRecBlk;
      std::vector<std::vector<Candidate>> parts(nrb);
      parallel_for(nrb, nthreads, [&](size_t bi) {
        auto& out = parts[bi];
        const size_t i1 = std::min(nkc, (bi + 1) * kRecBlk);
        out.reserve(i1 - bi * kRecBlk + 16);
        for (size_t i = bi * kRecBlk; i < i1; i++) expand(kc[i], out);
      }, 1);
      size_t total = 0;
      for (const auto& pt : parts) total += pt.size();
      expanded.reserve(total);
      for (const auto& pt : parts) expanded.insert(expanded.end(), pt.begin(), pt.end());
      kc = expanded.data();
      nkc = expanded.size();
    }
  }
  // bucket candidates by file (counting sort), then sort each file's few by (rule, end)
  std::vector<uint32_t> first(F + 1, 0);
  for (size_t i = 0; i < nkc; i++) first[kc[i].file + 1]++;
  for (uint32_t f = 0; f < F; f++) first[f + 1] += first[f];
  std::vector<Candidate> cand(nkc);
  {
    std::vector<uint32_t> fill(first.begin(), first.end() - 1);
    for (size_t i = 0; i < nkc; i++) cand[fill[kc[i].file]++] = kc[i];
  }
  auto by_rule_end = [](const Candidate& x, const Candidate& y) {
    return x.rule != y.rule ? x.rule < y.rule : x.end < y.end;
  };

  std::vector<uint32_t> hostonly;
  for (size_t r = 0; r < R; r++)
    if (plan.rule_hostonly[r] ||
        (ko.group_skipped && plan.rule_group[r] >= 0 && ko.group_skipped[plan.rule_group[r]]))
      hostonly.push_back((uint32_t)r);
  std::vector<uint8_t> kw_has_i(R, 0), kw_has_k(R, 0);
  for (size_t r = 0; r < R; r++)
    for (const auto& k : rs.rules[r].kw_lower) {
      kw_has_i[r] |= k.find('i') != std::string::npos;
      kw_has_k[r] |= k.find('k') != std::string::npos;
    }

  const uint64_t t_ser1 = __rdtsc();
  // Global.AllowPath (scanner.go:343-347): from the device when it decided the path
  auto path_ok = [&](uint32_t f) -> bool {
    if (ko.path_ok && ko.path_ok[f] < 2) return ko.path_ok[f] == 1;
    return path_allowed(rs, &plan, b.paths + b.path_offsets[f], b.path_offsets[f + 1] - b.path_offsets[f]);
  };
  // Files that need the exact scan: candidates, empty files, kernel overflow, folding
  // runes, or a gated rule without a GPU program.  The others only need Global.AllowPath,
  // settled here.  Two parallel passes over blocks of files: flags and counts, then slot
  // numbers in file order.
  out->status.resize(F);
  out->slot.resize(F);
  const size_t kBlk = 8192, nblk = (F + kBlk - 1) / kBlk;
  std::vector<uint32_t> bcount(nblk + 1, 0);
  parallel_for(nblk, nthreads, [&](size_t bi) {
    uint32_t cnt = 0;
    for (uint32_t f = (uint32_t)(bi * kBlk), fe = (uint32_t)std::min<size_t>(F, (bi + 1) * kBlk); f < fe; f++) {
      bool need = first[f] != first[f + 1] || b.offsets[f + 1] == b.offsets[f] ||
                  (ko.overflow && (ko.overflow[f] & 1)) || !hostonly.empty();
      if (!need && ko.sparse_kw) {
        need = (ko.overflow[f] & 2) != 0;
      } else if (!need) {
        const uint32_t* kw = ko.kw + (size_t)f * plan.kw_words;
        for (int k = plan.fb_kw0; k < plan.n_kw && !need; k++) need = (kw[k / 32] >> (k % 32)) & 1;
      }
      if (need) {
        out->slot[f] = 0;
        cnt++;
      } else {
        out->slot[f] = UINT32_MAX;
        out->status[f] = path_ok(f) ? kPathAllowed : kNoFindings;
      }
    }
    bcount[bi + 1] = cnt;
  }, 1);
  for (size_t bi = 0; bi < nblk; bi++) bcount[bi + 1] += bcount[bi];
  const uint32_t nslots = bcount[nblk];
  std::vector<uint32_t> need_files(nslots);
  parallel_for(nblk, nthreads, [&](size_t bi) {
    uint32_t k = bcount[bi];
    for (uint32_t f = (uint32_t)(bi * kBlk), fe = (uint32_t)std::min<size_t>(F, (bi + 1) * kBlk); f < fe; f++)
      if (out->slot[f] != UINT32_MAX) {
        out->slot[f] = k;
        need_files[k++] = f;
      }
  }, 1);
  out->res.clear();
  out->res.resize(nslots);
  // a sparse keyword array holds only the rows the device wrote (flag bit 2): every file
  // that needs resolution must have one (reading any other row would read stale bits).
  // Checked here on the caller, not inside the parallel pass: a throw from a pool worker
  // would terminate the process.
  if (ko.sparse_kw)
    for (uint32_t f : need_files)
      if (b.offsets[f + 1] != b.offsets[f] && !(ko.overflow[f] & 4))
        throw std::runtime_error("keyword row of a resolved file not written");

  static const bool prof = getenv("TSG_PROF") != nullptr;
  if (prof)
    fprintf(stderr, "resolve: setup %.1f Mcyc (candidate sort %.1f; %u files to scan)\n", (__rdtsc() - t_ser0) / 1e6,
            (t_ser1 - t_ser0) / 1e6, nslots);
  // TSG_PROF: per-thread cycle counters (no shared atomics in the loop)
  struct alignas(64) Slot {
    // fast files, candidate files, other files, count cand, scan_file, fold-rune keyword
    // windows, fold windows of bounded rules, fold DFA / group DFA whole-file runs
    uint64_t cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  };
  static std::atomic<int> next_tid{0};
  std::vector<Slot> slots(prof ? 256 : 0);
  std::atomic<int64_t> n_whole{0};
  const uint64_t t_par0 = prof ? __rdtsc() : 0;
  parallel_for(nslots, nthreads, [&](size_t si) {
    thread_local int tid = next_tid++ & 255;
    const uint64_t tp0 = prof ? __rdtsc() : 0;
    struct Tm {
      bool on;
      uint64_t t0;
      uint64_t* acc;
      ~Tm() {
        if (on) *acc += __rdtsc() - t0;
      }
    };
    const uint32_t f = need_files[si];
    const bool has_cand = first[f] != first[f + 1];
    Tm tm{prof, tp0, prof ? &slots[tid].cyc[has_cand ? 1 : 2] : nullptr};
    if (prof && has_cand) slots[tid].cyc[3]++;
    const char* pp = b.paths + b.path_offsets[f];
    const size_t pn = b.path_offsets[f + 1] - b.path_offsets[f];
    const uint8_t* content = b.data + b.offsets[f];
    const int64_t n = (int64_t)(b.offsets[f + 1] - b.offsets[f]);
    FileResult& res = out->res[out->slot[f]];
    struct SetStatus {
      FileResult& r;
      uint8_t& s;
      ~SetStatus() { s = r.status; }
    } set_status{res, out->status[f]};
    if (n == 0) {  // the kernels skip empty files; only empty matches are possible
      scan_file(rs, std::string(pp, pn), content, 0, nullptr, &res);
      return;
    }
    // (a sparse keyword array has this file's row: checked before the parallel pass)
    const uint32_t* kw = ko.kw + (size_t)f * plan.kw_words;
    // folding runes present: bit 0 U+0130, bit 1 U+212A, bit 2 U+017F
    uint32_t fbbits = 0;
    for (int k = plan.fb_kw0; k < plan.n_kw; k++)
      if ((kw[k / 32] >> (k % 32)) & 1) fbbits |= 1u << (k - plan.fb_kw0);
    // Keyword gate.  K1 bits are exact for the ASCII bytes of the file; bytes.ToLower
    // turns a non-ASCII rune into an ASCII letter only for U+0130 -> 'i' and U+212A -> 'k',
    // so a clear bit is uncertain only for keywords holding that letter.
    auto kw_state = [&](size_t r) -> uint8_t {
      switch (plan.rule_kw_mode[r]) {
        case kKwAlways: return 1;
        case kKwUnknown: return 2;
        default:
          for (uint32_t k : plan.rule_kws[r])
            if ((kw[k / 32] >> (k % 32)) & 1) return 1;
          if (ko.kw_unknown)
            for (uint32_t k : plan.rule_kws[r])
              if (ko.kw_unknown[k]) return 2;  // the kernels scanned the rule's group
          // 3: uncertain and the kernels did not scan the rule (its keyword bits were clear)
          if (((fbbits & 1) && kw_has_i[r]) || ((fbbits & 2) && kw_has_k[r])) return 3;
          return 0;
      }
    };
    // kernel overflow: resolve every rule over the whole file
    const bool ovf = ko.overflow && (ko.overflow[f] & 1);
    bool any_host = false;
    for (uint32_t r : hostonly)
      if (kw_state(r) != 0) any_host = true;
    if (first[f] == first[f + 1] && !ovf && !any_host && !fbbits) {  // no match possible
      res.status = path_ok(f) ? kPathAllowed : kNoFindings;
      return;
    }
    const std::string path(pp, pn);
    std::vector<RuleWindows> wins(R);
    std::vector<const RuleWindows*> wptr(R, nullptr);
    std::vector<uint8_t> kws(R);
    for (size_t r = 0; r < R; r++) kws[r] = kw_state(r);
    const uint64_t tk0 = prof ? __rdtsc() : 0;
    if (fbbits & 3) {
      // U+0130 / U+212A present: a keyword K1 did not see (its bit is clear; bits are exact
      // for ASCII) can only occur through one of those runes, i.e. inside a window of 3 bytes
      // per keyword letter around a rune.  Check the uncertain rules' keywords there instead
      // of over the whole file: not found -> the gate fails (0), found -> exact scan (2).
      std::vector<int64_t> runes;
      fold_rune_positions(content, n, 1 | 2, &runes);
      for (size_t r = 0; r < R; r++) {
        if (kws[r] != 3 || !rs.rules[r].kw_ascii) continue;
        bool hit = false;
        for (const auto& kw : rs.rules[r].kw_lower) {
          const int64_t span = 3 * (int64_t)kw.size();
          for (size_t i = 0; i < runes.size() && !hit; i++) {
            const int64_t a = std::max<int64_t>(0, runes[i] - span), e = std::min<int64_t>(n, runes[i] + span);
            hit = contains_fold_runes(content + a, (size_t)(e - a), kw);
          }
          if (hit) break;
        }
        kws[r] = hit ? 3 : 0;  // 3 -> whole-file exact resolution below
      }
    }
    if (prof) slots[tid].cyc[5] += __rdtsc() - tk0;
    if (ovf) {
      for (size_t r = 0; r < R; r++) {
        wins[r].whole = true;
        wptr[r] = &wins[r];
      }
    }
    for (uint32_t r : hostonly)
      if (kws[r] != 0) {
        wins[r].whole = true;
        wptr[r] = &wins[r];
      }
    // every match start lies in [end - winback, end] of some candidate end offset; the
    // reverse DFA narrows that to [leftmost start, end] or drops the candidate
    auto add_end = [&](RuleWindows& w, uint32_t r, int64_t end) {
      int64_t lo;
      if (const DFA* rev = plan.rule_rev[r].get()) {
        lo = reverse_match_start(*rev, content, end);
        if (lo < 0) return;
        lo = align_rune(content, n, lo);
      } else {
        const int64_t back = plan.rule_winback[r];
        lo = back < 0 ? 0 : align_rune(content, n, std::max<int64_t>(0, end - back));
      }
      w.iv.push_back({lo, end});
    };
    auto normalize = [](RuleWindows& w) {  // sort, merge touching windows
      std::sort(w.iv.begin(), w.iv.end());
      size_t o = 0;
      for (size_t i = 0; i < w.iv.size(); i++) {
        if (o && w.iv[i].first <= w.iv[o - 1].second + 1)
          w.iv[o - 1].second = std::max(w.iv[o - 1].second, w.iv[i].second);
        else
          w.iv[o++] = w.iv[i];
      }
      w.iv.resize(o);
    };
    std::sort(cand.begin() + first[f], cand.begin() + first[f + 1], by_rule_end);
    for (uint32_t k = first[f]; k < first[f + 1];) {
      uint32_t r = cand[k].rule;
      uint32_t e = k;
      while (e < first[f + 1] && cand[e].rule == r) e++;
      RuleWindows& w = wins[r];
      wptr[r] = &w;
      if (!w.whole) {
        for (uint32_t j = k; j < e && !w.whole; j++) {
          if (cand[j].end == kCandWhole) {
            w.whole = true;
            w.iv.clear();
          } else {
            add_end(w, r, cand[j].end);
          }
        }
        normalize(w);
      }
      k = e;
    }
    const uint64_t tf0 = prof ? __rdtsc() : 0;
    uint64_t tdfa = 0;
    if (fbbits & 6) {
      // The windows and whole-file runs below are only needed for rules whose keyword gate
      // passes.  A gate K1 left to the host (kws 2: an adapted hot keyword such as "key")
      // is settled exactly first, as scan_file would (scanner.go:164-176): random binary
      // blobs hold folding-rune byte pairs but rarely the keyword.
      std::map<std::string, bool> kwhit;
      for (size_t r = 0; r < R; r++) {
        if (kws[r] != 2 || !rs.rules[r].kw_ascii || rs.rules[r].kw_lower.empty()) continue;
        bool hit = false;
        for (const auto& kw : rs.rules[r].kw_lower) {
          auto it = kwhit.find(kw);
          if (it == kwhit.end())
            it = kwhit.emplace(kw, (fbbits & 3) ? contains_fold_runes(content, (size_t)n, kw)
                                                : contains_fold_ascii(content, (size_t)n, kw)).first;
          if ((hit = it->second)) break;
        }
        if (!hit) kws[r] = 0;
      }
      // U+212A / U+017F join ASCII letters under (?i), which the K1 anchors (literal
      // automaton, token-run counters) do not see: a match the kernels may have missed
      // contains one of them, so its start lies within rule_maxlen bytes before it.  A
      // rule without that bound runs its K2 DFA over the file here when its GPU program is
      // exact (relaxed programs leave these runes out of their sets), else the whole file.
      std::vector<int64_t> fold;
      fold_rune_positions(content, n, 2 | 4, &fold);
      // the unbounded rules in one pass of their combined fold DFA: threads injected up to
      // the last rune and followed until they die; an end before the first rune belongs to
      // a match without one (the kernels' candidates cover those)
      std::vector<uint8_t> done(R, 0);
      if (plan.fold_all_dfa && !fold.empty()) {
        const DFA& fd = *plan.fold_all_dfa;
        const size_t nf = plan.fold_rules.size();
        std::vector<uint8_t> want(nf, 0);
        bool any = false;
        for (size_t k = 0; k < nf; k++) {
          const uint32_t r = plan.fold_rules[k];
          want[k] = !(kws[r] == 0 || kws[r] == 3 || wins[r].whole);
          any |= want[k] != 0;
        }
        if (any) {
          const uint64_t td = prof ? __rdtsc() : 0;
          const int64_t q0 = fold.front(), q1 = fold.back();
          // (true: the tail past the last rune reached a state whose threads never die,
          // e.g. a (?s).* rule, and stopped there: its later ends are unknown, so every
          // wanted rule is resolved over the whole file instead)
          const bool cut = run_segment(fd, content, 0, (uint64_t)n, 0, (uint64_t)std::min<int64_t>(n, q1 + 1), ~0u,
                      [&](uint32_t mi, uint64_t pos) {
                        if ((int64_t)pos < q0) return;
                        const auto& m = fd.masks[mi];
                        for (size_t k = 0; k < nf; k++)
                          if (want[k] && ((m[k / 64] >> (k % 64)) & 1))
                            add_end(wins[plan.fold_rules[k]], plan.fold_rules[k], (int64_t)pos);
                      });
          if (prof) tdfa += __rdtsc() - td;
          for (size_t k = 0; k < nf; k++)
            if (want[k]) {
              const uint32_t r = plan.fold_rules[k];
              done[r] = 1;
              wptr[r] = &wins[r];
              if (cut) {
                wins[r].whole = true;
                wins[r].iv.clear();
              } else {
                normalize(wins[r]);
              }
            }
        }
      }
      for (size_t r = 0; r < R; r++) {
        if (done[r] || kws[r] == 0 || kws[r] == 3 || !rs.rules[r].regex || wins[r].whole || fold.empty()) continue;
        RuleWindows& w = wins[r];
        wptr[r] = &w;
        const int64_t ml = plan.rule_maxlen[r];
        if (ml >= 0) {
          for (int64_t q : fold) w.iv.push_back({align_rune(content, n, std::max<int64_t>(0, q - ml)), q});
        } else if (const DFA* fd = plan.rule_fold_dfa[r].get()) {
          // relaxed rule: its fold-rune DFA (a superset that accepts the runes) gives the
          // candidate ends over the file
          w.iv.clear();
          const uint64_t td = prof ? __rdtsc() : 0;
          run_segment(*fd, content, 0, (uint64_t)n, 0, (uint64_t)n, ~0u, [&](uint32_t mi, uint64_t pos) {
            if (fd->masks[mi][0] & 1) add_end(w, (uint32_t)r, (int64_t)pos);
          });
          if (prof) tdfa += __rdtsc() - td;
        } else if (plan.rule_group[r] >= 0 && plan.rule_relax[r] < 0) {
          // only an unrelaxed GPU program keeps U+017F / U+212A in its (?i) sets (relaxed
          // ones drop them, goregex.cpp Compiler::rune): a relaxed rule is resolved whole
          const GroupPlan& g = plan.groups[plan.rule_group[r]];
          size_t local = 0;
          while (g.rules[local] != r) local++;
          const DFA& d = *g.dfa;
          w.iv.clear();
          const uint64_t td = prof ? __rdtsc() : 0;
          run_segment(d, content, 0, (uint64_t)n, 0, (uint64_t)n, ~0u, [&](uint32_t mi, uint64_t pos) {
            if ((d.masks[mi][local / 64] >> (local % 64)) & 1) add_end(w, (uint32_t)r, (int64_t)pos);
          });
          if (prof) tdfa += __rdtsc() - td;
        } else {
          w.whole = true;
          w.iv.clear();
          continue;
        }
        normalize(w);
      }
    }
    if (prof) {
      slots[tid].cyc[6] += __rdtsc() - tf0 - tdfa;
      slots[tid].cyc[7] += tdfa;
    }
    // a rule whose keyword gate is uncertain and that the kernels did not scan (its
    // keyword bits were clear) is resolved over the whole file when the exact gate passes
    for (size_t r = 0; r < R; r++)
      if (kws[r] == 3) {
        kws[r] = 2;
        wins[r].whole = true;
        wptr[r] = &wins[r];
      }
    if (getenv("TSG_DEBUG_RESOLVE"))
      for (size_t r = 0; r < R; r++)
        if (wptr[r]) {
          fprintf(stderr, "file %u rule %s kws %d whole %d:", f, rs.rules[r].id.c_str(), kws[r], (int)wptr[r]->whole);
          for (auto& iv : wptr[r]->iv) fprintf(stderr, " [%ld,%ld]", (long)iv.first, (long)iv.second);
          fprintf(stderr, "\n");
        }
    FileGate gate;
    gate.kw_state = kws.data();
    gate.windows = wptr.data();
    gate.path_allowed = path_ok(f) ? 1 : 0;
    gate.ascii_fold_exact = (fbbits & 3) == 0;
    if (prof)
      for (size_t r = 0; r < R; r++)
        if (wptr[r] && (wptr[r]->whole || (!wptr[r]->iv.empty() && wptr[r]->iv[0].first == 0))) {
          n_whole++;
          if (getenv("TSG_PROF2") && n_whole < 40)
            fprintf(stderr, "whole-prefix: file %u rule %s n=%ld whole=%d iv0=[%ld,%ld] niv=%zu\n", f, rs.rules[r].id.c_str(), (long)n,
                    (int)wptr[r]->whole, wptr[r]->iv.empty() ? -1L : (long)wptr[r]->iv[0].first,
                    wptr[r]->iv.empty() ? -1L : (long)wptr[r]->iv[0].second, wptr[r]->iv.size());
        }
    const uint64_t ts0 = prof ? __rdtsc() : 0;
    scan_file(rs, path, content, (size_t)n, &gate, &res);
    if (prof) slots[tid].cyc[4] += __rdtsc() - ts0;
  });
  if (prof) {
    uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (const auto& sl : slots)
      for (int k = 0; k < 8; k++) t[k] += sl.cyc[k];
    fprintf(stderr, "resolve: parallel part %.1f Mcyc wall; thread Mcyc: no-candidate files %.1f, candidate files %.1f "
            "(%lu files, %ld whole-prefix rule scans; scan_file %.1f), other %.1f\n",
            (__rdtsc() - t_par0) / 1e6, t[0] / 1e6, t[1] / 1e6, (unsigned long)t[3], (long)n_whole, t[4] / 1e6,
            t[2] / 1e6);
    fprintf(stderr, "resolve: fold runes: keyword windows %.1f, bounded-rule windows %.1f, whole-file DFAs %.1f Mcyc\n",
            t[5] / 1e6, t[6] / 1e6, t[7] / 1e6);
  }
}

// Start offsets of the folding runes selected by `which` (1: U+0130 = C4 B0, 2: U+212A =
// E2 84 AA, 4: U+017F = C5 BF), in order.  SSE2 finds their lead bytes 16 at a time.
void fold_rune_positions(const uint8_t* s, int64_t n, uint32_t which, std::vector<int64_t>* out) {
  out->clear();
  const __m128i c4 = _mm_set1_epi8((char)0xC4), c5 = _mm_set1_epi8((char)0xC5), e2 = _mm_set1_epi8((char)0xE2);
  auto check = [&](int64_t q) {
    if ((which & 1) && s[q] == 0xC4 && q + 1 < n && s[q + 1] == 0xB0) out->push_back(q);
    else if ((which & 4) && s[q] == 0xC5 && q + 1 < n && s[q + 1] == 0xBF) out->push_back(q);
    else if ((which & 2) && s[q] == 0xE2 && q + 2 < n && s[q + 1] == 0x84 && s[q + 2] == 0xAA) out->push_back(q);
  };
  int64_t q = 0;
  for (; q + 16 <= n; q += 16) {
    const __m128i b = _mm_loadu_si128((const __m128i*)(s + q));
    uint32_t bits = (uint32_t)_mm_movemask_epi8(
        _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(b, c4), _mm_cmpeq_epi8(b, c5)), _mm_cmpeq_epi8(b, e2)));
    while (bits) {
      check(q + __builtin_ctz(bits));
      bits &= bits - 1;
    }
  }
  for (; q < n; q++) check(q);
}

// ------------------------------------------------------------------ kernel emulation

void k1_reference(const Plan& plan, const BatchView& bv, uint32_t chunk, std::vector<uint32_t>* kw,
                  std::vector<uint32_t>* ev) {
  const uint32_t F = bv.nfiles;
  const uint64_t total = bv.offsets[F];
  const DFA& d = *plan.kw_dfa;
  const int nc = d.nclasses;
  const int W = plan.kw_words;
  kw->assign((size_t)F * W, 0);
  ev->assign((total + chunk - 1) / chunk, 0);
  uint32_t s = d.start[kCtxBOT];
  uint32_t cu = 0, cd = 0, f = 0;
  for (uint64_t p = 0; p < total; p++) {
    while (bv.offsets[f + 1] <= p) f++;  // the file holding byte p (skips empty files)
    const uint8_t c = bv.data[p];
    s = d.next[(size_t)s * nc + d.cls[c]];
    uint32_t e = 0;
    // arrival in state s: the literals its match set holds end with byte p
    const uint32_t mi = d.eot_acc[s];
    if (mi) {
      const auto& m = d.masks[mi];
      const uint64_t avail = p - bv.offsets[f] + 1;
      for (int k = 0; k < plan.n_kw; k++)
        if (((m[k / 64] >> (k % 64)) & 1) && plan.kw_len[k] <= avail)
          (*kw)[(size_t)f * W + k / 32] |= 1u << (k % 32);
      e |= plan.kw_mask_events[mi];
    }
    cu = (plan.run_cls[c] & 1) ? cu + 1 : 0;
    cd = (plan.run_cls[c] & 2) ? cd + 1 : 0;
    if ((int)cu >= plan.run_k[0]) e |= kEvRunU;
    if ((int)cd >= plan.run_k[1]) e |= kEvRunD;
    (*ev)[p / chunk] |= e;
  }
  k1x_reference(plan, bv, chunk, kw, ev);
}

// K1X semantics (the hashed literals of large rule sets): every occurrence of a literal in
// the ASCII-lowercased stream ending at byte q sets its event bits on chunk q / chunk, and
// its keyword bit for the file holding q when the whole literal lies inside that file.
void k1x_reference(const Plan& plan, const BatchView& bv, uint32_t chunk, std::vector<uint32_t>* kw,
                   std::vector<uint32_t>* ev) {
  if (plan.x_lits.empty()) return;
  const uint64_t total = bv.offsets[bv.nfiles];
  std::unordered_map<uint32_t, std::vector<uint32_t>> by4;
  for (size_t i = 0; i < plan.x_lits.size(); i++) by4[x_prefix4((const uint8_t*)plan.x_lits[i].data())].push_back((uint32_t)i);
  auto low = [](uint8_t c) -> uint8_t { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; };
  for (uint64_t p = 0; p + 4 <= total; p++) {
    const uint8_t b4[4] = {low(bv.data[p]), low(bv.data[p + 1]), low(bv.data[p + 2]), low(bv.data[p + 3])};
    auto it = by4.find(x_prefix4(b4));
    if (it == by4.end()) continue;
    for (uint32_t i : it->second) {
      const std::string& L = plan.x_lits[i];
      if (p + L.size() > total) continue;
      size_t t = 4;
      while (t < L.size() && low(bv.data[p + t]) == (uint8_t)L[t]) t++;
      if (t < L.size()) continue;
      const uint64_t q = p + L.size() - 1;
      (*ev)[q / chunk] |= plan.x_event[i];
      if (plan.x_kw[i] >= 0) {
        const uint32_t f = (uint32_t)(std::upper_bound(bv.offsets, bv.offsets + bv.nfiles + 1, q) - bv.offsets) - 1;
        if (p >= bv.offsets[f]) (*kw)[(size_t)f * plan.kw_words + plan.x_kw[i] / 32] |= 1u << (plan.x_kw[i] % 32);
      }
    }
  }
}

// The list kernel's output form for one item (kernels.hip k2_list_pair / Lane::tail with
// word records): an accepting 16-B word (batch-aligned; its part inside [a, b) or the tail)
// becomes one kCandWord record {file, group, row before its first byte, that byte's offset};
// a tail stops at a word boundary past ext_cap or in an immortal state (kCandWhole for the
// group's rules); end-of-text accepts are per-rule candidates.  TSG_EMU_WORDREC selects it
// (tests: it drives resolve_batch's word expansion without a device).
static void emulate_words(const DFA& d, uint32_t gi, const std::vector<uint32_t>& rules, const uint8_t* data,
                          uint32_t f, uint64_t fs, uint64_t fe, uint64_t a, uint64_t b, uint32_t ext_cap,
                          std::vector<Candidate>* out) {
  const uint32_t nc = (uint32_t)d.nclasses, ncd = std::max<uint32_t>(2, nc);
  auto word_rec = [&](uint32_t s0, uint64_t p0) {
    out->push_back({f, kCandTrans | kCandWord | (gi << 16) | (s0 * ncd), (uint32_t)(p0 - fs)});
  };
  auto eot = [&](uint32_t s) {
    if (!d.eot_acc[s]) return;
    const auto& m = d.masks[d.eot_acc[s]];
    for (size_t k = 0; k < rules.size(); k++)
      if ((m[k / 64] >> (k % 64)) & 1) out->push_back({f, rules[k], (uint32_t)(fe - fs)});
  };
  // bytes [p, e) of one word from state s: the state after them, accept seen
  auto step = [&](uint32_t& s, uint64_t p, uint64_t e) {
    bool acc = false;
    for (; p < e; p++) {
      const size_t x = (size_t)s * nc + d.cls[data[p]];
      acc |= d.acc[x] != 0;
      s = d.next[x];
    }
    return acc;
  };
  uint32_t s = (a == fs) ? d.start[kCtxBOT] : d.start[DFA::ctx_of(data[a - 1], d)];
  for (uint64_t p = a; p < b;) {
    const uint64_t e = std::min<uint64_t>(b, (p | 15) + 1);
    const uint32_t s0 = s;
    if (step(s, p, e)) word_rec(s0, p);
    p = e;
  }
  if (b >= fe) {
    eot(s);
    return;
  }
  s = d.to_noinject[s];
  uint64_t q = b;
  while (q < fe && !d.dead[s]) {
    if (q - b >= ext_cap || (s < d.immortal.size() && d.immortal[s])) {
      for (uint32_t r : rules) out->push_back({f, r, kCandWhole});
      return;
    }
    const uint64_t e = std::min<uint64_t>(fe, (q | 15) + 1);
    const uint32_t s0 = s;
    if (step(s, q, e)) word_rec(s0, q);
    q = e;
  }
  if (q >= fe && !d.dead[s]) eot(s);
}

void emulate_kernels(const Plan& plan, const BatchView& bv, uint32_t chunk, uint32_t ext_cap,
                     KernelOutput* ko, std::vector<uint64_t>* group_item_bytes) {
  const uint32_t F = bv.nfiles;
  const bool word_recs = knobs().emu_wordrec.load() && plan.groups.size() <= 0x3FFF;
  std::vector<uint32_t> ev;
  k1_reference(plan, bv, chunk, &ko->kw, &ev);
  ko->cand.clear();
  ko->overflow.assign(F, 0);
  if (group_item_bytes) group_item_bytes->assign(plan.groups.size(), 0);
  for (size_t gi = 0; gi < plan.groups.size(); gi++) {
    const GroupPlan& g = plan.groups[gi];
    const uint32_t back = group_back(g, chunk);
    const DFA& d = *g.dfa;
    for (uint32_t f = 0; f < F; f++) {
      const uint64_t fs = bv.offsets[f], fe = bv.offsets[f + 1];
      if (fe == fs) continue;
      const uint32_t* kw = ko->kw.data() + (size_t)f * plan.kw_words;
      bool gate = g.always;
      for (int w = 0; w < plan.kw_words && !gate; w++) gate = (kw[w] & g.kwmask[w]) != 0;
      if (!gate) continue;
      const uint64_t c0 = fs / chunk, c1 = (fe - 1) / chunk;
      for (uint64_t c = c0; c <= c1; c++) {
        bool need = (g.events & kEvAlways) != 0;
        for (uint64_t q = c; q <= std::min<uint64_t>(c + back, c1) && !need; q++) need = (ev[q] & g.events) != 0;
        if (!need) continue;
        const uint64_t a = std::max<uint64_t>(fs, c * chunk), b = std::min<uint64_t>(fe, (c + 1) * chunk);
        if (group_item_bytes) (*group_item_bytes)[gi] += b - a;
        if (word_recs) {
          emulate_words(d, (uint32_t)gi, g.rules, bv.data, f, fs, fe, a, b, ext_cap, &ko->cand);
          continue;
        }
        bool o = run_segment(d, bv.data, fs, fe, a, b, ext_cap, [&](uint32_t mi, uint64_t pos) {
          const auto& m = d.masks[mi];
          for (size_t k = 0; k < g.rules.size(); k++)
            if ((m[k / 64] >> (k % 64)) & 1) ko->cand.push_back({f, g.rules[k], (uint32_t)pos});
        });
        if (o)  // a tail past ext_cap: the group's rules over the whole file (kCandWhole)
          for (uint32_t r : g.rules) ko->cand.push_back({f, r, kCandWhole});
      }
    }
  }
}

}  // namespace tsg
