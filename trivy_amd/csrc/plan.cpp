// GPU plan construction, host resolver, CPU batch path and kernel emulation.
#include "plan.hpp"

#include <algorithm>
#include <atomic>
#include <map>
#include <thread>

namespace tsg {

static bool is_ascii(const std::string& s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

std::unique_ptr<Plan> build_plan(const Ruleset& rs, const PlanOptions& opt, std::string* err) {
  auto p = std::make_unique<Plan>();
  const size_t R = rs.rules.size();
  p->rule_kw_mode.assign(R, kKwAlways);
  p->rule_kws.assign(R, {});
  p->rule_group.assign(R, -1);
  p->rule_hostonly.assign(R, 0);
  p->rule_maxlen.assign(R, -1);

  // ---- K1 keyword automaton
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
  {
    DFAOptions o;
    o.max_states = 32767;
    o.with_noinject = false;
    std::string e;
    p->kw_dfa = build_keyword_dfa(kws, o, &e);
    if (!p->kw_dfa) {
      if (err) *err = "keyword automaton: " + e;
      return nullptr;
    }
  }

  // ---- K2 rule groups (greedy packing under the state / table caps)
  DFAOptions one;
  one.max_states = opt.max_group_states;
  std::vector<uint32_t> cur;
  auto group_kwmask = [&](GroupPlan& g) {
    g.kwmask.assign(p->kw_words, 0);
    for (uint32_t r : g.rules) {
      if (p->rule_kw_mode[r] != kKwBits) {
        g.always = true;
        continue;
      }
      for (uint32_t k : p->rule_kws[r]) g.kwmask[k / 32] |= 1u << (k % 32);
    }
    for (int k = p->fb_kw0; k < p->n_kw; k++) g.kwmask[k / 32] |= 1u << (k % 32);
  };
  auto fits = [&](const DFA& d, size_t nrules) {
    return d.nstates <= opt.max_group_states &&
           (size_t)d.nstates * d.nclasses * 2 <= (size_t)opt.max_group_table_bytes &&
           (int)nrules <= opt.max_rules_per_group;
  };
  std::unique_ptr<DFA> cur_dfa;
  auto flush = [&]() {
    if (cur.empty()) return;
    GroupPlan g;
    g.dfa = std::move(cur_dfa);
    g.rules = cur;
    group_kwmask(g);
    for (uint32_t r : cur) p->rule_group[r] = (int)p->groups.size();
    p->groups.push_back(std::move(g));
    cur.clear();
  };
  p->rule_relax.assign(R, -1);
  p->rule_atoms.assign(R, -1);
  p->rule_winback.assign(R, -1);
  p->rule_prog.assign(R, Prog{});
  for (size_t r = 0; r < R; r++) {
    const RuleC& rule = rs.rules[r];
    if (!rule.regex) continue;
    p->rule_maxlen[r] = max_match_len(rule.regex->prog());
    p->rule_winback[r] = p->rule_maxlen[r];
    // exact program first, then ever stronger relaxations of counted repetitions, then
    // ever shorter prefixes of the top-level concatenation
    std::unique_ptr<DFA> single;
    for (int k : {-1, 32, 16, 8, 4, 2, 1, 0}) {
      Prog pr = k < 0 ? rule.regex->prog() : rule.regex->RelaxedProg(k);
      std::string e;
      auto d = build_dfa({&pr}, one, &e);
      if (d && fits(*d, 1)) {
        single = std::move(d);
        p->rule_relax[r] = k;
        p->rule_prog[r] = std::move(pr);
        break;
      }
    }
    for (int t = rule.regex->NumAtoms() - 1; !single && t >= 1; t--) {
      for (int k : {8, 2, 0}) {
        Prog pr = rule.regex->RelaxedProg(k, t);
        std::string e;
        auto d = build_dfa({&pr}, one, &e);
        if (d && fits(*d, 1)) {
          single = std::move(d);
          p->rule_relax[r] = k;
          p->rule_atoms[r] = t;
          p->rule_prog[r] = std::move(pr);
          p->rule_winback[r] = max_match_len(rule.regex->RelaxedProg(-1, t));
          break;
        }
      }
    }
    if (!single) {
      p->rule_hostonly[r] = 1;
      continue;
    }
    if (cur.empty()) {
      cur.push_back((uint32_t)r);
      cur_dfa = std::move(single);
      continue;
    }
    std::vector<const Prog*> progs;
    for (uint32_t q : cur) progs.push_back(&p->rule_prog[q]);
    progs.push_back(&p->rule_prog[r]);
    std::string e;
    auto merged = build_dfa(progs, one, &e);
    if (merged && fits(*merged, cur.size() + 1)) {
      cur.push_back((uint32_t)r);
      cur_dfa = std::move(merged);
    } else {
      flush();
      cur.push_back((uint32_t)r);
      cur_dfa = std::move(single);
    }
  }
  flush();

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
template <class F>
static void parallel_for(size_t n, int nthreads, F f) {
  if (nthreads <= 1 || n < 64) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  const size_t grain = 64;
  for (int t = 0; t < nthreads; t++) {
    th.emplace_back([&]() {
      for (;;) {
        size_t s = next.fetch_add(grain);
        if (s >= n) break;
        size_t e = std::min(n, s + grain);
        for (size_t i = s; i < e; i++) f(i);
      }
    });
  }
  for (auto& t : th) t.join();
}

static bool path_allowed(const Ruleset& rs, const Plan* plan, const std::string& path) {
  if (plan && plan->allow_path_dfa && is_ascii(path)) {
    std::vector<uint64_t> m;
    plan->allow_path_dfa->match_any((const uint8_t*)path.data(), path.size(), &m);
    for (uint64_t w : m)
      if (w) return true;
    return false;
  }
  return rs.AllowPath(path);
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

void resolve_batch(const Ruleset& rs, const Plan& plan, const BatchView& b,
                   const KernelOutput& ko, int nthreads, std::vector<FileResult>* out) {
  const uint32_t F = b.nfiles;
  const size_t R = rs.rules.size();
  out->assign(F, FileResult{});
  // bucket candidates by file, sorted by (rule, end)
  std::vector<Candidate> cand = ko.cand;
  std::sort(cand.begin(), cand.end(), [](const Candidate& x, const Candidate& y) {
    if (x.file != y.file) return x.file < y.file;
    if (x.rule != y.rule) return x.rule < y.rule;
    return x.end < y.end;
  });
  std::vector<uint32_t> first(F + 1, 0);
  for (const auto& c : cand) first[c.file + 1]++;
  for (uint32_t f = 0; f < F; f++) first[f + 1] += first[f];

  std::vector<uint32_t> hostonly;
  for (size_t r = 0; r < R; r++)
    if (plan.rule_hostonly[r]) hostonly.push_back((uint32_t)r);

  parallel_for(F, nthreads, [&](size_t fi) {
    const uint32_t f = (uint32_t)fi;
    std::string path(b.paths + b.path_offsets[f], b.path_offsets[f + 1] - b.path_offsets[f]);
    const uint8_t* content = b.data + b.offsets[f];
    const int64_t n = (int64_t)(b.offsets[f + 1] - b.offsets[f]);
    FileResult& res = (*out)[f];
    if (n == 0) {  // the kernels skip empty files; only empty matches are possible
      scan_file(rs, path, content, 0, nullptr, &res);
      return;
    }
    const uint32_t* kw = ko.kw.data() + (size_t)f * plan.kw_words;
    bool fb = false;
    for (int k = plan.fb_kw0; k < plan.n_kw; k++) fb |= (kw[k / 32] >> (k % 32)) & 1;
    auto kw_state = [&](size_t r) -> uint8_t {
      switch (plan.rule_kw_mode[r]) {
        case kKwAlways: return 1;
        case kKwUnknown: return 2;
        default:
          if (fb) return 2;
          for (uint32_t k : plan.rule_kws[r])
            if ((kw[k / 32] >> (k % 32)) & 1) return 1;
          return 0;
      }
    };
    // kernel overflow, or a folding rune (U+0130/U+212A/U+017F) the GPU programs ignore:
    // resolve every rule over the whole file
    const bool ovf = (!ko.overflow.empty() && ko.overflow[f]) || fb;
    bool any_host = false;
    for (uint32_t r : hostonly)
      if (kw_state(r) != 0) any_host = true;
    if (first[f] == first[f + 1] && !ovf && !any_host) {
      res.status = path_allowed(rs, &plan, path) ? kPathAllowed : kNoFindings;
      return;
    }
    std::vector<RuleWindows> wins(R);
    std::vector<const RuleWindows*> wptr(R, nullptr);
    std::vector<uint8_t> kws(R);
    for (size_t r = 0; r < R; r++) kws[r] = kw_state(r);
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
    for (uint32_t k = first[f]; k < first[f + 1];) {
      uint32_t r = cand[k].rule;
      uint32_t e = k;
      while (e < first[f + 1] && cand[e].rule == r) e++;
      RuleWindows& w = wins[r];
      wptr[r] = &w;
      if (!w.whole) {
        // every match start lies in [end - winback, end] of some candidate end offset
        const int64_t back = plan.rule_winback[r];
        for (uint32_t j = k; j < e; j++) {
          int64_t end = cand[j].end;
          int64_t lo = back < 0 ? 0 : align_rune(content, n, std::max<int64_t>(0, end - back));
          if (!w.iv.empty() && lo <= w.iv.back().second + 1) {
            w.iv.back().second = std::max<int64_t>(w.iv.back().second, end);
          } else {
            w.iv.push_back({lo, end});
          }
        }
      }
      k = e;
    }
    FileGate gate;
    gate.kw_state = kws.data();
    gate.windows = wptr.data();
    scan_file(rs, path, content, (size_t)n, &gate, &res);
  });
}

// ------------------------------------------------------------------ kernel emulation
namespace {

// One lane's work on one file segment [a, b) of file [fs, fe): inject mode over the
// segment, then (if the file continues) noinject mode until every thread started in
// the segment has died.  on_acc(mask_index, position_in_file).
template <class OnAcc>
bool run_segment(const DFA& d, const uint8_t* data, uint64_t fs, uint64_t fe, uint64_t a,
                 uint64_t b, uint32_t ext_cap, OnAcc on_acc) {
  const int nc = d.nclasses;
  uint32_t s = (a == fs) ? d.start[kCtxBOT] : d.start[DFA::ctx_of(data[a - 1], d)];
  for (uint64_t p = a; p < b; p++) {
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
    if (p - b >= ext_cap) return true;  // overflow: host resolves the file whole
    size_t e = (size_t)s * nc + d.cls[data[p]];
    if (d.acc[e]) on_acc(d.acc[e], p - fs);
    s = d.next[e];
    p++;
  }
  if (p == fe && !d.dead[s] && d.eot_acc[s]) on_acc(d.eot_acc[s], fe - fs);
  return false;
}

// K1: keywords are bounded, so the lane simply keeps going in inject mode for
// max_len - 1 bytes past its piece (every keyword occurrence that starts in the piece
// is seen; occurrences found in the overlap are real occurrences too).
template <class OnAcc>
void run_kw_segment(const DFA& d, const uint8_t* data, uint64_t fs, uint64_t fe, uint64_t a,
                    uint64_t b, OnAcc on_acc) {
  const int nc = d.nclasses;
  uint64_t ext = d.max_len > 1 ? (uint64_t)d.max_len - 1 : 0;
  uint64_t stop = std::min(fe, b + ext);
  uint32_t s = (a == fs) ? d.start[kCtxBOT] : d.start[DFA::ctx_of(data[a - 1], d)];
  for (uint64_t p = a; p < stop; p++) {
    size_t e = (size_t)s * nc + d.cls[data[p]];
    if (d.acc[e]) on_acc(d.acc[e], p - fs);
    s = d.next[e];
  }
  if (stop == fe && d.eot_acc[s]) on_acc(d.eot_acc[s], fe - fs);
}

}  // namespace

void emulate_kernels(const Plan& plan, const BatchView& bv, uint32_t chunk, uint32_t ext_cap,
                     KernelOutput* ko) {
  const uint32_t F = bv.nfiles;
  const uint64_t total = bv.offsets[F];
  ko->kw.assign((size_t)F * plan.kw_words, 0);
  ko->cand.clear();
  ko->overflow.assign(F, 0);
  const uint64_t nchunks = (total + chunk - 1) / chunk;
  for (int pass = 0; pass < 2; pass++) {
    for (uint64_t c = 0; c < nchunks; c++) {
      uint64_t a = c * chunk, b = std::min<uint64_t>(a + chunk, total);
      uint32_t f = (uint32_t)(std::upper_bound(bv.offsets, bv.offsets + F + 1, a) - bv.offsets) - 1;
      while (a < b && f < F) {
        uint64_t fs = bv.offsets[f], fe = bv.offsets[f + 1];
        if (fe == fs) {
          f++;
          continue;
        }
        uint64_t se = std::min(b, fe);
        if (pass == 0) {
          const DFA& d = *plan.kw_dfa;
          run_kw_segment(d, bv.data, fs, fe, a, se, [&](uint32_t mi, uint64_t) {
            const auto& m = d.masks[mi];
            for (int k = 0; k < plan.n_kw; k++)
              if ((m[k / 64] >> (k % 64)) & 1) ko->kw[(size_t)f * plan.kw_words + k / 32] |= 1u << (k % 32);
          });
        } else {
          const uint32_t* kw = ko->kw.data() + (size_t)f * plan.kw_words;
          for (const auto& g : plan.groups) {
            bool gate = g.always;
            for (int w = 0; w < plan.kw_words && !gate; w++) gate = (kw[w] & g.kwmask[w]) != 0;
            if (!gate) continue;
            const DFA& d = *g.dfa;
            bool o = run_segment(d, bv.data, fs, fe, a, se, ext_cap, [&](uint32_t mi, uint64_t pos) {
              const auto& m = d.masks[mi];
              for (size_t k = 0; k < g.rules.size(); k++)
                if ((m[k / 64] >> (k % 64)) & 1) ko->cand.push_back({f, g.rules[k], (uint32_t)pos});
            });
            if (o) ko->overflow[f] = 1;
          }
        }
        a = se;
        f++;
      }
    }
  }
}

}  // namespace tsg
