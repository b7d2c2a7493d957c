// C ABI, host part (rule compilation, CPU scans, test hooks).  See include/trivy_secret.h.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>

#include "internal.hpp"
#include "k1f.hpp"

namespace tsg {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

static void copy_err(const std::string& m, char* err, size_t len) {
  if (!err || len == 0) return;
  size_t n = std::min(len - 1, m.size());
  std::memcpy(err, m.data(), n);
  err[n] = 0;
}

static std::string str(const char* s) { return s ? std::string(s) : std::string(); }

static std::shared_ptr<Regexp> compile_opt(const char* src, std::string* err) {
  if (!src) return nullptr;
  std::string e;
  auto re = Regexp::Compile(src, &e);
  if (!re) *err = "regexp compile error: " + e;
  return re;
}

static int hw_threads(int n) {
  if (n > 0) return n;
  unsigned h = std::thread::hardware_concurrency();
  if (h == 0) h = 4;
  return (int)std::min<unsigned>(h, 16);
}

}  // namespace tsg

using namespace tsg;

extern "C" {

const char* tsg_last_error(void) { return g_last_error.c_str(); }

int tsg_ruleset_compile(const tsg_rule_desc* rules, uint32_t n_rules,
                        const tsg_allow_rule_desc* allow_rules, uint32_t n_allow_rules,
                        const char* const* exclude_regexes, uint32_t n_exclude_regexes,
                        tsg_ruleset** out, char* err, size_t err_len) {
  if (!out || (n_rules && !rules) || (n_allow_rules && !allow_rules) ||
      (n_exclude_regexes && !exclude_regexes)) {
    copy_err("bad argument", err, err_len);
    return fail(TSG_ERR_ARG, "bad argument");
  }
  try {
    auto h = std::make_unique<tsg_ruleset>();
    std::string e;
    auto allow_of = [&](const tsg_allow_rule_desc& a, AllowRuleC* o) -> bool {
      o->id = str(a.id);
      o->description = str(a.description);
      o->regex = compile_opt(a.regex, &e);
      if (a.regex && !o->regex) return false;
      o->path = compile_opt(a.path, &e);
      if (a.path && !o->path) return false;
      return true;
    };
    for (uint32_t i = 0; i < n_rules; i++) {
      const tsg_rule_desc& d = rules[i];
      RuleC r;
      r.id = str(d.id);
      r.category = str(d.category);
      r.title = str(d.title);
      r.severity = str(d.severity);
      r.secret_group_name = str(d.secret_group_name);
      r.regex = compile_opt(d.regex, &e);
      if (d.regex && !r.regex) goto bad;
      r.path = compile_opt(d.path, &e);
      if (d.path && !r.path) goto bad;
      for (uint32_t k = 0; k < d.n_keywords; k++) {
        std::string kw = str(d.keywords[k]), low;
        r.keywords.push_back(kw);
        go_to_lower((const uint8_t*)kw.data(), kw.size(), &low);  // strings.ToLower
        r.kw_lower.push_back(low);
        for (unsigned char ch : low) r.kw_ascii &= ch < 0x80;
      }
      for (uint32_t k = 0; k < d.n_allow_rules; k++) {
        AllowRuleC a;
        if (!allow_of(d.allow_rules[k], &a)) goto bad;
        r.allow.push_back(std::move(a));
      }
      for (uint32_t k = 0; k < d.n_exclude_regexes; k++) {
        auto re = compile_opt(d.exclude_regexes[k], &e);
        if (!re) goto bad;
        r.exclude.push_back(re);
      }
      if (r.regex && !r.secret_group_name.empty()) {
        const auto& names = r.regex->SubexpNames();
        for (size_t g = 0; g < names.size(); g++)
          if (names[g] == r.secret_group_name) r.group_idx.push_back((int)g);
      }
      h->rs.rules.push_back(std::move(r));
    }
    for (uint32_t k = 0; k < n_allow_rules; k++) {
      AllowRuleC a;
      if (!allow_of(allow_rules[k], &a)) goto bad;
      h->rs.allow.push_back(std::move(a));
    }
    for (uint32_t k = 0; k < n_exclude_regexes; k++) {
      auto re = compile_opt(exclude_regexes[k], &e);
      if (!re) goto bad;
      h->rs.exclude.push_back(re);
    }
    {
      PlanOptions po;
      // Rule sets of a few hundred rules get K2 groups of up to 2,048 states / 64 KiB (the
      // u16 row offsets' limit): the run-event groups, which scan the same chunks, merge 7 -> 6
      // on the builtin rules (K2 0.127 -> 0.118 ms, items 0.060 -> 0.056 ms per GiB,
      // profiles/r05/kn1).  Larger sets keep 1,024 / 48 KiB: the merged DFAs' construction
      // grows fast (1,083 rules: 8 -> 25 s).
      if (h->rs.rules.size() <= 256) {
        po.max_group_states = 2048;
        po.max_group_table_bytes = 64 * 1024;
      }
      if (knobs().group_states.load() > 0) po.max_group_states = (int)knobs().group_states.load();
      if (knobs().group_table_kib.load() > 0) po.max_group_table_bytes = (int)knobs().group_table_kib.load() * 1024;
      std::string pe;
      h->plan = build_plan(h->rs, po, &pe);
      if (!h->plan) {
        copy_err(pe, err, err_len);
        return fail(TSG_ERR_INTERNAL, pe);
      }
    }
    *out = h.release();
    return TSG_OK;
  bad:
    copy_err(e, err, err_len);
    return fail(TSG_ERR_CONFIG, e);
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    copy_err(ex.what(), err, err_len);
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

void tsg_ruleset_destroy(tsg_ruleset* rs) { delete rs; }

int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t path_len) {
  if (!rs || (!path && path_len)) return fail(TSG_ERR_ARG, "bad argument");
  return rs->rs.AllowPath(std::string(path ? path : "", path_len)) ? 1 : 0;
}

int tsg_ruleset_get_info(const tsg_ruleset* rs, tsg_ruleset_info* o) {
  if (!rs || !o) return fail(TSG_ERR_ARG, "bad argument");
  const Plan& p = *rs->plan;
  std::memset(o, 0, sizeof(*o));
  o->n_rules = (uint32_t)rs->rs.rules.size();
  o->n_keywords = (uint32_t)p.n_kw;
  o->n_groups = (uint32_t)p.groups.size();
  for (uint8_t h : p.rule_hostonly) o->n_hostonly += h;
  o->kw_states = (uint32_t)p.kw_dfa->nstates;
  o->kw_classes = (uint32_t)p.kw_dfa->nclasses;
  o->k1x_literals = (uint32_t)p.x_lits.size();
  uint64_t tb = (uint64_t)p.kw_dfa->nstates * p.kw_dfa->nclasses * 2;
  for (const auto& g : p.groups) {
    o->max_group_states = std::max<uint32_t>(o->max_group_states, (uint32_t)g.dfa->nstates);
    tb += (uint64_t)g.dfa->nstates * g.dfa->nclasses * 2;
  }
  o->table_bytes = tb;
  return TSG_OK;
}

int tsg_scan_cpu(const tsg_ruleset* rs, const char* path, size_t path_len, const uint8_t* content,
                 size_t len, tsg_result** out) {
  if (!rs || !out || (!content && len) || (!path && path_len)) return fail(TSG_ERR_ARG, "bad argument");
  try {
    FileResult fr;
    scan_file(rs->rs, std::string(path ? path : "", path_len), content, len, nullptr, &fr);
    auto r = std::make_unique<tsg_result>();
    serialize_results({fr}, &r->buf);
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_scan_cpu_batch(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                       uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                       int nthreads, tsg_result** out) {
  if (!rs || !out || !offsets || !path_offsets) return fail(TSG_ERR_ARG, "bad argument");
  try {
    BatchView b{data, offsets, nfiles, paths, path_offsets};
    std::vector<FileResult> res;
    scan_batch_cpu(rs->rs, b, hw_threads(nthreads), &res);
    auto r = std::make_unique<tsg_result>();
    serialize_results(res, &r->buf);
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_scan_batch_emulated(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                            uint32_t nfiles, const char* paths, const uint64_t* path_offsets,
                            uint32_t chunk, tsg_result** out) {
  if (!rs || !out || !offsets || !path_offsets || chunk == 0) return fail(TSG_ERR_ARG, "bad argument");
  try {
    BatchView b{data, offsets, nfiles, paths, path_offsets};
    KernelOutput ko;
    auto t0 = std::chrono::steady_clock::now();
    emulate_kernels(*rs->plan, b, chunk, 1u << 16, &ko);
    const std::string u = knob_kw_unknown();
    if (!u.empty()) {
      // test hook: as after K1 adaptation, these keywords' bits are not reported and their
      // gates are checked exactly on the host
      const Plan& p = *rs->plan;
      ko.kw_unknown.assign(p.n_kw, 0);
      std::string list(u);
      for (size_t r = 0; r < rs->rs.rules.size(); r++)
        for (size_t j = 0; j < p.rule_kws[r].size(); j++) {
          const std::string& kw = rs->rs.rules[r].kw_lower[j];
          if (("," + list + ",").find("," + kw + ",") == std::string::npos) continue;
          const uint32_t k = p.rule_kws[r][j];
          ko.kw_unknown[k] = 1;
          for (uint32_t f = 0; f < nfiles; f++) ko.kw[(size_t)f * p.kw_words + k / 32] &= ~(1u << (k % 32));
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    BatchResult res;
    resolve_batch(rs->rs, *rs->plan, b, ko.view(), hw_threads(0), &res);
    auto t2 = std::chrono::steady_clock::now();
    auto r = std::make_unique<tsg_result>();
    serialize_batch(res, &r->buf, hw_threads(0));
    auto t3 = std::chrono::steady_clock::now();
    if (getenv("TSG_PROF"))
      fprintf(stderr, "emulate %.1f ms resolve %.1f ms serialize %.1f ms (%zu candidates)\n",
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count(),
              std::chrono::duration<double, std::milli>(t3 - t2).count(), ko.cand.size());
    *out = r.release();
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_emulate_candidate_stats(const tsg_ruleset* rs, const uint8_t* data,
                                const uint64_t* offsets, uint32_t nfiles, uint32_t chunk,
                                uint64_t* cand_per_rule, uint64_t* gated_bytes_per_group) {
  if (!rs || !offsets || chunk == 0) return fail(TSG_ERR_ARG, "bad argument");
  try {
    std::vector<uint64_t> poff(nfiles + 1, 0);
    BatchView b{data, offsets, nfiles, "", poff.data()};
    KernelOutput ko;
    std::vector<uint64_t> gib;
    emulate_kernels(*rs->plan, b, chunk, 1u << 16, &ko, &gib);
    if (cand_per_rule) {
      std::fill(cand_per_rule, cand_per_rule + rs->rs.rules.size(), 0);
      for (const auto& c : ko.cand) cand_per_rule[c.rule]++;
    }
    if (gated_bytes_per_group) std::copy(gib.begin(), gib.end(), gated_bytes_per_group);
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_emulate_k1(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                   uint32_t nfiles, uint32_t chunk, uint32_t* kw, size_t kw_len, uint32_t* ev,
                   size_t ev_len) {
  if (!rs || !offsets || chunk == 0) return fail(TSG_ERR_ARG, "bad argument");
  try {
    std::vector<uint64_t> poff(nfiles + 1, 0);
    BatchView b{data, offsets, nfiles, "", poff.data()};
    std::vector<uint32_t> k, e;
    k1_reference(*rs->plan, b, chunk, &k, &e);
    if (kw) std::memcpy(kw, k.data(), sizeof(uint32_t) * std::min(kw_len, k.size()));
    if (ev) std::memcpy(ev, e.data(), sizeof(uint32_t) * std::min(ev_len, e.size()));
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_emulate_k1f(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                    uint32_t nfiles, uint32_t chunk, const uint32_t* quiet_ids, uint32_t nquiet,
                    uint32_t sample_kib, uint32_t* kw, size_t kw_len, uint32_t* ev, size_t ev_len,
                    uint64_t* stats) {
  if (!rs || !offsets || chunk == 0 || (nquiet && !quiet_ids)) return fail(TSG_ERR_ARG, "bad argument");
  try {
    const Plan& p = *rs->plan;
    std::vector<uint8_t> quiet(p.n_lit, 0);
    for (uint32_t i = 0; i < nquiet; i++) {
      if (quiet_ids[i] >= (uint32_t)p.n_lit) return fail(TSG_ERR_ARG, "no such K1 literal");
      quiet[quiet_ids[i]] = 1;
    }
    K1FTables t;
    std::string why;
    const size_t smp = std::min<uint64_t>((uint64_t)sample_kib << 10, offsets[nfiles]);
    if (!k1f_build(p, quiet, &t, &why, smp ? data : nullptr, smp)) return fail(TSG_ERR_CONFIG, "K1F does not apply: " + why);
    std::vector<uint64_t> poff(nfiles + 1, 0);
    BatchView b{data, offsets, nfiles, "", poff.data()};
    std::vector<uint32_t> k, e;
    uint64_t st[2];
    k1f_emulate(p, t, b, chunk, &k, &e, st);
    if (kw) std::memcpy(kw, k.data(), sizeof(uint32_t) * std::min(kw_len, k.size()));
    if (ev) std::memcpy(ev, e.data(), sizeof(uint32_t) * std::min(ev_len, e.size()));
    if (stats) {
      stats[0] = st[0];
      stats[1] = st[1];
      stats[2] = t.nlit;
      stats[3] = 0;
    }
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_INTERNAL, ex.what());
  }
}

int tsg_ruleset_rule_plan(const tsg_ruleset* rs, uint32_t rule, int32_t* group, int32_t* relax,
                          int64_t* max_len) {
  if (!rs || rule >= rs->rs.rules.size()) return fail(TSG_ERR_ARG, "bad argument");
  const Plan& p = *rs->plan;
  if (group) *group = p.rule_hostonly[rule] ? -1 : p.rule_group[rule];
  if (relax) *relax = p.rule_relax[rule];
  if (max_len) *max_len = p.rule_maxlen[rule];
  return TSG_OK;
}

int tsg_ruleset_rule_anchor(const tsg_ruleset* rs, uint32_t rule, uint32_t* event, int64_t* evdist,
                            char* desc, size_t desc_len) {
  if (!rs || rule >= rs->rs.rules.size()) return fail(TSG_ERR_ARG, "bad argument");
  const Plan& p = *rs->plan;
  if (event) *event = p.rule_event[rule];
  if (evdist) *evdist = p.rule_evdist[rule];
  copy_err(p.rule_anchor[rule], desc, desc_len);
  return TSG_OK;
}

int tsg_ruleset_k1_literal(const tsg_ruleset* rs, uint32_t i, uint8_t* buf, uint32_t cap,
                           uint32_t* len, uint32_t* event) {
  if (!rs || (!buf && cap)) return fail(TSG_ERR_ARG, "bad argument");
  const Plan& p = *rs->plan;
  if (i >= p.k1_lits.size()) return fail(TSG_ERR_ARG, "no such K1 literal");
  const std::string& s = p.k1_lits[i];
  if (buf) std::memcpy(buf, s.data(), std::min<size_t>(cap, s.size()));
  if (len) *len = (uint32_t)s.size();
  if (event) *event = p.lit_event[i];
  return TSG_OK;
}

int tsg_go_sort_perm(const uint8_t* keys, const uint64_t* key_offsets, const int64_t* secondary,
                     uint32_t n, uint32_t* perm) {
  if ((n && (!keys || !key_offsets || !perm))) return fail(TSG_ERR_ARG, "bad argument");
  try {
    go_sort_perm(keys, key_offsets, secondary, n, perm);
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return fail(TSG_ERR_NOMEM, "out of memory");
  }
}

const uint8_t* tsg_result_data(const tsg_result* r, size_t* len) {
  if (!r) {
    if (len) *len = 0;
    return nullptr;
  }
  if (len) *len = r->buf.size();
  return (const uint8_t*)r->buf.data();
}

void tsg_result_free(tsg_result* r) { delete r; }

int tsg_result_summary(const tsg_result* r, uint64_t* nfiles, uint64_t* files_with_findings,
                       uint64_t* findings) {
  if (!r) return fail(TSG_ERR_ARG, "bad argument");
  try {
    std::vector<size_t> rec;
    result_record_spans(r->buf, &rec);
    uint64_t ff = 0, nf = 0;
    for (size_t i = 0; i + 1 < rec.size(); i++) {
      uint32_t k;
      std::memcpy(&k, r->buf.data() + rec[i] + 1, 4);
      ff += k > 0;
      nf += k;
    }
    if (nfiles) *nfiles = rec.size() - 1;
    if (files_with_findings) *files_with_findings = ff;
    if (findings) *findings = nf;
    return TSG_OK;
  } catch (const std::exception& ex) {
    return fail(TSG_ERR_ARG, ex.what());
  }
}

// ---- test hooks
struct tsg_regex {
  std::shared_ptr<Regexp> re;
};

int tsg_regex_compile(const char* src, tsg_regex** out, char* err, size_t err_len) {
  if (!src || !out) return fail(TSG_ERR_ARG, "bad argument");
  std::string e;
  auto re = Regexp::Compile(src, &e);
  if (!re) {
    copy_err(e, err, err_len);
    return fail(TSG_ERR_CONFIG, e);
  }
  *out = new tsg_regex{re};
  return TSG_OK;
}

void tsg_regex_free(tsg_regex* re) { delete re; }

int tsg_regex_num_slots(const tsg_regex* re) { return re ? re->re->NumSlots() : TSG_ERR_ARG; }

int tsg_regex_match(const tsg_regex* re, const uint8_t* text, size_t len) {
  if (!re) return fail(TSG_ERR_ARG, "bad argument");
  return re->re->Match(text, len) ? 1 : 0;
}

int64_t tsg_regex_find_all(const tsg_regex* re, const uint8_t* text, size_t len, int submatch,
                           int64_t* out, size_t cap) {
  if (!re) return fail(TSG_ERR_ARG, "bad argument");
  std::vector<int64_t> v;
  re->re->FindAll(text, len, submatch != 0, &v);
  if (out) std::memcpy(out, v.data(), sizeof(int64_t) * std::min(cap, v.size()));
  return (int64_t)v.size();
}

int64_t tsg_regex_find_all_engine(const tsg_regex* re, const uint8_t* text, size_t len, int submatch,
                                  int engine, int64_t* out, size_t cap) {
  if (!re || engine < 0 || engine > 2) return fail(TSG_ERR_ARG, "bad argument");
  std::vector<int64_t> v;
  re->re->FindAll(text, len, submatch != 0, &v, 0, SIZE_MAX, engine);
  if (out) std::memcpy(out, v.data(), sizeof(int64_t) * std::min(cap, v.size()));
  return (int64_t)v.size();
}

int64_t tsg_regex_dfa_ends(const tsg_regex* re, const uint8_t* text, size_t len, uint32_t chunk,
                           int64_t* out, size_t cap) {
  if (!re || chunk == 0) return fail(TSG_ERR_ARG, "bad argument");
  DFAOptions o;
  o.max_states = 1 << 16;
  std::string e;
  auto d = build_dfa({&re->re->prog()}, o, &e);
  if (!d) return fail(TSG_ERR_INTERNAL, e);
  // one "group" with one rule, chunked exactly like the kernels
  Plan p;
  p.n_kw = 0;
  p.kw_words = 1;
  p.fb_kw0 = 0;
  p.kw_dfa = build_keyword_dfa({}, o, &e);
  p.kw_mask_events.assign(p.kw_dfa->masks.size(), 0);
  GroupPlan g;
  g.dfa = std::move(d);
  g.rules = {0};
  g.always = true;
  g.kwmask = {0};
  p.groups.push_back(std::move(g));
  uint64_t offs[2] = {0, len};
  uint64_t poffs[2] = {0, 0};
  BatchView b{text, offs, 1, "", poffs};
  KernelOutput ko;
  emulate_kernels(p, b, chunk, 1u << 30, &ko);
  std::vector<int64_t> ends;
  for (const auto& c : ko.cand) ends.push_back(c.end);
  std::sort(ends.begin(), ends.end());
  ends.erase(std::unique(ends.begin(), ends.end()), ends.end());
  if (out) std::memcpy(out, ends.data(), sizeof(int64_t) * std::min(cap, ends.size()));
  return (int64_t)ends.size();
}

}  // extern "C"
