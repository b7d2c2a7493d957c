// Concurrency stress of the C ABI for sanitizer builds (ThreadSanitizer / AddressSanitizer
// of the host C++, tests/test_sanitizers.py).  Everything runs on emulated contexts
// (TSG_CTX_EMULATE: the kernels' algorithm on the CPU over the real slots, lanes, tickets,
// queue and multi-context dispatcher), so no GPU is needed.  Each scenario's results must be
// byte-identical to the exact CPU path's:
//   1. tsg_scan_batch from 16 threads on one context
//   2. tsg_batch_upload + tsg_slot_submit + tsg_batch_collect(ticket) from 16 threads
//   3. tsg_queue_scan: 16 threads, one file per call (analyzer.go:419-443)
//   4. tsg_multi_scan_batch over 3 contexts from 4 threads (image.go:210-234)
//
// usage: stress RULES CORPUS_DIR    (files written by tests/test_sanitizers.py)
//   RULES: one rule per line, fields separated by \x1f: id, category, title, severity,
//          regex, keywords (\x1e-separated), secret group name; then "ALLOW" lines
//          (id, description, regex, path; "-" = absent)
//   CORPUS_DIR: data.bin, offsets.bin (u64), paths.bin, path_offsets.bin (u64)
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/trivy_secret.h"

namespace {

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  out.push_back(cur);
  return out;
}

std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

struct Batch {
  std::string data, paths;
  std::vector<uint64_t> off{0}, poff{0};
  uint32_t n() const { return (uint32_t)off.size() - 1; }
  void add(const char* d, uint64_t len, const char* p, uint64_t plen) {
    data.append(d, len);
    paths.append(p, plen);
    off.push_back(data.size());
    poff.push_back(paths.size());
  }
};

std::string take(tsg_result* r) {
  size_t n = 0;
  const uint8_t* p = tsg_result_data(r, &n);
  std::string s((const char*)p, n);
  tsg_result_free(r);
  return s;
}

std::atomic<int> g_fail{0};

void check(bool ok, const char* what, int i) {
  if (!ok) {
    std::fprintf(stderr, "FAIL %s (%d): %s\n", what, i, tsg_last_error());
    g_fail++;
  }
}

template <class F>
void threads(int n, F f) {
  std::vector<std::thread> th;
  for (int t = 0; t < n; t++) th.emplace_back(f, t);
  for (auto& t : th) t.join();
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: stress RULES CORPUS_DIR\n");
    return 2;
  }
  // ---- rules
  std::vector<std::vector<std::string>> rf, af;
  for (const auto& line : split(slurp(argv[1]), '\n')) {
    if (line.empty()) continue;
    auto f = split(line, '\x1f');
    if (f[0] == "ALLOW") af.push_back(std::vector<std::string>(f.begin() + 1, f.end()));
    else rf.push_back(f);
  }
  std::vector<std::vector<std::string>> kws(rf.size());
  std::vector<std::vector<const char*>> kwp(rf.size());
  std::vector<tsg_rule_desc> rules(rf.size());
  auto opt_str = [](const std::string& s) -> const char* { return s == "-" ? nullptr : s.c_str(); };
  for (size_t i = 0; i < rf.size(); i++) {
    if (!rf[i][5].empty()) kws[i] = split(rf[i][5], '\x1e');
    for (auto& k : kws[i]) kwp[i].push_back(k.c_str());
    tsg_rule_desc& d = rules[i];
    std::memset(&d, 0, sizeof d);
    d.id = rf[i][0].c_str();
    d.category = rf[i][1].c_str();
    d.title = rf[i][2].c_str();
    d.severity = rf[i][3].c_str();
    d.regex = rf[i][4].c_str();
    d.keywords = kwp[i].data();
    d.n_keywords = (uint32_t)kwp[i].size();
    d.secret_group_name = rf[i][6].c_str();
  }
  std::vector<tsg_allow_rule_desc> allow(af.size());
  for (size_t i = 0; i < af.size(); i++)
    allow[i] = tsg_allow_rule_desc{af[i][0].c_str(), af[i][1].c_str(), opt_str(af[i][2]), opt_str(af[i][3])};
  tsg_ruleset* rs = nullptr;
  char err[512];
  if (tsg_ruleset_compile(rules.data(), (uint32_t)rules.size(), allow.data(), (uint32_t)allow.size(), nullptr, 0,
                          &rs, err, sizeof err)) {
    std::fprintf(stderr, "compile: %s\n", err);
    return 2;
  }
  // ---- corpus, cut into batches of 1..N files
  const std::string dir = argv[2];
  const std::string data = slurp(dir + "/data.bin"), paths = slurp(dir + "/paths.bin");
  const std::string offb = slurp(dir + "/offsets.bin"), poffb = slurp(dir + "/path_offsets.bin");
  const uint64_t* off = (const uint64_t*)offb.data();
  const uint64_t* poff = (const uint64_t*)poffb.data();
  const uint32_t nfiles = (uint32_t)(offb.size() / 8 - 1);
  std::vector<Batch> batches;
  for (uint32_t f = 0, k = 0; f < nfiles; k++) {
    Batch b;
    const uint32_t want = 1 + (k * 7) % 23;
    for (uint32_t j = 0; j < want && f < nfiles; j++, f++)
      b.add(data.data() + off[f], off[f + 1] - off[f], paths.data() + poff[f], poff[f + 1] - poff[f]);
    batches.push_back(std::move(b));
  }
  std::vector<std::string> want(batches.size());
  for (size_t i = 0; i < batches.size(); i++) {
    const Batch& b = batches[i];
    tsg_result* r = nullptr;
    check(!tsg_scan_cpu_batch(rs, (const uint8_t*)b.data.data(), b.off.data(), b.n(), b.paths.data(), b.poff.data(), 2,
                              &r),
          "cpu batch", (int)i);
    want[i] = take(r);
  }
  std::printf("%u files, %zu batches, %zu rules\n", nfiles, batches.size(), rules.size());

  tsg_ctx_options o;
  std::memset(&o, 0, sizeof o);
  o.flags = TSG_CTX_EMULATE;
  o.chunk_bytes = 64;
  o.host_threads = 4;
  o.max_slots = 6;
  o.slot_mib = 1;
  tsg_ctx* c = nullptr;
  if (tsg_ctx_create(0, rs, &o, &c)) return 2;

  // 1. tsg_scan_batch
  threads(16, [&](int t) {
    for (size_t i = t; i < batches.size(); i += 16) {
      const Batch& b = batches[i];
      tsg_result* r = nullptr;
      if (tsg_scan_batch(c, (const uint8_t*)b.data.data(), b.off.data(), b.n(), b.paths.data(), b.poff.data(), &r)) {
        check(false, "tsg_scan_batch", (int)i);
        continue;
      }
      check(take(r) == want[i], "tsg_scan_batch result", (int)i);
    }
  });
  std::printf("scan_batch done\n");
  // 2. upload + ticketed submit / collect (two submissions per upload)
  threads(16, [&](int t) {
    for (size_t i = t; i < batches.size(); i += 16) {
      const Batch& b = batches[i];
      uint32_t sid;
      uint64_t t1, t2;
      if (tsg_batch_upload(c, (const uint8_t*)b.data.data(), b.off.data(), b.n(), b.paths.data(), b.poff.data(),
                           &sid) ||
          tsg_slot_submit(c, sid, b.n(), &t1) || tsg_slot_submit(c, sid, b.n(), &t2) || tsg_slot_release(c, sid)) {
        check(false, "upload/submit", (int)i);
        continue;
      }
      for (uint64_t tk : {t2, t1}) {
        tsg_result* r = nullptr;
        if (tsg_batch_collect(c, tk, &r)) {
          check(false, "collect", (int)i);
          continue;
        }
        check(take(r) == want[i], "ticket result", (int)i);
      }
    }
  });
  check(tsg_batch_pending(c) == 0, "nothing pending", 0);
  std::printf("tickets done\n");
  // 3. queue, one file per call
  tsg_queue* q = nullptr;
  if (tsg_queue_create(c, 300, &q)) return 2;
  threads(16, [&](int t) {
    for (uint32_t f = t; f < nfiles; f += 16) {
      tsg_result *r = nullptr, *e = nullptr;
      const char* p = paths.data() + poff[f];
      const size_t pl = poff[f + 1] - poff[f];
      const uint8_t* d = (const uint8_t*)data.data() + off[f];
      const size_t dl = off[f + 1] - off[f];
      if (tsg_queue_scan(q, p, pl, d, dl, &r) || tsg_scan_cpu(rs, p, pl, d, dl, &e)) {
        check(false, "queue", (int)f);
        continue;
      }
      check(take(r) == take(e), "queue result", (int)f);
    }
  });
  tsg_queue_destroy(q);
  tsg_ctx_destroy(c);
  std::printf("queue done\n");
  // 4. multi-context dispatcher
  const int devs[3] = {0, 1, 2};
  tsg_multi* m = nullptr;
  if (tsg_multi_create(devs, 3, rs, &o, &m)) return 2;
  threads(4, [&](int t) {
    for (size_t i = t; i < batches.size(); i += 4) {
      const Batch& b = batches[i];
      tsg_result* r = nullptr;
      if (tsg_multi_scan_batch(m, (const uint8_t*)b.data.data(), b.off.data(), b.n(), b.paths.data(), b.poff.data(),
                               &r)) {
        check(false, "multi", (int)i);
        continue;
      }
      check(take(r) == want[i], "multi result", (int)i);
    }
  });
  tsg_multi_destroy(m);
  std::printf("multi done\n");
  // 5. pipelined one-call layer / tree scans (1 MiB pieces) from 8 threads on one context,
  // each == the exact CPU path over the pageable pack of the same input
  {
    const std::string tar = slurp(dir + "/layer.tar");
    const std::string tree = dir + "/tree";
    std::string want_layer, want_tree;
    for (int which = 0; which < 2; which++) {
      tsg_layer* L = nullptr;
      const int rc = which == 0 ? tsg_layer_pack(rs, (const uint8_t*)tar.data(), tar.size(), nullptr, 0, nullptr, 0, "", &L)
                                : tsg_fs_pack(rs, tree.c_str(), nullptr, 0, nullptr, 0, "", &L);
      if (rc) return 2;
      tsg_layer_view v;
      tsg_layer_get(L, &v);
      tsg_result* r = nullptr;
      check(!tsg_scan_cpu_batch(rs, v.data, v.offsets, v.nfiles, (const char*)v.paths, v.path_offsets, 2, &r),
            "pack cpu", which);
      (which == 0 ? want_layer : want_tree) = take(r);
      tsg_layer_free(L);
    }
    tsg_ctx* c2 = nullptr;
    if (tsg_ctx_create(0, rs, &o, &c2)) return 2;
    threads(8, [&](int t) {
      for (int k = 0; k < 3; k++) {
        tsg_layer* L = nullptr;
        tsg_result* r = nullptr;
        const bool lay = (t + k) % 2 == 0;
        const int rc = lay ? tsg_layer_scan(c2, (const uint8_t*)tar.data(), tar.size(), nullptr, 0, nullptr, 0, "", &L, &r)
                           : tsg_fs_scan(c2, tree.c_str(), nullptr, 0, nullptr, 0, "", &L, &r);
        if (rc) {
          check(false, "pipelined scan", t);
          continue;
        }
        check(take(r) == (lay ? want_layer : want_tree), "pipelined scan result", t);
        tsg_layer_free(L);
      }
    });
    check(tsg_batch_pending(c2) == 0, "nothing pending after pipelined scans", 0);
    tsg_ctx_destroy(c2);
  }
  std::printf("pipelined scans done\n");
  tsg_ruleset_destroy(rs);
  std::printf(g_fail ? "FAILED %d\n" : "OK\n", g_fail.load());
  return g_fail ? 1 : 0;
}
