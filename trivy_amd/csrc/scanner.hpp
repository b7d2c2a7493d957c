// Host side of the secret engine: the rule set and the exact per-file Scan.
//
// Mirrors trivy pkg/fanal/secret/scanner.go:
//   Rule / AllowRule / ExcludeBlock / Global      scanner.go:23-94, 186-225
//   Scanner.Scan                                  scanner.go:341-416
//   FindLocations / FindSubmatchLocations         scanner.go:96-141
//   AllowLocation, getMatchSubgroupsLocations     scanner.go:143-158
//   Blocks (lazy exclude-block search)            scanner.go:227-265
//   censorLocation / toFinding / findLocation     scanner.go:418-502
//   sort.Slice(findings, RuleID, Match)           scanner.go:405-410 (Go 1.19 pdqsort_func)
// The GPU kernels only decide WHERE this exact code has to look (per-file keyword
// bits and per-rule candidate end offsets); everything that reaches the output is
// computed here with Go semantics.
#pragma once
#include <functional>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "goregex.hpp"

namespace tsg {

struct AllowRuleC {
  std::string id, description;
  std::shared_ptr<Regexp> regex, path;
};

struct RuleC {
  std::string id, category, title, severity;
  std::shared_ptr<Regexp> regex;  // may be null
  std::vector<std::string> keywords;
  std::shared_ptr<Regexp> path;
  std::vector<AllowRuleC> allow;
  std::vector<std::shared_ptr<Regexp>> exclude;
  std::string secret_group_name;
  // derived
  std::vector<std::string> kw_lower;  // strings.ToLower(kw)
  bool kw_ascii = true;               // every kw_lower is ASCII
  std::vector<int> group_idx;         // i where SubexpNames()[i] == secret_group_name
};

struct Ruleset {
  std::vector<RuleC> rules;
  std::vector<AllowRuleC> allow;
  std::vector<std::shared_ptr<Regexp>> exclude;

  bool AllowPath(const std::string& path) const;       // Global.AllowPath
  bool Allow(const uint8_t* m, size_t n) const;        // Global.Allow
};

struct Line {
  int32_t number;
  uint8_t flags;  // 1 IsCause, 2 FirstCause, 4 LastCause
  std::string content;
};

struct Finding {
  uint32_t rule;
  int32_t start_line, end_line;
  std::string match;
  std::vector<Line> lines;
};

enum FileStatus : uint8_t { kNoFindings = 0, kPathAllowed = 1, kHasFindings = 2 };

struct FileResult {
  uint8_t status = kNoFindings;
  std::vector<Finding> findings;
};

// Results of a batch resolved from kernel output: most files need no exact scan, so only
// those that did hold a FileResult.
struct BatchResult {
  std::vector<uint8_t> status;   // [nfiles] FileStatus
  std::vector<uint32_t> slot;    // [nfiles] index into res, or UINT32_MAX
  std::vector<FileResult> res;
};

// Where the exact matcher must look for one rule in one file.
struct RuleWindows {
  bool whole = false;                               // run FindAll over the whole file
  std::vector<std::pair<int64_t, int64_t>> iv;      // [lo, start_hi] intervals, sorted, disjoint
};

// Per-file gating decided by the GPU (null = CPU path: decide everything exactly).
struct FileGate {
  // kw_state[r]: 0 keyword gate known false, 1 known true, 2 unknown (check exactly)
  const uint8_t* kw_state = nullptr;
  // windows[r] == nullptr -> the rule has no candidate in this file (regex cannot match)
  const RuleWindows* const* windows = nullptr;
  // Global.AllowPath(path) already evaluated by the caller: 0 no, 1 yes, -1 not known
  int8_t path_allowed = -1;
  // the file holds neither U+0130 nor U+212A: an ASCII keyword is in bytes.ToLower(content)
  // iff it is in content under ASCII case folding (contains_fold_ascii)
  bool ascii_fold_exact = false;
};

bool contains_fold_ascii(const uint8_t* s, size_t n, const std::string& kw);
// the same for any content: U+0130 / U+212A count as 'i' / 'k' (bytes.ToLower)
bool contains_fold_runes(const uint8_t* s, size_t n, const std::string& kw);

// Exact Scan of one file (scanner.go:341-416).
void scan_file(const Ruleset& rs, const std::string& path, const uint8_t* content, size_t n,
               const FileGate* gate, FileResult* out);

// Rule.MatchKeywords (scanner.go:164-176) with the lowercased content computed once.
bool match_keywords(const RuleC& r, const std::string& lowered);

// Serialization of results (format documented in include/trivy_secret.h).
void serialize_batch(const BatchResult& br, std::string* out, int nthreads = 1);
// byte offset of each per-file record of a serialized result, and its end: file i is
// [rec[i], rec[i+1]) (throws on a malformed buffer)
void result_record_spans(const std::string& b, std::vector<size_t>* rec);

// f(i) for i in [0, n) on the process-wide worker pool (plan.cpp), `grain` indices a claim
void pool_for(size_t n, int nthreads, const std::function<void(size_t)>& f, size_t grain);
// the process-wide resolver pool holds at least this many worker threads
void pool_reserve(int threads);
// Global.AllowPath (scanner.go:55-57): the plan's path DFA for ASCII paths, else the exact VM
struct Plan;
bool path_allowed(const Ruleset& rs, const Plan* plan, const char* p, size_t n);
void serialize_results(const std::vector<FileResult>& res, std::string* out);
// sort.Slice (Go 1.19 pdqsort_func) of n items by (key bytes, then secondary): the order
// as a permutation (perm[k] = original index of the k-th item)
void go_sort_perm(const uint8_t* keys, const uint64_t* key_offsets, const int64_t* secondary, uint32_t n,
                  uint32_t* perm);

}  // namespace tsg
