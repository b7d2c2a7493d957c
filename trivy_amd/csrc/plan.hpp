// Compiled plan for the GPU pipeline of one rule set, and the host resolver.
//
//   K1  keyword automaton  : every distinct lowercased ASCII keyword of every rule
//                            (Rule.MatchKeywords, scanner.go:164-176) + two pseudo
//                            keywords for the only non-ASCII runes whose simple
//                            lowercase is ASCII (U+0130 -> 'i', U+212A -> 'k'); a file
//                            containing them gets its keyword gate checked exactly.
//   K2  rule-group DFAs    : the rules' regexes packed into groups (one DFA each,
//                            accept bit per rule); a group is scanned only over the
//                            files whose keyword bits gate at least one of its rules.
//   resolver (host)        : candidate end offsets -> exact windows -> scan_file.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "dfa.hpp"
#include "scanner.hpp"

namespace tsg {

enum KwMode : uint8_t { kKwAlways = 0, kKwBits = 1, kKwUnknown = 2 };

// Chunk events (K1 output, one u32 per chunk of the batch).  A rule group is scanned by
// K2 only over the chunks of its gated files that lie within `back` chunks before a
// chunk carrying one of its event bits (see Plan::rule_event).
constexpr uint32_t kEvRunU = 1u;        // run of >= run_k[0] bytes of class U
constexpr uint32_t kEvRunD = 2u;        // run of >= run_k[1] bytes of class D
constexpr int kEvLit0 = 2;              // bits 2..30: anchor literal classes
constexpr int kEvLitBits = 29;
constexpr uint32_t kEvAlways = 1u << 31;  // implicit in every chunk

struct GroupPlan {
  std::unique_ptr<DFA> dfa;
  std::vector<uint32_t> rules;   // group-local accept id -> global rule index
  std::vector<uint32_t> kwmask;  // keyword ids gating this group [kw_words]
  bool always = false;           // some member rule is not keyword-gated on the GPU
  uint32_t events = kEvAlways;   // OR of the member rules' event bits
  int64_t evdist = 0;            // max over members of Plan::rule_evdist
};

struct Plan {
  // K1: Aho-Corasick automaton over literal ids [0, n_kw) keywords (incl. the 3 fallback
  // pseudo keywords at fb_kw0..), [n_kw, n_lit) anchor literals that are not keywords.
  // Its accepts are state-based; kw_mask_events[m] = event bits of accept mask m.
  std::unique_ptr<DFA> kw_dfa;
  int n_kw = 0;        // keyword ids incl. the 3 fallback pseudo keywords at the end
  int n_lit = 0;
  int kw_words = 1;    // 32-bit words per file
  int fb_kw0 = 0;      // first fallback pseudo keyword id
  std::vector<uint32_t> kw_mask_events;
  std::vector<uint32_t> lit_event;     // [n_lit] event bits of each literal
  std::vector<std::string> k1_lits;    // [n_lit] the automaton's literals (ASCII case folded
                                       // when matched); a keyword left out is
                                       // never_literal() (dfa.hpp: matches nothing)
  std::vector<uint16_t> kw_len;        // [n_kw] byte length of each keyword literal
  // K1X: literals of >= 4 bytes that K1's LDS-resident automaton has no room for (large
  // user rule sets) -- keywords, and anchor literals with their event bits -- found by a
  // hashed 4-gram prefilter and exact verification (k1x_kernel).  Same semantics as
  // K1's: ASCII case folded, one stream, a keyword counts only inside one file.
  std::vector<std::string> x_lits;     // ASCII-lowercased literal bytes
  std::vector<int32_t> x_kw;           // keyword id, or -1 (anchor only)
  std::vector<uint32_t> x_event;       // event bits (0: keyword only)
  int x_step = 1;                      // K1X samples a 4-byte window every x_step bytes
  std::vector<uint8_t> x_j0;           // K1X windows of literal i: offsets x_j0[i] .. + x_step - 1
  // run classes for kEvRunU / kEvRunD: byte -> membership bit 0 (U) / 1 (D)
  uint8_t run_cls[256] = {0};
  int run_k[2] = {32, 12};
  int warm = 32;       // K1 warm-up bytes before a chunk (>= longest literal - 1, >= run_k - 1)
  // per rule: event bits (kEvAlways = none) and the largest distance in bytes from the
  // start of a match of the rule's GPU program to the event byte inside it; the
  // program keeps atoms [rule_first_atom, ...) of the regex
  std::vector<uint32_t> rule_event;
  std::vector<int64_t> rule_evdist;
  std::vector<int> rule_first_atom;
  std::vector<std::string> rule_anchor;  // description, for plan reports
  std::vector<uint8_t> rule_kw_mode;            // per rule
  std::vector<std::vector<uint32_t>> rule_kws;  // per rule: keyword ids
  std::vector<GroupPlan> groups;
  std::vector<int> rule_group;       // per rule: group index, -1 = no GPU DFA
  std::vector<uint8_t> rule_hostonly;  // regex without a GPU DFA (host scans gated files)
  std::vector<int64_t> rule_maxlen;  // longest EXACT match in bytes, -1 unbounded
  std::vector<int> rule_relax;       // relaxation used for the GPU program (-1 exact)
  std::vector<int> rule_atoms;       // GPU program = prefix of this many atoms (-1 = all)
  // a GPU end offset e says "a match may START in [e - winback, e]" (-1: anywhere before e)
  std::vector<int64_t> rule_winback;
  std::vector<Prog> rule_prog;       // the program the rule's GPU DFA was built from
  // reverse DFA of the exact program (null: state cap): bounds and filters the windows
  std::vector<std::unique_ptr<DFA>> rule_rev;
  // unbounded rules with a relaxed GPU program: a relaxed forward DFA that also accepts
  // U+017F / U+212A where (?i) folds s / k (null: state cap or not needed).  Run on the
  // host over a file holding those runes, it gives candidate ends instead of a whole-file
  // FindAll.
  std::vector<std::unique_ptr<DFA>> rule_fold_dfa;
  // The unbounded rules' fold programs (rule_fold_dfa's, or the GPU program of an unrelaxed
  // rule, which keeps U+017F / U+212A) in ONE forward DFA, accept id k = fold_rules[k]: one
  // pass over a file with folding runes gives every such rule's candidate ends (null: state
  // cap; the per-rule DFAs are used)
  std::unique_ptr<DFA> fold_all_dfa;
  std::vector<uint32_t> fold_rules;
  std::unique_ptr<DFA> allow_path_dfa;  // Global.AllowPath on ASCII paths
};

struct PlanOptions {
  int max_group_states = 1024;
  int max_group_table_bytes = 48 * 1024;
  int max_rules_per_group = 64;
  int max_kw_table_bytes = 96 * 1024;  // K1 transition table must stay LDS-resident
  bool anchors = true;                 // event windows (false: scan whole gated files)
};

std::unique_ptr<Plan> build_plan(const Ruleset& rs, const PlanOptions& opt, std::string* err);

// One GPU candidate: rule `rule` has a match ending at byte `end` of file `file`, or, with
// end == kCandWhole, the rule's K2 thread ran past ext_cap: resolve the rule over the whole
// file (only that rule: the other rules of the file keep their windows).
constexpr uint32_t kCandWhole = 0xFFFFFFFFu;
// Candidate.rule with this bit: a K2 transition record {group g = bits 16-30, table index ix
// = bits 0-15 (state * max(2, nclasses) + class of the group's DFA)}: the transition at
// `end` accepts, and its accept mask names the rules (expanded on the host, so the kernel
// looks up no mask per accepting byte)
constexpr uint32_t kCandTrans = 0x80000000u;
// with kCandTrans: a whole accepting 16-B word {file, kCandTrans | kCandWord | group << 16 |
// row before the byte at end, end}; the host replays it (groups then have 14 bits)
constexpr uint32_t kCandWord = 0x40000000u;
struct Candidate {
  uint32_t file;
  uint32_t rule;
  uint32_t end;
};

// What the kernels hand back for one batch, wherever it lives (pinned host buffers of the
// device pipeline, or the vectors of a CPU emulation).
struct KernelOutputView {
  const uint32_t* kw = nullptr;     // [nfiles * kw_words]
  const Candidate* cand = nullptr;
  size_t ncand = 0;
  const uint8_t* overflow = nullptr;    // [nfiles] or null: bit 0 = resolve the whole file exactly
  // overflow bit 1 = folding runes present (their keyword bits set), bit 2 = the file's
  // keyword row is written, and `kw` holds only those rows (files with candidates or a flag
  // set: the device's outputs kernel); otherwise `kw` is whole and folding runes are read
  // from it
  bool sparse_kw = false;
  const uint8_t* kw_unknown = nullptr;  // [n_kw] or null: keyword bits K1 no longer reports
  const uint8_t* path_ok = nullptr;     // [nfiles] or null: Global.AllowPath from the device
  // [groups] or null: groups K2 did not scan in this batch (item capacity); their rules are
  // resolved like rules without a GPU program
  const uint8_t* group_skipped = nullptr;
};

// Everything the kernels hand back for one batch.
struct KernelOutput {
  std::vector<uint32_t> kw;        // [nfiles * kw_words]
  std::vector<Candidate> cand;
  std::vector<uint8_t> overflow;   // [nfiles] 1 = resolve the whole file exactly
  // [n_kw] (or empty): keyword bits K1 no longer reports (a clear bit proves nothing)
  std::vector<uint8_t> kw_unknown;
  // [nfiles] (or empty): Global.AllowPath of each path computed on the device:
  // 0 / 1, or 2 = non-ASCII path, decided on the host
  std::vector<uint8_t> path_ok;
  KernelOutputView view() const {
    KernelOutputView v;
    v.kw = kw.data();
    v.cand = cand.data();
    v.ncand = cand.size();
    v.overflow = overflow.empty() ? nullptr : overflow.data();
    v.kw_unknown = kw_unknown.empty() ? nullptr : kw_unknown.data();
    v.path_ok = path_ok.empty() ? nullptr : path_ok.data();
    return v;
  }
};

struct BatchView {
  const uint8_t* data;
  const uint64_t* offsets;  // [nfiles + 1]
  uint32_t nfiles;
  const char* paths;
  const uint64_t* path_offsets;  // [nfiles + 1]
};

// Start offsets of the folding runes in s: which = 1 U+0130, 2 U+212A, 4 U+017F (ORed).
void fold_rune_positions(const uint8_t* s, int64_t n, uint32_t which, std::vector<int64_t>* out);

// Host resolution: exact findings for every file of the batch.
void resolve_batch(const Ruleset& rs, const Plan& plan, const BatchView& b,
                   const KernelOutputView& ko, int nthreads, BatchResult* out);

// Exact CPU path for a whole batch (no GPU).
void scan_batch_cpu(const Ruleset& rs, const BatchView& b, int nthreads,
                    std::vector<FileResult>* out);

// CPU emulation of the two kernels' algorithm (same chunking, same tables);
// used by the CPU tests and as the reference for the HIP kernels.
// group_item_bytes (optional, [groups]): bytes of the K2 items of each group.
void emulate_kernels(const Plan& plan, const BatchView& b, uint32_t chunk, uint32_t ext_cap,
                     KernelOutput* ko, std::vector<uint64_t>* group_item_bytes = nullptr);

// K1 semantics shared by the HIP kernel and the emulation: keyword bits of every file
// [nfiles * kw_words] and event bits of every chunk c = bytes [c*chunk, (c+1)*chunk).
// The automaton and the run counters run over the batch as ONE byte stream (they are not
// reset at file boundaries), so a chunk's event bits are a superset of its files' own.
// Keyword bits stay exact: an occurrence counts for file f only when the whole keyword
// lies inside f (its length is checked against the bytes of f before its last byte).
void k1_reference(const Plan& plan, const BatchView& b, uint32_t chunk,
                  std::vector<uint32_t>* kw, std::vector<uint32_t>* ev);
// The K1X part of k1_reference (Plan::x_lits), ORed into kw / ev.
void k1x_reference(const Plan& plan, const BatchView& b, uint32_t chunk,
                   std::vector<uint32_t>* kw, std::vector<uint32_t>* ev);

// K1X: the 4-byte little-endian prefix word of a (lowercased) literal or window
inline uint32_t x_prefix4(const uint8_t* b) {
  return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
}
// K1X prefilter: a blocked Bloom filter of 2^kXDwordBits dwords (128 KiB of LDS).  A
// window's hash picks one dword and two bits in it; the window passes when both are set.
constexpr int kXDwordBits = 15;
constexpr uint32_t kXDwords = 1u << kXDwordBits;
// Keys are folded windows: bit 5 of every byte set, so an ASCII letter and its capital agree
// (one OR per dword on the device instead of a lowercase).
constexpr uint32_t kXFold = 0x20202020u;
inline uint32_t x_fold(uint32_t w) { return w | kXFold; }
inline uint32_t x_hash(uint32_t w) { return w * 2654435761u; }
inline uint32_t x_dword(uint32_t h) { return h >> (32 - kXDwordBits); }
inline uint32_t x_bits(uint32_t h) { return 1u << ((h >> 12) & 31) | 1u << ((h >> 7) & 31); }

// Chunks of file f that K2 scans for group g (given the K1 output): chunk c of the file
// is an item iff the group is gated for f and a chunk in [c, c + back] (inside f)
// carries one of the group's event bits.  back = ceil(evdist / chunk).
inline uint32_t group_back(const GroupPlan& g, uint32_t chunk) {
  return (uint32_t)((g.evdist + chunk - 1) / chunk);
}

}  // namespace tsg
