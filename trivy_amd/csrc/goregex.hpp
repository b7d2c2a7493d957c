// Go 1.19 regexp semantics for the host side of the secret engine.
//
// The reference compiles every rule with Go's `regexp.Compile` (Perl flags) —
// trivy pkg/fanal/secret/scanner.go:64-81 — and matches with
// `FindAllIndex` / `FindAllSubmatchIndex` / `MatchString` (scanner.go:106,124,161,197,206,254).
// This is a from-scratch C++ implementation of that dialect:
//   * parser   : regexp/syntax parse rules (flags i m s U with group scoping, (?P<name>),
//                Perl/POSIX/Unicode classes, folding via SimpleFold orbits, {n,m} <= 1000)
//   * compiler : Go-shaped program (Alt/Cap/Empty/Match/Nop/Rune) incl. the x{n,m}
//                expansion and the nullable-star rule of regexp/syntax
//   * matcher  : Pike VM with leftmost-first priority, UTF-8 rune stepping where an
//                invalid byte is one U+FFFD rune of width 1, and Go's FindAll
//                empty-match iteration.
// It is the exact resolver the GPU candidates are confirmed with; the GPU kernels run
// DFAs built from the same program (dfa.hpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace tsg {

constexpr int32_t kMaxRune = 0x10FFFF;
constexpr int32_t kRuneError = 0xFFFD;
constexpr int32_t kEOT = -1;
// Pseudo rune used only in relaxed (GPU) programs: "any single byte >= 0x80".
constexpr int32_t kHighByteRune = 0x110000;

using Ranges = std::vector<std::pair<int32_t, int32_t>>;  // sorted, non-overlapping

// Shape of one element of a regex's flattened top-level concatenation, for choosing
// the GPU anchor of a rule (plan.cpp).  Runes U+017F / U+212A (the only non-ASCII
// members (?i) adds to ASCII letters) are ignored: files containing them are resolved
// whole on the host.
struct AtomInfo {
  int64_t min_bytes = 0, max_bytes = 0;  // bytes one occurrence consumes; max -1 = unbounded
  bool ascii_only = true;                // consumes only ASCII bytes
  uint64_t set[2] = {0, 0};              // ASCII bytes it can consume
  int lit = -1;                          // a single char, ASCII-case-folded: its lowercase
  bool lit_fold = false;                 // lit matched case-insensitively
};

// utf8.DecodeRune on b[pos:n]; returns width 0 at end of text.
int32_t decode_rune(const uint8_t* b, size_t n, size_t pos, int* width);

// unicode.SimpleFold orbit of r (sorted, includes r).
void fold_orbit(int32_t r, std::vector<int32_t>* out);
// unicode.ToLower (simple mapping)
int32_t simple_lower(int32_t r);
// bytes.ToLower (Go 1.19): ASCII fast path, else per-rune mapping with invalid -> U+FFFD
void go_to_lower(const uint8_t* b, size_t n, std::string* out);

enum EmptyOp : uint32_t {
  kBeginLine = 1, kEndLine = 2, kBeginText = 4, kEndText = 8, kWordBoundary = 16,
  kNoWordBoundary = 32,
};

inline bool is_word_byte(int32_t c) {
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
}
// lazyFlag.match(op) with r1 = rune before, r2 = rune after (kEOT at the ends)
bool empty_ok(uint32_t op, int32_t r1, int32_t r2);

enum class Op : uint8_t { Fail, Alt, Cap, Empty, Match, Nop, Rune };

struct Inst {
  Op op = Op::Fail;
  uint32_t out = 0;
  uint32_t arg = 0;  // Alt: second branch; Cap: slot; Empty: EmptyOp; Rune: index into Prog::runes
};

struct Prog {
  std::vector<Inst> inst;
  std::vector<Ranges> runes;
  uint32_t start = 0;
  int nslots = 2;  // 2 * (number of capture groups + 1)
  // [runes.size() * 2]: ASCII members of each rune set as a 128-bit map (matcher fast
  // path; filled by Regexp::Compile, empty for derived programs)
  std::vector<uint64_t> ascii;
  // regexp/syntax Prog.Prefix restricted to ASCII: the literal every match starts with (the
  // leading single-rune, case-sensitive instructions after Nop / Cap), or empty.  The
  // matchers jump between its occurrences while no thread is alive (regexp/exec.go
  // machine.match, backtrack.go), so a whole-file search costs a memmem where it can.
  std::string prefix;
};

class Regexp {
 public:
  Regexp();
  ~Regexp();
  // regexp.Compile; returns nullptr and sets *err on a syntax error.
  static std::shared_ptr<Regexp> Compile(const std::string& src, std::string* err);

  // A superset program for the GPU filter: every counted repetition x{n,m} with
  // m > k (or unbounded) becomes x{min(n,k),}.  Each match of the exact program is a
  // match of this one with the same start and end, so its DFA reports a superset of
  // the exact end offsets while avoiding the state blow-up of re-entrant counters
  // such as (?i)lob[a-z0-9_ .\-,]{0,25}.
  // natoms >= 0 keeps only that many leading elements of the (flattened) top-level
  // concatenation: each match of the regex then has a prefix match with the same start.
  // Non-ASCII members of rune sets become "one or more bytes >= 0x80" (kHighByteRune).
  // first_atom > 0 drops that many leading elements instead (a suffix program: every
  // match of the regex ends where a match of the suffix ends).
  Prog RelaxedProg(int k, int natoms = -1, int first_atom = 0, bool fold_high = false) const;
  int NumAtoms() const;
  std::vector<AtomInfo> Atoms() const;

  const std::string& source() const { return src_; }
  const std::vector<std::string>& SubexpNames() const { return names_; }
  int NumSlots() const { return prog_.nslots; }
  const Prog& prog() const { return prog_; }

  // regexp.MatchString / Match (unanchored search)
  bool Match(const uint8_t* b, size_t n) const;

  // regexp.FindAllSubmatchIndex(b, -1) (submatch=true, nslots per match) or
  // FindAllIndex (submatch=false, 2 per match), appended flattened to *out.
  //
  // Window extension used for exact resolution of GPU candidates: the FindAll
  // iteration starts at `lo` (with the whole text as context for assertions) and only
  // matches whose start is <= start_hi are produced.  With lo = 0 and
  // start_hi = n this is exactly Go's FindAll.
  // engine (tests): 0 auto, 1 Pike VM only, 2 bit-state backtracker where it fits
  void FindAll(const uint8_t* b, size_t n, bool submatch, std::vector<int64_t>* out,
               size_t lo = 0, size_t start_hi = SIZE_MAX, int engine = 0) const;

  // Go's FindAll iteration restricted to match STARTS inside the given windows
  // [lo, hi] (sorted, disjoint, lo on a rune boundary).  The iteration position and the
  // previous match end carry across windows, so the result equals FindAll whenever
  // every match start lies in some window -- matches may end beyond their window.
  void FindAllWindows(const uint8_t* b, size_t n, bool submatch,
                      const std::vector<std::pair<int64_t, int64_t>>& iv,
                      std::vector<int64_t>* out) const;

 private:
  struct Ast;
  std::string src_;
  std::vector<std::string> names_;
  Prog prog_;
  std::shared_ptr<Ast> ast_;
};

}  // namespace tsg
