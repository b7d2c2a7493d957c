// Byte-level DFAs for the GPU scan kernels and the host path gates.
//
// Built from the Go programs of goregex.hpp (one or many regexes at once; each
// regex gets an accept id).  Semantics: for every position p of a text, the DFA
// reports the set of regexes that have a match ENDING at p (any start) -- the
// "candidate end offsets" the host then resolves exactly.  It is exact on ASCII
// text; on non-ASCII text it is a superset (a rune class containing U+FFFD also
// accepts any single byte >= 0x80, and multi-byte runes are taken as their exact
// UTF-8 encodings), so it never misses a Go match.
//
// Empty-width assertions (^ $ \A \z \b \B, (?m) line anchors) are evaluated when
// the NEXT byte is known: the closure is taken at transition time from the
// previous-byte context stored in the state and the byte being consumed, so an
// accept is attached to a transition ("a match ends just before this byte") or to
// end-of-text (eot_acc).
//
// Two modes share one state space:
//   inject   : a fresh thread is started at every position (unanchored search)
//   noinject : no new threads; used after a chunk's end so a GPU lane can follow
//              the matches that STARTED inside its chunk to their end, exactly,
//              without any state from the neighbouring lanes.  A noinject state
//              with no live thread is `dead`.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "goregex.hpp"

namespace tsg {

enum Ctx : uint8_t { kCtxBOT = 0, kCtxNL = 1, kCtxWord = 2, kCtxOther = 3 };

struct DFA {
  int nregex = 0;
  int nstates = 0;
  int nclasses = 0;
  int mask_words = 1;               // 64-bit words per accept mask
  uint8_t cls[256] = {0};           // byte -> class
  std::vector<uint32_t> next;       // [nstates * nclasses] next state
  std::vector<uint32_t> acc;        // [nstates * nclasses] accept-mask index (0 = none)
  std::vector<uint32_t> eot_acc;    // [nstates] accept-mask index at end of text
  std::vector<std::vector<uint64_t>> masks;  // masks[0] = empty
  uint32_t start[4] = {0, 0, 0, 0};  // inject-mode start state per previous-byte context
  std::vector<uint32_t> to_noinject;  // [nstates] same threads, noinject mode
  std::vector<uint8_t> dead;         // [nstates] noinject and no live thread
  // [nstates] noinject states from which no dead state is reachable: their threads never all
  // die, so a tail entering one runs to the end of the file (e.g. after begin(?s).*end)
  std::vector<uint8_t> immortal;
  std::vector<uint8_t> noinject;     // [nstates] mode bit
  int64_t max_len = -1;              // longest match in bytes (-1 = unbounded)
  uint32_t anchored = 0;             // DFAOptions::anchored: noinject state of the start node
  // host fast path (reverse DFAs): per transition the next state's row (state * nclasses)
  // | 1 << 31 if the transition accepts | 1 << 30 if the next state is dead; see pack()
  std::vector<uint32_t> packed;
  void pack();

  // Host helper: accept mask (words) of regexes matching somewhere in b (MatchString).
  void match_any(const uint8_t* b, size_t n, std::vector<uint64_t>* out) const;
  static Ctx ctx_of(uint8_t c, const DFA& d);
  bool need_word = false, need_nl = false, need_bot = false;
};

// merges byte classes whose columns are equal in every state (build_dfa does)
void merge_equal_classes(DFA* d);
// fills DFA::immortal (build_dfa does; for DFAs assembled by hand)
void mark_immortal(DFA* d);

struct DFAOptions {
  int max_states = 8192;
  // build the noinject twin states (K2); K1 keywords are bounded and use an overlap instead
  bool with_noinject = true;
  // also build DFA::anchored (one thread at the NFA start, no injection)
  bool anchored = false;
};

// Build a DFA over `progs` (accept id = index).  Returns nullptr if the state
// cap is exceeded.
std::unique_ptr<DFA> build_dfa(const std::vector<const Prog*>& progs, const DFAOptions& opt,
                               std::string* err);

// Reverse DFA of a program for the host resolver: run from a candidate end e backwards
// (reverse_match_start) it finds the leftmost s such that [s, e) may match.  Empty-width
// assertions are dropped (a superset), so "no such s" proves no match ends at e.
std::unique_ptr<DFA> build_reverse_dfa(const Prog& prog, const DFAOptions& opt, std::string* err);
// -1: no match of the program ends at e; else the leftmost possible start.
int64_t reverse_match_start(const DFA& rev, const uint8_t* b, int64_t e);

// Longest match of a program in bytes (-1 = unbounded), over the byte-level NFA.
int64_t max_match_len(const Prog& prog);

// Literal keyword set, matched case-insensitively on ASCII letters (the GPU half of
// Rule.MatchKeywords, scanner.go:164-176).  Every literal is folded, the case-sensitive
// anchor literals of K2's events too (an event may only fire more often than the match it
// anchors, never less), so 'A' and 'a' share one byte class: 42 classes instead of 68 for
// the builtin rules, and the automaton fits 16-bit byte offsets (kernels.hip K1).
// A literal equal to never_literal() is a slot that matches nothing: it keeps its id (a
// keyword left out of K1, which K1X or the host checks) without adding to the automaton.
std::unique_ptr<DFA> build_keyword_dfa(const std::vector<std::string>& lower_keywords,
                                       const DFAOptions& opt, std::string* err);
inline const std::string& never_literal() {
  static const std::string s("\0\xff\0never", 8);
  return s;
}

}  // namespace tsg
