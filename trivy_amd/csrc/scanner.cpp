// Exact per-file Scan (host).  See scanner.hpp for the reference mapping.
#include <emmintrin.h>
#include "scanner.hpp"

#include <algorithm>
#include <map>
#include <atomic>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <x86intrin.h>
#include <emmintrin.h>

namespace tsg {

// ------------------------------------------------------------------ allow rules
static bool allow_path(const std::vector<AllowRuleC>& rules, const std::string& path) {
  for (const auto& r : rules)  // scanner.go:195-202
    if (r.path && r.path->Match((const uint8_t*)path.data(), path.size())) return true;
  return false;
}

static bool allow_match(const std::vector<AllowRuleC>& rules, const uint8_t* m, size_t n) {
  for (const auto& r : rules)  // scanner.go:204-211
    if (r.regex && r.regex->Match(m, n)) return true;
  return false;
}

bool Ruleset::AllowPath(const std::string& path) const { return allow_path(allow, path); }
bool Ruleset::Allow(const uint8_t* m, size_t n) const { return allow_match(allow, m, n); }

bool match_keywords(const RuleC& r, const std::string& lowered) {
  if (r.kw_lower.empty()) return true;  // scanner.go:165-167
  for (const auto& kw : r.kw_lower)
    if (lowered.find(kw) != std::string::npos) return true;
  return false;
}

// bytes.Contains(bytes.ToLower(s), kw) for an ASCII lowercase keyword kw, valid when s holds
// neither U+0130 nor U+212A: those are the only runes bytes.ToLower turns into ASCII, so
// the ASCII bytes of the lowered text are exactly the ASCII bytes of s, lowercased.
bool contains_fold_ascii(const uint8_t* s, size_t n, const std::string& kw) {
  const size_t m = kw.size();
  if (m == 0) return true;
  if (m > n) return false;
  const uint8_t c0 = (uint8_t)kw[0];
  const uint8_t u0 = (c0 >= 'a' && c0 <= 'z') ? (uint8_t)(c0 - 32) : c0;
  const __m128i v0 = _mm_set1_epi8((char)c0), v1 = _mm_set1_epi8((char)u0);
  auto rest = [&](size_t i) {
    for (size_t j = 1; j < m; j++) {
      uint8_t x = s[i + j];
      if (x >= 'A' && x <= 'Z') x |= 0x20;
      if (x != (uint8_t)kw[j]) return false;
    }
    return true;
  };
  const size_t last = n - m;  // last possible start
  size_t i = 0;
  for (; i + 16 <= last + 1; i += 16) {
    const __m128i b = _mm_loadu_si128((const __m128i*)(s + i));
    uint32_t bits = (uint32_t)_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(b, v0), _mm_cmpeq_epi8(b, v1)));
    while (bits) {
      const size_t k = i + (size_t)__builtin_ctz(bits);
      bits &= bits - 1;
      if (rest(k)) return true;
    }
  }
  for (; i <= last; i++)
    if ((s[i] == c0 || s[i] == u0) && rest(i)) return true;
  return false;
}

// bytes.Contains(bytes.ToLower(s), kw) for an ASCII lowercase keyword kw, for any s.
// bytes.ToLower maps exactly two non-ASCII runes to ASCII: U+0130 (C4 B0) -> 'i' and
// U+212A (E2 84 AA) -> 'k'; every other rune, and every invalid byte (U+FFFD), lowers to
// non-ASCII bytes.  Neither C4 nor E2 is a UTF-8 continuation byte, so those byte
// sequences always decode as the runes.  A keyword then occurs in the lowered text iff
// its letters occur contiguously in s, each as itself, its upper case, or for 'i' / 'k'
// as the rune's bytes -- without lowering (and copying) the file.
bool contains_fold_runes(const uint8_t* s, size_t n, const std::string& kw) {
  const size_t m = kw.size();
  if (m == 0) return true;
  auto at = [&](size_t i, size_t j, size_t* w) -> bool {  // kw[j] at s[i..]: width in *w
    const uint8_t c = (uint8_t)kw[j];
    if (i >= n) return false;
    uint8_t x = s[i];
    if (x >= 'A' && x <= 'Z') x |= 0x20;
    if (x == c) {
      *w = 1;
      return true;
    }
    if (c == 'i' && s[i] == 0xC4 && i + 1 < n && s[i + 1] == 0xB0) {
      *w = 2;
      return true;
    }
    if (c == 'k' && s[i] == 0xE2 && i + 2 < n && s[i + 1] == 0x84 && s[i + 2] == 0xAA) {
      *w = 3;
      return true;
    }
    return false;
  };
  const uint8_t c0 = (uint8_t)kw[0];
  const uint8_t u0 = (c0 >= 'a' && c0 <= 'z') ? (uint8_t)(c0 - 32) : c0;
  const uint8_t r0 = c0 == 'i' ? 0xC4 : c0 == 'k' ? 0xE2 : c0;  // the rune's lead byte
  const __m128i v0 = _mm_set1_epi8((char)c0), v1 = _mm_set1_epi8((char)u0), v2 = _mm_set1_epi8((char)r0);
  auto try_at = [&](size_t i) {
    size_t p = i;
    for (size_t j = 0; j < m; j++) {
      size_t w;
      if (!at(p, j, &w)) return false;
      p += w;
    }
    return true;
  };
  size_t i = 0;
  for (; i + 16 <= n; i += 16) {
    const __m128i b = _mm_loadu_si128((const __m128i*)(s + i));
    uint32_t bits = (uint32_t)_mm_movemask_epi8(
        _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(b, v0), _mm_cmpeq_epi8(b, v1)), _mm_cmpeq_epi8(b, v2)));
    while (bits) {
      const size_t k = i + (size_t)__builtin_ctz(bits);
      bits &= bits - 1;
      if (try_at(k)) return true;
    }
  }
  for (; i < n; i++)
    if ((s[i] == c0 || s[i] == u0 || s[i] == r0) && try_at(i)) return true;
  return false;
}

// ------------------------------------------------------------------ Go sort.Slice
// pdqsort_func from Go 1.19 sort/zsortfunc.go, restated over a vector with `less`.
namespace gosort {

template <class T, class L>
struct Data {
  std::vector<T>& x;
  L less;
  bool Less(int i, int j) const { return less(x[i], x[j]); }
  void Swap(int i, int j) { std::swap(x[i], x[j]); }
};

template <class D>
void insertion_sort(D& d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
}

template <class D>
void sift_down(D& d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
    if (!d.Less(first + root, first + child)) return;
    d.Swap(first + root, first + child);
    root = child;
  }
}

template <class D>
void heap_sort(D& d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) {
    d.Swap(first, first + i);
    sift_down(d, lo, i, first);
  }
}

enum Hint { kUnknown, kIncreasing, kDecreasing };

inline int bits_len(uint64_t x) {
  int n = 0;
  while (x) {
    n++;
    x >>= 1;
  }
  return n;
}

template <class D>
void break_patterns(D& d, int a, int b) {
  int length = b - a;
  if (length >= 8) {
    uint64_t r = (uint64_t)length;
    uint64_t modulus = 1ull << bits_len((uint64_t)length);
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13;
      r ^= r >> 17;
      r ^= r << 5;
      int other = (int)(r & (modulus - 1));
      if (other >= length) other -= length;
      d.Swap(idx - 1 + i, a + other);
    }
  }
}

template <class D>
void order2(D& d, int& a, int& b, int* swaps) {
  if (d.Less(b, a)) {
    (*swaps)++;
    std::swap(a, b);
  }
}

template <class D>
int median(D& d, int a, int b, int c, int* swaps) {
  order2(d, a, b, swaps);
  order2(d, b, c, swaps);
  order2(d, a, b, swaps);
  return b;
}

template <class D>
int choose_pivot(D& d, int a, int b, Hint* hint) {
  const int shortest_ninther = 50, max_swaps = 4 * 3;
  int l = b - a;
  int swaps = 0;
  int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
  if (l >= 8) {
    if (l >= shortest_ninther) {
      i = median(d, i - 1, i, i + 1, &swaps);
      j = median(d, j - 1, j, j + 1, &swaps);
      k = median(d, k - 1, k, k + 1, &swaps);
    }
    j = median(d, i, j, k, &swaps);
  }
  *hint = swaps == 0 ? kIncreasing : swaps == max_swaps ? kDecreasing : kUnknown;
  return j;
}

template <class D>
void reverse_range(D& d, int a, int b) {
  for (int i = a, j = b - 1; i < j; i++, j--) d.Swap(i, j);
}

template <class D>
bool partial_insertion_sort(D& d, int a, int b) {
  const int max_steps = 5, shortest_shifting = 50;
  int i = a + 1;
  for (int j = 0; j < max_steps; j++) {
    while (i < b && !d.Less(i, i - 1)) i++;
    if (i == b) return true;
    if (b - a < shortest_shifting) return false;
    d.Swap(i, i - 1);
    if (i - a >= 2) {
      for (int k = i - 1; k >= 1; k--) {
        if (!d.Less(k, k - 1)) break;
        d.Swap(k, k - 1);
      }
    }
    if (b - i >= 2) {
      for (int k = i + 1; k < b; k++) {
        if (!d.Less(k, k - 1)) break;
        d.Swap(k, k - 1);
      }
    }
  }
  return false;
}

template <class D>
int partition_equal(D& d, int a, int b, int pivot) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  for (;;) {
    while (i <= j && !d.Less(a, i)) i++;
    while (i <= j && d.Less(a, j)) j--;
    if (i > j) break;
    d.Swap(i, j);
    i++;
    j--;
  }
  return i;
}

template <class D>
int partition(D& d, int a, int b, int pivot, bool* already) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  while (i <= j && d.Less(i, a)) i++;
  while (i <= j && !d.Less(j, a)) j--;
  if (i > j) {
    d.Swap(j, a);
    *already = true;
    return j;
  }
  d.Swap(i, j);
  i++;
  j--;
  for (;;) {
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    if (i > j) break;
    d.Swap(i, j);
    i++;
    j--;
  }
  d.Swap(j, a);
  *already = false;
  return j;
}

template <class D>
void pdqsort(D& d, int a, int b, int limit) {
  const int max_insertion = 12;
  bool was_balanced = true, was_partitioned = true;
  for (;;) {
    int length = b - a;
    if (length <= max_insertion) {
      insertion_sort(d, a, b);
      return;
    }
    if (limit == 0) {
      heap_sort(d, a, b);
      return;
    }
    if (!was_balanced) {
      break_patterns(d, a, b);
      limit--;
    }
    Hint hint;
    int pivot = choose_pivot(d, a, b, &hint);
    if (hint == kDecreasing) {
      reverse_range(d, a, b);
      pivot = (b - 1) - (pivot - a);
      hint = kIncreasing;
    }
    if (was_balanced && was_partitioned && hint == kIncreasing) {
      if (partial_insertion_sort(d, a, b)) return;
    }
    if (a > 0 && !d.Less(a - 1, pivot)) {
      a = partition_equal(d, a, b, pivot);
      continue;
    }
    bool already;
    int mid = partition(d, a, b, pivot, &already);
    was_partitioned = already;
    int left_len = mid - a, right_len = b - mid;
    int balance_threshold = length / 8;
    if (left_len < right_len) {
      was_balanced = left_len >= balance_threshold;
      pdqsort(d, a, mid, limit);
      a = mid + 1;
    } else {
      was_balanced = right_len >= balance_threshold;
      pdqsort(d, mid + 1, b, limit);
      b = mid;
    }
  }
}

template <class T, class L>
void sort_slice(std::vector<T>& x, L less) {
  Data<T, L> d{x, less};
  pdqsort(d, 0, (int)x.size(), bits_len(x.size()));
}

}  // namespace gosort

void go_sort_perm(const uint8_t* keys, const uint64_t* key_offsets, const int64_t* secondary, uint32_t n,
                  uint32_t* perm) {
  std::vector<uint32_t> x(n);
  for (uint32_t i = 0; i < n; i++) x[i] = i;
  auto key = [&](uint32_t i, size_t* len) {
    *len = key_offsets[i + 1] - key_offsets[i];
    return keys + key_offsets[i];
  };
  gosort::sort_slice(x, [&](uint32_t a, uint32_t b) {
    size_t la, lb;
    const uint8_t* ka = key(a, &la);
    const uint8_t* kb = key(b, &lb);
    const int c = std::memcmp(ka, kb, std::min(la, lb));
    if (c != 0 || la != lb) return c != 0 ? c < 0 : la < lb;  // Go string <
    return secondary ? secondary[a] < secondary[b] : false;
  });
  std::memcpy(perm, x.data(), sizeof(uint32_t) * n);
}

// ------------------------------------------------------------------ materialise
namespace {

struct Loc {
  int64_t start, end;
};

// Blocks (scanner.go:227-265): exclude-block spans, searched lazily once per file
struct Blocks {
  const uint8_t* content;
  size_t n;
  const std::vector<std::shared_ptr<Regexp>>* regexes;
  bool done = false;
  std::vector<Loc> locs;

  bool Match(const Loc& b) {
    if (!done) {
      done = true;
      std::vector<int64_t> idx;
      for (const auto& re : *regexes) {
        idx.clear();
        re->FindAll(content, n, false, &idx);
        for (size_t k = 0; k + 1 < idx.size(); k += 2) locs.push_back({idx[k], idx[k + 1]});
      }
    }
    for (const auto& l : locs)
      if (l.start <= b.start && b.end <= l.end) return true;
    return false;
  }
};

// newlines in [p, p + n): SSE2 byte compares summed in 8-bit lanes (at most 255 blocks of
// 16 bytes per lane before a _mm_sad_epu8 widening), then a byte loop for the tail
int64_t count_nl(const char* p, int64_t n) {
  int64_t c = 0, i = 0;
  const __m128i nl = _mm_set1_epi8('\n');
  const __m128i zero = _mm_setzero_si128();
  while (n - i >= 32) {
    __m128i a0 = zero, a1 = zero;
    const int64_t blocks = std::min<int64_t>((n - i) / 32, 255);
    for (int64_t k = 0; k < blocks; k++, i += 32) {
      a0 = _mm_sub_epi8(a0, _mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i)), nl));
      a1 = _mm_sub_epi8(a1, _mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i + 16)), nl));
    }
    const __m128i s = _mm_add_epi64(_mm_sad_epu8(a0, zero), _mm_sad_epu8(a1, zero));
    c += _mm_cvtsi128_si64(s) + _mm_cvtsi128_si64(_mm_unpackhi_epi64(s, s));
  }
  for (; i < n; i++) c += p[i] == '\n';
  return c;
}

// The censored buffer of scanner.go:389-392 / censorLocation (:418-426) without copying
// the file: the content plus the censored spans (sorted, merged).  A newline inside a
// span is a '*' in the censored buffer, so the line helpers skip it.
struct Censored {
  const char* b;
  int64_t n;
  std::vector<Loc> cz;

  void finish() {  // sort and merge the spans
    std::sort(cz.begin(), cz.end(), [](const Loc& x, const Loc& y) { return x.start < y.start; });
    size_t o = 0;
    for (size_t i = 0; i < cz.size(); i++) {
      if (cz[i].end <= cz[i].start) continue;
      if (o && cz[i].start <= cz[o - 1].end) cz[o - 1].end = std::max(cz[o - 1].end, cz[i].end);
      else cz[o++] = cz[i];
    }
    cz.resize(o);
  }
  // the span holding p, or nullptr
  const Loc* span(int64_t p) const {
    auto it = std::upper_bound(cz.begin(), cz.end(), p, [](int64_t v, const Loc& l) { return v < l.start; });
    if (it == cz.begin()) return nullptr;
    --it;
    return p < it->end ? &*it : nullptr;
  }
  // the first span ending after a (spans are disjoint: ends are sorted too)
  std::vector<Loc>::const_iterator first_after(int64_t a) const {
    return std::partition_point(cz.begin(), cz.end(), [a](const Loc& l) { return l.end <= a; });
  }
  // newlines of the censored buffer in [a, e)
  int64_t count(int64_t a, int64_t e) const {
    int64_t c = count_nl(b + a, e - a);
    for (auto it = first_after(a); it != cz.end() && it->start < e; ++it) {
      const int64_t s = std::max(a, it->start), t = std::min(e, it->end);
      if (s < t) c -= count_nl(b + s, t - s);
    }
    return c;
  }
  // the first newline at or after x (n if none)
  int64_t next_nl(int64_t x) const {
    while (x < n) {
      const char* p = (const char*)std::memchr(b + x, '\n', (size_t)(n - x));
      if (!p) return n;
      const int64_t q = p - b;
      const Loc* l = span(q);
      if (!l) return q;
      x = l->end;
    }
    return n;
  }
  // the last newline before x (-1 if none)
  int64_t prev_nl(int64_t x) const {
    while (x > 0) {
      const char* p = (const char*)memrchr(b, '\n', (size_t)x);
      if (!p) return -1;
      const int64_t q = p - b;
      const Loc* l = span(q);
      if (!l) return q;
      x = l->start;
    }
    return -1;
  }
  void extract(int64_t a, int64_t e, std::string* out) const {
    out->assign(b + a, (size_t)(e - a));
    for (auto it = first_after(a); it != cz.end() && it->start < e; ++it) {
      const int64_t s = std::max(a, it->start), t = std::min(e, it->end);
      if (s < t) std::memset(&(*out)[s - a], '*', (size_t)(t - s));
    }
  }
};

// findLocation (scanner.go:445-502) over the censored buffer.  start_line (0-based) =
// newlines before start; the lines around the match are found from the match instead of
// a newline index of the whole file.
void find_location(int64_t start, int64_t end, const Censored& c, int64_t start_line, Finding* f) {
  const int64_t n = c.n;
  const int64_t line_start = c.prev_nl(start) + 1;  // after the last newline before start
  const int64_t line_end = c.next_nl(start);        // the first newline at or after start
  const int64_t end_line = start_line + c.count(start, end);
  if (line_end - line_start > 100) {
    int64_t ts = start - 30 < 0 ? 0 : start - 30;
    int64_t te = end + 20 > n ? n : end + 20;
    c.extract(ts, te, &f->match);
  } else {
    c.extract(line_start, line_end, &f->match);
  }
  // code lines [start_line - 2, end_line + 2), clamped to the lines of the file
  const int64_t code_start = start_line - 2 < 0 ? 0 : start_line - 2;
  int64_t ls = line_start;
  for (int64_t i = start_line; i > code_start; i--) ls = c.prev_nl(ls - 1) + 1;
  bool found_first = false;
  f->lines.clear();
  f->lines.reserve((size_t)(end_line + 2 - code_start));
  for (int64_t i = code_start; i < end_line + 2; i++) {
    const int64_t le = c.next_nl(ls);
    bool cause = i >= start_line && i <= end_line;
    Line ln;
    ln.number = (int32_t)(i + 1);
    ln.flags = (uint8_t)((cause ? 1 : 0) | ((!found_first && cause) ? 2 : 0));
    c.extract(ls, le, &ln.content);
    found_first = found_first || cause;
    f->lines.push_back(std::move(ln));
    if (le >= n) break;  // the last line of the file
    ls = le + 1;
  }
  for (auto it = f->lines.rbegin(); it != f->lines.rend(); ++it)
    if (it->flags & 1) {
      it->flags |= 4;
      break;
    }
  f->start_line = (int32_t)(start_line + 1);
  f->end_line = (int32_t)(end_line + 1);
}

}  // namespace

// TSG_PROF: per-phase cycle counters of scan_file (printed at exit)
static std::atomic<uint64_t> g_ph[8];
// per-thread phase sums in slots of their own (no shared cache line is written per lap:
// contended atomics would distort what they measure); PhDump adds the slots up
struct alignas(64) PhSlot {
  uint64_t v[8];
};
static PhSlot g_phslot[256];
static std::atomic<int> g_phslots{0};
static thread_local PhSlot* t_phslot = nullptr;
static PhSlot& ph_slot() {
  if (!t_phslot) t_phslot = &g_phslot[g_phslots++ & 255];
  return *t_phslot;
}
static std::atomic<uint64_t> g_rule_cyc[2048], g_rule_calls[2048], g_rule_bytes[2048];
static std::string g_rule_name[2048];  // rule ids seen by the profiler (names outlive rule sets)
static const bool g_prof = getenv("TSG_PROF") != nullptr;
struct PhDump {
  ~PhDump() {
    if (!g_prof) return;
    const char* nm[8] = {"allowpath", "rulegates", "lower", "findall", "allowmatch", "locate", "total", "nfiles"};
    for (int i = 0; i < 8; i++) {
      uint64_t t = g_ph[i];
      for (const auto& sl : g_phslot) t += sl.v[i];
      fprintf(stderr, "scan_file %-10s %.2f Mcyc\n", nm[i], t / 1e6);
    }
    std::vector<std::pair<uint64_t, size_t>> v;
    for (size_t r = 0; r < 2048; r++)
      if (g_rule_calls[r]) v.push_back({g_rule_cyc[r].load(), r});
    std::sort(v.rbegin(), v.rend());
    for (size_t i = 0; i < v.size() && i < 12; i++)
      fprintf(stderr, "  findall %-32s %8.2f Mcyc %7lu calls %10lu window bytes\n", g_rule_name[v[i].second].c_str(),
              v[i].first / 1e6, (unsigned long)g_rule_calls[v[i].second].load(), (unsigned long)g_rule_bytes[v[i].second].load());
  }
};
static PhDump g_phdump;
struct PhT {
  uint64_t t = g_prof ? __rdtsc() : 0;
  void lap(int i) {
    if (!g_prof) return;
    uint64_t n = __rdtsc();
    ph_slot().v[i] += n - t;
    t = n;
  }
};

void scan_file(const Ruleset& rs, const std::string& path, const uint8_t* content, size_t n,
               const FileGate* gate, FileResult* out) {
  PhT ph, tot;
  if (g_prof) ph_slot().v[7] += 1000000;
  struct TotL { PhT& t; ~TotL() { t.lap(6); } } totl{tot};
  out->findings.clear();
  out->status = kNoFindings;
  if ((gate && gate->path_allowed >= 0) ? gate->path_allowed == 1 : rs.AllowPath(path)) {  // scanner.go:343-347
    out->status = kPathAllowed;
    return;
  }
  ph.lap(0);
  std::string lowered;
  bool have_lowered = false;
  std::map<std::string, int8_t> kwcache;  // keyword -> 1 present, -1 absent
  Blocks global{content, n, &rs.exclude};
  std::vector<std::pair<uint32_t, Loc>> matched;
  Censored censored{(const char*)content, (int64_t)n, {}};
  std::vector<int64_t> idx;

  for (size_t ri = 0; ri < rs.rules.size(); ri++) {  // scanner.go:355
    const RuleC& r = rs.rules[ri];
    const RuleWindows* win = nullptr;
    if (gate) {
      // GPU: no candidate end offset for this rule -> its regex has no match here
      win = gate->windows[ri];
      if (!win) continue;
      if (gate->kw_state[ri] == 0) continue;
    }
    ph.lap(1);
    if (r.path && !r.path->Match((const uint8_t*)path.data(), path.size())) continue;
    if (allow_path(r.allow, path)) continue;
    ph.lap(1);
    if (gate && gate->kw_state[ri] == 2 && r.kw_ascii) {
      // exact keyword gate without lowering the file (per-keyword results cached)
      bool hit = r.kw_lower.empty();
      for (size_t k = 0; k < r.kw_lower.size() && !hit; k++) {
        const std::string& kw = r.kw_lower[k];
        int8_t& c = kwcache[kw];
        if (c == 0)
          c = (gate->ascii_fold_exact ? contains_fold_ascii(content, n, kw) : contains_fold_runes(content, n, kw)) ? 1 : -1;
        hit = c > 0;
      }
      ph.lap(2);
      if (!hit) continue;
    } else if (!gate || gate->kw_state[ri] == 2) {
      if (!have_lowered) {
        go_to_lower(content, n, &lowered);
        have_lowered = true;
      }
      if (!match_keywords(r, lowered)) {
        ph.lap(2);
        continue;
      }
      ph.lap(2);
    }
    if (!r.regex) continue;
    // FindLocations / FindSubmatchLocations (scanner.go:96-141)
    const bool sub = !r.secret_group_name.empty();
    const int ns = sub ? r.regex->NumSlots() : 2;
    idx.clear();
    const uint64_t tf0 = g_prof ? __rdtsc() : 0;
    if (!win || win->whole) {
      r.regex->FindAll(content, n, sub, &idx);
    } else {
      r.regex->FindAllWindows(content, n, sub, win->iv, &idx);
    }
    if (g_prof && ri < 2048) {
      if (g_rule_calls[ri] == 0 && g_rule_name[ri].empty()) g_rule_name[ri] = r.id;  // racy, names only
      g_rule_cyc[ri] += __rdtsc() - tf0;
      g_rule_calls[ri]++;
      uint64_t wb = 0;
      if (!win || win->whole) wb = n;
      else for (const auto& w : win->iv) wb += (uint64_t)(w.second - w.first + 1);
      g_rule_bytes[ri] += wb;
    }
    ph.lap(3);
    std::vector<Loc> locs;
    for (size_t k = 0; k + ns - 1 < idx.size(); k += ns) {
      int64_t s = idx[k], e = idx[k + 1];
      if (rs.Allow(content + s, e - s) || allow_match(r.allow, content + s, e - s)) continue;
      if (!sub) {
        locs.push_back({s, e});
      } else {
        for (int g : r.group_idx) locs.push_back({idx[k + 2 * g], idx[k + 2 * g + 1]});
      }
    }
    ph.lap(4);
    if (locs.empty()) continue;
    Blocks local{content, n, &r.exclude};
    for (const auto& loc : locs) {
      if (global.Match(loc) || local.Match(loc)) continue;
      if (loc.start < 0) continue;  // reference panics (slice bounds); never produced by valid rules
      matched.push_back({(uint32_t)ri, loc});
      censored.cz.push_back(loc);  // censorLocation
    }
  }
  ph.lap(4);
  if (matched.empty()) return;  // Secret{}
  // line numbers: newlines of the censored buffer counted once, in match-start order
  std::vector<uint32_t> order(matched.size());
  for (size_t k = 0; k < order.size(); k++) order[k] = (uint32_t)k;
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    return matched[x].second.start < matched[y].second.start;
  });
  out->findings.resize(matched.size());
  censored.finish();
  int64_t pos = 0, line = 0;
  for (uint32_t k : order) {
    const Loc& l = matched[k].second;
    line += censored.count(pos, l.start);
    pos = l.start;
    out->findings[k].rule = matched[k].first;
    find_location(l.start, l.end, censored, line, &out->findings[k]);
  }
  const auto& rules = rs.rules;
  gosort::sort_slice(out->findings, [&rules](const Finding& a, const Finding& b) {
    const std::string& ia = rules[a.rule].id;
    const std::string& ib = rules[b.rule].id;
    if (ia != ib) return ia < ib;
    return a.match < b.match;
  });
  out->status = kHasFindings;
  ph.lap(5);
}

// ------------------------------------------------------------------ serialization
static void put_u32(std::string* o, uint32_t v) { o->append((const char*)&v, 4); }
static void put_bytes(std::string* o, const std::string& s) {
  put_u32(o, (uint32_t)s.size());
  o->append(s);
}

namespace {
struct Writer {
  char* p;
  void u8(uint8_t v) { *p++ = (char)v; }
  void u32(uint32_t v) {
    std::memcpy(p, &v, 4);
    p += 4;
  }
  void bytes(const std::string& s) {
    u32((uint32_t)s.size());
    std::memcpy(p, s.data(), s.size());
    p += s.size();
  }
};
size_t findings_bytes(const FileResult& r) {
  size_t n = 0;
  for (const auto& f : r.findings) {
    n += 16 + f.match.size() + 4;
    for (const auto& ln : f.lines) n += 9 + ln.content.size();
  }
  return n;
}
void write_findings(Writer& w, const FileResult& r) {
  for (const auto& f : r.findings) {
    w.u32(f.rule);
    w.u32((uint32_t)f.start_line);
    w.u32((uint32_t)f.end_line);
    w.bytes(f.match);
    w.u32((uint32_t)f.lines.size());
    for (const auto& ln : f.lines) {
      w.u32((uint32_t)ln.number);
      w.u8(ln.flags);
      w.bytes(ln.content);
    }
  }
}
}  // namespace

void serialize_batch(const BatchResult& br, std::string* out, int nthreads) {
  const size_t F = br.status.size();
  // file ranges per thread: sizes, prefix offsets, then every range written in parallel
  const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)std::max(nthreads, 1), F / 32768));
  std::vector<size_t> lo(T + 1), bytes(T + 1, 0);
  for (size_t t = 0; t <= T; t++) lo[t] = F * t / T;
  auto range_bytes = [&](size_t t) {
    size_t n = 0;
    for (size_t f = lo[t]; f < lo[t + 1]; f++) {
      n += 5;
      if (br.slot[f] != UINT32_MAX) n += findings_bytes(br.res[br.slot[f]]);
    }
    bytes[t + 1] = n;
  };
  auto write_range = [&](size_t t) {
    Writer w{&(*out)[0] + 8 + bytes[t]};
    for (size_t f = lo[t]; f < lo[t + 1]; f++) {
      const uint32_t k = br.slot[f];
      if (k == UINT32_MAX) {
        w.u8(br.status[f]);
        w.u32(0);
      } else {
        const FileResult& r = br.res[k];
        w.u8(r.status);
        w.u32((uint32_t)r.findings.size());
        write_findings(w, r);
      }
    }
  };
  auto run = [&](auto fn) { pool_for(T, (int)T, [&](size_t t) { fn(t); }, 1); };
  run(range_bytes);
  for (size_t t = 0; t < T; t++) bytes[t + 1] += bytes[t];
  out->resize(8 + bytes[T]);
  Writer w{&(*out)[0]};
  w.u32(0x31475354u);  // "TSG1"
  w.u32((uint32_t)F);
  run(write_range);
}

void serialize_results(const std::vector<FileResult>& res, std::string* out) {
  out->clear();
  put_u32(out, 0x31475354u);  // "TSG1"
  put_u32(out, (uint32_t)res.size());
  for (const auto& r : res) {
    out->push_back((char)r.status);
    put_u32(out, (uint32_t)r.findings.size());
    for (const auto& f : r.findings) {
      put_u32(out, f.rule);
      put_u32(out, (uint32_t)f.start_line);
      put_u32(out, (uint32_t)f.end_line);
      put_bytes(out, f.match);
      put_u32(out, (uint32_t)f.lines.size());
      for (const auto& ln : f.lines) {
        put_u32(out, (uint32_t)ln.number);
        out->push_back((char)ln.flags);
        put_bytes(out, ln.content);
      }
    }
  }
}

static uint32_t rd_u32(const std::string& b, size_t& p) {
  if (p + 4 > b.size()) throw std::runtime_error("truncated result");
  uint32_t v;
  std::memcpy(&v, b.data() + p, 4);
  p += 4;
  return v;
}

void result_record_spans(const std::string& b, std::vector<size_t>* rec) {
  size_t p = 0;
  if (rd_u32(b, p) != 0x31475354u) throw std::runtime_error("bad result magic");
  const uint32_t n = rd_u32(b, p);
  rec->resize((size_t)n + 1);
  for (uint32_t i = 0; i < n; i++) {
    (*rec)[i] = p;
    p += 1;  // status
    const uint32_t nf = rd_u32(b, p);
    for (uint32_t f = 0; f < nf; f++) {
      p += 12;              // rule, start line, end line
      p += rd_u32(b, p);    // match
      const uint32_t nl = rd_u32(b, p);
      for (uint32_t l = 0; l < nl; l++) {
        p += 5;             // number, flags
        p += rd_u32(b, p);  // content
      }
    }
    if (p > b.size()) throw std::runtime_error("truncated result");
  }
  if (p != b.size()) throw std::runtime_error("trailing bytes after the last file record");
  (*rec)[n] = p;
}

}  // namespace tsg
