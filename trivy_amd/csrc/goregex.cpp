// Go 1.19 regexp dialect: parser, compiler and Pike VM.  See goregex.hpp.
#include "goregex.hpp"
#include "internal.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace tsg {

#include "unicode_tables.inc"

// ------------------------------------------------------------------ unicode helpers
int32_t decode_rune(const uint8_t* b, size_t n, size_t pos, int* width) {
  if (pos >= n) {
    *width = 0;
    return kEOT;
  }
  uint8_t c0 = b[pos];
  if (c0 < 0x80) {
    *width = 1;
    return c0;
  }
  auto cont = [&](size_t k, uint8_t lo, uint8_t hi) {
    return pos + k < n && b[pos + k] >= lo && b[pos + k] <= hi;
  };
  if (c0 >= 0xC2 && c0 <= 0xDF) {
    if (cont(1, 0x80, 0xBF)) {
      *width = 2;
      return ((c0 & 0x1F) << 6) | (b[pos + 1] & 0x3F);
    }
  } else if (c0 >= 0xE0 && c0 <= 0xEF) {
    uint8_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
    if (cont(1, lo, hi) && cont(2, 0x80, 0xBF)) {
      *width = 3;
      return ((c0 & 0x0F) << 12) | ((b[pos + 1] & 0x3F) << 6) | (b[pos + 2] & 0x3F);
    }
  } else if (c0 >= 0xF0 && c0 <= 0xF4) {
    uint8_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
    if (cont(1, lo, hi) && cont(2, 0x80, 0xBF) && cont(3, 0x80, 0xBF)) {
      *width = 4;
      return ((c0 & 0x07) << 18) | ((b[pos + 1] & 0x3F) << 12) | ((b[pos + 2] & 0x3F) << 6) |
             (b[pos + 3] & 0x3F);
    }
  }
  *width = 1;
  return kRuneError;
}

static const RunePair* find_pair(const RunePair* t, size_t n, int32_t r) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (t[m].a < r) lo = m + 1;
    else hi = m;
  }
  return (lo < n && t[lo].a == r) ? &t[lo] : nullptr;
}

void fold_orbit(int32_t r, std::vector<int32_t>* out) {
  out->clear();
  out->push_back(r);
  const size_t n = sizeof(kFoldNext) / sizeof(kFoldNext[0]);
  const RunePair* p = find_pair(kFoldNext, n, r);
  if (!p) return;
  int32_t x = p->b;
  while (x != r) {
    out->push_back(x);
    x = find_pair(kFoldNext, n, x)->b;
  }
  std::sort(out->begin(), out->end());
}

int32_t simple_lower(int32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  const RunePair* p = find_pair(kLower, sizeof(kLower) / sizeof(kLower[0]), r);
  return p ? p->b : r;
}

static void append_utf8(int32_t r, std::string* out) {
  if (r < 0 || r > kMaxRune || (r >= 0xD800 && r <= 0xDFFF)) r = kRuneError;
  if (r < 0x80) {
    out->push_back((char)r);
  } else if (r < 0x800) {
    out->push_back((char)(0xC0 | (r >> 6)));
    out->push_back((char)(0x80 | (r & 0x3F)));
  } else if (r < 0x10000) {
    out->push_back((char)(0xE0 | (r >> 12)));
    out->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    out->push_back((char)(0x80 | (r & 0x3F)));
  } else {
    out->push_back((char)(0xF0 | (r >> 18)));
    out->push_back((char)(0x80 | ((r >> 12) & 0x3F)));
    out->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    out->push_back((char)(0x80 | (r & 0x3F)));
  }
}

void go_to_lower(const uint8_t* b, size_t n, std::string* out) {
  out->clear();
  bool ascii = true;
  for (size_t i = 0; i < n; i++)
    if (b[i] >= 0x80) {
      ascii = false;
      break;
    }
  if (ascii) {
    out->resize(n);
    for (size_t i = 0; i < n; i++) {
      uint8_t c = b[i];
      (*out)[i] = (char)((c >= 'A' && c <= 'Z') ? c + 32 : c);
    }
    return;
  }
  out->reserve(n);
  size_t i = 0;
  while (i < n) {
    int w;
    int32_t r = decode_rune(b, n, i, &w);
    append_utf8(simple_lower(r), out);
    i += w;
  }
}

bool empty_ok(uint32_t op, int32_t r1, int32_t r2) {
  if (op == 0) return true;
  if (op & kBeginLine) {
    if (r1 != '\n' && r1 >= 0) return false;
    op &= ~kBeginLine;
  }
  if (op & kBeginText) {
    if (r1 >= 0) return false;
    op &= ~kBeginText;
  }
  if (op == 0) return true;
  if (op & kEndLine) {
    if (r2 != '\n' && r2 >= 0) return false;
    op &= ~kEndLine;
  }
  if (op & kEndText) {
    if (r2 >= 0) return false;
    op &= ~kEndText;
  }
  if (op == 0) return true;
  if (is_word_byte(r1) != is_word_byte(r2)) op &= ~kWordBoundary;
  else op &= ~kNoWordBoundary;
  return op == 0;
}

// ------------------------------------------------------------------ ranges
static Ranges clean(Ranges r) {
  std::sort(r.begin(), r.end());
  Ranges out;
  for (auto& p : r) {
    if (!out.empty() && (int64_t)p.first <= (int64_t)out.back().second + 1) {
      if (p.second > out.back().second) out.back().second = p.second;
    } else {
      out.push_back(p);
    }
  }
  return out;
}

static Ranges negate(const Ranges& in) {
  Ranges r = clean(in), out;
  int32_t next = 0;
  for (auto& p : r) {
    if (p.first > next) out.push_back({next, p.first - 1});
    next = p.second + 1;
  }
  if (next <= kMaxRune) out.push_back({next, kMaxRune});
  return out;
}

// appendFoldedRange: every rune plus its SimpleFold orbit
static Ranges fold(const Ranges& in) {
  Ranges out = in;
  const size_t n = sizeof(kFoldNext) / sizeof(kFoldNext[0]);
  std::vector<int32_t> orb;
  for (auto& p : in) {
    // walk only the runes that have orbits
    size_t lo = 0, hi = n;
    while (lo < hi) {
      size_t m = (lo + hi) / 2;
      if (kFoldNext[m].a < p.first) lo = m + 1;
      else hi = m;
    }
    for (size_t k = lo; k < n && kFoldNext[k].a <= p.second; k++) {
      fold_orbit(kFoldNext[k].a, &orb);
      for (int32_t x : orb) out.push_back({x, x});
    }
  }
  return clean(out);
}

static const Ranges kPerlD = {{'0', '9'}};
static const Ranges kPerlS = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}};
static const Ranges kPerlW = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};

struct PosixEnt {
  const char* name;
  Ranges r;
};
static const std::vector<PosixEnt>& posix_classes() {
  static const std::vector<PosixEnt> t = {
      {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
      {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
      {"ascii", {{0, 0x7F}}},
      {"blank", {{'\t', '\t'}, {' ', ' '}}},
      {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{'0', '9'}}},
      {"graph", {{'!', '~'}}},
      {"lower", {{'a', 'z'}}},
      {"print", {{' ', '~'}}},
      {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
      {"space", {{'\t', '\r'}, {' ', ' '}}},
      {"upper", {{'A', 'Z'}}},
      {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
      {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
  };
  return t;
}

// ------------------------------------------------------------------ AST
enum class NK : uint8_t {
  Empty, NoMatch, Rune, BOT, EOT, BOL, EOL, WB, NWB, Cap, Cat, Alt, Star, Plus, Quest, Repeat
};

struct Node {
  NK k = NK::Empty;
  bool greedy = true;
  int cap = 0, min = 0, max = 0;
  Ranges r;
  std::vector<int> sub;
};

enum : int { FOLD = 1, DOTNL = 2, ONELINE = 4, NONGREEDY = 8 };

struct ParseError {
  std::string msg;
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}

  int parse() {
    int n = parse_alt();
    if (i_ != s_.size()) fail("unexpected )");
    return n;
  }

  std::vector<Node> nodes;
  std::vector<std::string> names{""};
  int ncap = 0;

 private:
  const std::string& s_;
  size_t i_ = 0;
  int flags_ = ONELINE;  // Perl: ClassNL|OneLine|PerlX|UnicodeGroups

  [[noreturn]] void fail(const std::string& m) {
    throw ParseError{"error parsing regexp: " + m + ": `" + s_ + "`"};
  }
  int peek(size_t k = 0) const { return i_ + k < s_.size() ? (uint8_t)s_[i_ + k] : -1; }

  // next source rune (patterns are UTF-8)
  int32_t next_rune() {
    int w;
    int32_t r = decode_rune((const uint8_t*)s_.data(), s_.size(), i_, &w);
    if (r == kRuneError && w == 1) fail("invalid UTF-8");
    i_ += w;
    return r;
  }

  int add(Node n) {
    nodes.push_back(std::move(n));
    return (int)nodes.size() - 1;
  }
  int leaf(NK k) {
    Node n;
    n.k = k;
    return add(std::move(n));
  }
  int rune_node(Ranges r) {
    Node n;
    n.k = NK::Rune;
    n.r = std::move(r);
    return add(std::move(n));
  }
  int literal(int32_t r) {
    if (flags_ & FOLD) {
      std::vector<int32_t> orb;
      fold_orbit(r, &orb);
      Ranges rs;
      for (int32_t x : orb) rs.push_back({x, x});
      return rune_node(clean(rs));
    }
    return rune_node({{r, r}});
  }

  int parse_alt() {
    std::vector<int> alts{parse_concat()};
    while (peek() == '|') {
      i_++;
      alts.push_back(parse_concat());
    }
    if (alts.size() == 1) return alts[0];
    Node n;
    n.k = NK::Alt;
    n.sub = alts;
    return add(std::move(n));
  }

  int parse_concat() {
    std::vector<int> items;
    while (true) {
      int c = peek();
      if (c < 0 || c == '|' || c == ')') break;
      int a = parse_atom();
      if (a < 0) continue;
      items.push_back(parse_repeat(a));
    }
    if (items.empty()) return leaf(NK::Empty);
    if (items.size() == 1) return items[0];
    Node n;
    n.k = NK::Cat;
    n.sub = items;
    return add(std::move(n));
  }

  bool try_braces(int* lo, int* hi) {
    size_t j = i_ + 1;
    auto digits = [&](size_t k) {
      while (k < s_.size() && s_[k] >= '0' && s_[k] <= '9') k++;
      return k;
    };
    size_t k = digits(j);
    if (k == j) return false;
    long long a = std::stoll(s_.substr(j, std::min<size_t>(k - j, 9)));
    if (k - j > 9) a = 100000;
    long long b = a;
    j = k;
    if (j < s_.size() && s_[j] == ',') {
      j++;
      if (j < s_.size() && s_[j] == '}') {
        b = -1;
      } else {
        k = digits(j);
        if (k == j) return false;
        b = std::stoll(s_.substr(j, std::min<size_t>(k - j, 9)));
        if (k - j > 9) b = 100000;
        j = k;
      }
    }
    if (j >= s_.size() || s_[j] != '}') return false;
    i_ = j + 1;
    if (a > 1000 || b > 1000 || (b >= 0 && b < a)) fail("invalid repeat count");
    *lo = (int)a;
    *hi = (int)b;
    return true;
  }

  int parse_repeat(int atom) {
    bool last_rep = false;
    size_t rep_start = 0;
    while (true) {
      int c = peek();
      size_t start = i_;
      int lo, hi;
      NK k;
      if (c == '*') {
        i_++;
        k = NK::Star;
        lo = 0;
        hi = -1;
      } else if (c == '+') {
        i_++;
        k = NK::Plus;
        lo = 1;
        hi = -1;
      } else if (c == '?') {
        i_++;
        k = NK::Quest;
        lo = 0;
        hi = 1;
      } else if (c == '{') {
        if (!try_braces(&lo, &hi)) return atom;
        k = NK::Repeat;
      } else {
        return atom;
      }
      if (last_rep)
        fail("invalid nested repetition operator: `" + s_.substr(rep_start, i_ - rep_start) + "`");
      bool greedy = true;
      if (peek() == '?') {
        i_++;
        greedy = false;
      }
      if (flags_ & NONGREEDY) greedy = !greedy;
      Node n;
      n.k = k;
      n.min = lo;
      n.max = hi;
      n.greedy = greedy;
      n.sub = {atom};
      atom = add(std::move(n));
      last_rep = true;
      rep_start = start;
    }
  }

  int parse_atom() {
    int c = peek();
    if (c == '(') return parse_group();
    if (c == '[') return rune_node(parse_class());
    if (c == '*' || c == '+' || c == '?')
      fail(std::string("missing argument to repetition operator: `") + (char)c + "`");
    if (c == '{') {
      size_t save = i_;
      int lo, hi;
      if (try_braces(&lo, &hi)) fail("missing argument to repetition operator: `" + s_.substr(save, i_ - save) + "`");
    }
    if (c == '.') {
      i_++;
      if (flags_ & DOTNL) return rune_node({{0, kMaxRune}});
      return rune_node({{0, '\n' - 1}, {'\n' + 1, kMaxRune}});
    }
    if (c == '^') {
      i_++;
      return leaf((flags_ & ONELINE) ? NK::BOT : NK::BOL);
    }
    if (c == '$') {
      i_++;
      return leaf((flags_ & ONELINE) ? NK::EOT : NK::EOL);
    }
    if (c == '\\') return parse_backslash();
    return literal(next_rune());
  }

  void close() {
    if (peek() != ')') fail("missing closing )");
    i_++;
  }

  int parse_group() {
    i_++;
    int saved = flags_;
    if (s_.compare(i_, 3, "?P=") == 0) fail("invalid named capture");
    if (s_.compare(i_, 3, "?P<") == 0) {
      size_t end = s_.find('>', i_);
      if (end == std::string::npos) fail("invalid named capture");
      std::string name = s_.substr(i_ + 3, end - i_ - 3);
      bool ok = !name.empty();
      for (char ch : name)
        if (!(isalnum((unsigned char)ch) || ch == '_')) ok = false;
      if (!ok) fail("invalid named capture: `" + s_.substr(i_ - 1, end - i_ + 2) + "`");
      i_ = end + 1;
      int idx = ++ncap;
      names.push_back(name);
      int sub = parse_alt();
      close();
      flags_ = saved;
      Node n;
      n.k = NK::Cap;
      n.cap = idx;
      n.sub = {sub};
      return add(std::move(n));
    }
    if (peek() == '?') {
      size_t j = i_ + 1;
      bool neg = false, sawflag = false;
      int fl = flags_;
      char ch = 0;
      while (true) {
        if (j >= s_.size()) fail("missing closing )");
        ch = s_[j];
        if (ch == 'i') {
          fl = neg ? (fl & ~FOLD) : (fl | FOLD);
          sawflag = true;
        } else if (ch == 'm') {
          fl = neg ? (fl | ONELINE) : (fl & ~ONELINE);
          sawflag = true;
        } else if (ch == 's') {
          fl = neg ? (fl & ~DOTNL) : (fl | DOTNL);
          sawflag = true;
        } else if (ch == 'U') {
          fl = neg ? (fl & ~NONGREEDY) : (fl | NONGREEDY);
          sawflag = true;
        } else if (ch == '-') {
          if (neg) fail("invalid or unsupported Perl syntax");
          neg = true;
          sawflag = false;
        } else if (ch == ')' || ch == ':') {
          bool empty_flags = (j == i_ + 1);
          if ((neg && !sawflag) || (empty_flags && ch == ')'))
            fail("invalid or unsupported Perl syntax");
          break;
        } else {
          fail("invalid or unsupported Perl syntax");
        }
        j++;
      }
      i_ = j + 1;
      flags_ = fl;
      if (ch == ')') return -1;  // flags persist to the end of the enclosing group
      int sub = parse_alt();
      close();
      flags_ = saved;
      return sub;
    }
    int idx = ++ncap;
    names.push_back("");
    int sub = parse_alt();
    close();
    flags_ = saved;
    Node n;
    n.k = NK::Cap;
    n.cap = idx;
    n.sub = {sub};
    return add(std::move(n));
  }

  Ranges perl_group(char ch) {
    char lc = (char)tolower(ch);
    Ranges base = lc == 'd' ? kPerlD : lc == 's' ? kPerlS : kPerlW;
    if (flags_ & FOLD) base = fold(base);
    return isupper((unsigned char)ch) ? negate(base) : clean(base);
  }

  Ranges unicode_class() {
    bool neg = s_[i_ + 1] == 'P';
    size_t j = i_ + 2;
    if (j >= s_.size()) fail("invalid character class range");
    std::string name;
    if (s_[j] == '{') {
      size_t end = s_.find('}', j);
      if (end == std::string::npos) fail("invalid character class range");
      name = s_.substr(j + 1, end - j - 1);
      i_ = end + 1;
    } else {
      i_ = j;
      int32_t r = next_rune();
      std::string t;
      append_utf8(r, &t);
      name = t;
    }
    if (!name.empty() && name[0] == '^') {
      neg = !neg;
      name = name.substr(1);
    }
    Ranges rs;
    if (name == "Any") {
      rs = {{0, kMaxRune}};
    } else {
      bool found = false;
      for (const auto& c : kCats) {
        if (name == c.name) {
          for (int k = 0; k < c.n; k++) rs.push_back({c.r[k].a, c.r[k].b});
          found = true;
        }
      }
      if (!found) fail("invalid character class range: `\\p{" + name + "}`");
    }
    if (flags_ & FOLD) rs = fold(rs);
    return neg ? negate(rs) : clean(rs);
  }

  int parse_backslash() {
    int nx = peek(1);
    if (nx < 0) fail("trailing backslash at end of expression");
    switch (nx) {
      case 'A': i_ += 2; return leaf(NK::BOT);
      case 'z': i_ += 2; return leaf(NK::EOT);
      case 'b': i_ += 2; return leaf(NK::WB);
      case 'B': i_ += 2; return leaf(NK::NWB);
      case 'Q': {
        size_t end = s_.find("\\E", i_ + 2);
        std::string lit = end == std::string::npos ? s_.substr(i_ + 2) : s_.substr(i_ + 2, end - i_ - 2);
        i_ = end == std::string::npos ? s_.size() : end + 2;
        std::vector<int> items;
        size_t k = 0;
        while (k < lit.size()) {
          int w;
          int32_t r = decode_rune((const uint8_t*)lit.data(), lit.size(), k, &w);
          k += w;
          items.push_back(literal(r));
        }
        if (items.empty()) return -1;
        if (items.size() == 1) return items[0];
        Node n;
        n.k = NK::Cat;
        n.sub = items;
        return add(std::move(n));
      }
      case 'p':
      case 'P':
        return rune_node(unicode_class());
      case 'd': case 'D': case 's': case 'S': case 'w': case 'W':
        i_ += 2;
        return rune_node(perl_group((char)nx));
      default:
        return literal(parse_escape());
    }
  }

  int32_t parse_escape() {
    i_++;  // backslash
    if (i_ >= s_.size()) fail("trailing backslash at end of expression");
    int32_t c = next_rune();
    if (c >= '1' && c <= '7') {
      int d = peek();
      if (!(d >= '0' && d <= '7')) fail("invalid escape sequence: `\\" + std::string(1, (char)c) + "`");
    }
    if (c >= '0' && c <= '7') {
      int32_t r = c - '0';
      for (int k = 0; k < 2; k++) {
        int d = peek();
        if (d >= '0' && d <= '7') {
          r = r * 8 + (d - '0');
          i_++;
        } else {
          break;
        }
      }
      return r;
    }
    if (c == 'x') {
      auto hexv = [](int ch) {
        if (ch >= '0' && ch <= '9') return ch - '0';
        if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
        if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
        return -1;
      };
      if (peek() == '{') {
        size_t j = i_ + 1;
        int64_t r = 0;
        int nd = 0;
        while (j < s_.size() && hexv((uint8_t)s_[j]) >= 0) {
          r = r * 16 + hexv((uint8_t)s_[j]);
          if (r > kMaxRune) fail("invalid escape sequence");
          j++;
          nd++;
        }
        if (nd == 0 || j >= s_.size() || s_[j] != '}') fail("invalid escape sequence");
        i_ = j + 1;
        return (int32_t)r;
      }
      int h1 = hexv(peek()), h2 = hexv(peek(1));
      if (h1 < 0 || h2 < 0) fail("invalid escape sequence");
      i_ += 2;
      return h1 * 16 + h2;
    }
    switch (c) {
      case 'a': return 7;
      case 'f': return 12;
      case 'n': return 10;
      case 'r': return 13;
      case 't': return 9;
      case 'v': return 11;
    }
    if (c < 0x80 && !isalnum(c)) return c;
    std::string t;
    append_utf8(c, &t);
    fail("invalid escape sequence: `\\" + t + "`");
  }

  Ranges parse_class() {
    i_++;
    bool neg = false;
    if (peek() == '^') {
      neg = true;
      i_++;
    }
    Ranges rs;
    bool first = true;
    while (peek() != ']' || first) {
      if (peek() < 0) fail("missing closing ]");
      first = false;
      if (peek() == '[' && peek(1) == ':') {
        size_t end = s_.find(":]", i_ + 2);
        if (end != std::string::npos) {
          std::string name = s_.substr(i_ + 2, end - i_ - 2);
          bool pneg = !name.empty() && name[0] == '^';
          if (pneg) name = name.substr(1);
          const Ranges* base = nullptr;
          for (const auto& e : posix_classes())
            if (name == e.name) base = &e.r;
          if (!base) fail("invalid character class range: `[:" + name + ":]`");
          Ranges r2 = *base;
          if (flags_ & FOLD) r2 = fold(r2);
          if (pneg) r2 = negate(r2);
          rs.insert(rs.end(), r2.begin(), r2.end());
          i_ = end + 2;
          continue;
        }
      }
      if (peek() == '\\' && (peek(1) == 'p' || peek(1) == 'P')) {
        Ranges r2 = unicode_class();
        rs.insert(rs.end(), r2.begin(), r2.end());
        continue;
      }
      if (peek() == '\\' && peek(1) >= 0 && strchr("dDsSwW", peek(1))) {
        Ranges r2 = perl_group((char)peek(1));
        rs.insert(rs.end(), r2.begin(), r2.end());
        i_ += 2;
        continue;
      }
      int32_t lo = class_char(), hi = lo;
      if (peek() == '-' && peek(1) >= 0 && peek(1) != ']') {
        i_++;
        hi = class_char();
        if (hi < lo) fail("invalid character class range");
      }
      if (flags_ & FOLD) {
        Ranges r2 = fold({{lo, hi}});
        rs.insert(rs.end(), r2.begin(), r2.end());
      } else {
        rs.push_back({lo, hi});
      }
    }
    i_++;
    rs = clean(rs);
    return neg ? negate(rs) : rs;
  }

  int32_t class_char() {
    if (peek() < 0) fail("missing closing ]");
    if (peek() == '\\') return parse_escape();
    return next_rune();
  }
};

// ------------------------------------------------------------------ compiler
namespace {

struct Frag {
  uint32_t i = 0;
  std::vector<uint32_t> out;  // patch list: inst << 1 | (1 = arg)
  bool nullable = false;
};

class Compiler {
 public:
  // relax >= 0: GPU superset program -- every counted repetition x{n,m} whose bounds
  // exceed `relax` becomes x{min(n,relax),} (see Regexp::RelaxedProg)
  // fold_high: U+017F / U+212A count as non-ASCII members too (a superset that also
  // accepts the runes (?i) folds into s / k; the host's folding-rune path)
  Compiler(const std::vector<Node>& nodes, Prog* p, int relax = -1, bool fold_high = false)
      : n_(nodes), p_(p), relax_(relax), fold_high_(fold_high) {
    p_->inst.push_back(Inst{Op::Fail, 0, 0});
  }

  Frag compile(int idx) {
    const Node& nd = n_[idx];
    switch (nd.k) {
      case NK::NoMatch: return Frag{};
      case NK::Empty: return nop();
      case NK::Rune: return rune(nd.r);
      case NK::BOT: return empty(kBeginText);
      case NK::EOT: return empty(kEndText);
      case NK::BOL: return empty(kBeginLine);
      case NK::EOL: return empty(kEndLine);
      case NK::WB: return empty(kWordBoundary);
      case NK::NWB: return empty(kNoWordBoundary);
      case NK::Cap: {
        Frag bra = cap((uint32_t)nd.cap * 2);
        Frag sub = compile(nd.sub[0]);
        Frag ket = cap((uint32_t)nd.cap * 2 + 1);
        return cat(cat(bra, sub), ket);
      }
      case NK::Cat: {
        Frag f;
        bool firstf = true;
        for (int s : nd.sub) {
          if (firstf) {
            f = compile(s);
            firstf = false;
          } else {
            f = cat(f, compile(s));
          }
        }
        return firstf ? nop() : f;
      }
      case NK::Alt: {
        Frag f;
        for (int s : nd.sub) f = alt(f, compile(s));
        return f;
      }
      case NK::Star:
      case NK::Plus:
      case NK::Quest:
      case NK::Repeat:
        return repeat(nd);
    }
    return Frag{};
  }

  Frag finish(int root) {
    Frag f = compile(root);
    uint32_t m = inst(Op::Match);
    patch(f.out, m);
    p_->start = f.i;
    return f;
  }

  // a prefix of the flattened top-level concatenation (GPU filter programs)
  Frag finish_atoms(const std::vector<int>& atoms) {
    Frag f;
    if (atoms.empty()) {
      f = nop();
    } else {
      f = compile(atoms[0]);
      for (size_t i = 1; i < atoms.size(); i++) f = cat(f, compile(atoms[i]));
    }
    uint32_t m = inst(Op::Match);
    patch(f.out, m);
    p_->start = f.i;
    return f;
  }

 private:
  const std::vector<Node>& n_;
  Prog* p_;
  int relax_;
  bool fold_high_;

  uint32_t inst(Op op) {
    p_->inst.push_back(Inst{op, 0, 0});
    return (uint32_t)p_->inst.size() - 1;
  }
  void patch(const std::vector<uint32_t>& l, uint32_t v) {
    for (uint32_t x : l) {
      Inst& in = p_->inst[x >> 1];
      if (x & 1) in.arg = v;
      else in.out = v;
    }
  }
  Frag nop() {
    Frag f;
    f.i = inst(Op::Nop);
    f.out = {f.i << 1};
    f.nullable = true;
    return f;
  }
  Frag empty(uint32_t op) {
    Frag f;
    f.i = inst(Op::Empty);
    p_->inst[f.i].arg = op;
    f.out = {f.i << 1};
    f.nullable = true;
    return f;
  }
  Frag cap(uint32_t slot) {
    Frag f;
    f.i = inst(Op::Cap);
    p_->inst[f.i].arg = slot;
    f.out = {f.i << 1};
    f.nullable = true;
    if ((int)slot + 1 > p_->nslots) p_->nslots = (int)slot + 1;
    return f;
  }
  Frag rune1(const Ranges& r) {
    Frag f;
    f.i = inst(Op::Rune);
    p_->runes.push_back(r);
    p_->inst[f.i].arg = (uint32_t)p_->runes.size() - 1;
    f.out = {f.i << 1};
    f.nullable = false;
    return f;
  }
  Frag rune(const Ranges& r) {
    if (relax_ < 0 || r.empty() || r.back().second < 0x80) return rune1(r);
    // relaxed (GPU) program: the ASCII part stays exact, every non-ASCII member of the
    // set becomes "one or more bytes >= 0x80" -- a superset of any rune's encoding and of
    // an invalid byte -- so the byte DFA needs no UTF-8 sub-states
    Ranges ascii;
    bool other_high = false;
    for (auto& p : r) {
      if (p.first < 0x80) ascii.push_back({p.first, std::min<int32_t>(p.second, 0x7F)});
      for (int32_t lo = std::max<int32_t>(p.first, 0x80); lo <= p.second; lo++) {
        // U+017F / U+212A only enter a set through (?i) folding of s / k; files that
        // contain them are resolved whole on the host (K1 fallback keywords), so the
        // GPU program may ignore them
        if (fold_high_ || (lo != 0x17F && lo != 0x212A)) {
          other_high = true;
          break;
        }
      }
    }
    if (!other_high) return rune1(ascii);
    Frag high = plus(rune1({{kHighByteRune, kHighByteRune}}), false);
    if (ascii.empty()) return high;
    return alt(rune1(ascii), high);
  }
  Frag cat(Frag f1, Frag f2) {
    if (f1.i == 0 || f2.i == 0) return Frag{};
    patch(f1.out, f2.i);
    Frag f;
    f.i = f1.i;
    f.out = std::move(f2.out);
    f.nullable = f1.nullable && f2.nullable;
    return f;
  }
  Frag alt(Frag f1, Frag f2) {
    if (f1.i == 0) return f2;
    if (f2.i == 0) return f1;
    Frag f;
    f.i = inst(Op::Alt);
    p_->inst[f.i].out = f1.i;
    p_->inst[f.i].arg = f2.i;
    f.out = std::move(f1.out);
    f.out.insert(f.out.end(), f2.out.begin(), f2.out.end());
    f.nullable = f1.nullable || f2.nullable;
    return f;
  }
  Frag quest(Frag f1, bool nongreedy) {
    Frag f;
    f.i = inst(Op::Alt);
    if (nongreedy) {
      p_->inst[f.i].arg = f1.i;
      f.out = {f.i << 1};
    } else {
      p_->inst[f.i].out = f1.i;
      f.out = {(f.i << 1) | 1};
    }
    f.out.insert(f.out.end(), f1.out.begin(), f1.out.end());
    f.nullable = true;
    return f;
  }
  Frag loop(Frag f1, bool nongreedy) {
    Frag f;
    f.i = inst(Op::Alt);
    if (nongreedy) {
      p_->inst[f.i].arg = f1.i;
      f.out = {f.i << 1};
    } else {
      p_->inst[f.i].out = f1.i;
      f.out = {(f.i << 1) | 1};
    }
    patch(f1.out, f.i);
    f.nullable = true;
    return f;
  }
  Frag plus(Frag f1, bool nongreedy) {
    Frag l = loop(f1, nongreedy);
    Frag f;
    f.i = f1.i;
    f.out = std::move(l.out);
    f.nullable = f1.nullable;
    return f;
  }
  Frag star(Frag f1, bool nongreedy) {
    if (f1.nullable) return quest(plus(f1, nongreedy), nongreedy);  // golang.org/issue/46123
    return loop(f1, nongreedy);
  }

  bool is_empty_match(int idx) const { return n_[idx].k == NK::Empty; }

  // regexp/syntax Simplify of star/plus/quest/repeat, then compile
  Frag repeat(const Node& nd) {
    int sub = nd.sub[0];
    bool ng = !nd.greedy;
    NK k = nd.k;
    int lo = nd.min, hi = nd.max;
    if (k == NK::Repeat && relax_ >= 0 && (hi == -1 || hi > relax_)) {
      lo = std::min(lo, relax_);
      hi = -1;
    }
    if (k == NK::Repeat) {
      if (lo == 0 && hi == 0) return nop();
      if (hi == -1) {
        if (lo == 0) k = NK::Star;
        else if (lo == 1) k = NK::Plus;
      } else if (lo == 1 && hi == 1) {
        return compile(sub);
      }
    }
    // simplify1: op of an empty match is the empty match; x** -> x*
    if (k != NK::Repeat) {
      if (is_empty_match(sub)) return nop();
      const Node& s = n_[sub];
      if (s.k == k && s.greedy == nd.greedy) return compile(sub);
      if (k == NK::Star) return star(compile(sub), ng);
      if (k == NK::Plus) return plus(compile(sub), ng);
      return quest(compile(sub), ng);
    }
    if (is_empty_match(sub)) return nop();
    if (hi == -1) {  // x{n,} = x^(n-1) x+
      Frag f;
      bool firstf = true;
      for (int i = 0; i < lo - 1; i++) {
        Frag c = compile(sub);
        f = firstf ? c : cat(f, c);
        firstf = false;
      }
      Frag p = simplified_plus(sub, ng, nd.greedy);
      return firstf ? p : cat(f, p);
    }
    // x{n,m} = x^n (x(x(x)?)?)?  -- suffix built inside-out
    Frag f;
    bool firstf = true;
    for (int i = 0; i < lo; i++) {
      Frag c = compile(sub);
      f = firstf ? c : cat(f, c);
      firstf = false;
    }
    if (hi > lo) {
      Frag suffix = suffix_chain(sub, hi - lo, ng, nd.greedy);
      f = firstf ? suffix : cat(f, suffix);
      firstf = false;
    }
    return f;
  }

  Frag simplified_plus(int sub, bool ng, bool greedy) {
    const Node& s = n_[sub];
    if (s.k == NK::Plus && s.greedy == greedy) return compile(sub);
    return plus(compile(sub), ng);
  }

  // depth copies nested: (x(x(x)?)?)?  (depth = m - n)
  Frag suffix_chain(int sub, int depth, bool ng, bool greedy) {
    if (depth == 1) {
      const Node& s = n_[sub];
      if (s.k == NK::Quest && s.greedy == greedy) return compile(sub);
      return quest(compile(sub), ng);
    }
    Frag x = compile(sub);
    Frag rest = suffix_chain(sub, depth - 1, ng, greedy);
    return quest(cat(x, rest), ng);
  }
};

}  // namespace

struct Regexp::Ast {
  std::vector<Node> nodes;
  int root = 0;
  int ncap = 0;
};

// Prog.Prefix (regexp/syntax/prog.go) over ASCII runes: an ASCII byte never lies inside a
// multi-byte rune, so each occurrence found by memmem is a position the matchers visit.
static std::string literal_prefix(const Prog& p) {
  std::string s;
  uint32_t pc = p.start;
  for (size_t guard = 0; guard < p.inst.size() && pc != 0; guard++) {
    const Inst& i = p.inst[pc];
    if (i.op == Op::Nop || i.op == Op::Cap) {
      pc = i.out;
      continue;
    }
    if (i.op != Op::Rune) break;
    const Ranges& r = p.runes[i.arg];
    if (r.size() != 1 || r[0].first != r[0].second || r[0].first < 0 || r[0].first >= 0x80) break;
    s.push_back((char)r[0].first);
    pc = i.out;
  }
  return s;
}

// first occurrence of the program's prefix at or after pos (-1: none)
static int64_t next_prefix(const Prog& p, const uint8_t* b, size_t n, int64_t pos) {
  if ((size_t)pos >= n) return -1;
  const void* q = memmem(b + pos, n - (size_t)pos, p.prefix.data(), p.prefix.size());
  return q ? (int64_t)((const uint8_t*)q - b) : -1;
}

Regexp::Regexp() = default;
Regexp::~Regexp() = default;

std::shared_ptr<Regexp> Regexp::Compile(const std::string& src, std::string* err) {
  auto re = std::make_shared<Regexp>();
  try {
    Parser p(src);
    int root = p.parse();
    re->src_ = src;
    re->names_ = p.names;
    re->prog_.nslots = 2 * (p.ncap + 1);
    Compiler c(p.nodes, &re->prog_);
    c.finish(root);
    re->prog_.nslots = 2 * (p.ncap + 1);
    re->prog_.ascii.assign(re->prog_.runes.size() * 2, 0);
    for (size_t k = 0; k < re->prog_.runes.size(); k++)
      for (const auto& rg : re->prog_.runes[k])
        for (int32_t c = std::max<int32_t>(rg.first, 0); c <= std::min<int32_t>(rg.second, 127); c++)
          re->prog_.ascii[k * 2 + c / 64] |= 1ull << (c % 64);
    re->prog_.prefix = literal_prefix(re->prog_);
    re->ast_ = std::make_shared<Ast>();
    re->ast_->nodes = std::move(p.nodes);
    re->ast_->root = root;
    re->ast_->ncap = p.ncap;
  } catch (const ParseError& e) {
    if (err) *err = e.msg;
    return nullptr;
  }
  return re;
}

// top-level concatenation with captures and nested concatenations flattened
static void flatten_atoms(const std::vector<Node>& nodes, int idx, std::vector<int>* out) {
  const Node& n = nodes[idx];
  if (n.k == NK::Cat) {
    for (int s : n.sub) flatten_atoms(nodes, s, out);
  } else if (n.k == NK::Cap) {
    flatten_atoms(nodes, n.sub[0], out);
  } else {
    out->push_back(idx);
  }
}

int Regexp::NumAtoms() const {
  std::vector<int> atoms;
  flatten_atoms(ast_->nodes, ast_->root, &atoms);
  return (int)atoms.size();
}

Prog Regexp::RelaxedProg(int k, int natoms, int first_atom, bool fold_high) const {
  Prog p;
  p.nslots = 2 * (ast_->ncap + 1);
  Compiler c(ast_->nodes, &p, k, fold_high);
  if (natoms < 0 && first_atom <= 0) {
    c.finish(ast_->root);
  } else {
    std::vector<int> atoms;
    flatten_atoms(ast_->nodes, ast_->root, &atoms);
    size_t a = std::min<size_t>(atoms.size(), (size_t)std::max(first_atom, 0));
    size_t b = natoms < 0 ? atoms.size() : std::min<size_t>(atoms.size(), a + (size_t)natoms);
    c.finish_atoms(std::vector<int>(atoms.begin() + a, atoms.begin() + b));
  }
  p.nslots = 2 * (ast_->ncap + 1);
  return p;
}

// ------------------------------------------------------------------ atom shapes
static int utf8_width(int32_t r) { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; }

static AtomInfo node_info(const std::vector<Node>& nodes, int idx) {
  const Node& n = nodes[idx];
  AtomInfo a;
  auto cat = [](AtomInfo x, const AtomInfo& y) {
    x.min_bytes += y.min_bytes;
    x.max_bytes = (x.max_bytes < 0 || y.max_bytes < 0) ? -1 : x.max_bytes + y.max_bytes;
    x.ascii_only = x.ascii_only && y.ascii_only;
    x.set[0] |= y.set[0];
    x.set[1] |= y.set[1];
    x.lit = -1;
    return x;
  };
  switch (n.k) {
    case NK::Rune: {
      a.min_bytes = 1;
      a.max_bytes = 1;
      for (auto& p : n.r) {
        for (int32_t c = p.first; c <= std::min<int32_t>(p.second, 0x7F); c++)
          a.set[c >> 6] |= 1ull << (c & 63);
        if (p.second >= 0x80) {
          // the only non-ASCII members (?i) folds into ASCII letters (see AtomInfo)
          bool only_fold = true;
          for (int32_t c = std::max<int32_t>(p.first, 0x80); c <= p.second && only_fold; c++)
            only_fold = c == 0x17F || c == 0x212A;
          if (!only_fold) {
            a.ascii_only = false;
            a.max_bytes = std::max<int64_t>(a.max_bytes, utf8_width(p.second));
            if (p.first <= 0xFFFD && 0xFFFD <= p.second) a.max_bytes = std::max<int64_t>(a.max_bytes, 3);
          }
        }
      }
      const int cnt = __builtin_popcountll(a.set[0]) + __builtin_popcountll(a.set[1]);
      auto has = [&](int c) { return (a.set[c >> 6] >> (c & 63)) & 1; };
      if (a.ascii_only && cnt == 1) {
        int c = a.set[0] ? __builtin_ctzll(a.set[0]) : 64 + __builtin_ctzll(a.set[1]);
        a.lit = (c >= 'A' && c <= 'Z') ? c + 32 : c;
      } else if (a.ascii_only && cnt == 2) {
        for (int c = 'a'; c <= 'z'; c++)
          if (has(c) && has(c - 32)) {
            a.lit = c;
            a.lit_fold = true;
          }
      }
      return a;
    }
    case NK::Cap:
      return node_info(nodes, n.sub[0]);
    case NK::Cat: {
      for (size_t i = 0; i < n.sub.size(); i++) a = cat(a, node_info(nodes, n.sub[i]));
      if (n.sub.size() == 1) a = node_info(nodes, n.sub[0]);
      return a;
    }
    case NK::Alt: {
      bool first = true;
      for (int s : n.sub) {
        AtomInfo b = node_info(nodes, s);
        if (first) {
          a = b;
          first = false;
        } else {
          a.min_bytes = std::min(a.min_bytes, b.min_bytes);
          a.max_bytes = (a.max_bytes < 0 || b.max_bytes < 0) ? -1 : std::max(a.max_bytes, b.max_bytes);
          a.ascii_only = a.ascii_only && b.ascii_only;
          a.set[0] |= b.set[0];
          a.set[1] |= b.set[1];
          a.lit = -1;
        }
      }
      a.lit = -1;
      return a;
    }
    case NK::Star:
    case NK::Plus:
    case NK::Quest:
    case NK::Repeat: {
      AtomInfo b = node_info(nodes, n.sub[0]);
      int64_t lo = n.k == NK::Plus ? 1 : n.k == NK::Repeat ? n.min : 0;
      int64_t hi = n.k == NK::Quest ? 1 : n.k == NK::Repeat ? n.max : -1;
      a = b;
      a.lit = -1;
      a.min_bytes = lo * b.min_bytes;
      a.max_bytes = (hi < 0 || b.max_bytes < 0) ? (b.max_bytes == 0 ? 0 : -1) : hi * b.max_bytes;
      return a;
    }
    case NK::NoMatch:
    case NK::Empty:
    default:
      return a;  // assertions and empty: zero width
  }
}

std::vector<AtomInfo> Regexp::Atoms() const {
  std::vector<int> atoms;
  flatten_atoms(ast_->nodes, ast_->root, &atoms);
  std::vector<AtomInfo> out;
  for (int i : atoms) out.push_back(node_info(ast_->nodes, i));
  return out;
}

// ------------------------------------------------------------------ Pike VM
namespace {

inline bool rune_in(const Ranges& r, int32_t c) {
  if (c < 0) return false;
  if (r.size() <= 8) {
    for (auto& p : r) {
      if (c < p.first) return false;
      if (c <= p.second) return true;
    }
    return false;
  }
  size_t lo = 0, hi = r.size();
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (r[m].second < c) lo = m + 1;
    else hi = m;
  }
  return lo < r.size() && r[lo].first <= c;
}

struct Queue {
  std::vector<uint32_t> sparse;
  std::vector<std::pair<uint32_t, int>> dense;  // pc, thread (-1 = none)
  explicit Queue(size_t n) : sparse(n, 0) { dense.reserve(n); }
  bool contains(uint32_t pc) const {
    uint32_t j = sparse[pc];
    return j < dense.size() && dense[j].first == pc;
  }
};

class Machine {
 public:
  Machine(const Prog& p, int nslots) : p_(p), ns_(nslots), q0_(p.inst.size()), q1_(p.inst.size()) {
    matchcap_.assign(ns_ > 0 ? ns_ : 1, -1);
  }

  bool run(const uint8_t* b, size_t n, int64_t pos, int64_t start_hi) {
    matched_ = false;
    std::fill(matchcap_.begin(), matchcap_.end(), -1);
    Queue* runq = &q0_;
    Queue* nextq = &q1_;
    int w, w1 = 0;
    int32_t r = decode_rune(b, n, (size_t)pos, &w), r1 = kEOT;
    if (r != kEOT) r1 = decode_rune(b, n, (size_t)pos + w, &w1);
    int32_t fr1, fr2;  // flag (before, after)
    if (pos == 0) {
      fr1 = kEOT;
      fr2 = r;
    } else {
      fr1 = b[pos - 1];  // only word/newline-ness matters: any byte >= 0x80 is a non-word rune
      fr2 = r;
    }
    while (true) {
      if (runq->dense.empty()) {
        if (matched_) break;
        if (pos > start_hi) break;
        if (!p_.prefix.empty()) {  // no thread alive: the next match starts at a prefix
          const int64_t q = next_prefix(p_, b, n, pos);
          if (q < 0 || q > start_hi) break;
          if (q > pos) {
            pos = q;
            r = decode_rune(b, n, (size_t)pos, &w);
            r1 = kEOT;
            if (r != kEOT) r1 = decode_rune(b, n, (size_t)pos + w, &w1);
            fr1 = b[pos - 1];
            fr2 = r;
          }
        }
      }
      if (!matched_ && pos <= start_hi) {
        if (ns_ > 0) matchcap_[0] = pos;
        add2(*runq, p_.start, pos, -2, fr1, fr2, -1);
      }
      fr1 = r;
      fr2 = r1;
      step(*runq, *nextq, pos, pos + w, r, fr1, fr2);
      if (w == 0) break;
      if (ns_ == 0 && matched_) break;
      pos += w;
      r = r1;
      w = w1;
      if (r != kEOT) r1 = decode_rune(b, n, (size_t)pos + w, &w1);
      std::swap(runq, nextq);
    }
    clear(*nextq);
    clear(*runq);
    return matched_;
  }

  const std::vector<int64_t>& matchcap() const { return matchcap_; }

 private:
  const Prog& p_;
  int ns_;
  Queue q0_, q1_;
  std::vector<int64_t> matchcap_;
  std::vector<int64_t> pool_caps_;
  std::vector<int> free_;
  bool matched_ = false;

  int alloc() {
    if (!free_.empty()) {
      int t = free_.back();
      free_.pop_back();
      return t;
    }
    int t = (int)(pool_caps_.size() / (ns_ > 0 ? ns_ : 1));
    pool_caps_.resize(pool_caps_.size() + (ns_ > 0 ? ns_ : 1), -1);
    return t;
  }
  int64_t* caps(int t) { return pool_caps_.data() + (size_t)t * (ns_ > 0 ? ns_ : 1); }
  void release(int t) { free_.push_back(t); }
  void clear(Queue& q) {
    for (auto& d : q.dense)
      if (d.second >= 0) release(d.second);
    q.dense.clear();
  }

  int64_t* capp(int owner) { return owner == -2 ? matchcap_.data() : caps(owner); }

  // machine.add (regexp/exec.go). The capture array is named by its owner (a thread
  // id, or -2 for matchcap_) because alloc() can grow pool_caps_ and move it.
  int add2(Queue& q, uint32_t pc, int64_t pos, int owner, int32_t f1, int32_t f2, int t) {
  again:
    if (pc == 0) return t;
    if (q.contains(pc)) return t;
    size_t j = q.dense.size();
    q.dense.push_back({pc, -1});
    q.sparse[pc] = (uint32_t)j;
    const Inst& i = p_.inst[pc];
    switch (i.op) {
      case Op::Fail:
        break;
      case Op::Alt:
        t = add2(q, i.out, pos, owner, f1, f2, t);
        pc = i.arg;
        goto again;
      case Op::Empty:
        if (empty_ok(i.arg, f1, f2)) {
          pc = i.out;
          goto again;
        }
        break;
      case Op::Nop:
        pc = i.out;
        goto again;
      case Op::Cap:
        if ((int)i.arg < ns_) {
          int64_t opos = capp(owner)[i.arg];
          capp(owner)[i.arg] = pos;
          add2(q, i.out, pos, owner, f1, f2, -1);
          capp(owner)[i.arg] = opos;
        } else {
          pc = i.out;
          goto again;
        }
        break;
      case Op::Match:
      case Op::Rune: {
        if (t < 0) t = alloc();
        if (ns_ > 0 && t != owner) {
          int64_t* src = capp(owner);
          int64_t* dst = caps(t);
          if (src != dst) std::memcpy(dst, src, sizeof(int64_t) * ns_);
        }
        q.dense[j].second = t;
        t = -1;
        break;
      }
    }
    return t;
  }

  void step(Queue& runq, Queue& nextq, int64_t pos, int64_t next_pos, int32_t c, int32_t f1,
            int32_t f2) {
    for (size_t j = 0; j < runq.dense.size(); j++) {
      int t = runq.dense[j].second;
      if (t < 0) continue;
      const Inst& i = p_.inst[runq.dense[j].first];
      bool addit = false;
      bool cut = false;
      if (i.op == Op::Match) {
        if (ns_ > 0) {
          caps(t)[1] = pos;
          std::memcpy(matchcap_.data(), caps(t), sizeof(int64_t) * ns_);
        }
        // first-match mode: cut off all lower-priority threads
        for (size_t k = j + 1; k < runq.dense.size(); k++)
          if (runq.dense[k].second >= 0) release(runq.dense[k].second);
        cut = true;
        matched_ = true;
      } else if (c >= 0 && c < 128 && !p_.ascii.empty()) {
        addit = (p_.ascii[i.arg * 2 + (c >> 6)] >> (c & 63)) & 1;
      } else {
        addit = rune_in(p_.runes[i.arg], c);
      }
      if (addit) t = add2(nextq, i.out, next_pos, t, f1, f2, t);
      if (t >= 0) release(t);
      if (cut) break;
    }
    runq.dense.clear();
  }
};

}  // namespace

bool Regexp::Match(const uint8_t* b, size_t n) const {
  Machine m(prog_, 0);
  return m.run(b, n, 0, (int64_t)n);
}

// regexp's bit-state backtracker (regexp/backtrack.go): depth-first in priority order, so
// the first Match reached from a start position is that start's leftmost-first match, and a
// (pc, pos) pair is expanded at most once per search (a pair that failed fails again from
// any later start), which keeps the search linear in prog size x text span.  Go picks it
// for small programs and inputs; the results equal the Pike VM's.
class Backtracker {
 public:
  explicit Backtracker(const Prog& p, int nslots) : p_(p), ns_(nslots), np_(p.inst.size()) {
    cap_.assign(ns_, -1);
    matchcap_.assign(ns_, -1);
  }
  // budget for the visited bitmap (bits) above which the caller uses the Pike VM
  static constexpr uint64_t kMaxBits = 64ull << 20;
  // Go uses it only for programs of at most 500 instructions (backtrack.go maxBacktrackProg):
  // larger ones (long counted repetitions) visit too many (pc, pos) pairs
  static constexpr size_t kMaxProg = 500;
  bool fits(size_t n, int64_t pos) const {
    return np_ <= kMaxProg && (uint64_t)np_ * (uint64_t)(n - pos + 1) <= kMaxBits;
  }

  // leftmost-first match starting in [pos, start_hi] (rune steps), as Machine::run
  bool run(const uint8_t* b, size_t n, int64_t pos, int64_t start_hi) {
    b_ = b;
    n_ = (int64_t)n;
    base_ = pos;
    maxrow_ = -1;
    bool found = false;
    std::fill(matchcap_.begin(), matchcap_.end(), -1);
    for (int64_t s = pos; s <= n_ && s <= start_hi;) {
      if (!p_.prefix.empty()) {  // a match starts at a prefix occurrence
        const int64_t q = next_prefix(p_, b, n, s);
        if (q < 0 || q > start_hi) break;
        if (q > s && q - base_ > 4096) {  // far jump: restart the visited rows at q
          if (maxrow_ >= 0) {
            const uint64_t hi = ((uint64_t)(maxrow_ + 1) * np_ + 63) / 64;
            std::fill(visited_.begin(), visited_.begin() + std::min<uint64_t>(hi, visited_.size()), 0);
          }
          base_ = q;
          maxrow_ = -1;
        }
        s = q;
      }
      std::fill(cap_.begin(), cap_.end(), -1);
      if (ns_ > 0) cap_[0] = s;
      if (try_at(s)) {
        found = true;
        break;
      }
      if (s == n_) break;
      int w;
      decode_rune(b_, n, (size_t)s, &w);
      s += w;
    }
    // clear the rows touched (only the visited span costs)
    if (maxrow_ >= 0) {
      const uint64_t hi = ((uint64_t)(maxrow_ + 1) * np_ + 63) / 64;
      std::fill(visited_.begin(), visited_.begin() + std::min<uint64_t>(hi, visited_.size()), 0);
    }
    return found;
  }
  const std::vector<int64_t>& matchcap() const { return matchcap_; }

 private:
  struct Job {
    uint32_t pc;
    bool arg;
    int64_t pos;
  };
  const Prog& p_;
  int ns_;
  size_t np_;
  const uint8_t* b_ = nullptr;
  int64_t n_ = 0, base_ = 0, maxrow_ = -1;
  // per-thread visited bitmap, kept all-zero between runs (each run clears what it touched)
  static std::vector<uint64_t>& visited_buf() {
    thread_local std::vector<uint64_t> v;
    return v;
  }
  std::vector<uint64_t>& visited_ = visited_buf();
  std::vector<Job> jobs_;
  std::vector<int64_t> cap_, matchcap_;

  // rows are allocated as the search reaches them (zeroed once, kept zero between runs),
  // so a run costs what it explores, not the rest of the file
  void grow(int64_t row) {
    const size_t need = (size_t)(((uint64_t)(row + 1) * np_ + 63) / 64);
    if (need > visited_.size()) visited_.resize(std::max(need, visited_.size() * 2), 0);
  }
  bool visit(uint32_t pc, int64_t pos) {
    const int64_t row = pos - base_;
    if (row > maxrow_) {
      maxrow_ = row;
      grow(row);
    }
    const uint64_t k = (uint64_t)row * np_ + pc;
    uint64_t& w = visited_[k >> 6];
    const uint64_t bit = 1ull << (k & 63);
    if (w & bit) return false;
    w |= bit;
    return true;
  }
  int32_t before(int64_t pos) const { return pos > 0 ? (int32_t)b_[pos - 1] : kEOT; }
  int32_t at(int64_t pos) const { return pos < n_ ? (int32_t)b_[pos] : kEOT; }

  bool try_at(int64_t start) {
    jobs_.clear();
    jobs_.push_back({p_.start, false, start});
    while (!jobs_.empty()) {
      Job j = jobs_.back();
      jobs_.pop_back();
      uint32_t pc = j.pc;
      int64_t pos = j.pos;
      bool arg = j.arg;
      if (arg) goto skip;
    check:
      if (!visit(pc, pos)) continue;
    skip : {
      const Inst& in = p_.inst[pc];
      switch (in.op) {
        case Op::Fail:
          continue;
        case Op::Alt:
          if (arg) {
            arg = false;
            pc = in.arg;
            goto check;
          }
          jobs_.push_back({pc, true, pos});
          pc = in.out;
          goto check;
        case Op::Rune: {
          if (pos >= n_) continue;
          int w;
          const int32_t c = decode_rune(b_, (size_t)n_, (size_t)pos, &w);
          bool ok;
          if (c >= 0 && c < 128 && !p_.ascii.empty()) ok = (p_.ascii[in.arg * 2 + (c >> 6)] >> (c & 63)) & 1;
          else ok = rune_in(p_.runes[in.arg], c);
          if (!ok) continue;
          pos += w;
          pc = in.out;
          goto check;
        }
        case Op::Cap:
          if (arg) {
            cap_[in.arg] = pos;  // restore
            continue;
          }
          if ((int)in.arg < ns_) {
            jobs_.push_back({pc, true, cap_[in.arg]});
            cap_[in.arg] = pos;
          }
          pc = in.out;
          goto check;
        case Op::Empty:
          if (!empty_ok(in.arg, before(pos), at(pos))) continue;
          pc = in.out;
          goto check;
        case Op::Nop:
          pc = in.out;
          goto check;
        case Op::Match:
          if (ns_ > 1) cap_[1] = pos;
          std::copy(cap_.begin(), cap_.end(), matchcap_.begin());
          return true;
      }
    }
    }
    return false;
  }
};

// The leftmost-first match found from `pos` with whole-match positions only (2 slots: the
// cheap pass), then, for submatches, the same match re-run anchored at its start with every
// slot: the highest-priority thread that starts there ends at the same place, so the two
// passes give exactly the single full pass's result.
struct TwoPass {
  Machine whole, sub;
  Backtracker bt;
  bool submatch;
  int nslots;
  int engine;    // 0 auto, 1 Pike VM only, 2 backtracker where it fits
  int mode = 0;  // which matcher produced the last match: 0 whole, 1 sub, 2 backtracker
  TwoPass(const Prog& p, bool submatch_, int engine_ = 0)
      : whole(p, 2), sub(p, submatch_ ? p.nslots : 2), bt(p, submatch_ ? p.nslots : 2), submatch(submatch_),
        nslots(p.nslots), engine(engine_) {}
  bool run(const uint8_t* b, size_t n, int64_t pos, int64_t start_hi) {
    if (engine != 1 && bt.fits(n, pos) && !(engine == 0 && pike_only())) {
      mode = 2;
      return bt.run(b, n, pos, start_hi);
    }
    mode = 0;
    if (!whole.run(b, n, pos, start_hi)) return false;
    if (submatch && nslots > 2) {
      sub.run(b, n, whole.matchcap()[0], whole.matchcap()[0]);
      mode = 1;
    }
    return true;
  }
  const std::vector<int64_t>& matchcap() const {
    return mode == 2 ? bt.matchcap() : mode == 1 ? sub.matchcap() : whole.matchcap();
  }
  static bool pike_only() {
    const bool v = knobs().pike_only.load() != 0;  // tests: the Pike VM alone ("pike_only" knob)
    return v;
  }
};

void Regexp::FindAll(const uint8_t* b, size_t n, bool submatch, std::vector<int64_t>* out,
                     size_t lo, size_t start_hi, int engine) const {
  // regexp.allMatches (regexp/regexp.go)
  TwoPass m(prog_, submatch, engine);
  int64_t end = (int64_t)n;
  int64_t pos = (int64_t)lo, prev_end = -1;
  int64_t hi = start_hi == SIZE_MAX ? end : (int64_t)std::min<size_t>(start_hi, n);
  while (pos <= end) {
    if (pos > hi) break;
    if (!m.run(b, n, pos, hi)) break;
    const auto& mc = m.matchcap();
    bool accept = true;
    if (mc[1] == pos) {
      if (mc[0] == prev_end) accept = false;
      int w;
      decode_rune(b, n, (size_t)pos, &w);
      pos = w > 0 ? pos + w : end + 1;
    } else {
      pos = mc[1];
    }
    prev_end = mc[1];
    if (accept) {
      if (submatch) out->insert(out->end(), mc.begin(), mc.begin() + prog_.nslots);
      else out->insert(out->end(), mc.begin(), mc.begin() + 2);
    }
  }
}

void Regexp::FindAllWindows(const uint8_t* b, size_t n, bool submatch,
                            const std::vector<std::pair<int64_t, int64_t>>& iv,
                            std::vector<int64_t>* out) const {
  // Go's allMatches iteration, skipping the stretches in which no match can start:
  // `pos` and the previous match end carry from one window to the next, so a match
  // that runs past its window is handled exactly as the global iteration would.
  TwoPass m(prog_, submatch);
  const int64_t end = (int64_t)n;
  int64_t pos = 0, prev_end = -1;
  for (const auto& w : iv) {
    if (pos > end) break;
    if (w.first > pos) pos = w.first;
    const int64_t hi = std::min<int64_t>(w.second, end);
    while (pos <= end && pos <= hi) {
      if (!m.run(b, n, pos, hi)) {
        pos = hi + 1;  // no match starts in [pos, hi]
        break;
      }
      const auto& mc = m.matchcap();
      bool accept = true;
      if (mc[1] == pos) {
        if (mc[0] == prev_end) accept = false;
        int wd;
        decode_rune(b, n, (size_t)pos, &wd);
        pos = wd > 0 ? pos + wd : end + 1;
      } else {
        pos = mc[1];
      }
      prev_end = mc[1];
      if (accept) {
        if (submatch) out->insert(out->end(), mc.begin(), mc.begin() + prog_.nslots);
        else out->insert(out->end(), mc.begin(), mc.begin() + 2);
      }
    }
  }
}

}  // namespace tsg
