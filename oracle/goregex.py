"""Go 1.19 `regexp` restated on top of Python's `regex` engine (oracle only).

The reference compiles every rule with `regexp.Compile` (Perl flags:
ClassNL | OneLine | PerlX | UnicodeGroups) -- `pkg/fanal/secret/scanner.go:64-81`.
Python's regex dialect differs from Go's in the ways SURVEY.md Appendix A lists
(\\s/\\d/\\w/\\b are Unicode, `$` also matches before a final newline, mid-pattern
flags, case folding tables, duplicate group names, invalid UTF-8, the FindAll
empty-match rule).  So this module does not hand Go syntax to Python: it parses
the Go syntax itself (a restatement of regexp/syntax/parse.go), applies Go's
own case folding and class semantics, and emits a Python pattern in which every
character set is an explicit list of code-point ranges, every capture is a plain
numbered group in Go's order, and every empty-width assertion is an explicit
look-around.  No Python flag is ever used.

Text is decoded with `surrogateescape`, which yields exactly one code point per
invalid byte, as Go's `utf8.DecodeRune` yields one U+FFFD of width 1 (a class
that names U+FFFD explicitly would differ -- no rule does).  Offsets are mapped
back to bytes.
"""
import regex as _pyre

from . import gounicode as U

MAX = U.MAX_RUNE


class GoRegexpError(ValueError):
    pass


# ---------------------------------------------------------------- char sets
def _clean(ranges):
    rs = sorted(ranges)
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + 1:
            if hi > out[-1][1]:
                out[-1] = (out[-1][0], hi)
        else:
            out.append((lo, hi))
    return out


def _negate(ranges):
    out = []
    nxt = 0
    for lo, hi in _clean(ranges):
        if lo > nxt:
            out.append((nxt, lo - 1))
        nxt = hi + 1
    if nxt <= MAX:
        out.append((nxt, MAX))
    return out


def _fold_ranges(ranges):
    """appendFoldedRange (regexp/syntax/parse.go): add every SimpleFold orbit member."""
    out = list(ranges)
    orbit_table = U._orbits()
    for lo, hi in ranges:
        if hi - lo > 0x3000:
            # scan only the runes that have orbits
            for cp, orb in orbit_table.items():
                if lo <= cp <= hi:
                    out.extend((o, o) for o in orb)
        else:
            for cp in range(lo, hi + 1):
                orb = orbit_table.get(cp)
                if orb:
                    out.extend((o, o) for o in orb)
    return _clean(out)


PERL = {
    "d": [(0x30, 0x39)],
    "s": [(0x09, 0x0A), (0x0C, 0x0D), (0x20, 0x20)],
    "w": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
}
POSIX = {
    "alnum": [(0x30, 0x39), (0x41, 0x5A), (0x61, 0x7A)],
    "alpha": [(0x41, 0x5A), (0x61, 0x7A)],
    "ascii": [(0x00, 0x7F)],
    "blank": [(0x09, 0x09), (0x20, 0x20)],
    "cntrl": [(0x00, 0x1F), (0x7F, 0x7F)],
    "digit": [(0x30, 0x39)],
    "graph": [(0x21, 0x7E)],
    "lower": [(0x61, 0x7A)],
    "print": [(0x20, 0x7E)],
    "punct": [(0x21, 0x2F), (0x3A, 0x40), (0x5B, 0x60), (0x7B, 0x7E)],
    "space": [(0x09, 0x0D), (0x20, 0x20)],
    "upper": [(0x41, 0x5A)],
    "word": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
    "xdigit": [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66)],
}

FOLD, DOTNL, ONELINE, NONGREEDY = 1, 2, 4, 8
PERL_FLAGS = ONELINE  # ClassNL|PerlX|UnicodeGroups are always on; OneLine is the toggleable one


# ---------------------------------------------------------------- parser
class _Parser:
    def __init__(self, src):
        self.s = src
        self.i = 0
        self.flags = PERL_FLAGS
        self.ncap = 0
        self.names = [""]

    def peek(self, k=0):
        j = self.i + k
        return self.s[j] if j < len(self.s) else None

    def err(self, msg):
        raise GoRegexpError("error parsing regexp: %s: `%s`" % (msg, self.s))

    def parse(self):
        node = self.parse_alt()
        if self.i != len(self.s):
            self.err("unexpected )")
        return node

    def parse_alt(self):
        alts = [self.parse_concat()]
        while self.peek() == "|":
            self.i += 1
            alts.append(self.parse_concat())
        return alts[0] if len(alts) == 1 else ("alt", alts)

    def parse_concat(self):
        items = []
        while True:
            c = self.peek()
            if c is None or c == "|" or c == ")":
                break
            atom = self.parse_atom()
            if atom is None:
                continue
            atom = self.parse_repeat(atom)
            items.append(atom)
        if not items:
            return ("empty",)
        return items[0] if len(items) == 1 else ("cat", items)

    def parse_repeat(self, atom):
        last_was_rep = False
        while True:
            c = self.peek()
            start = self.i
            if c in ("*", "+", "?"):
                self.i += 1
                lo, hi = {"*": (0, -1), "+": (1, -1), "?": (0, 1)}[c]
            elif c == "{":
                r = self._try_braces()
                if r is None:
                    return atom
                lo, hi = r
            else:
                return atom
            if last_was_rep:
                self.err("invalid nested repetition operator: `%s`" % self.s[rep_start:self.i])
            greedy = True
            if self.peek() == "?":
                self.i += 1
                greedy = False
            if self.flags & NONGREEDY:
                greedy = not greedy
            if atom[0] == "empty_marker":
                self.err("missing argument to repetition operator")
            atom = ("rep", lo, hi, greedy, atom)
            last_was_rep = True
            rep_start = start

    def _try_braces(self):
        # {n} {n,} {n,m}; anything else is a literal '{'
        s, j = self.s, self.i + 1

        def digits(j):
            k = j
            while k < len(s) and s[k].isdigit() and s[k] < "\x80":
                k += 1
            return k

        k = digits(j)
        if k == j:
            return None
        lo = int(s[j:k])
        j = k
        hi = lo
        if j < len(s) and s[j] == ",":
            j += 1
            if j < len(s) and s[j] == "}":
                hi = -1
            else:
                k = digits(j)
                if k == j:
                    return None
                hi = int(s[j:k])
                j = k
        if j >= len(s) or s[j] != "}":
            return None
        self.i = j + 1
        if lo > 1000 or hi > 1000 or (hi >= 0 and hi < lo):
            self.err("invalid repeat count")
        return lo, hi

    def parse_atom(self):
        c = self.peek()
        if c == "(":
            return self.parse_group()
        if c == "[":
            return ("class", self.parse_class())
        if c in "*+?":
            self.err("missing argument to repetition operator: `%s`" % c)
        if c == ".":
            self.i += 1
            return ("any",) if self.flags & DOTNL else ("anynotnl",)
        if c == "^":
            self.i += 1
            return ("bot",) if self.flags & ONELINE else ("bol",)
        if c == "$":
            self.i += 1
            return ("eot",) if self.flags & ONELINE else ("eol",)
        if c == "\\":
            return self.parse_backslash()
        self.i += 1
        return self.literal(ord(c))

    def literal(self, r):
        return ("lit", r, bool(self.flags & FOLD))

    def parse_group(self):
        s = self.s
        self.i += 1
        saved = self.flags
        if s.startswith("?P<", self.i) or s.startswith("?P=", self.i):
            if s.startswith("?P=", self.i):
                self.err("invalid named capture")
            end = s.find(">", self.i)
            if end < 0:
                self.err("invalid named capture")
            name = s[self.i + 3:end]
            if not name or not all(ch.isalnum() or ch == "_" for ch in name) or not name.isascii():
                self.err("invalid named capture")
            self.i = end + 1
            self.ncap += 1
            idx = self.ncap
            self.names.append(name)
            sub = self.parse_alt()
            self._close()
            self.flags = saved
            return ("cap", idx, sub)
        if self.peek() == "?":
            # flags: (?flags) or (?flags:re)
            j = self.i + 1
            neg = False
            sawflag = False
            flags = self.flags
            while True:
                if j >= len(s):
                    self.err("missing closing )")
                ch = s[j]
                if ch == "i":
                    flags = (flags & ~FOLD) if neg else (flags | FOLD)
                    sawflag = True
                elif ch == "m":
                    flags = (flags | ONELINE) if neg else (flags & ~ONELINE)
                    sawflag = True
                elif ch == "s":
                    flags = (flags & ~DOTNL) if neg else (flags | DOTNL)
                    sawflag = True
                elif ch == "U":
                    flags = (flags & ~NONGREEDY) if neg else (flags | NONGREEDY)
                    sawflag = True
                elif ch == "-":
                    if neg:
                        self.err("invalid or unsupported Perl syntax")
                    neg = True
                    sawflag = False
                elif ch == ")" or ch == ":":
                    if (neg and not sawflag) or (j == self.i + 1):
                        if not (ch == ":" and j == self.i + 1):
                            self.err("invalid or unsupported Perl syntax")
                    break
                else:
                    self.err("invalid or unsupported Perl syntax")
                j += 1
            self.i = j + 1
            if ch == ")":
                # flags persist until the enclosing group closes
                self.flags = flags
                return None
            self.flags = flags
            sub = self.parse_alt()
            self._close()
            self.flags = saved
            return ("group", sub)
        self.ncap += 1
        idx = self.ncap
        self.names.append("")
        sub = self.parse_alt()
        self._close()
        self.flags = saved
        return ("cap", idx, sub)

    def _close(self):
        if self.peek() != ")":
            self.err("missing closing )")
        self.i += 1

    # -- escapes
    def parse_backslash(self):
        s = self.s
        nxt = self.peek(1)
        if nxt is None:
            self.err("trailing backslash at end of expression")
        if nxt == "A":
            self.i += 2
            return ("bot",)
        if nxt == "z":
            self.i += 2
            return ("eot",)
        if nxt == "b":
            self.i += 2
            return ("wb",)
        if nxt == "B":
            self.i += 2
            return ("nwb",)
        if nxt == "Q":
            end = s.find("\\E", self.i + 2)
            lit = s[self.i + 2:] if end < 0 else s[self.i + 2:end]
            self.i = len(s) if end < 0 else end + 2
            items = [self.literal(ord(ch)) for ch in lit]
            if not items:
                return None
            return items[0] if len(items) == 1 else ("cat", items)
        if nxt in "pP":
            return ("class", self.parse_unicode_class())
        if nxt in "dDsSwW":
            self.i += 2
            return ("class", self.perl_group(nxt))
        r = self.parse_escape()
        return self.literal(r)

    def perl_group(self, ch):
        base = PERL[ch.lower()]
        if self.flags & FOLD:
            base = _fold_ranges(base)
        return _negate(base) if ch.isupper() else _clean(base)

    def parse_unicode_class(self):
        s = self.s
        sign = -1 if s[self.i + 1] == "P" else 1
        j = self.i + 2
        if j >= len(s):
            self.err("invalid character class range")
        if s[j] == "{":
            end = s.find("}", j)
            if end < 0:
                self.err("invalid character class range")
            name = s[j + 1:end]
            self.i = end + 1
        else:
            name = s[j]
            self.i = j + 1
        if name.startswith("^"):
            sign = -sign
            name = name[1:]
        if name == "Any":
            rs = [(0, MAX)]
        elif name in U.CATEGORIES:
            rs = list(U.category_ranges(name))
        else:
            self.err("invalid character class range (unsupported in oracle: %s)" % name)
        if self.flags & FOLD:
            rs = _fold_ranges(rs)
        return _negate(rs) if sign < 0 else _clean(rs)

    def parse_escape(self):
        """regexp/syntax parseEscape: returns a rune, advances past it."""
        s = self.s
        self.i += 1  # backslash
        c = s[self.i]
        self.i += 1
        if "1" <= c <= "7":
            if not (self.peek() is not None and "0" <= self.peek() <= "7"):
                self.err("invalid escape sequence: `\\%s`" % c)
        if "0" <= c <= "7":
            r = ord(c) - 48
            for _ in range(2):
                d = self.peek()
                if d is not None and "0" <= d <= "7":
                    r = r * 8 + ord(d) - 48
                    self.i += 1
                else:
                    break
            return r
        if c == "x":
            if self.peek() == "{":
                end = s.find("}", self.i)
                if end < 0:
                    self.err("invalid escape sequence")
                h = s[self.i + 1:end]
                try:
                    r = int(h, 16)
                except ValueError:
                    self.err("invalid escape sequence")
                if not h or r > MAX:
                    self.err("invalid escape sequence")
                self.i = end + 1
                return r
            h = s[self.i:self.i + 2]
            if len(h) < 2 or any(ch not in "0123456789abcdefABCDEF" for ch in h):
                self.err("invalid escape sequence")
            self.i += 2
            return int(h, 16)
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if c in simple:
            return simple[c]
        if ord(c) < 0x80 and not c.isalnum():
            return ord(c)
        self.err("invalid escape sequence: `\\%s`" % c)

    # -- classes
    def parse_class(self):
        s = self.s
        self.i += 1
        sign = 1
        if self.peek() == "^":
            sign = -1
            self.i += 1
        ranges = []
        first = True
        while self.peek() != "]" or first:
            if self.peek() is None:
                self.err("missing closing ]")
            first = False
            if s.startswith("[:", self.i):
                end = s.find(":]", self.i + 2)
                if end >= 0:
                    name = s[self.i + 2:end]
                    neg = name.startswith("^")
                    if neg:
                        name = name[1:]
                    if name not in POSIX:
                        self.err("invalid character class range")
                    rs = POSIX[name]
                    if self.flags & FOLD:
                        rs = _fold_ranges(rs)
                    ranges.extend(_negate(rs) if neg else rs)
                    self.i = end + 2
                    continue
            if self.peek() == "\\" and self.peek(1) in ("p", "P"):
                ranges.extend(self.parse_unicode_class())
                continue
            if self.peek() == "\\" and self.peek(1) is not None and self.peek(1) in "dDsSwW":
                ranges.extend(self.perl_group(self.peek(1)))
                self.i += 2
                continue
            lo = self.class_char()
            hi = lo
            if self.peek() == "-" and self.peek(1) is not None and self.peek(1) != "]":
                self.i += 1
                hi = self.class_char()
                if hi < lo:
                    self.err("invalid character class range")
            if self.flags & FOLD:
                ranges.extend(_fold_ranges([(lo, hi)]))
            else:
                ranges.append((lo, hi))
        self.i += 1
        ranges = _clean(ranges)
        return _negate(ranges) if sign < 0 else ranges

    def class_char(self):
        c = self.peek()
        if c is None:
            self.err("missing closing ]")
        if c == "\\":
            return self.parse_escape()
        self.i += 1
        return ord(c)


# ---------------------------------------------------------------- emitter
def _esc(cp):
    return "\\U%08x" % cp


def _emit_set(ranges):
    if not ranges:
        return "(?!)"
    parts = []
    for lo, hi in ranges:
        parts.append(_esc(lo) if lo == hi else _esc(lo) + "-" + _esc(hi))
    return "[" + "".join(parts) + "]"


_W = "[0-9A-Za-z_]"


def _emit(node):
    k = node[0]
    if k == "lit":
        r, fold = node[1], node[2]
        if fold:
            orb = U.fold_orbit(r)
            if len(orb) > 1:
                return _emit_set(_clean([(o, o) for o in orb]))
        return _esc(r)
    if k == "class":
        return _emit_set(node[1])
    if k == "any":
        return "[\\U00000000-\\U0010ffff]"
    if k == "anynotnl":
        return "[^\\n]"
    if k == "bot":
        return "(?<![\\U00000000-\\U0010ffff])"
    if k == "eot":
        return "(?![\\U00000000-\\U0010ffff])"
    if k == "bol":
        return "(?:(?<![\\U00000000-\\U0010ffff])|(?<=\\n))"
    if k == "eol":
        return "(?:(?![\\U00000000-\\U0010ffff])|(?=\\n))"
    if k == "wb":
        return "(?:(?<=%s)(?!%s)|(?<!%s)(?=%s))" % (_W, _W, _W, _W)
    if k == "nwb":
        return "(?:(?<=%s)(?=%s)|(?<!%s)(?!%s))" % (_W, _W, _W, _W)
    if k == "empty":
        return ""
    if k == "cap":
        return "(" + _emit(node[2]) + ")"
    if k == "group":
        return "(?:" + _emit(node[1]) + ")"
    if k == "cat":
        return "".join("(?:" + _emit(x) + ")" if x[0] == "alt" else _emit(x) for x in node[1])
    if k == "alt":
        return "(?:" + "|".join(_emit(x) for x in node[1]) + ")"
    if k == "rep":
        lo, hi, greedy, sub = node[1], node[2], node[3], node[4]
        if lo == 0 and hi == -1:
            q = "*"
        elif lo == 1 and hi == -1:
            q = "+"
        elif lo == 0 and hi == 1:
            q = "?"
        elif hi == -1:
            q = "{%d,}" % lo
        elif lo == hi:
            q = "{%d}" % lo
        else:
            q = "{%d,%d}" % (lo, hi)
        if not greedy:
            q += "?"
        return "(?:" + _emit(sub) + ")" + q
    raise AssertionError(node)


# ---------------------------------------------------------------- text mapping
class _Text:
    """Decoded text + char-index -> byte-offset map."""

    __slots__ = ("s", "off", "nbytes")

    def __init__(self, b):
        self.nbytes = len(b)
        if b.isascii():
            self.s = b.decode("ascii")
            self.off = None
        else:
            self.s = b.decode("utf-8", "surrogateescape")
            off = [0] * (len(self.s) + 1)
            o = 0
            for k, ch in enumerate(self.s):
                off[k] = o
                cp = ord(ch)
                if 0xDC80 <= cp <= 0xDCFF:
                    o += 1
                elif cp < 0x80:
                    o += 1
                elif cp < 0x800:
                    o += 2
                elif cp < 0x10000:
                    o += 3
                else:
                    o += 4
            off[len(self.s)] = o
            self.off = off

    def b(self, k):
        if k < 0:
            return -1
        return k if self.off is None else self.off[k]


def _as_bytes(x):
    if isinstance(x, str):
        return x.encode("utf-8", "surrogateescape")
    return bytes(x)


class GoRegexp:
    """The subset of Go's *regexp.Regexp API used on the secret path."""

    def __init__(self, src):
        p = _Parser(src)
        ast = p.parse()
        self.src = src
        self.names = p.names
        self.ncap = p.ncap
        self.py_pattern = _emit(ast)
        try:
            self._re = _pyre.compile(self.py_pattern, _pyre.V0)
        except Exception as e:  # pragma: no cover
            raise GoRegexpError("oracle translation failed for %r: %s" % (src, e))

    def __repr__(self):
        return "GoRegexp(%r)" % self.src

    def SubexpNames(self):
        return list(self.names)

    def MatchString(self, s):
        return self._re.search(_Text(_as_bytes(s)).s) is not None

    def _all(self, b, n=-1):
        """regexp.allMatches (regexp/regexp.go): Go's FindAll iteration."""
        t = _Text(_as_bytes(b))
        s = t.s
        end = len(s)
        pos = 0
        prev_end = -1
        out = []
        while (n < 0 or len(out) < n) and pos <= end:
            m = self._re.search(s, pos)
            if m is None:
                break
            accept = True
            if m.end() == pos:
                if m.start() == prev_end:
                    accept = False
                pos = pos + 1 if pos < end else end + 1
            else:
                pos = m.end()
            prev_end = m.end()
            if accept:
                spans = []
                for g in range(self.ncap + 1):
                    a, z = m.span(g)
                    spans.append(t.b(a))
                    spans.append(t.b(z))
                out.append(spans)
        return out

    def FindAllIndex(self, b, n=-1):
        return [m[:2] for m in self._all(b, n)]

    def FindAllSubmatchIndex(self, b, n=-1):
        return self._all(b, n)


def MustCompile(src):
    return GoRegexp(src)
