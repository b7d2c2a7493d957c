"""Go 1.19 Unicode semantics used by the secret path (oracle restatement).

Go 1.19 ships Unicode 13.0.0 tables; Python 3.10's `unicodedata` is 13.0.0 too,
so the tables below are derived from it.

* `fold_orbit(r)`   -- the `unicode.SimpleFold` orbit of r (used by regexp (?i)).
* `simple_lower(r)` -- `unicode.ToLower` (simple mapping) used by `bytes.ToLower`.
* `go_to_lower(b)`  -- `bytes.ToLower` (bytes/bytes.go: ASCII fast path, else
                       `Map(unicode.ToLower, s)` where an invalid byte decodes to
                       U+FFFD and is re-encoded as EF BF BD).
* `decode_runes(b)` -- `utf8.DecodeRune` segmentation: (rune, width) pairs.
* `category_ranges(name)` -- `\\pX` tables.
"""
import functools
import sys
import unicodedata

MAX_RUNE = 0x10FFFF
RUNE_ERROR = 0xFFFD

# Go excludes the Turkic dotted/dotless I from simple folding orbits
# (CaseFolding.txt status T only), so they fold to nothing but themselves.
_NO_FOLD = {0x130, 0x131}


@functools.lru_cache(maxsize=1)
def _orbits():
    parent = {}

    def find(x):
        while parent.get(x, x) != x:
            parent[x] = parent.get(parent[x], parent[x])
            x = parent[x]
        return x

    def union(a, b):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)

    for cp in range(MAX_RUNE + 1):
        if 0xD800 <= cp <= 0xDFFF or cp in _NO_FOLD:
            continue
        c = chr(cp)
        for m in (c.casefold(), c.lower()):
            if len(m) == 1 and m != c and ord(m) not in _NO_FOLD:
                union(cp, ord(m))
    groups = {}
    members = set(parent.keys()) | set(parent.values())
    for cp in members:
        groups.setdefault(find(cp), set()).add(cp)
    orbit = {}
    for g in groups.values():
        if len(g) > 1:
            t = tuple(sorted(g))
            for cp in g:
                orbit[cp] = t
    return orbit


def fold_orbit(r):
    """All runes equivalent to r under Go's SimpleFold (sorted, includes r)."""
    return _orbits().get(r, (r,))


def simple_lower(r):
    if r == 0x130:
        return 0x69  # UnicodeData simple lowercase of U+0130 is U+0069
    if 0xD800 <= r <= 0xDFFF:
        return r
    m = chr(r).lower()
    return ord(m) if len(m) == 1 else r


def decode_rune(b, i):
    """utf8.DecodeRune(b[i:]) -> (rune, width). Invalid -> (U+FFFD, 1)."""
    n = len(b)
    c0 = b[i]
    if c0 < 0x80:
        return c0, 1
    if 0xC2 <= c0 <= 0xDF:
        if i + 1 < n and 0x80 <= b[i + 1] <= 0xBF:
            return ((c0 & 0x1F) << 6) | (b[i + 1] & 0x3F), 2
        return RUNE_ERROR, 1
    if 0xE0 <= c0 <= 0xEF:
        lo, hi = 0x80, 0xBF
        if c0 == 0xE0:
            lo = 0xA0
        elif c0 == 0xED:
            hi = 0x9F
        if i + 2 < n and lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF:
            return ((c0 & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F), 3
        return RUNE_ERROR, 1
    if 0xF0 <= c0 <= 0xF4:
        lo, hi = 0x80, 0xBF
        if c0 == 0xF0:
            lo = 0x90
        elif c0 == 0xF4:
            hi = 0x8F
        if (i + 3 < n and lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF
                and 0x80 <= b[i + 3] <= 0xBF):
            return (((c0 & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12)
                    | ((b[i + 2] & 0x3F) << 6) | (b[i + 3] & 0x3F)), 4
        return RUNE_ERROR, 1
    return RUNE_ERROR, 1


def go_to_lower(b):
    """bytes.ToLower (Go 1.19 bytes/bytes.go)."""
    if all(c < 0x80 for c in b):
        return b.lower()
    out = []
    i = 0
    n = len(b)
    while i < n:
        r, w = decode_rune(b, i)
        out.append(chr(simple_lower(r)))
        i += w
    return "".join(out).encode("utf-8", "surrogatepass")


@functools.lru_cache(maxsize=None)
def category_ranges(name):
    """Ranges for \\p{name} where name is a general category (L, Lu, N, ...)."""
    ranges = []
    start = None
    for cp in range(MAX_RUNE + 2):
        ok = False
        if cp <= MAX_RUNE:
            cat = unicodedata.category(chr(cp))
            # Go's one-letter tables are unions of the assigned two-letter ones (no Cn)
            ok = cat == name or (len(name) == 1 and cat[0] == name and cat != "Cn")
        if ok and start is None:
            start = cp
        elif not ok and start is not None:
            ranges.append((start, cp - 1))
            start = None
    return ranges


CATEGORIES = {"C", "Cc", "Cf", "Co", "Cs", "L", "Ll", "Lm", "Lo", "Lt", "Lu", "M", "Mc",
              "Me", "Mn", "N", "Nd", "Nl", "No", "P", "Pc", "Pd", "Pe", "Pf", "Pi", "Po",
              "Ps", "S", "Sc", "Sk", "Sm", "So", "Z", "Zl", "Zp", "Zs"}

if sys.maxunicode < MAX_RUNE:  # pragma: no cover
    raise RuntimeError("narrow Python build")
