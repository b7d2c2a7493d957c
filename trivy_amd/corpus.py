"""Seeded synthetic corpora for the secret-scan benchmarks and parity tests.

Not part of the scanning path: it produces BASELINE.json-shaped inputs (mixed
code/config text files, log-normal sizes with median ~6 KiB, planted secrets for
every builtin rule plus near misses, CRLF lines, long lines, multi-line PEM keys,
valid non-ASCII UTF-8, invalid bytes and the U+017F / U+212A folding runes) as one
packed byte stream + offsets + paths (trivy_amd.secret.Batch).

Text is sampled once into a base buffer from a vocabulary that includes the common
builtin keywords (key, sk, account, -----, lob, live_, pk., sg., ...), then tiled, so
generating 10 GiB is a memcpy-speed operation.
"""
import sre_parse
import warnings

import numpy as np

from .secret import Batch, builtin_rules

VOCAB = (
    "the a of to in is for on with as by at from it this that be are was not or and if else "
    "return def class import func var let const int str bool true false null None self new "
    "public private static void main print log error warn info debug value values name id "
    "data result results config settings options path file files dir url host port user "
    "users password token tokens secret secrets key keys api apikey access account accounts "
    "task tasks ask disk risk skip desk global blob lobby public_key pk. sg. msg. live_ "
    "test test_ example vendor buffer index item items list map dict set get put post "
    "request response client server http https json yaml xml html css js go py rs java "
    "for while break continue try catch except finally raise throw async await yield "
    "linear matrix vector hash sha256 md5 base64 encode decode encrypt decrypt cipher "
    "aws gcp azure cloud storage bucket region queue cache redis postgres mysql docker "
    "kubernetes deploy build release version commit branch merge SK "
    "----- ===== ##### // /* */ # -- ; { } ( ) [ ] < > => := = == != += -= && || "
    "0 1 2 3 42 100 1024 0x1f 3.14 2023-01-01 localhost 127.0.0.1 /usr/local/bin "
    "café naïve résumé über 日本語 中文 Ελληνικά кириллица emoji😀 ✓"
).split()


def _sample(node_list, rng, out):
    for op, av in node_list:
        name = str(op)
        if name == "LITERAL":
            out.append(chr(av))
        elif name == "NOT_LITERAL":
            c = chr(av)
            out.append("x" if c != "x" else "y")
        elif name == "ANY":
            out.append(rng.choice(list("abcxyz012 ")))
        elif name == "IN":
            chars = []
            neg = False
            for o2, a2 in av:
                n2 = str(o2)
                if n2 == "NEGATE":
                    neg = True
                elif n2 == "LITERAL":
                    chars.append(chr(a2))
                elif n2 == "RANGE":
                    chars.extend(chr(c) for c in range(a2[0], min(a2[1], 0x7E) + 1))
                elif n2 == "CATEGORY":
                    cat = str(a2)
                    if "DIGIT" in cat:
                        chars.extend("0123456789")
                    elif "SPACE" in cat:
                        chars.extend(" ")
                    elif "WORD" in cat:
                        chars.extend("abcXYZ019_")
            if neg:
                pool = [c for c in "abcdefghij0123456789 =:" if c not in chars] or ["#"]
                out.append(rng.choice(pool))
            else:
                out.append(rng.choice(chars or ["a"]))
        elif name == "BRANCH":
            _sample(av[1][rng.integers(len(av[1]))], rng, out)
        elif name == "SUBPATTERN":
            _sample(av[-1], rng, out)
        elif name in ("MAX_REPEAT", "MIN_REPEAT"):
            lo, hi, sub = av
            hi = lo + 3 if hi == sre_parse.MAXREPEAT else hi
            n = int(rng.integers(lo, hi + 1)) if hi > lo else lo
            if lo >= 8:
                n = lo + int(rng.integers(0, max(1, min(hi, lo + 4) - lo + 1)))
            for _ in range(n):
                _sample(sub, rng, out)
        elif name == "AT":
            pass
        elif name == "CATEGORY":
            out.append("0")
        else:  # pragma: no cover
            raise ValueError(name)


def sample_secret(regex, rng):
    """A string drawn from (a Python reading of) a rule regex; ASCII only."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        tree = sre_parse.parse(regex)
    out = []
    _sample(list(tree), rng, out)
    return "".join(out)


def _base_text(nbytes, rng):
    toks = [t.encode() for t in VOCAB]
    maxl = max(len(t) for t in toks)
    table = np.zeros((len(toks), maxl), dtype=np.uint8)
    lens = np.array([len(t) for t in toks])
    for i, t in enumerate(toks):
        table[i, :len(t)] = np.frombuffer(t, dtype=np.uint8)
    p = 1.0 / np.arange(1, len(toks) + 1) ** 0.6
    rng.shuffle(p)
    p /= p.sum()
    ntok = nbytes // 6 + 16
    ids = rng.choice(len(toks), size=ntok, p=p)
    seps = rng.choice(np.frombuffer(b"       ...,:;=()\n\n\n\"'\t", dtype=np.uint8), size=ntok)
    g = table[ids]
    mask = np.arange(maxl)[None, :] < lens[ids][:, None]
    body = np.concatenate([g, seps[:, None]], axis=1)
    mask = np.concatenate([mask, np.ones((ntok, 1), dtype=bool)], axis=1)
    text = body[mask]
    # ~10% of the newlines become CRLF
    nl = np.flatnonzero(text == 10)
    crlf = nl[rng.random(len(nl)) < 0.1]
    if len(crlf):
        text = np.insert(text, crlf, 13)
    return text[:nbytes]


# The three runes that change keyword gates or (?i) matching:
# U+017F (s under (?i)), U+212A (k under (?i); bytes.ToLower -> 'k'), U+0130
# (bytes.ToLower -> 'i').  Each line is planted whole, so some are real findings.
FOLD_PLANTS = [
    "ſecret=\"abcdefgh12\" KEY",
    "aws_secret_access_\u212aey = \"12ASD34qwe56CXZ78tyH10Tna543VBokN85RHCas\"",
    "A\u0130DA token \u0130ntercom_api_token = \"" + "b" * 60 + "\"",
    "\u212aEY=\"9f8e7d6c5b4a39281706\" aws_account_id: 1234-5678-9012",
]

FOLD = {ord("k"): "\u212a", ord("K"): "\u212a", ord("s"): "\u017f", ord("S"): "\u017f",
        ord("i"): "\u0130", ord("I"): "\u0130"}

EXTS = ["go", "py", "js", "ts", "yaml", "json", "sh", "env", "tf", "ini", "txt", "conf", "rb",
        "java", "md"]
DIRS = ["src", "pkg", "lib", "app", "cmd", "internal", "config", "deploy", "scripts", "web",
        "test", "vendor", "examples", "docs", "tools"]


def make_corpus(total_bytes, seed=1, plants_per_mib=1.0, median=6 * 1024, sigma=1.2,
                min_size=10, max_size=2 * 1024 * 1024, base_bytes=None, special=True,
                extra_plants=None, extra_per_mib=0.0, binary_frac=0.0):
    """Return (Batch, info).  Deterministic in `seed`.

    extra_plants / extra_per_mib: lines (e.g. configs.plant_lines of a user rule set) planted
    at that rate on top of the builtin plants (configs[3]).  binary_frac: that fraction of
    the files becomes random bytes behind a text-looking first 300 bytes, i.e. binary blobs
    that pass utils.IsBinary and reach Scan (configs[4])."""
    rng = np.random.default_rng(seed)
    base_bytes = base_bytes or int(min(total_bytes, 64 << 20))
    base = _base_text(base_bytes, rng)
    # file sizes
    sizes = []
    acc = 0
    while acc < total_bytes:
        n = int(rng.lognormal(np.log(median), sigma, size=4096).clip(min_size, max_size)[0])
        chunk = rng.lognormal(np.log(median), sigma, size=4096).clip(min_size, max_size).astype(np.int64)
        cs = np.cumsum(chunk)
        k = int(np.searchsorted(cs, total_bytes - acc)) + 1
        sizes.append(chunk[:k])
        acc += int(cs[min(k, len(cs)) - 1])
        del n
    sizes = np.concatenate(sizes)
    sizes[-1] -= max(0, int(sizes.sum()) - total_bytes)
    sizes = sizes[sizes > 0]
    nfiles = len(sizes)
    offsets = np.zeros(nfiles + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offsets[1:])
    total = int(offsets[-1])
    reps = -(-total // len(base))
    start = int(rng.integers(0, len(base)))
    data = np.empty(total + 16, dtype=np.uint8)
    pos = 0
    src = np.concatenate([base[start:], base[:start]])
    for _ in range(reps):
        n = min(len(src), total - pos)
        data[pos:pos + n] = src[:n]
        pos += n
        if pos >= total:
            break
    data[total:] = 0
    # plants: one valid sample of every builtin rule, round-robin, plus near misses
    rules, _ = builtin_rules()
    nplants = max(len(rules), int(plants_per_mib * total / (1 << 20)))
    pfiles = rng.integers(0, nfiles, size=nplants)
    planted = 0
    for i in range(nplants):
        f = int(pfiles[i])
        fs, fe = int(offsets[f]), int(offsets[f + 1])
        r = rules[i % len(rules)]
        s = sample_secret(r.Regex, rng)
        if i % 5 == 4:  # near miss: truncate the secret part
            s = s[: max(1, len(s) - 3)]
        line = ("\n" + s + "\n").encode()
        if fe - fs < len(line) + 1:
            continue
        at = fs + int(rng.integers(0, fe - fs - len(line)))
        data[at:at + len(line)] = np.frombuffer(line, dtype=np.uint8)
        planted += 1
    if extra_plants:
        nx = int(extra_per_mib * total / (1 << 20))
        xf = rng.integers(0, nfiles, size=nx)
        for i in range(nx):
            f = int(xf[i])
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            line = ("\n" + extra_plants[i % len(extra_plants)] + "\n").encode()
            if fe - fs < len(line) + 1:
                continue
            at = fs + int(rng.integers(0, fe - fs - len(line)))
            data[at:at + len(line)] = np.frombuffer(line, dtype=np.uint8)
            planted += 1
    if binary_frac:
        for f in np.flatnonzero(rng.random(nfiles) < binary_frac):
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            if fe - fs > 300:
                data[fs + 300:fe] = rng.integers(0, 256, size=fe - fs - 300, dtype=np.uint8)
    if special and nfiles > 100:
        # invalid bytes (0.1%), folding runes (0.01%), long lines (5%), PEM blocks (0.5%)
        for f in rng.choice(nfiles, size=max(1, nfiles // 1000), replace=False):
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            if fe - fs > 4:
                data[fs + int(rng.integers(0, fe - fs))] = int(rng.integers(0x80, 0x100))
        for k, f in enumerate(rng.choice(nfiles, size=max(3, nfiles // 10000), replace=False)):
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            w = FOLD_PLANTS[k % len(FOLD_PLANTS)].encode()
            if fe - fs > len(w) + 2:
                at = fs + int(rng.integers(0, fe - fs - len(w)))
                data[at:at + len(w)] = np.frombuffer(w, dtype=np.uint8)
        pem = ("-----BEGIN RSA PRIVATE KEY-----\n" + "\n".join(
            "".join(rng.choice(list("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"),
                               size=64)) for _ in range(8)) + "\n-----END RSA PRIVATE KEY-----\n").encode()
        for f in rng.choice(nfiles, size=max(1, nfiles // 200), replace=False):
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            if fe - fs > len(pem) + 2:
                at = fs + int(rng.integers(0, fe - fs - len(pem)))
                data[at:at + len(pem)] = np.frombuffer(pem, dtype=np.uint8)
        for f in rng.choice(nfiles, size=max(1, nfiles // 20), replace=False):
            fs, fe = int(offsets[f]), int(offsets[f + 1])
            if fe - fs > 300:
                at = fs + int(rng.integers(0, fe - fs - 250))
                seg = data[at:at + 250]
                seg[seg == 10] = 32
    # paths
    d = rng.integers(0, len(DIRS), size=nfiles)
    d2 = rng.integers(0, len(DIRS), size=nfiles)
    e = rng.integers(0, len(EXTS), size=nfiles)
    pb = [("%s/%s/f%d.%s" % (DIRS[a], DIRS[b], i, EXTS[c])).encode()
          for i, (a, b, c) in enumerate(zip(d, d2, e))]
    plen = np.array([len(x) for x in pb], dtype=np.uint64)
    poffs = np.zeros(nfiles + 1, dtype=np.uint64)
    np.cumsum(plen, out=poffs[1:])
    paths = np.frombuffer(b"".join(pb), dtype=np.uint8)
    batch = Batch(data, offsets, paths, poffs)
    return batch, {"files": nfiles, "bytes": total, "planted": planted, "seed": seed}


def fold_runes_batch(seed, nbytes=1 << 20, plants=300, frac=0.3):
    """Seeded corpus in which `frac` of the files have some k/s/i letters turned into the
    folding runes (U+212A, U+017F, U+0130), mostly inside and around planted secrets and
    keywords, plus hand-made files with a folding rune inside the secret or keyword of
    common rules.  Stresses the one place where the kernels' anchors are not exact."""
    from .secret import ScanArgs
    rng = np.random.default_rng(seed)
    b, _ = make_corpus(nbytes, seed=seed, plants_per_mib=plants)
    args = []
    for i in range(b.nfiles):
        c = bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])])
        if rng.random() < frac and len(c) > 0:
            t = bytearray()
            p = float(rng.choice([0.002, 0.02, 0.2]))
            for ch in c:
                if ch in FOLD and rng.random() < p:
                    t += FOLD[ch].encode()
                else:
                    t.append(ch)
            c = bytes(t)
        args.append(ScanArgs(b.path(i), c))
    hand = [
        "aws_secret_access_\u212aey = \"12ASD34qwe56CXZ78tyH10Tna543VBokN85RHCas\"\n",
        "AWS_\u017fECRET_ACCESS_KEY=12ASD34qwe56CXZ78tyH10Tna543VBokN85RHCas\n",
        "ghp_0123456789abcdefghij\u212almnopqrstuvwxyz\n",
        "\u0130ntercom_api_token = \"" + "a" * 60 + "\"\n",
        "gitlab_\u017fecret glpat-0123456789abcdefghij\n",
        "-----BEGIN RSA PRIVATE KEY-----\nMIIEabc\n-----END RSA PRIVATE KEY-----\n",
        "twitch_api_\u212aey = '" + "x" * 30 + "'\n",
        "facebook_token = '" + "a" * 31 + "\u212a'\n",
    ] + [w + "\n" for w in FOLD_PLANTS]
    for j, h in enumerate(hand):
        args.append(ScanArgs("hand/f%d.txt" % j, h.encode()))
    return Batch.from_args(args)


def k1_edge_batch(literals, seed, nfiles=400):
    """Seeded batch of K1 edge cases for a rule set's K1 literals (Scanner.k1_literals()):
    every literal in random letter case at the start and at the end of a file, split across
    two files at every position, at the batch's first and last byte; class-U runs of 30-34
    bytes and class-D runs of 10-14 bytes at every offset mod 16, also across file
    boundaries; CR/LF, '-' next to CR, high and zero bytes; tiny and empty files.  The
    filter-and-verify K1 (K1F) and the automaton must agree with k1_reference on it."""
    from .secret import ScanArgs
    rng = np.random.default_rng(seed)

    def rcase(b):
        return bytes(c - 32 if 97 <= c <= 122 and rng.random() < 0.5 else c for c in b)

    def filler(n):
        pool = b"abcxyz \n\r-_.=/+0123456789\x00\x80\xc4\xe2\xff\t"
        return bytes(pool[int(i)] for i in rng.integers(0, len(pool), n))

    lits = [s for s, _ in literals if s]
    files = [rcase(lits[0]) + filler(int(rng.integers(0, 40)))]  # the batch's first byte
    for s in lits:
        files.append(rcase(s) + filler(int(rng.integers(0, 40))))
        files.append(filler(int(rng.integers(0, 40))) + rcase(s))
        for cut in range(1, len(s)):
            files.append(filler(int(rng.integers(0, 8))) + rcase(s[:cut]))
            files.append(rcase(s[cut:]) + filler(int(rng.integers(0, 8))))
    for n in range(30, 35):
        for off in range(17):
            tok = bytes(rng.choice(list(b"aZ09+/=_.-"), n))
            files.append(filler(off) + tok + filler(int(rng.integers(0, 20))))
            files.append(filler(off) + tok[: n // 2])
            files.append(tok[n // 2:] + filler(3))
    for n in range(10, 15):
        for off in range(17):
            dig = bytes(rng.choice(list(b"0123456789-"), n))
            files.append(filler(off) + dig + b"\r-\r" + filler(int(rng.integers(0, 20))))
            files.append(filler(off) + dig[: n // 2])
            files.append(dig[n // 2:] + filler(2))
    while len(files) < nfiles:
        k = int(rng.integers(0, 4))
        if k == 0:
            files.append(b"")
        elif k == 1:
            files.append(filler(int(rng.integers(1, 4))))
        else:
            parts = [filler(int(rng.integers(0, 60)))]
            for _ in range(int(rng.integers(0, 4))):
                parts.append(rcase(lits[int(rng.integers(0, len(lits)))]))
                parts.append(filler(int(rng.integers(0, 30))))
            files.append(b"".join(parts))
    order = list(range(1, len(files)))
    rng.shuffle(order)
    files = [files[0]] + [files[i] for i in order] + [filler(5) + rcase(lits[-1])]  # ... and its last
    return Batch.from_args([ScanArgs("e/%d.txt" % i, c) for i, c in enumerate(files)])
