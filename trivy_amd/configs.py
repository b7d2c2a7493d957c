"""Seeded rule-set configurations for the BASELINE parity configs beyond the builtins.

    user_rules_doc(n, seed)    configs[3]: n user-defined rules in trivy-secret.yaml form
                               (SURVEY.md §8d "Config 4"): generic-family clones with
                               random keyword names, rules with no keywords, unbounded
                               (?s).* rules between literals, and DFA state-blowup
                               patterns that force the NFA / host-only fallback.  Every
                               rule has a `secret` group (scanner.go:148-158).
    allow_exclude_doc(seed)    configs[4]: global and per-rule allow rules (regex and
                               path) and exclude blocks (scanner.go:50-57, :178-265).
    plant_lines(doc, rng, k)   lines that match rules of `doc`, to mix into a corpus.

The documents are plain dicts in the YAML schema of ParseConfig (scanner.go:27-47), so
they go through trivy_amd.secret.config_from_dict exactly like a parsed file.
"""
import string

import numpy as np

_ALNUM = string.ascii_lowercase + string.digits


def _name(rng, lo=5, hi=12):
    n = int(rng.integers(lo, hi + 1))
    return "".join(rng.choice(list(string.ascii_lowercase), size=n))


def user_rules_doc(n=1000, seed=4):
    """configs[3]: 60 % generic clones, 20 % keyword-less, 10 % unbounded, 10 % blow-up."""
    rng = np.random.default_rng(seed)
    rules = []
    seen = set()
    for i in range(n):
        kind = i % 10
        name = _name(rng)
        while name in seen:
            name = _name(rng)
        seen.add(name)
        rid = "user-%04d-%s" % (i, name)
        r = {"id": rid, "category": "user", "title": "User rule %d" % i,
             "severity": ["LOW", "MEDIUM", "HIGH", "CRITICAL", ""][i % 5],
             "secret-group-name": "secret"}
        if kind < 6:    # generic-family clone (builtin-rules.go generic pattern)
            r["regex"] = (r"(?i)(?:%s)(?:[0-9a-z\-_\t .]{0,20})(?:[\s|']|[\s|\"]){0,3}"
                          r"(?:=|>|:=|\|\|:|<=|=>|:)(?:'|\"|\s|=|\x60){0,5}"
                          r"(?P<secret>[0-9a-z]{16,32})(?:['|\"|\n|\r|\s|\x60]|$)" % name)
            r["keywords"] = [name]
        elif kind < 8:  # no keywords: always scanned
            r["regex"] = r"%s_(?P<secret>[A-Z0-9]{20})\b" % name.upper()
        elif kind < 9:  # unbounded between two literals
            r["regex"] = r"(?s)begin_%s(?P<secret>.*)end_%s" % (name, name)
            r["keywords"] = ["begin_" + name]
        else:           # DFA state blow-up: counted overlap / k-th symbol from the end
            if i % 20 == 9:
                r["regex"] = r"%s(?P<secret>[a-z0-9]{1,40}x[a-f0-9]{20,40})" % name
            else:
                r["regex"] = r"%s(?P<secret>(a|b)*a(a|b){15})" % name
            r["keywords"] = [name]
        rules.append(r)
    return {"rules": rules}


def allow_exclude_doc(seed=5):
    """configs[4]: allow rules and exclude blocks around builtin and custom rules."""
    return {
        "rules": [
            {"id": "custom-token", "category": "custom", "title": "Custom token", "severity": "HIGH",
             "regex": r"(?i)(?P<key>(custom_token))(=|:).{0,5}['\"](?P<secret>[0-9a-zA-Z\-_=]{8,64})['\"]",
             "secret-group-name": "secret", "keywords": ["custom_token"],
             "allow-rules": [{"id": "skip-test-values", "regex": "TESTVALUE"},
                             {"id": "skip-fixtures", "path": r"fixtures/"}],
             "exclude-block": {"description": "local block",
                               "regexes": [r"--- ignore block start ---(.|\s)*--- ignore block stop ---"]}},
        ],
        "allow-rules": [{"id": "global-example", "regex": "EXAMPLEKEY"},
                        {"id": "global-docs", "path": r"\.rst$"}],
        "exclude-block": {"description": "global block",
                          "regexes": [r"-----BEGIN IGNORE-----(.|\s)*?-----END IGNORE-----"]},
    }


def plant_lines(doc, rng, k):
    """k lines, each matching (or nearly matching) a random rule of `doc`."""
    rules = doc.get("rules") or []
    out = []
    for _ in range(k):
        r = rules[int(rng.integers(0, len(rules)))]
        rid = r["id"]
        name = rid.split("-", 2)[-1] if rid.startswith("user-") else "custom_token"
        tok = "".join(rng.choice(list(_ALNUM), size=int(rng.integers(12, 36))))
        kind = int(rng.integers(0, 6))
        if kind == 0:
            out.append("%s = '%s'" % (name, tok))
        elif kind == 1:
            out.append("%s_%s" % (name.upper(), tok.upper()[:20].ljust(20, "Q")))
        elif kind == 2:
            out.append("begin_%s %s\n%s end_%s" % (name, tok, tok[::-1], name))
        elif kind == 3:
            out.append("%s%sx%s" % (name, tok[:10], "abcdef0123456789"[:int(rng.integers(18, 30)) % 16] * 2))
        elif kind == 4:
            out.append("%s%s" % (name, "".join(rng.choice(["a", "b"], size=int(rng.integers(14, 30))))))
        else:
            out.append("custom_token: '%s' TESTVALUE" % tok if rng.random() < 0.3 else
                       "custom_token='%s'" % tok)
    return out


def mixed_batch(doc, nbytes, seed, plants_per_file=0.3, binary_frac=0.0):
    """A seeded corpus (trivy_amd.corpus) with lines of `plant_lines` mixed into files,
    and (configs[4]) binary blobs: random bytes, half with a text-looking first 300 bytes
    so that they pass utils.IsBinary (utils.go:71-89)."""
    from trivy_amd import corpus
    from trivy_amd import secret as S
    rng = np.random.default_rng(seed)
    base, _ = corpus.make_corpus(nbytes, seed=seed, plants_per_mib=50)
    args = []
    for i in range(base.nfiles):
        c = bytes(base.data[int(base.offsets[i]):int(base.offsets[i + 1])])
        if rng.random() < plants_per_file:
            lines = c.split(b"\n")
            for ln in plant_lines(doc, rng, int(rng.integers(1, 4))):
                lines.insert(int(rng.integers(0, len(lines) + 1)), ln.encode())
            if rng.random() < 0.05:
                lines.insert(0, b"--- ignore block start ---")
                lines.append(b"--- ignore block stop ---")
            c = b"\n".join(lines)
        path = base.path(i)
        if rng.random() < 0.03:
            path = "fixtures/" + path
        args.append(S.ScanArgs(path, c))
        if binary_frac and rng.random() < binary_frac:
            blob = rng.integers(0, 256, size=int(rng.integers(64, 4096)), dtype=np.uint8).tobytes()
            if rng.random() < 0.5:
                blob = (b"custom_token='abcdefgh12345678' " * 10)[:300] + blob
            args.append(S.ScanArgs("blob/%d.bin" % i, blob))
    return args


_LOREM = (b"lorem ipsum dolor sit amet consectetur adipiscing elit sed do eiusmod tempor "
          b"incididunt ut labore et dolore magna aliqua enim ad minim veniam quis nostrud "
          b"exercitation ullamco laboris nisi aliquip ex ea commodo consequat duis aute irure in "
          b"reprehenderit voluptate velit esse cillum fugiat nulla pariatur excepteur sint "
          b"occaecat cupidatat non proident sunt culpa qui officia deserunt mollit anim id est "
          b"laborum").split()


def big_text(nbytes, seed=7):
    """A large text entry ("some entries >= 200 MiB"): filler words
    that hold no rule keyword, and secrets planted at known places: a GitHub token in the
    first line, an AWS key at the middle, private-key blocks straddling the 2 MiB / 16 MiB /
    middle offsets (K1 segments, K2 chunks and items, ingest pieces all break inside them),
    a Slack token near the end and a private-key block whose END line is the file's last
    bytes.  Returns (bytes, {plant name: byte offset})."""
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, len(_LOREM), size=nbytes // 5 + 16)
    parts, n = [], 0
    for k, i in enumerate(idx):
        w = _LOREM[i] + (b"\n" if k % 12 == 11 else b" ")
        parts.append(w)
        n += len(w)
        if n >= nbytes:
            break
    buf = bytearray(b"".join(parts)[:nbytes])
    alnum = string.ascii_letters + string.digits
    upper = string.ascii_uppercase + "234567"
    b64 = string.ascii_letters + string.digits + "+/"

    def pem():
        lines = ["".join(rng.choice(list(b64), size=64)) for _ in range(6)]
        return ("-----BEGIN RSA PRIVATE KEY-----\n" + "\n".join(lines) + "\n-----END RSA PRIVATE KEY-----").encode()

    plants = {}

    def put(name, at, blob):
        at = max(0, min(at, len(buf) - len(blob)))
        buf[at:at + len(blob)] = blob
        plants[name] = at
    put("github", 0, ("GITHUB_TOKEN=ghp_%s\n" % "".join(rng.choice(list(alnum), size=36))).encode())
    put("aws", nbytes // 2 + 4096, ("\naws_access_key_id = AKIA%s\n" % "".join(rng.choice(list(upper), size=16))).encode())
    for name, at in (("pem_2mib", 2 << 20), ("pem_16mib", 16 << 20), ("pem_mid", nbytes // 2)):
        if at + 1024 < nbytes:
            blob = b"\n" + pem() + b"\n"
            put(name, at - len(blob) // 2, blob)
    put("slack", nbytes - 4096, ("\nSLACK=xoxb-%s-%s-%s\n" % (
        "".join(rng.choice(list(string.digits), size=12)), "".join(rng.choice(list(string.digits), size=12)),
        "".join(rng.choice(list(alnum), size=24)))).encode())
    blob = b"\n" + pem()
    put("pem_end", len(buf) - len(blob), blob)
    return bytes(buf), plants


def layer_tar(nbytes, seed=3, binary_frac=0.05, big=()):
    """configs[2] (SURVEY.md §8d "Config 3"): an uncompressed image-layer tar built from the
    seeded corpus, with directory entries, symlinks/hardlinks (no content), whiteouts,
    an opaque marker, a system dir (`proc/`, skipped by the walker), `.git` and
    `node_modules` trees, binary blobs and PAX long names; `big`: sizes of large text entries
    (big_text), written between the corpus files.  Returns the tar bytes."""
    import io
    import tarfile
    from trivy_amd import corpus
    rng = np.random.default_rng(seed)
    base, _ = corpus.make_corpus(nbytes, seed=seed, plants_per_mib=50)
    buf = io.BytesIO()
    dirs = set()

    def add(tf, name, typ, data=b"", link=""):
        ti = tarfile.TarInfo(name)
        ti.type = typ
        ti.linkname = link
        ti.size = len(data) if typ in (tarfile.REGTYPE, tarfile.AREGTYPE) else 0
        tf.addfile(ti, io.BytesIO(data) if ti.size else None)

    with tarfile.open(fileobj=buf, mode="w", format=tarfile.PAX_FORMAT) as tf:
        for i in range(base.nfiles):
            c = bytes(base.data[int(base.offsets[i]):int(base.offsets[i + 1])])
            p = base.path(i).lstrip("/")
            r = rng.random()
            if r < 0.02:
                p = "proc/%d/%s" % (i, p.rsplit("/", 1)[-1])
            elif r < 0.03:
                p = "srv/.git/objects/%d" % i
            elif r < 0.04:
                p = "app/node_modules/%s" % p
            elif r < 0.05:
                p = "deep/" + "/".join("d%d" % k for k in range(24)) + "/" + p
            d = p.rsplit("/", 1)[0] if "/" in p else ""
            parts = d.split("/") if d else []
            for k in range(1, len(parts) + 1):
                dd = "/".join(parts[:k])
                if dd not in dirs:
                    dirs.add(dd)
                    add(tf, dd + "/", tarfile.DIRTYPE)
            add(tf, p, tarfile.REGTYPE, c)
            r = rng.random()
            if r < 0.01:
                add(tf, p + ".lnk", tarfile.SYMTYPE, link=p)
            elif r < 0.02:
                add(tf, p + ".hard", tarfile.LNKTYPE, link=p)
            elif r < 0.025:
                add(tf, (d + "/" if d else "") + ".wh." + "gone%d" % i, tarfile.REGTYPE)
            elif r < 0.026:
                add(tf, (d + "/" if d else "") + ".wh..wh..opq", tarfile.REGTYPE)
            if binary_frac and rng.random() < binary_frac:
                blob = rng.integers(0, 256, size=int(rng.integers(64, 4096)),
                                    dtype=np.uint8).tobytes()
                if rng.random() < 0.5:
                    blob = c[:300].replace(b"\0", b" ") + blob
                add(tf, "blob/%d.dat" % i, tarfile.REGTYPE, blob)
            for k, size in enumerate(big):
                if i == (k + 1) * base.nfiles // (len(big) + 1):
                    if "opt/big" not in dirs:
                        dirs.add("opt/big")
                        add(tf, "opt/", tarfile.DIRTYPE)
                        add(tf, "opt/big/", tarfile.DIRTYPE)
                    add(tf, "opt/big/text%d.log" % k, tarfile.REGTYPE, big_text(size, seed=seed + k)[0])
        add(tf, "etc/.wh..wh..opq", tarfile.REGTYPE)
        add(tf, "etc/.wh.hostname", tarfile.REGTYPE)
    return buf.getvalue()


def source_tree(root, nbytes=200 << 20, seed=0, binary_frac=0.0, binary_text_head=0.5, extra_plants=None,
                extra_per_mib=0.0):
    """configs[0] (SURVEY.md §8d "Config 1"): a seeded source tree on disk for `trivy fs
    --scanners secret`.  Files come from the corpus generator (log-normal sizes, median
    6 KiB; every builtin rule planted, near misses included; md/test/vendor/example/docs
    paths that the builtin allow rules cover), plus explicit AWS / GitHub / Slack tokens,
    and entries the walker or `Required` skips: a .git dir, node_modules, lockfiles, a
    tiny file.  binary_frac: that share of the tree's bytes are binary blobs (random bytes,
    sizes like the text files', under bin/); binary_text_head of them start with 300 bytes
    of text, so utils.IsBinary (utils.go:71-89) passes them to Scan, the others it drops
    (configs[4]: 30 %, half with a text head).  extra_plants / extra_per_mib: lines planted
    on top (a user rule set's, configs.plant_lines).  Returns {"files": written regular
    files, "bytes": their total, "binary_files", "binary_text_head_files"}."""
    import os
    from trivy_amd import corpus
    rng = np.random.default_rng(seed)
    aws = ["aws_access_key_id = AKIA%s" % "".join(rng.choice(list(string.ascii_uppercase + "234567"), size=16))
           for _ in range(8)]
    aws += ["aws_secret_access_key = \"%s\"" % "".join(rng.choice(list(_ALNUM + "ABCDEFGHIJ/+"), size=40))
            for _ in range(8)]
    gh = ["token: %s_%s" % (p, "".join(rng.choice(list(_ALNUM + "ABCDEFGHIJKLMNOP"), size=36)))
          for p in ("ghp", "gho", "ghu", "ghs", "ghr") for _ in range(3)]
    slack = ["SLACK_TOKEN=xoxb-%d-%d-%s" % (rng.integers(10 ** 9, 10 ** 10), rng.integers(10 ** 9, 10 ** 10),
                                           "".join(rng.choice(list(_ALNUM), size=24))) for _ in range(8)]
    slack += ["https://hooks.slack.com/services/T%s/B%s/%s" % (
        "".join(rng.choice(list(string.ascii_uppercase + string.digits), size=8)),
        "".join(rng.choice(list(string.ascii_uppercase + string.digits), size=8)),
        "".join(rng.choice(list(_ALNUM), size=24))) for _ in range(4)]
    extra = [x for t in zip(aws, gh, slack) for x in t] + aws[8:] + gh[8:] + slack[8:]
    text_bytes = int(nbytes * (1.0 - binary_frac))
    b, info = corpus.make_corpus(text_bytes, seed=seed, plants_per_mib=5.0,
                                 extra_plants=extra + list(extra_plants or []),
                                 extra_per_mib=8.0 + extra_per_mib)
    nfiles, total = 0, 0
    for i in range(b.nfiles):
        p = os.path.join(root, b.path(i))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        data = b.data[int(b.offsets[i]):int(b.offsets[i + 1])]
        with open(p, "wb") as f:
            f.write(data.tobytes())
        nfiles += 1
        total += len(data)
    nbin = nhead = 0
    if binary_frac > 0:
        # blob sizes drawn like the text files' (from the corpus offsets), random content
        sizes = np.diff(b.offsets.astype(np.int64))
        left = nbytes - text_bytes
        os.makedirs(os.path.join(root, "bin"), exist_ok=True)
        while left > 0:
            n = int(min(left, max(16, sizes[int(rng.integers(0, len(sizes)))])))
            blob = rng.integers(0, 256, size=n, dtype=np.uint8)
            if rng.random() < binary_text_head:
                i = int(rng.integers(0, b.nfiles))
                head = b.data[int(b.offsets[i]):int(b.offsets[i]) + min(300, n)]
                blob[:len(head)] = head
                if len(head) < min(300, n):  # a short text file: printable filler after it
                    blob[len(head):min(300, n)] = ord("x")
                nhead += 1
            with open(os.path.join(root, "bin", "blob%06d.dat" % nbin), "wb") as f:
                f.write(blob.tobytes())
            nbin += 1
            nfiles += 1
            total += n
            left -= n
    planted = "\n".join(aws[:2] + gh[:2] + slack[:2]).encode()
    for rel in (".git/config", "node_modules/pkg/index.js", "package-lock.json", "go.sum",
                "src/tiny.txt"):
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(planted if rel != "src/tiny.txt" else b"AKIA")
        nfiles += 1
        total += len(planted) if rel != "src/tiny.txt" else 4
    return {"files": nfiles, "bytes": total, "planted": info["planted"], "seed": seed,
            "binary_files": nbin, "binary_text_head_files": nhead}
