#!/usr/bin/env python3
"""Turn the reference's own test expectations for the secret path into JSON fixtures.

Sources (read as text; the Go composite literals are parsed, nothing is executed):
  pkg/fanal/secret/scanner_test.go:24-765            26 Scan cases + their testdata/
  pkg/fanal/analyzer/secret/secret_test.go:16-223     5 Analyze + 5 Required cases
  integration/testdata/secrets.json.golden            `trivy fs` secrets golden
  integration/testdata/fixtures/fs/secrets/*          its inputs

Output: tests/golden/reference_cases.json plus copies of the input data files under
tests/golden/reference/ (data files the reference's tests hold).  Run here once:
    python tools/gen_reference_fixtures.py /root/reference
"""
import json
import os
import re
import shutil
import sys

TOK = re.compile(r"""\s*(?:(?P<raw>`[^`]*`)|(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+)|"""
                 r"""(?P<id>[A-Za-z_][A-Za-z0-9_.]*)|(?P<p>[{}\[\]:,&*()]))""", re.S)


def go_str(tok):
    if tok[0] == "`":
        return tok[1:-1]
    body = tok[1:-1]
    out, i = [], 0
    esc = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'"}
    while i < len(body):
        if body[i] == "\\":
            out.append(esc[body[i + 1]])
            i += 2
        else:
            out.append(body[i])
            i += 1
    return "".join(out)


class Lit:
    def __init__(self, src, env):
        self.toks = []
        pos = 0
        while pos < len(src):
            m = TOK.match(src, pos)
            if not m or m.end() == pos:
                if src[pos:].strip() == "":
                    break
                raise ValueError("tokenize at %r" % src[pos:pos + 40])
            kind = m.lastgroup
            self.toks.append((kind, m.group(kind)))
            pos = m.end()
        self.i = 0
        self.env = env

    def peek(self, k=0):
        return self.toks[self.i + k] if self.i + k < len(self.toks) else (None, None)

    def take(self, val=None):
        t = self.toks[self.i]
        if val is not None and t[1] != val:
            raise ValueError("expected %r got %r" % (val, t))
        self.i += 1
        return t

    def value(self):
        kind, v = self.peek()
        if v == "&":
            self.take()
            return self.value()
        if kind in ("raw", "str"):
            self.take()
            return go_str(v)
        if kind == "num":
            self.take()
            return int(v)
        if v == "[":
            self.take("[")
            self.take("]")
            self.take()  # element type
            return self.body(list_=True)
        if v == "{":
            return self.body(list_=False)
        if kind == "id":
            self.take()
            if self.peek()[1] == "{":
                return self.body(list_=False)
            if v == "true":
                return True
            if v == "false":
                return False
            if v == "nil":
                return None
            return self.env[v]
        raise ValueError("bad value %r" % (v,))

    def body(self, list_):
        self.take("{")
        if list_:
            out = []
            while self.peek()[1] != "}":
                out.append(self.value())
                if self.peek()[1] == ",":
                    self.take()
            self.take("}")
            return out
        out = {}
        while self.peek()[1] != "}":
            if self.peek(1)[1] == ":":
                k = self.take()[1]
                self.take(":")
                out[k] = self.value()
            else:  # unkeyed element of an elided-type slice
                out.setdefault("__items__", []).append(self.value())
            if self.peek()[1] == ",":
                self.take()
        self.take("}")
        return out


def extract_block(src, start_pat):
    m = re.search(start_pat, src)
    j = src.index("{", m.end() - 1)
    depth = 0
    for k in range(j, len(src)):
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[m.start():k + 1], k + 1
    raise ValueError


def finding_json(f):
    lines = []
    for ln in f.get("Code", {}).get("Lines", []) or []:
        lines.append({
            "Number": ln.get("Number", 0), "Content": ln.get("Content", ""),
            "IsCause": ln.get("IsCause", False), "Annotation": ln.get("Annotation", ""),
            "Truncated": ln.get("Truncated", False), "Highlighted": ln.get("Highlighted", ""),
            "FirstCause": ln.get("FirstCause", False), "LastCause": ln.get("LastCause", False)})
    return {"RuleID": f.get("RuleID", ""), "Category": f.get("Category", ""),
            "Severity": f.get("Severity", ""), "Title": f.get("Title", ""),
            "StartLine": f.get("StartLine", 0), "EndLine": f.get("EndLine", 0),
            "Code": {"Lines": lines or None}, "Match": f.get("Match", "")}


def secret_json(s):
    if s is None:
        return None
    fs = s.get("Findings")
    return {"FilePath": s.get("FilePath", ""),
            "Findings": None if fs is None else [finding_json(f) for f in fs]}


def parse_test_file(path, env):
    src = open(path).read()
    for m in re.finditer(r"\n\t(want\w+) := types\.SecretFinding\{", src):
        blk, _ = extract_block(src[m.start():], r"types\.SecretFinding\{")
        env[m.group(1)] = Lit(blk, env).value()
    return src


def parse_table(src, env, start_pat):
    _, end = extract_block(src, start_pat)      # the anonymous struct type
    rest = src[end:]
    blk, _ = extract_block(rest, r"\{")        # the table literal
    return Lit(blk, env).value()


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    here = os.path.dirname(os.path.abspath(__file__))
    out_dir = os.path.join(here, "..", "tests", "golden")
    data_dir = os.path.join(out_dir, "reference")
    os.makedirs(data_dir, exist_ok=True)

    rules_src = open(os.path.join(ref, "pkg/fanal/secret/builtin-rules.go")).read()
    env = {"secret." + m.group(1): m.group(2) for m in re.finditer(
        r'(Category\w+)\s*=\s*types\.SecretRuleCategory\("([^"]*)"\)', rules_src)}

    # ---- scanner_test.go
    sdir = os.path.join(ref, "pkg/fanal/secret")
    src = parse_test_file(os.path.join(sdir, "scanner_test.go"), env)
    table = parse_table(src, env, r"tests := \[\]struct \{")
    scanner_cases = []
    for t in table["__items__"]:
        scanner_cases.append({
            "name": t["name"], "config": t.get("configPath", ""),
            "input": t["inputFilePath"], "want": secret_json(t.get("want", {}))})
    sd = os.path.join(data_dir, "secret")
    os.makedirs(os.path.join(sd, "testdata"), exist_ok=True)
    for fn in os.listdir(os.path.join(sdir, "testdata")):
        shutil.copyfile(os.path.join(sdir, "testdata", fn), os.path.join(sd, "testdata", fn))

    # ---- analyzer secret_test.go
    adir = os.path.join(ref, "pkg/fanal/analyzer/secret")
    env2 = dict(env)
    src = parse_test_file(os.path.join(adir, "secret_test.go"), env2)
    m = re.search(r"func TestSecretAnalyzer", src)
    table = parse_table(src[m.start():], env2, r"tests := \[\]struct \{")
    analyzer_cases = []
    for t in table["__items__"]:
        want = t.get("want")
        if want is not None:
            want = {"Secrets": [secret_json(s) for s in want["Secrets"]["__items__"]]} \
                if isinstance(want["Secrets"], dict) else \
                {"Secrets": [secret_json(s) for s in want["Secrets"]]}
        analyzer_cases.append({"name": t["name"], "config": t.get("configPath", ""),
                               "input": t["filePath"], "dir": t.get("dir", ""), "want": want})
    m = re.search(r"func TestSecretRequire", src)
    table = parse_table(src[m.start():], env2, r"tests := \[\]struct \{")
    required_cases = [{"name": t["name"], "input": t["filePath"], "want": t["want"]}
                      for t in table["__items__"]]
    ad = os.path.join(data_dir, "analyzer")
    if os.path.exists(ad):
        shutil.rmtree(ad)
    shutil.copytree(os.path.join(adir, "testdata"), os.path.join(ad, "testdata"))
    for root, dirs, files in os.walk(ad):
        os.chmod(root, 0o755)
        for f in files:
            os.chmod(os.path.join(root, f), 0o644)

    # ---- integration golden
    golden = json.load(open(os.path.join(ref, "integration/testdata/secrets.json.golden")))
    fx = os.path.join(ref, "integration/testdata/fixtures/fs/secrets")
    idir = os.path.join(data_dir, "integration", "secrets")
    os.makedirs(idir, exist_ok=True)
    for fn in os.listdir(fx):
        shutil.copyfile(os.path.join(fx, fn), os.path.join(idir, fn))
    integ = {"config": "trivy-secret.yaml", "results": [
        {"Target": r["Target"], "Secrets": r["Secrets"]} for r in golden["Results"]
        if r.get("Class") == "secret"]}

    out = {
        "source": {
            "scanner": "pkg/fanal/secret/scanner_test.go:24-765",
            "analyzer": "pkg/fanal/analyzer/secret/secret_test.go:16-223",
            "integration": "integration/testdata/secrets.json.golden (fs_test.go:213-219)",
        },
        "scanner_cases": scanner_cases,
        "analyzer_cases": analyzer_cases,
        "required_cases": required_cases,
        "integration": integ,
    }
    with open(os.path.join(out_dir, "reference_cases.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print("scanner cases:", len(scanner_cases), "analyzer:", len(analyzer_cases),
          "required:", len(required_cases))


if __name__ == "__main__":
    main()
