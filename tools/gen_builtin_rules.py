#!/usr/bin/env python3
"""Extract trivy's builtin secret-rule DATA into JSON.

Reads (as text, never executes) the reference's rule tables:
  pkg/fanal/secret/builtin-rules.go:9-67   (category constants)
  pkg/fanal/secret/builtin-rules.go:70-77  (quote/connect/startSecret/endSecret/aws)
  pkg/fanal/secret/builtin-rules.go:79-782 (83 rules)
  pkg/fanal/secret/builtin-allow-rules.go:3-64 (12 path allow rules)
and writes trivy_amd/rules/builtin_rules.json. The output is pure data (rule ids,
titles, regex source strings, keywords); `fmt.Sprintf` splices are evaluated here.

Run once in the build container (the reference does not exist on the GPU box):
    python tools/gen_builtin_rules.py /root/reference
"""
import json
import os
import re
import sys


def go_string(tok):
    """Decode one Go string literal (raw `...` or interpreted "...")."""
    if tok.startswith("`"):
        return tok[1:-1]
    assert tok.startswith('"')
    body = tok[1:-1]
    out = []
    i = 0
    while i < len(body):
        c = body[i]
        if c == "\\":
            n = body[i + 1]
            simple = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'"}
            if n in simple:
                out.append(simple[n])
                i += 2
                continue
            raise ValueError("unsupported escape in %r" % tok)
        out.append(c)
        i += 1
    return "".join(out)


STR = r'(`[^`]*`|"(?:[^"\\]|\\.)*")'


def parse_rules(src, consts, cats):
    rules = []
    body = src[src.index("var builtinRules = []Rule{"):]
    # split entries at top-level "\t{\n" lines
    entries = re.split(r"\n\t\{\n", body)[1:]
    for ent in entries:
        r = {}
        m = re.search(r"\bID:\s*" + STR, ent)
        r["id"] = go_string(m.group(1))
        m = re.search(r"\bCategory:\s*(\w+)", ent)
        r["category"] = cats[m.group(1)]
        m = re.search(r"\bTitle:\s*" + STR, ent)
        r["title"] = go_string(m.group(1))
        m = re.search(r"\bSeverity:\s*" + STR, ent)
        r["severity"] = go_string(m.group(1)) if m else ""
        m = re.search(r"\bRegex:\s*MustCompile\(fmt\.Sprintf\(" + STR + r",\s*([^)]*)\)\)", ent)
        if m:
            fmtstr = go_string(m.group(1))
            args = [a.strip() for a in m.group(2).split(",") if a.strip()]
            vals = [consts[a] for a in args]
            assert fmtstr.count("%s") == len(vals), r["id"]
            r["regex"] = _sprintf(fmtstr, vals)
        else:
            m = re.search(r"\bRegex:\s*MustCompile\(" + STR + r"\)", ent)
            r["regex"] = go_string(m.group(1))
        m = re.search(r"\bSecretGroupName:\s*" + STR, ent)
        r["secret_group_name"] = go_string(m.group(1)) if m else ""
        m = re.search(r"\bKeywords:\s*\[\]string\{(.*?)\}", ent, re.S)
        r["keywords"] = [go_string(t) for t in re.findall(STR, m.group(1))] if m else []
        rules.append(r)
    return rules


def _sprintf(fmtstr, vals):
    parts = fmtstr.split("%s")
    out = parts[0]
    for v, p in zip(vals, parts[1:]):
        out += v + p
    return out


def parse_allow(src):
    rules = []
    for ent in re.split(r"\n\t\{\n", src)[1:]:
        r = {}
        r["id"] = go_string(re.search(r"\bID:\s*" + STR, ent).group(1))
        r["description"] = go_string(re.search(r"\bDescription:\s*" + STR, ent).group(1))
        m = re.search(r"\bPath:\s*MustCompile\(" + STR + r"\)", ent)
        r["path"] = go_string(m.group(1)) if m else None
        m = re.search(r"\bRegex:\s*MustCompile\(" + STR + r"\)", ent)
        r["regex"] = go_string(m.group(1)) if m else None
        rules.append(r)
    return rules


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    base = os.path.join(ref, "pkg/fanal/secret")
    src = open(os.path.join(base, "builtin-rules.go")).read()
    cats = {m.group(1): go_string(m.group(2)) for m in
            re.finditer(r"(Category\w+)\s*=\s*types\.SecretRuleCategory\(" + STR + r"\)", src)}
    consts = {m.group(1): go_string(m.group(2)) for m in
              re.finditer(r"^\t(quote|connect|startSecret|endSecret|aws)\s*=\s*" + STR, src, re.M)}
    rules = parse_rules(src, consts, cats)
    allow = parse_allow(open(os.path.join(base, "builtin-allow-rules.go")).read())
    assert len(rules) == 83, len(rules)
    assert len(allow) == 12, len(allow)
    out = {
        "source": "trivy pkg/fanal/secret/builtin-rules.go:79-782, builtin-allow-rules.go:3-64",
        "rules": rules,
        "allow_rules": allow,
    }
    here = os.path.dirname(os.path.abspath(__file__))
    dst = os.path.join(here, "..", "trivy_amd", "rules", "builtin_rules.json")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
        f.write("\n")
    print("wrote", dst, len(rules), "rules,", len(allow), "allow rules")


if __name__ == "__main__":
    main()
