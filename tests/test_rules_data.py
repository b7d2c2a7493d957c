"""The product's rule data (trivy_amd/rules/builtin_rules.json) against the reference's
Go source, re-read here with a parser independent of tools/gen_builtin_rules.py.

gen_builtin_rules.py splits the rule table with regexes; this test tokenizes the Go
source (string literals, identifiers, punctuation), walks the composite literal
`var builtinRules = []Rule{ ... }` by brace depth, and evaluates the only expression forms
the table uses: string literals, the pattern constants, `MustCompile(x)` and
`fmt.Sprintf(fmt, args...)` with `%s` verbs.  Every field of every rule and allow rule is
compared, so a transcription error in any of the 83 rules fails here, not only in the
dozen rules the reference fixtures exercise.

Reads /root/reference as text (it is absent on the GPU box: skipped there)."""
import json
import os

import pytest

REF = "/root/reference/pkg/fanal/secret"
RULES_JSON = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "trivy_amd", "rules", "builtin_rules.json")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference source not present")


def tokenize(src):
    """Go tokens: ('str', value) | ('id', name) | ('p', char).  Comments are dropped."""
    toks, i, n = [], 0, len(src)
    esc = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'"}
    while i < n:
        c = src[i]
        if c.isspace():
            i += 1
        elif src.startswith("//", i):
            i = src.index("\n", i)
        elif src.startswith("/*", i):
            i = src.index("*/", i) + 2
        elif c == "`":
            j = src.index("`", i + 1)
            toks.append(("str", src[i + 1:j]))
            i = j + 1
        elif c == '"':
            out, j = [], i + 1
            while src[j] != '"':
                if src[j] == "\\":
                    out.append(esc[src[j + 1]])
                    j += 2
                else:
                    out.append(src[j])
                    j += 1
            toks.append(("str", "".join(out)))
            i = j + 1
        elif c.isalnum() or c == "_":
            j = i
            while j < n and (src[j].isalnum() or src[j] == "_"):
                j += 1
            toks.append(("id", src[i:j]))
            i = j
        else:
            toks.append(("p", c))
            i += 1
    return toks


class Walker:
    def __init__(self, toks, consts):
        self.t, self.k, self.consts = toks, 0, consts

    def peek(self, o=0):
        return self.t[self.k + o]

    def take(self, kind=None, val=None):
        tok = self.t[self.k]
        assert kind is None or tok[0] == kind, tok
        assert val is None or tok[1] == val, tok
        self.k += 1
        return tok

    def expr(self):
        kind, v = self.take()
        if kind == "str":
            return v
        if kind == "id" and v == "MustCompile":
            self.take("p", "(")
            x = self.expr()
            self.take("p", ")")
            return x
        if kind == "id" and v == "fmt":
            self.take("p", ".")
            self.take("id", "Sprintf")
            self.take("p", "(")
            args = [self.expr()]
            while self.peek() == ("p", ","):
                self.take()
                args.append(self.expr())
            self.take("p", ")")
            fmt, rest = args[0], args[1:]
            assert fmt.count("%s") == len(rest) and "%" not in fmt.replace("%s", "")
            for a in rest:
                fmt = fmt.replace("%s", a, 1)
            return fmt
        if kind == "id" and v == "types":  # types.SecretRuleCategory("X")
            self.take("p", ".")
            self.take("id")
            self.take("p", "(")
            x = self.expr()
            self.take("p", ")")
            return x
        if kind == "id" and v == "nil":
            return None
        if kind == "id" and v == "[":
            raise AssertionError
        if kind == "id":
            return self.consts[v]
        if (kind, v) == ("p", "["):  # []string{...}
            self.take("p", "]")
            self.take("id", "string")
            self.take("p", "{")
            out = []
            while self.peek() != ("p", "}"):
                out.append(self.expr())
                if self.peek() == ("p", ","):
                    self.take()
            self.take("p", "}")
            return out
        raise AssertionError((kind, v))

    def struct(self):
        """{ Field: expr, ... } -> dict"""
        self.take("p", "{")
        d = {}
        while self.peek() != ("p", "}"):
            name = self.take("id")[1]
            self.take("p", ":")
            d[name] = self.expr()
            if self.peek() == ("p", ","):
                self.take()
        self.take("p", "}")
        return d

    def slice_of_structs(self, var):
        while not (self.peek() == ("id", var) and self.peek(1) == ("p", "=")):
            self.k += 1
        self.k += 2
        self.take("p", "[")
        self.take("p", "]")
        self.take("id")
        self.take("p", "{")
        out = []
        while self.peek() != ("p", "}"):
            out.append(self.struct())
            if self.peek() == ("p", ","):
                self.take()
        return out


def consts_of(toks):
    """Every `Name = "lit"` / `Name = types.SecretRuleCategory("lit")` in const blocks."""
    consts = {}
    w = Walker(toks, consts)
    for i in range(len(toks) - 2):
        if toks[i][0] == "id" and toks[i + 1] == ("p", "=") and i > 0 and toks[i - 1][1] != "var":
            if toks[i + 2][0] == "str" or toks[i + 2] == ("id", "types"):
                w.k = i + 2
                consts[toks[i][1]] = w.expr()
    return consts


def test_builtin_rules_match_go_source():
    src = open(os.path.join(REF, "builtin-rules.go")).read()
    toks = tokenize(src)
    consts = consts_of(toks)
    rules = Walker(toks, consts).slice_of_structs("builtinRules")
    mine = json.load(open(RULES_JSON))
    assert len(rules) == len(mine["rules"]) == 83
    for go, j in zip(rules, mine["rules"]):
        assert j["id"] == go["ID"]
        assert j["category"] == go["Category"], go["ID"]
        assert j["title"] == go["Title"], go["ID"]
        assert j["severity"] == go.get("Severity", ""), go["ID"]
        assert j["regex"] == go["Regex"], go["ID"]
        assert j["secret_group_name"] == go.get("SecretGroupName", ""), go["ID"]
        assert j["keywords"] == go.get("Keywords", []), go["ID"]
        assert set(go) <= {"ID", "Category", "Title", "Severity", "Regex", "SecretGroupName",
                           "Keywords"}, go["ID"]


def test_builtin_allow_rules_match_go_source():
    src = open(os.path.join(REF, "builtin-allow-rules.go")).read()
    toks = tokenize(src)
    allow = Walker(toks, {}).slice_of_structs("builtinAllowRules")
    mine = json.load(open(RULES_JSON))["allow_rules"]
    assert len(allow) == len(mine)
    for go, j in zip(allow, mine):
        assert j["id"] == go["ID"]
        assert j["description"] == go.get("Description", ""), go["ID"]
        assert j["regex"] == go.get("Regex"), go["ID"]
        assert j["path"] == go.get("Path"), go["ID"]
