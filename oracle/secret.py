"""Restatement of trivy's secret scanner (oracle only; see oracle/__init__.py).

Follows, function by function:
  pkg/fanal/secret/scanner.go            (Config/Rule/AllowRule/ExcludeBlock, Scan, censor,
                                          toFinding, findLocation)
  pkg/fanal/secret/builtin-rules.go      (data: trivy_amd/rules/builtin_rules.json)
  pkg/fanal/analyzer/secret/secret.go    (Analyze, Required, skip lists)
  pkg/fanal/utils/utils.go:71-89         (IsBinary)
  pkg/fanal/analyzer/analyzer.go:212-223 (AnalysisResult.Sort, secrets part)

Values are plain dicts mirroring Go's types.Secret / types.SecretFinding /
types.Code / types.Line; Go `string` fields that come from file content are
kept as `bytes` so invalid UTF-8 survives exactly as Go keeps it.
"""
import json
import os

import yaml

from . import gosort
from .goregex import GoRegexp, MustCompile
from .gounicode import go_to_lower

_RULES_JSON = os.path.join(os.path.dirname(__file__), "..", "trivy_amd", "rules",
                           "builtin_rules.json")


class ConfigError(ValueError):
    pass


# ------------------------------------------------------------------ rule types
class AllowRule:
    def __init__(self, id="", description="", regex=None, path=None):
        self.ID = id
        self.Description = description
        self.Regex = regex
        self.Path = path


def allow_rules_allow_path(rules, path):           # scanner.go:195-202
    for r in rules:
        if r.Path is not None and r.Path.MatchString(path):
            return True
    return False


def allow_rules_allow(rules, match):               # scanner.go:204-211
    for r in rules:
        if r.Regex is not None and r.Regex.MatchString(match):
            return True
    return False


class ExcludeBlock:
    def __init__(self, description="", regexes=None):
        self.Description = description
        self.Regexes = regexes or []


class Rule:
    def __init__(self, id="", category="", title="", severity="", regex=None, keywords=None,
                 path=None, allow_rules=None, exclude_block=None, secret_group_name=""):
        self.ID = id
        self.Category = category
        self.Title = title
        self.Severity = severity
        self.Regex = regex
        self.Keywords = keywords or []
        self.Path = path
        self.AllowRules = allow_rules or []
        self.ExcludeBlock = exclude_block or ExcludeBlock()
        self.SecretGroupName = secret_group_name

    def MatchPath(self, path):                     # scanner.go:160-162
        return self.Path is None or self.Path.MatchString(path)

    def MatchKeywords(self, content):              # scanner.go:164-176
        if len(self.Keywords) == 0:
            return True
        for kw in self.Keywords:
            # bytes.ToLower(content) once per keyword, as the reference does
            if go_to_lower(kw.encode("utf-8", "surrogateescape")) in go_to_lower(content):
                return True
        return False

    def AllowPath(self, path):
        return allow_rules_allow_path(self.AllowRules, path)

    def Allow(self, match):
        return allow_rules_allow(self.AllowRules, match)

    def getMatchSubgroupsLocations(self, match_locs):  # scanner.go:148-158
        locs = []
        for i, name in enumerate(self.Regex.SubexpNames()):
            if name == self.SecretGroupName:
                locs.append((match_locs[2 * i], match_locs[2 * i + 1]))
        return locs


# ------------------------------------------------------------------ builtins
def _load_builtins():
    d = json.load(open(_RULES_JSON))
    rules = [Rule(id=r["id"], category=r["category"], title=r["title"], severity=r["severity"],
                  regex=MustCompile(r["regex"]), keywords=list(r["keywords"]),
                  secret_group_name=r["secret_group_name"]) for r in d["rules"]]
    allow = [AllowRule(id=a["id"], description=a["description"],
                       regex=MustCompile(a["regex"]) if a["regex"] is not None else None,
                       path=MustCompile(a["path"]) if a["path"] is not None else None)
             for a in d["allow_rules"]]
    return rules, allow


_BUILTIN = None


def builtins():
    global _BUILTIN
    if _BUILTIN is None:
        _BUILTIN = _load_builtins()
    return _BUILTIN


# ------------------------------------------------------------------ config
class Config:
    def __init__(self):
        self.EnableBuiltinRuleIDs = []
        self.DisableRuleIDs = []
        self.DisableAllowRuleIDs = []
        self.CustomRules = []
        self.CustomAllowRules = []
        self.ExcludeBlock = ExcludeBlock()


def _re(v):
    if v is None:
        return None
    try:
        return GoRegexp(str(v))
    except ValueError as e:
        raise ConfigError("regexp compile error: %s" % e)


def _str(v):
    return "" if v is None else str(v)


def _allow_rules(lst):
    return [AllowRule(id=_str(a.get("id")), description=_str(a.get("description")),
                      regex=_re(a.get("regex")), path=_re(a.get("path"))) for a in (lst or [])]


def _exclude_block(d):
    d = d or {}
    return ExcludeBlock(description=_str(d.get("description")),
                        regexes=[_re(x) for x in (d.get("regexes") or [])])


def config_from_dict(doc):
    if not isinstance(doc, dict):
        raise ConfigError("secrets config decode error")
    c = Config()
    c.EnableBuiltinRuleIDs = [str(x) for x in (doc.get("enable-builtin-rules") or [])]
    c.DisableRuleIDs = [str(x) for x in (doc.get("disable-rules") or [])]
    c.DisableAllowRuleIDs = [str(x) for x in (doc.get("disable-allow-rules") or [])]
    for r in doc.get("rules") or []:
        c.CustomRules.append(Rule(
            id=_str(r.get("id")), category=_str(r.get("category")), title=_str(r.get("title")),
            severity=_str(r.get("severity")), regex=_re(r.get("regex")),
            keywords=[str(k) for k in (r.get("keywords") or [])], path=_re(r.get("path")),
            allow_rules=_allow_rules(r.get("allow-rules")),
            exclude_block=_exclude_block(r.get("exclude-block")),
            secret_group_name=_str(r.get("secret-group-name"))))
    c.CustomAllowRules = _allow_rules(doc.get("allow-rules"))
    c.ExcludeBlock = _exclude_block(doc.get("exclude-block"))
    return c


def ParseConfig(config_path):                      # scanner.go:267-291
    if not config_path:
        return None
    if not os.path.exists(config_path):
        return None
    with open(config_path, "rb") as f:
        doc = yaml.safe_load(f)
    if doc is None:
        raise ConfigError("secrets config decode error: EOF")
    return config_from_dict(doc)


class Scanner:
    def __init__(self, rules, allow_rules, exclude_block):
        self.Rules = rules
        self.AllowRules = allow_rules
        self.ExcludeBlock = exclude_block

    def AllowPath(self, path):
        return allow_rules_allow_path(self.AllowRules, path)

    def Allow(self, match):
        return allow_rules_allow(self.AllowRules, match)

    # -------------------------------------------------------------- matching
    def AllowLocation(self, r, content, loc):      # scanner.go:143-146
        match = content[loc[0]:loc[1]]
        return self.Allow(match) or r.Allow(match)

    def FindLocations(self, r, content):           # scanner.go:96-120
        if r.Regex is None:
            return []
        if r.SecretGroupName != "":
            return self.FindSubmatchLocations(r, content)
        locs = []
        for idx in r.Regex.FindAllIndex(content, -1):
            loc = (idx[0], idx[1])
            if self.AllowLocation(r, content, loc):
                continue
            locs.append(loc)
        return locs

    def FindSubmatchLocations(self, r, content):   # scanner.go:122-141
        out = []
        for m in r.Regex.FindAllSubmatchIndex(content, -1):
            loc = (m[0], m[1])
            if self.AllowLocation(r, content, loc):
                continue
            out.extend(r.getMatchSubgroupsLocations(m))
        return out

    def Scan(self, file_path, content):            # scanner.go:341-416
        if self.AllowPath(file_path):
            return {"FilePath": file_path, "Findings": None}
        censored = None
        matched = []
        global_blocks = _Blocks(content, self.ExcludeBlock.Regexes)
        for rule in self.Rules:
            if not rule.MatchPath(file_path):
                continue
            if rule.AllowPath(file_path):
                continue
            if not rule.MatchKeywords(content):
                continue
            locs = self.FindLocations(rule, content)
            if not locs:
                continue
            local_blocks = _Blocks(content, rule.ExcludeBlock.Regexes)
            for loc in locs:
                if global_blocks.Match(loc) or local_blocks.Match(loc):
                    continue
                if loc[0] < 0:
                    # the reference panics here (slice bounds); never planted by our corpora
                    raise RuntimeError("secret group did not participate in the match")
                matched.append((rule, loc))
                if censored is None:
                    censored = bytearray(content)
                censored[loc[0]:loc[1]] = b"*" * (loc[1] - loc[0])
        findings = [to_finding(rule, loc, bytes(censored)) for rule, loc in matched]
        if not findings:
            return {"FilePath": "", "Findings": None}
        gosort.sort_slice(findings, _finding_less)
        return {"FilePath": file_path, "Findings": findings}


def _finding_less(a, b):                           # scanner.go:405-410
    if a["RuleID"] != b["RuleID"]:
        return a["RuleID"].encode() < b["RuleID"].encode()
    return a["Match"] < b["Match"]


class _Blocks:                                     # scanner.go:227-265 (lazy once)
    def __init__(self, content, regexes):
        self.content = content
        self.regexes = regexes
        self.locs = None

    def Match(self, block):
        if self.locs is None:
            self.locs = []
            for rx in self.regexes:
                for r in rx.FindAllIndex(self.content, -1):
                    self.locs.append((r[0], r[1]))
        for s, e in self.locs:
            if s <= block[0] and block[1] <= e:
                return True
        return False


def NewScanner(config):                            # scanner.go:293-329
    b_rules, b_allow = builtins()
    if config is None:
        return Scanner(list(b_rules), list(b_allow), ExcludeBlock())
    enabled = list(b_rules)
    if config.EnableBuiltinRuleIDs:
        enabled = [r for r in b_rules if r.ID in config.EnableBuiltinRuleIDs]
    enabled = enabled + config.CustomRules
    rules = [r for r in enabled if r.ID not in config.DisableRuleIDs]
    allow = [a for a in list(b_allow) + config.CustomAllowRules
             if a.ID not in config.DisableAllowRuleIDs]
    return Scanner(rules, allow, config.ExcludeBlock)


# ------------------------------------------------------------------ materialise
def to_finding(rule, loc, content):                # scanner.go:428-441
    start_line, end_line, code, match_line = find_location(loc[0], loc[1], content)
    return {
        "RuleID": rule.ID,
        "Category": rule.Category,
        "Severity": "UNKNOWN" if rule.Severity == "" else rule.Severity,
        "Title": rule.Title,
        "StartLine": start_line,
        "EndLine": end_line,
        "Code": code,
        "Match": match_line,
    }


SECRET_HIGHLIGHT_RADIUS = 2


def find_location(start, end, content):            # scanner.go:445-502
    start_line_num = content.count(b"\n", 0, start)
    line_start = content.rfind(b"\n", 0, start)
    line_start = 0 if line_start == -1 else line_start + 1
    line_end = content.find(b"\n", start)
    if line_end == -1:
        line_end = len(content)
    match = content[start:end]
    match_line = content[line_start:line_end]
    if len(match_line) > 100:
        ts = 0 if start - 30 < 0 else start - 30
        te = len(content) if end + 20 > len(content) else end + 20
        match_line = content[ts:te]
    end_line_num = start_line_num + match.count(b"\n")
    lines = content.split(b"\n")
    code_start = max(start_line_num - SECRET_HIGHLIGHT_RADIUS, 0)
    code_end = min(end_line_num + SECRET_HIGHLIGHT_RADIUS, len(lines))
    out = []
    found_first = False
    for i, raw in enumerate(lines[code_start:code_end]):
        real = code_start + i
        in_cause = start_line_num <= real <= end_line_num
        out.append({"Number": real + 1, "Content": raw, "IsCause": in_cause, "Annotation": "",
                    "Truncated": False, "Highlighted": raw,
                    "FirstCause": (not found_first) and in_cause, "LastCause": False})
        found_first = found_first or in_cause
    for ln in reversed(out):
        if ln["IsCause"]:
            ln["LastCause"] = True
            break
    return start_line_num + 1, end_line_num + 1, {"Lines": out or None}, match_line


# ------------------------------------------------------------------ analyzer
SKIP_FILES = ["go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
              "Pipfile.lock", "Gemfile.lock"]
SKIP_DIRS = [".git", "node_modules"]
SKIP_EXTS = [".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm",
             ".zip", ".gz", ".gzip", ".tar", ".pyc"]


def IsBinary(content, file_size):                  # utils.go:71-89
    head = content[:min(file_size, 300)]
    for b in head:
        if b < 7 or b == 11 or (13 < b < 27) or (27 < b < 0x20) or b == 0x7F:
            return True
    return False


def _go_base(p):
    """filepath.Base"""
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p[p.rfind("/") + 1:]


def _go_ext(name):
    i = name.rfind(".")
    j = name.rfind("/")
    return name[i:] if i > j else ""


class SecretAnalyzer:                              # analyzer/secret/secret.go
    def __init__(self, config_path=""):
        self.config_path = config_path
        self.scanner = NewScanner(ParseConfig(config_path))

    def Required(self, file_path, size):           # secret.go:112-150
        if size < 10:
            return False
        k = file_path.rfind("/")
        d, name = file_path[:k + 1], file_path[k + 1:]
        dirs = d.split("/")
        for sd in SKIP_DIRS:
            if sd in dirs:
                return False
        if name in SKIP_FILES:
            return False
        if _go_base(self.config_path) == file_path:
            return False
        if _go_ext(name) in SKIP_EXTS:
            return False
        if self.scanner.AllowPath(file_path):
            return False
        return True

    def Analyze(self, file_path, content, dir):    # secret.go:78-110
        if IsBinary(content, len(content)):
            return None
        fp = file_path
        if dir == "":
            fp = "/" + fp
        res = self.scanner.Scan(fp, content)
        if not res["Findings"]:
            return None
        return {"Secrets": [res]}


def sort_secrets(secrets):                         # analyzer.go:212-223
    gosort.sort_slice(secrets, lambda a, b: a["FilePath"].encode() < b["FilePath"].encode())
    for s in secrets:
        if s["Findings"]:
            gosort.sort_slice(s["Findings"], lambda a, b: (
                a["RuleID"].encode() < b["RuleID"].encode() if a["RuleID"] != b["RuleID"]
                else a["StartLine"] < b["StartLine"]))
    return secrets
