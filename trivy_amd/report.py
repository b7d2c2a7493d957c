"""The consumers of secret findings after the scan, restated for end-to-end parity:

  apply_layers(blobs)          applier.ApplyLayers, secret part: every finding stamped with
                               its layer, files merged across layers by path
                               (pkg/fanal/applier/docker.go:88-93, 134-142, 182-184,
                               269-297)
  secrets_to_results(secrets)  scanner/local.Scanner.secretsToResults
                               (pkg/scanner/local/scan.go:373-385)
  fs_report(name, results)     types.Report of a filesystem artifact (pkg/types/report.go)
  write_json(report)           report.JSONWriter.Write: json.MarshalIndent(report, "", "  ")
                               + a newline (pkg/report/json.go:20-29), with Go's encoding/json
                               string rules (HTML-safe escapes, invalid UTF-8 -> U+FFFD)

Secrets are the dicts of trivy_amd.secret (Go's types.Secret shape).
"""
import copy

# v1.ConfigFile zero value as encoding/json writes it (go-containerregistry): what a
# filesystem artifact's Metadata.ImageConfig holds (integration/testdata/*.json.golden)
_EMPTY_IMAGE_CONFIG = {"architecture": "", "created": "0001-01-01T00:00:00Z", "os": "",
                       "rootfs": {"type": "", "diff_ids": None}, "config": {}}


def _layer(digest="", diff_id="", created_by=""):
    """types.Layer: every field omitempty (artifact.go:20-24)."""
    d = {}
    if digest:
        d["Digest"] = digest
    if diff_id:
        d["DiffID"] = diff_id
    if created_by:
        d["CreatedBy"] = created_by
    return d


def apply_layers(blobs):
    """blobs: [{"Digest", "DiffID", "CreatedBy", "Secrets": [Secret]}] from the lowest layer
    up.  Returns the merged secrets: one per file path; a file's findings are the newest
    layer's plus those of lower layers whose RuleID it does not have (mergeSecrets).  The
    reference iterates a Go map here (unspecified order); this returns path order."""
    merged = {}
    for blob in blobs:
        lay = _layer(blob.get("Digest", ""), blob.get("DiffID", ""), blob.get("CreatedBy", ""))
        for sec in blob.get("Secrets") or []:
            new = copy.deepcopy(sec)
            for f in new["Findings"] or []:
                f["Layer"] = dict(lay)
            old = merged.get(new["FilePath"])
            if old is not None:
                # secretFindingsContains checks the growing newSecret.Findings
                # (applier/docker.go:280-284, :290-297): of several lower-layer findings with
                # a RuleID the upper layer lacks, only the first is kept
                have = {f["RuleID"] for f in new["Findings"] or []}
                for f in old["Findings"] or []:
                    if f["RuleID"] not in have:
                        new["Findings"] = (new["Findings"] or []) + [f]
                        have.add(f["RuleID"])
            merged[new["FilePath"]] = new
    return [merged[k] for k in sorted(merged)]


def secrets_to_results(secrets):
    return [{"Target": s["FilePath"], "Class": "secret", "Secrets": s["Findings"]} for s in secrets]


def _finding(f):
    """types.SecretFinding in field order; Layer is a struct (never omitted)."""
    lines = f["Code"]["Lines"]
    out_lines = None
    if lines is not None:
        out_lines = []
        for ln in lines:
            d = {"Number": ln["Number"], "Content": ln["Content"], "IsCause": ln["IsCause"],
                 "Annotation": ln.get("Annotation", ""), "Truncated": ln.get("Truncated", False)}
            hl = ln.get("Highlighted", b"")
            if hl not in (b"", ""):  # `json:"Highlighted,omitempty"` (misconf.go:51)
                d["Highlighted"] = hl
            d["FirstCause"] = ln["FirstCause"]
            d["LastCause"] = ln["LastCause"]
            out_lines.append(d)
    return {"RuleID": f["RuleID"], "Category": f["Category"], "Severity": f["Severity"],
            "Title": f["Title"], "StartLine": f["StartLine"], "EndLine": f["EndLine"],
            "Code": {"Lines": out_lines}, "Match": f["Match"], "Layer": f.get("Layer", {})}


def fs_report(artifact_name, results):
    """types.Report of `trivy fs` (SchemaVersion 2, ArtifactType "filesystem")."""
    rep = {"SchemaVersion": 2, "ArtifactName": artifact_name, "ArtifactType": "filesystem",
           "Metadata": {"ImageConfig": _EMPTY_IMAGE_CONFIG}}
    res = []
    for r in results:
        d = {"Target": r["Target"], "Class": r["Class"]}
        if r["Secrets"]:
            d["Secrets"] = [_finding(f) for f in r["Secrets"]]
        res.append(d)
    if res:
        rep["Results"] = res
    return rep


def _go_string(v):
    r"""encoding/json string encoding: invalid UTF-8 -> U+FFFD, HTML-safe <, >, & and the
    line/paragraph separators escaped, control characters as \n \r \t or \u00XX."""
    if isinstance(v, (bytes, bytearray)):
        s = bytes(v).decode("utf-8", "replace")
    else:
        s = v.encode("utf-8", "surrogateescape").decode("utf-8", "replace")
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _encode(v, indent, level, out):
    pad = indent * level
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, (str, bytes, bytearray)):
        out.append(_go_string(v))
    elif isinstance(v, dict):
        if not v:
            out.append("{}")
            return
        out.append("{\n")
        items = list(v.items())
        for i, (k, x) in enumerate(items):
            out.append(pad + indent + _go_string(k) + ": ")
            _encode(x, indent, level + 1, out)
            out.append(",\n" if i + 1 < len(items) else "\n")
        out.append(pad + "}")
    elif isinstance(v, (list, tuple)):
        if not v:
            out.append("[]")
            return
        out.append("[\n")
        for i, x in enumerate(v):
            out.append(pad + indent)
            _encode(x, indent, level + 1, out)
            out.append(",\n" if i + 1 < len(v) else "\n")
        out.append(pad + "]")
    else:
        raise TypeError(type(v))


def write_json(report):
    """JSONWriter.Write: MarshalIndent(report, "", "  ") followed by a newline."""
    out = []
    _encode(report, "  ", 0, out)
    return "".join(out) + "\n"
