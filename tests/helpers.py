"""Shared test helpers: canonical JSON-able form of types.Secret values."""
import json
import os

from tests.conftest import GOLDEN


def _s(v):
    if isinstance(v, (bytes, bytearray)):
        return bytes(v).decode("utf-8", "surrogateescape")
    return v


def canon_secret(sec):
    if sec is None:
        return None
    fs = sec.get("Findings")
    out = {"FilePath": sec.get("FilePath", ""), "Findings": None}
    if fs is not None:
        out["Findings"] = []
        for f in fs:
            lines = f["Code"]["Lines"]
            out["Findings"].append({
                "RuleID": f["RuleID"], "Category": f["Category"], "Severity": f["Severity"],
                "Title": f["Title"], "StartLine": f["StartLine"], "EndLine": f["EndLine"],
                "Code": {"Lines": None if lines is None else [
                    {"Number": ln["Number"], "Content": _s(ln["Content"]),
                     "IsCause": ln["IsCause"], "Annotation": ln.get("Annotation", ""),
                     "Truncated": ln.get("Truncated", False),
                     "Highlighted": _s(ln["Highlighted"]), "FirstCause": ln["FirstCause"],
                     "LastCause": ln["LastCause"]} for ln in lines]},
                "Match": _s(f["Match"])})
    return out


def reference_cases():
    with open(os.path.join(GOLDEN, "reference_cases.json")) as f:
        return json.load(f)
