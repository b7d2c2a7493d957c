"""The secret part of trivy's RPC layer: the protobuf messages of
rpc/common/service.proto:117-121 (Layer), :145-158 (Line, Code) and :160-177
(SecretFinding, Secret), and the converters of pkg/rpc/convert.go between them and the
secret dicts of trivy_amd.secret (Go's types.Secret shape):

  ConvertToRPCCode / ConvertFromRPCCode                 convert.go:63-80, :285-302
  ConvertToRPCSecrets / ConvertToRPCSecretFindings      convert.go:82-110
  ConvertFromRPCSecretFindings / ConvertFromRPCSecrets  convert.go:304-335
  ConvertToRPCLayer / ConvertFromRPCLayer               convert.go:230-236, :419-427

What a client/server `trivy` pair sends for secrets, so results of this scanner can cross
the reference's RPC boundary unchanged.  The message classes are built at import from a
descriptor written here (no protoc in this image); field numbers and types follow the
.proto, so the wire bytes are the reference's.

Go behaviour kept:
  * ConvertToRPC* always sets Code and Layer (non-nil pointers), so they are present on the
    wire even when empty;
  * ConvertFromRPCSecretFindings copies Layer.CreatedBy, ConvertFromRPCLayer does not;
  * a nil Code or Layer on a received finding dereferences nil in Go (a panic): here
    ValueError;
  * proto3 `string` fields must be valid UTF-8 (protobuf-go refuses to marshal otherwise):
    a Match or line Content that is not raises ValueError here;
  * int32 conversions wrap like Go's int32(x).
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="trivy_amd/rpc/common_secret.proto",
                                            package="trivy.common", syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = ".trivy.common." + tname
        return m

    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    S, I32, B, M = _F.TYPE_STRING, _F.TYPE_INT32, _F.TYPE_BOOL, _F.TYPE_MESSAGE
    msg("Layer", [("digest", 1, S, opt, None), ("diff_id", 2, S, opt, None),
                  ("created_by", 3, S, opt, None)])
    msg("Line", [("number", 1, I32, opt, None), ("content", 2, S, opt, None),
                 ("is_cause", 3, B, opt, None), ("annotation", 4, S, opt, None),
                 ("truncated", 5, B, opt, None), ("highlighted", 6, S, opt, None),
                 ("first_cause", 7, B, opt, None), ("last_cause", 8, B, opt, None)])
    msg("Code", [("lines", 1, M, rep, "Line")])
    sf = msg("SecretFinding", [("rule_id", 1, S, opt, None), ("category", 2, S, opt, None),
                               ("severity", 3, S, opt, None), ("title", 4, S, opt, None),
                               ("start_line", 5, I32, opt, None), ("end_line", 6, I32, opt, None),
                               ("code", 7, M, opt, "Code"), ("match", 8, S, opt, None),
                               ("layer", 10, M, opt, "Layer")])
    sf.reserved_range.add(start=9, end=10)  # deprecated 'deleted'
    msg("Secret", [("filepath", 1, S, opt, None), ("findings", 2, M, rep, "SecretFinding")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = getattr(message_factory, "GetMessageClass", None)
    out = {}
    for name in ("Layer", "Line", "Code", "SecretFinding", "Secret"):
        d = pool.FindMessageTypeByName("trivy.common." + name)
        out[name] = get(d) if get else message_factory.MessageFactory(pool).GetPrototype(d)
    return out


_M = _build()
Layer, Line, Code, SecretFinding, Secret = (_M[k] for k in ("Layer", "Line", "Code", "SecretFinding", "Secret"))


def _int32(x):
    x = int(x) & 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def _str(v, what):
    """A Go string (bytes or str) as a proto3 string: valid UTF-8 or ValueError."""
    if isinstance(v, (bytes, bytearray)):
        try:
            return bytes(v).decode("utf-8")
        except UnicodeDecodeError as e:
            raise ValueError("proto: %s contains invalid UTF-8" % what) from e
    try:
        v.encode("utf-8")
    except UnicodeEncodeError as e:  # (surrogate-escaped bytes)
        raise ValueError("proto: %s contains invalid UTF-8" % what) from e
    return v


def ConvertToRPCCode(code):
    """convert.go:63-80: &common.Code{Lines: ...} (never nil)."""
    out = Code()
    for ln in (code or {}).get("Lines") or []:
        out.lines.add(number=_int32(ln["Number"]), content=_str(ln["Content"], "Line.content"),
                      is_cause=bool(ln["IsCause"]), annotation=_str(ln.get("Annotation", ""), "Line.annotation"),
                      truncated=bool(ln.get("Truncated", False)),
                      highlighted=_str(ln.get("Highlighted", ""), "Line.highlighted"),
                      first_cause=bool(ln["FirstCause"]), last_cause=bool(ln["LastCause"]))
    return out


def ConvertToRPCLayer(layer):
    """convert.go:230-236: &common.Layer{Digest, DiffId, CreatedBy} (never nil)."""
    layer = layer or {}
    return Layer(digest=layer.get("Digest", ""), diff_id=layer.get("DiffID", ""),
                 created_by=layer.get("CreatedBy", ""))


def ConvertToRPCSecretFindings(findings):
    """convert.go:93-110."""
    out = []
    for f in findings or []:
        m = SecretFinding(rule_id=f["RuleID"], category=str(f["Category"]), severity=f["Severity"],
                          title=f["Title"], end_line=_int32(f["EndLine"]), start_line=_int32(f["StartLine"]),
                          match=_str(f["Match"], "SecretFinding.match"))
        m.code.CopyFrom(ConvertToRPCCode(f.get("Code")))
        m.code.SetInParent()  # (present even with no lines, like Go's non-nil pointer)
        m.layer.CopyFrom(ConvertToRPCLayer(f.get("Layer")))
        m.layer.SetInParent()
        out.append(m)
    return out


def ConvertToRPCSecrets(secrets):
    """convert.go:82-91: []*common.Secret{Filepath, Findings}."""
    out = []
    for s in secrets or []:
        m = Secret(filepath=s["FilePath"])
        m.findings.extend(ConvertToRPCSecretFindings(s["Findings"]))
        out.append(m)
    return out


def ConvertFromRPCCode(rpc_code):
    """convert.go:285-302; lines come back as str (Go strings).  A nil Code panics in Go."""
    if rpc_code is None:
        raise ValueError("nil Code (a nil pointer dereference in convert.go:287)")
    lines = [{"Number": int(ln.number), "Content": ln.content, "IsCause": ln.is_cause, "Annotation": ln.annotation,
              "Truncated": ln.truncated, "Highlighted": ln.highlighted, "FirstCause": ln.first_cause,
              "LastCause": ln.last_cause} for ln in rpc_code.lines]
    return {"Lines": lines or None}


def ConvertFromRPCLayer(rpc_layer):
    """convert.go:419-427: Digest and DiffID only (CreatedBy is not copied)."""
    d = {}
    if rpc_layer is not None:
        if rpc_layer.digest:
            d["Digest"] = rpc_layer.digest
        if rpc_layer.diff_id:
            d["DiffID"] = rpc_layer.diff_id
    return d


def ConvertFromRPCSecretFindings(rpc_findings):
    """convert.go:304-324 (Layer with CreatedBy, built inline)."""
    out = []
    for f in rpc_findings or []:
        if not f.HasField("code"):
            raise ValueError("nil Code (a nil pointer dereference in convert.go:287)")
        if not f.HasField("layer"):
            raise ValueError("nil Layer (a nil pointer dereference in convert.go:316)")
        lay = {}
        for k, v in (("Digest", f.layer.digest), ("DiffID", f.layer.diff_id), ("CreatedBy", f.layer.created_by)):
            if v:
                lay[k] = v
        out.append({"RuleID": f.rule_id, "Category": f.category, "Severity": f.severity, "Title": f.title,
                    "StartLine": int(f.start_line), "EndLine": int(f.end_line), "Code": ConvertFromRPCCode(f.code),
                    "Match": f.match, "Layer": lay})
    return out or None


def ConvertFromRPCSecrets(rpc_secrets):
    """convert.go:326-335."""
    out = [{"FilePath": s.filepath, "Findings": ConvertFromRPCSecretFindings(s.findings)} for s in rpc_secrets or []]
    return out or None
