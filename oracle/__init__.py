"""CPU oracle for trivy's secret-scan hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-Python restatement of the reference algorithm
(`pkg/fanal/secret/scanner.go`, `pkg/fanal/analyzer/secret/secret.go`,
`pkg/fanal/utils/utils.go`) and of the Go 1.19 standard-library semantics it
depends on (`regexp`, `bytes.ToLower`, `unicode.SimpleFold`, `sort.Slice`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import it, and only as the checker / the timed CPU baseline.  The product path
(`trivy_amd`) never imports anything from here.

Parity pin: the oracle is checked against every fixture the reference's own
tests hold for this path (tests/golden/reference_cases.json, extracted from
`pkg/fanal/secret/scanner_test.go:24-765`,
`pkg/fanal/analyzer/secret/secret_test.go:16-223` and
`integration/testdata/secrets.json.golden`).  Behaviour those fixtures do not
cover (non-ASCII folding, invalid UTF-8, sort ties > 12) follows the Go 1.19
documentation/source structure and is labelled "derived" in the tests.
"""
