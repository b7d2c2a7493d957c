"""MI355X-native engine for trivy's secret-scan hot path (pkg/fanal/secret Scanner.Scan).

Public API mirrors the reference (trivy_amd.secret, trivy_amd.analyzer); the compute
lives in libtrivy_secret.so (include/trivy_secret.h): Go-regexp engine, DFA compiler,
exact resolver and the gfx950 kernels.
"""
