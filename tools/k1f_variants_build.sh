#!/bin/bash
# Measurement variants of K1F for tools/gpu_k1f_variants.sh (profiles/r05/kv1): patched copies of
# kernels.hip built under /tmp; all but the default compute WRONG results (timing only).
# measurement variants of K1F (results NOT exact for most): built from a patched copy of kernels.hip
set -e
cd /root/repo
python -m trivy_amd.build >/dev/null
objs=$(ls trivy_amd/build/*.o | grep -v kernels.hip.o)
build() {
  name=$1; pyexpr=$2
  mkdir -p /tmp/kv/$name
  python3 - "$pyexpr" > /tmp/kv/$name/kernels.hip <<'PY'
import sys
s = open('/root/repo/trivy_amd/csrc/kernels.hip').read()
exec(sys.argv[1])
sys.stdout.write(s)
PY

  /opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -fPIC -Wno-unused-function -Iinclude -I/root/repo/trivy_amd/csrc \
    -c /tmp/kv/$name/kernels.hip -o /tmp/kv/$name/kernels.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o trivy_amd/libtrivy_secret_$name.so $objs /tmp/kv/$name/kernels.o -lpthread
  echo built $name
}
# no verification (the drain is a no-op)
build nover "s = s.replace('      L.verify(x.x, x.y & 0xFu, x.y >> 16, narr);', '      (void)x;')" &
# no run events and no listing: tile() only
build tileonly "s = s.replace('    if (__builtin_expect(bu | bd, 0)) {', '    if (__builtin_expect(bu | bd, 0) && A.total == 7) {').replace('    if (__builtin_expect(hb != 0, 0)) {', '    if (__builtin_expect(hb != 0, 0) && A.total == 7) {')" &
# loads only: the tile is an XOR of the word (LDS untouched)
build loadonly "s = s.replace('    const uint32_t rb = L.tile(v, cy, g);', '    g[0] = v.x ^ v.y; g[1] = v.z ^ v.w; g[2] = 0; g[3] = 0; const uint32_t rb = (v.x == 0x12345678u) ? 1u : 0u;').replace('    if (__builtin_expect(hb != 0, 0)) {', '    if (__builtin_expect(hb != 0, 0) && A.total == 7) {')" &
# LDS lookups kept, no R / flags / runs: OR of the 16 entries
build ldsonly "s = s.replace('    const uint32_t ao = k1f_and3(e[13].x, e[14].y, e[15].z), bo = e[14].x & e[15].y, co = e[15].x;', '    uint32_t acc = 0;\n#pragma unroll\n    for (int k = 0; k < 16; k++) acc ^= e[k].x ^ e[k].y ^ e[k].z ^ e[k].w;\n    g[0] = acc; g[1] = g[2] = g[3] = 0;\n    return acc == 0x12345678u ? 1u : 0u;\n    const uint32_t ao = k1f_and3(e[13].x, e[14].y, e[15].z), bo = e[14].x & e[15].y, co = e[15].x;').replace('    if (__builtin_expect(hb != 0, 0)) {', '    if (__builtin_expect(hb != 0, 0) && A.total == 7) {')" &
wait
