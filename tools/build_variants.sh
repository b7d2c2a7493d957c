# Build measurement variants of libtrivy_secret.so: the same sources with other K1
# compile-time settings (tools/k1sweep.py with TSG_LIB_VARIANT=<name>).
set -e
cd "$(dirname "$0")/.."
python -m trivy_amd.build
build() {
  name=$1; shift
  mkdir -p /tmp/tsgv_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -fPIC "$@" -Iinclude -c trivy_amd/csrc/gpu.hip -o /tmp/tsgv_$name/gpu.o
  objs=$(ls trivy_amd/build/*.o | grep -v gpu.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o trivy_amd/libtrivy_secret_$name.so $objs /tmp/tsgv_$name/gpu.o -lpthread
}
for v in "$@"; do
  case $v in
    pf*) build $v -DK1_PF=${v#pf} ;;
    nolds) build $v -DK1_EXP_NO_CLS -DK1_EXP_NO_TAB ;;
    coal) build $v -DK1_EXP_COAL ;;
    coalnolds) build $v -DK1_EXP_COAL -DK1_EXP_NO_CLS -DK1_EXP_NO_TAB ;;
    noruns) build $v -DK1_EXP_NO_RUNS ;;
    coalnoruns) build $v -DK1_EXP_COAL -DK1_EXP_NO_RUNS ;;
    nocls) build $v -DK1_EXP_NO_CLS ;;
  esac
done
