# Build measurement variants of libtrivy_secret.so: the same sources with other K1
# compile-time settings (select one with TSG_LIB_VARIANT=<name>, e.g. tools/gpu_sweep.sh).
#   usage: tools/build_variants.sh NAME...
set -e
cd "$(dirname "$0")/.."
python -m trivy_amd.build
build() {
  name=$1; shift
  mkdir -p /tmp/tsgv_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -Iinclude \
    -c trivy_amd/csrc/kernels.hip -o /tmp/tsgv_$name/kernels.o
  objs=$(ls trivy_amd/build/*.o | grep -v kernels.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o trivy_amd/libtrivy_secret_$name.so $objs /tmp/tsgv_$name/kernels.o -lpthread
}
for v in "$@"; do
  case $v in
    ob4w4) build $v -DK1_UNROLL=4 ;;
    nolds) build $v -DK1_EXP_NO_CLS -DK1_EXP_NO_TAB ;;
    noruns) build $v -DK1_EXP_NO_RUNS ;;
    nocls) build $v -DK1_EXP_NO_CLS ;;
    notab) build $v -DK1_EXP_NO_TAB ;;
    k2ctr) build $v -DK2_TRACE_CTR ;;
    coal) build $v -DK1_EXP_COAL ;;
    clspf8) build $v -DK1_CLSPF=8 ;;
    clspf8_ip) build $v -DK1_CLSPF=8 -DK1_INPLACE ;;
    clspf4) build $v -DK1_CLSPF=4 ;;
    clspf4_ip) build $v -DK1_CLSPF=4 -DK1_INPLACE ;;
    inplace) build $v -DK1_INPLACE ;;
    u4) build $v -DK1_UNROLL=4 ;;
    k2twobuf) build $v -DK2_TWOBUF ;;
    x1) build $v -DK1X_WORDS=1 ;;
    x8) build $v -DK1X_WORDS=8 ;;
    nostep) build $v -DK1_EXP_NOSTEP ;;
    noload) build $v -DK1_EXP_NOLOAD ;;
    noload_nolds) build $v -DK1_EXP_NOLOAD -DK1_EXP_NO_CLS -DK1_EXP_NO_TAB ;;
    nolds_coal) build $v -DK1_EXP_NO_CLS -DK1_EXP_NO_TAB -DK1_EXP_COAL ;;
  esac
done
