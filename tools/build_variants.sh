# Build measurement variants of libtrivy_secret.so: the same sources with other compile-time
# settings (select one with TSG_LIB_VARIANT=<name>).  Every variant computes the same results.
# (Round 4's K1X verify bisection used part-timing builds that computed wrong results; they
# are not kept in the product source: profiles/r04/xv/ holds their timings.)
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
    legacy) build $v -DK1_LEGACY ;;      # K1: the legacy layout (class words, index rows)
    u16) build $v -DK1_UNROLL=16 ;;      # K1: bytes unrolled per word
    u4) build $v -DK1_UNROLL=4 ;;
    ns3) build $v -DK1_CHAINS=3 ;;       # K1: chains per lane
    ns4) build $v -DK1_CHAINS=4 ;;
    k2ctr) build $v -DK2_TRACE_CTR ;;    # K2: per-entry counters (TSG_K2_TRACE)
    k2noinl) build $v -DK2_NOINL ;;      # K2: rare paths out of line
    k2w4) build $v -DK2_W=4 ;;           # K2: at least 4 waves per SIMD (<= 128 VGPRs, 38 spilled)
    x1) build $v -DK1X_WORDS=1 ;;        # K1X: words per lane per round
    x8) build $v -DK1X_WORDS=8 ;;
    xdiag) build $v -DK1X_DIAG ;;
    f16) build $v -DK1F_ALL16=1 ;;       # K1F: all 16 entries of a tile read at once
    fq64) build $v -DK1F_QUEUE=64 ;;     # K1F: the register queue with the small verification ring
    ftr) build $v -DK1F_WTRACE=1 ;;      # K1F: per-wave trace (TSG_K1F_TRACE, tools/k1ftrace.py)
    ftr0) build $v -DK1F_WTRACE=1 -DK1F_SHARES=0 ;;  # the same with equal wave ranges
    fe) build $v -DK1F_SHARES=0 ;;       # K1F: equal wave ranges
    fs8) build $v -DK1F_STEAL=8 ;;       # K1F: reserve 1/8 of a block's tiles, claimed in chunks
    fs16) build $v -DK1F_STEAL=16 ;;     # K1F: reserve 1/16 of a block's tiles
    fs4) build $v -DK1F_STEAL=4 ;;       # K1F: reserve 1/4
    fc16) build $v -DK1F_STEAL=8 -DK1F_STEAL_CHUNK=16 ;;  # K1F: 16-tile reserve chunks
    fc4) build $v -DK1F_STEAL=8 -DK1F_STEAL_CHUNK=4 ;;
    gs1) build $v -DGATES_STAMPS=0xFFFFFFFFu ;;  # gates: every block stamps the chain's start
    fnoend) build $v -DK1F_NO_END_ATOMICS=1 ;;  # K1F: no block-end counters / stamp (timing probe; stats read 0)
    ib0) build $v -DITEMS_BASE_IN_COUNT=0 ;;  # items: the emit pass reserves the blocks' ranges
    fd2) build $v -DK1F_DEPTH=2 ;;       # K1F: register queue depths
    fd3) build $v -DK1F_DEPTH=3 ;;        # K1X: verify counters in k2_long_tails (slot probes),
                                         # k2_tail_bytes (entries examined), k2_tail_max (matches)
  esac
done
