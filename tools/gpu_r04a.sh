set -o pipefail
bash tools/gpu_quick.sh r04a || exit $?
out=gpurun_out/r04a
echo "== kab user1000" && timeout -k 10 300 python -u tools/kab.py 1024 5 --rules user1000 > $out/kab_user1000.json 2>&1 || { tail $out/kab_user1000.json; exit 4; }
cat $out/kab_user1000.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== trace user1000" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tu -o run -- python tools/kab.py 1024 3 --rules user1000 > $out/tu.out 2>&1 || { tail $out/tu.out; exit 5; }
cut -c1-150 $out/tu/run_kernel_stats.csv
