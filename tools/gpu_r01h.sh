set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/kbench.py 4 256 > gpurun_out/kb_wide.log 2>&1
TSG_K1_NARROW=1 timeout -k 10 300 python -u tools/kbench.py 4 256 > gpurun_out/kb_narrow.log 2>&1
TSG_K1_GRID=16 timeout -k 10 300 python -u tools/kbench.py 4 256 > gpurun_out/kb_wide_g16.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pw -o pw --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/pw.log 2>&1
TSG_K1_NARROW=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pn -o pn --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/pn.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/prof/ps -o ps --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/ps.log 2>&1
