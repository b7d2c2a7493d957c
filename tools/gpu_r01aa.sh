set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/k1sweep.py 4 cls16 > gpurun_out/k1sweep.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES -d gpurun_out/prof/ps3 -o ps3 --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/ps3.log 2>&1
