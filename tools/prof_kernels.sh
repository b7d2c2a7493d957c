set -e

mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 tools/kprof.py 1 2 > gpurun_out/prof/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/prof/p1 -o p1 --output-format csv -- python3 tools/kprof.py 1 1 > gpurun_out/prof/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/p2 -o p2 --output-format csv -- python3 tools/kprof.py 1 1 > gpurun_out/prof/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof/p3 -o p3 --output-format csv -- python3 tools/kprof.py 1 1 > gpurun_out/prof/p3.log 2>&1
ls -R gpurun_out/prof | head -30
