#!/bin/bash
# fs ingest floor on the GPU box's host: the e2e tree, then tools/fs_read_floor at 16 threads
set -o pipefail
out=gpurun_out/${1:-fsfloor}
mkdir -p $out
g++ -O2 -o /tmp/fs_read_floor tools/fs_read_floor.cpp -lpthread || exit 2
python -c "from trivy_amd import configs; configs.source_tree('/tmp/tsg_floor/tree', 200 << 20, seed=1)" || exit 3
for m in 0 1 2; do timeout -k 5 60 /tmp/fs_read_floor /tmp/tsg_floor/tree 16 $m | tail -2; done | tee $out/floor.txt
