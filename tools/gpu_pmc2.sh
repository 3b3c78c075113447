#!/bin/bash
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE in separate runs) of bench.py INCLUDING the
# labelling pass and the STREAM copy (the copy's known bytes calibrate the FETCH_SIZE factor).
# usage: [BX="--batch-size 800"] bash tools/gpu_pmc2.sh TAG CONFIG
set -o pipefail
TAG=${1:-pmc}; CFG=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BA="--config $CFG --steps 64 --warmup 16 --no-cpu-baseline --kernel-iters 32 ${BX:-}"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $R/bench.py $BA > $O/fetch.log 2>&1 || { echo fetch pass failed; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 $R/bench.py $BA > $O/write.log 2>&1 || { echo write pass failed; tail -20 $O/write.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/fetch $O/write --config $CFG ${BX:-} --out $O/pmc_traffic.json || exit 1
