#!/bin/bash
# PMC passes (one counter group per run, as MI355X_MICROARCH.md prescribes) + phase stamps.
# usage: bash tools/gpu_pmc.sh TAG CONFIG [bench args...]
set -o pipefail
TAG=${1:-pmc}; CFG=${2:-c3}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BA="--config $CFG --steps 64 --warmup 16 --no-cpu-baseline --no-label-pass --kernel-iters 32 $@"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $R/bench.py $BA > $O/fetch.log 2>&1 || { echo fetch pass failed; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 $R/bench.py $BA > $O/write.log 2>&1 || { echo write pass failed; tail -20 $O/write.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/fetch $O/write --config $CFG --out $O/pmc_traffic.json || exit 1
timeout -k 10 180 python3 -u tools/phase_stamps.py --config $CFG > $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
