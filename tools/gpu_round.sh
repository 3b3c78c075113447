#!/bin/bash
# One GPU-box pass: smoke, gpu tests, bench, rocprofv3 kernel-trace stats of the bench.
# usage: bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { echo tests failed; tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 300 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat
