#!/bin/bash
# Default bench line + rocprofv3 kernel-trace stats of the same command (the profile the
# bench's per-kernel durations must agree with).   usage: bash tools/gpu_bench_prof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-bp}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py "$@" > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
head -4 $O/prof/run_kernel_stats.csv
python3 -c "
import json; d=json.load(open('$O/prof_bench.json')); print('under rocprof: value', d['value'], d['kernel_us'])"
