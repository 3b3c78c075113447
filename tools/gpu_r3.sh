#!/bin/bash
# Round-3 GPU pass: smoke, every -m gpu test (verbose, bf16 tolerance report), the default
# bench line, rocprofv3 kernel-trace stats of the same bench.   usage: bash tools/gpu_r3.sh TAG [bench args]
set -o pipefail
TAG=${1:-r3}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --maxfail=6 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/gputests.log | tail -15
grep -E "^(rescal|c5|hybrid)" $O/gputests.log | head -20
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 400 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernel_us'], d['roofline']['kernel'], d['roofline']['frac'], 'cpu', d.get('cpu_baseline',{}).get('runs'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
head -8 $O/prof/run_kernel_stats.csv
