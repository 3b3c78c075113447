#!/bin/bash
# C5 (RESCAL, bf16 MFMA): GPU tests, a bench line and rocprofv3 kernel stats of the C5 bench.
# usage: bash tools/gpu_c5.sh TAG
set -o pipefail
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gputests.log 2>&1 || { echo tests failed; tail -60 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 256 --warmup 32 > $O/bench_c5.json 2> $O/bench_c5.err || { echo bench failed; tail -20 $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, d['roofline'].get('frac'), d['roofline'].get('frac_of_measured_peak'), d.get('mfma_bf16_peak'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -20
