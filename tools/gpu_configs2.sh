#!/bin/bash
# Every GPU test, then one bench line per BASELINE config (C3 at the driver's 20 steps).
# usage: bash tools/gpu_configs2.sh TAG
set -o pipefail
TAG=${1:-cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/gputests.log 2>&1 || { echo tests failed; tail -60 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench c3 failed; tail -20 $O/bench_c3.err; exit 1; }
for C in c2 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $C --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_$C.json 2> $O/bench_$C.err || { echo bench $C failed; tail -20 $O/bench_$C.err; exit 1; }
done
for C in c3 c2 c4 c5; do
  python3 -c "import json; d=json.load(open('$O/bench_$C.json')); print('$C', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
