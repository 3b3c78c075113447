#!/bin/bash
# C5: bilinear GPU tests, two bench lines, rocprof kernel stats.   usage: bash tools/gpu_c5quick.sh TAG
set -o pipefail
O=gpurun_out/${1:-c5q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rescal or hybrid or bil or bf16 or bitwise" > $O/gputests.log 2>&1 || { echo tests failed; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for v in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_$v.json 2> $O/bench_$v.err || { echo bench failed; tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('c5', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof -o run -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $R/$O/prof.log 2>&1 || { echo prof failed; exit 1; }
find $R/$O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-110 | head -10
