#!/bin/bash
# Product-timing A/B: bench.py (kernel durations from dispatch-stamped events) against
# prebuilt variant libraries.   usage: [BS=batch] [CFG=c5] bash tools/gpu_libab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
i=0
for L in "$@"; do
  RAE_LIB=$R/$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps 256 --batch-size ${BS:-100} --config ${CFG:-c3} > $O/bench_$i.json 2> $O/bench_$i.err || { echo bench $L failed; tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$i.json')); print('$L', 'l=${BS:-100}', 'value', round(d['value']), 'ms/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
  i=$((i+1))
done
