#!/bin/bash
# A/B of bench.py over (environment, library) variants, repeated in rotation.
# usage: [BS=batch] [CFG=c3] [REP=2] bash tools/gpu_envab.sh TAG "ENV=V;lib.so" "ENV=V;lib.so" ...
# (an empty lib part means the product library; ENV may be empty)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
n=0
for rep in $(seq ${REP:-2}); do
  for v in "$@"; do
    E=${v%%;*}; L=${v#*;}
    if [ -n "$L" ]; then LE="RAE_LIB=$R/$L"; else LE=""; fi
    env $E $LE timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps ${STEPS:-256} --warmup 32 --batch-size ${BS:-100} --config ${CFG:-c3} > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench [$v] failed"; tail -20 $O/bench_$n.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/bench_$n.json')); print('[$v]', 'l=${BS:-100}', 'value', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
    n=$((n+1))
  done
done
