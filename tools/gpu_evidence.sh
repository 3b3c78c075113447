#!/bin/bash
# Round evidence pass: tools/gpu_r2.sh (smoke, GPU tests, the driver's bench command, a long
# bench, rocprofv3 kernel stats), the PMC traffic passes, and one bench line per other config.
# usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
bash tools/gpu_r2.sh $TAG || exit 1
bash tools/gpu_pmc2.sh $TAG/pmc c3 || exit 1
cd $R
for C in c2 c5 c4; do
  timeout -k 10 400 python3 -u bench.py --config $C --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_$C.json 2> $O/bench_$C.err || { echo bench $C failed; tail -20 $O/bench_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$C.json')); print('$C', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
