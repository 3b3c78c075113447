#!/bin/bash
# Quick forward iteration: phase stamps (diag build) + C3 bench priv_rows auto / off.
set -o pipefail
TAG=${1:-s5q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "${STAMPS:-1}" ]; then
  timeout -k 10 200 python3 -u tools/phase_stamps.py --config c3 > $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
  grep -v amdgpu.ids $O/stamps.log | head -8
fi
for f in auto off auto; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps 256 --kernel-form priv_rows=$f > $O/bench_$f.json 2> $O/bench_$f.err || { echo bench failed; tail -20 $O/bench_$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$f.json')); print('priv_rows=$f', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
