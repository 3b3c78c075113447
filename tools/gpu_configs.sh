#!/bin/bash
# Bench lines for the other BASELINE.json configs on one GPU (C2, C5, and C4's shape at l=100).
# usage: bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-configs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in c2 c5 c4; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --steps 256 > $O/bench_$c.json 2> $O/bench_$c.err || { echo bench $c failed; tail -20 $O/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$c.json'))
print('$c', round(d['value']), 'ex/s', round(d['ms_per_step']*1e3, 2), 'us/step', d['roofline']['kernel'], round(d['roofline']['frac'], 3), {k: round(v, 2) for k, v in d['kernel_us'].items()}, 'label', d['label_pass'] and round(d['label_pass']['frac'], 3), 'copy', d['hbm_copy'] and round(d['hbm_copy']['GBs']))"
done
