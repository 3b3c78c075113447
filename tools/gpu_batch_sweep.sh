#!/bin/bash
# Single-GPU batch sweep: how forward / update / step time grow with the batch, the data
# behind the data-parallel scaling estimate (the update runs over the GLOBAL batch G*l).
# usage: bash tools/gpu_batch_sweep.sh TAG [batch sizes...]
set -o pipefail
TAG=${1:-sweep}; shift
SIZES=${@:-200 400 800}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for b in $SIZES; do
  EXTRA=""; [ $b -ge 4096 ] && EXTRA="--steps 64 --warmup 16"     # an epoch has N/b batches
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-label-pass --batch-size $b $EXTRA \
      > $O/bench_l$b.json 2> $O/bench_l$b.err || { echo bench l=$b failed; tail -20 $O/bench_l$b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_l$b.json'))
print('l=$b value', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
