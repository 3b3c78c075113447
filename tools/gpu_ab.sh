#!/bin/bash
# A/B diagnostic pass: phase stamps for each variant library, then a short bench of the
# product library.   usage: bash tools/gpu_ab.sh TAG "VARIANT1" "VARIANT2" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
i=0
for v in "$@"; do
  echo "=== variant [$v]" | tee -a $O/stamps.log
  RAE_VARIANT="$v" timeout -k 10 150 python3 -u tools/phase_stamps.py --config c3 >> $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
  i=$((i+1))
done
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernel_us'])"
