#!/bin/bash
# Round-6 A/B of kernel forms on one config: bench line + rocprofv3 kernel stats per form.
#   usage: bash tools/gpu_ab6.sh TAG CONFIG FORM [FORM ...]    (FORM: key=value or "default")
set -o pipefail
TAG=$1; C=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for f in "$@"; do
  kf=""; [ "$f" != default ] && kf="--kernel-form $f"
  t=$(echo $f | tr -c 'a-zA-Z0-9' _)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/ab_${C}_$t -o run \
    -- python3 $R/bench.py --config $C --no-cpu-baseline --no-label-pass $kf > $O/ab_${C}_$t.json 2> $O/ab_${C}_$t.err) \
    || { echo "ab $C $f failed"; tail -20 $O/ab_${C}_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab_${C}_$t.json'))
print('$C $f', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
  cut -d, -f1,2,4 $O/ab_${C}_$t/run_kernel_stats.csv | head -9 | cut -c1-110
done
echo ALL_OK
