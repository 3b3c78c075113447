#!/bin/bash
# Private-rows pass: every GPU test, then C3 bench lines with priv_rows auto / off (256 steps).
set -o pipefail
TAG=${1:-s5p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo gpu tests failed; tail -60 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
for f in auto off auto off; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps 256 --kernel-form priv_rows=$f > $O/bench_$f.json 2> $O/bench_$f.err || { echo bench failed; tail -20 $O/bench_$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$f.json')); print('priv_rows=$f', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, d['config']['kernel_forms'])"
done
[ $# -gt 1 ] && shift && bash tools/gpu_libab.sh $TAG/ab relation-autoencoder_amd/rae/librae_hip.so "$@"
exit 0
