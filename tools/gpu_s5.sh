#!/bin/bash
# Session-5 pass: the GPU tests selected by K (pytest -k; K=none skips them), then the C3 forward /
# update phase stamps of a diagnostic build (extra -D flags in RAE_VARIANT), then the bench A/B
# of the product library against variant libraries.   usage: [K=expr] [STAMPS=1] [CFG=c5] bash tools/gpu_s5.sh TAG [lib.so ...]
set -o pipefail
TAG=${1:-s5}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "${K:-}" != "none" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/gputests.log 2>&1 || { echo gpu tests failed; tail -40 $O/gputests.log; exit 1; }
  tail -3 $O/gputests.log
fi
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 200 python3 -u tools/phase_stamps.py --config c3 > $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
  grep -v amdgpu.ids $O/stamps.log
fi
if [ -n "${CFG:-}" ]; then      # the bench line of one config + rocprofv3 kernel stats of it
  timeout -k 10 300 python3 -u bench.py --config $CFG --no-cpu-baseline --no-label-pass --steps 256 > $O/bench_$CFG.json 2> $O/bench_$CFG.err || { echo bench failed; tail -20 $O/bench_$CFG.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$CFG.json')); print('$CFG', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$CFG -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $O/prof_$CFG.json 2> $O/prof_$CFG.err || { echo prof failed; tail -20 $O/prof_$CFG.err; exit 1; }
  cut -c1-120 $O/prof_$CFG/run_kernel_stats.csv | head -12
  cd $R
fi
[ $# -gt 0 ] && bash tools/gpu_libab.sh $TAG/ab relation-autoencoder_amd/rae/librae_hip.so "$@"
exit 0
