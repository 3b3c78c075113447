#!/bin/bash
# GPU tests (parity) + phase stamps + short bench.   usage: bash tools/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=$1; K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > $O/gputests.log 2>&1 || { echo tests failed; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 150 python3 -u tools/phase_stamps.py --config c3 > $O/stamps.log 2>&1 || { echo stamps failed; tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-label-pass > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernel_us'])"
