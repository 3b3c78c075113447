#!/bin/bash
# Session-4 pass: the GPU tests (K = pytest -k expression, default all), then the bench A/B of
# the product library against variant libraries.   usage: [K=expr] bash tools/gpu_s4.sh TAG [lib.so ...]
set -o pipefail
TAG=${1:-s4}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "${K:-}" != "none" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/gputests.log 2>&1 || { echo gpu tests failed; tail -40 $O/gputests.log; exit 1; }
  tail -3 $O/gputests.log
fi
[ $# -gt 0 ] && bash tools/gpu_libab.sh $TAG/ab relation-autoencoder_amd/rae/librae_hip.so "$@"
exit 0
