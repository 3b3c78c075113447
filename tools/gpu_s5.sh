#!/bin/bash
# Session-5 pass: the GPU tests selected by K (pytest -k; K=none skips them), then the C3 forward /
# update phase stamps of a diagnostic build (extra -D flags in RAE_VARIANT), then the bench A/B
# of the product library against variant libraries.   usage: [K=expr] [STAMPS=1] bash tools/gpu_s5.sh TAG [lib.so ...]
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
[ $# -gt 0 ] && bash tools/gpu_libab.sh $TAG/ab relation-autoencoder_amd/rae/librae_hip.so "$@"
exit 0
