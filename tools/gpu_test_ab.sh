#!/bin/bash
# GPU tests of the in-tree library, then a product-timing A/B of prebuilt variant libraries at
# several batch sizes.   usage: [CFG=c3] [BSS="100 800"] bash tools/gpu_test_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gputests.log 2>&1 || { echo tests failed; tail -60 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
for BS in ${BSS:-100 800}; do
  BS=$BS CFG=${CFG:-c3} bash tools/gpu_libab.sh $TAG/l$BS "$@" || exit 1
done
