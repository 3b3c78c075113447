#!/bin/bash
# Full -m gpu suite on the in-tree library, then a bench A/B over prebuilt variant libraries.
# usage: [CFG=c5] bash tools/gpu_testab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 || { echo tests failed; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
bash $R/tools/gpu_libab.sh $TAG "$@"
