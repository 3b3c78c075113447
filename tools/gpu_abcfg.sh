#!/bin/bash
# bench A/B of variant libraries over several configs.   usage: bash tools/gpu_abcfg.sh TAG "c2 c4 c3" lib1.so ...
set -o pipefail
TAG=$1; CFGS=$2; shift 2
for c in $CFGS; do CFG=$c bash tools/gpu_libab.sh $TAG/$c "$@" | sed "s/^/$c /" || exit 1; done
