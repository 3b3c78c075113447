#!/bin/bash
# Build a variant librae_hip.so with extra -D flags for A/B timing (bench.py via RAE_LIB).
# usage: bash tools/build_variant.sh OUT.so [-DFLAG=V ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; shift
FLAGS=$(cd $R/relation-autoencoder_amd && python3 -c "from rae import _lib; print(' '.join(_lib.BUILD_FLAGS))")
/opt/rocm/bin/hipcc $FLAGS "$@" -DRAE_BUILD_ID=\"variant\" $R/relation-autoencoder_amd/csrc/rae.hip -o $OUT
