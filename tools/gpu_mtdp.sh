#!/bin/bash
# C5: bilinear GPU tests, then the bench with dP in the M-tile pass (default) and with k_bil_dp2.
set -o pipefail
O=gpurun_out/${1:-mtdp}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rescal or hybrid or bil or bf16" > $O/gputests.log 2>&1 || { echo tests failed; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for v in 1 0 1 0; do
  RAE_MTDP=$v timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_$v.json 2> $O/bench_$v.err || { echo bench failed; tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('RAE_MTDP=$v', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
