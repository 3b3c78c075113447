#!/bin/bash
# Round evidence pass: tools/gpu_r2.sh (smoke, GPU tests, the driver's bench command, a long
# bench, rocprofv3 kernel stats), the PMC traffic passes, and one bench line per other config.
# usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
bash tools/gpu_r2.sh $TAG || exit 1
bash tools/gpu_pmc2.sh $TAG/pmc c3 || exit 1
BX="--batch-size 800 --no-label-pass" bash tools/gpu_pmc2.sh $TAG/pmc800 c3 || exit 1
cd $R
for C in c2 c5 c4; do
  timeout -k 10 400 python3 -u bench.py --config $C --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_$C.json 2> $O/bench_$C.err || { echo bench $C failed; tail -20 $O/bench_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$C.json')); print('$C', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
# C5 MFMA utilisation: one PMC pass (2 SQ + 1 GRBM counters) + the kernel stats of the same
# command for the span-based figure
mkdir -p $O/c5mfma && cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/c5mfma/pmc -o run -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $O/c5mfma/pmc.log 2>&1 || { echo c5 mfma pass failed; tail -20 $O/c5mfma/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c5mfma/stats -o run -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $O/c5mfma/stats.log 2>&1 || { echo c5 stats failed; tail -20 $O/c5mfma/stats.log; exit 1; }
cd $R
python3 tools/pmc_mfma.py $O/c5mfma/pmc --stats $(find $O/c5mfma/stats -name "*kernel_stats.csv" | head -1) --out $O/c5mfma/pmc_mfma.json | grep -B1 -A7 "k_bil_mt\|k_bil_dp2\|k_bil_rows" | head -60
# batch sweep (global batch on one GPU: the replicated update's cost at G ranks), 8192 last
bash tools/gpu_batch_sweep.sh $TAG/sweep 100 400 800 1024 1600 8192 || exit 1
