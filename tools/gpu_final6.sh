#!/bin/bash
# Round-6 evidence passes on the final build.   usage: bash tools/gpu_final6.sh TAG STEP [STEP ...]
#   pmc:<cfg>    FETCH_SIZE / WRITE_SIZE passes of bench.py --config cfg (c3: with the labelling
#                pass, so k_label's traffic is in the same file) -> profiles/r06_<cfg>_pmc_traffic.json
#                on the box (bench lines after it report traffic_current) + gpurun_out/TAG/
#   sq           SQ wave-cycle split of the C3 step kernels (k_forward / k_update)
#   mfma         MFMA busy cycles of the C5 step kernels
#   bench:<cfg>  bench.py line (c3: the default run with CPU baseline and labelling pass)
#   stats:<cfg>  rocprofv3 --kernel-trace --stats of the same bench command
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
args() {   # bench arguments of a config's evidence line
  if [ "$1" = c3 ]; then echo "--config c3"; else echo "--config $1 --no-cpu-baseline --no-label-pass"; fi
}
for st in "$@"; do
  case $st in
    pmc:*)
      c=${st#pmc:}
      BA="--config $c --steps 64 --warmup 16 --no-cpu-baseline --kernel-iters 32"
      [ "$c" = c3 ] || BA="$BA --no-label-pass"
      for p in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $p -f csv -d $O/pmc_$c/$p -o run \
          -- python3 $R/bench.py $BA > $O/pmc_${c}_$p.log 2>&1) || { echo "pmc $c $p failed"; tail -20 $O/pmc_${c}_$p.log; exit 1; }
      done
      python3 tools/pmc_traffic.py $O/pmc_$c/FETCH_SIZE $O/pmc_$c/WRITE_SIZE $BA \
        --out $O/r06_${c}_pmc_traffic.json > $O/pmc_${c}_post.log 2>&1 || { echo "pmc $c post failed"; tail -20 $O/pmc_${c}_post.log; exit 1; }
      cp $O/r06_${c}_pmc_traffic.json profiles/
      python3 -c "
import json; d=json.load(open('$O/r06_${c}_pmc_traffic.json'))
print('pmc $c', {k: (round(v['traffic_bytes']/1e6, 2) if isinstance(v, dict) and 'traffic_bytes' in v else None) for k, v in d.get('per_kernel', {}).items()})" | cut -c1-600 ;;
    sq)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT -f csv \
        -d $O/sq -o run -- python3 $R/bench.py --config c3 --steps 64 --warmup 16 --no-cpu-baseline \
        --no-label-pass --kernel-iters 32 > $O/sq.log 2>&1) || { echo sq failed; tail -20 $O/sq.log; exit 1; }
      python3 tools/pmc_sq.py $O/sq --kernels k_forward,k_update --out $O/r06_c3_pmc_sq.json | grep -A12 fractions | head -30 ;;
    mfma)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
        GRBM_GUI_ACTIVE -f csv -d $O/mfma -o run -- python3 $R/bench.py --config c5 --steps 64 --warmup 16 \
        --no-cpu-baseline --no-label-pass --kernel-iters 32 > $O/mfma.log 2>&1) || { echo mfma failed; tail -20 $O/mfma.log; exit 1; }
      # mfma_util_span needs the kernels' average durations: this tag's stats:c5 pass if it ran
      # first, else the committed summary
      ST=$O/r06_c5_kernel_stats.csv; [ -f $ST ] || ST=profiles/r06_c5_kernel_stats.csv
      python3 tools/pmc_mfma.py $O/mfma --stats $ST --out $O/r06_c5_pmc_mfma.json > $O/mfma_post.log 2>&1 || { echo mfma post failed; tail $O/mfma_post.log; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/r06_c5_pmc_mfma.json'))['per_kernel']
for k, v in d.items():
    if v.get('mfma_busy_cycles'): print(k[:60], 'util', round(v['mfma_util'], 4), 'span', round(v.get('mfma_util_span', 0), 4), 'us', round(v['avg_duration_us'], 2))" ;;
    bench:*)
      c=${st#bench:}
      timeout -k 10 600 python3 -u bench.py $(args $c) > $O/r06_${c}_bench.json 2> $O/bench_$c.err \
        || { echo "$c bench failed"; tail -20 $O/bench_$c.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/r06_${c}_bench.json')); r=d['roofline']
print('$c', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, 'frac', round(r['frac'], 4), 'traffic', r.get('traffic'), r.get('traffic_current'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" ;;
    stats:*)
      c=${st#stats:}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_$c -o run \
        -- python3 $R/bench.py $(args $c) --no-cpu-baseline > $O/stats_$c.json 2> $O/stats_$c.err) \
        || { echo "stats $c failed"; tail -20 $O/stats_$c.err; exit 1; }
      cp $O/stats_$c/run_kernel_stats.csv $O/r06_${c}_kernel_stats.csv
      cut -c1-120 $O/stats_$c/run_kernel_stats.csv | head -10 ;;
    drv)
      # the driver's exact command (BENCH_rNN.json): 20 timed steps, 5 warm-up, CPU baseline
      timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r06_c3_bench_driver_cmd.json 2> $O/drv.err \
        || { echo drv bench failed; tail -30 $O/drv.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/r06_c3_bench_driver_cmd.json')); r=d['roofline']
print('drv', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, 'frac', round(r['frac'], 4), 'traffic_current', r.get('traffic_current'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" ;;
    drvstats)
      # rocprofv3 summary of the driver's exact command
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/drvstats -o run \
        -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/drvstats.json 2> $O/drvstats.err) \
        || { echo "drvstats failed"; tail -20 $O/drvstats.err; exit 1; }
      cp $O/drvstats/run_kernel_stats.csv $O/r06_c3_driver_cmd_kernel_stats.csv
      cut -c1-120 $O/drvstats/run_kernel_stats.csv | head -6 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo ALL_OK
