#!/bin/bash
# Round-6 GPU passes.  usage: bash tools/gpu_r6.sh TAG STEP [STEP ...]
#   smoke           __graft_entry__.smoke()
#   tests:<expr>    pytest -m gpu -k <expr> (tests/, thread timeouts)
#   alltests        every -m gpu test
#   bench[:cfg]     bench.py (default C3 line; cfg c2/c4/c5: no CPU baseline, no label pass)
#   dpmodel:<cfg>:<G>:<l>[:form]  tools/probes/dp_update_model.py (cost model, rank 0)
#   prof[:cfg]      rocprofv3 --kernel-trace --stats of bench.py
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for st in "$@"; do
  case $st in
    smoke)
      timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    tests:*)
      k=${st#tests:}
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -k "$k" -v -s --timeout 900 \
        --timeout-method thread -p no:cacheprovider > $O/tests_$(echo $k | tr -c 'a-zA-Z0-9' _).log 2>&1 \
        || { echo "tests $k failed"; grep -E "FAILED|Error|assert" $O/tests_*.log | head -30; exit 1; }
      grep -E "passed|failed|labels:|emu " $O/tests_$(echo $k | tr -c 'a-zA-Z0-9' _).log | tail -20 ;;
    alltests)
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread \
        -p no:cacheprovider > $O/alltests.log 2>&1 \
        || { echo tests failed; grep -E "FAILED|Error" $O/alltests.log | head -20; tail -5 $O/alltests.log; exit 1; }
      tail -2 $O/alltests.log ;;
    drv)
      # the driver's exact command (BENCH_rNN.json): 20 timed steps, 5 warm-up
      timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err \
        || { echo drv bench failed; tail -30 $O/drv.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/drv.json')); print('drv', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), 'hostq', round(d['timed_region_host_queue_us'],1), {k: round(v, 2) for k, v in d['kernel_us'].items()}, 'cpu', d.get('cpu_baseline', {}).get('value'))" ;;
    drvq)
      # the driver's command without the CPU baseline / label pass (timing only)
      timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-label-pass > $O/drvq.json 2> $O/drvq.err \
        || { echo drvq bench failed; tail -30 $O/drvq.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/drvq.json')); print('drvq', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), 'hostq', round(d['timed_region_host_queue_us'],1), {k: round(v, 2) for k, v in d['kernel_us'].items()})" ;;
    rep:*)
      # the driver's command n times (timing only; "rep:3" or "rep:3:--no-index-overlap")
      a=${st#rep:}; n=${a%%:*}; x=""; [ "$a" != "$n" ] && x=${a#*:}
      for i in $(seq 1 $n); do
        timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-label-pass $x > $O/rep_$i.json 2> $O/rep_$i.err \
          || { echo rep bench failed; tail -30 $O/rep_$i.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/rep_$i.json')); print('rep $x', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), 'hostq', round(d['timed_region_host_queue_us'],1), 'idx', round(d['index_build_us_per_batch'], 3), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
      done ;;
    b512)
      timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-label-pass > $O/b512.json 2> $O/b512.err \
        || { echo b512 bench failed; tail -30 $O/b512.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b512.json')); print('b512', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), 'hostq', round(d['timed_region_host_queue_us'],1), {k: round(v, 2) for k, v in d['kernel_us'].items()})" ;;
    hosttrace)
      # host time of every call inside the timed region (driver command, timing only)
      timeout -k 10 300 python3 -u tools/probes/bench_host_trace.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-label-pass > $O/hosttrace.json 2> $O/hosttrace.err \
        || { echo hosttrace failed; tail -30 $O/hosttrace.err; exit 1; }
      tail -25 $O/hosttrace.err ;;
    bench)
      timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err \
        || { echo bench failed; tail -30 $O/bench.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench.json')); print('c3', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, 'frac', round(d['roofline']['frac'], 3), 'cpu', d.get('cpu_baseline', {}).get('value'))" ;;
    bench:*)
      c=${st#bench:}
      timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --no-label-pass > $O/bench_$c.json 2> $O/bench_$c.err \
        || { echo $c bench failed; tail -20 $O/bench_$c.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})" ;;
    dpmodel:*)
      a=${st#dpmodel:}; IFS=: read -r c G l f <<< "$a"; ff=""; tg=${c}_G${G}_l${l}
      if [ -n "$f" ]; then ff="--kernel-form $f"; tg=${tg}_$(echo $f | tr -c 'a-zA-Z0-9' _); fi
      timeout -k 10 600 python3 -u tools/probes/dp_update_model.py --config $c --G $G --l $l $ff > $O/dpmodel_$tg.json 2> $O/dpmodel_$tg.err \
        || { echo dpmodel failed; tail -20 $O/dpmodel_$tg.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/dpmodel_$tg.json'))
for k in ('single','replicated','partitioned','p2p'):
    v=d.get(k)
    if v: print(k, {x: (round(y,2) if isinstance(y,float) else y) for x,y in v.items() if x!='kernel_forms'})
print('projection', {k: v for k, v in d['projection'].items() if k!='assumptions'})" ;;
    dpprof:*)
      a=${st#dpprof:}; l=${a%%:*}; f=""; tg=$l
      if [ "$a" != "$l" ]; then f="--kernel-form ${a#*:}"; tg=${l}_$(echo ${a#*:} | tr -c 'a-zA-Z0-9' _); fi
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv \
        -d $O/dpprof_$tg -o run -- python3 $R/tools/probes/dp_update_model.py --l $l $f \
        > $O/dpprof_$tg.json 2> $O/dpprof_$tg.err) || { echo dpprof failed; tail -30 $O/dpprof_$tg.err; exit 1; }
      cut -c1-150 $O/dpprof_$tg/run_kernel_stats.csv | head -20 ;;
    prof|prof:*)
      c=${st#prof}; c=${c#:}; c=${c:-c3}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv \
        -d $O/prof_$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --no-label-pass \
        > $O/prof_$c.json 2> $O/prof_$c.err) || { echo prof failed; tail -30 $O/prof_$c.err; exit 1; }
      cut -c1-120 $O/prof_$c/run_kernel_stats.csv | head -12 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo ALL_OK
