#!/bin/bash
# Round evidence pass on the current build: C3 PMC traffic (into profiles/ on the box, so the
# bench line below reports it as current), smoke, every GPU test, the default bench line,
# rocprofv3 kernel stats of the same bench, C5 bench + kernel stats.   usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/gpu_pmc.sh $TAG/pmc c3 > $O/pmc.log 2>&1 || { echo pmc failed; tail -20 $O/pmc.log; exit 1; }
cp $O/pmc/pmc_traffic.json profiles/r03_c3_pmc_traffic.json
python3 -c "import json; d=json.load(open('$O/pmc/pmc_traffic.json')); print('pmc', {k: v for k, v in d.items() if k != 'kernels'})" | cut -c1-400
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/gputests.log | head; tail -5 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernel_us'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('traffic_current'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
cut -c1-110 $O/prof/run_kernel_stats.csv | head -8
cd $R
K=none CFG=c5 bash tools/gpu_s5.sh $TAG/c5 || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 256 --kernel-form priv_rows=off > $O/bench_c5_privoff.json 2> $O/bench_c5_privoff.err || { echo c5 privoff bench failed; tail -20 $O/bench_c5_privoff.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5_privoff.json')); print('c5 priv_rows=off', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
for c in c2 c4; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --no-label-pass > $O/bench_$c.json 2> $O/bench_$c.err || { echo $c bench failed; tail -20 $O/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
done
