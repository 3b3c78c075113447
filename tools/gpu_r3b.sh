#!/bin/bash
# Round-3 measurement pass: C3 PMC traffic passes + phase stamps, the C3 split-forward A/B,
# the C5 bench + rocprofv3 stats + decoder / M-tile stamps.   usage: bash tools/gpu_r3b.sh TAG
set -o pipefail
TAG=${1:-r3b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/gpu_pmc.sh $TAG/pmc c3 || exit 1
cd $R
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 --kernel-form sp_forward=split > $O/bench_split.json 2> $O/bench_split.err || { echo split bench failed; tail -20 $O/bench_split.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_split.json')); print('c3 split', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), d['kernel_us'], d['config']['kernel_forms'])"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_fused.json 2> $O/bench_fused.err || { echo bench failed; tail -20 $O/bench_fused.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_fused.json')); print('c3 fused', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), d['kernel_us'])"
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline --steps 256 --warmup 32 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 bench failed; tail -20 $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()}, d['roofline'].get('frac'), d['roofline'].get('frac_of_measured_peak'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_c5 -o run -- python3 $R/bench.py --config c5 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $O/prof_c5.json 2> $O/prof_c5.err || { echo prof failed; tail -30 $O/prof_c5.err; exit 1; }
cut -c1-150 $O/prof_c5/run_kernel_stats.csv | head -12
cd $R
timeout -k 10 200 python3 -u tools/bil_stamps.py --config c5 > $O/bil_stamps.log 2>&1 || { echo bil stamps failed; tail -20 $O/bil_stamps.log; exit 1; }
grep -v amdgpu.ids $O/bil_stamps.log
