#!/bin/bash
# Round-2 GPU pass: host probe, smoke, every GPU test, the driver's bench command, a long bench,
# and a rocprofv3 kernel-trace of the driver's command.   usage: bash tools/gpu_r2.sh TAG
set -o pipefail
TAG=${1:-r2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'omp', os.environ.get('OMP_NUM_THREADS'))";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; free -g | head -2; } > $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo tests failed; tail -60 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo bench20 failed; tail -30 $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench512.json 2> $O/bench512.err || { echo bench512 failed; tail -30 $O/bench512.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench512.json')); print('512:', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -30 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat
