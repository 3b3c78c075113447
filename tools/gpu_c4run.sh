set -o pipefail
O=gpurun_out/r2c4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread  > $O/gputests.log 2>&1 || { echo tests failed; tail -60 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline --no-label-pass --steps 256 --warmup 32 > $O/bench_c4.json 2> $O/bench_c4.err || { echo bench failed; tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', round(d['value']), 'us/step', round(d['ms_per_step']*1e3, 2), {k: round(v, 2) for k, v in d['kernel_us'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --no-cpu-baseline --no-label-pass --steps 64 --warmup 8 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo prof failed; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-140 | head -14
