set -o pipefail
R=$(pwd); O=$R/gpurun_out/r2d; mkdir -p $O
timeout -k 10 120 ./build/stream_probe > $O/stream_probe.txt 2>&1 || { echo probe failed; cat $O/stream_probe.txt; exit 1; }
cat $O/stream_probe.txt
bash tools/gpu_pmc2.sh r2d/pmc c3 || exit 1
timeout -k 10 200 python3 -u tools/phase_stamps.py --config c3 > $O/stamps_l100.log 2>&1 || { echo stamps failed; tail -20 $O/stamps_l100.log; exit 1; }
grep -v amdgpu.ids $O/stamps_l100.log
timeout -k 10 300 python3 -u tools/phase_stamps.py --config c3 --batch-size 800 > $O/stamps_l800.log 2>&1 || { echo stamps800 failed; tail -20 $O/stamps_l800.log; exit 1; }
grep -v amdgpu.ids $O/stamps_l800.log
