set -o pipefail
R=$(pwd); O=$R/gpurun_out/r2e; mkdir -p $O
bash tools/gpu_test_ab.sh r2e build/ab/head.so build/ab/vh32.so build/ab/cap0.so relation-autoencoder_amd/rae/librae_hip.so build/ab/cap1024.so build/ab/cap3072.so || exit 1
timeout -k 10 200 python3 -u tools/phase_stamps.py --config c3 > $O/stamps_l100.log 2>&1 || { echo stamps failed; tail -20 $O/stamps_l100.log; exit 1; }
grep -v amdgpu.ids $O/stamps_l100.log
timeout -k 10 300 python3 -u tools/phase_stamps.py --config c3 --batch-size 800 > $O/stamps_l800.log 2>&1 || { echo stamps800 failed; tail -20 $O/stamps_l800.log; exit 1; }
grep -v amdgpu.ids $O/stamps_l800.log
