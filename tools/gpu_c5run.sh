bash tools/gpu_c5.sh r2z || exit 1
timeout -k 10 300 python3 -u tools/bil_stamps.py --config c5 > gpurun_out/r2z/bil_stamps.log 2>&1; grep -v amdgpu gpurun_out/r2z/bil_stamps.log
