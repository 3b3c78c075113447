set -o pipefail
O=gpurun_out/r2rep; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "test_bf16_mfma_path_tracks_oracle" -p no:cacheprovider > $O/run_$i.log 2>&1; echo "mtdp=1 run $i rc=$?"; grep -h "relative distance\|passed\|failed" $O/run_$i.log | tail -2
done
for i in 1 2; do
  RAE_MTDP=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "test_bf16_mfma_path_tracks_oracle" -p no:cacheprovider > $O/run0_$i.log 2>&1; echo "mtdp=0 run $i rc=$?"; grep -h "relative distance\|passed\|failed" $O/run0_$i.log | tail -2
done
exit 0
