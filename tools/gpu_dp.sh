set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03dp; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=4 --timeout 600 --timeout-method thread -p no:cacheprovider -k "partitioned or global_batch_800 or many_relations or gpu_ranks" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -20
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/probes/dp_update_model.py --G 8 --l 100 > $O/model_l100.json 2> $O/model.err && cat $O/model_l100.json
timeout -k 10 300 python -u tools/probes/dp_update_model.py --G 8 --l 1024 > $O/model_l1024.json 2>> $O/model.err && cat $O/model_l1024.json
