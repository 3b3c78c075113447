set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/g5; mkdir -p $O; cd $R
for L in relation-autoencoder_amd/rae/librae_hip.so variants/pipe_plain.so variants/pipe_nopush.so; do
  t=$(basename $L .so)
  RAE_LIB=$R/$L timeout -k 10 300 python3 -u tools/probes/dp_update_model.py --config c3 --G 8 --l 100 --modes p2p_pipe > $O/dp_$t.json 2> $O/dp_$t.err || { echo "$L failed"; tail -20 $O/dp_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dp_$t.json')); v=d['p2p_pipe']
print('$t', {k: round(v[k],2) for k in ('forward','update','graph_step','graph_step_with_index')}, 'eff', round(d['projection']['p2p_pipe']['efficiency'],4))"
done
