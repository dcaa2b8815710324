# A/B: row-stride log-softmax (softmax_variant 11/12) vs column walk; split gradient (grad_variant 4) and
# row-stride gradient (3) vs default; re-sized copy probe. Parity of the new variants first.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3a; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "variant" > $O/pytest.log 2>&1 && \
V='[{},{"softmax_variant":11},{"softmax_variant":12},{"softmax_variant":11,"softmax_grid_per_cu":32},{"softmax_variant":12,"softmax_grid_per_cu":32},{"grad_variant":4},{"grad_variant":3}]' && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/b0.json 2> $O/b0.err
echo rc=$?
tail -n 3 $O/pytest.log
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
cat $O/b0.json
