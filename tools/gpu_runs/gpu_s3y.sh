# log-softmax restricted to the alignment window for alignment-restricted calls: whole GPU suite, then the headline
# with k = 0 / 2 / 10 and the unrestricted headline
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3y; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --align-k 2 > $O/b_k2.json 2> $O/b_k2.err && \
timeout -k 10 200 python bench.py --no-cpu --align-k 0 > $O/b_k0.json 2> $O/b_k0.err && \
timeout -k 10 200 python bench.py --no-cpu --align-k 10 > $O/b_k10.json 2> $O/b_k10.err && \
timeout -k 10 200 python bench.py --no-cpu > $O/b.json 2> $O/b.err
echo rc=$?
tail -n 2 $O/pytest.log
for f in b_k0 b_k2 b_k10 b; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels'].items()}, d['roofline']['live_rows'], d['config'].get('window_rows_per_gpu'), d['loss_check'])"; done
