# scattered column order for the gradient kernel only (col_scatter=2): A/B on two buffer pairs, three processes;
# then two bench processes with the same-buffer copy probe
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3l; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variant or occupancy" > $O/pytest.log 2>&1 && \
V='[{},{"col_scatter":2},{"grads_buf":1,"acts_buf":1},{"grads_buf":1,"acts_buf":1,"col_scatter":2}]' && \
for i in 1 2 3; do
  timeout -k 10 300 python tools/kbench.py --ws-first --rounds 4 --buffers 2 --variants "$V" > $O/kb_$i.json 2> $O/kb_$i.err || break
done && \
timeout -k 10 200 python bench.py --no-cpu > $O/b1.json 2> $O/b1.err && \
timeout -k 10 200 python bench.py --no-cpu --tune col_scatter=2 > $O/b2.json 2> $O/b2.err
echo rc=$?
tail -n 2 $O/pytest.log
for i in 1 2 3; do python -c "
import json; d=json.load(open('$O/kb_$i.json'))
print('proc $i')
for v in d['variants']: print('   ', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
for f in b1 b2; do python -c "
import json; d=json.load(open('$O/$f.json')); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], d['kernels']['grad'], d['kernels']['log_softmax'], r['copy_gbps_same_buffers'], r['frac_of_copy_same_buffers'])"; done
