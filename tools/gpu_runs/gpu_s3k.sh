# scattered column order (col_scatter) vs in order, across two acts / two grads buffers, four processes:
# does spreading the active window over the whole buffer remove the placement-dependent slow mode?
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3k; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variant" > $O/pytest.log 2>&1 && \
V='[{},{"col_scatter":1},{"grads_buf":1,"acts_buf":1},{"grads_buf":1,"acts_buf":1,"col_scatter":1}]' && \
for i in 1 2 3 4; do
  timeout -k 10 300 python tools/kbench.py --ws-first --rounds 3 --buffers 2 --variants "$V" > $O/kb_$i.json 2> $O/kb_$i.err || break
done
echo rc=$?
tail -n 2 $O/pytest.log
for i in 1 2 3 4; do python -c "
import json; d=json.load(open('$O/kb_$i.json'))
print('proc $i')
for v in d['variants']: print('   ', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
