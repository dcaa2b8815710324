# staged-coefficient gradient kernel (grad_variant 5/6) + fp32 blank/label coefficients: parity (default and
# variant 5 over the whole parity file), in-process A/B, then bench in separate processes to see the
# process-to-process spread of the gradient kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3c; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
MRNNT_TUNE=grad_variant=5,softmax_variant=13 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest5.log 2>&1 && \
V='[{},{"grad_variant":5},{"grad_variant":6},{"grad_variant":5,"grad_grid_per_cu":8},{"grad_variant":6,"grad_grid_per_cu":8},{"grad_variant":5,"grad_grid_per_cu":0}]' && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu --steps 5 > $O/b0_$i.json 2> $O/b0_$i.err && \
  timeout -k 10 200 python bench.py --no-cpu --steps 5 --tune grad_variant=5 > $O/b5_$i.json 2> $O/b5_$i.err && \
  timeout -k 10 200 python bench.py --no-cpu --steps 5 --tune grad_variant=6 > $O/b6_$i.json 2> $O/b6_$i.err || break
done
echo rc=$?
tail -n 2 $O/pytest.log $O/pytest5.log
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
for f in $O/b*_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['grad']['avg_ms'], d['kernels']['log_softmax']['avg_ms'], d['roofline']['box_copy_gbps'])"; done
