set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r28
mkdir -p $O
cd $R
V='[{},{"grad_variant":4},{"grad_variant":2},{"grad_variant":4,"grad_grid_per_cu":16}]'
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python bench.py --no-cpu --tune grad_variant=4 > $O/b4.json 2> $O/b4.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/b0.json 2> $O/b0.err && \
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "variant or occupancy" > $O/pt.log 2>&1
echo rc=$?
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
for f in $O/b4.json $O/b0.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['kernels'])"; done
tail -n 2 $O/pt.log
