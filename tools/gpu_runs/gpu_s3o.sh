# simplified dispatch: lean softmax and staged gradient now also for rows of < 96 vectors; parity + c2 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3o; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
V='[{},{"softmax_variant":0,"grad_variant":0},{"softmax_variant":15},{"grad_variant":6}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 7 --config c2 --variants "$V" > $O/kb_c2.json 2> $O/kb_c2.err && \
timeout -k 10 300 python bench.py --config c2 --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python bench.py --config c2 --no-cpu --tune softmax_variant=0 --tune grad_variant=0 > $O/bench_c2_old.json 2> $O/bench_c2_old.err
echo rc=$?
tail -n 2 $O/pytest.log
python -c "
import json; d=json.load(open('$O/kb_c2.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,4) for k,x in v['median_ms'].items()})"
for f in bench_c2 bench_c2_old; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernels'])"; done
