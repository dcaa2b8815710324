# occupancy-8 lean softmax (variant 16) A/B; non-blocking length upload: bench step overhead vs kernel sum
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3i; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variant or golden or known" > $O/pytest.log 2>&1 && \
V='[{},{"softmax_variant":16},{"softmax_variant":15}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 200 python bench.py --no-cpu > $O/b1.json 2> $O/b1.err && \
timeout -k 10 200 python bench.py --no-cpu --tune softmax_variant=16 > $O/b2.json 2> $O/b2.err
echo rc=$?
tail -n 2 $O/pytest.log
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
for f in b1 b2; do python -c "
import json; d=json.load(open('$O/$f.json')); k=d['kernels']; s=sum(v['avg_ms'] for v in k.values())
print('$f', d['value'], d['ms_per_step'], 'kernels sum', round(s,3), 'overhead', round(d['ms_per_step']-s,3), k)"; done
