# new defaults (lean log-softmax, staged gradient): whole GPU suite, then old-vs-new A/B on the other configs
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3e; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
V='[{},{"softmax_variant":2,"grad_variant":0}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --config c2 --variants "$V" > $O/kb_c2.json 2> $O/kb_c2.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --config ragged64 --variants "$V" > $O/kb_r64.json 2> $O/kb_r64.err && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 3 --config c5 --variants "$V" > $O/kb_c5.json 2> $O/kb_c5.err && \
timeout -k 10 200 python bench.py --no-cpu --acts-dtype bf16 > $O/bf.json 2> $O/bf.err && \
timeout -k 10 200 python bench.py --no-cpu --acts-dtype f16 > $O/f16.json 2> $O/f16.err
echo rc=$?
tail -n 2 $O/pytest.log
for c in c2 r64 c5; do python -c "
import json; d=json.load(open('$O/kb_$c.json'))
for v in d['variants']: print('$c', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
for f in bf f16; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernels'])"; done
