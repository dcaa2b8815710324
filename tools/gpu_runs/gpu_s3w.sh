# halo recursion as the default (dp_halo=2, single wave without halo for S+1 <= 64): whole GPU suite, A/B vs the
# per-step-barrier recursion (dp_halo=0) on c2, headline, ragged64
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3w; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
V='[{},{"dp_halo":0},{"dp_halo":1}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 7 --config c2 --variants "$V" > $O/kb_c2.json 2> $O/kb_c2.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --config ragged64 --variants "$V" > $O/kb_r64.json 2> $O/kb_r64.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err
echo rc=$?
tail -n 2 $O/pytest.log
for f in kb_c2 kb kb_r64; do python -c "
import json; d=json.load(open('$O/$f.json'))
for v in d['variants']: print('$f', v['knobs'], {k:round(x,4) for k,x in v['median_ms'].items()})"; done
python -c "
import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['kernels'])"
