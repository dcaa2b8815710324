# lean log-softmax (softmax_variant 13/14/15: DPP merges, uniform captures, lane-parallel epilogue): parity,
# then in-process A/B against the column-walk default at f32 and bf16
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3b; mkdir -p $O; cd $R
MRNNT_TUNE=softmax_variant=13 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
V='[{},{"softmax_variant":13},{"softmax_variant":14},{"softmax_variant":15}]' && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python bench.py --no-cpu --tune softmax_variant=13 > $O/b13.json 2> $O/b13.err && \
timeout -k 10 300 python bench.py --no-cpu --acts-dtype bf16 > $O/bf0.json 2> $O/bf0.err && \
timeout -k 10 300 python bench.py --no-cpu --acts-dtype bf16 --tune softmax_variant=13 > $O/bf13.json 2> $O/bf13.err && \
timeout -k 10 300 python bench.py --no-cpu --acts-dtype bf16 --tune softmax_variant=15 > $O/bf15.json 2> $O/bf15.err
echo rc=$?
tail -n 3 $O/pytest.log
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
for f in b13 bf0 bf13 bf15; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernels'])"; done
