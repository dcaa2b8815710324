# recursion shapes (dp_variant 1: 2 cells per lane, half the waves; 2: 4 cells per lane): parity, A/B on the
# headline and ragged64; accuracy-vs-reference-fp32 test output
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3t; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "variant or accuracy or long_label or alignment or golden" > $O/pytest.log 2>&1 && \
V='[{},{"dp_variant":1},{"dp_variant":2}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --config ragged64 --variants "$V" > $O/kb_r64.json 2> $O/kb_r64.err
echo rc=$?
grep -E "passed|failed|accuracy vs" $O/pytest.log | tail -4
for f in kb kb_r64; do python -c "
import json; d=json.load(open('$O/$f.json'))
for v in d['variants']: print('$f', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
