# halo recursion v2 (whole prefetch blocks, dp_halo=1: 8-step, 2: 16-step blocks): parity with dp_halo=2 over the
# halo path on, then A/B on the headline and ragged64
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3v; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variant" > $O/pytest_v.log 2>&1 && \
MRNNT_TUNE=dp_halo=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_halo.log 2>&1 && \
V='[{},{"dp_halo":1},{"dp_halo":2}]' && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 5 --config ragged64 --variants "$V" > $O/kb_r64.json 2> $O/kb_r64.err
echo rc=$?
tail -n 2 $O/pytest_v.log $O/pytest_halo.log
for f in kb kb_r64; do python -c "
import json; d=json.load(open('$O/$f.json'))
for v in d['variants']: print('$f', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
