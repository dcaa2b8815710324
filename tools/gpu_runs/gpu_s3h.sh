# does scattered physical memory (small mapping fragments) slow the gradient kernel? kbench with the big
# buffers allocated after punching 2 MiB / 64 MiB holes into 100 GB, variants: staged (5), per-row (0),
# row-stride (3), staged on a smaller grid
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3h; mkdir -p $O; cd $R
V='[{},{"grad_variant":0},{"grad_variant":3},{"grad_variant":5,"grad_grid_per_cu":8},{"softmax_variant":2}]'
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 3 --variants "$V" > $O/kb_clean.json 2> $O/kb_clean.err && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 3 --variants "$V" --fragment-gb 100 --fragment-mib 2 > $O/kb_f2.json 2> $O/kb_f2.err && \
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 3 --variants "$V" --fragment-gb 100 --fragment-mib 64 > $O/kb_f64.json 2> $O/kb_f64.err
echo rc=$?
for f in clean f2 f64; do python -c "
import json; d=json.load(open('$O/kb_$f.json'))
for v in d['variants']: print('$f', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
