set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r27
mkdir -p $O
cd $R
V='[{},{"softmax_variant":8},{"softmax_variant":9},{"softmax_variant":0},{"softmax_variant":8,"softmax_grid_per_cu":32}]'
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 5 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python bench.py --acts-dtype bf16 --no-cpu --tune softmax_variant=8 > $O/bf16_v8.json 2> $O/bf16_v8.err && \
timeout -k 10 300 python bench.py --no-cpu --tune softmax_variant=8 > $O/f32_v8.json 2> $O/f32_v8.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/f32_def.json 2> $O/f32_def.err
echo rc=$?
python -c "
import json; d=json.load(open('$O/kb.json'))
for v in d['variants']: print(v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"
for f in $O/*_v8.json $O/f32_def.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['kernels'])"; done
