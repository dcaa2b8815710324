set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r26
mkdir -p $O
cd $R
for v in 2 3 4; do
timeout -k 10 300 python bench.py --acts-dtype bf16 --no-cpu --tune softmax_variant=$v > $O/bf16_v$v.json 2> $O/bf16_v$v.err || exit 1
done
echo rc=$?
for f in $O/bf16_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['kernels'])"; done
