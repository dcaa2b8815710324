set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r25
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python bench.py --acts-dtype bf16 --no-cpu > $O/bench_bf16.json 2> $O/bench_bf16.err && \
timeout -k 10 300 python bench.py --config ragged64 --no-cpu > $O/bench_ragged64.json 2> $O/bench_ragged64.err && \
timeout -k 10 400 python bench.py --config c5 --no-cpu --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 600 python tools/scaling_emulation.py > $O/scaling.json 2> $O/scaling.err
echo rc=$?
for f in $O/bench_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'])"; done
tail -n 3 $O/*.err | grep -v amdgpu.ids
