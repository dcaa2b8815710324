# pooled profiling events: configs[1] bench line (launch-bound size) before/after, headline unchanged
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4l; mkdir -p $O; cd $R
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python bench.py --config c2 > $O/bench_c2_default.json 2> $O/bench_c2_default.err && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
for f in bench_c2 bench_c2_default bench; do python -c "
import json,sys;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"; done
