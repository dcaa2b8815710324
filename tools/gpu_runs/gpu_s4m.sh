# timing events without the system fence: step time with per-kernel events on vs off (configs[1]), bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4m; mkdir -p $O; cd $R
timeout -k 10 200 python -u tools/debug/host_overhead.py > $O/host.json 2> $O/host.err && \
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
head -12 $O/host.json
for f in bench_c2 bench; do python -c "
import json,sys;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"; done
