set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab3
mkdir -p $O
cd $R
V='[{"grads_offset_kb":0},{"grads_offset_kb":4},{"grads_offset_kb":64},{"grads_offset_kb":1024},{"grads_offset_kb":2048},{"grads_offset_kb":2052},{"grads_offset_kb":4096},{"grads_offset_kb":6144},{"dp_variant":0},{"grads_offset_kb":0,"grad_grid_per_cu":0}]'
timeout -k 10 400 python tools/kbench.py --rounds 4 --variants "$V" > $O/kbench_off.json 2> $O/kbench_off.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/bench2.json 2> $O/bench2.err
echo rc=$?
