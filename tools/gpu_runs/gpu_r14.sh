set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r14
mkdir -p $O
cd $R
V='[{},{"occ_skip":0},{"softmax_variant":3},{"grad_grid_per_cu":0},{"grad_grid_per_cu":0,"occ_skip":0}]'
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 4 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err
echo rc=$?
