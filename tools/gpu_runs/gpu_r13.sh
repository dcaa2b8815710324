set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r13
mkdir -p $O
cd $R
V='[{},{"softmax_variant":0},{"softmax_variant":3},{"softmax_variant":4},{"softmax_variant":5},{"softmax_variant":6},{"softmax_variant":7},{"grad_variant":2},{"grad_grid_per_cu":16},{"grad_grid_per_cu":0}]'
timeout -k 10 400 python tools/kbench.py --ws-first --rounds 4 --variants "$V" > $O/kb.json 2> $O/kb.err
echo rc=$?
