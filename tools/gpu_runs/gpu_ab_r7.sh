set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab7
mkdir -p $O
cd $R
V='[{},{"softmax_variant":3,"softmax_grid_per_cu":16},{"softmax_variant":3,"softmax_grid_per_cu":32},{"softmax_variant":3,"softmax_grid_per_cu":64},{"grad_variant":3,"grad_grid_per_cu":16},{"grad_variant":3,"grad_grid_per_cu":32},{"grad_variant":3,"grad_grid_per_cu":64}]'
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not fullsize" > $O/pytest.log 2>&1 && \
timeout -k 10 500 python tools/kbench.py --rounds 4 --variants "$V" > $O/kbench.json 2> $O/kbench.err
echo rc=$?
tail -n 3 $O/pytest.log
