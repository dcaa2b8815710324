set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab5
mkdir -p $O
cd $R
V='[{"nt_load":0},{"nt_load":1},{"nt_load":1,"nt_store":0},{"nt_load":1,"grad_grid_per_cu":16},{"nt_load":1,"grad_grid_per_cu":48},{"nt_load":1,"softmax_grid_per_cu":32},{"nt_load":1,"dp_variant":4},{"nt_load":1,"softmax_variant":0},{"nt_load":1,"grad_variant":2}]'
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not fullsize" > $O/pytest.log 2>&1 && \
timeout -k 10 500 python tools/kbench.py --rounds 4 --variants "$V" > $O/kbench.json 2> $O/kbench.err && \
timeout -k 10 300 python tools/kbench.py --config c2 --rounds 6 --variants '[{"dp_variant":1},{"dp_variant":4},{"dp_variant":3},{"dp_variant":0}]' > $O/kbench_c2.json 2> $O/kbench_c2.err && \
timeout -k 10 300 python tools/kbench.py --config ragged --rounds 3 --variants '[{"dp_variant":1},{"dp_variant":4},{"dp_variant":3}]' > $O/kbench_ragged.json 2> $O/kbench_ragged.err
echo rc=$?
tail -n 3 $O/pytest.log
