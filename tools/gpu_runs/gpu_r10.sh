set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r10
mkdir -p $O
cd $R
V='[{},{"grad_grid_per_cu":0},{"grad_variant":3,"grad_grid_per_cu":32},{"grad_variant":2},{"softmax_grid_per_cu":32}]'
timeout -k 10 300 python tools/kbench.py --config ragged --rank 7/8 --rounds 3 --variants "$V" > $O/kb_r7of8.json 2> $O/kb_r7of8.err && \
timeout -k 10 300 python tools/kbench.py --config ragged --rank 0/8 --rounds 3 --variants "$V" > $O/kb_r0of8.json 2> $O/kb_r0of8.err && \
timeout -k 10 300 python tools/kbench.py --config headline --rounds 3 --variants "$V" > $O/kb_head.json 2> $O/kb_head.err
echo rc=$?
