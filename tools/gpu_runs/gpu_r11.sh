set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r11
mkdir -p $O
cd $R
V='[{},{"occ_skip":0},{"grad_variant":2},{"grad_variant":2,"occ_skip":0}]'
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rs > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python tools/kbench.py --config headline --rounds 4 --variants "$V" > $O/kb_head.json 2> $O/kb_head.err && \
timeout -k 10 300 python tools/kbench.py --config ragged --rank 7/8 --rounds 4 --variants "$V" > $O/kb_r7of8.json 2> $O/kb_r7of8.err
echo rc=$?
tail -n 3 $O/pytest.log
cat $O/bench.json
