set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab4
mkdir -p $O
cd $R
V='[{},{"dp_variant":2},{"softmax_variant":2},{"grad_variant":2},{"softmax_variant":2,"grad_variant":2,"dp_variant":2},{"dp_variant":0}]'
timeout -k 10 400 python -m pytest tests -m gpu -q -x -k "not fullsize" > $O/pytest.log 2>&1 && \
timeout -k 10 400 python tools/kbench.py --rounds 4 --variants "$V" > $O/kbench.json 2> $O/kbench.err && \
timeout -k 10 600 python -m pytest tests/test_gpu_fullsize.py -q -x > $O/pytest_full.log 2>&1
echo rc=$?
tail -3 $O/pytest.log $O/pytest_full.log
