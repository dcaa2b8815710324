set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r8
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rs > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
tail -n 5 $O/pytest.log
cat $O/bench.json
