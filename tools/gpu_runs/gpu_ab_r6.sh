set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab6
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not fullsize" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --rounds 4 --variants '[{"dp_variant":1},{"dp_variant":4},{"dp_variant":3}]' > $O/kbench.json 2> $O/kbench.err && \
timeout -k 10 300 python tools/kbench.py --config c2 --rounds 6 --variants '[{"dp_variant":1},{"dp_variant":4},{"dp_variant":0}]' > $O/kbench_c2.json 2> $O/kbench_c2.err && \
timeout -k 10 300 python tools/kbench.py --config ragged64 --rounds 3 --variants '[{"dp_variant":1},{"dp_variant":4},{"dp_variant":3}]' > $O/kbench_ragged64.json 2> $O/kbench_ragged64.err
echo rc=$?
tail -n 3 $O/pytest.log
