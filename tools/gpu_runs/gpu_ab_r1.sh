set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab1
cd $R
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/ab1/pytest.log 2>&1 && \
timeout -k 10 400 python tools/kbench.py --rounds 5 > gpurun_out/ab1/kbench.json 2> gpurun_out/ab1/kbench.err
echo rc=$?
tail -3 gpurun_out/ab1/pytest.log
