# Full GPU validation: every gpu-marked test, the driver's smoke(), the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-full}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
tail -n 3 $O/pytest_gpu.log
cat $O/smoke.log $O/bench.json
