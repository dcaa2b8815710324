# full-size tests incl. the new alignment-restricted headline test
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4f; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
