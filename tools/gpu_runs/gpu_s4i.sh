# seeded random sweep of the HIP path against the oracle
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4i; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo rc=$?
grep -E "FAILED|passed|failed" $O/pytest.log | tail -20
