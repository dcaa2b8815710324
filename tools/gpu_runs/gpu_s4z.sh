# 17 M lattice columns (grid cap of the hardware-scheduled streaming launches)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4z; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k "32bit_dispatch or very_large_vocabulary" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest.log | tail -8
