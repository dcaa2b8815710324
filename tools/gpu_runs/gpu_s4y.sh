# B = 70000 utterances with alignment (band kernel grid y capped at 65535), plus the alignment parity tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4y; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "grid_y or alignment or many_utterances" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -20
