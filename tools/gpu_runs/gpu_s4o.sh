# new edge cases: S + 1 = 2048 (largest label length), batches of 257-1000 utterances
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4o; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "long_label or many_utterances" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest.log | tail -20
