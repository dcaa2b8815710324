# NaN zero-rows for ll = -inf (reference semantics): infeasible-alignment test, vocabulary-size sweep, parity suite
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4t; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
MRNNT_FUZZ_V=1,4,8,12,4096,5000,10000 MRNNT_FUZZ_FIRST=5000 MRNNT_FUZZ_CASES=400 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
tail -3 $O/parity.log
grep -E "^FAILED|passed|failed|Error" $O/fuzz.log | tail -20
