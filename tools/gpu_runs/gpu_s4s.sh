# fuzz sweep over other vocabulary sizes: V = 1 (blank only), 4, 8, 12 (one vector), 4096, 5000, 10000
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4s; mkdir -p $O; cd $R
MRNNT_FUZZ_V=1,4,8,12,4096,5000,10000 MRNNT_FUZZ_FIRST=5000 MRNNT_FUZZ_CASES=400 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed|Error" $O/fuzz.log | tail -30
