# long seeded sweep: 2000 further random cases of tests/test_gpu_fuzz.py (seeds 160-2159)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4p; mkdir -p $O; cd $R
MRNNT_FUZZ_FIRST=160 MRNNT_FUZZ_CASES=2000 timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" $O/fuzz.log | tail -30
