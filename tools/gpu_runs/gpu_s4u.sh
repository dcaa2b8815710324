# fuzz sweeps: extreme logit spreads (x10, x30, x100) and long T with short S (up to 600 extra frames)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4u; mkdir -p $O; cd $R
MRNNT_FUZZ_SCALE=10,30,100 MRNNT_FUZZ_FIRST=7000 MRNNT_FUZZ_CASES=400 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz_scale.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" $O/fuzz_scale.log | tail -20
MRNNT_FUZZ_V=2,5,16,64,256 MRNNT_FUZZ_T_EXTRA=600 MRNNT_FUZZ_FIRST=9000 MRNNT_FUZZ_CASES=300 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz_longT.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" $O/fuzz_longT.log | tail -20
