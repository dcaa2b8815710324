# long seeded sweeps: 4000 default cases (seeds 20000-23999), 1000 through dp_halo=0 + grad_variant=3 + softmax 0
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5a; mkdir -p $O; cd $R
MRNNT_FUZZ_FIRST=20000 MRNNT_FUZZ_CASES=4000 timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q -p no:randomly --timeout 300 --timeout-method thread > $O/fuzz_default.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" $O/fuzz_default.log | tail -12
MRNNT_FUZZ_TUNE=dp_halo=0,grad_variant=3,softmax_variant=0 MRNNT_FUZZ_FIRST=30000 MRNNT_FUZZ_CASES=1000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/fuzz_variants.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed" $O/fuzz_variants.log | tail -12
