# more seeded sweeps: two other launch-variant sets and odd vocabulary sizes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5g; mkdir -p $O; cd $R
run() { tag=$1; shift; env "$@" timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -k test_random_case_vs_oracle -q --timeout 300 --timeout-method thread > $O/$tag.log 2>&1; echo "$tag rc=$? $(tail -1 $O/$tag.log)"; grep -E "^FAILED" $O/$tag.log | head -5; }
run variants_a MRNNT_FUZZ_TUNE=softmax_variant=14,grad_variant=6,col_scatter=0 MRNNT_FUZZ_FIRST=40000 MRNNT_FUZZ_CASES=800
run variants_b MRNNT_FUZZ_TUNE=occ_skip=0,dp_halo=1,softmax_variant=15 MRNNT_FUZZ_FIRST=50000 MRNNT_FUZZ_CASES=800
run odd_v MRNNT_FUZZ_V=6,7,9,33,65,127,129,513,1025 MRNNT_FUZZ_FIRST=60000 MRNNT_FUZZ_CASES=800
