# fused joint sweep with long utterances (T up to 200, S up to 90)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4v; mkdir -p $O; cd $R
MRNNT_JOINT_BIG=1 MRNNT_FUZZ_FIRST=1000 MRNNT_JOINT_CASES=150 timeout -k 10 1000 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed|^E  .*Assert" $O/fuzz.log | tail -30
