# long seeded sweep of the fused joint path: 600 random cases (seeds 0-599)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4q; mkdir -p $O; cd $R
MRNNT_FUZZ_FIRST=0 MRNNT_JOINT_CASES=600 timeout -k 10 1000 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
grep -E "^FAILED|passed|failed|Error" $O/fuzz.log | tail -30
