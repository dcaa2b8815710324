# joint activation build with a rational tanh (one v_rcp per element instead of v_exp + v_rcp): parity, sweeps, bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5e; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -q --timeout 300 --timeout-method thread > $O/joint.log 2>&1
echo rc=$?; tail -1 $O/joint.log
MRNNT_FUZZ_FIRST=0 MRNNT_JOINT_CASES=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/joint_fuzz.log 2>&1
echo rc=$?; grep -E "^FAILED|passed|failed" $O/joint_fuzz.log | tail -6
MRNNT_JOINT_BIG=1 MRNNT_FUZZ_FIRST=1000 MRNNT_JOINT_CASES=100 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/joint_fuzz_big.log 2>&1
echo rc=$?; grep -E "^FAILED|passed|failed" $O/joint_fuzz_big.log | tail -6
for H in 512 256 128; do
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H > $O/jb_h${H}.json 2> $O/jb.err || exit 1
  python -c "
import json;d=json.load(open('$O/jb_h${H}.json'));print('H=$H', d['fused']['ms_per_step'], json.dumps(d['fused']['kernels_ms']), d['fused']['joint_fwd_frac'])"
done
