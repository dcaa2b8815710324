# dbias through the dweight GEMM (ones column in Hact, ABI v3 hact_ld): joint parity + sweeps, then A/B vs G.sum
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5b; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py tests/test_capi_host.py -q --timeout 300 --timeout-method thread > $O/joint.log 2>&1 && \
MRNNT_FUZZ_FIRST=0 MRNNT_JOINT_CASES=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/joint_fuzz.log 2>&1 && \
MRNNT_JOINT_BIG=1 MRNNT_FUZZ_FIRST=1000 MRNNT_JOINT_CASES=100 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/joint_fuzz_big.log 2>&1
echo rc=$?
tail -1 $O/joint.log; tail -1 $O/joint_fuzz.log; tail -1 $O/joint_fuzz_big.log
for H in 512 256 128; do for rep in 1 2; do
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H > $O/jb_h${H}_gemm_$rep.json 2> $O/jb.err && \
  MRNNT_JOINT_BIAS_SUM=1 timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H > $O/jb_h${H}_sum_$rep.json 2> $O/jb.err || exit 1
done; done
for f in $O/jb_h*.json; do python -c "
import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['fused']['ms_per_step'], json.dumps(d['fused']['kernels_ms']))"; done
