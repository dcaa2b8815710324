# widened sweeps: acts path through every launch variant (+ cost-only forward), fused joint random cases
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4k; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
r1=$?
echo fuzz rc=$r1
tail -n 25 $O/fuzz.log
if [ $r1 -eq 0 ] || [ $r1 -eq 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_joint.py -q --timeout 300 --timeout-method thread > $O/joint.log 2>&1
  echo joint rc=$?
  tail -n 25 $O/joint.log
fi
