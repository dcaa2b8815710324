# joint activation build with batched enc/pred loads (new) vs one k-step at a time (ab/pkg_old)
# runs of tools/joint_bench.py, plus the joint tests on the new build
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4e; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 300 python tools/joint_bench.py --no-unfused > $O/new_$i.json 2> $O/new_$i.err && \
  MRNNT_LIB=$R/ab/pkg_old/libmonotonic_rnnt_amd.so timeout -k 10 300 python tools/joint_bench.py --no-unfused > $O/old_$i.json 2> $O/old_$i.err || break
done
echo rc=$?
tail -n 1 $O/pytest.log
for f in new_1 old_1 new_2 old_2; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['fused']['ms_per_step'], d['fused']['kernels_ms'])"; done
