# pipelined joint kernels (joint_pipe=1): parity tests, then A/B timing against the plain loop
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r33; mkdir -p $O; cd $R
MRNNT_TUNE=joint_pipe=1 timeout -k 10 600 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_pipe.log 2>&1
echo pytest_rc=$? ; tail -n 5 $O/pytest_pipe.log
for v in 0 1 0 1; do
  timeout -k 10 240 python tools/joint_bench.py --no-unfused --steps 5 --tune joint_pipe=$v >> $O/joint_h512.json 2>> $O/err.log || exit 1
done
for v in 0 1; do
  timeout -k 10 240 python tools/joint_bench.py --no-unfused --steps 5 --H 256 --tune joint_pipe=$v >> $O/joint_h256.json 2>> $O/err.log || exit 1
done
python - <<'PY'
import json
for f in ['gpurun_out/r33/joint_h512.json','gpurun_out/r33/joint_h256.json']:
    for l in open(f):
        d=json.loads(l); print(f[-14:], d['tune'], d['fused']['kernels_ms'], d['fused']['ms_per_step'])
PY
