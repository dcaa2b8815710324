# persistent joint forward (joint_pipe=2, two 4-wave workgroups per CU, phase offset): parity + offset sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r36; mkdir -p $O; cd $R
MRNNT_TUNE=joint_pipe=2 timeout -k 10 600 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest.log 2>&1
echo pytest_rc=$?; tail -n 3 $O/pytest.log
run() { local lab=$1; shift; local args=""; for t in "$@"; do args="$args --tune $t"; done
  timeout -k 10 240 python tools/joint_bench.py --no-unfused --steps 5 $args | sed "s/^/$lab /" >> $O/ab.txt 2>> $O/err.log; }
for rep in 1 2; do
  run plain joint_pipe=0 && run off0 joint_pipe=2 joint_offset=0 && run off4 joint_pipe=2 joint_offset=4 && \
  run off9 joint_pipe=2 joint_offset=9 && run off14 joint_pipe=2 joint_offset=14 || exit 1
done
python3 - <<'PY'
import json
for l in open('/root/repo/gpurun_out/r36/ab.txt'):
    lab, js = l.split(' ', 1); d = json.loads(js)
    print(f"{lab:8s}", d['fused']['kernels_ms'], d['fused']['ms_per_step'])
PY
