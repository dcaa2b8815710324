# final check of the round-end tree: whole GPU suite, smoke, bench; then the joint dbias A/B at H = 384 / 640
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
TAG=full_s5d bash tools/gpu_full.sh || exit 1
O=$R/gpurun_out/s5d; mkdir -p $O
for H in 384 640; do
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H > $O/jb_h${H}_gemm.json 2> $O/jb.err && \
  MRNNT_JOINT_BIAS_SUM=1 timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H > $O/jb_h${H}_sum.json 2> $O/jb.err || exit 1
done
for f in $O/jb_h*.json; do python -c "
import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['fused']['ms_per_step'], json.dumps(d['fused']['kernels_ms']))"; done
