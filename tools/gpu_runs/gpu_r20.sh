set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r20
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_joint.log 2>&1 && \
for H in 512 256; do for v in 0 1; do
timeout -k 10 300 python tools/joint_bench.py --no-unfused --H $H --tune joint_variant=$v > $O/jb_h${H}_v$v.json 2> $O/jb_h${H}_v$v.err || exit 1
done; done
echo rc=$?
tail -n 2 $O/pytest_joint.log
for f in $O/jb_*.json; do python -c "
import json; d=json.load(open('$f')); f=d['fused']; print('$f'.split('/')[-1], f['ms_per_step'], f['kernels_ms'], f['joint_fwd_frac'], f['joint_bwd_frac'])"; done
