set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r19
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_joint.log 2>&1 && \
timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/jb_head.json 2> $O/jb_head.err && \
timeout -k 10 600 python tools/joint_bench.py --no-unfused --H 256 > $O/jb_h256.json 2> $O/jb_h256.err
echo rc=$?
tail -n 3 $O/pytest_joint.log
cat $O/jb_head.json $O/jb_h256.json
