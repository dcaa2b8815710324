set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r21
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_joint.log 2>&1 && \
timeout -k 10 600 python tools/joint_bench.py > $O/jb_h512.json 2> $O/jb_h512.err && \
timeout -k 10 600 python tools/joint_bench.py --H 256 > $O/jb_h256.json 2> $O/jb_h256.err
echo rc=$?
tail -n 2 $O/pytest_joint.log
cat $O/jb_h512.json $O/jb_h256.json
