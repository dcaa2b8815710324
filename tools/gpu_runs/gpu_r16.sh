set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r16
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_joint.log 2>&1 && \
timeout -k 10 300 python tools/joint_bench.py --B 8 --steps 3 > $O/jb_small.json 2> $O/jb_small.err && \
timeout -k 10 600 python tools/joint_bench.py > $O/jb_head.json 2> $O/jb_head.err
echo rc=$?
tail -n 2 $O/pytest_joint.log
cat $O/jb_small.json $O/jb_head.json
tail -n 5 $O/jb_head.err
