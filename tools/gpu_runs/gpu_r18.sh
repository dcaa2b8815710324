set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r18
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_joint.py -q -x > $O/pytest_joint.log 2>&1 && \
timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/jb_head.json 2> $O/jb_head.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 3 --warmup 1 > $O/jb_prof.json 2> $O/jb_prof.err
echo rc=$?
tail -n 3 $O/pytest_joint.log
cat $O/jb_head.json
