set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r15
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_joint.py -m gpu -q -x -rs > $O/pytest_joint.log 2>&1
echo rc=$?
tail -n 40 $O/pytest_joint.log
