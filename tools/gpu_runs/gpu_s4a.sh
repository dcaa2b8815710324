# joint reduce: clear/flush only the label range a block of frames touches; joint tests + alignment-window test,
# joint bench with and without alignment restriction
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4a; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "joint or alignment" > $O/pytest.log 2>&1 && \
timeout -k 10 600 python tools/joint_bench.py --align-k 2 --no-unfused > $O/jb_k2.json 2> $O/jb_k2.err && \
timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/jb.json 2> $O/jb.err
echo rc=$?
tail -n 2 $O/pytest.log
cat $O/jb_k2.json $O/jb.json
