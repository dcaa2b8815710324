# row-parallel (sparse) joint reduce: joint tests with the reduce forced each way, joint bench aligned / unaligned
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4b; mkdir -p $O; cd $R
MRNNT_TUNE=joint_reduce_sparse=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest_sparse.log 2>&1 && \
MRNNT_TUNE=joint_reduce_sparse=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dense.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "alignment" > $O/pytest_align.log 2>&1 && \
timeout -k 10 600 python tools/joint_bench.py --align-k 2 --no-unfused > $O/jb_k2.json 2> $O/jb_k2.err && \
timeout -k 10 600 python tools/joint_bench.py --align-k 2 --no-unfused --tune joint_reduce_sparse=1 > $O/jb_k2_dense.json 2> $O/jb_k2_dense.err && \
timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/jb.json 2> $O/jb.err
echo rc=$?
tail -n 1 $O/pytest_sparse.log $O/pytest_dense.log $O/pytest_align.log
for f in jb_k2 jb_k2_dense jb; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['fused']['ms_per_step'], d['fused']['utt_per_s'], d['fused']['kernels_ms'])"; done
