#!/bin/bash
# Round 3: dbias from the gradient pass against the ones column of the dweight GEMM at H = 128 / 256 / 384.
# Output under gpurun_out/db2/.
set -e
O=gpurun_out/db2
mkdir -p $O
MRNNT_JOINT_DBIAS=pass timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread > $O/pytest_joint_dbias_pass.log 2>&1
for r in 1 2; do
for H in 128 256 384; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H $H > $O/h${H}_column_$r.json
MRNNT_JOINT_DBIAS=pass timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H $H > $O/h${H}_pass_$r.json
done
done
echo done
