#!/bin/bash
# Round 3: dbias summed inside the 16x16x32 gradient pass (ABI v8 mrnnt_joint_problem.dbias) -- the whole GPU suite,
# then the H = 512 joint step with it and with the separate G.sum (MRNNT_JOINT_BIAS_SUM=1). Output under gpurun_out/db/.
set -e
O=gpurun_out/db
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for r in 1 2; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 > $O/h512_fused_db_$r.json
MRNNT_JOINT_BIAS_SUM=1 timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 > $O/h512_gsum_$r.json
done
echo done
