#!/bin/bash
# Round 3: fused-joint launch variants -- parity of every variant, then an A/B in one box: forward tile (32x32 ring
# 2 / 4 / 8, 16x16) and backward tile (16x16 default, 32x32) at H = 512 and 256. Output under gpurun_out/j16b/.
set -e
O=gpurun_out/j16b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread > $O/pytest_joint.log 2>&1
for r in 1 2; do
for t in "joint_ring=2" "joint_ring=4" "joint_ring=8" "joint_mfma=16" "joint_bwd_mfma=32"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --tune $t > $O/h512_${t}_$r.json
done
done
for t in "joint_ring=2" "joint_ring=4" "joint_ring=8" "joint_bwd_mfma=32"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H 256 --tune $t > $O/h256_${t}.json
done
echo done
