#!/bin/bash
# Round 3: persistent 8-wave joint forward (joint_fwd_persist, development build): parity, then A/B in one box.
# Output under gpurun_out/persist/.
set -e
O=gpurun_out/persist
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "persist" > $O/pytest_persist.log 2>&1
MRNNT_FUZZ_TUNE="joint_fwd_persist=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "random or vs_host or alignment or blank_last" > $O/pytest_persist_fuzz.log 2>&1
for r in 1 2; do
for t in "joint_fwd_persist=0" "joint_fwd_persist=1"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --tune $t > $O/h512_${t}_$r.json
done
done
for H in 256 640; do
for t in "joint_fwd_persist=0" "joint_fwd_persist=1"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H $H --tune $t > $O/h${H}_${t}.json
done
done
echo done
