#!/bin/bash
# Round 3: fewer vector instructions in the 8-wave joint forward (joint_fwd_opt, development build): parity, then A/B
# in one box at H = 512 / 256. Output under gpurun_out/fwdopt/.
set -e
O=gpurun_out/fwdopt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "fwd_opt" > $O/pytest_fwdopt.log 2>&1
MRNNT_FUZZ_TUNE="joint_fwd_opt=3" timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "random or vs_host or alignment or blank_last" > $O/pytest_fwdopt_fuzz.log 2>&1
for r in 1 2; do
for t in "joint_fwd_opt=0" "joint_fwd_opt=1" "joint_fwd_opt=2" "joint_fwd_opt=3"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --tune $t > $O/h512_${t}_$r.json
done
done
for t in "joint_fwd_opt=0" "joint_fwd_opt=3"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H 256 --tune $t > $O/h256_${t}.json
done
echo done
