#!/bin/bash
# Round 3: the pipelined one-wave-per-SIMD joint forward (development build): parity of every variant, then an A/B
# against the 8-wave forward at H = 512 / 384 / 256. Output under gpurun_out/pipe/.
#   joint_pipe=1: MFMA gaps carry the softmax, the next tile's build, the W DMA and the fragment loads
#   joint_pipe=3: the same without the DMA / loads in the gaps;  joint_pipe=0: the 8-wave kernel
set -e
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "pipe" > $O/pytest_pipe.log 2>&1
MRNNT_FUZZ_TUNE="joint_pipe=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k "random or vs_host or alignment or blank_last" > $O/pytest_pipe_fuzz.log 2>&1
for r in 1 2; do
for t in "joint_pipe=0" "joint_pipe=1" "joint_pipe=3"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --tune $t > $O/h512_${t}_$r.json
done
done
for H in 384 256; do
for t in "joint_pipe=0" "joint_pipe=1"; do
timeout -k 10 300 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --H $H --tune $t > $O/h${H}_${t}.json
done
done
echo done
