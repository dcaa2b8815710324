#!/bin/bash
# Round-3 final build: seeded fuzz sweep with a fresh seed range (1,000 loss cases + 120 fused-joint cases).
O=gpurun_out/sw
mkdir -p $O
MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=130000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/fuzz_1000_seed130000.log 2>&1 && \
MRNNT_JOINT_CASES=120 MRNNT_FUZZ_FIRST=5000 timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread -k random > $O/joint_fuzz_120_seed5000.log 2>&1
echo rc_fuzz=$?
