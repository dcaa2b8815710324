#!/bin/bash
O=gpurun_out/jt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 120 --timeout-method thread > $O/pytest_joint.log 2>&1
echo rc=$?
tail -n 2 $O/pytest_joint.log
