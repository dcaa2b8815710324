#!/bin/bash
O=gpurun_out/pipe_dbg
mkdir -p $O
timeout -k 10 60 ./tools/debug/dot2_probe > $O/dot2.txt 2>&1
cat $O/dot2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -q --timeout 120 --timeout-method thread -k "pipe" > $O/pytest_pipe.log 2>&1
echo rc=$?
grep -E "passed|failed" $O/pytest_pipe.log | tail -3
grep -E "^FAILED" $O/pytest_pipe.log | head -20
