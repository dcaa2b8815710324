#!/bin/bash
# Round-3 final build: configs[4] whole batch, all 64 costs against the oracle (CPU oracle minutes: a heartbeat file
# under gpurun_out keeps the run visibly alive). Output under gpurun_out/sw/.
O=gpurun_out/sw
mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
MRNNT_FULL_BATCH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_chunks.py -x -v -rs --timeout 840 --timeout-method thread > $O/c5_full_batch.log 2>&1
rc=$?
kill $HB
echo rc_c5=$rc
