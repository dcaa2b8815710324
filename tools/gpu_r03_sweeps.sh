#!/bin/bash
# Round-3 final build: the opt-in full-batch oracle sweeps (all 64 headline utterances, all 512 configs[3] costs,
# all 64 configs[4] costs) and a seeded fuzz sweep with a fresh seed, incl. 120 fused-joint cases.
# Output under gpurun_out/sw/.
O=gpurun_out/sw
mkdir -p $O
export MRNNT_FULL_BATCH=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v -rs --timeout 360 --timeout-method thread -k "full_batch or all_64" > $O/full_batch_headline.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_c4_shards.py -x -v -rs --timeout 480 --timeout-method thread > $O/c4_full_batch.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5_chunks.py -x -v -rs --timeout 360 --timeout-method thread > $O/c5_full_batch.log 2>&1
echo rc_full=$?
