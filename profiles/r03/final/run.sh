#!/bin/bash
# Round-3 final-build profiles: headline under rocprofv3 --kernel-trace --stats; the fused joint (H = 512) kernel
# stats; SQ / GRBM counters of the joint kernels with the backward on the 16x16x32 tile (default) and on the
# 32x32x16 tile (round 2), each counter pass its own run. Output under gpurun_out/fp/.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/fp
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/headline -- python3 $R/bench.py --config headline --steps 10 --warmup 3 > $O/headline.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/joint_stats -- python3 $R/tools/joint_bench.py --no-unfused --steps 5 --warmup 2 > $O/joint_h512.json
for t in "joint_bwd_mfma=16" "joint_bwd_mfma=32"; do
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq_$t -- python3 $R/tools/joint_bench.py --no-unfused --steps 2 --warmup 1 --tune $t > $O/pmc_sq_$t.json
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_grbm_$t -- python3 $R/tools/joint_bench.py --no-unfused --steps 2 --warmup 1 --tune $t > $O/pmc_grbm_$t.json
done
python3 $R/tools/pmc_kernel.py $O/pmc_sq_joint_bwd_mfma=16 $O/pmc_grbm_joint_bwd_mfma=16 --match joint_ > $O/pmc_joint_bwd16.txt
python3 $R/tools/pmc_kernel.py $O/pmc_sq_joint_bwd_mfma=32 $O/pmc_grbm_joint_bwd_mfma=32 --match joint_ > $O/pmc_joint_bwd32.txt
echo done
