#!/bin/bash
# Joint (H = 512) profiling round: kernel stats of the fused step (our kernels and the hipBLASLt GEMMs), then the SQ
# and GRBM counters of the joint kernels, each counter pass its own run. Output under gpurun_out/joint_$TAG/.
set -o pipefail
TAG=${TAG:-r04}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/joint_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
J="$R/tools/joint_bench.py --no-unfused"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $J --steps 5 --warmup 2 > $O/joint_h512.json 2> $O/stats.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -- python3 $J --steps 2 --warmup 1 > $O/pmc_sq.json 2> $O/pmc_sq.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d $O/pmc_sq2 -- python3 $J --steps 2 --warmup 1 > $O/pmc_sq2.json 2> $O/pmc_sq2.err && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_grbm -- python3 $J --steps 2 --warmup 1 > $O/pmc_grbm.json 2> $O/pmc_grbm.err && \
python3 $R/tools/pmc_kernel.py $O/pmc_sq $O/pmc_sq2 $O/pmc_grbm --match joint_ > $O/pmc_joint.txt
echo rc=$?
