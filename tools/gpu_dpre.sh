#!/bin/bash
# The dpre GEMM study (round 6): variant / ablation A/B of mrnnt_joint_dpre in one process (tools/dpre_bench.py,
# development build), then SQ / TA / TCC counters of one variant, each counter pass its own run.
#   TAG=dpre2 VARIANTS='[...]' PMC_VARIANT='{"joint_dpre_nw": 8}' bash tools/gpu_dpre.sh
set -o pipefail
TAG=${TAG:-dpre}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/tools/dpre_bench.py"
timeout -k 10 300 python3 $B --reps 20 --variants "$VARIANTS" > $O/bench.json 2> $O/bench.err || exit 1
[ -z "$PMC_VARIANT" ] && exit 0
P="[$PMC_VARIANT]"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $B --reps 3 --variants "$P" > $O/stats.json 2> $O/stats.err && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -- python3 $B --reps 2 --variants "$P" > $O/pmc_sq.json 2> $O/pmc_sq.err && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_sq2 -- python3 $B --reps 2 --variants "$P" > $O/pmc_sq2.json 2> $O/pmc_sq2.err && \
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_ta -- python3 $B --reps 2 --variants "$P" > $O/pmc_ta.json 2> $O/pmc_ta.err && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 $B --reps 2 --variants "$P" > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 $B --reps 2 --variants "$P" > $O/pmc_write.json 2> $O/pmc_write.err
rc=$?
python3 $R/tools/pmc_kernel.py $O/pmc_sq $O/pmc_sq2 $O/pmc_ta $O/pmc_fetch $O/pmc_write --match dpre --match Cijk > $O/pmc.txt
echo rc=$rc
exit $rc
