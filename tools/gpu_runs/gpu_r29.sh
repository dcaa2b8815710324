set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r29
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 3 --warmup 1 > $O/jb_stats.json 2> $O/jb_stats.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 1 --warmup 1 > $O/p1.json 2> $O/p1.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $O/p2 -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 1 --warmup 1 > $O/p2.json 2> $O/p2.err
echo rc=$?
python3 $R/tools/pmc_kernel.py $O/p1 $O/p2 --match joint_fwd --match joint_bwd
