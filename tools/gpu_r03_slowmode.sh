# Round 3: log-softmax read-side counters over four acts buffers per process, two passes
# (each its own process, so its own four buffers), plus the D2H-copy trace of an eager device-lengths step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_slow
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
V='[{"acts_buf":0},{"acts_buf":1},{"acts_buf":2},{"acts_buf":3}]'
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/d2h_device -o run -- python3 $R/tools/d2h_check.py --lengths device > $O/d2h_device.log 2>&1 && \
timeout -k 10 30 rocprofv3 --list-avail > $O/counters_avail.txt 2>&1; \
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum --output-format csv -d $O/pmc_a -o run -- python3 $R/tools/kbench.py --config headline --rounds 2 --acts-buffers 4 --variants "$V" > $O/kbench_a.json 2> $O/kbench_a.err && \
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY --output-format csv -d $O/pmc_b -o run -- python3 $R/tools/kbench.py --config headline --rounds 2 --acts-buffers 4 --variants "$V" > $O/kbench_b.json 2> $O/kbench_b.err
echo rc=$?
