# Round-5 GPU steps, chained with && (each under its own time limit); MODE picks the set.
#   full  : every gpu-marked test, smoke(), the default bench line, configs[1] graph bench
#   c2    : configs[1] HIP-graph bench + rocprofv3 kernel stats of it
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05}
mkdir -p $O
cd $R
case ${MODE:-full} in
full)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
  timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
  timeout -k 10 300 python bench.py --config c2 --graph --steps 2000 --warmup 200 > $O/bench_c2_graph.json 2> $O/bench_c2_graph.err
  rc=$?; echo rc=$rc; tail -n 3 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json $O/bench_c2_graph.json; exit $rc ;;
joint)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1 && \
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_h512.json 2> $O/joint_h512.err && \
  MRNNT_JOINT_DH=mfma timeout -k 10 300 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_h512_mfma.json 2> $O/joint_h512_mfma.err
  rc=$?; echo rc=$rc; tail -n 3 $O/pytest_joint.log; cat $O/joint_h512.json $O/joint_h512_mfma.json; exit $rc ;;
reduce)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1 && \
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_h512.json 2> $O/joint_h512.err && \
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --steps 5 --tune joint_reduce_pf=1 > $O/joint_h512_pf1.json 2> $O/joint_h512_pf1.err
  rc=$?; echo rc=$rc; tail -n 3 $O/pytest_joint.log; cat $O/joint_h512.json $O/joint_h512_pf1.json; exit $rc ;;
redab)
  [ -n "$AB" ] || AB='[{"joint_probe":0},{"joint_probe":4}]'
  timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1 && \
  timeout -k 10 400 python tools/joint_bench.py --no-unfused --steps 3 --ab "$AB" > $O/joint_ab.json 2> $O/joint_ab.err && \
  cd /tmp && export TMPDIR=/tmp && \
  for form in 0 1; do \
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_red_sq_form$form -- python3 $R/tools/joint_bench.py --no-unfused --steps 1 --warmup 1 --tune joint_probe=$((4*form)) > $O/pmc_red_sq_form$form.json 2> $O/pmc_red_sq_form$form.err || exit 1; \
    python3 $R/tools/pmc_kernel.py $O/pmc_red_sq_form$form --match reduce > $O/pmc_red_sq_form$form.txt || exit 1; \
  done
  rc=$?; echo rc=$rc; tail -n 2 $O/pytest_joint.log; python3 -c "import json;d=json.load(open('$O/joint_ab.json'));[print(v['knobs'],v['median_ms']) for v in d['ab']]"; cat $O/pmc_red_sq_form0.txt $O/pmc_red_sq_form1.txt; exit $rc ;;
sweeps)
  # opt-in full-batch parity runs (minutes of CPU oracle each: a heartbeat file shows the run alive)
  mkdir -p $O/tests
  ( while true; do date > $O/tests/heartbeat; sleep 30; done ) &
  HB=$!
  MRNNT_FULL_BATCH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -v -rs --timeout 600 --timeout-method thread -s > $O/tests/full_batch_headline_64utt.log 2>&1 && \
  MRNNT_FULL_BATCH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_shards.py -v -rs --timeout 600 --timeout-method thread -s > $O/tests/c4_full_batch_costs_512utt.log 2>&1 && \
  MRNNT_FULL_BATCH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_chunks.py -v -rs --timeout 600 --timeout-method thread -s > $O/tests/c5_full_batch_costs_64utt.log 2>&1
  rc=$?; kill $HB; echo rc=$rc; tail -n 3 $O/tests/*.log; exit $rc ;;
fuzz)
  mkdir -p $O/tests
  MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=150000 timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/tests/fuzz_1000_seed150000.log 2>&1 && \
  MRNNT_JOINT_CASES=120 MRNNT_FUZZ_FIRST=7000 timeout -k 10 500 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/tests/joint_fuzz_120_seed7000.log 2>&1
  rc=$?; echo rc=$rc; tail -n 2 $O/tests/*fuzz*.log; exit $rc ;;
final)
  # the round's closing measurements on the final library: full suite, smoke, bench lines, PMC traffic
  MODE=full bash $R/tools/gpu_r05.sh && \
  TAG=r05 bash $R/tools/gpu_profile.sh && \
  MODE=c2 TAG=r05final bash $R/tools/gpu_r05.sh
  rc=$?; echo rc=$rc; exit $rc ;;
fwdab)
  # the plain exp-sum forward (product) against the running max forced on (joint_probe bit 3)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1 && \
  timeout -k 10 300 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_h512.json 2> $O/joint_h512.err && \
  timeout -k 10 400 python tools/joint_bench.py --no-unfused --steps 3 --ab '[{"joint_probe":0},{"joint_probe":8}]' > $O/joint_fwd_ab.json 2> $O/joint_fwd_ab.err
  rc=$?; echo rc=$rc; tail -n 3 $O/pytest_joint.log; cat $O/joint_h512.json; python3 -c "import json;d=json.load(open('$O/joint_fwd_ab.json'));[print(v) for v in d['ab']]"; exit $rc ;;
libab)
  # product library (plain exp-sum forward) against the previous commit's product library (running max, ablib/),
  # alternating processes on one box
  for i in 1 2 3; do \
    timeout -k 10 200 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_new_$i.json 2> $O/joint_new_$i.err || exit 1; \
    MRNNT_LIB_PATH=$R/ablib/lib_head_runmax.so timeout -k 10 200 python tools/joint_bench.py --no-unfused --steps 5 > $O/joint_old_$i.json 2> $O/joint_old_$i.err || exit 1; \
  done
  rc=$?; echo rc=$rc; for f in $O/joint_new_*.json $O/joint_old_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));k=d['fused'];print('$f'.split('/')[-1],k['ms_per_step'],k['kernels_ms'])"; done; exit $rc ;;
post)
  # after the development-build stamp change: the forward A/B again, the headline bench line (carrying the PMC
  # traffic record of the same sources), the joint random sweep over the plain / running-max forward, then the sweeps
  MODE=fwdab TAG=${TAG:-r05} bash $R/tools/gpu_r05.sh && \
  timeout -k 10 300 python bench.py > $O/bench_post.json 2> $O/bench_post.err && \
  mkdir -p $O/tests && \
  MRNNT_JOINT_CASES=120 MRNNT_FUZZ_FIRST=9000 timeout -k 10 500 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/tests/joint_fuzz_120_seed9000.log 2>&1
  rc=$?; echo rc=$rc; cat $O/bench_post.json; tail -n 2 $O/tests/joint_fuzz_120_seed9000.log; [ $rc = 0 ] || exit $rc
  MODE=sweeps TAG=${TAG:-r05} bash $R/tools/gpu_r05.sh; exit $? ;;
probeab)
  # the forward's load probes again in the unstamped development build (1: every pred load on row 0, 2: every enc load
  # on frame 0; results wrong, timing only), interleaved in one process
  timeout -k 10 400 python tools/joint_bench.py --no-unfused --steps 3 --ab-rounds 4 --ab '[{"joint_probe":0},{"joint_probe":1},{"joint_probe":2},{"joint_probe":3}]' > $O/joint_probe_ab.json 2> $O/joint_probe_ab.err
  rc=$?; echo rc=$rc; python3 -c "import json;d=json.load(open('$O/joint_probe_ab.json'));[print(v['knobs'],v['step_ms_median'],v['median_ms']) for v in d['ab']]"; exit $rc ;;
jtrace)
  timeout -k 10 300 python tools/joint_trace.py $O/joint_trace.json > $O/joint_trace.txt 2>&1
  rc=$?; echo rc=$rc; cat $O/joint_trace.txt | tail -6; exit $rc ;;
fuzzvar)
  # seeded sweeps through other launch variants of the development build (MRNNT_FUZZ_TUNE)
  mkdir -p $O/tests
  MRNNT_FUZZ_TUNE="dp_halo=0,grad_variant=3" MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=160000 timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/tests/fuzz_1000_seed160000_dphalo0_grad3.log 2>&1 && \
  MRNNT_FUZZ_TUNE="chase=0" MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=170000 timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/tests/fuzz_1000_seed170000_chase0.log 2>&1 && \
  MRNNT_FUZZ_TUNE="chase_stage=0,chase_wait_us=0" MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=180000 timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/tests/fuzz_1000_seed180000_direct_selfhelp.log 2>&1
  rc=$?; echo rc=$rc; tail -n 2 $O/tests/fuzz_1000_seed1[678]*.log; exit $rc ;;
cgrid)
  timeout -k 10 300 python tools/kbench.py --config c2 --rounds 30 --variants '[{"chase_grid_per_cu":0},{"chase_grid_per_cu":4},{"chase_grid_per_cu":6},{"chase_grid_per_cu":8},{"chase_grid_per_cu":12},{"chase_grid_per_cu":16}]' > $O/chase_grid.json 2> $O/chase_grid.err
  rc=$?; echo rc=$rc; python3 -c "import json;d=json.load(open('$O/chase_grid.json'));[print(v['knobs'],round(v['median_ms']['chase']*1e3,2)) for v in d['variants']]"; exit $rc ;;
hasan)
  # the GPU library's host orchestration under ASan / UBSan (a child pytest process; a heartbeat file shows it alive)
  ( while true; do date > $O/hasan_heartbeat; sleep 30; done ) &
  HB=$!
  timeout -k 10 1100 python -u -m pytest tests/test_gpu_host_asan.py -x -v -rs --timeout 1050 --timeout-method thread > $O/pytest_host_asan.log 2>&1
  rc=$?; kill $HB; echo rc=$rc; tail -n 30 $O/pytest_host_asan.log; exit $rc ;;
dpre)
  timeout -k 10 300 python tools/dpre_bench.py > $O/dpre_bench.json 2> $O/dpre_bench.err && \
  timeout -k 10 300 python -u -m pytest tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread -k dpre > $O/pytest_dpre.log 2>&1
  rc=$?; echo rc=$rc; cat $O/dpre_bench.json; tail -n 2 $O/pytest_dpre.log; exit $rc ;;
dprepmc)
  cd /tmp && export TMPDIR=/tmp
  J="$R/tools/dpre_bench.py --reps 2 --variants [{\"joint_dpre_nw\":0}]"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -- python3 $J > $O/pmc_sq.json 2> $O/pmc_sq.err && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d $O/pmc_sq2 -- python3 $J > $O/pmc_sq2.json 2> $O/pmc_sq2.err && \
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_grbm -- python3 $J > $O/pmc_grbm.json 2> $O/pmc_grbm.err && \
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 $J > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 $J > $O/pmc_write.json 2> $O/pmc_write.err && \
  python3 $R/tools/pmc_kernel.py $O/pmc_sq $O/pmc_sq2 $O/pmc_grbm $O/pmc_fetch $O/pmc_write --match dpre --match Cijk > $O/pmc_dpre.txt
  rc=$?; echo rc=$rc; cat $O/pmc_dpre.txt; exit $rc ;;
dbg)
  timeout -k 10 300 python tools/debug/chase_state_diff.py > $O/chase_state_diff.txt 2>&1
  rc=$?; echo rc=$rc; cat $O/chase_state_diff.txt | tail -40; exit $rc ;;
ctrace)
  timeout -k 10 300 python tools/chase_trace.py $O/chase_trace.json > $O/chase_trace.txt 2>&1
  rc=$?; echo rc=$rc; cat $O/chase_trace.txt | tail -5; exit $rc ;;
c2)
  timeout -k 10 300 python bench.py --config c2 --graph --steps 2000 --warmup 200 > $O/bench_c2_graph.json 2> $O/bench_c2_graph.err && \
  cd /tmp && export TMPDIR=/tmp && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_stats -o run --output-format csv -- python3 $R/bench.py --config c2 --graph --steps 2000 --warmup 200 --no-cpu --no-lengths-ab > $O/bench_c2_graph_prof.json 2> $O/bench_c2_graph_prof.err
  rc=$?; echo rc=$rc; cat $O/bench_c2_graph.json; exit $rc ;;
esac
