# Round-6 GPU steps, chained with && (each under its own time limit); MODE picks the set. Output under
# gpurun_out/$TAG (default r06).
#   first : joint tests + the new uniform-acts oracle test, headline bench lines on N(0,1) / U[0,1) logits and with
#           every in-band row live (development build, occ_skip=0), then the joint step's kernel stats + SQ counters on
#           the shipping library
#   walk  : walk / loader progress inside the configs[1] chase launch (tools/walk_trace.py; probe 4: no ring reads)
#   full  : every gpu-marked test, smoke(), the default bench line, configs[1] graph bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06}
mkdir -p $O
cd $R
sha() { python3 -c "import hashlib,sys;print(hashlib.sha256(open(sys.argv[1],'rb').read()).hexdigest())" $1; }
case ${MODE:-full} in
first)
  sha monotonic-rnnt_amd/libmonotonic_rnnt_amd.so > $O/lib_sha256.txt
  timeout -k 10 400 python -u -m pytest tests/test_gpu_joint.py -x -q -rs --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1 && \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v -rs -s --timeout 300 --timeout-method thread -k uniform > $O/pytest_uniform.log 2>&1 && \
  timeout -k 10 300 python bench.py > $O/bench_normal.json 2> $O/bench_normal.err && \
  timeout -k 10 300 python bench.py --acts-dist uniform > $O/bench_uniform.json 2> $O/bench_uniform.err && \
  timeout -k 10 300 python bench.py --tune occ_skip=0 --no-cpu > $O/bench_allrows.json 2> $O/bench_allrows.err && \
  timeout -k 10 300 python bench.py --acts-dist uniform --tune occ_skip=0 --no-cpu > $O/bench_uniform_allrows.json 2> $O/bench_uniform_allrows.err && \
  TAG=r06 bash tools/gpu_joint_profile.sh > $O/joint_profile.txt 2>&1
  rc=$?; echo rc=$rc; tail -n 2 $O/pytest_joint.log $O/pytest_uniform.log
  for f in normal uniform allrows uniform_allrows; do python3 -c "
import json,sys;d=json.load(open('$O/bench_$f.json'));r=d['roofline'];k=d['kernels']
print('$f',d['value'],d['ms_per_step'],'live',r['live_rows'],'/',r['inband_rows'],'frac',r['frac'],'grad',k['grad']['avg_ms'],'lsm',k['log_softmax']['avg_ms'])"; done
  cat $O/joint_profile.txt; exit $rc ;;
walk)
  W="python tools/walk_trace.py"
  timeout -k 10 200 $W $O/walk_p1e0.json chase_pair=1 chase_early_free=0 > $O/walk_p1e0.txt 2>&1 && \
  timeout -k 10 200 $W $O/walk_p1e1.json chase_pair=1 chase_early_free=1 > $O/walk_p1e1.txt 2>&1 && \
  timeout -k 10 200 $W $O/walk_p2e1.json chase_pair=2 chase_early_free=1 > $O/walk_p2e1.txt 2>&1 && \
  timeout -k 10 200 $W $O/walk_p2e1_noring.json chase_pair=2 chase_early_free=1 chase_probe=4 > $O/walk_p2e1_noring.txt 2>&1 && \
  timeout -k 10 200 $W $O/walk_p1e1_noring.json chase_pair=1 chase_early_free=1 chase_probe=4 > $O/walk_p1e1_noring.txt 2>&1 && \
  timeout -k 10 300 python tools/kbench.py --config c2 --rounds 40 --variants '[{"chase_pair":1,"chase_early_free":0},{"chase_pair":1,"chase_early_free":1},{"chase_pair":2,"chase_early_free":0},{"chase_pair":2,"chase_early_free":1}]' > $O/kbench_c2_pair_early.json 2> $O/kbench.err
  rc=$?; echo rc=$rc; for f in p1e0 p1e1 p2e1 p2e1_noring p1e1_noring; do echo == $f; tail -n 4 $O/walk_$f.txt; done
  python3 -c "
import json;d=json.load(open('$O/kbench_c2_pair_early.json'))
for v in d['variants']: print(v['knobs'], {k: round(x*1e3,2) for k,x in v['median_ms'].items() if x})"; exit $rc ;;
walkprobe)
  W="python tools/walk_trace.py"
  for pr in 4 5 6 7; do
    timeout -k 10 200 $W $O/walk_p1_probe$pr.json chase_pair=1 chase_early_free=1 chase_probe=$pr > $O/walk_p1_probe$pr.txt 2>&1 || exit $?
  done
  for pr in 4 5 6 7; do echo == probe $pr; grep "alpha walk" $O/walk_p1_probe$pr.txt; done; exit 0 ;;
chase)
  timeout -k 10 400 python -u -m pytest tests/test_gpu_chase.py -x -q -rs --timeout 120 --timeout-method thread > $O/pytest_chase.log 2>&1
  rc=$?; tail -n 3 $O/pytest_chase.log; [ $rc -eq 0 ] || exit $rc
  VARS="cur r05chase" TAG=$TAG/var MODE=chasevar bash $R/tools/gpu_r06.sh; exit $? ;;
chaseprod)
  cd /tmp && export TMPDIR=/tmp
  for i in 1 2; do
    for v in new old; do
      if [ $v = old ]; then export MRNNT_LIB_PATH=$R/monotonic-rnnt_amd/abl/libmonotonic_rnnt_amd_r05chase.so; else unset MRNNT_LIB_PATH; fi
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$i -o run --output-format csv -- python3 $R/bench.py --config c2 --graph --steps 2000 --warmup 200 --no-cpu > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit 1
    done
  done
  unset MRNNT_LIB_PATH; cd $R
  for f in $O/prof_*; do echo == $f; find $f -name "*kernel_stats.csv" -exec grep chase {} \; | cut -d, -f1-4; done
  exit 0 ;;
chasevar)
  cd /tmp && export TMPDIR=/tmp
  for i in 1 2; do
    for v in ${VARS:-cur r05chase p3r16 p2r16 p1r16 p2r32}; do
      if [ $v = cur ]; then unset MRNNT_LIB_PATH; else export MRNNT_LIB_PATH=$R/monotonic-rnnt_amd/abl/libmonotonic_rnnt_amd_$v.so; fi
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$i -o run --output-format csv -- python3 $R/bench.py --config c2 --graph --steps 2000 --warmup 200 --no-cpu > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit 1
    done
  done
  unset MRNNT_LIB_PATH; cd $R
  for f in $O/prof_*; do python3 -c "
import csv,json
r={x['Name'].split('(')[0].split('<')[-1][:40]:round(float(x['AverageNs'])/1000,2) for x in csv.DictReader(open('$f/run_kernel_stats.csv')) if 'chase' in x['Name']}
print('$f'.split('/')[-1], r)"; done
  exit 0 ;;
reducetrace)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -x -q -rs --timeout 300 --timeout-method thread > $O/pytest_joint.log 2>&1
  rc=$?; tail -n 2 $O/pytest_joint.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python tools/reduce_trace.py $O/reduce_trace.json > $O/reduce_trace.txt 2>&1 && \
  timeout -k 10 600 python tools/joint_bench.py --no-unfused --ab '[{"joint_probe":64},{"joint_probe":0}]' --ab-rounds 9 > $O/joint_h512.json 2> $O/joint_h512.err && \
  MRNNT_JOINT_CAPTURABLE=1 timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/joint_h512_capturable.json 2> $O/joint_h512_capturable.err
  rc=$?; tail -n 1 $O/reduce_trace.txt | cut -c1-600; python3 -c "
import json
for f in ('joint_h512','joint_h512_capturable'):
    d=json.load(open('$O/%s.json'%f)); print(f, d['fused']['ms_per_step'], d['fused']['kernels_ms'])
for v in json.load(open('$O/joint_h512.json'))['ab']: print(v['knobs'], v['step_ms_median'], v['median_ms'])"; exit $rc ;;
benches)
  b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; exit 1; }; \
        python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('traffic'))"; }
  b headline
  b headline_uniform --acts-dist uniform
  b headline_allrows --tune occ_skip=0 --no-cpu
  b headline_uniform_allrows --acts-dist uniform --tune occ_skip=0 --no-cpu
  b c2_graph --config c2 --graph --steps 2000 --warmup 200 --no-cpu
  b c2_eager --config c2 --steps 200 --warmup 20 --no-cpu
  b headline_bf16 --acts-dtype bf16 --no-cpu
  b ragged64 --config ragged64 --no-cpu
  b align_k2 --align-k 2 --no-cpu
  b c5 --config c5 --steps 2 --warmup 1 --no-cpu
  timeout -k 10 600 python tools/joint_bench.py > $O/joint_h512.json 2> $O/joint_h512.err || exit 1
  MRNNT_JOINT_CAPTURABLE=1 timeout -k 10 600 python tools/joint_bench.py --no-unfused > $O/joint_h512_capturable.json 2> $O/joint_h512_capturable.err || exit 1
  timeout -k 10 600 python tools/joint_bench.py --H 256 --no-unfused > $O/joint_h256.json 2> $O/joint_h256.err || exit 1
  python3 -c "
import json
for f in ('joint_h512','joint_h512_capturable','joint_h256'):
    d=json.load(open('$O/%s.json'%f)); print(f, d['fused']['ms_per_step'], d['fused']['utt_per_s'], d['fused']['kernels_ms'], (d.get('unfused') or {}).get('ms_per_step'))"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c2 -o run --output-format csv -- python3 $R/bench.py --config c2 --graph --steps 500 --warmup 100 --no-cpu > $O/bench_c2_graph_rocprof.json 2> $O/bench_c2_graph_rocprof.err && \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rocprof_joint -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 3 --warmup 1 > $O/joint_h512_rocprof.json 2> $O/joint_h512_rocprof.err
  rc=$?; rm -f $O/rocprof_c2/run_kernel_trace.csv $O/rocprof_joint/run_kernel_trace.csv; exit $rc ;;
sweeps)
  sha() { python3 -c "import hashlib,sys;print(hashlib.sha256(open(sys.argv[1],'rb').read()).hexdigest())" $1; }
  L="library $(sha monotonic-rnnt_amd/libmonotonic_rnnt_amd.so)"
  P="python -u -m pytest -q -rs --timeout 600 --timeout-method thread"
  f() { n=$1; shift; echo "$L" > $O/$n.log; timeout -k 10 900 env "$@" >> $O/$n.log 2>&1; rc=$?; tail -n 1 $O/$n.log; [ $rc -eq 0 ] || exit $rc; }
  if [ "${SET:-a}" = b ]; then
  [ -z "$ONLY_C5" ] && f full_batch_headline_64utt MRNNT_FULL_BATCH=1 $P tests/test_gpu_fullsize.py -k full_batch
  [ -z "$ONLY_C5" ] && f c4_full_batch_costs_512utt MRNNT_FULL_BATCH=1 $P tests/test_gpu_c4_shards.py
  f c5_full_batch_costs_64utt MRNNT_FULL_BATCH=1 $P -s -v tests/test_gpu_c5_chunks.py
  exit 0; fi
  f fuzz_1000_seed200000 MRNNT_FUZZ_CASES=1000 MRNNT_FUZZ_FIRST=200000 $P tests/test_gpu_fuzz.py -k test_random_case_vs_oracle
  f fuzz_500_seed210000_chase_pair3 MRNNT_FUZZ_CASES=500 MRNNT_FUZZ_FIRST=210000 MRNNT_FUZZ_TUNE=chase_pair=3 $P tests/test_gpu_fuzz.py -k test_random_case_vs_oracle
  f fuzz_500_seed220000_chase_pair2 MRNNT_FUZZ_CASES=500 MRNNT_FUZZ_FIRST=220000 MRNNT_FUZZ_TUNE=chase_pair=2 $P tests/test_gpu_fuzz.py -k test_random_case_vs_oracle
  f joint_fuzz_120_seed11000 MRNNT_JOINT_CASES=120 MRNNT_FUZZ_FIRST=11000 $P tests/test_gpu_joint.py -k random_cases
  exit 0 ;;
full)
  sha monotonic-rnnt_amd/libmonotonic_rnnt_amd.so > $O/lib_sha256.txt
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
  timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
  timeout -k 10 300 python bench.py --config c2 --graph --steps 2000 --warmup 200 > $O/bench_c2_graph.json 2> $O/bench_c2_graph.err
  rc=$?; echo rc=$rc; tail -n 3 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json $O/bench_c2_graph.json; exit $rc ;;
esac
