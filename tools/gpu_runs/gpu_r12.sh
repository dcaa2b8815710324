set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r12
mkdir -p $O
cd $R
V='[{},{"occ_skip":0}]'
timeout -k 10 300 python bench.py --no-cpu > $O/bench_skip.json 2> $O/bench_skip.err && \
timeout -k 10 300 python bench.py --no-cpu --tune occ_skip=0 > $O/bench_noskip.json 2> $O/bench_noskip.err && \
timeout -k 10 300 python tools/kbench.py --rounds 4 --variants "$V" > $O/kb.json 2> $O/kb.err && \
timeout -k 10 300 python tools/kbench.py --ws-first --rounds 4 --variants "$V" > $O/kb_wsfirst.json 2> $O/kb_wsfirst.err
echo rc=$?
