set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1b
mkdir -p $O
cd $R
timeout -k 10 300 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1 && \
timeout -k 10 400 python tools/kbench.py --rounds 5 > $O/kbench.json 2> $O/kbench.err && \
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py > $O/bench_prof.json 2> $O/bench_prof.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_write.json 2> $O/pmc_write.err
echo rc=$?
tail -2 $O/pytest.log
cat $O/bench.json
