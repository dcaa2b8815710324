# One profiling round: bench line, rocprofv3 kernel stats of the same command, FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes, summarised into profiles/$TAG by tools/pmc_summary.py.
set -o pipefail
TAG=${TAG:-r04}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --no-lengths-ab > $O/bench_prof.json 2> $O/bench_prof.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-lengths-ab > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-lengths-ab > $O/pmc_write.json 2> $O/pmc_write.err && \
python3 $R/tools/pmc_summary.py --stats $O/stats --fetch $O/fetch --write $O/write --bench $O/bench_prof.json --tag $TAG > $O/summary.json && \
cp -r $R/profiles $O/profiles_out
echo rc=$?
