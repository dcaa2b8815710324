set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r1
cd $R
timeout -k 10 400 python bench.py > gpurun_out/r1/bench.json 2> gpurun_out/r1/bench.err && \
cat gpurun_out/r1/bench.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1/prof -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/r1/bench_prof.json 2> $R/gpurun_out/r1/bench_prof.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r1/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/r1/pmc_fetch.json 2> $R/gpurun_out/r1/pmc_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r1/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/r1/pmc_write.json 2> $R/gpurun_out/r1/pmc_write.err
echo rc=$?
