# Profiling round for a non-headline configuration: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE in separate
# --pmc passes, summarised by tools/pmc_summary.py into profiles/$TAG/*_$CONFIG_$DTYPE.* (the headline f32 round is
# tools/gpu_profile.sh). CONFIG=c2|ragged64|c5|headline, DTYPE=f32|bf16|f16.
set -o pipefail
TAG=${TAG:-r02}; CONFIG=${CONFIG:-c2}; DTYPE=${DTYPE:-f32}; STEPS=${STEPS:-50}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_${TAG}_${CONFIG}_${DTYPE}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config $CONFIG --acts-dtype $DTYPE"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $B --steps $STEPS --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B --steps 3 --warmup 1 --no-cpu > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B --steps 3 --warmup 1 --no-cpu > $O/pmc_write.json 2> $O/pmc_write.err && \
python3 $R/tools/pmc_summary.py --stats $O/stats --fetch $O/fetch --write $O/write --bench $O/bench_prof.json --tag $TAG --config $CONFIG --dtype $DTYPE > $O/summary.json && \
mkdir -p $O/profiles_out && cp $R/profiles/$TAG/*_${CONFIG}_${DTYPE}* $R/profiles/$TAG/kernel_stats_${CONFIG}*.csv $O/profiles_out/
echo rc=$?
