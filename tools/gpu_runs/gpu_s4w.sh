# final refresh (NaN rows for ll = -inf, sweeps): GPU suite, smoke, bench, rocprof + PMC, other configs
# (tools/gpu_full.sh), rocprofv3 stats + FETCH/WRITE PMC passes (tools/gpu_profile.sh), other configs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
TAG=full_s4w bash tools/gpu_full.sh && \
TAG=r01 bash tools/gpu_profile.sh && cd $R && \
O=$R/gpurun_out/s4w_cfg && mkdir -p $O && \
timeout -k 10 200 python bench.py --config c2 > $O/bench_c2.json 2> $O/c2.err && \
timeout -k 10 200 python bench.py --config ragged64 --no-cpu > $O/bench_ragged64.json 2> $O/r64.err && \
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 5 > $O/bench_c5.json 2> $O/c5.err && \
timeout -k 10 200 python bench.py --acts-dtype bf16 --no-cpu > $O/bench_bf16.json 2> $O/bf16.err
echo rc=$?
