# refresh after the halo recursion: GPU suite + smoke + bench (gpu_full.sh), rocprofv3 stats + PMC
# (gpu_profile.sh), the other configs, the C4 scaling emulation
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
TAG=full_s3x bash tools/gpu_full.sh && \
TAG=r01 bash tools/gpu_profile.sh && cd $R && \
O=$R/gpurun_out/s3x_cfg && mkdir -p $O && \
timeout -k 10 200 python bench.py --config c2 > $O/bench_c2.json 2> $O/c2.err && \
timeout -k 10 200 python bench.py --config ragged64 --no-cpu > $O/bench_ragged64.json 2> $O/r64.err && \
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 5 > $O/bench_c5.json 2> $O/c5.err && \
timeout -k 10 200 python bench.py --acts-dtype bf16 --no-cpu > $O/bench_bf16.json 2> $O/bf16.err && \
timeout -k 10 600 python tools/scaling_emulation.py > $O/scaling_c4.json 2> $O/scaling_c4.err
echo rc=$?
