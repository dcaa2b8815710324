set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r9
mkdir -p $O
cd $R
TAG=r01 bash tools/gpu_profile.sh && \
cd $R && timeout -k 10 600 python tools/scaling_emulation.py > $O/scaling.json 2> $O/scaling.err
echo rc=$?
cat $O/scaling.json | head -5
